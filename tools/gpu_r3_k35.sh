#!/bin/bash
# K35 fused step: kernel parity tests, schedule / chain / shard bitwise tests, then the
# driver-window bench with and without K35. Stops at the first failing GPU step.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_step.py > $O/step_tests.log 2>&1
rc=$?; tail -3 $O/step_tests.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 900 $T tests/test_gpu_e2e.py tests/test_gpu_chain.py tests/test_gpu_shard.py > $O/bitwise_tests.log 2>&1
rc=$?; tail -3 $O/bitwise_tests.log; [ $rc -le 1 ] || exit $rc
for v in fused k3k5; do
  A=""; [ $v = k3k5 ] && A="--no-fused-step"
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval $A > $O/$v.short$rep 2>&1 || exit 4
    echo "$v short/$rep: $(grep -o '"value": [0-9.]*' $O/$v.short$rep | head -n1) $(grep -o '"us_per_step": [0-9.]*' $O/$v.short$rep | head -n1)"
  done
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval $A > $O/$v.default 2>&1 || exit 5
  echo "$v default: $(grep -o '"value": [0-9.]*' $O/$v.default | head -n1) $(grep -o '"kernels_us": {[^}]*}' $O/$v.default | head -n1)"
done
echo done
