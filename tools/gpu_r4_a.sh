#!/bin/bash
# Round-4 check: flush-rows kernel + K36 parity, the fused path's step / chain tests,
# then the driver-window bench (twice) and its kernel trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 300 $PT tests/test_gpu_kernels.py -k "flush or deferred" > $O/tests_k.log 2>&1
rc=$?; tail -2 $O/tests_k.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 500 $PT tests/test_gpu_group.py tests/test_gpu_step.py tests/test_gpu_e2e.py tests/test_gpu_chain.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 11
for i in 1 2; do
  timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $O/bench_short_$i.log 2>&1 || exit 4
  tail -1 $O/bench_short_$i.log | cut -c1-160
done
bash tools/trace_short.sh || exit 5
cat gpurun_out/prof_short/tw.txt | head -70
