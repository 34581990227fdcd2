#!/bin/bash
# K35 with staged contribution ids: parity tests, bitwise chain, driver-window and
# default benches, kernel trace of the driver window. Stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_step.py tests/test_gpu_e2e.py tests/test_gpu_chain.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
b() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval "$@" > $O/$tag 2>&1 || exit 4
  echo "$tag: $(grep -o '"value": [0-9.]*' $O/$tag | head -n1) $(grep -o '"kernels_us": {[^}]*}' $O/$tag | head -n1)"
}
b short_a --warmup 5 --steps 20; b short_b --warmup 5 --steps 20
b default
BENCH_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
  python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $O/trace.log 2>&1 || exit 6
python tools/check_timed_window.py $O/trace $O/timed_window.json > $O/tw.txt
head -60 $O/tw.txt
echo done
