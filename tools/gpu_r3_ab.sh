#!/bin/bash
# Parity tests of the step path, then default-window and short benches (tag from $1).
# Stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3ab_${1:-x}
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_step.py tests/test_gpu_e2e.py tests/test_gpu_chain.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
b() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --in-memory "$@" > $O/$tag 2>&1 || { tail -5 $O/$tag; exit 4; }
  echo "$tag: $(grep -o '"value": [0-9.]*' $O/$tag | head -n1) $(grep -o '"kernels_us": {[^}]*}' $O/$tag | head -n1)"
}
b default; b default2; b short --warmup 5 --steps 20
BENCH_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- \
  python bench.py --no-cpu-baseline --no-eval --in-memory > $O/trace_bench.log 2>&1 || exit 5
python tools/k35_gaps.py $O/tr > $O/gaps.txt || exit 6
head -4 $O/gaps.txt
echo done
