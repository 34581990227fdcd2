#!/bin/bash
# Driver-window fill: parity tests of the step path, then short (--warmup 5 --steps 20)
# benches with chunk-ramp variants, the default window, and one marked short trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3fill2
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_step.py tests/test_gpu_e2e.py tests/test_gpu_chain.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
b() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --in-memory "$@" > $O/$tag 2>&1 || { tail -5 $O/$tag; exit 4; }
  echo "$tag: $(grep -o '"value": [0-9.]*' $O/$tag | head -n1) $(grep -o '"kernels_us": {[^}]*}' $O/$tag | head -n1)"
}
S="--warmup 5 --steps 20"
b base $S; b base2 $S
b r4444 $S --ramp 4,4,4,4,8,16,32; b r2444 $S --ramp 2,4,4,4,8,16,32; b r468 $S --ramp 4,6,8,10,12,16,24,32
b default; b default_r4444 --ramp 4,4,4,4,8,16,32
BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- \
  python bench.py --no-cpu-baseline --no-eval --in-memory $S > $O/trace_bench.log 2>&1 || exit 5
echo done
