#!/bin/bash
# K35 with split rows after removing the sweep: parity tests, then the default bench
# at flush periods 64 / 32 / 48 / 96. Stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3f2
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_step.py tests/test_gpu_e2e.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
b() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --in-memory "$@" > $O/$tag 2>&1 || { tail -5 $O/$tag; exit 4; }
  echo "$tag: $(grep -o '"value": [0-9.]*' $O/$tag | head -n1) $(grep -o '"kernels_us": {[^}]*}' $O/$tag | head -n1)"
}
b f64; b f32 --flush-every 32; b f48 --flush-every 48; b f96 --flush-every 96; b f64b
echo done
