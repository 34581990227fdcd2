#!/bin/bash
# K10 tests, then the C4 timed-step kernel breakdown and the C4 line.
set -u
export TMPDIR=/tmp
O=gpurun_out/k10b
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_mlp.py tests/test_gpu_deepfm.py > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit 10
MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_C4 -o run -- \
  python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_C4.log 2>&1 || exit 7
python tools/step_breakdown.py $O/tr_C4 32 $O/C4_step.json > $O/C4_step.txt || exit 8
head -45 $O/C4_step.txt | cut -c1-160
timeout -k 10 300 python tools/bench_models.py --configs C4 --steps 64 --warmup 8 --no-cpu-baseline --out $O/c4.json > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 3; }
python -c "import json; r=json.load(open('$O/c4.json')); r=r[0] if isinstance(r,list) else r; print(json.dumps({k: r.get(k) for k in ('value','ms_per_step')}))"
echo done
