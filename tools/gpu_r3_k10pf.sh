#!/bin/bash
# K10 with the layer-boundary prefetch: its tests, then the C4 line.
set -u
export TMPDIR=/tmp
O=gpurun_out/k10pf
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu \
  tests/test_gpu_mlp.py tests/test_gpu_deepfm.py tests/test_gpu_graph_step.py tests/test_gpu_configs.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
for rep in 1 2; do
  timeout -k 10 300 python tools/bench_models.py --configs C4 --steps 64 --warmup 8 --no-cpu-baseline --out $O/c4_$rep.json > $O/c4_$rep.log 2>&1 || { tail -20 $O/c4_$rep.log; exit 3; }
  python -c "import json; r=json.load(open('$O/c4_$rep.json')); r=r[0] if isinstance(r,list) else r; print(json.dumps({k: r.get(k) for k in ('value','ms_per_step')}), r['k10_fwd']['launch_us'], r['k10_bwd']['call_us'])"
done
echo done
