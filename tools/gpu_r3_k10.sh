#!/bin/bash
# K10 fused MLP: its tests + the DeepFM / graph-step / shard tests, the C4 line, then the
# C2 driver-window trace. Stops at the first failing step.
set -u
export TMPDIR=/tmp
O=gpurun_out/k10
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_mlp.py tests/test_gpu_deepfm.py tests/test_gpu_graph_step.py \
  tests/test_gpu_shard.py > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 300 python tools/bench_models.py --configs C4 --steps 64 --warmup 8 --no-cpu-baseline --out $O/c4.json > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 3; }
python -c "import json; r=json.load(open('$O/c4.json')); r=r[0] if isinstance(r,list) else r; print(json.dumps({k: r.get(k) for k in ('value','ms_per_step','roofline')})[:1500])"
bash tools/trace_short.sh || exit 4
cat gpurun_out/prof_short/tw.txt | head -60
echo done
