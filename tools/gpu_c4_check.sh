#!/bin/bash
# C4 DeepFM: graphed vs eager step (samples/s), kernel trace of the graphed run, DeepFM tests.
set -u
export TMPDIR=/tmp
O=gpurun_out/c4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_graph_step.py tests/test_gpu_deepfm.py tests/test_gpu_deferred.py > $O/t.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/t.log; exit 3; }
tail -1 $O/t.log
timeout -k 10 600 python tools/bench_models.py --configs C4 --steps 100 --warmup 10 --no-cpu-baseline --out $O/c4_graph.json > $O/c4_graph.log 2>&1 || { echo "graph rc=$?"; tail $O/c4_graph.log; exit 3; }
timeout -k 10 600 python tools/bench_models.py --configs C4 --steps 100 --warmup 10 --no-cpu-baseline --eager-step --out $O/c4_eager.json > $O/c4_eager.log 2>&1 || { echo "eager rc=$?"; tail $O/c4_eager.log; exit 3; }
grep -h '"value"' $O/c4_graph.log $O/c4_eager.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/bench_models.py --configs C4 --steps 100 --warmup 10 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof rc=$?"; exit 3; }
echo prof-ok
