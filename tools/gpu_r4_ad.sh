#!/bin/bash
# Round-4: deferred Adam with a capped grid (blocks loop over rows) — tests, C3 / C4 / C2.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4ad
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 900 $PT tests/test_gpu_deferred.py tests/test_gpu_kernels.py tests/test_gpu_sasrec.py \
  tests/test_gpu_deepfm.py tests/test_gpu_graph_step.py tests/test_gpu_e2e.py tests/test_gpu_chain.py \
  tests/test_gpu_dp.py tests/test_gpu_shard.py tests/test_gpu_step.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 500 python tools/bench_models.py --configs C3,C4 --no-cpu-baseline > $O/m.log 2>&1 || exit 4
grep '^{' $O/m.log | cut -c1-170
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-eval > $O/drv.log 2>&1 || exit 5
grep '^{' $O/drv.log | cut -c1-150
