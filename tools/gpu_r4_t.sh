#!/bin/bash
# Round-4: onesweep device-wide sort — sort / reduce tests, SASRec tests, C3 trace + line.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 400 $PT tests/test_gpu_kernels.py -k "sort or scatter or reduce" > $O/tests_k.log 2>&1
rc=$?; tail -3 $O/tests_k.log; [ $rc -eq 0 ] || exit 9
timeout -k 10 700 $PT tests/test_gpu_sasrec.py tests/test_gpu_deferred.py tests/test_gpu_graph_step.py \
  tests/test_gpu_configs.py tests/test_gpu_lightgcn.py tests/test_gpu_shard.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
O3=gpurun_out/r4t/c3 bash tools/gpu_r4_r.sh 2>&1 | sed 's/^/C3: /' | grep -E "us/step|C3: \{" | head -30
