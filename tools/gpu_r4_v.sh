#!/bin/bash
# Round-4: second-level merges — kernel tests, SASRec / deferred tests, C3 trace + line.
set -u
export TMPDIR=/tmp
O=${OV:-gpurun_out/r4v}
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 400 $PT tests/test_gpu_kernels.py -k "merge or reduce or sort or scatter" > $O/tests_k.log 2>&1
rc=$?; tail -3 $O/tests_k.log; [ $rc -eq 0 ] || exit 9
timeout -k 10 700 $PT tests/test_gpu_sasrec.py tests/test_gpu_deferred.py tests/test_gpu_graph_step.py \
  tests/test_gpu_configs.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
O3=$O/c3 bash tools/gpu_r4_r.sh 2>&1 | grep -E "us/step|^\{" | head -40
