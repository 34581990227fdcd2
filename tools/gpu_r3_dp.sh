#!/bin/bash
# Segment-relative reduction chunks: kernel tests, deferred / DeepFM / SASRec parity, and
# the 2-rank sharded-vs-replicated (bitwise) and sharded-vs-one-process tests.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3dp
mkdir -p $O
T="python -u -m pytest -x -v -s -p no:cacheprovider --timeout 400 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_kernels.py -k "segment or scatter" > $O/tests_k.log 2>&1 || { tail -20 $O/tests_k.log; exit 3; }
tail -1 $O/tests_k.log
timeout -k 10 900 $T tests/test_gpu_deferred.py tests/test_gpu_deepfm.py tests/test_gpu_sasrec.py tests/test_gpu_dp.py > $O/tests.log 2>&1
rc=$?; grep -E "max \\||passed|failed|Error" $O/tests.log | tail -40; exit $rc
