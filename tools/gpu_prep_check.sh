#!/bin/bash
# Sampler + chunk-prep changes: sampler tests, walk phase profile, then the fused checks.
set -u
export TMPDIR=/tmp
O=gpurun_out/walk
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "sampler or walk or used or repeatable" tests/test_gpu_sampled_eval.py > $O/t.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/t.log; exit 3; }
tail -1 $O/t.log
MIREC_LIB=recbole_amd/_lib/alt/walkprof.so timeout -k 10 200 python tools/probe_walk.py > $O/prof_new.log 2>&1 || { echo prof fail; tail $O/prof_new.log; exit 3; }
grep rep $O/prof_new.log | tail -1
bash tools/gpu_fused_check.sh
