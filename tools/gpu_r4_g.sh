#!/bin/bash
# Round-4: per-block 8-bit sort — tests, phase timing on C4's keys.
set -u
O=gpurun_out/r4g
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 300 $PT tests/test_gpu_kernels.py -k "segment_sort" > $O/tests_sort.log 2>&1
rc=$?; tail -2 $O/tests_sort.log; [ $rc -eq 0 ] || exit 9
timeout -k 10 120 python tools/probe_r8.py > $O/default.log 2>&1 || exit 3
MIREC_LIB=recbole_amd/_lib/alt/r8probe.so timeout -k 10 120 python tools/probe_r8.py > $O/probe.log 2>&1 || exit 4
cat $O/default.log $O/probe.log
