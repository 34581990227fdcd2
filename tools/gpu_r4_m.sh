#!/bin/bash
# Round-4: K3 defaults (6 waves, non-temporal gradient stores) — K3 tests, gather probe.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 600 $PT tests/test_gpu_kernels.py tests/test_gpu_step.py tests/test_gpu_dp.py \
  tests/test_gpu_shard.py tests/test_gpu_e2e.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
for i in 1 2; do
  timeout -k 10 120 python tools/gather_probe.py > $O/g$i.log 2>&1 || exit 3
  cut -c1-200 $O/g$i.log
done
