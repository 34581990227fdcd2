#!/bin/bash
# Round-4: K36 / K4s parity, then the preparation latency probe.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 400 $PT tests/test_gpu_group.py tests/test_gpu_spec_walk.py > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 300 python tools/probe_prep.py > $O/probe.log 2>&1 || { tail $O/probe.log; exit 4; }
grep '^{' $O/probe.log
timeout -k 10 300 python tools/host_timeline.py --reps 3 > $O/host.log 2>&1 || { tail $O/host.log; exit 5; }
tail -45 $O/host.log
