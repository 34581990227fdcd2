#!/bin/bash
# Round-4: DPP block scan + chained block sort — the whole GPU suite, then C4.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 1000 $PT tests/ > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 120 python tools/probe_r8.py > $O/r8.log 2>&1 || exit 3
cut -c1-120 $O/r8.log
for i in 1 2; do
  timeout -k 10 300 python tools/bench_models.py --configs C4 --no-cpu-baseline > $O/c4_$i.log 2>&1 || exit 4
  grep '^{' $O/c4_$i.log | cut -c1-200
done
