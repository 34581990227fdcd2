#!/bin/bash
# Round-4: DPP group sums — the whole GPU suite, then the C2 bench (driver and default windows).
set -u
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 1000 $PT tests/ > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv_$i.log 2>&1 || exit 4
  grep '^{' $O/bench_drv_$i.log | cut -c1-160
done
timeout -k 10 400 python bench.py > $O/bench_def.log 2>&1 || exit 5
grep '^{' $O/bench_def.log | cut -c1-160
