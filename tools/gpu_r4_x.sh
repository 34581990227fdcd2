#!/bin/bash
# Round-4 measurement pass: the whole GPU suite, smoke, C2 bench (default and driver
# windows, kernel stats), the model configurations with CPU baselines.
set -u
export TMPDIR=/tmp
O=${OX:-gpurun_out/r4x}
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 900 $PT tests/ > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 11
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_def.log 2>&1 || exit 4
grep '^{' $O/bench_def.log > $O/bench_def.json; cut -c1-150 $O/bench_def.json
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv.log 2>&1 || exit 5
grep '^{' $O/bench_drv.log | cut -c1-150
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_def -o run -- \
  python bench.py > $O/prof_def.log 2>&1 || exit 6
timeout -k 10 900 python tools/bench_models.py --out $O/r04_models.json > $O/models.log 2>&1 || exit 7
grep '^{' $O/models.log | cut -c1-170
