#!/bin/bash
# Round-4 profiles: gather PMC (separate FETCH / WRITE passes), C2 driver-window kernel
# stats, C2 bench lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 120 python tools/gather_probe.py --out $O/gather_probe.json > $O/gp.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- \
  python tools/gather_probe.py > $O/pf.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- \
  python tools/gather_probe.py > $O/pw.log 2>&1 || exit 5
python tools/gather_pmc.py $O/pmc_fetch $O/pmc_write $O/gather_probe.json $O/r04_gather.json || exit 6
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit 7
grep '^{' $O/prof.log | cut -c1-160
