#!/bin/bash
# Round-4: default-window C2 bench and the driver-window kernel stats.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_def.log 2>&1 || exit 5
grep '^{' $O/bench_def.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- \
  python bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit 6
grep '^{' $O/prof.log | cut -c1-160
