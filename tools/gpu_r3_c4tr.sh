#!/bin/bash
# C4 timed-step kernel trace (markers) -> per-step breakdown.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3c4tr
mkdir -p $O
MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_C4 -o run -- \
  python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_C4.log 2>&1 || exit 7
python tools/step_breakdown.py $O/tr_C4 32 $O/C4_step.json > $O/C4_step.txt || exit 8
head -40 $O/C4_step.txt
