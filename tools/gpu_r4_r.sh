#!/bin/bash
# Round-4: C3 step trace and line.
set -u
export TMPDIR=/tmp
O=${O3:-gpurun_out/r4r}
mkdir -p $O
MODELS_MARKERS=1 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/tr_C3 -o run -- \
  python tools/bench_models.py --configs C3 --steps 8 --warmup 3 --no-cpu-baseline > $O/tr_C3.log 2>&1 || exit 7
python tools/step_breakdown.py $O/tr_C3 8 $O/C3_step.json > $O/C3_step.txt || exit 8
head -40 $O/C3_step.txt | cut -c1-140
timeout -k 10 500 python tools/bench_models.py --configs C3 --no-cpu-baseline > $O/c3.log 2>&1 || exit 9
grep '^{' $O/c3.log | cut -c1-300
