#!/bin/bash
# Host-side timeline of the C2 driver window, then the C4 timed-step kernel breakdown.
set -u
export TMPDIR=/tmp
O=gpurun_out/host
mkdir -p $O
timeout -k 10 300 python tools/host_timeline.py > $O/host.txt 2>&1 || { tail -20 $O/host.txt; exit 3; }
tail -60 $O/host.txt
MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_C4 -o run -- \
  python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_C4.log 2>&1 || exit 7
python tools/step_breakdown.py $O/tr_C4 32 $O/C4_step.json > $O/C4_step.txt || exit 8
head -60 $O/C4_step.txt | cut -c1-200
echo done
