#!/bin/bash
# Round-end refresh: smoke, GPU tests, C2 bench lines, rocprofv3 kernel trace of the
# default C2 bench (tools/gpu_check.sh), then the C3/C4/C5 model lines with CPU baselines.
# Each GPU step has its own time limit; a crash / timeout ends the script.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
PROF=1 bash tools/gpu_check.sh || exit $?
grep -q ABORT gpurun_out/summary.txt && exit 5
timeout -k 10 500 python tools/bench_models.py --out gpurun_out/models.json > gpurun_out/models.log 2>&1
rc=$?; echo "models rc=$rc"; grep '^{' gpurun_out/models.log | cut -c1-300
exit $rc
