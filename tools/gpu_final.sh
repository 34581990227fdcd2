#!/bin/bash
# Round-end refresh: C3/C4/C5 model lines (with CPU baselines) and a rocprofv3 kernel
# trace of the default C2 bench. Each GPU step has its own time limit.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python tools/bench_models.py --out gpurun_out/models.json > gpurun_out/models.log 2>&1
rc=$?; echo "models rc=$rc"; grep '^{' gpurun_out/models.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
SMOKE=0 TESTS=0 BENCH=0 PROF=1 bash tools/gpu_check.sh
