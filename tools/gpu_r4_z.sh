#!/bin/bash
# Round-4: the first timed chunk prepared on the model stream (MIREC_MAIN_FIRST=1) vs
# the prep / group streams — driver-window lines and the timeline.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4z2
mkdir -p $O
for v in 0 1; do
  for i in 1 2 3; do
    MIREC_MAIN_FIRST=$v timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-eval > $O/drv_${v}_$i.log 2>&1 || exit 4
    echo "main_first=$v $(grep '^{' $O/drv_${v}_$i.log | cut -c70-100)"
  done
done
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
MIREC_MAIN_FIRST=1 timeout -k 10 500 $PT tests/test_gpu_chain.py tests/test_gpu_e2e.py > $O/tests.log 2>&1 || exit 9
tail -1 $O/tests.log
MIREC_MAIN_FIRST=1 bash tools/trace_short.sh || exit 5
head -30 gpurun_out/prof_short/tw.txt
