#!/bin/bash
# Kernel trace of the default C2 bench (timed window between trace markers) ->
# per-step breakdown; K35 durations and the gaps between consecutive K35 launches.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3t
mkdir -p $O
BENCH_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
  python bench.py --no-cpu-baseline --no-eval --in-memory > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 3; }
grep -o '"value": [0-9.]*' $O/bench.log | head -n1
python tools/step_breakdown.py $O/tr $(python -c "import json,re;print(json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])['steps'])") $O/c2_step.json > $O/c2_step.txt || exit 4
head -24 $O/c2_step.txt
python tools/k35_gaps.py $O/tr > $O/gaps.txt || exit 5
cat $O/gaps.txt
echo done
