#!/bin/bash
# C2 driver window (--warmup 5 --steps 20): the default vs variants of the pipeline start,
# then the kernel timeline of the default.
set -u
export TMPDIR=/tmp
O=gpurun_out/fill
mkdir -p $O
run() {  # name, extra args
  local name=$1; shift
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval --in-memory "$@" > $O/$name.$rep.log 2>&1 || { tail -5 $O/$name.$rep.log; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('$O/$name.$rep.log') if l.startswith('{')][0]); print('$name', d['value'], d['ms_per_step'], d['config']['chunk_plan_timed'])"
  done
}
run default
run side --no-main-first
run r2 --ramp 2,4,8,16,32
run r3 --ramp 3,6,12,24
run r6 --ramp 6,8,16,32
bash tools/trace_short.sh || exit 4
head -60 gpurun_out/prof_short/tw.txt
echo done
