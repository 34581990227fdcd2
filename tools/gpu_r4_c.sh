#!/bin/bash
# Round-4: parity of the new kernels (K36, K4s, K35 rows-per-workgroup, sparse flush,
# K3 at ids) and the fused chain; executed-work counters; the preparation probe; the host
# timeline; driver-window A/B runs of the variants; the kernel trace of the default.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 700 $PT tests/test_gpu_group.py tests/test_gpu_spec_walk.py tests/test_gpu_step.py \
  tests/test_gpu_e2e.py tests/test_gpu_chain.py tests/test_gpu_kernels.py tests/test_gpu_shard.py > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit 10
MIREC_LIB=recbole_amd/_lib/alt/work.so timeout -k 10 300 python tools/probe_step_work.py --out $O/k35_work.json > $O/work.log 2>&1 || { tail $O/work.log; exit 3; }
python -c "import json; d=json.load(open('$O/k35_work.json')); print(json.dumps(d['timed_region'])[:700]); print(json.dumps(d['measurement_window']['per_launch']))"
timeout -k 10 300 python tools/probe_prep.py > $O/probe.log 2>&1 || { tail $O/probe.log; exit 4; }
grep '^{' $O/probe.log
timeout -k 10 200 python tools/host_timeline.py --reps 2 > $O/host.log 2>&1 || { tail $O/host.log; exit 5; }
tail -34 $O/host.log
run() {   # name "env assignments" bench-args...
  local name=$1 envs=$2; shift 2
  for i in 1 2; do
    env MIREC_X=1 $envs timeout -k 10 200 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval "$@" > $O/b_${name}_$i.log 2>&1 || return 1
    echo "$name $i $(tail -1 $O/b_${name}_$i.log | sed 's/.*"value": \([0-9.]*\).*/\1/')"
  done
}
run default "" || exit 6
run mainfirst "" --main-first || exit 6
run ramp4_16 "" --ramp 4,16 || exit 6
run ramp2_18 "" --ramp 2,18 || exit 6
run nospec "MIREC_SPEC_WALK=0" || exit 6
run rpb1 "MIREC_LIB=recbole_amd/_lib/alt/k35_rpb1.so" || exit 6
run w5 "MIREC_LIB=recbole_amd/_lib/alt/k35_w5.so" || exit 6
run noacq "MIREC_LIB=recbole_amd/_lib/alt/k35_noacq.so" || exit 6
run wt "MIREC_LIB=recbole_amd/_lib/alt/k35_wt.so" || exit 6
bash tools/trace_short.sh || exit 7
cat gpurun_out/prof_short/tw.txt | head -80
