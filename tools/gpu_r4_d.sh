#!/bin/bash
# Round-4: K36 phase timing (early-exit probe builds), chunk-plan (ramp) A/B of the
# driver window, w5 A/B.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 500 $PT tests/test_gpu_spec_walk.py tests/test_gpu_chain.py tests/test_gpu_kernels.py -k "adam or flush or spec or chain" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 200 python tools/probe_prep.py --reps 30 > $O/probe.log 2>&1 || { tail $O/probe.log; exit 3; }
grep '^{' $O/probe.log
for v in 1 2 3 4; do
  MIREC_LIB=recbole_amd/_lib/alt/grp$v.so timeout -k 10 200 python tools/probe_prep.py --reps 30 > $O/grp$v.log 2>&1 || { tail $O/grp$v.log; exit 3; }
  echo "grp$v $(grep '"batches": 4' $O/grp$v.log)"
done
run() {   # name "env assignments" bench-args...
  local name=$1 envs=$2; shift 2
  for i in 1 2 3; do
    env MIREC_X=1 $envs timeout -k 10 200 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval "$@" > $O/b_${name}_$i.log 2>&1 || return 1
    echo "$name $i $(tail -1 $O/b_${name}_$i.log | sed 's/.*"value": \([0-9.]*\).*/\1/')"
  done
}
run default "" || exit 6
run nopk "MIREC_LIB=recbole_amd/_lib/alt/nopk.so" || exit 6
run r20 "" --ramp 20 || exit 6
run r16 "" --ramp 16 || exit 6
run r12 "" --ramp 12 || exit 6
run r8 "" --ramp 8 || exit 6
run r20mf "" --ramp 20 --main-first || exit 6
run w5 "MIREC_LIB=recbole_amd/_lib/alt/k35_w5.so" || exit 6
run w5r20 "MIREC_LIB=recbole_amd/_lib/alt/k35_w5.so" --ramp 20 || exit 6
