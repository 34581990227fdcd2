#!/bin/bash
# Round-4: K10 forward group size A/B (4 vs 8 slices per prefetch group) on C4.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4ae
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
MIREC_LIB=recbole_amd/_lib/alt/fwdpf2.so timeout -k 10 400 $PT tests/test_gpu_mlp.py > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit 10
for v in base fwdu4 fwdpf2 base fwdu4 fwdpf2; do
  if [ $v != base ]; then export MIREC_LIB=recbole_amd/_lib/alt/$v.so; else unset MIREC_LIB; fi
  timeout -k 10 300 python tools/bench_models.py --configs C4 --no-cpu-baseline > $O/c4_$v.log 2>&1 || exit 4
  echo "$v $(grep '^{' $O/c4_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["launch_us"], d["roofline"]["frac"])')"
done
