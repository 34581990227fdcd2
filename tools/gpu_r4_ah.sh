#!/bin/bash
# Round-4: K35 last-adder acquire (buffer_inv sc1 per split row) vs none (probe build
# tools/build_variant.sh noacq -DMIREC_STEP_NO_ACQUIRE), C2 bench A/B. Measurement only.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4ah
mkdir -p $O
for v in base noacq base noacq base noacq; do
  if [ $v != base ]; then export MIREC_LIB=$PWD/recbole_amd/_lib/alt/$v.so; else unset MIREC_LIB; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_$v.log 2>&1 || exit 4
  echo "$v drv $(grep '^{' $O/drv_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
for v in base noacq; do
  if [ $v != base ]; then export MIREC_LIB=$PWD/recbole_amd/_lib/alt/$v.so; else unset MIREC_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/def_$v.log 2>&1 || exit 5
  echo "$v def $(grep '^{' $O/def_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
