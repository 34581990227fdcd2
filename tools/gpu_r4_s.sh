#!/bin/bash
# Round-4: K35 variants A/B (whole look-ahead rows, 7-wave budget) on the C2 windows.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
MIREC_LIB=recbole_amd/_lib/alt/whole.so timeout -k 10 600 $PT tests/test_gpu_step.py tests/test_gpu_e2e.py > $O/tests_whole.log 2>&1
rc=$?; tail -1 $O/tests_whole.log; [ $rc -eq 0 ] || exit 10
for v in base whole w7; do
  if [ $v != base ]; then export MIREC_LIB=recbole_amd/_lib/alt/$v.so; else unset MIREC_LIB; fi
  for i in 1 2; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_${v}_$i.log 2>&1 || exit 4
    echo "$v drv $(grep '^{' $O/drv_${v}_$i.log | cut -c70-110)"
  done
  timeout -k 10 400 python bench.py > $O/def_$v.log 2>&1 || exit 5
  echo "$v def $(grep '^{' $O/def_$v.log | cut -c70-110)"
done
