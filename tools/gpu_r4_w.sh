#!/bin/bash
# Round-4: deferred-Adam workgroup size A/B (64 vs 256 lanes) on C3 / C4; fixup prefetch.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4w
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
MIREC_LIB=recbole_amd/_lib/alt/dblk256.so timeout -k 10 700 $PT tests/test_gpu_deferred.py tests/test_gpu_kernels.py -k "deferred or reduce or merge or adam" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
for v in base dblk256; do
  if [ $v != base ]; then export MIREC_LIB=recbole_amd/_lib/alt/$v.so; else unset MIREC_LIB; fi
  timeout -k 10 500 python tools/bench_models.py --configs C3,C4 --no-cpu-baseline > $O/m_$v.log 2>&1 || exit 4
  echo $v; grep '^{' $O/m_$v.log | cut -c1-170
done
unset MIREC_LIB
MIREC_LIB=recbole_amd/_lib/alt/work.so timeout -k 10 600 python tools/probe_step_work.py --warmup 64 --steps 256 --out $O/r04_k35_work_w64_s256.json > $O/work.log 2>&1 || exit 6
MIREC_LIB=recbole_amd/_lib/alt/work.so timeout -k 10 300 python tools/probe_step_work.py --warmup 5 --steps 20 --out $O/r04_k35_work_w5_s20.json > $O/work5.log 2>&1 || exit 7
tail -3 $O/work.log | cut -c1-200
