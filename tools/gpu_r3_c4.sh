#!/bin/bash
# C4 A/B: reduction piece length for d <= 16 (32 / 16 / 8), DeepFM parity tests per variant.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3c4
mkdir -p $O
for v in base ch16 ch8; do
  if [ $v = base ]; then unset MIREC_LIB; else export MIREC_LIB=recbole_amd/_lib/alt/$v.so; fi
  timeout -k 10 300 python -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_gpu_deepfm.py tests/test_gpu_deferred.py > $O/t_$v.log 2>&1 || { tail -5 $O/t_$v.log; exit 3; }
  timeout -k 10 300 python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline --out $O/c4_$v.json > $O/c4_$v.log 2>&1 || { tail -5 $O/c4_$v.log; exit 4; }
  python -c "import json; r=json.load(open('$O/c4_$v.json')); r=r[0] if isinstance(r,list) else r; print('$v', r['value'], r['ms_per_step'])"
done
echo done
