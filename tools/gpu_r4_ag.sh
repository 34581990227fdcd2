#!/bin/bash
# Round-4: relaxed agent-scope tickets / status words (no buffer_wbl2 / buffer_inv per
# block) in the chained sorts, onesweep cleanup, dense-Adam advance, chunk finish and the
# MLP dropout counter. Variant: tools/build_variant.sh relaxed (from the edited tree).
set -u
export TMPDIR=/tmp
O=gpurun_out/r4ag
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
export MIREC_LIB=$PWD/recbole_amd/_lib/alt/relaxed.so
timeout -k 10 600 $PT tests/test_gpu_kernels.py tests/test_gpu_deepfm.py tests/test_gpu_mlp.py \
  tests/test_gpu_e2e.py tests/test_gpu_chain.py tests/test_gpu_sasrec.py > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit 10
for v in base relaxed base relaxed; do
  if [ $v != base ]; then export MIREC_LIB=$PWD/recbole_amd/_lib/alt/$v.so; else unset MIREC_LIB; fi
  timeout -k 10 300 python tools/bench_models.py --configs C4,C3 --no-cpu-baseline > $O/m_$v.log 2>&1 || exit 4
  echo "$v $(grep '^{' $O/m_$v.log | python -c 'import json,sys
for l in sys.stdin: d=json.loads(l); print(d["config"].get("workload","?")[:12], d["value"], end=" | ")')"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_$v.log 2>&1 || exit 5
  echo "$v drv $(grep '^{' $O/drv_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
