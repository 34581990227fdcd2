#!/bin/bash
# Round-4: K35 join memory orders — the memory-model form (MIREC_STEP_HANDOFF_FORMAL build "formal") vs the write-through
# hand-off with explicit drains (default). Tests on the default library,
# then C2 driver-window and default-window bench A/B.
# build the variant first: tools/build_variant.sh formal -DMIREC_STEP_HANDOFF_FORMAL
set -u
export TMPDIR=/tmp
O=gpurun_out/r4af
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 500 $PT tests/test_gpu_step.py tests/test_gpu_chain.py tests/test_gpu_e2e.py tests/test_gpu_deferred.py > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit 10
for v in formal base formal base formal base; do
  if [ $v != base ]; then export MIREC_LIB=recbole_amd/_lib/alt/$v.so; else unset MIREC_LIB; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_$v.log 2>&1 || exit 4
  echo "$v drv $(grep '^{' $O/drv_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
for v in formal base; do
  if [ $v != base ]; then export MIREC_LIB=recbole_amd/_lib/alt/$v.so; else unset MIREC_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/def_$v.log 2>&1 || exit 5
  echo "$v def $(grep '^{' $O/def_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
