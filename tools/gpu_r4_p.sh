#!/bin/bash
# Round-4: K35 grid order (touched rows before look-ahead, look-ahead slots looping) —
# K35 tests, C2 driver/default windows, stamps.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 600 $PT tests/test_gpu_step.py tests/test_gpu_chain.py tests/test_gpu_e2e.py \
  tests/test_c2_atomic_path.py tests/test_gpu_group.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv_$i.log 2>&1 || exit 4
  grep '^{' $O/bench_drv_$i.log | cut -c1-150
done
timeout -k 10 400 python bench.py > $O/bench_def.log 2>&1 || exit 5
grep '^{' $O/bench_def.log | cut -c1-150
MIREC_LIB=recbole_amd/_lib/alt/step_stamps.so timeout -k 10 300 python tools/probe_step_stamps.py --warmup 96 --steps 24 > $O/stamps.jsonl 2> $O/stamps.err || exit 6
tail -2 $O/stamps.jsonl
