#!/bin/bash
# Round-4: K35 grid pieces (segment tails last) + C4 launch folds (BCE mean, unit seed,
# step advance) — tests, C2 benches, stamps, C4 trace and lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 900 $PT tests/test_gpu_step.py tests/test_gpu_chain.py tests/test_gpu_e2e.py \
  tests/test_c2_atomic_path.py tests/test_gpu_group.py tests/test_gpu_deepfm.py \
  tests/test_gpu_graph_step.py tests/test_gpu_deferred.py tests/test_gpu_mlp.py \
  tests/test_gpu_configs.py tests/test_gpu_sasrec.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv_$i.log 2>&1 || exit 4
  grep '^{' $O/bench_drv_$i.log | cut -c1-150
done
timeout -k 10 400 python bench.py > $O/bench_def.log 2>&1 || exit 5
grep '^{' $O/bench_def.log | cut -c1-150
MIREC_LIB=recbole_amd/_lib/alt/step_stamps.so timeout -k 10 300 python tools/probe_step_stamps.py --warmup 96 --steps 24 > $O/stamps.jsonl 2> $O/stamps.err || exit 6
MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_C4 -o run -- \
  python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_C4.log 2>&1 || exit 7
python tools/step_breakdown.py $O/tr_C4 32 $O/C4_step.json > $O/C4_step.txt || exit 8
head -14 $O/C4_step.txt | cut -c1-120
for i in 1 2; do
  timeout -k 10 300 python tools/bench_models.py --configs C4 --no-cpu-baseline > $O/c4_$i.log 2>&1 || exit 9
  grep '^{' $O/c4_$i.log | cut -c1-200
done
