#!/bin/bash
# Round-4: DeepFM keys formed inside the chained sort — tests, C4 trace + lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4ab
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 400 $PT tests/test_gpu_kernels.py -k "flush or adam or deferred" > $O/tests_k.log 2>&1
rc=$?; tail -2 $O/tests_k.log; [ $rc -eq 0 ] || exit 9
timeout -k 10 700 $PT tests/test_gpu_deepfm.py tests/test_gpu_deferred.py tests/test_gpu_graph_step.py \
  tests/test_gpu_mlp.py tests/test_gpu_configs.py tests/test_gpu_shard.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_C4 -o run -- \
  python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_C4.log 2>&1 || exit 7
python tools/step_breakdown.py $O/tr_C4 32 $O/C4_step.json > $O/C4_step.txt || exit 8
head -40 $O/C4_step.txt | cut -c1-120
for i in 1 2; do
  timeout -k 10 300 python tools/bench_models.py --configs C4 --no-cpu-baseline > $O/c4_$i.log 2>&1 || exit 4
  grep '^{' $O/c4_$i.log | cut -c1-200
done
