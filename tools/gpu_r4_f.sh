#!/bin/bash
# Round-4: the 8-bit block sort (segment sort tests), then C4 tests, C4 step trace and lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 300 $PT tests/test_gpu_kernels.py -k "segment_sort" > $O/tests_sort.log 2>&1
rc=$?; tail -3 $O/tests_sort.log; [ $rc -eq 0 ] || exit 9
timeout -k 10 600 $PT tests/test_gpu_deepfm.py tests/test_gpu_mlp.py tests/test_gpu_configs.py \
  -k "not c3 and not c5" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_C4 -o run -- \
  python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_C4.log 2>&1 || exit 7
python tools/step_breakdown.py $O/tr_C4 32 $O/C4_step.json > $O/C4_step.txt || exit 8
head -30 $O/C4_step.txt | cut -c1-120
for i in 1 2; do
  timeout -k 10 300 python tools/bench_models.py --configs C4 --no-cpu-baseline > $O/c4_$i.log 2>&1 || exit 4
  grep '^{' $O/c4_$i.log | cut -c1-200
done
