#!/bin/bash
# Round-3 model measurements, in the order the model lines read their inputs: kernel
# traces of the C4 and C3 timed steps (markers) -> per-step breakdowns into profiles/
# (the C4 roofline follows the breakdown's dominant kernel); FETCH / WRITE passes of the
# C4 step's kernels -> profiles/r03_models_pmc.json; then the C3-C5 lines with CPU
# baselines (-> models.json). Stops at the first failing step.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu \
  tests/test_gpu_mlp.py tests/test_gpu_deepfm.py tests/test_gpu_graph_step.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 10
for c in C4 C3; do
  MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$c -o run -- \
    python tools/bench_models.py --configs $c --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_$c.log 2>&1 || exit 7
  python tools/step_breakdown.py $O/tr_$c 32 $O/${c}_step.json > $O/${c}_step.txt || exit 8
  cp $O/${c}_step.json profiles/r03_${c}_step.json
  head -24 $O/${c}_step.txt | cut -c1-120
done
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4fetch -o run -- \
  python tools/bench_models.py --configs C4 --steps 4 --warmup 2 --no-cpu-baseline > $O/c4fetch.log 2>&1 || exit 4
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c4write -o run -- \
  python tools/bench_models.py --configs C4 --steps 4 --warmup 2 --no-cpu-baseline > $O/c4write.log 2>&1 || exit 5
python tools/models_pmc.py $O/c4fetch $O/c4write $O/models_pmc.json mlp_fwd_kernel mlp_bwd_data_kernel \
  mlp_bwd_weight_kernel ctx_fm_bwd_kernel ctx_fm_fwd segsort_lds_kernel || exit 6
cp $O/models_pmc.json profiles/r03_models_pmc.json
cat $O/models_pmc.json | head -40
timeout -k 10 700 python tools/bench_models.py --out $O/models.json > $O/models.log 2>&1
rc=$?; echo "models rc=$rc"; grep '^{' $O/models.log | cut -c1-250; [ $rc -eq 0 ] || exit 3
echo done
