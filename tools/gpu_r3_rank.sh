#!/bin/bash
# Rank sort v3: the blocks-sort test, then the C4 step breakdown with the rank sort and
# with the radix sort (MIREC_BLOCKS_RADIX=1), then the C4 line.
set -u
export TMPDIR=/tmp
O=gpurun_out/rank
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_kernels.py -k "segment_sort_blocks or reduce2" tests/test_gpu_deepfm.py tests/test_gpu_mlp.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
for v in rank radix; do
  if [ $v = radix ]; then export MIREC_BLOCKS_RADIX=1; fi
  MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- \
    python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_$v.log 2>&1 || exit 7
  python tools/step_breakdown.py $O/tr_$v 32 $O/C4_$v.json > $O/C4_$v.txt || exit 8
  echo "== $v"; sed -n 4,6p $O/C4_$v.txt; grep -E "rank_|segsort|concat|mlp_" $O/C4_$v.txt | cut -c1-100
done
unset MIREC_BLOCKS_RADIX
timeout -k 10 300 python tools/bench_models.py --configs C4 --steps 64 --warmup 8 --no-cpu-baseline --out $O/c4.json > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 3; }
python -c "import json; r=json.load(open('$O/c4.json')); r=r[0] if isinstance(r,list) else r; print(json.dumps({k: r.get(k) for k in ('value','ms_per_step')}))"
echo done
