set -u
O=gpurun_out/r6o; mkdir -p $O
export TMPDIR=/tmp
for c in C3 C4; do
  rm -rf $O/tr_$c
  MODELS_MARKERS=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$c -o run -- python tools/bench_models.py --configs $c --steps 8 --warmup 4 --no-cpu-baseline > $O/tr_$c.log 2>&1 || { echo FAIL $c; tail -20 $O/tr_$c.log; exit 3; }
  python tools/step_breakdown.py $O/tr_$c 8 $O/${c}_step.json > $O/${c}_step.txt || exit 4
  head -12 $O/${c}_step.txt
done
timeout -k 10 700 python tools/bench_models.py --configs C3,C4,C5 --out $O/models.json > $O/models.log 2>&1 || { echo FAIL models; tail -20 $O/models.log; exit 3; }
grep '^{' $O/models.log | cut -c1-300
