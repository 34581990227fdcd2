set -u
O=gpurun_out/r6c4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/probe_flush.py > $O/probe_flush.log 2>&1 || { echo FAIL probe; tail -20 $O/probe_flush.log; exit 3; }
tail -8 $O/probe_flush.log
c=C4
rm -rf $O/tr_$c
MODELS_MARKERS=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$c -o run -- python tools/bench_models.py --configs $c --steps 64 --warmup 8 --no-cpu-baseline > $O/tr_$c.log 2>&1 || { echo FAIL $c; tail -20 $O/tr_$c.log; exit 3; }
python tools/step_breakdown.py $O/tr_$c 64 $O/${c}_step.json > $O/${c}_step.txt || exit 4
head -24 $O/${c}_step.txt
