set -u
O=gpurun_out/r6fin; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/bench_models.py --configs C3,C4,C5 --out $O/models.json > $O/models.log 2>&1 || { echo FAIL models; tail -20 $O/models.log; exit 3; }
grep '^{' $O/models.log | cut -c1-200
timeout -k 10 600 python -u bench.py --warmup 5 --steps 20 > $O/full.log 2>&1 || { echo FAIL full; tail -20 $O/full.log; exit 3; }
grep '^{' $O/full.log | cut -c1-300
