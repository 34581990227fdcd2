set -u
O=gpurun_out/r6i; mkdir -p $O
export TMPDIR=/tmp
rm -rf $O/trace
BENCH_MARKERS=1 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --dp-mode sharded --exchange ipc --batch-rows 16384 --warmup 5 --steps 40 --chunk 16 --no-cpu-baseline --no-eval > $O/b4096.log 2>&1 || { echo FAIL; tail -20 $O/b4096.log; exit 3; }
python tools/check_timed_window.py $O/trace $O/tw.json > $O/tw.txt || exit 4
grep '^{' $O/b4096.log | python -c 'import json,sys
d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("kernels_us"))'
