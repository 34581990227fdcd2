set -u
O=gpurun_out/r6h; mkdir -p $O
export TMPDIR=/tmp
for ex in ipc rccl; do
  rm -rf $O/trace_$ex
  BENCH_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace_$ex -o run -- python bench.py --dp-mode sharded --exchange $ex --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $O/trace_$ex.log 2>&1 || { echo FAIL $ex; tail -20 $O/trace_$ex.log; exit 3; }
  python tools/check_timed_window.py $O/trace_$ex $O/tw_$ex.json > $O/tw_$ex.txt || exit 4
  head -30 $O/tw_$ex.txt
done
