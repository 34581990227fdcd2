set -u
O=gpurun_out/r6p; mkdir -p $O
for ex in rccl ipc; do
  MIREC_BENCH_ONE_DEVICE=1 timeout -k 10 500 python bench.py --gpus 2 --exchange $ex --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $O/n2_$ex.log 2>&1 || { echo FAIL $ex; tail -30 $O/n2_$ex.log; exit 3; }
  grep '^{' $O/n2_$ex.log | python -c 'import json,sys
d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d["n_gpus"], d["config"]["parallelism"], d.get("kernels_us"))' $ex
done
timeout -k 10 300 python tools/event_timeline.py --reps 3 > $O/event_timeline.log 2>&1 || { echo FAIL timeline; tail -20 $O/event_timeline.log; exit 3; }
grep -A12 "^rep 2" $O/event_timeline.log
