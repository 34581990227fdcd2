set -o pipefail
for r in 4,8,16,32 2,4,8,16,32 1,2,4,8,16,32 2,6,12,24,48 3,6,12,24; do
  for k in 1 2; do
    timeout -k 10 200 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval --ramp $r > gpurun_out/ramp.log 2>&1 || exit 3
    echo "$r $(grep '^{' gpurun_out/ramp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["chunk_plan_timed"])')" | tee -a gpurun_out/ramps.txt
  done
done
