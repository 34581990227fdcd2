set -o pipefail
for c in 32 48 64 96; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-eval --chunk $c > gpurun_out/fe.log 2>&1 || { tail -20 gpurun_out/fe.log; exit 3; }
  echo "default C=$c $(grep '^{' gpurun_out/fe.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_step"])')" | tee -a gpurun_out/fc.txt
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-eval --chunk $c --warmup 5 --steps 20 > gpurun_out/fe.log 2>&1 || { tail -20 gpurun_out/fe.log; exit 3; }
  echo "short C=$c $(grep '^{' gpurun_out/fe.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/fc.txt
done
