set -o pipefail
for f in 64 256 1024 100000; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-eval --flush-every $f > gpurun_out/fe.log 2>&1 || { tail -20 gpurun_out/fe.log; exit 3; }
  echo "default $f $(grep '^{' gpurun_out/fe.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_step"])')" | tee -a gpurun_out/fe.txt
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-eval --flush-every $f --warmup 5 --steps 20 > gpurun_out/fe.log 2>&1 || { tail -20 gpurun_out/fe.log; exit 3; }
  echo "short $f $(grep '^{' gpurun_out/fe.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/fe.txt
done
