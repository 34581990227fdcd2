set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_chain.py tests/test_gpu_popularity.py tests/test_gpu_e2e.py tests/test_gpu_alias.py > gpurun_out/wt.log 2>&1 || { tail -30 gpurun_out/wt.log; exit 3; }
tail -2 gpurun_out/wt.log
for k in 1 2 3; do
timeout -k 10 200 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > gpurun_out/bs.log 2>&1 || exit 4
grep '^{' gpurun_out/bs.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("short", d["value"])'
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-eval > gpurun_out/bs.log 2>&1 || exit 5
grep '^{' gpurun_out/bs.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("default", d["value"])'
timeout -k 10 300 python tools/event_timeline.py --reps 2 > gpurun_out/evt.log 2>&1
