set -o pipefail
timeout -k 10 1100 python tools/bench_models.py --out gpurun_out/r02_models.json > gpurun_out/models.log 2>&1 || { tail -30 gpurun_out/models.log; exit 3; }
grep '^{' gpurun_out/models.log | cut -c1-200
