set -o pipefail
timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > gpurun_out/bs1.log 2>&1 && \
timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > gpurun_out/bs2.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_chain.py tests/test_gpu_e2e.py tests/test_gpu_shard.py tests/test_gpu_distributed.py tests/test_gpu_alias.py > gpurun_out/t.log 2>&1 && \
TRACE_OPTS=--hip-runtime-trace bash tools/trace_short.sh
