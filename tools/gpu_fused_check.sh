#!/bin/bash
# Fused-path changes: fused/sharded/e2e/chain tests, the driver's short bench line
# under a marked kernel trace (timed-window timeline), and the default bench line.
set -u
export TMPDIR=/tmp
O=gpurun_out/fused
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_e2e.py tests/test_gpu_chain.py tests/test_gpu_shard.py tests/test_gpu_distributed.py \
  tests/test_gpu_kernels.py ${EXTRA_TESTS:-} > $O/t.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/t.log; exit 3; }
tail -2 $O/t.log
timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $O/bench_short.log 2>&1 || { echo bench fail; tail $O/bench_short.log; exit 3; }
tail -1 $O/bench_short.log | cut -c1-200
bash tools/trace_short.sh || exit 3
timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval > $O/bench_default.log 2>&1 || { echo bench fail; tail $O/bench_default.log; exit 3; }
tail -1 $O/bench_default.log | cut -c1-200
