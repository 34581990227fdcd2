#!/bin/bash
# K5 changes: Adam kernel tests, deferred-schedule model tests, fused e2e, probes, bench lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/k5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_deferred.py tests/test_gpu_e2e.py tests/test_gpu_chain.py \
  > $O/t.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/t.log; exit 3; }
tail -2 $O/t.log
timeout -k 10 200 python tools/probe_adam.py --gap 64 > $O/steady.log 2>&1 && \
  timeout -k 10 200 python tools/probe_adam.py --gap 20 --state fresh > $O/fresh.log 2>&1 || { echo probe fail; exit 3; }
cat $O/steady.log $O/fresh.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $O/bench_short.log 2>&1 || { echo bench fail; tail $O/bench_short.log; exit 3; }
tail -1 $O/bench_short.log | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval > $O/bench_default.log 2>&1 || { echo bench fail; tail $O/bench_default.log; exit 3; }
tail -1 $O/bench_default.log | cut -c1-200
