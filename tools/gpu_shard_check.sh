#!/bin/bash
# Sharded-path GPU session: tests, then the bench on one rank through the sharded
# protocol over a real 1-rank RCCL group (torchrun), then the short bench line.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_shard.py > $OUT/shard.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/shard.log; exit 3; }
tail -3 $OUT/shard.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --dp-mode sharded --warmup 64 --steps 256 --no-cpu-baseline --no-eval \
  > $OUT/bench_shard1.log 2>&1 || { echo "bench shard rc=$?"; tail -20 $OUT/bench_shard1.log; exit 3; }
tail -1 $OUT/bench_shard1.log | cut -c1-600
timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $OUT/bench_short.log 2>&1 || { echo "short rc=$?"; exit 3; }
tail -1 $OUT/bench_short.log | cut -c1-300
