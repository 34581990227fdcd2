#!/bin/bash
# Round-3 first GPU session: shard tests (plan status / overflow re-plan), K2 block-scan
# variant vs default (probe + driver-window bench), the untraced event timeline of the
# driver window. Stops at the first failing GPU step.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r3a/shard_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3a/shard_tests.log; [ $rc -le 1 ] || exit $rc
for v in k2bs default; do
  if [ $v = default ]; then L=recbole_amd/_lib/libmirec.so; else L=recbole_amd/_lib/alt/$v.so; fi
  MIREC_LIB=$L timeout -k 10 120 python tools/probe_segsort.py > gpurun_out/r3a/$v.probe 2>&1 || exit 3
  for rep in 1 2; do
    MIREC_LIB=$L timeout -k 10 200 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > gpurun_out/r3a/$v.bench$rep 2>&1 || exit 4
    echo "$v/$rep: $(grep -o '"value": [0-9.]*' gpurun_out/r3a/$v.bench$rep | head -n1)"
  done
done
timeout -k 10 200 python tools/event_timeline.py > gpurun_out/r3a/timeline.txt 2>&1 || exit 5
echo done
