#!/bin/bash
# K2 LDS sort: workgroup-size variants (tools/build_variant.sh) — probe latency and the
# driver-window bench line of each. Stops at the first failing GPU step.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/sortv
for v in ${VARIANTS:-d5 d6 default}; do
  if [ $v = default ]; then L=recbole_amd/_lib/libmirec.so; else L=recbole_amd/_lib/alt/$v.so; fi
  MIREC_LIB=$L timeout -k 10 120 python tools/probe_segsort.py > gpurun_out/sortv/$v.probe 2>&1 || exit 3
  MIREC_LIB=$L timeout -k 10 200 python bench.py --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/sortv/$v.bench 2>&1 || exit 4
  echo "$v: $(grep -o '"value": [0-9.]*' gpurun_out/sortv/$v.bench | head -n1)"
done
