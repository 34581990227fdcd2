#!/bin/bash
# Flush kernel geometry A/B (rows per block 1 / 4 / 16): short (driver) and default windows.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3fv
mkdir -p $O
b() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --in-memory "$@" > $O/$tag 2>&1 || { tail -5 $O/$tag; exit 4; }
  echo "$tag: $(grep -o '"value": [0-9.]*' $O/$tag | head -n1) $(grep -o '"kernels_us": {[^}]*}' $O/$tag | head -n1)"
}
b short64 --warmup 5 --steps 20
MIREC_LIB=recbole_amd/_lib/alt/flush256.so b short256 --warmup 5 --steps 20
MIREC_LIB=recbole_amd/_lib/alt/flush1024.so b short1024 --warmup 5 --steps 20
b default64
MIREC_LIB=recbole_amd/_lib/alt/flush256.so b default256
MIREC_LIB=recbole_amd/_lib/alt/flush1024.so b default1024
echo done
