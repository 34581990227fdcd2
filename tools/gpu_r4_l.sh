#!/bin/bash
# Round-4: K3 gather variants (register budget, non-temporal gradient stores).
set -u
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 120 python tools/gather_probe.py > $O/base.log 2>&1 || exit 3
grep big $O/base.log | cut -c1-220
for v in k3nt k3nt6; do
  MIREC_LIB=recbole_amd/_lib/alt/$v.so timeout -k 10 120 python tools/gather_probe.py > $O/$v.log 2>&1 || exit 4
  echo $v; grep big $O/$v.log | cut -c1-220
done
