#!/bin/bash
# Driver-window fill: short (--warmup 5 --steps 20) benches with ramp variants and the
# flush geometry variants; one marked trace of the default short run.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3fill
mkdir -p $O
b() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --in-memory --warmup 5 --steps 20 "$@" > $O/$tag 2>&1 || { tail -5 $O/$tag; exit 4; }
  echo "$tag: $(grep -o '"value": [0-9.]*' $O/$tag | head -n1) $(grep -o '"kernels_us": {[^}]*}' $O/$tag | head -n1)"
}
b base; b base2
b r1 --ramp 1,2,4,8,16,32; b r2 --ramp 2,4,8,16,32; b r1b --ramp 1,3,8,16,32
MIREC_LIB=recbole_amd/_lib/alt/flush256.so b f256
MIREC_LIB=recbole_amd/_lib/alt/flush1024.so b f1024
BENCH_MARKERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- \
  python bench.py --no-cpu-baseline --no-eval --in-memory --warmup 5 --steps 20 > $O/trace_bench.log 2>&1 || exit 5
python tools/check_timed_window.py $O/tr > $O/window.txt 2>&1 || true
echo done
