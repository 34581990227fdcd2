#!/bin/bash
# K35 timing probes (variants without the look-ahead / without the touched rows) and
# PMC passes of the K35 kernel (VALU / wave counters, FETCH_SIZE, WRITE_SIZE).
set -u
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
b() {  # tag, lib, args...
  local tag=$1 lib=$2; shift 2
  MIREC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --in-memory "$@" > $O/$tag 2>&1 || exit 4
  echo "$tag: $(grep -o '"value": [0-9.]*' $O/$tag | head -n1) $(grep -o '"kernels_us": {[^}]*}' $O/$tag | head -n1)"
}
L=recbole_amd/_lib
b full $L/libmirec.so --steps 64 --warmup 64
b noahead $L/alt/step_noahead.so --steps 64 --warmup 64
b notouched $L/alt/step_notouched.so --steps 64 --warmup 64
b k3k5 $L/libmirec.so --steps 64 --warmup 64 --no-fused-step
A="python bench.py --no-cpu-baseline --no-eval --in-memory --steps 64 --warmup 64"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $A > $O/trace.log 2>&1 || exit 5
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM --output-format csv -d $O/sq -o run -- $A > $O/sq.log 2>&1 || exit 6
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $A > $O/fetch.log 2>&1 || exit 7
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $A > $O/write.log 2>&1 || exit 8
echo done
