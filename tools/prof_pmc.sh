#!/bin/bash
# Kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes
# (MI355X_MICROARCH.md §rocprofv3 PMC slots: they don't fit one pass).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; exit 3; }
echo trace-ok; tail -1 $OUT/trace.log | cut -c1-300
if [ "${PMC:-1}" = "1" ]; then
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python bench.py $ARGS --no-eval > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; exit 3; }
echo fetch-ok
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python bench.py $ARGS --no-eval > $OUT/write.log 2>&1 || { echo "write rc=$?"; exit 3; }
echo write-ok
# VALU issue view of the VALU-bound K5 kernels (SQ block: 4 of its 8 slots)
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU \
  SQ_WAVE_CYCLES --output-format csv -d $OUT/valu -o run -- \
  python bench.py $ARGS --no-eval > $OUT/valu.log 2>&1 || { echo "valu rc=$?"; exit 3; }
echo valu-ok
fi
find $OUT -name "*.csv" | head -20
