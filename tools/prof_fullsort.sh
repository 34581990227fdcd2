#!/bin/bash
set -u
export TMPDIR=/tmp
OUT=gpurun_out/fsprof; mkdir -p $OUT
timeout -k 10 300 python tools/bench_fullsort.py > $OUT/plain.log 2>&1 || exit 3
cat $OUT/plain.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $OUT/sq -o run -- python tools/bench_fullsort.py --reps 1 > $OUT/sq.log 2>&1 || { echo sq fail; tail $OUT/sq.log; exit 3; }
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA --output-format csv -d $OUT/mfma -o run -- python tools/bench_fullsort.py --reps 1 > $OUT/mfma.log 2>&1 || { echo mfma fail; tail $OUT/mfma.log; exit 3; }
echo done
