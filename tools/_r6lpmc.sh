set -u
O=gpurun_out/r6lpmc; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python tools/probe_linear.py > $O/probe.log 2>&1 || { echo FAIL probe; tail -20 $O/probe.log; exit 3; }
tail -1 $O/probe.log
rm -rf $O/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/pmc -o run -- python tools/probe_linear.py > $O/pmc.log 2>&1 || { echo FAIL pmc; tail -20 $O/pmc.log; exit 3; }
echo pmc ok
