set -u
O=gpurun_out/r6apmc; mkdir -p $O
export TMPDIR=/tmp
rm -rf $O/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/pmc -o run -- python tools/probe_attn.py > $O/pmc.log 2>&1 || { echo FAIL pmc; tail -20 $O/pmc.log; exit 3; }
tail -1 $O/pmc.log
