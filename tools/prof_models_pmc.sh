#!/bin/bash
# FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, MI355X_MICROARCH.md §HBM/rocprofv3)
# over tools/bench_models.py for one config -> gpurun_out/pmc_<cfg>/{fetch,write}
set -u
export TMPDIR=/tmp
CFG=${1:-C5}
OUT=gpurun_out/pmc_$CFG
mkdir -p $OUT
ARGS="--configs $CFG --steps ${STEPS:-16} --no-cpu-baseline ${EXTRA:-}"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
    python tools/bench_models.py $ARGS > $OUT/$c.log 2>&1 || { echo "$c rc=$?"; exit 3; }
  echo $c-ok
done
