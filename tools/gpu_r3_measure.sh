#!/bin/bash
# Round-3 measurements: (1) the K3 gather at B=65,536 on C2 tables and on 2M-row tables
# past the LLC, with FETCH_SIZE / WRITE_SIZE passes; (2) kernel traces of the C3 and C4
# timed steps (trace markers) -> per-step breakdowns. Stops at the first failing step.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 120 python tools/gather_probe.py --out $O/gather.json > $O/gather.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/gfetch -o run -- \
  python tools/gather_probe.py > $O/gfetch.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/gwrite -o run -- \
  python tools/gather_probe.py > $O/gwrite.log 2>&1 || exit 5
python tools/gather_pmc.py $O/gfetch $O/gwrite $O/gather.json $O/gather_pmc.json > /dev/null || exit 6
echo gather-ok
for c in C4 C3; do
  MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$c -o run -- \
    python tools/bench_models.py --configs $c --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_$c.log 2>&1 || exit 7
  python tools/step_breakdown.py $O/tr_$c 32 $O/${c}_step.json > $O/${c}_step.txt || exit 8
  head -30 $O/${c}_step.txt
done
echo done
