#!/bin/bash
# Model configurations C3-C5 with CPU baselines (-> models.json), then kernel traces of
# the C4 and C3 timed steps (trace markers) -> per-step breakdowns. Stops at the first
# failing step.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3m2
mkdir -p $O
timeout -k 10 600 python tools/bench_models.py --out $O/models.json > $O/models.log 2>&1
rc=$?; echo "models rc=$rc"; grep '^{' $O/models.log | cut -c1-300; [ $rc -eq 0 ] || exit 3
for c in ${TRACE_CONFIGS:-C4 C3}; do
  MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$c -o run -- \
    python tools/bench_models.py --configs $c --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_$c.log 2>&1 || exit 7
  python tools/step_breakdown.py $O/tr_$c 32 $O/${c}_step.json > $O/${c}_step.txt || exit 8
  head -40 $O/${c}_step.txt
done
echo done
