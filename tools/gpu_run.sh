#!/bin/bash
# The one GPU-session runner (replaces the per-session gpu_r3_* / gpu_r4_* scripts).
#
#   bash tools/gpu_run.sh OUTDIR TASK [TASK ...]
#
# Tasks run in order, each under its own time limit; any failure ends the script (a
# crash / fault / timeout must not be followed by more GPU work). Tasks:
#   smoke            __graft_entry__.smoke()
#   tests[:ARGS]     pytest -m gpu (ARGS: test files / -k, ':'-separated words -> spaces)
#   drv[:N]          N driver-window bench lines (--warmup 5 --steps 20), default 3
#   def[:N]          N default-window bench lines (64 + 256 steps), default 1
#   full             one driver-window bench with eval + gather + CPU baseline (BENCH line)
#   trace            kernel + HIP runtime trace of the driver window (tools/trace_short.sh)
#   stats            rocprofv3 --kernel-trace --stats of the driver window
#   pmc              FETCH_SIZE / WRITE_SIZE / VALU passes of the driver window (separate runs)
#   models[:CFGS]    tools/bench_models.py (CFGS comma list, default C3,C4,C5)
#   mstats:CFG       kernel trace + stats of bench_models for one config
#   mpmc:CFG         FETCH_SIZE / WRITE_SIZE passes of bench_models for one config
#   py:SCRIPT[:ARGS] python SCRIPT ARGS (a probe under tools/)
# Env: BENCH_ARGS (extra bench.py flags), MIREC_LIB (alternative library build).
set -u
export TMPDIR=/tmp
O=${1:?outdir}; shift
mkdir -p "$O"
S="$O/summary.txt"
: > "$S"
say() { echo "$*" | tee -a "$S"; }
run() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    say "FAIL $name rc=$rc"
    tail -30 "$O/$name.log" | cut -c1-400 | tee -a "$S"
    exit 3
  fi
}
line() {  # the bench JSON line's headline fields
  grep '^{' "$1" | python -c 'import json,sys
d=json.loads(sys.stdin.read()); r=d.get("roofline",{})
print(d["value"], d["ms_per_step"], d.get("kernels_us"), "frac", r.get("frac"), r.get("bound"))'
}
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread"
for task in "$@"; do
  name=${task%%:*}
  arg=""
  [ "$name" != "$task" ] && arg=${task#*:}
  case $name in
    smoke)
      run smoke 300 python __graft_entry__.py smoke
      say "smoke: $(tail -1 $O/smoke.log | cut -c1-300)";;
    tests)
      run tests 1100 $PT -m gpu ${arg//:/ }
      say "tests: $(tail -1 $O/tests.log)";;
    drv)
      for i in $(seq 1 ${arg:-3}); do
        run drv_$i 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval ${BENCH_ARGS:-}
        say "drv $i: $(line $O/drv_$i.log)"
      done;;
    def)
      for i in $(seq 1 ${arg:-1}); do
        run def_$i 400 python bench.py --no-cpu-baseline --no-eval ${BENCH_ARGS:-}
        say "def $i: $(line $O/def_$i.log)"
      done;;
    full)
      run full 600 python bench.py --warmup 5 --steps 20 ${BENCH_ARGS:-}
      say "full: $(line $O/full.log)";;
    trace)
      rm -rf "$O/trace"; mkdir -p "$O/trace"
      BENCH_MARKERS=1 run trace 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv \
        -d "$O/trace" -o run -- python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval \
        ${BENCH_ARGS:-}
      python tools/check_timed_window.py "$O/trace" "$O/timed_window.json" > "$O/tw.txt" || exit 4
      say "trace: $(head -3 $O/tw.txt | tr -d '\n')";;
    stats)
      rm -rf "$O/stats"
      run stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- \
        python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval ${BENCH_ARGS:-}
      say "stats: $(line $O/stats.log)";;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"; do
        tag=${c%% *}
        rm -rf "$O/pmc_$tag"
        run pmc_$tag 300 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$tag" -o run -- \
          python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval ${BENCH_ARGS:-}
        say "pmc $tag ok"
      done;;
    models)
      run models 700 python tools/bench_models.py --configs ${arg:-C3,C4,C5} --no-cpu-baseline \
        --out "$O/models.json"
      say "models: $(grep '^{' $O/models.log | cut -c1-200 | tr '\n' ' ')";;
    mstats)
      rm -rf "$O/mstats_$arg"
      run mstats_$arg 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/mstats_$arg" \
        -o run -- python tools/bench_models.py --configs $arg --no-cpu-baseline
      say "mstats $arg ok";;
    mpmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        rm -rf "$O/mpmc_${arg}_$c"
        run mpmc_${arg}_$c 500 rocprofv3 --pmc $c --output-format csv -d "$O/mpmc_${arg}_$c" -o run -- \
          python tools/bench_models.py --configs $arg --steps 16 --no-cpu-baseline
        say "mpmc $arg $c ok"
      done;;
    py)
      script=${arg%%:*}
      rest=""
      [ "$script" != "$arg" ] && rest=${arg#*:}
      PYN=$(( ${PYN:-0} + 1 ))
      log=py_$(basename $script .py)_$PYN
      run $log 600 python -u $script ${rest//:/ }
      say "py $script: $(tail -3 $O/$log.log | tr '\n' ' ' | cut -c1-400)";;
    *)
      say "unknown task $task"; exit 2;;
  esac
done
say "done"
