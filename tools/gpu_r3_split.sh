#!/bin/bash
# K35 with split rows: parity tests, bitwise chains, A/B benches vs the K3 + K5
# launches, and the stamp probe. Stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_step.py tests/test_gpu_e2e.py tests/test_gpu_chain.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
b() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --in-memory "$@" > $O/$tag 2>&1 || exit 4
  echo "$tag: $(grep -o '"value": [0-9.]*' $O/$tag | head -n1) $(grep -o '"kernels_us": {[^}]*}' $O/$tag | head -n1)"
}
b k35_short --warmup 5 --steps 20; b k3k5_short --warmup 5 --steps 20 --no-fused-step
b k35_default; b k3k5_default --no-fused-step
b k35_short2 --warmup 5 --steps 20; b k35_default2
MIREC_LIB=recbole_amd/_lib/alt/step_stamps.so timeout -k 10 300 python tools/probe_step_stamps.py --warmup 96 --steps 12 > $O/stamps.jsonl 2> $O/stamps.err || { tail -5 $O/stamps.err; exit 6; }
python - <<'PY'
import json
for l in open('gpurun_out/r3h/stamps.jsonl'):
    r = json.loads(l)
    print(r['batch'], r['makespan_us'], {k: r[k]['end'] for k in ('share_users','share_items','ahead_users','ahead_items','touched_users','touched_items') if r.get(k)})
PY
echo done
