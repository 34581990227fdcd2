#!/bin/bash
# C4 / C3 with the dominant-kernel rooflines (live HIP events), then the K8 backward's
# FETCH / WRITE passes (a short C4 run under rocprofv3 --pmc). Stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3mod
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_deepfm.py tests/test_gpu_deferred.py tests/test_gpu_graph_step.py tests/test_gpu_configs.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 300 python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline --out $O/c4.json > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 3; }
python -c "import json; r=json.load(open('$O/c4.json')); r=r[0] if isinstance(r,list) else r; print(json.dumps({k: r.get(k) for k in ('value','ms_per_step','roofline','k8_fwd')})[:1500])"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4fetch -o run -- \
  python tools/bench_models.py --configs C4 --steps 4 --warmup 2 --no-cpu-baseline > $O/c4fetch.log 2>&1 || { tail -5 $O/c4fetch.log; exit 4; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c4write -o run -- \
  python tools/bench_models.py --configs C4 --steps 4 --warmup 2 --no-cpu-baseline > $O/c4write.log 2>&1 || { tail -5 $O/c4write.log; exit 5; }
python tools/models_pmc.py $O/c4fetch $O/c4write $O/models_pmc.json ctx_fm_bwd_kernel ctx_fm_fwd_kernel || exit 6
timeout -k 10 400 python tools/bench_models.py --configs C3 --steps 16 --warmup 4 --no-cpu-baseline --out $O/c3.json > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 7; }
python -c "import json; r=json.load(open('$O/c3.json')); r=r[0] if isinstance(r,list) else r; print(json.dumps({k: r.get(k) for k in ('value','ms_per_step','roofline')})[:1500])"
echo done
