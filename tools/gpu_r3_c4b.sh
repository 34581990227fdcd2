#!/bin/bash
# C4 after the fixup owner list and the unrolled FM reduce: parity tests (kernels,
# DeepFM, deferred, SASRec, 2-rank DP), C4 bench.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3c4b
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 400 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_kernels.py -k "segment or scatter" > $O/tk.log 2>&1 || { tail -20 $O/tk.log; exit 3; }
tail -1 $O/tk.log
timeout -k 10 900 $T tests/test_gpu_deferred.py tests/test_gpu_deepfm.py tests/test_gpu_sasrec.py tests/test_gpu_dp.py tests/test_gpu_graph_step.py > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 4; }
tail -1 $O/t.log
timeout -k 10 300 python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline --out $O/c4.json > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 5; }
python -c "import json; r=json.load(open('$O/c4.json')); r=r[0] if isinstance(r,list) else r; print(r['value'], r['ms_per_step'], r['k8_fwd'])"
echo done
