#!/bin/bash
# K10 v4 + compacted flush: their tests and the C2 parity chain, the C4 step breakdown,
# then the C2 lines (driver window twice, default once) and the driver-window timeline.
set -u
export TMPDIR=/tmp
O=gpurun_out/v4
mkdir -p $O
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_mlp.py tests/test_gpu_deepfm.py tests/test_gpu_kernels.py \
  tests/test_gpu_step.py tests/test_gpu_e2e.py tests/test_gpu_chain.py tests/test_gpu_deferred.py tests/test_gpu_graph_step.py > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit 10
MODELS_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_C4 -o run -- \
  python tools/bench_models.py --configs C4 --steps 32 --warmup 8 --no-cpu-baseline > $O/tr_C4.log 2>&1 || exit 7
python tools/step_breakdown.py $O/tr_C4 32 $O/C4_step.json > $O/C4_step.txt || exit 8
head -12 $O/C4_step.txt | cut -c1-120
for rep in 1 2; do
  timeout -k 10 200 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $O/short.$rep.log 2>&1 || { tail -5 $O/short.$rep.log; exit 3; }
  grep '^{' $O/short.$rep.log | cut -c1-200
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval > $O/default.log 2>&1 || { tail -5 $O/default.log; exit 4; }
grep '^{' $O/default.log | cut -c1-200
python -c "import json; d=json.loads([l for l in open('$O/default.log') if l.startswith('{')][0]); print(d['kernels_us'])"
bash tools/trace_short.sh || exit 5
tail -8 gpurun_out/prof_short/tw.txt
echo done
