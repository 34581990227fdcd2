set -u
export TMPDIR=/tmp
O=gpurun_out/walk
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "sampler or walk or used" > $O/t.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/t.log; exit 3; }
tail -2 $O/t.log
timeout -k 10 300 python tools/bench_walk.py --keys 512 4096 > $O/walk.log 2>&1 || { echo walk fail; tail $O/walk.log; exit 3; }
grep -v amdgpu $O/walk.log | tail -3
timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $O/bench_short.log 2>&1 || { echo bench fail; tail $O/bench_short.log; exit 3; }
tail -1 $O/bench_short.log | cut -c1-200
