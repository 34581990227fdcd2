set -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/c4prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o run -- python tools/bench_models.py --configs C4 --steps 100 --warmup 8 --no-cpu-baseline > gpurun_out/c4p.log 2>&1 || { tail -20 gpurun_out/c4p.log; exit 3; }
