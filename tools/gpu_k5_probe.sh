set -u
export TMPDIR=/tmp
O=gpurun_out/k5
mkdir -p $O
timeout -k 10 120 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
timeout -k 10 200 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "chunk_finish" > $O/t.log 2>&1 || { echo "test fail"; tail -20 $O/t.log; exit 3; }
timeout -k 10 200 python tools/probe_adam.py --gap 64 > $O/steady.log 2>&1 && timeout -k 10 200 python tools/probe_adam.py --gap 20 --state fresh > $O/fresh.log 2>&1 || { echo probe fail; exit 3; }
cat $O/steady.log $O/fresh.log | grep -v amdgpu.ids
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/pmc1 -o run -- python tools/probe_adam.py --gap 64 --reps 3 > $O/pmc1.log 2>&1 || { echo pmc1 fail; tail $O/pmc1.log; exit 3; }
timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $O/bench_short.log 2>&1 || { echo bench fail; tail $O/bench_short.log; exit 3; }
tail -1 $O/bench_short.log | cut -c1-300
