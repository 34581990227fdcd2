set -u
O=gpurun_out/r6ap; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu tests/test_gpu_attention.py > $O/tests.log 2>&1 || { echo FAIL tests; tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
MIREC_LIB=recbole_amd/_lib/probe_atfast.so timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu tests/test_gpu_attention.py > $O/tests_fast.log 2>&1 || { echo FAIL fast tests; tail -30 $O/tests_fast.log; }
tail -1 $O/tests_fast.log
timeout -k 10 120 python -u tools/probe_attn.py > $O/probe_main.log 2>&1 || { echo FAIL probe; tail -20 $O/probe_main.log; exit 3; }
echo main; tail -1 $O/probe_main.log
MIREC_LIB=recbole_amd/_lib/probe_atfast.so timeout -k 10 120 python -u tools/probe_attn.py > $O/probe_fast.log 2>&1 || { echo FAIL probe fast; tail -20 $O/probe_fast.log; exit 3; }
echo fast; tail -1 $O/probe_fast.log
