set -u
O=gpurun_out/r6fb; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "flush or deferred" > $O/tests.log 2>&1 || { echo FAIL tests; tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for v in main fb1 fb2; do
  if [ $v = main ]; then L=""; else L=recbole_amd/_lib/probe_$v.so; fi
  MIREC_LIB=${L:-recbole_amd/_lib/libmirec.so} timeout -k 10 200 python -u tools/probe_flush.py > $O/probe_$v.log 2>&1 || { echo FAIL probe $v; tail -20 $O/probe_$v.log; exit 3; }
  echo $v; tail -1 $O/probe_$v.log
done
