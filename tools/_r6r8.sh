set -u
O=gpurun_out/r6r8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 170 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_deepfm.py -k "sort or block or deepfm or DeepFM" > $O/tests.log 2>&1 || { echo FAIL tests; tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for v in main r8512; do
  if [ $v = main ]; then L=recbole_amd/_lib/libmirec.so; else L=recbole_amd/_lib/probe_$v.so; fi
  MIREC_LIB=$L timeout -k 10 400 python tools/bench_models.py --configs C4 --no-cpu-baseline > $O/c4_$v.log 2>&1 || { echo FAIL $v; tail -20 $O/c4_$v.log; exit 3; }
  echo $v; grep '^{' $O/c4_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['k2_grouping']['launch_us'])"
done
