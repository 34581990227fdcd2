set -u
O=gpurun_out/r6sk; mkdir -p $O
export TMPDIR=/tmp
for v in sk1 sk8; do
  MIREC_LIB=recbole_amd/_lib/probe_$v.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_deferred.py tests/test_gpu_kernels.py -k "adam or deferred or flush or replay" > $O/tests_$v.log 2>&1 || { echo FAIL tests $v; tail -30 $O/tests_$v.log; exit 3; }
  echo $v; tail -1 $O/tests_$v.log
done
for v in main sk1 sk8; do
  if [ $v = main ]; then L=recbole_amd/_lib/libmirec.so; else L=recbole_amd/_lib/probe_$v.so; fi
  MIREC_LIB=$L timeout -k 10 300 python tools/bench_models.py --configs C3 --no-cpu-baseline > $O/c3_$v.log 2>&1 || { echo FAIL $v; tail -20 $O/c3_$v.log; exit 3; }
  echo $v; grep '^{' $O/c3_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])"
done
rm -rf $O/st
MIREC_LIB=recbole_amd/_lib/probe_sk1.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o run -- python tools/bench_models.py --configs C3 --no-cpu-baseline > $O/st.log 2>&1 || { echo FAIL st; exit 3; }
echo done
