set -u
O=gpurun_out/r6v; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_run.sh $O tests:tests/test_gpu_mlp.py:tests/test_gpu_deepfm.py || exit 3
for v in ks2 ks1; do
  lib=recbole_amd/_lib/libmirec.so; [ $v = ks1 ] && lib=recbole_amd/_lib/probe_ks1.so
  rm -rf $O/st_$v
  MIREC_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_$v -o run -- python tools/bench_models.py --configs C4 --no-cpu-baseline > $O/m_$v.log 2>&1 || { echo FAIL $v; tail -20 $O/m_$v.log; exit 3; }
  grep '^{' $O/m_$v.log | python -c 'import json,sys
d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d["k10_fwd"]["launch_us"])' $v
  python - $O/st_$v/run_kernel_stats.csv $v <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'mlp' in r['Name']: print(sys.argv[2], r['Name'][:40], r['Calls'], r['AverageNs'])
PY
done
