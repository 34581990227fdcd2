set -u
O=gpurun_out/r6s; mkdir -p $O; export TMPDIR=/tmp
for v in skipc skipca; do
  lib=""; lib=recbole_amd/_lib/probe_$v.so
  rm -rf $O/st_$v
  MIREC_LIB=${lib:-recbole_amd/_lib/libmirec.so} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_$v -o run -- python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-eval > $O/$v.log 2>&1 || { echo FAIL $v; tail -20 $O/$v.log; exit 3; }
  python - $O/st_$v/run_kernel_stats.csv $v <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'bpr_adam_step' in r['Name'] or 'flush_scan' in r['Name']: print(sys.argv[2], r['Name'][:40], r['Calls'], r['AverageNs'])
PY
done
