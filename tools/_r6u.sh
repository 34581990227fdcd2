set -u
O=gpurun_out/r6u; mkdir -p $O; export TMPDIR=/tmp
rm -rf $O/pmc
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/pmc -o run -- python tools/bench_models.py --configs C4 --steps 8 --warmup 4 --no-cpu-baseline > $O/pmc.log 2>&1 || { echo FAIL pmc; tail -20 $O/pmc.log; exit 3; }
python - $O/pmc <<'PY'
import csv,glob,sys,collections
f=glob.glob(sys.argv[1]+'/**/*counter_collection.csv',recursive=True)[0]
agg=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'].split('(')[0][:50]
    if 'mlp' not in k and 'radix8' not in k: continue
    agg[k][r['Counter_Name']]+=float(r['Counter_Value']); cnt[k].add(r['Dispatch_Id'])
for k,v in agg.items():
    n=len(cnt[k]); print(k, n, {c: round(x/n) for c,x in v.items()})
PY
