set -u
O=gpurun_out/r6t; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_run.sh $O tests:tests/test_gpu_linear_finish.py:tests/test_gpu_sasrec.py || exit 3
rm -rf $O/tr_C3
MODELS_MARKERS=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_C3 -o run -- python tools/bench_models.py --configs C3 --steps 8 --warmup 4 --no-cpu-baseline > $O/tr_C3.log 2>&1 || { echo FAIL trace; tail -20 $O/tr_C3.log; exit 3; }
python tools/step_breakdown.py $O/tr_C3 8 $O/C3_step.json > /dev/null || exit 4
python -c "
import json;d=json.load(open('$O/C3_step.json'));print('wall/step',d['wall_us_per_step'],'launches',d['launches_per_step'])
[print(x['kernel'][:50],x['launches_per_step'],x['avg_us'],x['us_per_step']) for x in d['kernels'] if 'finish' in x['kernel']]"
timeout -k 10 500 python tools/bench_models.py --configs C3 --no-cpu-baseline > $O/m.log 2>&1 || { echo FAIL models; exit 3; }
grep '^{' $O/m.log | cut -c1-200
