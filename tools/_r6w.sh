set -u
O=gpurun_out/r6w; mkdir -p $O
bash tools/gpu_run.sh $O tests:tests/test_gpu_kernels.py:tests/test_gpu_configs.py:tests/test_gpu_case_study.py || exit 3
for d in 128 64 256; do
  for v in new old; do
    lib=recbole_amd/_lib/libmirec.so; [ $v = old ] && lib=recbole_amd/_lib/probe_fsold.so
    MIREC_LIB=$lib timeout -k 10 300 python tools/bench_fullsort.py --d $d --reps 3 > $O/fs_${d}_$v.log 2>&1 || { echo FAIL $d $v; tail $O/fs_${d}_$v.log; exit 3; }
    echo "d=$d $v: $(tail -2 $O/fs_${d}_$v.log | tr '\n' ' ')"
  done
done
