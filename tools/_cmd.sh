set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_deepfm.py tests/test_gpu_graph_step.py tests/test_gpu_configs.py tests/test_gpu_dp.py > gpurun_out/st.log 2>&1 || { tail -40 gpurun_out/st.log; exit 3; }
tail -2 gpurun_out/st.log
timeout -k 10 400 python tools/bench_models.py --configs C4 --no-cpu-baseline > gpurun_out/c4.log 2>&1 || { tail -20 gpurun_out/c4.log; exit 4; }
grep '^{' gpurun_out/c4.log | cut -c1-200
