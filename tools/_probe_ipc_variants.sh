mkdir -p gpurun_out/r6f
run() { # tag variant [env]
  tag=$1; v=$2; shift 2
  env "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 500)) tools/probe_ipc_adam.py $v --warmup 5 --steps 20 --no-cpu-baseline --no-eval > gpurun_out/r6f/$tag.log 2>&1 || { echo FAIL $tag; tail -20 gpurun_out/r6f/$tag.log; exit 3; }
  grep '^{' gpurun_out/r6f/$tag.log | python -c 'import json,sys
d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d.get("kernels_us"))' $tag
}
run ipc_noarrive ipc MIREC_LIB=recbole_amd/_lib/probe_noarrive.so && run nopush_noarrive nopush MIREC_LIB=recbole_amd/_lib/probe_noarrive.so
