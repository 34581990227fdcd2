#!/bin/bash
# The sharded C2 step at one rank under torchrun, both exchanges (rccl / ipc): per-launch
# HIP-event times of gather / push, K3 (bpr), the owner Adam, and the step rate.
#   bash tools/ipc_probe.sh OUTDIR
set -u
O=${1:?outdir}; mkdir -p "$O"
for ex in rccl ipc; do
  MIREC_EXCHANGE=$ex timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
    --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 1 \
    --dp-mode sharded --warmup 5 --steps 20 --no-cpu-baseline --no-eval > "$O/sharded_$ex.log" 2>&1 || {
      echo "FAIL sharded $ex"; tail -20 "$O/sharded_$ex.log"; exit 3; }
  grep '^{' "$O/sharded_$ex.log" | python -c 'import json,sys
d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d.get("kernels_us"))' $ex
done
