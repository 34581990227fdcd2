"""Probe: can an RCCL all_gather_into_tensor be captured in a HIP graph here?
(world size 1, in-place, like FusedBPRTrainStep._exchange). Prints one line."""
import os

import torch
import torch.distributed as tdist

os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
os.environ.setdefault('MASTER_PORT', '29611')
torch.cuda.set_device(0)
tdist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
x = torch.arange(1024, dtype=torch.float32, device='cuda')
tdist.all_gather_into_tensor(x, x[:1024])          # warm the communicator
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
try:
    with torch.cuda.graph(g, stream=s):
        x.mul_(2)
        tdist.all_gather_into_tensor(x, x[:1024])
        x.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    x.fill_(1)
    g.replay()
    torch.cuda.synchronize()
    print('capture ok', float(x[0].item()) == 3.0)
except Exception as e:  # noqa: BLE001
    print('capture failed:', type(e).__name__, str(e)[:300])
tdist.destroy_process_group()
