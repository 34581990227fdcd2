"""Probe: the row-sharded step on a 1-rank nccl (RCCL) group, step by step with
progress lines (eager first, then captured chunk graphs)."""
import os
import pathlib
import sys
import tempfile
import time

import torch
import torch.distributed as tdist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=os.environ.get('PORT', '29931'), RANK='0',
                  WORLD_SIZE='1')
t0 = time.time()
say = lambda m: print(f'[{time.time() - t0:6.1f}s] {m}', flush=True)
torch.cuda.set_device(0)
tdist.init_process_group('nccl', device_id=torch.device('cuda', 0))
say('init ok')
x = torch.ones(4, device='cuda')
y = torch.empty(4, device='cuda')
tdist.all_to_all_single(y, x)
torch.cuda.synchronize()
say(f'eager all_to_all ok {y.tolist()}')
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.graph(g, stream=s):
    tdist.all_to_all_single(y, x * 2)
torch.cuda.current_stream().wait_stream(s)
say('captured all_to_all')
g.replay()
torch.cuda.synchronize()
say(f'replayed all_to_all {y.tolist()}')
from test_gpu_e2e import _pipeline
from recbole_amd.trainer.fused import ShardedBPRTrainStep
from recbole_amd.trainer.optim import FusedAdam
tmp = tempfile.mkdtemp()
for graph in (False, True):
    config, train, valid, test, model = _pipeline(pathlib.Path(tmp), epochs=2)
    opt = FusedAdam(model.parameters(), lr=config['learning_rate'])
    step = ShardedBPRTrainStep(model, opt, train, chunk=4, dist=tdist.group.WORLD,
                               use_graph=graph)
    say(f'step built graph={graph}')
    nb = step.begin_epoch()
    say(f'begin_epoch ok ({nb} batches)')
    step.run_batches(0, nb)
    torch.cuda.synchronize()
    say('batches ok')
    losses = step.end_epoch()
    say(f'epoch ok loss0={losses[0]:.6f}')
    step.close()
    del step
say('graphs released')
del g
import gc
gc.collect()
torch.cuda.synchronize()
say('destroying')
tdist.destroy_process_group()
say('done')
