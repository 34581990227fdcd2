"""Data-parallel fused step on the GPU: 2 ranks (gloo, both on cuda:0) each with
half of every global batch must end bit-identical to ONE process running the
global batch (weights, Adam state, per-batch losses), over epochs with a ragged
last batch and partial chunks. The RCCL backend differs only in the collective
(an in-place all_gather_into_tensor); the 8-GPU run is the driver's."""
import os

import numpy as np
import pytest
import torch
from conftest import free_port
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

EPOCHS, CHUNK = 2, 4


def _pipeline(root, batch_rows):
    import pathlib
    from test_gpu_e2e import _pipeline as pipe
    return pipe(pathlib.Path(root), train_batch_size=batch_rows, epochs=EPOCHS)


def _train(step):
    losses = []
    for _ in range(EPOCHS):
        nb = step.begin_epoch()
        step.run_batches(0, min(5, nb))
        step.run_batches(min(5, nb), nb)
        losses += step.end_epoch()
    st = [step.opt.state[p][k].cpu() for p in (step.pU, step.pI)
          for k in ('exp_avg', 'exp_avg_sq')]
    return [step.pU.detach().cpu(), step.pI.detach().cpu()] + st, losses


def _worker(rank, port, root, q):
    import torch.distributed as tdist
    from recbole_amd.trainer.fused import FusedBPRTrainStep
    from recbole_amd.trainer.optim import FusedAdam
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=2)
    try:
        torch.cuda.set_device(0)
        config, train, valid, test, model = _pipeline(root, 256)
        opt = FusedAdam(model.parameters(), lr=config['learning_rate'])
        step = FusedBPRTrainStep(model, opt, train, chunk=CHUNK, dist=tdist.group.WORLD)
        tensors, losses = _train(step)
        q.put((rank, step.Bg, [t.numpy() for t in tensors], losses))   # by value
    finally:
        tdist.destroy_process_group()


def test_two_ranks_equal_one_gpu_global_batch(tmp_path):
    from recbole_amd.trainer.fused import FusedBPRTrainStep
    from recbole_amd.trainer.optim import FusedAdam
    root = str(tmp_path)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=600) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    config, train, valid, test, model = _pipeline(root, 512)
    opt = FusedAdam(model.parameters(), lr=config['learning_rate'])
    step = FusedBPRTrainStep(model, opt, train, chunk=CHUNK)
    assert train.dataset.inter_num % step.B != 0            # a ragged last batch
    ref_t, ref_l = _train(step)
    for rank, Bg, tensors, losses in got:
        assert Bg == step.B
        assert losses == ref_l, rank
        for a, b in zip(ref_t, tensors):
            assert np.array_equal(a.numpy(), b), (rank, np.abs(a.numpy() - b).max())
