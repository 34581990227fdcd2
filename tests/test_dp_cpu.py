"""Data-parallel helpers of the generic trainer path (recbole_amd/trainer/dist.py)
on CPU gloo ranks (world size 2): slicing of a global batch (incl. the sampler's
j*B + k layout of SSM negatives), the dense-gradient bucket all-reduce, the stash
all-gather in rank order, the global loss, and the sharded full-sort flag gather."""
import os

import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

G = 2


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=G)
    try:
        from recbole_amd.data.interaction import Interaction
        from recbole_amd.trainer.dist import DataParallelStep, active_group
        dp = DataParallelStep(active_group())
        B, N = 6, 3
        inter = Interaction({'u': torch.arange(B), 'seq': torch.arange(B * 4).view(B, 4),
                             'neg': torch.arange(N * B) + 100})
        loc, shard = dp.local_slice(inter)
        odd, shard_odd = dp.local_slice(Interaction({'u': torch.arange(5)}))
        lin = torch.nn.Linear(3, 2)
        with torch.no_grad():
            lin.weight.fill_(1.0)
            lin.bias.zero_()
        x = torch.full((1, 3), float(rank + 1))
        (lin(x).sum() * dp.loss_scale()).backward()

        class _Opt:
            _deferred = {'t': {'stash': [(torch.full((2, 4), float(rank)),
                                          torch.tensor([rank, 10 + rank]), None)]}}
        dp.exchange(lin, _Opt)
        rows, keys, _ = _Opt._deferred['t']['stash'][0]
        gl = dp.global_loss(torch.tensor(float(rank)))
        s, e, b = dp.user_block(5)
        flags = torch.arange(s, e).view(-1, 1).repeat(1, 2)
        allf = dp.gather_rows(flags, 5, b)
        q.put((rank, shard, loc['u'].tolist(), loc['seq'].tolist(), loc['neg'].tolist(),
               shard_odd, len(odd['u']), lin.weight.grad.tolist(), rows.tolist(),
               keys.tolist(), float(gl), allf.tolist()))
    finally:
        tdist.destroy_process_group()


def test_dp_helpers_two_ranks():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(G)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(G))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, shard, u, seq, neg, shard_odd, n_odd, wg, rows, keys, gl, allf in out:
        assert shard and not shard_odd and n_odd == 5
        assert u == [3 * rank, 3 * rank + 1, 3 * rank + 2]
        assert seq == [[4 * k + t for t in range(4)] for k in u]
        # j*B + k layout: rank's k in [3r, 3r+3) for every j
        assert neg == [100 + j * 6 + k for j in range(3) for k in u]
        # d/dW of sum(W x)/G summed over ranks: (1 + 2) / 2 per entry
        assert wg == [[1.5] * 3, [1.5] * 3]
        assert rows == [[0.0] * 4] * 2 + [[1.0] * 4] * 2 and keys == [0, 10, 1, 11]
        assert gl == 0.5
        assert allf == [[i, i] for i in range(5)]
