"""Row-sharded tables (csrc/shard.hip, trainer/fused.py ShardedBPRTrainStep) on
the GPU:
  * the exchange plans and the owner's slice of the grouping, bit for bit against
    the specification (trainer/exchange.py ShardLayout) for G = 1, 2, 3, 8, every
    rank, full and ragged batches, and the overflow status;
  * the sharded step on one rank (G = 1, no process group) bit-identical to the
    single-GPU fused step (weights, Adam state, losses; graph and eager);
  * 2 ranks (gloo, both on cuda:0) bit-identical to ONE process running the global
    batch (ragged last batch, partial chunks);
  * the RCCL code path (a 1-rank nccl group: all-to-all + all-gather inside the
    captured chunk graphs) equal to the single-GPU step."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT, free_port
from recbole_amd.trainer.exchange import ShardLayout

pytestmark = pytest.mark.gpu

EPOCHS, CHUNK = 2, 4


@pytest.mark.parametrize('G,Bc', [(1, 48), (2, 96), (3, 144), (3, 100), (8, 384), (8, 170)])
def test_shard_plan_and_own_match_spec(dev, G, Bc):
    from recbole_amd import ops
    from recbole_amd._native import check, lib
    B, T, nU, nI = 48, 4, 301, 523
    cap = min((2 + T) * B, -(-5 * (2 + T) * B // (4 * G)) + 64)
    lay = ShardLayout(G, B, T, nU, nI, cap)
    g = torch.Generator().manual_seed(G * 1000 + Bc)
    users = torch.randint(0, nU, (Bc,), generator=g)
    items = torch.randint(1, nI, ((1 + T) * Bc,), generator=g)
    items[:Bc // 3] = 5                                        # a hot item
    ud, idv = users.to(dev), items.to(dev)
    L = lib()
    st = torch.cuda.current_stream().cuda_stream
    keyed = {}
    for tag, ids, S in (('u', ud, lay.SU), ('i', idv, lay.SI)):
        k = torch.empty_like(ids)
        check(L.mirec_shard_keys(ids.data_ptr(), ids.numel(), G, S, k.data_ptr(), st), 'keys')
        assert torch.equal(k.cpu(), lay.keys(ids.cpu(), S))
        n = ids.numel()
        perm = torch.empty(n, dtype=torch.int32, device=dev)
        uniq = torch.empty(n, dtype=torch.int32, device=dev)
        seg = torch.empty(n + 1, dtype=torch.int32, device=dev)
        nu = torch.zeros(1, dtype=torch.int32, device=dev)
        ops.segment_sort_batched(k, n, G * S, perm, uniq, seg, nu)
        keyed[tag] = (perm, uniq, seg, nu, S)
    M = G * cap
    KI = (1 + T) * Bc
    for r in range(G):
        fwd = torch.empty(M, dtype=torch.int64, device=dev)
        map2 = torch.full((Bc + KI,), -7, dtype=torch.int32, device=dev)
        pos = torch.full(((2 + T) * B,), -1, dtype=torch.int64, device=dev)
        bwd = torch.empty(M, dtype=torch.int32, device=dev)
        status = torch.zeros(2, dtype=torch.int32, device=dev)
        check(L.mirec_shard_plan(ud.data_ptr(), idv.data_ptr(), 1, Bc, B, T, G, r, cap,
                                 fwd.data_ptr(), map2.data_ptr(), pos.data_ptr(), bwd.data_ptr(),
                                 status.data_ptr(), st), 'plan')
        efwd, emap, epos, ebwd, over = lay.plan(users, items, r)
        assert not over and status.tolist() == [0, lay.largest_message(users, items)]
        assert torch.equal(fwd.cpu(), efwd)
        assert torch.equal(bwd.cpu(), ebwd)
        n_r = max(0, min(B, Bc - r * B))
        assert torch.equal(pos.cpu()[:(2 + T) * n_r], epos[:(2 + T) * n_r])
        owned = emap >= 0
        assert torch.equal(map2.cpu()[owned], emap[owned])
        for tag, off in (('u', 0), ('i', Bc)):
            perm, uniq, seg, nu, S = keyed[tag]
            n = perm.numel()
            own = torch.empty(n, dtype=torch.int32, device=dev)
            oseg = torch.empty(n + 1, dtype=torch.int32, device=dev)
            on = torch.zeros(1, dtype=torch.int32, device=dev)
            p2 = torch.full((n,), -9, dtype=torch.int32, device=dev)
            check(L.mirec_shard_own(uniq.data_ptr(), seg.data_ptr(), nu.data_ptr(),
                                    perm.data_ptr(), n, 1, None, None, map2.data_ptr(), Bc + KI,
                                    off, S, r, own.data_ptr(), oseg.data_ptr(), on.data_ptr(),
                                    p2.data_ptr(), None, None, st), 'own')
            nn = int(nu.item())
            e_own, e_seg, e_p, e_p2 = lay.own(uniq.cpu()[:nn], seg.cpu()[:nn + 1], perm.cpu(),
                                             map2.cpu(), off, S, r)
            k = int(on.item())
            assert k == e_own.numel()
            assert torch.equal(own.cpu()[:k], e_own)
            assert torch.equal(oseg.cpu()[:k + 1], e_seg)
            assert torch.equal(p2.cpu()[e_p], e_p2)
    # a too-small cap is reported on every rank (with the largest message), and the
    # overflowing slots get the in-range position 0 instead of stale values
    for r in range(G):
        status = torch.zeros(2, dtype=torch.int32, device=dev)
        bufs = [torch.empty(G * 2, dtype=torch.int64, device=dev),
                torch.full((Bc + KI,), 1 << 30, dtype=torch.int32, device=dev),
                torch.full(((2 + T) * B,), 1 << 40, dtype=torch.int64, device=dev),
                torch.empty(G * 2, dtype=torch.int32, device=dev)]
        check(L.mirec_shard_plan(ud.data_ptr(), idv.data_ptr(), 1, Bc, B, T, G, r, 2,
                                 *[b.data_ptr() for b in bufs], status.data_ptr(), st), 'plan')
        assert status.tolist() == [-4, lay.largest_message(users, items)]
        n_r = max(0, min(B, Bc - r * B))
        if n_r:                          # a ragged batch leaves the last ranks no positives
            assert int(bufs[2][:(2 + T) * n_r].max()) < 2 * G
        owned = (torch.cat([users, items]) % G == r).to(dev)
        if bool(owned.any()):
            assert int(bufs[1][owned].max()) < 2 * G


@pytest.mark.parametrize('G,nb,per', [(1, 3, 240), (2, 4, 240), (3, 2, 1000), (8, 5, 2560)])
def test_owner_filtered_grouping_matches_global(dev, G, nb, per):
    """mirec_shard_select + K2 on the selected keys + mirec_shard_own_sel give every rank
    the same owned rows, the same look-ahead lists and, per owned row, the same
    contributions in the same order as mirec_shard_own on the global grouping."""
    from recbole_amd import ops
    from recbole_amd._native import check, lib
    S, L = 97, lib()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(G * 7 + per)
    ids = torch.randint(0, G * S, (nb * per,), generator=g)
    ids[:per // 4] = 5                                         # a hot row
    idd = ids.to(dev)
    map2 = torch.randperm(nb * per, generator=g).to(torch.int32).to(dev)   # stand-in plan

    def group(keys, stride, space):
        n = keys.numel()
        out = [torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32,
               device=dev), torch.empty(nb * (stride + 1), dtype=torch.int32, device=dev),
               torch.zeros(nb, dtype=torch.int32, device=dev)]
        ops.segment_sort_batched(keys, stride, space, *out)
        ah = torch.empty(n, dtype=torch.int32, device=dev)
        nah = torch.zeros(nb, dtype=torch.int32, device=dev)
        ops.uniq_ahead_diff(out[1], out[3], stride, nb, ah, nah)
        return out + [ah, nah]

    def owned(res, stride, r, sel=None):
        perm, uniq, seg, nu, ah, nah = res
        own = torch.empty(nb * per, dtype=torch.int32, device=dev)
        oseg = torch.empty(nb * (per + 1), dtype=torch.int32, device=dev)
        on = torch.zeros(nb, dtype=torch.int32, device=dev)
        p2 = torch.full((nb * per,), -9, dtype=torch.int32, device=dev)
        oa = torch.empty(nb * per, dtype=torch.int32, device=dev)
        ona = torch.zeros(nb, dtype=torch.int32, device=dev)
        args = [uniq.data_ptr(), seg.data_ptr(), nu.data_ptr(), perm.data_ptr(), stride, nb,
                ah.data_ptr(), nah.data_ptr(), map2.data_ptr(), per, 0, S, r]
        outs = [own.data_ptr(), oseg.data_ptr(), on.data_ptr(), p2.data_ptr(), oa.data_ptr(),
                ona.data_ptr(), st]
        if sel is None:
            check(L.mirec_shard_own(*args, *outs), 'own')
        else:
            check(L.mirec_shard_own_sel(*args, sel.data_ptr(), per, *outs), 'own_sel')
        rows = []
        for c in range(nb):
            k = int(on[c])
            o = own[c * per:c * per + k].tolist()
            sg = oseg[c * (per + 1):c * (per + 1) + k + 1].tolist()
            p = p2[c * per:(c + 1) * per].tolist()
            rows.append((o, [p[sg[x]:sg[x + 1]] for x in range(k)],
                         oa[c * per:c * per + int(ona[c])].tolist() if c + 1 < nb else None))
        return rows

    most_owned = max(int(((ids[c * per:(c + 1) * per] % G) == r).sum())
                     for c in range(nb) for r in range(G))
    cap_sel = min(per, most_owned + 16)            # padded batches on every rank
    keyed = torch.empty_like(idd)
    check(L.mirec_shard_keys(idd.data_ptr(), idd.numel(), G, S, keyed.data_ptr(), st), 'keys')
    glob = group(keyed, per, G * S)
    for r in range(G):
        keys = torch.empty(nb * cap_sel, dtype=torch.int64, device=dev)
        sel = torch.empty(nb * cap_sel, dtype=torch.int32, device=dev)
        most = torch.zeros(1, dtype=torch.int32, device=dev)
        check(L.mirec_shard_select(idd.data_ptr(), nb, per, G, S, r, cap_sel, keys.data_ptr(),
                                   sel.data_ptr(), most.data_ptr(), st), 'select')
        counts = [int(((ids[c * per:(c + 1) * per] % G) == r).sum()) for c in range(nb)]
        assert int(most) == max(counts) <= cap_sel
        assert owned(group(keys, cap_sel, G * S + 1), cap_sel, r, sel) == owned(glob, per, r)
    # an over-full batch is reported (the caller re-selects at full size)
    most = torch.zeros(1, dtype=torch.int32, device=dev)
    keys = torch.empty(nb * 8, dtype=torch.int64, device=dev)
    sel = torch.empty(nb * 8, dtype=torch.int32, device=dev)
    check(L.mirec_shard_select(idd.data_ptr(), nb, per, G, S, 0, 8, keys.data_ptr(),
                               sel.data_ptr(), most.data_ptr(), st), 'select')
    assert int(most) > 8


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


@pytest.mark.parametrize('graph', [True, False])
def test_sharded_solo_equals_fused(tmp_path, graph):
    from recbole_amd.trainer.fused import FusedBPRTrainStep, ShardedBPRTrainStep
    from recbole_amd.trainer.optim import FusedAdam
    out = []
    for cls in (FusedBPRTrainStep, ShardedBPRTrainStep):
        config, train, valid, test, model = _pipeline(str(tmp_path), 512)
        opt = FusedAdam(model.parameters(), lr=config['learning_rate'])
        out.append(_train(cls(model, opt, train, chunk=CHUNK, use_graph=graph)))
    (ta, la), (tb, lb) = out
    assert la == lb
    for a, b in zip(ta, tb):
        assert torch.equal(a, b)


@pytest.mark.parametrize('graph', [True, False])
def test_sharded_cap_overflow_replans(tmp_path, graph):
    """A cap below the largest message: the chunk is re-planned with a larger cap
    before it runs (no step on a truncated plan; graphs recaptured) — results
    bit-identical to the fused single-GPU step."""
    cap = 64
    from recbole_amd.trainer.fused import FusedBPRTrainStep, ShardedBPRTrainStep
    from recbole_amd.trainer.optim import FusedAdam
    out = []
    for cls, kw in ((FusedBPRTrainStep, {}), (ShardedBPRTrainStep, {'cap': cap})):
        config, train, valid, test, model = _pipeline(str(tmp_path), 512)
        opt = FusedAdam(model.parameters(), lr=config['learning_rate'])
        step = cls(model, opt, train, chunk=CHUNK, use_graph=graph, **kw)
        out.append(_train(step))
        if kw:
            assert step.cap_growths >= 1 and step.cap > cap
    (ta, la), (tb, lb) = out
    assert la == lb
    for a, b in zip(ta, tb):
        assert torch.equal(a, b)


def _worker(rank, port, root, q, cap=None, exchange='rccl', sel=None, world=2):
    import torch.distributed as tdist
    from recbole_amd.trainer.fused import ShardedBPRTrainStep
    from recbole_amd.trainer.optim import FusedAdam
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        config, train, valid, test, model = _pipeline(root, 256)
        opt = FusedAdam(model.parameters(), lr=config['learning_rate'])
        step = ShardedBPRTrainStep(model, opt, train, chunk=CHUNK, dist=tdist.group.WORLD,
                                   cap=cap, exchange=exchange)
        assert step.exchange == exchange
        if sel is not None:                       # owner-filtered grouping too small: the
            step.cap_sel = dict(sel)              # chunks are re-selected at full size
        sel_growths0 = step.sel_growths
        tensors, losses = _train(step)
        assert cap is None or step.cap_growths >= 1
        assert sel is None or step.sel_growths > sel_growths0
        if step.win is not None:                  # no wait gave up (end_epoch raises too)
            assert step.win.status() == 0
        step.close()
        q.put((rank, step.Bg, step.SU, [t.numpy() for t in tensors], losses))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize('cap,exchange,sel,world', [(None, 'rccl', None, 2), (40, 'rccl', None, 2),
                                                    (None, 'rccl', {'u': 4, 'i': 12}, 2),
                                                    (None, 'ipc', None, 2), (40, 'ipc', None, 2),
                                                    (None, 'rccl', None, 3), (None, 'ipc', None, 3)])
def test_sharded_ranks_equal_one_gpu_global_batch(tmp_path, cap, exchange, sel, world):
    """world ranks (2, 3) bitwise equal to one process on the global batch.
    cap=40: every rank detects the same overflow and grows cap identically.
    sel: an owner-filtered grouping too small for the batches' owned slots — every chunk
    is re-selected at full size before it runs (ShardedBPRTrainStep._grow_sel).
    exchange='ipc': the rows go through the peer windows (csrc/comm.hip: IPC-mapped, in-
    kernel stores, flags on the GPU). Both ranks share cuda:0 here, so this pins the flag /
    counter protocol, the push lists and the owner-Adam fold — NOT the cross-device mapping
    over xGMI, which no test on a one-GPU box can reach (hence RCCL stays the default)."""
    from recbole_amd.trainer.fused import FusedBPRTrainStep
    from recbole_amd.trainer.optim import FusedAdam
    root = str(tmp_path)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, root, q, cap, exchange, sel, world))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    config, train, valid, test, model = _pipeline(root, 256 * world)
    opt = FusedAdam(model.parameters(), lr=config['learning_rate'])
    step = FusedBPRTrainStep(model, opt, train, chunk=CHUNK)
    assert train.dataset.inter_num % step.B != 0            # a ragged last batch
    ref_t, ref_l = _train(step)
    for rank, Bg, SU, tensors, losses in got:
        assert Bg == step.B and SU == -(-step.nU // world)
        assert losses == ref_l, rank
        for a, b in zip(ref_t, tensors):
            assert np.array_equal(a.numpy(), b), (rank, np.abs(a.numpy() - b).max())


NCCL_SCRIPT = r'''
import os, sys, pathlib, torch, torch.distributed as tdist
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], 'tests'))
os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=sys.argv[3], RANK='0', WORLD_SIZE='1')
torch.cuda.set_device(0)
tdist.init_process_group('nccl', device_id=torch.device('cuda', 0))
from test_gpu_e2e import _pipeline
from recbole_amd.trainer.fused import FusedBPRTrainStep, ShardedBPRTrainStep
from recbole_amd.trainer.optim import FusedAdam
res = []
for cls, dist in ((FusedBPRTrainStep, None), (ShardedBPRTrainStep, tdist.group.WORLD)):
    config, train, valid, test, model = _pipeline(pathlib.Path(sys.argv[2]), epochs=2)
    opt = FusedAdam(model.parameters(), lr=config['learning_rate'])
    step = cls(model, opt, train, chunk=4, dist=dist)
    assert step.use_graph
    losses = []
    for _ in range(2):
        losses += step.run_epoch()
    res.append((losses, step.pU.detach().cpu(), step.pI.detach().cpu()))
    step.close()                 # captured collectives go before destroy_process_group
    del step
assert res[0][0] == res[1][0]
assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])
tdist.destroy_process_group()
print('NCCL_OK')
'''


def test_sharded_rccl_path_one_rank(tmp_path):
    script = tmp_path / 'nccl_one_rank.py'
    script.write_text(NCCL_SCRIPT)
    port = str(free_port())
    out = subprocess.run([sys.executable, str(script), ROOT, str(tmp_path), port],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and 'NCCL_OK' in out.stdout, out.stderr[-3000:]
