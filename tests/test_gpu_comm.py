"""The generic cross-GPU entry points of the C-ABI (mirec_alltoallv_rows_f32,
mirec_allreduce_sum_f32; csrc/comm.hip) with 2 and 3 ranks (spawned processes, a gloo group
for the IPC handle exchange, all on cuda:0 — this covers the flag / barrier protocol,
not xGMI itself):
  * ragged send_counts, the received blocks and recv_counts exact;
  * all-reduce bit-identical to the rank-order sum torch computes on the host;
  * calls back to back and interleaved (alltoallv, allreduce, alltoallv, ...) with no
    host sync between them — the entry / exit barriers keep a fast rank from
    overwriting a window block its peer has not consumed;
  * the status word stays 0 (no wait gave up), and mirec_shard_next's push lists
    against their specification."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import free_port

pytestmark = pytest.mark.gpu

WCAP, D, ROUNDS = 96, 64, 6


def _data(rank, r, WORLD):
    g = torch.Generator().manual_seed(1000 * r + rank)
    send = torch.randn(WORLD, WCAP, D, generator=g)
    counts = torch.randint(0, WCAP + 1, (WORLD,), generator=g)
    counts[(rank + r) % WORLD] = WCAP if r % 3 == 0 else 0       # full and empty blocks
    vec = torch.randn(WCAP * D // 2, generator=g)
    return send, counts, vec


def _worker(rank, port, q, WORLD):
    import ctypes

    import torch.distributed as tdist
    from recbole_amd._native import check, lib
    from recbole_amd.trainer.comm import PeerWindows
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=WORLD)
    try:
        torch.cuda.set_device(0)
        dev = torch.device('cuda', 0)
        win = PeerWindows(tdist.group.WORLD, WCAP, D, dev)
        assert win.shared_device
        L = lib()
        st = torch.cuda.current_stream(dev).cuda_stream
        outs = []
        keep = []
        for r in range(ROUNDS):                       # no host sync inside the loop
            send, counts, vec = _data(rank, r, WORLD)
            s_d, c_d = send.to(dev), counts.to(dev)
            recv = torch.full((WORLD, WCAP, D), -7.0, device=dev)
            rc = torch.full((WORLD,), -1, dtype=torch.int64, device=dev)
            check(L.mirec_alltoallv_rows_f32(win.comm, s_d.data_ptr(), c_d.data_ptr(),
                                             recv.data_ptr(), rc.data_ptr(), D, ctypes.c_void_p(st)),
                  'mirec_alltoallv_rows_f32')
            buf = vec.to(dev)
            check(L.mirec_allreduce_sum_f32(win.comm, buf.data_ptr(), buf.numel(), ctypes.c_void_p(st)),
                  'mirec_allreduce_sum_f32')
            keep.append((s_d, c_d))
            outs.append((recv, rc, buf))
        torch.cuda.synchronize(dev)
        status = win.status()
        res = [(a.cpu().numpy(), b.cpu().numpy(), c.cpu().numpy()) for a, b, c in outs]
        win.close()
        q.put((rank, status, res))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize('WORLD', [2, 3])
def test_alltoallv_and_allreduce_ranks(WORLD):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, WORLD)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = dict((r, (s, res)) for r, s, res in (q.get(timeout=300) for _ in range(WORLD)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for me in range(WORLD):
        status, res = got[me]
        assert status == 0, me
        for r, (recv, rc, buf) in enumerate(res):
            exp_sum = None
            for src in range(WORLD):
                send, counts, vec = _data(src, r, WORLD)
                n = int(counts[me])
                assert rc[src] == n, (me, r, src)
                np.testing.assert_array_equal(recv[src, :n], send[me, :n].numpy())
                assert (recv[src, n:] == -7.0).all()
                exp_sum = vec.clone() if exp_sum is None else exp_sum + vec   # rank order
            np.testing.assert_array_equal(buf, exp_sum.numpy())


@pytest.mark.parametrize('per,nb', [(64, 5), (300, 3)])
def test_shard_next_matches_spec(dev, per, nb):
    """mirec_shard_next: where each entry of step c's owned lists sits in step c+1's."""
    from recbole_amd._native import check, lib
    rng = np.random.default_rng(per + nb)
    own = np.zeros((nb, per), np.int32)
    n = np.zeros(nb, np.int32)
    ah = np.zeros((nb, per), np.int32)
    nah = np.zeros(nb, np.int32)
    lists = []
    for c in range(nb):
        k = int(rng.integers(0, per + 1))
        lists.append(np.sort(rng.choice(4 * per, k, replace=False)).astype(np.int32))
        own[c, :k], n[c] = lists[-1], k
    for c in range(nb - 1):
        a = np.setdiff1d(lists[c + 1], lists[c]).astype(np.int32)
        ah[c, :a.size], nah[c] = a, a.size
    T = lambda x: torch.as_tensor(x.reshape(-1), device=dev)
    nt = torch.full((nb * per,), -9, dtype=torch.int32, device=dev)
    na = torch.full((nb * per,), -9, dtype=torch.int32, device=dev)
    od, ond, ad, andv = T(own), T(n), T(ah), T(nah)
    check(lib().mirec_shard_next(od.data_ptr(), ond.data_ptr(), ad.data_ptr(), andv.data_ptr(),
                                 per, nb, nt.data_ptr(), na.data_ptr(),
                                 torch.cuda.current_stream(dev).cuda_stream), 'mirec_shard_next')
    nt, na = nt.cpu().numpy().reshape(nb, per), na.cpu().numpy().reshape(nb, per)
    for c in range(nb - 1):
        pos = {int(v): j for j, v in enumerate(lists[c + 1])}
        assert [pos.get(int(v), -1) for v in lists[c]] == nt[c, :n[c]].tolist()
        assert [pos.get(int(v), -1) for v in ah[c, :nah[c]]] == na[c, :nah[c]].tolist()
        assert (na[c, :nah[c]] >= 0).all()       # the look-ahead rows are all read next
