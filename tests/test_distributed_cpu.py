"""The data-parallel exchange protocol on CPU (gloo, world size 2).

Each rank computes the per-contribution gradient rows of ITS slice of a global
BPR batch (torch-CPU autograd with the global-batch mean, the oracle's model),
packs them in the trainer/exchange.py layout, all-gathers, and sums every table
row's contributions through the GLOBAL batch's grouping remapped to packed rows.
The result must equal — bit for bit — the same grouped sums of one process that
computed the whole global batch; this is what makes the fused GPU step with G
ranks bit-identical to one GPU running the global batch."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

from recbole_amd.trainer.exchange import ExchangeLayout

G, B, T, D, NU, NI = 2, 6, 3, 8, 11, 17


def _batch():
    g = torch.Generator().manual_seed(7)
    EU = torch.randn(NU, D, generator=g)
    EI = torch.randn(NI, D, generator=g)
    users = torch.randint(0, 4, (G * B,), generator=g)            # repeats across ranks
    items = torch.randint(0, 6, ((1 + T) * G * B,), generator=g)  # row r = j*G*B + k
    return EU, EI, users, items


def _contrib_rows(EU, EI, users, pos, neg, R_total):
    """d loss / d (gathered rows) of the reference's BPR (bpr.py:74-83, loss.py:48)
    for positives users[k], pos[k], neg[j*n + k]; mean over the GLOBAL R_total rows."""
    n = users.numel()
    u = EU[users].clone().requires_grad_()
    p = EI[pos].clone().requires_grad_()
    q = EI[neg].clone().requires_grad_()
    ur, pr = u.repeat(T, 1), p.repeat(T, 1)
    x = (ur * pr).sum(-1) - (ur * q).sum(-1)
    loss = -torch.log(1e-10 + torch.sigmoid(x)).sum() / R_total
    loss.backward()
    return u.grad, torch.cat([p.grad, q.grad]).view(1 + T, n, D)


def _grouped(rows, keys, perm_rows, n_rows):
    """Row sums in the order of a stable sort of `keys` (K2's grouping)."""
    order = np.argsort(keys.numpy(), kind='stable')
    out = torch.zeros(n_rows, D)
    for c in order:
        out[keys[c]] += rows[perm_rows[c]]
    return out


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=G)
    EU, EI, users, items = _batch()
    lay = ExchangeLayout(G, B, T, D)
    lu = lay.local_users(users, rank).reshape(-1)
    li = lay.local_items(items, rank).reshape(1 + T, B)
    gU, gI = _contrib_rows(EU, EI, lu, li[0], li[1:].reshape(-1), G * B * T)
    xbuf = torch.zeros(G, lay.R, D)
    xbuf[rank, :B] = gU
    xbuf[rank, lay.item0:lay.loss0] = gI.reshape(-1, D)
    parts = list(xbuf.unbind(0))
    tdist.all_gather(parts, parts[rank].clone())
    flat = xbuf.view(-1, D)
    cu = torch.arange(G * B, dtype=torch.int32)
    ci = torch.arange((1 + T) * G * B, dtype=torch.int32)
    sumU = _grouped(flat, users, lay.user_rows(cu).long(), NU)
    sumI = _grouped(flat, items, lay.item_rows(ci).long(), NI)
    q.put((rank, sumU, sumI))
    tdist.destroy_process_group()


def test_exchange_layout_remaps_are_bijections():
    lay = ExchangeLayout(3, 5, 2, 4)
    u = lay.user_rows(torch.arange(15)).tolist()
    i = lay.item_rows(torch.arange(45)).tolist()
    assert len(set(u) | set(i)) == 60
    assert all(0 <= r < 3 * lay.R for r in u + i)
    assert all(lay.loss0 > r % lay.R for r in u + i)       # never the loss rows


def test_two_rank_exchange_equals_global_batch():
    EU, EI, users, items = _batch()
    gU, gI = _contrib_rows(EU, EI, users, items[:G * B], items[G * B:], G * B * T)
    refU = _grouped(gU, users, torch.arange(G * B), NU)
    refI = _grouped(gI.reshape(-1, D), items, torch.arange((1 + T) * G * B), NI)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(G)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(G)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, sumU, sumI in got:
        assert torch.equal(sumU, refU), rank
        assert torch.equal(sumI, refI), rank
