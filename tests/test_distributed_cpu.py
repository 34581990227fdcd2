"""The data-parallel exchange protocol on CPU (gloo, world size 2).

Each rank computes, for ITS slice of a global BPR batch, the per-row coefficients
coef_r = d loss / d (pos_score - neg_score) (torch-CPU autograd with the global-batch
mean, the oracle's model) and the per-positive losses, packs them in the
trainer/exchange.py layout, all-gathers, and rebuilds the gradient rows of the
GLOBAL batch from the rows and the gathered coefficients (the arithmetic of
mirec_bpr_contrib_f32), then sums every table row's contributions through the
global batch's grouping. The result must equal — bit for bit — the same grouped
sums of one process that computed the whole global batch; this is what makes the
fused GPU step with G ranks bit-identical to one GPU running the global batch."""
import os

import numpy as np
import torch
from conftest import free_port
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


def _coef(EU, EI, users, pos, neg, R_total):
    """Per-row d loss / d x and per-positive losses of the reference's BPR
    (bpr.py:74-83, loss.py:48) for rows (users[k], pos[k], neg[j*n + k]), mean over
    the GLOBAL R_total rows."""
    n = users.numel()
    u, p, q = EU[users], EI[pos], EI[neg]
    ur, pr = u.repeat(T, 1), p.repeat(T, 1)
    x = ((ur * pr).sum(-1) - (ur * q).sum(-1)).detach().requires_grad_()
    per_row = -torch.log(1e-10 + torch.sigmoid(x))
    (per_row.sum() / R_total).backward()
    return x.grad.view(T, n), per_row.detach().view(T, n).sum(0)


def _rows(EU, EI, users, pos, neg, coef):
    """Gradient rows from the coefficients, in the order of mirec_bpr_contrib_f32:
    du = sum_j (c*p - c*n_j), dp = sum_j c*u, dn_j = -c*u."""
    n = users.numel()
    u, p = EU[users], EI[pos]
    q = EI[neg].view(T, n, D)
    gu = torch.zeros(n, D)
    gp = torch.zeros(n, D)
    gn = torch.empty(T, n, D)
    for j in range(T):
        c = coef[j].unsqueeze(1)
        gu = gu + (c * p - c * q[j])
        gp = gp + c * u
        gn[j] = -c * u
    return gu, torch.cat([gp.unsqueeze(0), gn]).view(1 + T, n, D)


def _grouped(rows, keys, n_rows):
    """Row sums in the order of a stable sort of `keys` (K2's grouping)."""
    order = np.argsort(keys.numpy(), kind='stable')
    out = torch.zeros(n_rows, D)
    for c in order:
        out[keys[c]] += rows[c]
    return out


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=G)
    EU, EI, users, items = _batch()
    lay = ExchangeLayout(G, B, T, D)
    lu = lay.local_users(users, rank).reshape(-1)
    li = lay.local_items(items, rank).reshape(1 + T, B)
    coef, loss = _coef(EU, EI, lu, li[0], li[1:].reshape(-1), G * B * T)
    buf = torch.zeros(G, lay.W)
    buf[rank, :B] = loss
    buf[rank, lay.coef0:] = coef.reshape(-1)
    parts = list(buf.unbind(0))
    tdist.all_gather(parts, parts[rank].clone())
    cg = lay.coef_global(buf).view(T, G * B)
    gU, gI = _rows(EU, EI, users, items[:G * B], items[G * B:], cg)
    sumU = _grouped(gU, users, NU)
    sumI = _grouped(gI.reshape(-1, D), items, NI)
    # by value (numpy): a torch tensor would travel as a shared-memory handle that
    # dies with this process
    q.put((rank, sumU.numpy(), sumI.numpy(), lay.gathered_losses(buf).reshape(-1).numpy()))
    tdist.destroy_process_group()


def test_exchange_layout_blocks():
    lay = ExchangeLayout(3, 5, 2, 4)
    buf = torch.arange(3 * lay.W, dtype=torch.float32)
    assert lay.gathered_losses(buf).reshape(-1).tolist() == \
        [g * lay.W + k for g in range(3) for k in range(5)]
    cg = lay.coef_global(buf).view(2, 15)
    # global row (j, g*B + k) <- rank g's local coefficient j*B + k
    for j in range(2):
        for g in range(3):
            for k in range(5):
                assert cg[j, g * 5 + k] == g * lay.W + lay.coef0 + j * 5 + k


def test_two_rank_exchange_equals_global_batch():
    EU, EI, users, items = _batch()
    coef, loss = _coef(EU, EI, users, items[:G * B], items[G * B:], G * B * T)
    gU, gI = _rows(EU, EI, users, items[:G * B], items[G * B:], coef)
    refU = _grouped(gU, users, NU)
    refI = _grouped(gI.reshape(-1, D), items, NI)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(G)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(G)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, sumU, sumI, losses in got:
        assert np.array_equal(sumU, refU.numpy()), rank
        assert np.array_equal(sumI, refI.numpy()), rank
        assert np.array_equal(losses, loss.numpy()), rank
