"""K35 (csrc/step.hip, mirec_bpr_adam_step_f32): one launch per BPR training step —
the owners of the touched rows form their own gradient contributions (BPR forward +
backward, bpr.py:74-83, loss.py:43-49), add them in grouping order and apply the
deferred Adam step, and the look-ahead rows replay — bit for bit against the two
launches it replaces (K3 mirec_bpr_fwd_bwd_f32 + K5 mirec_adam_deferred_f32), on
tables held in parity buffers (state t in buffer t & 1).

Cases: d in {64, 128, 256}; T = 3, 4 and 6 (a partial negative group; negatives past
the 4 a contribution record holds); an even and an odd step; duplicate users; a hot
item with 40 or 80 positive slots (a split row: its contributions dealt out in shares
of 2 to other blocks of the launch, the last to arrive sums them); batches whose items
come from 3 or 5 ids (more shares than the 256 a batch deals out: the rest stay with
the row's own block, past its 62 staged records); look-ahead rows lagging 0..7 steps, in
their parity buffer with the other buffer poisoned (NaN); zero-state rows. After the
launch the arrival counters are zero again."""
import numpy as np
import pytest
import torch

from recbole_amd import ops
from recbole_amd.ops import ADAM_ZERO_STATE, Segments

pytestmark = pytest.mark.gpu


def _consts(dev, n=32):
    from recbole_amd.trainer.optim import FusedAdam
    opt = FusedAdam([torch.nn.Parameter(torch.zeros(4, device=dev))], lr=1e-3)
    return torch.as_tensor(opt.step_constants(1, n).reshape(-1), device=dev)


def _grouping(keys, space):
    segs = Segments(keys.numel(), keys.device)
    ws = ops.segment_sort_batched(keys, keys.numel(), space, segs.perm, segs.uniq, segs.seg,
                                  segs.n_uniq)
    segs.ws = ws
    return segs


def build_case(dev, d, T, s, Bc, few):
    """Inputs of one K35 launch (step s) and the K3 + K5 reference result on them."""
    g = torch.Generator().manual_seed(d * 100 + T * 10 + s)
    nU, nI = 257, 301
    # batch 0 (the step) and batch 1 (whose rows the look-ahead completes)
    user0 = torch.randint(0, nU, (Bc,), generator=g)
    user0[5] = user0[17] = user0[60]                       # a user with 3 positives
    user1 = torch.randint(0, nU, (Bc,), generator=g)
    items0 = torch.randint(1, nI, ((1 + T) * Bc,), generator=g)
    if few:                                                 # every item row a split row
        items0 = torch.randint(1, 1 + few, ((1 + T) * Bc,), generator=g)
    hot = 40 if s % 2 == 0 else 80                          # > 64: two id-table refills
    items0[:hot] = 7                                        # hot item: `hot` positive slots
    items0[Bc + 3] = 7                                      # ... and a negative slot
    items1 = torch.randint(1, nI, ((1 + T) * Bc,), generator=g)
    pU = torch.randn(nU, d, generator=g) * 0.1
    pI = torch.randn(nI, d, generator=g) * 0.1
    mU, vU = torch.randn(nU, d, generator=g) * 1e-3, torch.rand(nU, d, generator=g) * 1e-5
    mI, vI = torch.randn(nI, d, generator=g) * 1e-3, torch.rand(nI, d, generator=g) * 1e-5
    # step counts: rows batch 0 reads are current (s); others lag 0..7; some zero-state
    lastU = s - torch.randint(0, 8, (nU,), generator=g, dtype=torch.int32)
    lastI = s - torch.randint(0, 8, (nI,), generator=g, dtype=torch.int32)
    lastU[user0] = s
    lastI[items0] = s
    for m, v, last, read in ((mU, vU, lastU, user0), (mI, vI, lastI, items0)):
        zs = torch.zeros(last.numel(), dtype=torch.bool)
        zs[torch.randint(0, last.numel(), (last.numel() // 6,), generator=g)] = True
        zs[read] = zs[read] & (torch.arange(read.numel()) % 2 == 0)   # some read rows too
        m[zs], v[zs] = 0.0, 0.0
        last[zs] = ADAM_ZERO_STATE
    to = lambda x: x.to(dev)
    consts = _consts(dev)
    base = torch.tensor([s - 3], dtype=torch.int32, device=dev)     # step = base + 3
    grad_scale = float(np.float32(1.0) / np.float32(Bc * T))

    gu0, gi0 = _grouping(to(user0), nU), _grouping(to(items0), nI)
    gu1, gi1 = _grouping(to(user1), nU), _grouping(to(items1), nI)
    ahead = []
    for a, b, n in ((gu0, gu1, nU), (gi0, gi1, nI)):
        # rows batch 1 reads and batch 0 does not touch (the chunk layout of 2 batches)
        stride = max(a.uniq.numel(), b.uniq.numel())
        U = torch.zeros(2 * stride, dtype=torch.int32, device=dev)
        N = torch.zeros(2, dtype=torch.int32, device=dev)
        U[:a.uniq.numel()] = a.uniq
        U[stride:stride + b.uniq.numel()] = b.uniq
        N[0], N[1] = a.n_uniq[0], b.n_uniq[0]
        out = torch.zeros(2 * stride, dtype=torch.int32, device=dev)
        n_out = torch.zeros(2, dtype=torch.int32, device=dev)
        ops.uniq_ahead_diff(U, N, stride, 2, out, n_out)
        ahead.append((out[:stride].clone(), n_out[:1].clone()))
    assert int(ahead[0][1]) > 0 and int(ahead[1][1]) > 0

    # ---- reference: K3 on the single current tables, then K5 deferred
    rU, rI = to(pU.clone()), to(pI.clone())
    rmU, rvU, rmI, rvI = to(mU.clone()), to(vU.clone()), to(mI.clone()), to(vI.clone())
    rlU, rlI = to(lastU.clone()), to(lastI.clone())
    o = ops.bpr_fwd_bwd(rU, rI, to(user0), to(items0[:Bc]), to(items0[Bc:]), T,
                        grad_scale=grad_scale)
    tabs = ops.adam_tables([
        {'p': rU, 'm': rmU, 'v': rvU, 'rows': o['gU'], 'segs': gu0, 'last': rlU,
         'ahead': ahead[0]},
        {'p': rI, 'm': rmI, 'v': rvI, 'rows': o['gI'], 'segs': gi0, 'last': rlI,
         'ahead': ahead[1]}])
    ops.adam_multi(tabs, d, consts, base, 3, schedule='deferred',
                   n_max_uniq=[Bc, (1 + T) * Bc])

    # ---- K35 inputs on parity buffers: row state t in buffer t & 1, the other poisoned
    bufs = []
    for p, last in ((pU, lastU), (pI, lastI)):
        P = [torch.full_like(p, float('nan')), torch.full_like(p, float('nan'))]
        for par in (0, 1):
            sel = (last & 1) == par
            P[par][sel] = p[sel]
        zs = last == ADAM_ZERO_STATE                       # zero-state: both buffers
        P[0][zs], P[1][zs] = p[zs], p[zs]
        bufs.append([to(P[0]), to(P[1])])
    return dict(d=d, T=T, s=s, Bc=Bc, dev=dev, bufs=bufs, mv=[to(x) for x in (mU, vU, mI, vI)],
                last=[to(lastU), to(lastI)], gu0=gu0, gi0=gi0, ahead=ahead, consts=consts,
                base=base, grad_scale=grad_scale, user0=to(user0), items0=to(items0), nU=nU,
                nI=nI, ref=dict(p=(rU, rI), m=(rmU, rmI), v=(rvU, rvI), last=(rlU, rlI),
                                loss_k=o['loss_k']))


def run_k35(c, stream=None):
    """K35 on fresh copies of the case's inputs (on `stream`, default current); returns
    the state it leaves: parity buffers, m, v, last, loss_k and the scratch."""
    d, T, Bc, dev = c['d'], c['T'], c['Bc'], c['dev']
    with torch.cuda.stream(stream or torch.cuda.current_stream(dev)):
        bufs = [[b.clone() for b in pair] for pair in c['bufs']]
        fmU, fvU, fmI, fvI = (x.clone() for x in c['mv'])
        flU, flI = (x.clone() for x in c['last'])
        tabs2 = ops.adam_tables([
            {'p': bufs[0][0], 'p_alt': bufs[0][1], 'm': fmU, 'v': fvU, 'grouping': c['gu0'],
             'last': flU, 'ahead': c['ahead'][0]},
            {'p': bufs[1][0], 'p_alt': bufs[1][1], 'm': fmI, 'v': fvI, 'grouping': c['gi0'],
             'last': flI, 'ahead': c['ahead'][1]}])
        loss_k = torch.full((Bc,), float('nan'), device=dev)
        recs = ops.step_records(c['user0'], c['items0'], 1, Bc, T, c['nU'], c['nI'], c['gu0'],
                                c['gi0'])
        scratch = ops.step_scratch(Bc, T, d, dev)
        ops.bpr_adam_step(tabs2, [Bc, (1 + T) * Bc], d, c['items0'], Bc, T, c['grad_scale'],
                          loss_k, recs, scratch, c['consts'], c['base'], 3)
    return dict(bufs=bufs, m=(fmU, fmI), v=(fvU, fvI), last=(flU, flI), loss_k=loss_k,
                scratch=scratch)


def check_k35(c, r):
    """Every word of the K35 result against the K3 + K5 reference."""
    s, ref = c['s'], c['ref']
    assert int(r['scratch'][1].abs().sum()) == 0 and int(r['scratch'][3].abs().sum()) == 0
    assert torch.equal(r['loss_k'], ref['loss_k'])
    for q in range(2):
        P, rp, rl, fl = r['bufs'][q], ref['p'][q], ref['last'][q], r['last'][q]
        assert torch.equal(rl, fl)
        assert torch.equal(ref['m'][q], r['m'][q]) and torch.equal(ref['v'][q], r['v'][q])
        moved = (fl == s + 1)                              # touched + look-ahead rows
        assert int(moved.sum()) > 0
        wb = P[(s + 1) & 1]
        assert torch.equal(wb[moved], rp[moved])
        # rows not moved keep their state in their own buffer
        keep = ~moved & (fl != ADAM_ZERO_STATE)
        src = torch.where(((fl & 1) == 1)[:, None], P[1], P[0])
        assert torch.equal(src[keep], rp[keep])


@pytest.mark.parametrize('d,T,s,Bc,few', [(64, 3, 6, 96, 0), (128, 4, 7, 96, 0),
                                          (128, 4, 10, 96, 0), (256, 3, 9, 96, 0),
                                          (128, 6, 8, 96, 0), (128, 4, 12, 640, 5),
                                          (64, 3, 11, 640, 3)])
def test_bpr_adam_step_equals_k3_k5(dev, d, T, s, Bc, few):
    c = build_case(dev, d, T, s, Bc, few)
    r = run_k35(c)
    torch.cuda.synchronize()
    check_k35(c, r)


def test_bpr_adam_step_rejects_bad_tables(dev):
    from recbole_amd._native import NativeError
    d, Bc, T = 64, 8, 2
    p = torch.zeros(10, d, device=dev)
    g = _grouping(torch.zeros(Bc, dtype=torch.int64, device=dev), 10)
    tabs = ops.adam_tables([{'p': p, 'm': p, 'v': p, 'grouping': g,
                             'last': torch.zeros(10, dtype=torch.int32, device=dev)}] * 2)
    consts = _consts(dev)
    base = torch.zeros(1, dtype=torch.int32, device=dev)
    z = torch.zeros(3 * Bc, dtype=torch.int64, device=dev)
    recs = ops.step_records(z[:Bc], z, 1, Bc, T, 10, 10, g, _grouping(z, 10))
    with pytest.raises(NativeError):            # no parity buffer
        ops.bpr_adam_step(tabs, [Bc, 3 * Bc], d, z, Bc, T, 0.1, torch.zeros(Bc, device=dev), recs,
                          ops.step_scratch(Bc, T, d, dev), consts, base)
