"""K9e (csrc/attn.hip): the attention core of MultiHeadAttention (reference
recbole/model/layers.py:338-407) against a float64 torch restatement of the same lines
(scores = q k^T / sqrt(dh) + mask; softmax; dropout; @ v; permute + view), forward and
all three input gradients: fp32 tolerance 1e-4 relative / 2e-5 absolute. With dropout the
restatement applies the keep bits the kernel saved (their layout: csrc/attn.hip header),
and the draws are checked for rate, freshness per forward (device counter) and
reproducibility."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _mask(B, L, g, kind):
    if kind == 'sasrec':                    # sasrec.py get_attention_mask: causal x padding
        lens = torch.randint(1, L + 1, (B,), generator=g)
        seq = (torch.arange(L)[None, :] < lens[:, None]).long()
        ext = seq[:, None, None, :] * (torch.triu(torch.ones(L, L), 1) == 0).long()[None, None]
        return (1.0 - ext.float()) * -10000.0
    return torch.randn(B, 1, L, L, generator=g)     # any additive mask


def _ref(q, k, v, mask, H, keep=None, p=0.0):
    B, L, D = q.shape
    dh = D // H
    t = lambda x: x.view(B, L, H, dh).permute(0, 2, 1, 3)
    s = t(q) @ t(k).transpose(-1, -2) / np.sqrt(dh) + mask
    pr = torch.softmax(s, -1)
    if keep is not None:
        pr = pr * keep / (1 - p)
    return (pr @ t(v)).permute(0, 2, 1, 3).reshape(B, L, D)


def _keep_from_words(words, B, H, L):
    """[B*H, 64] uint64 ballot words -> [B, H, L, L] keep mask (word (w*4+c)*4+r, bit
    li + 16*lk holds row 16w + 4lk + r, column 16c + li)."""
    w = words.cpu().numpy().view(np.uint64).reshape(B * H, 4, 4, 4)
    bits = ((w[..., None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)
    keep = np.zeros((B * H, 64, 64), bool)
    for wv in range(4):
        for c in range(4):
            for r in range(4):
                for lk in range(4):
                    keep[:, 16 * wv + 4 * lk + r, 16 * c:16 * c + 16] = \
                        bits[:, wv, c, r, 16 * lk:16 * lk + 16]
    return torch.as_tensor(keep[:, :L, :L].reshape(B, H, L, L))


def _run(dev, q, k, v, mask, H, p=0.0, rng=None, g=None):
    from recbole_amd._native import check, lib, ptr
    B, L, _ = q.shape
    qd, kd, vd = (x.to(dev).contiguous() for x in (q, k, v))
    md = mask.to(dev).contiguous()
    out = torch.full_like(qd, 7.0)
    lse = torch.empty(B * H, 64, device=dev)
    keep = torch.zeros(B * H, 64, dtype=torch.int64, device=dev) if p > 0 else None
    seed, counter, _ = rng if p > 0 else (0, None, None)
    st = torch.cuda.current_stream(dev).cuda_stream
    check(lib().mirec_attn_fwd_f32(ptr(qd), ptr(kd), ptr(vd), ptr(md), B, L, H, p, seed,
                                   ptr(counter) if p > 0 else None, ptr(out), ptr(lse),
                                   ptr(keep) if p > 0 else None, st), 'attn_fwd')
    res = {'out': out, 'keep': keep}
    if g is not None:
        gd = g.to(dev).contiguous()
        dq, dk, dv = (torch.full_like(qd, 7.0) for _ in range(3))
        check(lib().mirec_attn_bwd_f32(ptr(qd), ptr(kd), ptr(vd), ptr(md), ptr(gd), ptr(lse),
                                       ptr(keep) if p > 0 else None,
                                       ptr(counter) if p > 0 else None, B, L, H, p, ptr(dq),
                                       ptr(dk), ptr(dv), st), 'attn_bwd')
        res.update(dq=dq, dk=dk, dv=dv)
    torch.cuda.synchronize(dev)
    return {k_: (x.cpu() if x is not None else None) for k_, x in res.items()}


def _check(got, want, name):
    torch.testing.assert_close(got, want.float(), rtol=1e-4, atol=2e-5, msg=name)


@pytest.mark.parametrize('B,L,H,kind', [(37, 50, 2, 'sasrec'), (5, 64, 1, 'sasrec'),
                                        (9, 1, 2, 'sasrec'), (16, 17, 3, 'random'),
                                        (3, 33, 2, 'random')])
def test_k9e_matches_restatement(dev, B, L, H, kind):
    g = torch.Generator().manual_seed(B * 100 + L)
    q, k, v = (torch.randn(B, L, H * 64, generator=g) for _ in range(3))
    mask = _mask(B, L, g, kind)
    go = torch.randn(B, L, H * 64, generator=g)
    got = _run(dev, q, k, v, mask, H, g=go)
    qq, kk, vv = (x.double().requires_grad_() for x in (q, k, v))
    want = _ref(qq, kk, vv, mask.double(), H)
    want.backward(go.double())
    _check(got['out'], want.detach(), 'out')
    _check(got['dq'], qq.grad, 'dq')
    _check(got['dk'], kk.grad, 'dk')
    _check(got['dv'], vv.grad, 'dv')


def test_k9e_dropout(dev):
    B, L, H, p = 24, 50, 2, 0.3
    g = torch.Generator().manual_seed(5)
    q, k, v = (torch.randn(B, L, H * 64, generator=g) for _ in range(3))
    mask = _mask(B, L, g, 'sasrec')
    go = torch.randn(B, L, H * 64, generator=g)
    rng = (12345, torch.zeros(1, dtype=torch.int64, device=dev),
           torch.zeros(1, dtype=torch.int32, device=dev))
    got = _run(dev, q, k, v, mask, H, p, rng, go)
    assert int(rng[1].item()) == 1      # the backward advanced the counter
    keep = _keep_from_words(got['keep'], B, H, L)
    rate = keep.float().mean().item()
    assert abs(rate - (1 - p)) < 0.01, rate
    qq, kk, vv = (x.double().requires_grad_() for x in (q, k, v))
    want = _ref(qq, kk, vv, mask.double(), H, keep.double(), p)
    want.backward(go.double())
    _check(got['out'], want.detach(), 'out')
    _check(got['dq'], qq.grad, 'dq')
    _check(got['dk'], kk.grad, 'dk')
    _check(got['dv'], vv.grad, 'dv')
    # the next forward draws a new mask; the same counter value draws the same one
    again = _run(dev, q, k, v, mask, H, p, rng)
    assert not torch.equal(again['keep'], got['keep'])
    rng[1].fill_(0)
    same = _run(dev, q, k, v, mask, H, p, rng)
    assert torch.equal(same['keep'], got['keep']) and torch.equal(same['out'], got['out'])


def test_multihead_attention_module_k9e(dev):
    """MultiHeadAttention through K9e equals the torch path (SDPA) of the same module,
    eval mode, forward and parameter gradients."""
    from recbole_amd.model import layers
    torch.manual_seed(3)
    m = layers.MultiHeadAttention(2, 128, 0.0, 0.0, 1e-12).to(dev).eval()
    B, L = 19, 50
    g = torch.Generator().manual_seed(4)
    x = torch.randn(B, L, 128, generator=g).to(dev)
    mask = _mask(B, L, g, 'sasrec').to(dev)
    outs = []
    for k9e in (True, False):
        layers.K9E = k9e
        try:
            m.zero_grad()
            y = m(x, mask)
            y.square().sum().backward()
            outs.append((y.detach().cpu(), [p.grad.detach().cpu().clone() for p in m.parameters()]))
        finally:
            layers.K9E = True
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-4, atol=2e-5)
    for a, b in zip(outs[0][1], outs[1][1]):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4)


def test_sasrec_attention_mask_kernel_bitwise(dev):
    """SASRec.get_attention_mask on the GPU (one launch) equals the reference's seven-op
    construction (sasrec.py:91-105) bit for bit, -0.0 entries included."""
    g = torch.Generator().manual_seed(8)
    B, L = 33, 50
    lens = torch.randint(0, L + 1, (B,), generator=g)
    seq = torch.randint(1, 1000, (B, L), generator=g) * (torch.arange(L)[None, :] < lens[:, None])
    seq[3, 7] = 0                                   # a gap inside a sequence
    ext = (seq > 0).long()[:, None, None, :] * \
        (torch.triu(torch.ones((1, L, L)), diagonal=1) == 0).unsqueeze(1).long()
    want = (1.0 - ext.to(torch.float32)) * -10000.0
    from recbole_amd._native import check, lib, ptr
    got = torch.empty(B, 1, L, L, device=dev)
    sd = seq.to(dev)
    check(lib().mirec_seq_attn_mask_f32(ptr(sd), B, L, ptr(got),
                                        torch.cuda.current_stream(dev).cuda_stream), 'mask')
    assert torch.equal(got.cpu().view(torch.int32), want.view(torch.int32))
