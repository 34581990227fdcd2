"""K9d with the hidden dropout folded in (csrc/seq.hip, mirec_add_ln_drop_fwd/bwd_f32):
LayerNorm(dropout(a) + b) of the transformer blocks (reference layers.py:338-461) against a
float64 torch restatement that applies the keep flags of the kernel's draw specification
(restated in numpy below: key = splitmix64(seed + c), element e kept iff the 32-bit half
e & 1 of splitmix64(key ^ (e >> 1)) is below 2^32 (1 - p)); forward, dA, dB, dgamma, dbeta
(fp32, 1e-4 relative), the drawn word and the backward's advance of the device counter."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix(z):
    with np.errstate(over='ignore'):
        z = (z + np.uint64(0x9E3779B97F4A7C15)) & M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
        return z ^ (z >> np.uint64(31))


def _keep(seed, c, n_elems, p):
    key = _mix(np.uint64((seed + c) & 0xFFFFFFFFFFFFFFFF))
    e = np.arange(n_elems, dtype=np.uint64)
    h = _mix(key ^ (e >> np.uint64(1)))
    half = np.where((e & np.uint64(1)) == 1, h >> np.uint64(32), h & np.uint64(0xFFFFFFFF))
    thr = min(4294967295, int(np.ldexp(1.0 - p, 32)))
    return half < np.uint64(thr)


@pytest.mark.parametrize('d', [64, 128])
@pytest.mark.parametrize('p', [0.1, 0.5])
def test_add_ln_drop_matches_restatement(dev, d, p):
    from recbole_amd._native import check, lib, ptr
    n, eps, seed = 3001, 1e-12, 987654321
    g = torch.Generator().manual_seed(d + int(p * 10))
    a, b, gy = (torch.randn(n, d, generator=g) for _ in range(3))
    gamma, beta = torch.rand(d, generator=g) + 0.5, torch.randn(d, generator=g)
    ad, bd, gd, gmd, btd = (t.to(dev).contiguous() for t in (a, b, gy, gamma, beta))
    counter = torch.full((1,), 41, dtype=torch.int64, device=dev)
    drawn = torch.full((1,), -1, dtype=torch.int64, device=dev)
    out = torch.empty_like(ad)
    mean, rstd = torch.empty(n, device=dev), torch.empty(n, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    L = lib()
    check(L.mirec_add_ln_drop_fwd_f32(ptr(ad), ptr(bd), n, d, ptr(gmd), ptr(btd), eps, p, seed,
                                      ptr(counter), ptr(drawn), ptr(out), ptr(mean), ptr(rstd),
                                      st), 'fwd')
    torch.cuda.synchronize(dev)
    assert int(counter.item()) == 41 and int(drawn.item()) == 41    # read, not advanced
    parts = L.mirec_seq_embed_ln_partials(n)
    dxa, dxb = torch.empty_like(ad), torch.empty_like(ad)
    pg, pb = torch.empty(parts, d, device=dev), torch.empty(parts, d, device=dev)
    check(L.mirec_add_ln_drop_bwd_f32(ptr(ad), ptr(bd), n, d, ptr(gmd), ptr(mean), ptr(rstd),
                                      ptr(gd), p, seed, ptr(drawn), ptr(counter), ptr(dxa),
                                      ptr(dxb), ptr(pg), ptr(pb), st), 'bwd')
    torch.cuda.synchronize(dev)
    assert int(counter.item()) == 42 and int(drawn.item()) == 41   # the backward advanced it
    keep = torch.as_tensor(_keep(seed, 41, n * d, p).reshape(n, d))
    assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    A, B = a.double().requires_grad_(), b.double().requires_grad_()
    G, Bt = gamma.double().requires_grad_(), beta.double().requires_grad_()
    y = torch.nn.functional.layer_norm(A * keep / (1 - p) + B, (d,), G, Bt, eps)
    y.backward(gy.double())
    tol = dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out.cpu(), y.detach().float(), **tol)
    torch.testing.assert_close(dxa.cpu(), A.grad.float(), **tol)
    torch.testing.assert_close(dxb.cpu(), B.grad.float(), **tol)
    torch.testing.assert_close(pg.sum(0).cpu(), G.grad.float(), rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(pb.sum(0).cpu(), Bt.grad.float(), rtol=1e-4, atol=2e-3)


def test_ffn_block_folded_dropout_trains(dev):
    """FeedForward in training mode with dropout 0.3 runs through the folded K9d (the
    module's draw counter advances once per forward + backward, and once per forward under
    no_grad) and its gradients are finite; in eval mode it equals the unfused path."""
    from recbole_amd.model import layers
    torch.manual_seed(5)
    ffn = layers.FeedForward(128, 256, 0.3, 'gelu', 1e-12).to(dev)
    x = torch.randn(300, 50, 128, device=dev, requires_grad=True)
    ffn.train()
    y = ffn(x)
    y.square().mean().backward()
    rng = ffn.dropout._ln_drop_rng
    assert int(rng[1].item()) == 1
    with torch.no_grad():
        ffn(x)
    assert int(rng[1].item()) == 2
    assert torch.isfinite(x.grad).all() and all(torch.isfinite(p.grad).all() for p in ffn.parameters())
    ffn.eval()
    with torch.no_grad():
        a = ffn(x)
        layers.K9D_DROP = False
        try:
            b = ffn(x)
        finally:
            layers.K9D_DROP = True
    torch.testing.assert_close(a, b)


@pytest.mark.parametrize('p', [0.2, 0.5])
def test_seq_embed_ln_drop_matches_restatement(dev, p):
    """K9a with SASRec's embedding dropout folded in (mirec_seq_embed_ln_drop_fwd/bwd_f32,
    through _SeqEmbedLNFn): dropout(LayerNorm(E[seq] + P[t])) of the reference
    sasrec.py:107-114 against float64 torch applying the same keep flags (element index
    (b L + t) d + j); forward and the gradients of E (rows 1..), P, gamma and beta; the
    counter is read by the forward and advanced by the backward."""
    from recbole_amd.model.sequential_recommender.sasrec import _SeqEmbedLNFn
    B, L, d, n_items, eps, seed = 97, 50, 64, 500, 1e-12, 4242
    g = torch.Generator().manual_seed(int(p * 10))
    E, P = torch.randn(n_items, d, generator=g), torch.randn(L, d, generator=g)
    gamma, beta = torch.rand(d, generator=g) + 0.5, torch.randn(d, generator=g)
    seq = torch.randint(0, n_items, (B, L), generator=g)
    gy = torch.randn(B, L, d, generator=g)
    rng = (seed, torch.full((1,), 7, dtype=torch.int64, device=dev))
    Ed, Pd, Gd, Bd = (t.to(dev).requires_grad_() for t in (E, P, gamma, beta))
    y = _SeqEmbedLNFn.apply(Ed, Pd, Gd, Bd, seq.to(dev), eps, p, rng)
    torch.cuda.synchronize(dev)
    assert int(rng[1].item()) == 7
    y.backward(gy.to(dev))
    torch.cuda.synchronize(dev)
    assert int(rng[1].item()) == 8
    keep = torch.as_tensor(_keep(seed, 7, B * L * d, p).reshape(B, L, d))
    assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    E64, P64, G64, B64 = (t.double().requires_grad_() for t in (E, P, gamma, beta))
    x = E64[seq] + P64[None]
    want = torch.nn.functional.layer_norm(x, (d,), G64, B64, eps) * keep / (1 - p)
    want.backward(gy.double())
    tol = dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(y.detach().cpu(), want.detach().float(), **tol)
    torch.testing.assert_close(Ed.grad.cpu()[1:], E64.grad[1:].float(), **tol)
    torch.testing.assert_close(Pd.grad.cpu(), P64.grad.float(), rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(Gd.grad.cpu(), G64.grad.float(), rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(Bd.grad.cpu(), B64.grad.float(), rtol=1e-4, atol=2e-3)
