"""K11 (csrc/linear.hip): nn.Linear over tall inputs on fp32 MFMA — the forward
y = x W^T + b and the data gradient dx = dy W — against float64 torch at every built width
pair, row counts around the 128-row tile (1, 127, 128, 129, 5,000 and 40,000), with and
without bias; and SASRec's Linear autograd Function (K11 + the split-K weight gradient)
against torch autograd. fp32 tolerance 1e-4 relative / 1e-5 absolute."""
import pytest
import torch

pytestmark = pytest.mark.gpu

WIDTHS = [(64, 64), (64, 128), (64, 256), (128, 64), (128, 128), (128, 256), (256, 64),
          (256, 128)]


@pytest.mark.parametrize('K,N', WIDTHS)
@pytest.mark.parametrize('M', [1, 127, 129, 5000])
def test_k11_forward_and_data_grad(dev, K, N, M):
    from recbole_amd.model import layers
    g = torch.Generator().manual_seed(K * 7 + N + M)
    x = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    gy = torch.randn(M, N, generator=g)
    xd, Wd, bd, gd = (t.to(dev) for t in (x, W, b, gy))
    for bias in (bd, None):
        y = layers.linear_rows(xd, Wd, bias).cpu()
        want = x.double() @ W.double().t() + (b.double() if bias is not None else 0)
        torch.testing.assert_close(y, want.float(), rtol=1e-4, atol=1e-5)
    gx = layers.linear_rows_grad(gd, Wd).cpu()
    torch.testing.assert_close(gx, (gy.double() @ W.double()).float(), rtol=1e-4, atol=1e-5)


def test_k11_tall_rows_and_layout(dev):
    """40,000 rows (the persistent tile loop runs several tiles per workgroup) and a
    3-D input [B, L, K] as the transformer passes it."""
    from recbole_amd.model import layers
    g = torch.Generator().manual_seed(1)
    x = torch.randn(800, 50, 128, generator=g)
    W = torch.randn(256, 128, generator=g) / 128 ** 0.5
    b = torch.randn(256, generator=g)
    y = layers.linear_rows(x.to(dev), W.to(dev), b.to(dev)).cpu()
    assert y.shape == (800, 50, 256)
    torch.testing.assert_close(y, (x.double() @ W.double().t() + b.double()).float(),
                               rtol=1e-4, atol=1e-5)


def test_k11_linear_function_matches_autograd(dev):
    """layers.linear (K11 forward + data gradient, split-K weight gradient) equals torch's
    nn.Linear forward and all three gradients."""
    from recbole_amd.model import layers
    torch.manual_seed(0)
    lin = torch.nn.Linear(128, 256).to(dev)
    x = torch.randn(400, 50, 128, device=dev, requires_grad=True)
    gy = torch.randn(400, 50, 256, device=dev)
    y = layers.linear(lin, x)
    y.backward(gy)
    got = [y.detach().cpu(), x.grad.cpu(), lin.weight.grad.cpu(), lin.bias.grad.cpu()]
    x.grad = None
    lin.zero_grad()
    xr = x.detach().cpu().double().requires_grad_()
    Wr = lin.weight.detach().cpu().double().requires_grad_()
    br = lin.bias.detach().cpu().double().requires_grad_()
    yr = torch.nn.functional.linear(xr, Wr, br)
    yr.backward(gy.cpu().double())
    # dW and db sum 20,000 rows (entries ~ 1e2): fp32 accumulation, absolute slack scaled
    for a, e, atol in zip(got, [yr.detach(), xr.grad, Wr.grad, br.grad], (1e-5, 1e-5, 2e-3, 2e-3)):
        torch.testing.assert_close(a, e.float(), rtol=1e-4, atol=atol)


def test_k11_data_grad_accumulates(dev):
    """mirec_linear_bwd_data_f32 with accumulate: gx += gy W (in place)."""
    from recbole_amd.model import layers
    g = torch.Generator().manual_seed(9)
    gy = torch.randn(3000, 128, generator=g)
    W = torch.randn(128, 64, generator=g) / 8
    prev = torch.randn(3000, 64, generator=g)
    acc = prev.to(dev)
    out = layers.linear_rows_grad(gy.to(dev), W.to(dev), acc=acc)
    assert out.data_ptr() == acc.data_ptr()
    torch.testing.assert_close(out.cpu(), (prev.double() + gy.double() @ W.double()).float(),
                               rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize('with_res', [True, False])
def test_qkv_fn_matches_three_linears(dev, with_res):
    """_QKVFn (the three projections, one accumulated input gradient) equals three
    separate nn.Linear calls: outputs and all seven gradients; its fourth output (x, the
    block's residual input) brings its gradient into the same buffer (with_res), or is
    left unused."""
    from recbole_amd.model import layers
    torch.manual_seed(1)
    lins = [torch.nn.Linear(128, 128).to(dev) for _ in range(3)]
    x = torch.randn(400, 50, 128, device=dev, requires_grad=True)
    gs = [torch.randn(400, 50, 128, device=dev) for _ in range(4)]
    outs = layers._QKVFn.apply(x, *[p for l in lins for p in (l.weight, l.bias)])
    n = 4 if with_res else 3
    torch.autograd.backward(outs[:n], gs[:n])
    got = [o.detach().cpu() for o in outs[:3]] + [x.grad.cpu()] + \
        [p.grad.cpu() for l in lins for p in (l.weight, l.bias)]
    xr = x.detach().cpu().double().requires_grad_()
    ps = [p.detach().cpu().double().requires_grad_() for l in lins for p in (l.weight, l.bias)]
    refs = [torch.nn.functional.linear(xr, ps[2 * i], ps[2 * i + 1]) for i in range(3)]
    torch.autograd.backward(refs + [xr] * (n - 3), [t.cpu().double() for t in gs[:n]])
    want = [r.detach() for r in refs] + [xr.grad] + [p.grad for p in ps]
    atols = [1e-5] * 4 + [2e-3] * 6          # weight / bias grads sum 20,000 rows
    for a, e, atol in zip(got, want, atols):
        torch.testing.assert_close(a, e.float(), rtol=1e-4, atol=atol)


@pytest.mark.parametrize('n_in,n_out', [(128, 256), (128, 128)])
def test_linear_res_fn_matches_linear_plus_residual(dev, n_in, n_out):
    """_LinearResFn (FeedForward's dense_1 with its input passed through for the residual):
    x's gradient = gy W + the residual's gradient, accumulated in K11's epilogue."""
    from recbole_amd.model import layers
    torch.manual_seed(2)
    lin = torch.nn.Linear(n_in, n_out).to(dev)
    x = torch.randn(400, 50, n_in, device=dev, requires_grad=True)
    gy, gr = torch.randn(400, 50, n_out, device=dev), torch.randn(400, 50, n_in, device=dev)
    y, res = layers._LinearResFn.apply(x, lin.weight, lin.bias)
    assert torch.equal(res, x)
    gr0 = gr.clone()
    torch.autograd.backward([y, res], [gy, gr])
    assert torch.equal(gr, gr0)               # the handed-over gradient is not written
    xr = x.detach().cpu().double().requires_grad_()
    W, b = (t.detach().cpu().double().requires_grad_() for t in (lin.weight, lin.bias))
    yr = torch.nn.functional.linear(xr, W, b)
    torch.autograd.backward([yr, xr], [gy.cpu().double(), gr.cpu().double()])
    torch.testing.assert_close(y.detach().cpu(), yr.detach().float(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(x.grad.cpu(), xr.grad.float(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(lin.weight.grad.cpu(), W.grad.float(), rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(lin.bias.grad.cpu(), b.grad.float(), rtol=1e-4, atol=2e-3)
