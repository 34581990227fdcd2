"""mirec_linear_grad_finish_f32 (csrc/context.hip): the tail of nn.Linear's backward over
SASRec's tall inputs (reference layers.py:338-461 through torch's Linear backward) —
the sum of the split-K weight-gradient partials (in partial order: bit for bit the
sequential float32 sum) and the bias column sum (fixed chunk order: run-to-run
identical, within 1e-5 of float64) — and _SplitKLinearFn's gradients against
nn.Linear's."""
import numpy as np
import pytest
import torch

from recbole_amd import ops
from recbole_amd._native import check, lib, ptr, stream_handle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('C,n_out,n_in,K', [(32, 128, 128, 102400), (1, 256, 128, 70001),
                                            (8, 384, 128, 4096), (2, 4, 8, 3)])
def test_finish_sums(dev, C, n_out, n_in, K):
    g = torch.Generator(device='cpu').manual_seed(C * 7 + K)
    P = torch.randn(C, n_out, n_in, generator=g).to(dev)
    G = torch.randn(K, n_out, generator=g).to(dev)
    outs = []
    for _ in range(2):
        dW = P[0].clone() if C == 1 else torch.empty(n_out, n_in, device=dev)
        src = dW if C == 1 else P
        db = torch.empty(n_out, device=dev)
        scratch = torch.empty(lib().mirec_linear_grad_finish_scratch(K, n_out), device=dev)
        check(lib().mirec_linear_grad_finish_f32(ptr(src), C, n_out * n_in, ptr(dW), ptr(G), K,
                                                 n_out, ptr(db), ptr(scratch),
                                                 ptr(ops.finish_ticket(dev, 'linear')),
                                                 stream_handle()), 'finish')
        outs.append((dW, db))
    torch.cuda.synchronize()
    ref = P[0].cpu().numpy().copy()
    for c in range(1, C):
        ref = ref + P[c].cpu().numpy()                    # float32, c order
    assert np.array_equal(outs[0][0].cpu().numpy(), ref)
    want = G.double().sum(0).cpu()
    torch.testing.assert_close(outs[0][1].double().cpu(), want, rtol=1e-5, atol=1e-5 * K ** 0.5)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert int(ops.finish_ticket(dev, 'linear').item()) == 0


def test_splitk_linear_matches_nn_linear(dev):
    from recbole_amd.model.layers import linear
    torch.manual_seed(3)
    lin = torch.nn.Linear(128, 256).to(dev)
    x = torch.randn(2048, 50, 128, device=dev, requires_grad=True)
    gy = torch.randn(2048, 50, 256, device=dev)
    y = linear(lin, x)
    y.backward(gy)
    got = (x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone())
    x.grad = None
    lin.weight.grad = lin.bias.grad = None
    lin(x).backward(gy)
    # dW and db sum 102,400 rows (|values| ~ 300): another summation order than the
    # library GEMM's moves them by a few fp32 ulps of that magnitude
    for a, b, atol in zip(got, (x.grad, lin.weight.grad, lin.bias.grad), (1e-3, 2e-2, 2e-2)):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=atol)
