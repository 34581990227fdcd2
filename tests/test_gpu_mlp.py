"""K10 (csrc/mlp.hip): DeepFM's deep part — MLPLayers (Dropout -> Linear -> ReLU,
reference layers.py:30-86) + the prediction Linear — against a float64 torch-CPU
restatement of the same modules with the dropout masks of the draw specification
(tests/mlp_spec.py). Tolerances (fp32 MFMA vs fp64): outputs and gradients 1e-4
relative + 1e-5 absolute. The masks themselves are checked exactly (any flipped
element moves the fp64 comparison by far more than the tolerance, and the saved
layer-0 mask is compared bit for bit)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from recbole_amd.model.layers import MLPLayers
from recbole_amd.model import mlp as k10
from tests.mlp_spec import keep_mask

pytestmark = pytest.mark.gpu


def _modules(dims, out, p, dev, seed=7):
    torch.manual_seed(seed)
    mlp = MLPLayers(dims, p).to(dev)
    pred = nn.Linear(dims[-1], out).to(dev)
    for m in list(mlp.modules()) + [pred]:
        if isinstance(m, nn.Linear):
            nn.init.xavier_normal_(m.weight)
            nn.init.normal_(m.bias, std=0.1)
    return mlp, pred


def _reference(mlp, pred, x, masks, p):
    """float64 forward with explicit masks (None: no dropout)."""
    lins = [m for m in mlp.mlp_layers if isinstance(m, nn.Linear)]
    h = x.double()
    scale = np.float32(1.0 / (1.0 - p)) if masks is not None else None
    params = []
    for l, m in enumerate(lins):
        W = m.weight.detach().cpu().double().requires_grad_(True)
        b = m.bias.detach().cpu().double().requires_grad_(True)
        params += [W, b]
        if masks is not None:
            h = h * torch.from_numpy(masks[l]).double() * float(scale)
        h = torch.relu(h @ W.t() + b)
    W = pred.weight.detach().cpu().double().requires_grad_(True)
    b = pred.bias.detach().cpu().double().requires_grad_(True)
    params += [W, b]
    return h @ W.t() + b, params


@pytest.mark.parametrize('dims,out,B,p', [([624, 128, 128, 128], 1, 2048, 0.2),
                                          ([624, 128, 128, 128], 1, 2048, 0.0),
                                          ([40, 24, 8], 3, 37, 0.5),
                                          ([16, 256], 1, 300, 0.1),
                                          # wide layer 0 (>= 256): ragged rows, column
                                          # groups and K halves, 2 and 3 layers
                                          ([520, 72, 36], 3, 300, 0.3),
                                          ([272, 12], 5, 37, 0.0),
                                          ([960, 20], 1, 129, 0.5)])
def test_fused_deep_matches_reference(dev, dims, out, B, p):
    mlp, pred = _modules(dims, out, p, dev)
    mlp.train()
    x = torch.randn(B, dims[0], device=dev, requires_grad=True)
    assert k10.fused_supported(mlp, pred, x)
    st = k10._state(mlp, dev)
    c0 = int(st.counter.item())
    y = k10.fused_deep(mlp, pred, x)
    assert int(st.counter.item()) == c0 + (1 if p > 0 else 0)
    gy = torch.randn_like(y)
    y.backward(gy)
    masks = None
    if p > 0:
        thr = k10.keep_threshold(p)
        masks = [keep_mask(st.seed, c0, l, B, dims[l], thr) for l in range(len(dims))]
        frac = masks[0].mean()
        assert abs(frac - (1 - p)) < 0.02 + 3 / np.sqrt(masks[0].size)
    xr = x.detach().cpu().double().requires_grad_(True)
    yr, params = _reference(mlp, pred, xr, masks, p)
    yr.backward(gy.cpu().double())
    torch.testing.assert_close(y.detach().cpu().double(), yr.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(x.grad.cpu().double(), xr.grad, rtol=1e-4, atol=1e-5)
    lins = [m for m in mlp.mlp_layers if isinstance(m, nn.Linear)] + [pred]
    for l, m in enumerate(lins):
        torch.testing.assert_close(m.weight.grad.cpu().double(), params[2 * l].grad,
                                   rtol=1e-4, atol=1e-5, msg=f'dW{l}')
        torch.testing.assert_close(m.bias.grad.cpu().double(), params[2 * l + 1].grad,
                                   rtol=1e-4, atol=1e-5, msg=f'db{l}')


def test_masks_change_per_forward_and_eval_has_none(dev):
    dims = [64, 32]
    mlp, pred = _modules(dims, 1, 0.3, dev)
    x = torch.randn(128, 64, device=dev)
    mlp.train()
    with torch.no_grad():
        y1 = k10.fused_deep(mlp, pred, x)
        y2 = k10.fused_deep(mlp, pred, x)
    assert not torch.equal(y1, y2)                 # counter advanced: new masks
    mlp.eval()
    with torch.no_grad():
        ye = k10.fused_deep(mlp, pred, x)
        yt = pred(mlp(x))
    torch.testing.assert_close(ye, yt, rtol=1e-4, atol=1e-5)


def test_fixed_order_is_run_to_run_identical(dev):
    dims = [624, 128, 128, 128]
    mlp, pred = _modules(dims, 1, 0.0, dev)
    x = torch.randn(2048, 624, device=dev, requires_grad=True)
    grads = []
    for _ in range(2):
        for m in list(mlp.parameters()) + list(pred.parameters()):
            m.grad = None
        x.grad = None
        k10.fused_deep(mlp, pred, x).sum().backward()
        grads.append([x.grad.clone()] + [m.grad.clone() for m in
                                         list(mlp.parameters()) + list(pred.parameters())])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_saved_layer0_mask_is_the_spec(dev):
    dims, B, p = [48, 16], 33, 0.25
    mlp, pred = _modules(dims, 1, p, dev)
    mlp.train()
    x = torch.randn(B, 48, device=dev, requires_grad=True)
    st = k10._state(mlp, dev)
    c0 = int(st.counter.item())
    y = k10.fused_deep(mlp, pred, x)
    m0 = y.grad_fn.keep[-1].cpu().numpy().astype(bool)
    np.testing.assert_array_equal(m0, keep_mask(st.seed, c0, 0, B, 48, k10.keep_threshold(p)))
