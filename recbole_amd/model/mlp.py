"""Host side of K10 (csrc/mlp.hip): DeepFM's deep part — MLPLayers followed by the
prediction Linear (reference recbole/model/layers.py:30-86, deepfm.py:40-43,61) — as
one forward and two backward launches on fp32 MFMA.

fused_deep(mlp_layers, predict, x) returns predict(mlp_layers(x)) with the same
modules, parameters and autograd semantics: the parameter gradients land in .grad
as nn.Linear's would. Dropout draws come from a counter-based generator (spec in
csrc/mlp.hip, numpy restatement in tests/mlp_spec.py) keyed by torch's initial seed
and a device counter the forward advances, so a captured training step draws new
masks at every replay. Shapes K10 does not cover (another activation, BatchNorm,
widths above 1024 or not multiples of 4) keep the modules' torch path.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.nn as nn

from recbole_amd import ops
from recbole_amd._native import MLP_MAX_LAYERS, MlpDesc, check, lib, ptr, stream_handle


def _linears(mlp_layers, predict):
    lins = [m for m in mlp_layers.mlp_layers if isinstance(m, nn.Linear)]
    return lins + [predict]


def fused_supported(mlp_layers, predict, x) -> bool:
    """K10 covers ReLU MLPLayers without BatchNorm whose widths fit its tiles."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2):
        return False
    if getattr(mlp_layers, 'use_bn', False):
        return False
    act = getattr(mlp_layers, 'activation', 'relu')
    if not (isinstance(act, str) and act.lower() == 'relu'):
        return False
    lins = _linears(mlp_layers, predict)
    if len(lins) > MLP_MAX_LAYERS or not isinstance(predict, nn.Linear):
        return False
    dims = [lins[0].in_features] + [m.out_features for m in lins]
    if any(d < 1 or d > 1024 for d in dims) or any(d % 4 for d in dims[:-1]):
        return False
    if dims[0] != x.shape[1]:
        return False
    # the row-block kernels' two LDS tiles (16 rows each; widths of even / odd index)
    pad = lambda w: (w + 15) // 16 * 16 + 4
    if 16 * 4 * (pad(max(dims[0::2])) + pad(max(dims[1::2]))) > 65536:
        return False
    for m in lins:
        w = m.weight
        if not (w.is_cuda and w.dtype == torch.float32 and w.is_contiguous() and
                w.data_ptr() % 16 == 0):
            return False
    return True


class _State(object):
    """Per-MLPLayers K10 state: the draw counter, the forward's arrival word and the wide
    backward's hand-off counters (zero between launches) on the device."""

    WCOUNT = 4096              # wave tiles of the wide backward's weight gradients, at most

    def __init__(self, device):
        self.counter = torch.zeros(1, dtype=torch.int64, device=device)
        self.arrive = torch.zeros(1, dtype=torch.int32, device=device)
        self.wcount = torch.zeros(self.WCOUNT, dtype=torch.int32, device=device)
        self.seed = int(torch.initial_seed()) & 0xFFFFFFFFFFFFFFFF


def _state(mlp_layers, device):
    st = getattr(mlp_layers, '_mirec_k10', None)
    if st is None or st.counter.device != device:
        st = _State(device)
        mlp_layers._mirec_k10 = st
    return st


def keep_threshold(p):
    """32-bit threshold of Dropout(p): a draw u is kept iff u < threshold."""
    return min(int(np.floor((1.0 - float(p)) * 2.0 ** 32)), 0xFFFFFFFF)


def dropout_scale(p):
    return float(np.float32(1.0 / (1.0 - float(p)))) if p < 1 else 0.0


class _DeepFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, mlp_layers, n_lin, x, *params):
        dev = x.device
        x = x.contiguous()
        B = x.shape[0]
        Ws, bs = params[0::2], params[1::2]
        L = n_lin
        dims = [x.shape[1]] + [w.shape[0] for w in Ws]
        p = float(mlp_layers.dropout)
        train = bool(mlp_layers.training) and p > 0
        d = MlpDesc()
        d.n_layers = L
        for j, v in enumerate(dims):
            d.dims[j] = v
        for l in range(L):
            d.dropout[l] = 1 if (train and l < L - 1) else 0   # the prediction layer: none
            d.relu[l] = 1 if l < L - 1 else 0
            d.W[l] = ptr(Ws[l])
            d.b[l] = ptr(bs[l]) if bs[l] is not None else None
        st = _state(mlp_layers, dev)
        d.keep_threshold = keep_threshold(p) if train else 0xFFFFFFFF
        d.scale = dropout_scale(p) if train else 1.0
        d.seed = st.seed
        d.counter, d.arrive = ptr(st.counter), ptr(st.arrive)
        d.wscratch = d.wcount = None
        E = lambda *s, dt=torch.float32: torch.empty(*s, dtype=dt, device=dev)
        keep = []
        grad = torch.is_grad_enabled() or any(ctx.needs_input_grad)
        if grad or train:
            for l in range(1, L):
                t = E(B, dims[l])
                keep.append(t)
                d.xs[l] = ptr(t)
            if train:
                x0 = E(B, dims[0])
                m0 = E(B, dims[0], dt=torch.uint8)
                keep += [x0, m0]
                d.xs[0], d.mask0 = ptr(x0), ptr(m0)
        y = E(B, dims[L])
        with ops.timed_launch('mlp_fwd'):
            rc = lib().mirec_mlp_fwd_f32(ctypes.byref(d), ptr(x), B, ptr(y), 1 if train else 0,
                                         stream_handle())
        check(rc, 'mirec_mlp_fwd_f32')
        ctx.desc, ctx.keep, ctx.dims, ctx.L, ctx.state = d, keep, dims, L, st
        ctx.has_bias = [b is not None for b in bs]
        ctx.save_for_backward(x, *Ws)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, *Ws = ctx.saved_tensors
        if ctx.keep is None:
            # the descriptor's saved-activation pointers point into ctx.keep, released by
            # the first backward: a second one (retain_graph=True) would read freed memory
            raise RuntimeError('K10 MLP: backward through the same graph a second time is not '
                               'supported (its saved activations were released)')
        d, dims, L = ctx.desc, ctx.dims, ctx.L
        dev, B = x.device, x.shape[0]
        gy = gy.contiguous()
        E = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)
        gz = [E(B, dims[l + 1]) for l in range(L - 1)]
        for l, t in enumerate(gz):
            d.gz[l] = ptr(t)
        dW = [torch.empty_like(w) for w in Ws]
        db = [E(dims[l + 1]) if ctx.has_bias[l] else None for l in range(L)]
        for l in range(L):
            d.dW[l] = ptr(dW[l])
            d.db[l] = ptr(db[l])
        gx = E(B, dims[0])
        # the wide backward (layer 0's data and every weight gradient over the whole chip)
        # hands block partials over through a scratch buffer and zeroed counters
        nf, nc = ctypes.c_int64(0), ctypes.c_int64(0)
        wide = lib().mirec_mlp_bwd_workspace(ctypes.byref(d), B, ctypes.byref(nf), ctypes.byref(nc))
        check(min(wide, 0), 'mirec_mlp_bwd_workspace')
        scratch = None
        if wide == 1 and nc.value <= ctx.state.wcount.numel():
            scratch = E(nf.value)
            d.wscratch, d.wcount = ptr(scratch), ptr(ctx.state.wcount)
        with ops.timed_launch('mlp_bwd'):            # two launches: data, weight gradients
            rc = lib().mirec_mlp_bwd_f32(ctypes.byref(d), ptr(x), ptr(gy), B, ptr(gx),
                                         stream_handle())
        check(rc, 'mirec_mlp_bwd_f32')
        ctx.keep = None
        out = [None, None, gx]
        for l in range(L):
            out += [dW[l], db[l]]
        return tuple(out)


def fused_deep(mlp_layers, predict, x):
    """predict(mlp_layers(x)) through K10 (x: [B, dims[0]] fp32 on the GPU)."""
    lins = _linears(mlp_layers, predict)
    params = []
    for m in lins:
        params += [m.weight, m.bias]
    return _DeepFn.apply(mlp_layers, len(lins), x, *params)


def deep_forward(mlp_layers, predict, x):
    """K10 where it applies, the modules' torch path otherwise."""
    if fused_supported(mlp_layers, predict, x):
        return fused_deep(mlp_layers, predict, x)
    return predict(mlp_layers(x))
