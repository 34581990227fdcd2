"""Layers used by the context-aware path (mirror of recbole/model/layers.py:30-171,
905-1062). Same module structure, parameter names and construction order as the
reference, so checkpoints interoperate and the CPU-generator draws of module
construction and init line up.

The DeepFM hot path does not call FMEmbedding / FMFirstOrderLinear /
BaseFactorizationMachine forward: ContextRecommender runs all three in the
fused K8 kernel (csrc/context.hip) over these modules' weights. Their forward
methods remain, in torch ops, for user code that composes them directly.
"""
import copy
import math

import numpy as np
import torch
import torch.nn as nn
from torch.nn.init import normal_

from recbole_amd import ops
from recbole_amd._native import check, lib, ptr, stream_handle
from recbole_amd.utils import FeatureType


def activation_layer(activation_name='relu', emb_dim=None):
    """layers.py:89-118."""
    if activation_name is None:
        return None
    if isinstance(activation_name, str):
        name = activation_name.lower()
        if name == 'sigmoid':
            return nn.Sigmoid()
        if name == 'tanh':
            return nn.Tanh()
        if name == 'relu':
            return nn.ReLU()
        if name == 'leakyrelu':
            return nn.LeakyReLU()
        if name == 'none':
            return None
        raise NotImplementedError(f'activation function {activation_name} is not implemented')
    if issubclass(activation_name, nn.Module):
        return activation_name()
    raise NotImplementedError(f'activation function {activation_name} is not implemented')


class MLPLayers(nn.Module):
    """[Dropout -> Linear -> (BatchNorm) -> activation] per layer (layers.py:30-86)."""

    def __init__(self, layers, dropout=0., activation='relu', bn=False, init_method=None):
        super().__init__()
        self.layers = layers
        self.dropout = dropout
        self.activation = activation
        self.use_bn = bn
        self.init_method = init_method
        mods = []
        for input_size, output_size in zip(self.layers[:-1], self.layers[1:]):
            mods.append(nn.Dropout(p=self.dropout))
            mods.append(nn.Linear(input_size, output_size))
            if self.use_bn:
                mods.append(nn.BatchNorm1d(num_features=output_size))
            act = activation_layer(self.activation, output_size)
            if act is not None:
                mods.append(act)
        self.mlp_layers = nn.Sequential(*mods)
        if self.init_method is not None:
            self.apply(self.init_weights)

    def init_weights(self, module):
        if isinstance(module, nn.Linear):
            if self.init_method == 'norm':
                normal_(module.weight.data, 0, 0.01)
            if module.bias is not None:
                module.bias.data.fill_(0.0)

    def forward(self, input_feature):
        return self.mlp_layers(input_feature)


class FMEmbedding(nn.Module):
    """One table for all token fields, field f's ids shifted by offsets[f]
    (layers.py:121-144)."""

    def __init__(self, field_dims, offsets, embed_dim):
        super().__init__()
        self.embedding = nn.Embedding(int(sum(field_dims)), embed_dim)
        self.offsets = offsets

    def forward(self, input_x):
        input_x = input_x + input_x.new_tensor(self.offsets).unsqueeze(0)
        return self.embedding(input_x)


class BaseFactorizationMachine(nn.Module):
    """0.5 * ((sum_f e)^2 - sum_f e^2), summed over the embedding axis when
    reduce_sum (layers.py:147-171)."""

    def __init__(self, reduce_sum=True):
        super().__init__()
        self.reduce_sum = reduce_sum

    def forward(self, input_x):
        square_of_sum = torch.sum(input_x, dim=1) ** 2
        sum_of_square = torch.sum(input_x ** 2, dim=1)
        output = square_of_sum - sum_of_square
        if self.reduce_sum:
            output = torch.sum(output, dim=1, keepdim=True)
        return 0.5 * output


def _split_fields(config, dataset):
    """Token / token_seq / float field names and sizes in dataset.fields() order,
    the label skipped (abstract_recommender.py:185-200, layers.py:913-928)."""
    label = config['LABEL_FIELD']
    tok, tok_dims, seq, seq_dims, flt, flt_dims = [], [], [], [], [], []
    for name in dataset.fields():
        if name == label:
            continue
        ftype = dataset.field2type[name]
        if ftype == FeatureType.TOKEN:
            tok.append(name)
            tok_dims.append(dataset.num(name))
        elif ftype == FeatureType.TOKEN_SEQ:
            seq.append(name)
            seq_dims.append(dataset.num(name))
        else:
            flt.append(name)
            flt_dims.append(dataset.num(name))
    return tok, tok_dims, seq, seq_dims, flt, flt_dims


class FMFirstOrderLinear(nn.Module):
    """First-order weights of every field + a bias (layers.py:905-1062)."""

    def __init__(self, config, dataset, output_dim=1):
        super().__init__()
        self.field_names = dataset.fields()
        self.LABEL = config['LABEL_FIELD']
        self.device = config['device']
        (self.token_field_names, self.token_field_dims, self.token_seq_field_names,
         self.token_seq_field_dims, self.float_field_names,
         self.float_field_dims) = _split_fields(config, dataset)
        if len(self.token_field_dims) > 0:
            self.token_field_offsets = np.array((0, *np.cumsum(self.token_field_dims)[:-1]),
                                                dtype=np.int64)
            self.token_embedding_table = FMEmbedding(self.token_field_dims,
                                                     self.token_field_offsets, output_dim)
        if len(self.float_field_dims) > 0:
            self.float_embedding_table = nn.Embedding(int(np.sum(self.float_field_dims)),
                                                      output_dim)
        if len(self.token_seq_field_dims) > 0:
            self.token_seq_embedding_table = nn.ModuleList()
            for dim in self.token_seq_field_dims:
                self.token_seq_embedding_table.append(nn.Embedding(dim, output_dim))
        self.bias = nn.Parameter(torch.zeros((output_dim,)), requires_grad=True)


def _wgrad(x, gy, W, has_b):
    """(dW, db) of y = x W^T + b over the rows of x: the weight gradient dW = dY^T X as a
    batched GEMM over C row blocks, then summed — the library picks a 32x32-tile kernel for
    the single [out, K] x [K, in] product, which leaves most CUs idle at K = 10^5 (SASRec
    on C3); C blocks give C times the tiles — with the bias column sum in the same finish
    launch."""
    n_in, n_out = W.shape[1], W.shape[0]
    x2 = x.reshape(-1, n_in)
    g2 = gy.reshape(-1, n_out)
    K = x2.shape[0]
    C = 1
    while K % (2 * C) == 0 and K // (2 * C) >= 2048 and C < 64:
        C *= 2
    if C > 1:
        P = torch.bmm(g2.view(C, K // C, n_out).transpose(1, 2), x2.view(C, K // C, n_in))
        dW = torch.empty_like(W)
    else:
        P = dW = g2.t().mm(x2)
    db = None
    if has_b and (n_out % 4 or n_in % 4):        # outside the finish kernel's shapes
        if C > 1:
            dW = P.sum(0)
        return dW, g2.sum(0)
    if has_b or C > 1:
        # the C partials' sum and the bias column sum in one launch (two torch
        # reductions before)
        g2 = g2.contiguous()
        if has_b:
            db = torch.empty(n_out, dtype=torch.float32, device=gy.device)
        scratch = torch.empty(max(lib().mirec_linear_grad_finish_scratch(K, n_out), 2),
                              dtype=torch.float32, device=gy.device)
        check(lib().mirec_linear_grad_finish_f32(
            ptr(P), C, n_out * n_in, ptr(dW), ptr(g2), K, n_out, ptr(db) if db is not None
            else None, ptr(scratch), ptr(ops.finish_ticket(gy.device, 'linear')),
            stream_handle()), 'mirec_linear_grad_finish_f32')
    return dW, db


class _SplitKLinearFn(torch.autograd.Function):
    """nn.Linear over tall inputs: forward and input gradient through K11
    (linear_rows / linear_rows_grad), weight and bias gradients through _wgrad."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return linear_rows(x, W, b)

    @staticmethod
    def backward(ctx, gy):
        x, W = ctx.saved_tensors
        dx = linear_rows_grad(gy, W)
        dW, db = _wgrad(x, gy, W, ctx.has_b)
        return dx, dW, db


class _LinearResFn(torch.autograd.Function):
    """_SplitKLinearFn whose input also feeds a residual (FeedForward: dense_1(x) and the
    LayerNorm(... + x)): the second output is x itself (a view), and the backward adds
    gy W to that output's gradient in K11's epilogue (mirec_linear_bwd_data_acc_f32, into
    a new buffer: the handed-over gradient is not written) — autograd's add of the two
    input gradients (a [B L, d] torch add per block) goes."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return linear_rows(x, W, b), x.view_as(x)

    @staticmethod
    def backward(ctx, gy, gres):
        x, W = ctx.saved_tensors
        dx = linear_rows_grad(gy.contiguous(), W, acc=gres, in_place=False)
        dW, db = _wgrad(x, gy, W, ctx.has_b)
        return dx, dW, db


class _QKVFn(torch.autograd.Function):
    """The query / key / value Linears of MultiHeadAttention over one input (layers.py
    :338-407): three K11 products forward; backward, the input gradient of all three in
    one buffer — dx = gq Wq, then += gk Wk, += gv Wv in K11's accumulating epilogue —
    instead of three buffers and autograd's two adds. The fourth output is x itself (a
    view) for the block's residual LayerNorm; the first product starts from its gradient
    (read by K11's epilogue into a new buffer, as _LinearResFn), so that add goes too."""

    @staticmethod
    def forward(ctx, x, Wq, bq, Wk, bk, Wv, bv):
        ctx.save_for_backward(x, Wq, Wk, Wv)
        ctx.has_b = (bq is not None, bk is not None, bv is not None)
        return (linear_rows(x, Wq, bq), linear_rows(x, Wk, bk), linear_rows(x, Wv, bv),
                x.view_as(x))

    @staticmethod
    def backward(ctx, gq, gk, gv, gres):
        x, Wq, Wk, Wv = ctx.saved_tensors
        dx, own = gres, False                 # own: dx is this backward's buffer
        out = []
        for g, W, hb in ((gq, Wq, ctx.has_b[0]), (gk, Wk, ctx.has_b[1]), (gv, Wv, ctx.has_b[2])):
            if g is None:
                out += [None, None]
                continue
            g = g.contiguous()
            dx = linear_rows_grad(g, W, acc=dx, in_place=own)
            own = True
            out += list(_wgrad(x, g, W, hb))
        if dx is None:
            dx = torch.zeros_like(x)
        return (dx, *out)


def linear(module, x):
    """module(x): K11 for tall GPU inputs (with the split-K weight gradient when training)."""
    if x.is_cuda and x.numel() // x.shape[-1] >= 16384:
        if x.requires_grad or module.weight.requires_grad and torch.is_grad_enabled():
            return _SplitKLinearFn.apply(x, module.weight, module.bias)
        return linear_rows(x, module.weight, module.bias)
    return module(x)


K11 = True      # the tall Linears through K11 (csrc/linear.hip) where the widths allow


def _k11(x, n_in, n_out):
    """K11 where its widths allow (C3 step trace: the four 128 x 128 products 68-80 -> 49 us
    each; the 256-wide forward / data-gradient four 72-124 -> 82-88 us, 362 -> 340 us in
    all)."""
    return (K11 and x.is_cuda and x.dtype == torch.float32 and x.data_ptr() % 16 == 0
            and lib().mirec_linear_shape_ok(n_in, n_out) != 0)


def linear_rows(x, W, b):
    """x W^T + b over the rows of x (K11 where it applies, else the library)."""
    n_out, n_in = W.shape
    if not _k11(x, n_in, n_out):
        return nn.functional.linear(x, W, b)
    x2 = x.reshape(-1, n_in).contiguous()
    y = torch.empty(x2.shape[0], n_out, dtype=torch.float32, device=x.device)
    check(lib().mirec_linear_fwd_f32(ptr(x2), x2.shape[0], n_in, n_out, ptr(W.detach().contiguous()),
                                     ptr(b.detach()) if b is not None else None, ptr(y),
                                     stream_handle()), 'mirec_linear_fwd_f32')
    return y.view(*x.shape[:-1], n_out)


def linear_rows_grad(gy, W, acc=None, in_place=True):
    """dL/dx = gy W of linear_rows (K11 where it applies, else the library); acc: a
    previous input gradient of the same shape, added to — in place (in_place: a buffer
    of the caller's own), or into a new buffer (a gradient autograd handed over, which
    must not be written: mirec_linear_bwd_data_acc_f32 reads it in the epilogue)."""
    n_out, n_in = W.shape
    if not _k11(gy, n_in, n_out):
        gx = torch.matmul(gy, W)
        if acc is None:
            return gx
        return acc.add_(gx) if in_place else acc + gx
    g2 = gy.reshape(-1, n_out).contiguous()
    Wc = W.detach().contiguous()
    if acc is not None and not in_place:
        a2 = acc.reshape(-1, n_in).contiguous()
        assert a2.shape[0] == g2.shape[0]
        gx = torch.empty(g2.shape[0], n_in, dtype=torch.float32, device=gy.device)
        check(lib().mirec_linear_bwd_data_acc_f32(ptr(g2), g2.shape[0], n_out, n_in, ptr(Wc),
                                                  ptr(a2), ptr(gx), stream_handle()),
              'mirec_linear_bwd_data_acc_f32')
        return gx.view(*gy.shape[:-1], n_in)
    if acc is None:
        gx = torch.empty(g2.shape[0], n_in, dtype=torch.float32, device=gy.device)
    else:
        gx = acc.view(-1, n_in)
        assert gx.is_contiguous() and gx.shape[0] == g2.shape[0]
    check(lib().mirec_linear_bwd_data_f32(ptr(g2), g2.shape[0], n_out, n_in, ptr(Wc), ptr(gx),
                                          int(acc is not None), stream_handle()),
          'mirec_linear_bwd_data_f32')
    return gx.view(*gy.shape[:-1], n_in)


def colsums(jobs):
    """Column sums of up to four [n, m] row-major buffers in ONE launch
    (mirec_colsum_multi_f32: each job with mirec_colsum_f32's tile, the same bits);
    jobs = [(x, n, m, out)]. The LayerNorm backwards' dgamma / dbeta (and K9a's dP) went
    as one launch each (11 colsum launches of ~7.6 us a C3 step)."""
    import ctypes
    nj = len(jobs)
    check(lib().mirec_colsum_multi_f32((ctypes.c_void_p * nj)(*[ptr(j[0]) for j in jobs]),
                                       (ctypes.c_int64 * nj)(*[j[1] for j in jobs]),
                                       (ctypes.c_int64 * nj)(*[j[2] for j in jobs]),
                                       (ctypes.c_void_p * nj)(*[ptr(j[3]) for j in jobs]),
                                       nj, stream_handle()), 'mirec_colsum_multi_f32')


class _AddLNFn(torch.autograd.Function):
    """LayerNorm(a + b) (K9d, mirec_add_ln_fwd/bwd_f32): the residual sum is never
    materialised; the backward returns the same dx for both inputs."""

    @staticmethod
    def forward(ctx, a, b, gamma, beta, eps):
        a, b = a.contiguous(), b.contiguous()
        d = a.shape[-1]
        n = a.numel() // d
        out = torch.empty_like(a)
        mean = torch.empty(n, dtype=torch.float32, device=a.device)
        rstd = torch.empty(n, dtype=torch.float32, device=a.device)
        check(lib().mirec_add_ln_fwd_f32(ptr(a), ptr(b), n, d, ptr(gamma.detach()),
                                         ptr(beta.detach()), eps, ptr(out), ptr(mean),
                                         ptr(rstd), stream_handle()), 'mirec_add_ln_fwd_f32')
        ctx.save_for_backward(a, b, gamma, mean, rstd)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b, gamma, mean, rstd = ctx.saved_tensors
        d = a.shape[-1]
        n = a.numel() // d
        parts = lib().mirec_seq_embed_ln_partials(n)
        dx = torch.empty_like(a)
        pg = torch.empty(parts, d, dtype=torch.float32, device=a.device)
        pb = torch.empty(parts, d, dtype=torch.float32, device=a.device)
        check(lib().mirec_add_ln_bwd_f32(ptr(a), ptr(b), n, d, ptr(gamma.detach()), ptr(mean),
                                         ptr(rstd), ptr(g.contiguous()), ptr(dx), ptr(pg),
                                         ptr(pb), stream_handle()), 'mirec_add_ln_bwd_f32')
        dgamma = torch.empty_like(gamma)
        dbeta = torch.empty_like(gamma)
        colsums([(pg, parts, d, dgamma), (pb, parts, d, dbeta)])
        return dx, dx, dgamma, dbeta, None


class _AddLNDropFn(torch.autograd.Function):
    """LayerNorm(dropout(a) + b) (K9d with the dropout folded in, mirec_add_ln_drop_fwd/bwd_f32):
    no dropped copy of a in HBM, no separate dropout kernels; rng = (seed, device counter,
    unused) of the calling module; the backward advances the counter."""

    @staticmethod
    def forward(ctx, a, b, gamma, beta, eps, p, rng):
        a, b = a.contiguous(), b.contiguous()
        d = a.shape[-1]
        n = a.numel() // d
        out = torch.empty_like(a)
        mean = torch.empty(n, dtype=torch.float32, device=a.device)
        rstd = torch.empty(n, dtype=torch.float32, device=a.device)
        drawn = torch.empty(1, dtype=torch.int64, device=a.device)
        seed, counter, _ = rng
        check(lib().mirec_add_ln_drop_fwd_f32(ptr(a), ptr(b), n, d, ptr(gamma.detach()),
                                              ptr(beta.detach()), eps, float(p), seed,
                                              ptr(counter), ptr(drawn), ptr(out), ptr(mean),
                                              ptr(rstd), stream_handle()),
              'mirec_add_ln_drop_fwd_f32')
        ctx.save_for_backward(a, b, gamma, mean, rstd, drawn)
        ctx.p, ctx.seed, ctx.counter = p, seed, counter
        return out

    @staticmethod
    def backward(ctx, g):
        a, b, gamma, mean, rstd, drawn = ctx.saved_tensors
        d = a.shape[-1]
        n = a.numel() // d
        parts = lib().mirec_seq_embed_ln_partials(n)
        dxa, dxb = torch.empty_like(a), torch.empty_like(a)
        pg = torch.empty(parts, d, dtype=torch.float32, device=a.device)
        pb = torch.empty(parts, d, dtype=torch.float32, device=a.device)
        check(lib().mirec_add_ln_drop_bwd_f32(ptr(a), ptr(b), n, d, ptr(gamma.detach()),
                                              ptr(mean), ptr(rstd), ptr(g.contiguous()),
                                              float(ctx.p), ctx.seed, ptr(drawn),
                                              ptr(ctx.counter), ptr(dxa), ptr(dxb), ptr(pg),
                                              ptr(pb), stream_handle()),
              'mirec_add_ln_drop_bwd_f32')
        dgamma = torch.empty_like(gamma)
        dbeta = torch.empty_like(gamma)
        colsums([(pg, parts, d, dgamma), (pb, parts, d, dbeta)])
        return dxa, dxb, dgamma, dbeta, None, None, None


_DROP_SITES = [0]


def _drop_rng(owner, dev):
    """(seed, device draw counter, ticket) of a module's folded dropout: the seed from the
    device generator's initial seed (no CPU generator draw) and the module's index."""
    st = getattr(owner, '_ln_drop_rng', None)
    if st is None or st[1].device != dev:
        if not hasattr(owner, '_ln_drop_index'):
            owner._ln_drop_index = _DROP_SITES[0]
            _DROP_SITES[0] += 1
        seed = (torch.cuda.default_generators[dev.index or 0].initial_seed() * 0x85EBCA6B
                + 0x1000 + owner._ln_drop_index) & ((1 << 64) - 1)
        st = (seed, torch.zeros(1, dtype=torch.int64, device=dev),
              torch.zeros(1, dtype=torch.int32, device=dev))
        owner._ln_drop_rng = st
    return st


K9D_DROP = True     # the hidden dropout before add_layer_norm folded into K9d


def add_layer_norm(hidden, input_tensor, ln, drop=None, owner=None):
    """ln(drop(hidden) + input_tensor) — the fused K9d kernel on the GPU (fp32, d in
    {32, 64, 128, 256}; drop: the nn.Dropout on hidden, folded in while training with
    p > 0), the modules themselves otherwise."""
    fused = (hidden.is_cuda and hidden.dtype == torch.float32
             and hidden.shape[-1] in (32, 64, 128, 256) and ln.elementwise_affine
             and hidden.shape == input_tensor.shape)
    p = drop.p if (drop is not None and drop.training) else 0.0
    if fused and p > 0 and K9D_DROP and p < 1:
        rng = _drop_rng(owner if owner is not None else drop, hidden.device)
        out = _AddLNDropFn.apply(hidden, input_tensor, ln.weight, ln.bias, float(ln.eps), p, rng)
        if not out.requires_grad:             # no backward will advance the draw counter
            rng[1].add_(1)
        return out
    if drop is not None:
        hidden = drop(hidden)
    if fused:
        return _AddLNFn.apply(hidden, input_tensor, ln.weight, ln.bias, float(ln.eps))
    return ln(hidden + input_tensor)


class _GeluFn(torch.autograd.Function):
    """x * 0.5 * (1 + erf(x / sqrt(2))) and its derivative, one kernel each."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        check(lib().mirec_gelu_fwd_f32(ptr(x), x.numel(), ptr(y), stream_handle()),
              'mirec_gelu_fwd_f32')
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, g):
        x, = ctx.saved_tensors
        dx = torch.empty_like(x)
        check(lib().mirec_gelu_bwd_f32(ptr(x), ptr(g.contiguous()), x.numel(), ptr(dx),
                                       stream_handle()), 'mirec_gelu_bwd_f32')
        return dx


SDPA = True     # fallback for shapes K9e does not take: torch's fused scaled_dot_product_attention
K9E = True      # MultiHeadAttention's core through K9e (csrc/attn.hip) where it applies
_ATTN_MODULES = [0]


class _AttnFn(torch.autograd.Function):
    """K9e (csrc/attn.hip): softmax(q k^T / sqrt(dh) + mask) -> dropout(p) -> @ v for the
    [B, L, H*64] Linear outputs q, k, v (L <= 64), the context returned as [B, L, H*64]
    (the reference's permute(0, 2, 1, 3) + view, layers.py:391-397, without the copy).
    rng = (seed, device counter, unused) when p > 0; the backward advances the counter."""

    @staticmethod
    def forward(ctx, q, k, v, mask, H, p, rng):
        B, L, _ = q.shape
        out = torch.empty_like(q)
        lse = torch.empty(B * H, 64, dtype=torch.float32, device=q.device)
        keep = torch.empty(B * H, 64, dtype=torch.int64, device=q.device) if p > 0 else None
        seed, counter, _ = rng if p > 0 else (0, None, None)
        check(lib().mirec_attn_fwd_f32(ptr(q), ptr(k), ptr(v), ptr(mask), B, L, H, float(p),
                                       seed, ptr(counter) if p > 0 else None, ptr(out), ptr(lse),
                                       ptr(keep) if p > 0 else None, stream_handle()),
              'mirec_attn_fwd_f32')
        ctx.save_for_backward(q, k, v, mask, lse, keep)
        ctx.H, ctx.p, ctx.counter = H, p, counter
        return out

    @staticmethod
    def backward(ctx, g):
        q, k, v, mask, lse, keep = ctx.saved_tensors
        B, L, _ = q.shape
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        check(lib().mirec_attn_bwd_f32(ptr(q), ptr(k), ptr(v), ptr(mask), ptr(g.contiguous()),
                                       ptr(lse), ptr(keep) if keep is not None else None,
                                       ptr(ctx.counter) if keep is not None else None, B, L,
                                       ctx.H, float(ctx.p), ptr(dq), ptr(dk), ptr(dv),
                                       stream_handle()), 'mirec_attn_bwd_f32')
        return dq, dk, dv, None, None, None, None


def attn_k9e_applies(q, mask, n_heads, head_size):
    """K9e's shapes: fp32 CUDA [B, L, H*64] with L <= 64 and a float32 additive mask of
    B*L*L elements ([B, 1, L, L], contiguous) that needs no gradient."""
    if not (K9E and q.is_cuda and q.dtype == torch.float32 and q.dim() == 3 and head_size == 64
            and 1 <= q.shape[1] <= 64 and q.shape[2] == n_heads * 64):
        return False
    B, L = q.shape[0], q.shape[1]
    return (isinstance(mask, torch.Tensor) and mask.dtype == torch.float32 and mask.is_cuda
            and mask.is_contiguous() and mask.numel() == B * L * L and not mask.requires_grad
            and tuple(mask.shape[-2:]) == (L, L))


class MultiHeadAttention(nn.Module):
    """layers.py:338-407 (same parameters and op sequence; library GEMMs)."""

    def __init__(self, n_heads, hidden_size, hidden_dropout_prob, attn_dropout_prob,
                 layer_norm_eps):
        super().__init__()
        if hidden_size % n_heads != 0:
            raise ValueError(f'The hidden size ({hidden_size}) is not a multiple of the number '
                             f'of attention heads ({n_heads})')
        self.num_attention_heads = n_heads
        self.attention_head_size = int(hidden_size / n_heads)
        self.all_head_size = self.num_attention_heads * self.attention_head_size
        self.query = nn.Linear(hidden_size, self.all_head_size)
        self.key = nn.Linear(hidden_size, self.all_head_size)
        self.value = nn.Linear(hidden_size, self.all_head_size)
        self.attn_dropout = nn.Dropout(attn_dropout_prob)
        self.dense = nn.Linear(hidden_size, hidden_size)
        self.LayerNorm = nn.LayerNorm(hidden_size, eps=layer_norm_eps)
        self.out_dropout = nn.Dropout(hidden_dropout_prob)
        self._attn_index = _ATTN_MODULES[0]    # K9e dropout stream of this module
        _ATTN_MODULES[0] += 1
        self._attn_rng = None

    def _k9e_rng(self, dev):
        """(seed, device draw counter, ticket) of this module's K9e dropout: the seed
        from the device generator's initial seed (torch.manual_seed sets it; no CPU
        generator draw, so the reference's CPU random streams are untouched) and the
        module's construction index."""
        if self._attn_rng is None or self._attn_rng[1].device != dev:
            seed = (torch.cuda.default_generators[dev.index or 0].initial_seed()
                    * 0x9E3779B1 + self._attn_index) & ((1 << 64) - 1)
            self._attn_rng = (seed, torch.zeros(1, dtype=torch.int64, device=dev),
                              torch.zeros(1, dtype=torch.int32, device=dev))
        return self._attn_rng

    def transpose_for_scores(self, x):
        x = x.view(*(x.size()[:-1] + (self.num_attention_heads, self.attention_head_size)))
        return x.permute(0, 2, 1, 3)

    def forward(self, input_tensor, attention_mask):
        if (input_tensor.is_cuda and input_tensor.numel() // input_tensor.shape[-1] >= 16384
                and torch.is_grad_enabled() and input_tensor.requires_grad):
            ql, kl, vl, res = _QKVFn.apply(input_tensor, self.query.weight, self.query.bias,
                                           self.key.weight, self.key.bias, self.value.weight,
                                           self.value.bias)
        else:
            res = input_tensor
            ql = linear(self.query, input_tensor)
            kl = linear(self.key, input_tensor)
            vl = linear(self.value, input_tensor)
        if attn_k9e_applies(ql, attention_mask, self.num_attention_heads,
                            self.attention_head_size):
            p = self.attn_dropout.p if self.training else 0.0
            rng = self._k9e_rng(ql.device) if p > 0 else None
            ctx = _AttnFn.apply(ql.contiguous(), kl.contiguous(), vl.contiguous(),
                                attention_mask, self.num_attention_heads, p, rng)
            if rng is not None and not ctx.requires_grad:   # no backward to advance it
                rng[1].add_(1)
            return add_layer_norm(linear(self.dense, ctx), res, self.LayerNorm,
                                  drop=self.out_dropout)
        q = self.transpose_for_scores(ql)
        k = self.transpose_for_scores(kl)
        v = self.transpose_for_scores(vl)
        if input_tensor.is_cuda and SDPA:
            # softmax(q k^T / sqrt(dh) + mask) with dropout on the weights, @ v: the same
            # computation in torch's fused attention (no copies of the permuted q, k, v)
            p = self.attn_dropout.p if self.training else 0.0
            ctx = nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=attention_mask,
                                                             dropout_p=p)
            ctx = ctx.permute(0, 2, 1, 3).contiguous()
        else:
            scores = torch.matmul(q, k.transpose(-1, -2))
            scores = scores / math.sqrt(self.attention_head_size)
            scores = scores + attention_mask
            probs = nn.Softmax(dim=-1)(scores)
            probs = self.attn_dropout(probs)
            ctx = torch.matmul(probs, v).permute(0, 2, 1, 3).contiguous()
        ctx = ctx.view(*(ctx.size()[:-2] + (self.all_head_size,)))
        return add_layer_norm(linear(self.dense, ctx), res, self.LayerNorm,
                              drop=self.out_dropout)


class FeedForward(nn.Module):
    """layers.py:410-461."""

    def __init__(self, hidden_size, inner_size, hidden_dropout_prob, hidden_act, layer_norm_eps):
        super().__init__()
        self.dense_1 = nn.Linear(hidden_size, inner_size)
        self.intermediate_act_fn = self.get_hidden_act(hidden_act)
        self.dense_2 = nn.Linear(inner_size, hidden_size)
        self.LayerNorm = nn.LayerNorm(hidden_size, eps=layer_norm_eps)
        self.dropout = nn.Dropout(hidden_dropout_prob)

    def get_hidden_act(self, act):
        return {'gelu': self.gelu, 'relu': nn.functional.relu, 'swish': self.swish,
                'tanh': torch.tanh, 'sigmoid': torch.sigmoid}[act]

    def gelu(self, x):
        if x.is_cuda and x.dtype == torch.float32:
            return _GeluFn.apply(x)
        return x * 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0)))

    def swish(self, x):
        return x * torch.sigmoid(x)

    def forward(self, input_tensor):
        x = input_tensor
        if (x.is_cuda and x.numel() // x.shape[-1] >= 16384 and torch.is_grad_enabled()
                and x.requires_grad):
            h, res = _LinearResFn.apply(x, self.dense_1.weight, self.dense_1.bias)
        else:
            h, res = linear(self.dense_1, x), x
        hidden = linear(self.dense_2, self.intermediate_act_fn(h))
        return add_layer_norm(hidden, res, self.LayerNorm, drop=self.dropout)


class TransformerLayer(nn.Module):
    """layers.py:464-490."""

    def __init__(self, n_heads, hidden_size, intermediate_size, hidden_dropout_prob,
                 attn_dropout_prob, hidden_act, layer_norm_eps):
        super().__init__()
        self.multi_head_attention = MultiHeadAttention(n_heads, hidden_size, hidden_dropout_prob,
                                                       attn_dropout_prob, layer_norm_eps)
        self.feed_forward = FeedForward(hidden_size, intermediate_size, hidden_dropout_prob,
                                        hidden_act, layer_norm_eps)

    def forward(self, hidden_states, attention_mask):
        return self.feed_forward(self.multi_head_attention(hidden_states, attention_mask))


class TransformerEncoder(nn.Module):
    """layers.py:493-552 (n_layers deep copies of one TransformerLayer)."""

    def __init__(self, n_layers=2, n_heads=2, hidden_size=64, inner_size=256,
                 hidden_dropout_prob=0.5, attn_dropout_prob=0.5, hidden_act='gelu',
                 layer_norm_eps=1e-12):
        super().__init__()
        layer = TransformerLayer(n_heads, hidden_size, inner_size, hidden_dropout_prob,
                                 attn_dropout_prob, hidden_act, layer_norm_eps)
        self.layer = nn.ModuleList([copy.deepcopy(layer) for _ in range(n_layers)])

    def forward(self, hidden_states, attention_mask, output_all_encoded_layers=True):
        out = []
        for layer_module in self.layer:
            hidden_states = layer_module(hidden_states, attention_mask)
            if output_all_encoded_layers:
                out.append(hidden_states)
        if not output_all_encoded_layers:
            out.append(hidden_states)
        return out
