"""Autograd wrappers of the K8 kernels (csrc/context.hip) for ContextRecommender.

_CtxFMFn:      field embeddings of a batch -> (concat [B, F, d], y_fm [B]) where
               y_fm = first-order term + FM second-order term; backward gives the
               dense gradients nn.Embedding(sparse=False) would (zero tables +
               K2-grouped, fixed-order scatter of the per-contribution rows).
_SigmoidBCEFn: mean BCE of sigmoid(y_fm + y_deep) (deepfm.py:66-73).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from recbole_amd import ops
from recbole_amd._native import CtxField, check, lib, ptr, stream_handle

TOKEN, TOKEN_SEQ, FLOAT = 0, 1, 2


class FieldLayout:
    """The concat-order field list of a ContextRecommender: (kind, name, index)
    with index = token field number / token_seq field number / float column."""

    def __init__(self, token_names, seq_names, float_names, token_offsets):
        self.token_names = list(token_names)
        self.seq_names = list(seq_names)
        self.float_names = list(float_names)
        self.token_offsets = [int(x) for x in token_offsets] if len(token_names) else []
        # field-major keys (id + offset) then fall in increasing, disjoint ranges per field
        self.blocks_ok = all(a < b for a, b in zip(self.token_offsets, self.token_offsets[1:]))
        self.n_fields = len(self.token_names) + len(self.seq_names) + len(self.float_names)
        self._dev_offsets = {}

    def offsets_on(self, device):
        """token_offsets as an int64 device tensor (uploaded once per device: a
        pageable host-to-device copy per step would stall the stream)."""
        t = self._dev_offsets.get(device)
        if t is None:
            t = torch.as_tensor(self.token_offsets, dtype=torch.int64, device=device)
            self._dev_offsets[device] = t
        return t


def _col(interaction, name, dtype):
    t = interaction[name]
    if t.dtype != dtype:
        t = t.to(dtype)
    return t.contiguous()


def build_fields(layout, interaction, tables, grads=None):
    """ctypes array of mirec_ctx_field (host) + the tensors it points at.
    tables: dict T, T1, Ef, Ef1, seq (list), seq1 (list) of weight tensors."""
    arr = (CtxField * layout.n_fields)()
    keep = []
    f = 0
    for i, name in enumerate(layout.token_names):
        ids = _col(interaction, name, torch.int64)
        keep.append(ids)
        fd = arr[f]
        fd.kind, fd.seq_len, fd.ids, fd.offset = TOKEN, 1, ptr(ids), layout.token_offsets[i]
        fd.table, fd.table1, fd.n_rows = ptr(tables['T']), ptr(tables['T1']), tables['T'].shape[0]
        if grads is not None:
            d = tables['T'].shape[1]
            fd.grad = ptr(grads['T']) + 4 * i * grads['B'] * d
            fd.grad1 = ptr(grads['T1']) + 4 * i * grads['B']
            fd.keys = ptr(grads['keys']) + 8 * i * grads['B']
            fd.grad_ld, fd.grad1_ld = d, 1
        f += 1
    for i, name in enumerate(layout.seq_names):
        ids = _col(interaction, name, torch.int64)
        keep.append(ids)
        fd = arr[f]
        fd.kind, fd.seq_len, fd.ids = TOKEN_SEQ, ids.shape[1], ptr(ids)
        fd.table, fd.table1 = ptr(tables['seq'][i]), ptr(tables['seq1'][i])
        fd.n_rows = tables['seq'][i].shape[0]
        if grads is not None:
            fd.grad, fd.grad1 = ptr(grads['seq'][i]), ptr(grads['seq1'][i])
        f += 1
    n_float = len(layout.float_names)
    for j, name in enumerate(layout.float_names):
        vals = _col(interaction, name, torch.float32).view(-1)
        keep.append(vals)
        fd = arr[f]
        fd.kind, fd.seq_len, fd.vals, fd.offset = FLOAT, 1, ptr(vals), j
        fd.table, fd.table1 = ptr(tables['Ef']), ptr(tables['Ef1'])
        fd.n_rows = tables['Ef'].shape[0]
        if grads is not None:
            d = tables['Ef'].shape[1]
            fd.grad = ptr(grads['Ef']) + 4 * j * d
            fd.grad1 = ptr(grads['Ef1']) + 4 * j
            fd.grad_ld, fd.grad1_ld = n_float * d, n_float
        f += 1
    return arr, keep


def _upload(arr, device):
    """The batch's field descriptors to the device through kernel arguments
    (mirec_write_bytes): stream-ordered with no host staging buffer to recycle, and
    recorded by value when the step is being captured into a graph."""
    raw = bytes(arr)
    n = (len(raw) + 3) // 4 * 4
    out = torch.empty(max(n, 4), dtype=torch.uint8, device=device)
    buf = ctypes.create_string_buffer(raw, n)
    check(lib().mirec_write_bytes(ptr(out), buf, n, stream_handle()), 'mirec_write_bytes')
    return out


def _grad_buffers(layout, interaction, B, d, keys, dev):
    """The backward's per-contribution gradient buffers (written by K8's backward)."""
    nt, nf = len(layout.token_names), len(layout.float_names)
    E = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)
    seq_ids = [_col(interaction, n, torch.int64) for n in layout.seq_names]
    return {'B': B, 'keys': keys,
            'T': E(nt * B, d) if nt else None, 'T1': E(nt * B, 1) if nt else None,
            'Ef': E(B, nf * d) if nf else None, 'Ef1': E(B, nf) if nf else None,
            'seq': [E(ids.numel(), d) for ids in seq_ids],
            'seq1': [E(ids.numel(), 1) for ids in seq_ids]}


def ctx_fm_forward(layout, interaction, tables, B, d, bias, keys=None, grads=None):
    """K8 forward. grads (the backward's buffers, _grad_buffers): the field descriptors
    then also carry the gradient pointers, so the backward reuses them (one descriptor
    upload per step instead of two)."""
    dev = bias.device
    arr, keep = build_fields(layout, interaction, tables, grads)
    if keys is not None and grads is None:
        for i in range(len(layout.token_names)):
            arr[i].keys = ptr(keys) + 8 * i * B
    fields_dev = _upload(arr, dev)
    concat = torch.empty(B, layout.n_fields, d, dtype=torch.float32, device=dev)
    y_fm = torch.empty(B, dtype=torch.float32, device=dev)
    # first-order terms + FM sums of the batch: written here, read by the backward
    work = torch.empty(max(1, lib().mirec_ctx_fm_work_floats(B, layout.n_fields, d)),
                       dtype=torch.float32, device=dev)
    with ops.timed_launch('ctx_fm_fwd'):
        rc = lib().mirec_ctx_fm_fwd_f32(ptr(fields_dev), layout.n_fields, B, d, ptr(bias),
                                        ptr(concat), ptr(y_fm), ptr(work), stream_handle())
    check(rc, "mirec_ctx_fm_fwd_f32")
    keep.append(fields_dev)
    keep.append(work)
    return concat, y_fm, keep


class _CtxFMFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, layout, interaction, T, T1, Ef, Ef1, bias, *seq_tables):
        ns = len(layout.seq_names)
        seq, seq1 = list(seq_tables[:ns]), list(seq_tables[ns:])
        d = (T if T is not None else (Ef if Ef is not None else seq[0])).shape[1]
        B = interaction.length
        tables = {'T': T, 'T1': T1, 'Ef': Ef, 'Ef1': Ef1, 'seq': seq, 'seq1': seq1}
        tables = {k: (v.detach() if isinstance(v, torch.Tensor) else
                      [x.detach() for x in v] if isinstance(v, list) else v)
                  for k, v in tables.items()}
        keys = torch.empty(len(layout.token_names) * B, dtype=torch.int64, device=bias.device)
        h = getattr(T, '_mirec_deferred', None) if T is not None else None
        h1 = getattr(T1, '_mirec_deferred', None) if T1 is not None else None
        # the first-order [V, 1] table is read by the same keys: caught up with T (one
        # launch, mirec_adam_deferred_pair_f32) when the same optimizer runs both
        pair = T1 if (h1 is not None and h1 is h) else None
        if h is not None:                     # deferred Adam: complete the rows read
            # keys[f*B + i] = id + the field's table offset, every field in one launch
            cols = [_col(interaction, n, torch.int64) for n in layout.token_names]
            nt = len(cols)
            status = getattr(h, '_sort_status', None)
            if (layout.blocks_ok and 0 < B <= ops.CHAIN_MAX_BLOCK_N and 1 < nt <= 64
                    and status is not None and status.numel() > nt):
                # the keys formed and grouped (one LDS sort per field block, chained) in
                # one launch
                keys, segs = ops.segment_sort_fields(cols, layout.token_offsets, B, T.shape[0],
                                                     status)
                ctx.segs = h.catch_up(T, keys, segs=segs, pair=pair)
            else:
                cptr = (ctypes.c_void_p * nt)(*[ptr(x) for x in cols])
                offs = (ctypes.c_int64 * nt)(*layout.token_offsets)
                check(lib().mirec_offset_keys(cptr, offs, nt, B, ptr(keys), stream_handle()),
                      'mirec_offset_keys')
                # one key block per field (ranges increase with the field offsets): K2
                # sorts each field's B keys in LDS instead of a device-wide radix sort
                blocks = B if (layout.blocks_ok and 0 < B <= 8192 and nt > 1) else None
                ctx.segs = h.catch_up(T, keys, blocks=blocks, pair=pair)
            if h1 is not None and pair is None:   # the first-order [V, 1] table, same rows
                h1.catch_up(T1, keys, ctx.segs)
        else:
            ctx.segs = None
            h1 = None
        grads = None
        if any(ctx.needs_input_grad[2:]):
            grads = _grad_buffers(layout, interaction, B, d, keys, bias.device)
        concat, y_fm, keep = ctx_fm_forward(layout, interaction, tables, B, d, bias.detach(), keys,
                                            grads)
        ctx.fm_work, ctx.fields_dev, ctx.grads, ctx.keep = keep[-1], keep[-2], grads, keep
        ctx.layout, ctx.interaction, ctx.tables, ctx.B, ctx.d = layout, interaction, tables, B, d
        ctx.deferred_T = T if h is not None else None
        ctx.deferred_T1 = T1 if h1 is not None else None
        ctx.save_for_backward(concat, keys)
        return concat, y_fm

    @staticmethod
    def backward(ctx, g_concat, g_fm):
        concat, keys = ctx.saved_tensors
        if ctx.keep is None:        # the descriptors point into buffers the first backward freed
            raise RuntimeError('K8 context fields: backward through the same graph a second '
                               'time is not supported (its saved buffers were released)')
        layout, tables, B, d = ctx.layout, ctx.tables, ctx.B, ctx.d
        dev = concat.device
        nt, ns, nf = len(layout.token_names), len(layout.seq_names), len(layout.float_names)
        if g_fm is None:
            g_fm = torch.zeros(B, dtype=torch.float32, device=dev)
        g_fm = g_fm.contiguous()
        seq_ids = [_col(ctx.interaction, n, torch.int64) for n in layout.seq_names]
        grads, fields_dev = ctx.grads, ctx.fields_dev    # descriptors of the forward
        gc = None if g_concat is None else g_concat.contiguous()
        with ops.timed_launch('ctx_fm_bwd'):
            rc = lib().mirec_ctx_fm_bwd_f32(ptr(fields_dev), layout.n_fields, B, d, ptr(concat),
                                            ptr(gc), ptr(g_fm), ptr(ctx.fm_work),
                                            stream_handle())
        check(rc, "mirec_ctx_fm_bwd_f32")
        dT = dT1 = dEf = dEf1 = None
        if nt:
            T = tables['T']
            segs = ctx.segs if ctx.segs is not None else ops.segment_sort(keys, T.shape[0])
            if ctx.deferred_T is not None:    # compact rows to the deferred optimizer
                ctx.deferred_T._mirec_deferred.stash(ctx.deferred_T, grads['T'], keys, segs)
            else:
                dT = ops.segment_scatter_add(grads['T'], segs, torch.zeros_like(T))
            if ctx.deferred_T1 is not None:
                ctx.deferred_T1._mirec_deferred.stash(ctx.deferred_T1, grads['T1'], keys, segs)
            else:
                dT1 = ops.segment_scatter_add(grads['T1'], segs, torch.zeros_like(tables['T1']))
        # the float-field, first-order float and bias gradients: column sums, one launch
        dbias = torch.empty(1, dtype=torch.float32, device=dev)
        jobs = [(g_fm, 1, dbias)]
        if nf:
            dEf = torch.empty_like(tables['Ef'])
            dEf1 = torch.empty_like(tables['Ef1'])
            jobs = [(grads['Ef'], nf * d, dEf), (grads['Ef1'], nf, dEf1)] + jobs
        nj = len(jobs)
        check(lib().mirec_colsum_multi_f32((ctypes.c_void_p * nj)(*[ptr(j[0]) for j in jobs]),
                                           (ctypes.c_int64 * nj)(*[B] * nj),
                                           (ctypes.c_int64 * nj)(*[j[1] for j in jobs]),
                                           (ctypes.c_void_p * nj)(*[ptr(j[2]) for j in jobs]),
                                           nj, stream_handle()), "mirec_colsum_multi_f32")
        dseq, dseq1 = [], []
        for i, ids in enumerate(seq_ids):
            segs = ops.segment_sort(ids.view(-1), tables['seq'][i].shape[0])
            dseq.append(ops.segment_scatter_add(grads['seq'][i], segs,
                                                torch.zeros_like(tables['seq'][i])))
            dseq1.append(ops.segment_scatter_add(grads['seq1'][i], segs,
                                                 torch.zeros_like(tables['seq1'][i])))
        ctx.keep = ctx.grads = ctx.fields_dev = None      # the forward's buffers: done
        return (None, None, dT, dT1, dEf, dEf1, dbias, *dseq, *dseq1)


_UNIT = {}


def unit_grad(device):
    """A persistent 0-dim 1.0 per device. backward() seeded with it hands this very tensor
    to the loss Function at the root (autograd passes the seed object through sums), which
    then skips multiplying its gradient by the seed (x * 1 = x exactly): one launch fewer
    per step. Allocate it outside any graph capture."""
    key = str(device)
    if key not in _UNIT:
        _UNIT[key] = torch.ones((), dtype=torch.float32, device=device)
    return _UNIT[key]


class _SigmoidBCEFn(torch.autograd.Function):
    """nn.BCELoss()(sigmoid(y_fm + y_deep), label) (deepfm.py:45, 66-73): loss terms, their
    fixed-order mean and the logit gradient in one launch (mirec_sigmoid_bce_mean_f32)."""

    @staticmethod
    def forward(ctx, y_fm, y_deep, label):
        B = y_fm.numel()
        yd = y_deep.detach().reshape(-1).contiguous()
        lab = label.detach().to(torch.float32).contiguous()
        loss = torch.empty((), dtype=torch.float32, device=y_fm.device)
        dz = torch.empty(B, dtype=torch.float32, device=y_fm.device)
        gs = float(np.float32(1.0) / np.float32(B))
        rc = lib().mirec_sigmoid_bce_mean_f32(ptr(y_fm.detach().contiguous()), ptr(yd), ptr(lab),
                                              B, gs, None, ptr(loss), ptr(dz), stream_handle())
        check(rc, "mirec_sigmoid_bce_mean_f32")
        ctx.save_for_backward(dz)
        ctx.deep_shape = y_deep.shape
        return loss

    @staticmethod
    def backward(ctx, g):
        (dz,) = ctx.saved_tensors
        if g is not _UNIT.get(str(g.device)):      # the unit seed: dz * 1 = dz
            dz = dz * g
        return dz, dz.view(ctx.deep_shape), None


def sigmoid_prob(y_fm, y_deep):
    """sigmoid(y_fm + y_deep) on the device (DeepFM.forward's output)."""
    B = y_fm.numel()
    yd = None if y_deep is None else y_deep.detach().reshape(-1).contiguous()
    prob = torch.empty(B, dtype=torch.float32, device=y_fm.device)
    rc = lib().mirec_sigmoid_bce_f32(ptr(y_fm.detach().contiguous()), ptr(yd), None, B, 1.0,
                                     ptr(prob), None, None, stream_handle())
    check(rc, "mirec_sigmoid_bce_f32")
    return prob
