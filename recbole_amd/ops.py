"""Thin torch-tensor wrappers over the libmirec.so C-ABI (include/mirec.h).

Every device function here launches a hand-written gfx950 kernel on the current
HIP stream. Inputs must already be device tensors of the stated dtype; nothing is
copied to the host and nothing falls back to PyTorch or the CPU — a tensor on
the wrong device or a missing library raises. The host_* functions are the
library's CPU data-pipeline primitives (numpy arrays in and out).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from recbole_amd._native import NativeError, check, lib, ptr, stream_handle

# Per-launch HIP events of named kernels, collected while a dict is installed here
# ({name: [(start, end), ...]}; tools/bench_models.py): the measuring tool times a
# model step's dominant kernel on the stream it runs on. None: no events.
KERNEL_EVENTS = None


class timed_launch(object):
    """`with timed_launch(name): <one native launch>` — records a start / end event pair
    on the current stream when KERNEL_EVENTS holds `name` (nothing otherwise)."""

    def __init__(self, name):
        self.name = name
        self.ev = None

    def __enter__(self):
        if KERNEL_EVENTS is not None and self.name in KERNEL_EVENTS:
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self.ev[0].record()
        return self

    def __exit__(self, *exc):
        if self.ev is not None:
            self.ev[1].record()
            KERNEL_EVENTS[self.name].append(self.ev)
        return False


def _dev(t: torch.Tensor, dtype, name: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise NativeError(f"{name} must live on the GPU (got {t.device}); no CPU fallback exists")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t


# ---------------------------------------------------------------- K4 sampler
def sample_walk(random_list: torch.Tensor, pr_dev: torch.Tensor, keys: torch.Tensor, num: int,
                used_ptr: torch.Tensor | None, used_cols: torch.Tensor | None, n_key_space: int,
                reject: bool, batch_keys: int | None = None, n_batches: int = 1,
                out: torch.Tensor | None = None, status: torch.Tensor | None = None,
                ws: torch.Tensor | None = None, out_stride: int = 0,
                used_bits: torch.Tensor | None = None, n_bits: int = 0) -> torch.Tensor:
    """Bit-exact cyclic-walk negative sampling (sampler.py:82-154). Membership
    comes from `used_bits` (see used_bitmap) when given, else the CSR."""
    _dev(random_list, torch.int32, "random_list")
    _dev(pr_dev, torch.int64, "pr_dev")
    _dev(keys, torch.int64, "keys")
    n_keys = keys.numel()
    if batch_keys is None:
        batch_keys = max(n_keys, 1)
    if out is None:
        out = torch.empty(n_keys * num, dtype=torch.int64, device=keys.device)
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=keys.device)
    if reject and used_bits is None:
        _dev(used_ptr, torch.int64, "used_ptr")
        _dev(used_cols, torch.int32, "used_cols")
    if reject and used_bits is not None:
        _dev(used_bits, torch.int32, "used_bits")
    wsz = lib().mirec_sample_walk_workspace_size(batch_keys, num)
    if ws is None or ws.numel() < wsz:
        ws = torch.empty(wsz, dtype=torch.uint8, device=keys.device)
    bits = reject and used_bits is not None
    rc = lib().mirec_sample_walk(ptr(random_list), random_list.numel(), ptr(pr_dev), ptr(keys),
                                 n_keys, batch_keys, n_batches, num,
                                 ptr(used_ptr) if reject and not bits else None,
                                 ptr(used_cols) if reject and not bits else None,
                                 ptr(used_bits) if bits else None, n_bits if bits else 0,
                                 n_key_space,
                                 1 if reject else 0, ptr(out), out_stride, ptr(status), ptr(ws),
                                 ws.numel(),
                                 stream_handle())
    check(rc, "mirec_sample_walk")
    return out


def sample_walk_spec(random_list: torch.Tensor, pr_dev: torch.Tensor, users: torch.Tensor,
                     batch_keys: int, n_batches: int, num: int, used_ptr, used_cols,
                     n_key_space: int, reject: bool, r_mean: float, r_sd: float,
                     out: torch.Tensor | None = None, out_stride: int = 0, status=None,
                     used_bits=None, n_bits: int = 0, items=None, user_keys=None,
                     item_keys=None, key_stride: int = 0) -> torch.Tensor:
    """K4s (mirec_sample_walk_spec): the walk of n_batches batches of batch_keys keys
    (users[b*batch_keys:]) by speculation — the same values, pointer and status as
    sample_walk, bit for bit; r_mean / r_sd size the windows (Sampler.walk_stats)."""
    _dev(random_list, torch.int32, "random_list")
    _dev(pr_dev, torch.int64, "pr_dev")
    _dev(users, torch.int64, "users")
    dev = users.device
    if out is None:
        out = torch.empty(n_batches * batch_keys * num, dtype=torch.int64, device=dev)
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=dev)
    bits = reject and used_bits is not None
    wsz = lib().mirec_sample_walk_spec_workspace_size(batch_keys, num, min(n_batches, 16),
                                                      r_mean, r_sd)
    ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
    rc = lib().mirec_sample_walk_spec(
        ptr(random_list), random_list.numel(), ptr(pr_dev), ptr(users), ptr(items), n_batches,
        batch_keys, num, ptr(used_ptr) if reject and not bits else None,
        ptr(used_cols) if reject and not bits else None, ptr(used_bits) if bits else None,
        n_bits if bits else 0, n_key_space, 1 if reject else 0, float(r_mean), float(r_sd),
        ptr(out), out_stride, ptr(user_keys), ptr(item_keys), key_stride, ptr(status), ptr(ws),
        ws.numel(), stream_handle())
    check(rc, "mirec_sample_walk_spec")
    return out


def sample_walk_segments(random_list: torch.Tensor, pr_dev: torch.Tensor, keys: torch.Tensor,
                         seg_ptr: torch.Tensor, max_seg_keys: int, num: int,
                         used_ptr: torch.Tensor | None, used_cols: torch.Tensor | None,
                         n_key_space: int, reject: bool, used_bits: torch.Tensor | None = None,
                         n_bits: int = 0, status: torch.Tensor | None = None) -> torch.Tensor:
    """Successive sample_by_key_ids calls, call s over keys[seg_ptr[s]:seg_ptr[s+1]]
    (device int64 seg_ptr), in one launch; values of call s at seg_ptr[s]*num."""
    _dev(random_list, torch.int32, "random_list")
    _dev(pr_dev, torch.int64, "pr_dev")
    _dev(keys, torch.int64, "keys")
    _dev(seg_ptr, torch.int64, "seg_ptr")
    out = torch.empty(keys.numel() * num, dtype=torch.int64, device=keys.device)
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=keys.device)
    bits = reject and used_bits is not None
    if reject and not bits:
        _dev(used_ptr, torch.int64, "used_ptr")
        _dev(used_cols, torch.int32, "used_cols")
    if bits:
        _dev(used_bits, torch.int32, "used_bits")
    ws = torch.empty(lib().mirec_sample_walk_workspace_size(max(max_seg_keys, 1), max(num, 1)),
                     dtype=torch.uint8, device=keys.device)
    rc = lib().mirec_sample_walk_segments(
        ptr(random_list), random_list.numel(), ptr(pr_dev), ptr(keys), ptr(seg_ptr),
        seg_ptr.numel() - 1, max_seg_keys, num,
        ptr(used_ptr) if reject and not bits else None,
        ptr(used_cols) if reject and not bits else None,
        ptr(used_bits) if bits else None, n_bits if bits else 0, n_key_space,
        1 if reject else 0, ptr(out), ptr(status), ptr(ws), ws.numel(), stream_handle())
    check(rc, "mirec_sample_walk_segments")
    return out


def copy_many(dst: list, src: list) -> None:
    """dst[i].copy_(src[i]) for same-size contiguous device tensors, in one launch
    (mirec_copy_many)."""
    n = len(dst)
    if n == 0:
        return
    S = (ctypes.c_void_p * n)()
    D = (ctypes.c_void_p * n)()
    N = (ctypes.c_int64 * n)()
    for i, (d, s) in enumerate(zip(dst, src)):
        if not (d.is_cuda and s.is_cuda and d.is_contiguous() and s.is_contiguous()):
            raise NativeError("copy_many: contiguous device tensors only")
        nb = d.numel() * d.element_size()
        if s.numel() * s.element_size() != nb:
            raise ValueError(f"copy_many: size mismatch at {i}")
        S[i], D[i], N[i] = s.data_ptr(), d.data_ptr(), nb
    check(lib().mirec_copy_many(S, D, N, n, stream_handle()), "mirec_copy_many")


def host_counting_order(keys, key_space: int) -> np.ndarray:
    """Stable sort permutation of integer keys in [0, key_space) (host, O(n))."""
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    order = np.empty(len(keys), dtype=np.int64)
    check(lib().mirec_host_counting_order(keys.ctypes.data, len(keys), int(key_space),
                                          order.ctypes.data), "mirec_host_counting_order")
    return order


def host_csr_build(keys, vals, n_keys: int) -> tuple:
    """(ptr int64[n_keys+1], cols int32) of the distinct (key, value) pairs, each
    row ascending (host, counting pass + per-row sort)."""
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    vals = np.ascontiguousarray(vals, dtype=np.int64)
    ptr = np.empty(int(n_keys) + 1, dtype=np.int64)
    cols = np.empty(max(len(keys), 1), dtype=np.int32)
    nnz = lib().mirec_host_csr_build(keys.ctypes.data, vals.ctypes.data, len(keys), int(n_keys),
                                     ptr.ctypes.data, cols.ctypes.data)
    if nnz < 0:
        check(int(nnz), "mirec_host_csr_build")
    return ptr, cols[:nnz].copy()


def alias_build(counts) -> tuple:
    """Host-side Vose alias table of non-negative integer counts: (thr uint32[n],
    alias int32[n]) numpy arrays (mirec_alias_build)."""
    counts = np.ascontiguousarray(counts, dtype=np.int64)
    n = len(counts)
    thr = np.empty(n, dtype=np.uint32)
    alias = np.empty(n, dtype=np.int32)
    check(lib().mirec_alias_build(counts.ctypes.data, n, thr.ctypes.data, alias.ctypes.data),
          "mirec_alias_build")
    return thr, alias


def sample_alias(thr: torch.Tensor, alias: torch.Tensor, seed: int, counter: int,
                 keys: torch.Tensor, num: int, used_ptr: torch.Tensor | None,
                 used_cols: torch.Tensor | None, n_key_space: int, reject: bool,
                 batch_keys: int | None = None, out: torch.Tensor | None = None,
                 out_stride: int = 0, status: torch.Tensor | None = None,
                 used_bits: torch.Tensor | None = None, n_bits: int = 0) -> torch.Tensor:
    """Alias-table fast-mode draws (NON-PARITY, mirec_sample_alias): `thr` is the
    uint32 threshold table viewed as int32 on the device, `alias` int32."""
    _dev(thr, torch.int32, "thr")
    _dev(alias, torch.int32, "alias")
    _dev(keys, torch.int64, "keys")
    n_keys = keys.numel()
    if batch_keys is None:
        batch_keys = max(n_keys, 1)
    if out is None:
        out = torch.empty(n_keys * num, dtype=torch.int64, device=keys.device)
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=keys.device)
    bits = reject and used_bits is not None
    if reject and not bits:
        _dev(used_ptr, torch.int64, "used_ptr")
        _dev(used_cols, torch.int32, "used_cols")
    if bits:
        _dev(used_bits, torch.int32, "used_bits")
    rc = lib().mirec_sample_alias(
        ptr(thr), ptr(alias), thr.numel(), seed & (2 ** 64 - 1), counter, ptr(keys), n_keys,
        batch_keys, num, ptr(used_ptr) if reject and not bits else None,
        ptr(used_cols) if reject and not bits else None, ptr(used_bits) if bits else None,
        n_bits if bits else 0, n_key_space, 1 if reject else 0, ptr(out), out_stride,
        ptr(status), stream_handle())
    check(rc, "mirec_sample_alias")
    return out


def used_bitmap(used_ptr: torch.Tensor, used_cols: torch.Tensor, n_keys: int,
                n_bits: int) -> torch.Tensor:
    """Per-key used-id bitmap [n_keys, ceil(n_bits/32)] (int32 words) of a CSR."""
    _dev(used_ptr, torch.int64, "used_ptr")
    _dev(used_cols, torch.int32, "used_cols")
    words = (n_bits + 31) // 32
    bits = torch.empty(max(n_keys * words, 1), dtype=torch.int32, device=used_ptr.device)
    rc = lib().mirec_used_bitmap_build(ptr(used_ptr), ptr(used_cols), n_keys, n_bits, ptr(bits),
                                       stream_handle())
    check(rc, "mirec_used_bitmap_build")
    return bits


# ---------------------------------------------------------------- K1 gather
def gather_rows(table: torch.Tensor, idx: torch.Tensor, out: torch.Tensor | None = None):
    if not table.is_cuda or not idx.is_cuda:
        raise NativeError("gather_rows: tensors must live on the GPU")
    if not table.is_contiguous():
        raise ValueError("table must be contiguous")
    idx = idx.contiguous()
    row_shape = table.shape[1:]
    if out is None:
        out = torch.empty((idx.numel(),) + tuple(row_shape), dtype=table.dtype,
                          device=table.device)
    row_bytes = table.element_size() * (table[0].numel() if table.dim() > 1 else 1)
    if idx.dtype == torch.int64:
        fn = lib().mirec_gather_rows
    elif idx.dtype == torch.int32:
        fn = lib().mirec_gather_rows_i32idx
    else:
        raise TypeError("idx must be int32 or int64")
    rc = fn(ptr(table), table.shape[0], row_bytes, ptr(idx), idx.numel(), ptr(out),
            stream_handle())
    check(rc, "mirec_gather_rows")
    return out


def window_gather(col: torch.Tensor, start: torch.Tensor, length: torch.Tensor, L: int,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """out[i, t] = col[start[i] + t] if t < length[i] else 0 (sequence windows)."""
    _dev(start, torch.int64, "start")
    _dev(length, torch.int64, "length")
    if not col.is_cuda or not col.is_contiguous():
        raise NativeError("window_gather: col must be a contiguous GPU tensor")
    n = start.numel()
    if out is None:
        out = torch.empty(n, L, dtype=col.dtype, device=col.device)
    rc = lib().mirec_window_gather(ptr(col), col.element_size(), ptr(start), ptr(length), n, L,
                                   ptr(out), stream_handle())
    check(rc, "mirec_window_gather")
    return out


# ---------------------------------------------------------------- K3 BPR
def bpr_fwd_bwd(EU, EI, user, pos, neg, times: int, gamma: float = 1e-10,
                grad_scale: float | None = None, grads: bool = True, scores: bool = False,
                out: dict | None = None) -> dict:
    """Fused BPR forward/backward on the pairwise layout (bpr.py:74-83, loss.py:47-49)."""
    _dev(EU, torch.float32, "EU")
    _dev(EI, torch.float32, "EI")
    for n_, t_ in (("user", user), ("pos", pos), ("neg", neg)):
        _dev(t_, torch.int64, n_)
    B = user.numel()
    d = EU.shape[1]
    if EI.shape[1] != d or pos.numel() != B or neg.numel() != B * times:
        raise ValueError("bpr_fwd_bwd: inconsistent shapes")
    if grad_scale is None:
        grad_scale = float(torch.tensor(1.0, dtype=torch.float32) /
                           torch.tensor(float(B * times), dtype=torch.float32))
    o = {} if out is None else out
    dev = EU.device
    if "loss_k" not in o:
        o["loss_k"] = torch.empty(B, dtype=torch.float32, device=dev)
    if scores:
        o.setdefault("pos_score", torch.empty(B, dtype=torch.float32, device=dev))
        o.setdefault("neg_score", torch.empty(B * times, dtype=torch.float32, device=dev))
    if grads:
        o.setdefault("gU", torch.empty(B, d, dtype=torch.float32, device=dev))
        o.setdefault("gI", torch.empty((1 + times) * B, d, dtype=torch.float32, device=dev))
    rc = lib().mirec_bpr_fwd_bwd_f32(ptr(EU), EU.shape[0], ptr(EI), EI.shape[0], d, ptr(user),
                                     ptr(pos), ptr(neg), B, times, gamma, grad_scale,
                                     ptr(o["loss_k"]), ptr(o.get("pos_score")),
                                     ptr(o.get("neg_score")), ptr(o.get("gU")),
                                     ptr(o.get("gI")), stream_handle())
    check(rc, "mirec_bpr_fwd_bwd_f32")
    return o


def bpr_fwd_coef(EU, EI, user, pos, neg, times: int, grad_scale: float, gamma: float = 1e-10):
    """K3 forward only: (loss_k [B], coef [times*B]) with coef[r] = d loss / d x_r
    (the data-parallel step's exchanged quantity)."""
    B = user.numel()
    for n_, t_ in (("user", user), ("pos", pos), ("neg", neg)):
        _dev(t_, torch.int64, n_)
    loss_k = torch.empty(B, dtype=torch.float32, device=EU.device)
    coef = torch.empty(max(B * times, 1), dtype=torch.float32, device=EU.device)
    rc = lib().mirec_bpr_fwd_coef_f32(ptr(EU), EU.shape[0], ptr(EI), EI.shape[0], EU.shape[1],
                                      ptr(user), ptr(pos), ptr(neg), B, times, gamma,
                                      grad_scale, ptr(loss_k), ptr(coef), stream_handle())
    check(rc, "mirec_bpr_fwd_coef_f32")
    return loss_k, coef[:B * times]


def bpr_contrib(EU, EI, user, pos, neg, times: int, coef, coef_block: int | None = None,
                coef_stride: int | None = None):
    """Gradient rows (gU [B,d], gI [(1+times)B,d]) of a batch rebuilt from its
    coefficients (mirec_bpr_contrib_f32); default: the single-rank layout."""
    B, d = user.numel(), EU.shape[1]
    _dev(coef, torch.float32, "coef")
    block = B if coef_block is None else coef_block
    stride = times * block if coef_stride is None else coef_stride
    gU = torch.empty(B, d, dtype=torch.float32, device=EU.device)
    gI = torch.empty((1 + times) * B, d, dtype=torch.float32, device=EU.device)
    rc = lib().mirec_bpr_contrib_f32(ptr(EU), EU.shape[0], ptr(EI), EI.shape[0], d, ptr(user),
                                     ptr(pos), ptr(neg), B, times, ptr(coef), block, stride,
                                     ptr(gU), ptr(gI), stream_handle())
    check(rc, "mirec_bpr_contrib_f32")
    return gU, gI


def dot_rows(EU, EI, u, i, out=None):
    """score[r] = <EU[u[r]], EI[i[r]]> (BPR.predict, bpr.py:85-89)."""
    _dev(EU, torch.float32, "EU")
    _dev(EI, torch.float32, "EI")
    u = u.contiguous()
    i = i.contiguous()
    _dev(u, torch.int64, "u")
    _dev(i, torch.int64, "i")
    if out is None:
        out = torch.empty(u.numel(), dtype=torch.float32, device=EU.device)
    rc = lib().mirec_dot_rows_f32(ptr(EU), EU.shape[0], ptr(EI), EI.shape[0], EU.shape[1], ptr(u),
                                  ptr(i), u.numel(), ptr(out), stream_handle())
    check(rc, "mirec_dot_rows_f32")
    return out


def fixed_sum(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    _dev(x, torch.float32, "x")
    if out is None:
        out = torch.empty(1, dtype=torch.float32, device=x.device)
    check(lib().mirec_sum_f32(ptr(x), x.numel(), ptr(out), stream_handle()), "mirec_sum_f32")
    return out


# ---------------------------------------------------------------- K2 grouping
class Segments:
    """Grouping of contribution rows by table row (output of K2)."""

    __slots__ = ("perm", "uniq", "seg", "n_uniq", "n", "ws", "pos_seg")

    def __init__(self, n: int, device, ws_bytes: int = 0):
        cap = max(n, 1)
        self.n = n
        self.pos_seg = None      # int32[n]: the segment of each sorted position, if the sort gave it
        self.perm = torch.empty(cap, dtype=torch.int32, device=device)
        self.uniq = torch.empty(cap, dtype=torch.int32, device=device)
        self.seg = torch.empty(cap + 1, dtype=torch.int32, device=device)
        self.n_uniq = torch.empty(1, dtype=torch.int32, device=device)   # every sort writes it
        self.ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=device)


ONESWEEP_MIN = 8193          # above the single-workgroup LDS sort
_SORT_STATUS = {}
_RETIRED = []    # superseded shared scratch buffers: never freed (see _sort_status)


def _sort_status(device, words):
    """Zeroed look-back / histogram words of the onesweep sort, one buffer per device —
    every call leaves it zero; calls are stream-ordered (the model's stream; a graph's
    warm-up and capture streams wait for each other), as for _scatter_ws. None while a
    graph capture is running and the buffer does not exist yet or is too small (the
    caller then takes the radix path).

    A buffer that is replaced by a larger one stays allocated for the life of the
    process: a HIP graph captured earlier holds its pointer and replays against it, and
    memory handed back to the caching allocator could be reused for other data, so a
    replay would read garbage look-back words (and scatter outside its outputs). A
    retired buffer is still zero (every call leaves it so) and only graphs use it."""
    key = str(device)
    buf = _SORT_STATUS.get(key)
    if buf is None or buf.numel() < words:
        if torch.cuda.is_current_stream_capturing():
            return None
        if buf is not None:
            _RETIRED.append(buf)
        buf = torch.zeros(max(words, 1 << 16), dtype=torch.int32, device=device)
        _SORT_STATUS[key] = buf
    return buf


def segment_sort(keys: torch.Tensor, key_space: int, segs: Segments | None = None) -> Segments:
    _dev(keys, torch.int64, "keys")
    n = keys.numel()
    wsz = lib().mirec_segment_sort_workspace_size(n, key_space)
    if segs is None or segs.n < n or segs.ws.numel() < wsz:
        segs = Segments(n, keys.device, wsz)
    status = None
    if ONESWEEP_MIN <= n < (1 << 30):
        status = _sort_status(keys.device, lib().mirec_segment_sort_onesweep_status_words(n))
    if status is not None:
        if segs.pos_seg is None or segs.pos_seg.numel() < n:
            segs.pos_seg = torch.empty(n, dtype=torch.int32, device=keys.device)
        rc = lib().mirec_segment_sort_onesweep(
            ptr(keys), n, key_space, ptr(segs.perm), ptr(segs.uniq), ptr(segs.seg),
            ptr(segs.n_uniq), ptr(segs.pos_seg), ptr(segs.ws), segs.ws.numel(), ptr(status),
            status.numel(), stream_handle())
        check(rc, "mirec_segment_sort_onesweep")
        return segs
    segs.pos_seg = None
    rc = lib().mirec_segment_sort(ptr(keys), n, key_space, ptr(segs.perm), ptr(segs.uniq),
                                  ptr(segs.seg), ptr(segs.n_uniq), ptr(segs.ws), segs.ws.numel(),
                                  stream_handle())
    check(rc, "mirec_segment_sort")
    return segs


CHAIN_MAX_BLOCK_N, CHAIN_MAX_BLOCKS = 4096, 256


def segment_sort_blocks(keys: torch.Tensor, block_n: int, key_space: int,
                        status: torch.Tensor | None = None) -> Segments:
    """segment_sort for keys in blocks of block_n whose key ranges increase block to
    block (every key of block b below every key of block b+1): same outputs, each
    block sorted in LDS. With `status` (int32, zero, >= n_blocks + 1 entries; left
    zero) and block_n <= 4,096, <= 256 blocks: one launch (mirec_segment_sort_blocks_
    chained); otherwise the sort + concatenation pair (mirec_segment_sort_blocks)."""
    _dev(keys, torch.int64, "keys")
    n = keys.numel()
    nb = -(-n // max(block_n, 1))
    if (status is not None and n > 0 and block_n <= CHAIN_MAX_BLOCK_N
            and nb <= CHAIN_MAX_BLOCKS):
        _dev(status, torch.int32, "status")
        segs = Segments(n, keys.device)
        segs.pos_seg = torch.empty(n, dtype=torch.int32, device=keys.device)
        with timed_launch('k2_blocks'):
            rc = lib().mirec_segment_sort_blocks_chained(
                ptr(keys), n, block_n, key_space, ptr(segs.perm), ptr(segs.uniq), ptr(segs.seg),
                ptr(segs.n_uniq), ptr(status), status.numel(), ptr(segs.pos_seg),
                stream_handle())
        check(rc, "mirec_segment_sort_blocks_chained")
        return segs
    segs = Segments(n, keys.device, lib().mirec_segment_sort_blocks_workspace_size(n, block_n))
    with timed_launch('k2_blocks'):              # two launches: the block sorts, the concat
        rc = lib().mirec_segment_sort_blocks(ptr(keys), n, block_n, key_space, ptr(segs.perm),
                                             ptr(segs.uniq), ptr(segs.seg), ptr(segs.n_uniq),
                                             ptr(segs.ws), segs.ws.numel(), stream_handle())
    check(rc, "mirec_segment_sort_blocks")
    return segs


def segment_sort_fields(cols, offsets, B: int, key_space: int, status: torch.Tensor):
    """DeepFM's token keys (field f: cols[f] + offsets[f], ranges increasing with f) formed
    and grouped in one launch (mirec_segment_sort_fields_chained): (keys [F * B] int64,
    Segments with pos_seg). status: the chained sort's zeroed words (>= F + 1)."""
    nf = len(cols)
    for c in cols:
        _dev(c, torch.int64, "field column")
    _dev(status, torch.int32, "status")
    dev = cols[0].device
    n = nf * B
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    segs = Segments(n, dev)
    segs.pos_seg = torch.empty(n, dtype=torch.int32, device=dev)
    cptr = (ctypes.c_void_p * nf)(*[ptr(c) for c in cols])
    offs = (ctypes.c_int64 * nf)(*[int(o) for o in offsets])
    with timed_launch('k2_blocks'):
        rc = lib().mirec_segment_sort_fields_chained(
            cptr, offs, nf, B, key_space, ptr(keys), ptr(segs.perm), ptr(segs.uniq),
            ptr(segs.seg), ptr(segs.n_uniq), ptr(status), status.numel(), ptr(segs.pos_seg),
            stream_handle())
    check(rc, "mirec_segment_sort_fields_chained")
    return keys, segs


def segment_sort_batched(keys: torch.Tensor, batch_n: int, key_space: int, perm, uniq, seg,
                         n_uniq, ws=None):
    """K2 over consecutive batches of `batch_n` keys, one workgroup per batch."""
    _dev(keys, torch.int64, "keys")
    n = keys.numel()
    nb = max(1, -(-n // max(batch_n, 1)))
    wsz = lib().mirec_segment_sort_workspace_size(nb * batch_n, key_space)
    if ws is None or ws.numel() < wsz:
        ws = torch.empty(wsz, dtype=torch.uint8, device=keys.device)
    rc = lib().mirec_segment_sort_batched(ptr(keys), n, batch_n, key_space, ptr(perm), ptr(uniq),
                                          ptr(seg), ptr(n_uniq), ptr(ws), ws.numel(),
                                          stream_handle())
    check(rc, "mirec_segment_sort_batched")
    return ws


def uniq_ahead_diff(uniq, n_uniq, stride: int, n_batches: int, out, n_out):
    """out[b*stride..] = uniq(b+1) minus uniq(b) (batched segment-sort layout)."""
    for n_, t_ in (("uniq", uniq), ("n_uniq", n_uniq), ("out", out), ("n_out", n_out)):
        _dev(t_, torch.int32, n_)
    rc = lib().mirec_uniq_ahead_diff(ptr(uniq), ptr(n_uniq), stride, n_batches, ptr(out),
                                     ptr(n_out), stream_handle())
    check(rc, "mirec_uniq_ahead_diff")


_SCATTER_WS = {}


def _scatter_ws(device, nbytes):
    """Per-device scratch of the chunked scatter (stream-ordered reuse: every
    launch on the stream finishes with it before the next one starts)."""
    key = str(device)
    buf = _SCATTER_WS.get(key)
    if buf is None or buf.numel() < nbytes:
        if buf is not None:                  # a captured graph may hold it (_sort_status)
            _RETIRED.append(buf)
        buf = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, device=device)
        _SCATTER_WS[key] = buf
    return buf


def segment_scatter_add(rows: torch.Tensor, segs: Segments, dense: torch.Tensor) -> torch.Tensor:
    _dev(rows, torch.float32, "rows")
    _dev(dense, torch.float32, "dense")
    d = rows.shape[1]
    wsz = lib().mirec_segment_scatter_add_workspace_size(segs.n, d)
    ws = _scatter_ws(rows.device, wsz)
    rc = lib().mirec_segment_scatter_add_f32(ptr(rows), d, ptr(segs.perm), ptr(segs.uniq),
                                             ptr(segs.seg), ptr(segs.n_uniq), segs.n, ptr(dense),
                                             dense.shape[0], ptr(ws), ws.numel(),
                                             stream_handle())
    check(rc, "mirec_segment_scatter_add_f32")
    return dense


def segment_reduce(rows: torch.Tensor, segs: Segments):
    """(compact [n, d] with row u = sum of segment u's contributions, identity
    Segments over it with the same uniq / n_uniq) — each touched table row's
    gradient as one row for K5."""
    _dev(rows, torch.float32, "rows")
    n, d = segs.n, rows.shape[1]
    out = torch.empty(max(n, 1), d, dtype=torch.float32, device=rows.device)
    ws = _scatter_ws(rows.device, lib().mirec_segment_scatter_add_workspace_size(n, d))
    pos_seg = getattr(segs, 'pos_seg', None)
    if pos_seg is not None and pos_seg is not getattr(segs, 'perm', None):
        rc = lib().mirec_segment_reduce_pos_seg_f32(ptr(rows), d, ptr(segs.perm), ptr(pos_seg),
                                                    ptr(segs.uniq), ptr(segs.seg),
                                                    ptr(segs.n_uniq), n, ptr(out), ptr(ws),
                                                    ws.numel(), stream_handle())
    else:
        rc = lib().mirec_segment_reduce_f32(ptr(rows), d, ptr(segs.perm), ptr(segs.uniq),
                                            ptr(segs.seg), ptr(segs.n_uniq), n, ptr(out),
                                            ptr(ws), ws.numel(), stream_handle())
    check(rc, "mirec_segment_reduce_f32")
    ident = Segments.__new__(Segments)
    ident.n = n
    iota = _iota(rows.device, max(n, 1) + 1)       # identity perm / seg: no launch per call
    ident.perm = iota[:max(n, 1)]
    ident.seg = iota[:max(n, 1) + 1]
    ident.uniq, ident.n_uniq, ident.ws = segs.uniq, segs.n_uniq, segs.ws
    ident.pos_seg = ident.perm
    return out, ident


def segment_merge2(a, b, a_pre=False):
    """Union of two reduced sources of one table — a, b: (compact rows, identity Segments
    with uniq / n_uniq) as segment_reduce returns them — into (rows, identity Segments):
    the second-level segment_reduce of their concatenation, bit for bit, in two launches
    (mirec_segment_merge2_f32). a_pre: a is a previous merge's output."""
    (ra, sa), (rb, sb) = a, b
    _dev(ra, torch.float32, "rows a")
    _dev(rb, torch.float32, "rows b")
    d = ra.shape[1]
    if rb.shape[1] != d:
        raise ValueError("segment_merge2: row widths differ")
    capA, capB = sa.n, sb.n
    cap = max(capA + capB, 1)
    dev = ra.device
    out = torch.empty(cap, d, dtype=torch.float32, device=dev)
    uniq = torch.empty(cap, dtype=torch.int32, device=dev)
    n_uniq = torch.empty(1, dtype=torch.int32, device=dev)
    ws = _scatter_ws(dev, 8 * cap)
    status = _sort_status(dev, cap // 512 + 2)
    if status is None:
        raise NativeError("segment_merge2: no status buffer inside a capture (run one step "
                          "eagerly first)")
    rc = lib().mirec_segment_merge2_f32(ptr(sa.uniq), ptr(sa.n_uniq), capA, ptr(ra),
                                        ptr(sb.uniq), ptr(sb.n_uniq), capB, ptr(rb), d,
                                        1 if a_pre else 0, ptr(uniq), ptr(n_uniq), ptr(out),
                                        ptr(ws), ws.numel(), ptr(status), status.numel(),
                                        stream_handle())
    check(rc, "mirec_segment_merge2_f32")
    ident = Segments.__new__(Segments)
    ident.n = cap
    iota = _iota(dev, cap + 1)
    ident.perm = iota[:cap]
    ident.seg = iota[:cap + 1]
    ident.uniq, ident.n_uniq, ident.ws = uniq, n_uniq, sa.ws
    ident.pos_seg = ident.perm
    return out, ident


def segment_reduce2(rows: torch.Tensor, rows1: torch.Tensor, segs: Segments):
    """segment_reduce of a [n, d] source (2 <= d <= 16) and a [n, 1] source grouped by
    the same segments, in one pass: (compact, compact1, identity Segments), bit for bit
    the two separate reductions."""
    _dev(rows, torch.float32, "rows")
    _dev(rows1, torch.float32, "rows1")
    n, d = segs.n, rows.shape[1]
    out = torch.empty(max(n, 1), d, dtype=torch.float32, device=rows.device)
    out1 = torch.empty(max(n, 1), 1, dtype=torch.float32, device=rows.device)
    ws = _scatter_ws(rows.device, lib().mirec_segment_scatter_add_workspace_size(n, d + 1))
    if getattr(segs, 'pos_seg', None) is not None:     # the chained sort's position -> segment
        rc = lib().mirec_segment_reduce2_pos_seg_f32(
            ptr(rows), d, ptr(rows1), ptr(segs.perm), ptr(segs.pos_seg), ptr(segs.uniq),
            ptr(segs.seg), ptr(segs.n_uniq), n, ptr(out), ptr(out1), ptr(ws), ws.numel(),
            stream_handle())
    else:
        rc = lib().mirec_segment_reduce2_f32(ptr(rows), d, ptr(rows1), ptr(segs.perm),
                                             ptr(segs.uniq), ptr(segs.seg), ptr(segs.n_uniq), n,
                                             ptr(out), ptr(out1), ptr(ws), ws.numel(),
                                             stream_handle())
    check(rc, "mirec_segment_reduce2_f32")
    ident = Segments.__new__(Segments)
    ident.n = n
    iota = _iota(rows.device, max(n, 1) + 1)
    ident.perm = iota[:max(n, 1)]
    ident.seg = iota[:max(n, 1) + 1]
    ident.uniq, ident.n_uniq, ident.ws = segs.uniq, segs.n_uniq, segs.ws
    ident.pos_seg = ident.perm
    return out, out1, ident


_IOTA = {}


def _iota(device, n):
    """0, 1, ..., n-1 as a persistent int32 device tensor (grown on demand; read only).
    Allocated outside any graph capture the first time a size is needed."""
    key = str(device)
    t = _IOTA.get(key)
    if t is None or t.numel() < n:
        if torch.cuda.is_current_stream_capturing():   # graph-pool memory: not cached
            return torch.arange(n, dtype=torch.int32, device=device)
        if t is not None:                    # a captured graph may hold it (_sort_status)
            _RETIRED.append(t)
        t = _IOTA[key] = torch.arange(max(n, 1 << 16), dtype=torch.int32, device=device)
    return t[:n]


# ---------------------------------------------------------------- K5 Adam
def adam_flat_multi(specs, step_consts, step_idx, beta1=0.9, beta2=0.999, eps=1e-8,
                    weight_decay=0.0, advance_ticket=None):
    """Dense Adam steps of several parameters in one launch per 16 (specs: dicts with
    p, m, v, g — contiguous float32 device tensors of one size each). advance_ticket (an
    int32 [1] device tensor, zero between calls): step_idx is the device step counter and
    the last launch advances it by one after reading it."""
    from recbole_amd._native import FlatParam
    _dev(step_consts, torch.float32, "step_consts")
    _dev(step_idx, torch.int32, "step_idx")
    for i in range(0, len(specs), 16):
        part = specs[i:i + 16]
        arr = (FlatParam * len(part))()
        for t, sp in zip(arr, part):
            for n_ in ("p", "m", "v", "g"):
                x = _dev(sp[n_], torch.float32, n_)
                if not x.is_contiguous() or x.numel() != sp["p"].numel():
                    raise ValueError(f"adam_flat_multi: {n_} must be contiguous, numel of p")
            t.p, t.m, t.v, t.g, t.n = (ptr(sp["p"]), ptr(sp["m"]), ptr(sp["v"]), ptr(sp["g"]),
                                       sp["p"].numel())
        if advance_ticket is not None and i + 16 >= len(specs):
            _dev(advance_ticket, torch.int32, "advance_ticket")
            check(lib().mirec_adam_flat_multi_advance_f32(
                arr, len(part), ptr(step_consts), ptr(step_idx), ptr(advance_ticket), beta1,
                beta2, eps, weight_decay, stream_handle()), "mirec_adam_flat_multi_advance_f32")
            continue
        check(lib().mirec_adam_flat_multi_f32(arr, len(part), ptr(step_consts), ptr(step_idx),
                                              beta1, beta2, eps, weight_decay, stream_handle()),
              "mirec_adam_flat_multi_f32")


def adam_step(p, m, v, step_consts, step_idx, rows=None, segs: Segments | None = None,
              dense_grad=None, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0):
    """One dense Adam step over every row of p (K5); the gradient is the grouped
    compact rows (rows + segs) and/or a dense gradient tensor."""
    for n_, t_ in (("p", p), ("m", m), ("v", v)):
        _dev(t_, torch.float32, n_)
    _dev(step_consts, torch.float32, "step_consts")
    _dev(step_idx, torch.int32, "step_idx")
    if dense_grad is not None:
        _dev(dense_grad, torch.float32, "dense_grad")
    if p.dim() == 2 and p.shape[1] in (16, 32, 64, 128, 256):
        n_rows, d = p.shape
    elif segs is not None:
        raise ValueError("grouped gradients need a 2-D table of width 16..256")
    elif p.numel() % 4 == 0:
        n_rows, d = p.numel() // 4, 4
    else:
        if dense_grad is None:
            raise ValueError("adam_step: a flat parameter needs a dense gradient")
        rc = lib().mirec_adam_flat_f32(ptr(p), ptr(m), ptr(v), p.numel(), ptr(dense_grad),
                                       ptr(step_consts), ptr(step_idx), beta1, beta2, eps,
                                       weight_decay, stream_handle())
        check(rc, "mirec_adam_flat_f32")
        return
    rc = lib().mirec_adam_sparse_grad_f32(
        ptr(p), ptr(m), ptr(v), n_rows, d, ptr(rows),
        ptr(segs.perm) if segs else None, ptr(segs.uniq) if segs else None,
        ptr(segs.seg) if segs else None, ptr(segs.n_uniq) if segs else None,
        segs.n if segs else 0, ptr(dense_grad), ptr(step_consts), ptr(step_idx), beta1, beta2,
        eps, weight_decay, stream_handle())
    check(rc, "mirec_adam_sparse_grad_f32")


ADAM_ZERO_STATE = 0x7fffffff   # MIREC_ADAM_ZERO_STATE (include/mirec.h)


def zero_state_marks(m, v, last, weight_decay=0.0):
    """Set the deferred schedule's step counts for a new window in place:
    last[r] = ADAM_ZERO_STATE where row r's m and v are all +0 (a fixed point of
    the zero-gradient Adam step when weight_decay == 0: flushes and look-aheads
    skip it), else 0."""
    if weight_decay != 0:
        last.zero_()
        return last
    zs = (m.view(torch.int32) == 0).all(1) & (v.view(torch.int32) == 0).all(1)
    last.copy_(torch.where(zs, ADAM_ZERO_STATE, 0).to(torch.int32))
    return last


def reset_marks(last):
    """Window start for counts that already carry zero-state marks: every count
    that is not a mark restarts at 0 (marks stay: those rows are still +0)."""
    last.masked_fill_(last != ADAM_ZERO_STATE, 0)
    return last


def adam_tables(specs):
    """ctypes array of mirec_adam_table from dicts with keys p, m, v (2-D float32
    tables of one width) and optional rows + segs (grouped gradient), dense_grad,
    last (int32 per-row step counts of the deferred schedule), ahead ((rows, count)
    int32 device tensors: rows the next batch reads and this one does not touch,
    completed by the deferred schedule for the next forward pass)."""
    from recbole_amd._native import AdamTable
    arr = (AdamTable * len(specs))()
    for t, s in zip(arr, specs):
        for n_ in ("p", "m", "v"):
            _dev(s[n_], torch.float32, n_)
        t.p, t.m, t.v, t.n_rows = ptr(s["p"]), ptr(s["m"]), ptr(s["v"]), s["p"].shape[0]
        segs = s.get("segs")
        if segs is not None:
            _dev(s["rows"], torch.float32, "rows")
            t.rows, t.perm, t.uniq = ptr(s["rows"]), ptr(segs.perm), ptr(segs.uniq)
            t.seg, t.n_uniq = ptr(segs.seg), ptr(segs.n_uniq)
        if s.get("dense_grad") is not None:
            t.dense_grad = ptr(_dev(s["dense_grad"], torch.float32, "dense_grad"))
        if s.get("last") is not None:
            t.last = ptr(_dev(s["last"], torch.int32, "last"))
        if s.get("ahead") is not None:
            au, an = s["ahead"]
            t.ahead_uniq = ptr(_dev(au, torch.int32, "ahead_uniq"))
            t.ahead_n_uniq = ptr(_dev(an, torch.int32, "ahead_n_uniq"))
        if s.get("p_alt") is not None:            # parity buffer (bpr_adam_step)
            t.p_alt = ptr(_dev(s["p_alt"], torch.float32, "p_alt"))
        if s.get("segs") is None and s.get("grouping") is not None:   # no gradient rows
            g = s["grouping"]
            t.perm, t.uniq, t.seg, t.n_uniq = ptr(g.perm), ptr(g.uniq), ptr(g.seg), ptr(g.n_uniq)
    return arr


def step_records(user_keys, item_keys, n_batches: int, Bc: int, times: int, n_users: int,
                 n_items: int, gu, gi, out=None):
    """K35 records (mirec_step_records) of n_batches batches from their K2 groupings
    gu / gi (Segments or any object with perm, uniq, seg, n_uniq; per-batch strides Bc
    and (1+T)*Bc): (u_rec, u_crec, i_rec, i_crec) int32 device tensors (`out`: the
    caller's four buffers)."""
    for n_, t_ in (("user_keys", user_keys), ("item_keys", item_keys)):
        _dev(t_, torch.int64, n_)
    dev = user_keys.device
    KI = (1 + times) * Bc
    if out is None:
        out = [torch.empty(n_batches * n, dtype=torch.int32, device=dev)
               for n in (step_record_ints(Bc), Bc * 8, step_record_ints(KI), KI * 8)]
    rc = lib().mirec_step_records(ptr(user_keys), ptr(item_keys), n_batches, Bc, times, n_users,
                                  n_items, ptr(gu.perm), ptr(gu.uniq), ptr(gu.seg),
                                  ptr(gu.n_uniq), ptr(gi.perm), ptr(gi.uniq), ptr(gi.seg),
                                  ptr(gi.n_uniq), *[ptr(o) for o in out], None, None, None, None,
                                  stream_handle())
    check(rc, "mirec_step_records")
    return out


def chunk_group(user_keys, item_keys, n_batches: int, Bc: int, times: int, n_users: int,
                n_items: int, outs: dict, records: bool = True, ahead: bool = True):
    """K36 (mirec_chunk_group): the groupings, K35 records and look-ahead lists of a
    chunk in one launch, into the int32 device tensors of `outs` (keys u_perm, u_uniq,
    u_seg, u_nu, i_perm, i_uniq, i_seg, i_nu, and u_rec, u_crec, i_rec, i_crec /
    u_ahead, u_nah, i_ahead, i_nah when asked for). Returns False (nothing launched)
    when the shapes are outside its one-workgroup form."""
    for n_, t_ in (("user_keys", user_keys), ("item_keys", item_keys)):
        _dev(t_, torch.int64, n_)
    names = ["u_perm", "u_uniq", "u_seg", "u_nu", "i_perm", "i_uniq", "i_seg", "i_nu"]
    rec = ["u_rec", "u_crec", "i_rec", "i_crec"]
    ah = ["u_ahead", "u_nah", "i_ahead", "i_nah"]
    args = [ptr(outs[k]) for k in names]
    args += [ptr(outs[k]) for k in rec] if records else [None] * 4
    args += [ptr(outs[k]) for k in ah] if ahead else [None] * 4
    rc = lib().mirec_chunk_group(ptr(user_keys), ptr(item_keys), n_batches, Bc, times, n_users,
                                 n_items, *args, stream_handle())
    if rc < 0:
        check(rc, "mirec_chunk_group")
    return rc == 1


def step_record_ints(per: int) -> int:
    """int32 per batch of one table's K35 record region (mirec_step_record_ints)."""
    n = lib().mirec_step_record_ints(per)
    if n < 0:
        raise ValueError(f"step_record_ints: bad per {per}")
    return n


def step_scratch(Bc: int, times: int, d: int, device):
    """K35 hand-off scratch (u_part, u_join, i_part, i_join): contribution vectors of
    split rows per grouped position, and zeroed arrival counters per row slot and per
    look-ahead slot; reusable by every launch of the same stream (each launch leaves
    the counters zero)."""
    KI = (1 + times) * Bc
    return [torch.empty(Bc * d, dtype=torch.float32, device=device),
            torch.zeros(2 * Bc, dtype=torch.int32, device=device),
            torch.empty(KI * d, dtype=torch.float32, device=device),
            torch.zeros(2 * KI, dtype=torch.int32, device=device)]


def bpr_adam_step(tables, n_max_uniq, d: int, items, Bc: int, times: int, grad_scale: float,
                  loss_k, records, scratch, step_consts, step_base, step_off: int = 0,
                  gamma: float = 1e-10, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0):
    """K35: one training step (BPR forward/backward + the touched rows' deferred Adam
    step + look-ahead) in one launch; tables = adam_tables([users, items]) with p_alt and
    a grouping (n_uniq); records = step_records(...) of this batch; scratch =
    step_scratch(Bc, times, d)."""
    import ctypes
    _dev(items, torch.int64, "items")
    nm = (ctypes.c_int64 * 2)(*n_max_uniq)
    rc = lib().mirec_bpr_adam_step_f32(tables, nm, d, ptr(items), Bc, times, gamma, grad_scale,
                                       ptr(loss_k), *[ptr(r) for r in records],
                                       *[ptr(x) for x in scratch], ptr(step_consts),
                                       ptr(step_base), step_off, beta1, beta2, eps, weight_decay,
                                       stream_handle())
    check(rc, "mirec_bpr_adam_step_f32")


def adam_multi(tables, d: int, step_consts, step_base, step_off: int = 0,
               schedule: str = "streamed", n_max_uniq=None, beta1=0.9, beta2=0.999, eps=1e-8,
               weight_decay=0.0, flush_rows=None):
    """K5 over several tables in one launch: schedule 'streamed' (every row),
    'deferred' (touched rows, replaying skipped zero-gradient steps), 'deferred_pair'
    (two tables, widths d and 1, same semantics, one launch) or 'flush'
    (flush_rows: rows per wave per table, mirec_adam_flush_rows_f32; None = one wave
    per row)."""
    import ctypes
    _dev(step_consts, torch.float32, "step_consts")
    _dev(step_base, torch.int32, "step_base")
    args = (ptr(step_consts), ptr(step_base), step_off, beta1, beta2, eps, weight_decay,
            stream_handle())
    if schedule == "streamed":
        rc = lib().mirec_adam_multi_f32(tables, len(tables), d, *args)
    elif schedule == "deferred":
        nm = (ctypes.c_int64 * len(tables))(*n_max_uniq)
        rc = lib().mirec_adam_deferred_f32(tables, len(tables), nm, d, *args)
    elif schedule == "deferred_pair":          # tables: ([V, d], [V, 1]), one launch
        nm = (ctypes.c_int64 * 2)(*n_max_uniq)
        rc = lib().mirec_adam_deferred_pair_f32(tables, nm, d, *args)
    elif schedule == "flush" and flush_rows is not None:
        rpw = (ctypes.c_int32 * len(tables))(*flush_rows)
        rc = lib().mirec_adam_flush_rows_f32(tables, len(tables), d, rpw, *args)
    elif schedule == "flush":
        rc = lib().mirec_adam_flush_f32(tables, len(tables), d, *args)
    else:
        raise ValueError(f"unknown schedule {schedule!r}")
    check(rc, f"adam_multi[{schedule}]")


_TICKETS = {}


def finish_ticket(device, tag=''):
    """Per-device zeroed int32 of mirec_chunk_finish (tag '') or another kernel's
    last-block ticket (left zero by every launch)."""
    key = (str(device), tag)
    t = _TICKETS.get(key)
    if t is None:
        t = _TICKETS[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return t


def chunk_finish(loss_k, n: int, stride: int, n_steps: int, denom: float, loss_hist, step_base):
    _dev(loss_k, torch.float32, "loss_k")
    _dev(step_base, torch.int32, "step_base")
    rc = lib().mirec_chunk_finish(ptr(loss_k), n, stride, n_steps, float(denom), ptr(loss_hist),
                                  ptr(step_base), ptr(finish_ticket(loss_k.device)),
                                  stream_handle())
    check(rc, "mirec_chunk_finish")


def step_finish(loss_k, denom: float, loss_hist, step_idx):
    _dev(loss_k, torch.float32, "loss_k")
    _dev(step_idx, torch.int32, "step_idx")
    rc = lib().mirec_step_finish(ptr(loss_k), loss_k.numel(), float(denom), ptr(loss_hist),
                                 ptr(step_idx), stream_handle())
    check(rc, "mirec_step_finish")


# ---------------------------------------------------------------- K6 full sort
def fullsort_topk(Uq, EI, K: int, hist_ptr=None, hist_cols=None, pos_ptr=None, pos_cols=None,
                  out: dict | None = None, n_split: int = 1) -> dict:
    _dev(Uq, torch.float32, "Uq")
    _dev(EI, torch.float32, "EI")
    nq, d = Uq.shape
    if EI.shape[1] != d:
        raise ValueError("fullsort_topk: embedding sizes differ")
    for n_, t_, dt in (("hist_ptr", hist_ptr, torch.int64), ("hist_cols", hist_cols, torch.int32),
                       ("pos_ptr", pos_ptr, torch.int64), ("pos_cols", pos_cols, torch.int32)):
        if t_ is not None:
            _dev(t_, dt, n_)
    o = {} if out is None else out
    dev = Uq.device
    o.setdefault("scores", torch.empty(nq, K, dtype=torch.float32, device=dev))
    o.setdefault("ids", torch.empty(nq, K, dtype=torch.int32, device=dev))
    if pos_ptr is not None:
        o.setdefault("pos_flags", torch.empty(nq, K, dtype=torch.uint8, device=dev))
    if n_split > 1:                      # item range split over n_split workgroups + merge
        wsz = lib().mirec_fullsort_topk_split_workspace_size(nq, K, n_split)
        ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
        with timed_launch('fullsort'):
            rc = lib().mirec_fullsort_topk_split_f32(
                ptr(Uq), nq, ptr(EI), EI.shape[0], d, ptr(hist_ptr), ptr(hist_cols),
                ptr(pos_ptr), ptr(pos_cols), K, n_split, ptr(ws), wsz, ptr(o["scores"]),
                ptr(o["ids"]), ptr(o.get("pos_flags")), stream_handle())
        check(rc, "mirec_fullsort_topk_split_f32")
        o["_ws"] = ws
        return o
    with timed_launch('fullsort'):
        rc = lib().mirec_fullsort_topk_f32(ptr(Uq), nq, ptr(EI), EI.shape[0], d, ptr(hist_ptr),
                                           ptr(hist_cols), ptr(pos_ptr), ptr(pos_cols), K,
                                           ptr(o["scores"]), ptr(o["ids"]),
                                           ptr(o.get("pos_flags")), stream_handle())
    check(rc, "mirec_fullsort_topk_f32")
    return o


def score_matrix(Uq, EI, out=None):
    _dev(Uq, torch.float32, "Uq")
    _dev(EI, torch.float32, "EI")
    if out is None:
        out = torch.empty(Uq.shape[0], EI.shape[0], dtype=torch.float32, device=Uq.device)
    rc = lib().mirec_score_matrix_f32(ptr(Uq), Uq.shape[0], ptr(EI), EI.shape[0], Uq.shape[1],
                                      ptr(out), stream_handle())
    check(rc, "mirec_score_matrix_f32")
    return out


# ---------------------------------------------------------------- K7 graph propagation
def _rows_ref(t):
    """mirec_rows_ref from None, a [n, d] tensor, or a (lo, hi) pair of row blocks."""
    from recbole_amd._native import RowsRef
    if t is None:
        return RowsRef(None, None, 0)
    if isinstance(t, tuple):
        lo, hi = t
        _dev(lo, torch.float32, "rows.lo")
        _dev(hi, torch.float32, "rows.hi")
        return RowsRef(ptr(lo), ptr(hi), lo.shape[0])
    _dev(t, torch.float32, "rows")
    return RowsRef(ptr(t), None, t.shape[0])


def _rows_n(t):
    if t is None:
        return None
    if isinstance(t, tuple):
        return t[0].shape[0] + t[1].shape[0], t[0].shape[1]
    return t.shape[0], t.shape[1]


class SpmmPlan:
    """Device CSR of a square sparse matrix plus the K7 load-balancing plan:
    every row is cut into units of at most `piece` nonzeros (include/mirec.h)."""

    def __init__(self, row_ptr: np.ndarray, cols: np.ndarray, vals: np.ndarray, device,
                 piece: int = 256, max_units: int = 1024):
        row_ptr = np.asarray(row_ptr, dtype=np.int64)
        n = len(row_ptr) - 1
        deg = np.diff(row_ptr)
        # hub rows (a Zipf head item has millions of edges) are cut into at most
        # max_units units so the fixup of their partials stays short
        n_units_row = np.minimum(np.maximum(1, -(-deg // piece)), max_units)
        first_unit = np.concatenate([[0], np.cumsum(n_units_row)])
        n_units = int(first_unit[-1])
        unit_row = np.repeat(np.arange(n, dtype=np.int32), n_units_row)
        k_in_row = np.arange(n_units, dtype=np.int64) - first_unit[:-1][unit_row]
        # near-equal split of row r's deg nonzeros over its units
        unit_beg = row_ptr[:-1][unit_row] + (k_in_row * deg[unit_row]) // n_units_row[unit_row]
        unit_beg = np.concatenate([unit_beg, [row_ptr[-1]]])
        split = n_units_row > 1
        unit_slot = np.full(n_units, -1, dtype=np.int32)
        in_split = split[unit_row]
        unit_slot[in_split] = np.arange(int(in_split.sum()), dtype=np.int32)
        fix_row = np.nonzero(split)[0].astype(np.int32)
        fix_ptr = np.concatenate([[0], np.cumsum(n_units_row[split])]).astype(np.int32)
        self.n_rows, self.nnz, self.piece = n, int(row_ptr[-1]), piece
        self.n_units, self.n_fix, self.n_slots = n_units, len(fix_row), int(fix_ptr[-1])
        T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=device)
        self.row_ptr, self.cols, self.vals = T(row_ptr), T(cols.astype(np.int32)), \
            T(vals.astype(np.float32))
        self.unit_row, self.unit_beg, self.unit_slot = T(unit_row), T(unit_beg), T(unit_slot)
        self.fix_row, self.fix_ptr = T(fix_row), T(fix_ptr)
        self._partial = {}

    def partial(self, d, device):
        if self.n_slots == 0:
            return None
        if d not in self._partial:
            self._partial[d] = torch.empty(self.n_slots, d, dtype=torch.float32, device=device)
        return self._partial[d]


def spmm_csr(plan: SpmmPlan, x, y=None, add=None, add_scale: float = 1.0, acc_in=None,
             acc_out=None, acc_scale: float = 1.0):
    """One K7 launch: y = A @ x (+ add_scale*add); Y = y; ACC_OUT = (ACC_IN + y)*acc_scale.
    Each operand is None, a [n, d] tensor or a (lo, hi) pair of row blocks."""
    from recbole_amd._native import SpmmEpilogue
    n, d = _rows_n(x)
    if n != plan.n_rows:
        raise ValueError(f"spmm_csr: x has {n} rows, the matrix {plan.n_rows}")
    for name, t in (("y", y), ("add", add), ("acc_in", acc_in), ("acc_out", acc_out)):
        if t is not None and _rows_n(t) != (n, d):
            raise ValueError(f"spmm_csr: {name} shape {_rows_n(t)} != {(n, d)}")
    if y is None and acc_out is None:
        raise ValueError("spmm_csr: nothing to write")
    dev = plan.row_ptr.device
    part = plan.partial(d, dev)
    ep = SpmmEpilogue(_rows_ref(add), add_scale, _rows_ref(y), _rows_ref(acc_in),
                      _rows_ref(acc_out), acc_scale)
    xr = _rows_ref(x)
    rc = lib().mirec_spmm_csr_f32(ptr(plan.row_ptr), ptr(plan.cols), ptr(plan.vals), plan.n_rows,
                                  d, ptr(plan.unit_row), ptr(plan.unit_beg), ptr(plan.unit_slot),
                                  plan.n_units, plan.piece, ptr(plan.fix_row), ptr(plan.fix_ptr),
                                  plan.n_fix, ptr(part), ctypes.byref(xr), ctypes.byref(ep),
                                  stream_handle())
    check(rc, "mirec_spmm_csr_f32")


def gather_sqnorm(table, idx, out=None):
    """out[i] = ||table[idx[i]]||^2 (EmbLoss, loss.py:79-84)."""
    _dev(table, torch.float32, "table")
    _dev(idx, torch.int64, "idx")
    if out is None:
        out = torch.empty(idx.numel(), dtype=torch.float32, device=table.device)
    rc = lib().mirec_gather_sqnorm_f32(ptr(table), table.shape[0], table.shape[1], ptr(idx),
                                       idx.numel(), ptr(out), stream_handle())
    check(rc, "mirec_gather_sqnorm_f32")
    return out


def gather_scale_rows(table, idx, scale_dev, out=None):
    """out[i, :] = scale_dev[0] * table[idx[i], :]."""
    _dev(table, torch.float32, "table")
    _dev(idx, torch.int64, "idx")
    _dev(scale_dev, torch.float32, "scale")
    if out is None:
        out = torch.empty(idx.numel(), table.shape[1], dtype=torch.float32, device=table.device)
    rc = lib().mirec_gather_scale_rows_f32(ptr(table), table.shape[0], table.shape[1], ptr(idx),
                                           idx.numel(), ptr(scale_dev), ptr(out),
                                           stream_handle())
    check(rc, "mirec_gather_scale_rows_f32")
    return out
