"""Fused train step and full-sort evaluation for embedding models (BPR-MF).

One training step of Trainer._train_epoch (trainer.py:157-174) for a pairwise
model with learner 'adam', as hand-written gfx950 kernels with no host
synchronisation inside the epoch. The work splits by dependency:

data side (depends only on ids; runs AHEAD on a side stream, CHUNK batches per launch)
  K4 sampler walk  (sampler.py:103-154)   negatives of CHUNK future batches, written
                                           straight into per-batch [pos | neg] key rows
  K2 segment sort  (embedding backward)   rows grouped by table row, one workgroup/batch
model side (main stream, per batch)
  K3 fused BPR     (bpr.py:74-83)         loss rows + per-row gradients
  K5 dense Adam    (optim.Adam.step)      every row of BOTH tables in one launch,
                                           grouped gradients summed on the fly
  step_finish                             per-step mean loss kept on the device

The batch is a contiguous slice of the train table resident in HBM, shuffled
once per epoch with torch.randperm on the CPU generator (interaction.py:272-276)
and re-ordered on the device with the K1 gather. Per-batch losses are read
back once per epoch (the reference reads `losses.item()` every batch).

Chunks are double-buffered (the side stream fills slot s^1 while the main
stream consumes slot s, ordered by HIP events). Every model-side pointer of a
chunk is relative to its slot, and the Adam constants / loss history / step
counter live in persistent device buffers, so the CHUNK steps of a slot are
captured ONCE into a HIP graph and replayed for every chunk that lands in it
(one host launch per CHUNK steps instead of three per step).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from recbole_amd import ops
from recbole_amd._native import AdamTable, check, lib


class _Slot(object):
    """Buffers of one chunk of prepared batches."""

    def __init__(self, C, B, T, dev):
        KI = (1 + T) * B
        self.user_keys = torch.empty(C * B, dtype=torch.int64, device=dev)
        self.item_keys = torch.empty(C * KI, dtype=torch.int64, device=dev)
        self.u_perm = torch.empty(C * B, dtype=torch.int32, device=dev)
        self.u_uniq = torch.empty(C * B, dtype=torch.int32, device=dev)
        self.u_seg = torch.empty(C * (B + 1), dtype=torch.int32, device=dev)
        self.u_nu = torch.zeros(C, dtype=torch.int32, device=dev)
        self.i_perm = torch.empty(C * KI, dtype=torch.int32, device=dev)
        self.i_uniq = torch.empty(C * KI, dtype=torch.int32, device=dev)
        self.i_seg = torch.empty(C * (KI + 1), dtype=torch.int32, device=dev)
        self.i_nu = torch.zeros(C, dtype=torch.int32, device=dev)
        self.ready = torch.cuda.Event()
        self.free = torch.cuda.Event()
        self.free_recorded = False
        self.chunk = None            # (first batch, n batches, batch size)
        self.graph = None            # HIP graph of a full chunk's model-side steps


class FusedBPRTrainStep(object):
    """Device buffers and launch sequence of the fused pairwise train step."""

    CHUNK = 64

    def __init__(self, model, optimizer, train_data, chunk=None, use_graph=True):
        self.model = model
        self.opt = optimizer
        self.data = train_data
        (self.pU, self.nU), (self.pI, self.nI) = model.fused_embedding_tables()
        self.device = self.pU.device
        self.B = train_data.step                   # positives per batch
        self.times = train_data.times              # negatives per positive
        self.uid_field = train_data.uid_field
        self.iid_field = train_data.iid_field
        self.C = chunk or self.CHUNK
        self.use_graph = use_graph
        B, T, d = self.B, self.times, self.pU.shape[1]
        self.d = d
        dev = self.device
        self.gU = torch.empty(B, d, dtype=torch.float32, device=dev)
        self.gI = torch.empty((1 + T) * B, d, dtype=torch.float32, device=dev)
        self.loss_k = torch.empty(B, dtype=torch.float32, device=dev)
        self.slots = [_Slot(self.C, B, T, dev), _Slot(self.C, B, T, dev)]
        self.samp_ws = torch.empty(lib().mirec_sample_walk_workspace_size(B, T),
                                   dtype=torch.uint8, device=dev)
        self.sort_ws = None
        self.prep_stream = torch.cuda.Stream(device=dev)
        self.loss_hist = torch.zeros(1, dtype=torch.float32, device=dev)
        self.consts = torch.zeros(2, dtype=torch.float32, device=dev)
        self.step_idx = torch.zeros(1, dtype=torch.int32, device=dev)
        self.kernel_events = None   # list -> HIP events around the K5 launches (bench.py)
        self.opt._ensure_state(self.pU)
        self.opt._ensure_state(self.pI)
        self._tables = (AdamTable * 2)()
        g = self.opt.param_groups[0]
        self._adam_args = (g['betas'][0], g['betas'][1], g['eps'], g['weight_decay'])

    # ------------------------------------------------------------------ data side
    def _chunks(self):
        n = self._users.numel()
        full = n // self.B
        out = [(b0, min(self.C, full - b0), self.B) for b0 in range(0, full, self.C)]
        if n % self.B:
            out.append((full, 1, n % self.B))
        return out

    def _prepare(self, slot, chunk):
        b0, nb, Bc = chunk
        T = self.times
        KI = (1 + T) * Bc
        if slot.free_recorded:
            self.prep_stream.wait_event(slot.free)
        with torch.cuda.stream(self.prep_stream):
            s0 = b0 * self.B
            users = slot.user_keys[:nb * Bc]
            users.copy_(self._users[s0:s0 + nb * Bc])
            keys = slot.item_keys[:nb * KI].view(nb, 1 + T, Bc)
            keys[:, 0, :].copy_(self._items[s0:s0 + nb * Bc].view(nb, Bc))
            neg = slot.item_keys[Bc:nb * KI]                    # first batch's neg row
            self.data.sampler.launch_batches(users, Bc, nb, T, neg, out_stride=KI,
                                             ws=self.samp_ws)
            self.sort_ws = ops.segment_sort_batched(users, Bc, self.nU, slot.u_perm,
                                                    slot.u_uniq, slot.u_seg, slot.u_nu,
                                                    ws=self.sort_ws)
            self.sort_ws = ops.segment_sort_batched(slot.item_keys[:nb * KI], KI, self.nI,
                                                    slot.i_perm, slot.i_uniq, slot.i_seg,
                                                    slot.i_nu, ws=self.sort_ws)
            slot.ready.record(self.prep_stream)
        slot.chunk = chunk

    # ------------------------------------------------------------------ model side
    def _step(self, slot, c, Bc, stream):
        """Model-side kernels of batch c of `slot` (batch size Bc); every pointer
        is relative to the slot or a persistent buffer (graph-capturable)."""
        T = self.times
        KI = (1 + T) * Bc
        user_p = slot.user_keys.data_ptr() + 8 * c * Bc
        keys_p = slot.item_keys.data_ptr() + 8 * c * KI
        L = lib()
        st = stream.cuda_stream
        rc = L.mirec_bpr_fwd_bwd_f32(self.pU.data_ptr(), self.nU, self.pI.data_ptr(), self.nI,
                                     self.d, user_p, keys_p, keys_p + 8 * Bc, Bc, T, 1e-10,
                                     self._grad_scale(Bc), self.loss_k.data_ptr(), None, None,
                                     self.gU.data_ptr(), self.gI.data_ptr(), st)
        check(rc, 'mirec_bpr_fwd_bwd_f32')
        stU = self.opt.state[self.pU]
        stI = self.opt.state[self.pI]
        t = self._tables
        t[0].p, t[0].m, t[0].v, t[0].n_rows = (self.pU.data_ptr(), stU['exp_avg'].data_ptr(),
                                               stU['exp_avg_sq'].data_ptr(), self.nU)
        t[0].rows, t[0].perm = self.gU.data_ptr(), slot.u_perm.data_ptr() + 4 * c * Bc
        t[0].uniq = slot.u_uniq.data_ptr() + 4 * c * Bc
        t[0].seg = slot.u_seg.data_ptr() + 4 * c * (Bc + 1)
        t[0].n_uniq, t[0].dense_grad = slot.u_nu.data_ptr() + 4 * c, None
        t[1].p, t[1].m, t[1].v, t[1].n_rows = (self.pI.data_ptr(), stI['exp_avg'].data_ptr(),
                                               stI['exp_avg_sq'].data_ptr(), self.nI)
        t[1].rows, t[1].perm = self.gI.data_ptr(), slot.i_perm.data_ptr() + 4 * c * KI
        t[1].uniq = slot.i_uniq.data_ptr() + 4 * c * KI
        t[1].seg = slot.i_seg.data_ptr() + 4 * c * (KI + 1)
        t[1].n_uniq, t[1].dense_grad = slot.i_nu.data_ptr() + 4 * c, None
        ev = self.kernel_events
        if ev is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        rc = L.mirec_adam_multi_f32(t, 2, self.d, self.consts.data_ptr(),
                                    self.step_idx.data_ptr(), *self._adam_args, st)
        check(rc, 'mirec_adam_multi_f32')
        if ev is not None:
            e1.record(stream)
            ev.append((e0, e1))
        rc = L.mirec_step_finish(self.loss_k.data_ptr(), Bc, float(Bc * T),
                                 self.loss_hist.data_ptr(), self.step_idx.data_ptr(), st)
        check(rc, 'mirec_step_finish')

    def _grad_scale(self, Bc):
        R = Bc * self.times
        if getattr(self, '_gs_R', None) != R:
            self._gs_R = R
            self._gs = float(np.float32(1.0) / np.float32(R))
        return self._gs

    def _graph_for(self, slot):
        if slot.graph is None:
            g = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(device=self.device)
            cap.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.graph(g, stream=cap):
                for c in range(self.C):
                    self._step(slot, c, self.B, cap)
            torch.cuda.current_stream(self.device).wait_stream(cap)
            slot.graph = g
        return slot.graph

    # ------------------------------------------------------------------ epoch API
    def begin_epoch(self):
        """Shuffle (reference order of RNG use), stage the epoch's Adam constants,
        and start preparing the first chunks; returns the number of batches."""
        data = self.data
        if data.shuffle:
            data._shuffle()                     # randperm (CPU RNG) + device reorder
        inter = data.dataset.inter_feat
        self._users = inter[self.uid_field]
        self._items = inter[self.iid_field]
        if not self._users.is_cuda:
            raise RuntimeError('fused train step needs the train table on the GPU')
        self.n_batches = nb = math.ceil(self._users.numel() / self.B)
        table = self.opt.step_constants(self.opt.n_steps + 1, max(nb, 1)).reshape(-1)
        if self.consts.numel() < table.size:   # persistent buffers (graph-captured pointers)
            self.consts = torch.zeros(table.size, dtype=torch.float32, device=self.device)
            self.loss_hist = torch.zeros(max(nb, 1), dtype=torch.float32, device=self.device)
            for s in self.slots:
                s.graph = None
        self.consts[:table.size].copy_(torch.from_numpy(table))
        self.loss_hist.zero_()
        self.step_idx.zero_()
        if self.use_graph and nb >= self.C:
            for s in self.slots:                # capture up front: capture synchronizes
                self._graph_for(s)
        self.prep_stream.wait_stream(torch.cuda.current_stream(self.device))
        self._plan = self._chunks()
        self._next_chunk = 0
        self._cur = None                       # chunk index being consumed
        for s in self.slots:
            s.free_recorded = False
        self._issue_prep()
        self._issue_prep()
        return nb

    def _issue_prep(self):
        k = self._next_chunk
        if k >= len(self._plan):
            return
        self._prepare(self.slots[k % 2], self._plan[k])
        self._next_chunk += 1

    def _enter_chunk(self, k, stream):
        if self._cur == k:
            return
        if self._cur is not None:              # previous chunk fully enqueued
            prev = self.slots[self._cur % 2]
            prev.free.record(stream)
            prev.free_recorded = True
        while self._next_chunk <= k + 1 and self._next_chunk < len(self._plan):
            self._issue_prep()
        stream.wait_event(self.slots[k % 2].ready)
        self._cur = k

    def run_batches(self, b_start, b_end):
        """Enqueue batches [b_start, b_end) in order (no host sync). Whole chunks
        replay their captured graph; partial chunks launch eagerly."""
        stream = torch.cuda.current_stream(self.device)
        b = b_start
        while b < b_end:
            k = self._chunk_of(b)
            b0, nb, Bc = self._plan[k]
            self._enter_chunk(k, stream)
            slot = self.slots[k % 2]
            c0, c1 = b - b0, min(nb, b_end - b0)
            if (self.use_graph and c0 == 0 and c1 == nb == self.C and Bc == self.B
                    and self.kernel_events is None):
                self._graph_for(slot).replay()
            else:
                for c in range(c0, c1):
                    self._step(slot, c, Bc, stream)
            b = b0 + c1

    def launch_batch(self, b):
        self.run_batches(b, b + 1)

    def _chunk_of(self, b):
        full = self._users.numel() // self.B
        if b >= full:
            return len(self._plan) - 1
        return b // self.C

    def end_epoch(self, n_done=None):
        """Account the optimizer steps and read the per-batch losses back (one sync)."""
        n_done = self.n_batches if n_done is None else n_done
        stream = torch.cuda.current_stream(self.device)
        stream.wait_stream(self.prep_stream)
        self.opt.advance(n_done)
        self.data.pr = 0
        return [float(x) for x in self.loss_hist[:n_done].cpu().numpy()]

    def run_epoch(self):
        """One epoch; returns the list of per-batch mean losses (host floats)."""
        nb = self.begin_epoch()
        self.run_batches(0, nb)
        return self.end_epoch()


def fused_full_sort_eval(model, eval_data, topk_evaluator, user_batch=1 << 20):
    """Trainer.evaluate for a FULL loader (trainer.py:355-412) on K6: scores,
    pad/history mask, top-K and positive flags in one kernel per user batch; only
    the [n_users, K] positive matrix returns to the host for the metric
    reduction (evaluators.py:122-141)."""
    dev = model.fused_item_table().device
    K = max(topk_evaluator.topk)
    uids = torch.as_tensor(eval_data.uid_list, dtype=torch.int64, device=dev)
    hist_ptr = torch.as_tensor(eval_data.hist_ptr, device=dev)
    hist_cols = torch.as_tensor(eval_data.hist_cols if len(eval_data.hist_cols)
                                else np.zeros(1, np.int32), device=dev)
    pos_ptr = torch.as_tensor(eval_data.pos_ptr, device=dev)
    pos_cols = torch.as_tensor(eval_data.pos_cols, device=dev)
    EI = model.fused_item_table().contiguous()
    n = uids.numel()
    flags = torch.empty(n, K, dtype=torch.uint8, device=dev)
    for s in range(0, n, user_batch):
        e = min(n, s + user_batch)
        Uq = model.fused_user_vectors(uids[s:e]).contiguous()
        o = {'pos_flags': flags[s:e]}
        ops.fullsort_topk(Uq, EI, K, hist_ptr=hist_ptr[s:e + 1], hist_cols=hist_cols,
                          pos_ptr=pos_ptr[s:e + 1], pos_cols=pos_cols, out=o)
    pos_idx = flags.cpu().numpy().astype(bool)
    return topk_evaluator.evaluate_pos_idx(pos_idx, eval_data.get_pos_len_list())
