"""Fused train step and full-sort evaluation for embedding models (BPR-MF).

One training step of Trainer._train_epoch (trainer.py:157-174) for a pairwise
model with learner 'adam', as hand-written gfx950 kernels with no host
synchronisation inside the epoch. The work splits by dependency:

data side (depends only on ids; runs AHEAD on a side stream, CHUNK batches per launch)
  K4 sampler walk  (sampler.py:103-154)   negatives of CHUNK future batches, written
                                           straight into per-batch [pos | neg] key rows
  K2 segment sort  (embedding backward)   rows grouped by table row, one workgroup/batch
model side (main stream, per batch)
  K3 fused BPR     (bpr.py:74-83)         loss rows + per-row gradients (G > 1: forward +
                                           coefficient exchange + rebuild of the rows)
  K5 dense Adam    (optim.Adam.step)      both tables in one launch, grouped gradients
                                           summed on the fly; schedule 'deferred' (default)
                                           or 'streamed', bit-identical (see adam.hip)
  chunk_finish                            per-step mean losses kept on the device
  K5 flush         ('deferred' only)      once per chunk: every row caught up

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

Deferred Adam: the reference's dense Adam moves every row every step, but a row
with a zero gradient moves as a function of its own (p, m, v) and the step
constants only. The deferred schedule applies those zero-gradient steps when the
row is next touched (or at the per-chunk flush), with the same per-element
arithmetic, so the parameters after a flush are bit-identical to the streamed
schedule's while a step moves only the rows its batch touches. Parameters are
complete after end_epoch() / sync_params().
"""
from __future__ import annotations

import ctypes
import logging
import math
import os

import numpy as np
import torch

from recbole_amd import ops
from recbole_amd._native import AdamTable, check, lib
from recbole_amd.trainer.exchange import ExchangeLayout

# K35 record widths (int32 per touched-row slot / per grouped position, include/mirec.h
# mirec_step_records)
REC_CONTRIB = 8
ADAM_MODES = ('deferred', 'streamed')


_PREP_STREAMS = {}


def _prep_streams_for(dev, n=2):
    """n side streams whose hardware queues are neither the current stream's nor
    each other's.

    HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES, 4 by
    default) round-robin; a side stream that lands on the main stream's queue
    runs in order with it, so the chunk preparation would run behind the model
    steps instead of beside them (and two prep streams on one queue would run
    the walk and the grouping in order again). Probe: hold the current stream
    and the streams already chosen busy with spin kernels and see whether an
    event on the candidate completes meanwhile (a dedicated high-priority or
    CU-masked queue avoids the sharing too, but measured 4-8x slower kernels on
    both queues: the extra queue oversubscribes the hardware queue slots). Falls
    back to the first candidates."""
    key = (str(dev), n)
    got = _PREP_STREAMS.get(key)
    if got is not None:
        return got
    import time
    main = torch.cuda.current_stream(dev)
    chosen, spare = [], []
    for _ in range(16):
        if len(chosen) == n:
            break
        cand = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize(dev)
        for busy in [main] + chosen:
            with torch.cuda.stream(busy):
                torch.cuda._sleep(int(2.4e3 * 3000))      # ~3 ms of spinning
        ev = torch.cuda.Event()
        with torch.cuda.stream(cand):
            torch.cuda._sleep(1)
            ev.record(cand)
        t0 = time.perf_counter()
        free = False
        while time.perf_counter() - t0 < 1.5e-3:
            if ev.query():
                free = True
                break
        torch.cuda.synchronize(dev)
        (chosen if free else spare).append(cand)
    while len(chosen) < n:
        chosen.append(spare.pop(0) if spare else torch.cuda.Stream(device=dev))
    _PREP_STREAMS[key] = chosen
    return chosen


class _Slot(object):
    """Buffers of one chunk of prepared batches (global-batch keys and groupings;
    for G > 1 also this rank's local key slices)."""

    def __init__(self, C, B, T, G, dev, ahead):
        Bg = G * B
        KI = (1 + T) * Bg
        self.user_keys = torch.empty(C * Bg, dtype=torch.int64, device=dev)
        self.item_keys = torch.empty(C * KI, dtype=torch.int64, device=dev)
        if G > 1:
            self.lu = torch.empty(C * B, dtype=torch.int64, device=dev)
            self.li = torch.empty(C * (1 + T) * B, dtype=torch.int64, device=dev)
        self.u_perm = torch.empty(C * Bg, dtype=torch.int32, device=dev)
        self.u_uniq = torch.empty(C * Bg, dtype=torch.int32, device=dev)
        self.u_seg = torch.empty(C * (Bg + 1), dtype=torch.int32, device=dev)
        self.u_nu = torch.zeros(C, dtype=torch.int32, device=dev)
        self.i_perm = torch.empty(C * KI, dtype=torch.int32, device=dev)
        self.i_uniq = torch.empty(C * KI, dtype=torch.int32, device=dev)
        self.i_seg = torch.empty(C * (KI + 1), dtype=torch.int32, device=dev)
        self.i_nu = torch.zeros(C, dtype=torch.int32, device=dev)
        if ahead:                    # deferred Adam: rows batch c+1 reads, batch c does not touch
            self.u_ahead = torch.empty(C * Bg, dtype=torch.int32, device=dev)
            self.u_nah = torch.zeros(C, dtype=torch.int32, device=dev)
            self.i_ahead = torch.empty(C * KI, dtype=torch.int32, device=dev)
            self.i_nah = torch.zeros(C, dtype=torch.int32, device=dev)
        self.records = None          # K35 row / contribution records (FusedBPRTrainStep)
        self.ready = torch.cuda.Event()
        self.walked = torch.cuda.Event()
        self.free = torch.cuda.Event()
        # torch creates an event's HIP object at its first record (hipEventCreate, tens of
        # microseconds of host time): record each one now, so a timed region never pays it
        cur = torch.cuda.current_stream(dev)
        for ev in (self.ready, self.walked, self.free):
            ev.record(cur)
        self.free_recorded = False
        self.group_pending = False   # walked, grouping not yet issued
        self.chunk = None            # (first global batch, n batches, global batch size)
        self.graphs = {}             # (n batches, entry, flush) -> HIP graph of the model side


class FusedBPRTrainStep(object):
    """Device buffers and launch sequence of the fused pairwise train step.

    Data parallel over G ranks (`dist` = a torch.distributed process group, or None
    for one GPU): one optimizer step consumes a GLOBAL batch of G*B positives, rank g
    runs K3's forward on positives [g*B, (g+1)*B) of it (losses + one coefficient per
    row), one all-gather (RCCL over xGMI) exchanges those (trainer/exchange.py: 4 B per
    row instead of a d-float gradient row), and every rank rebuilds the global batch's
    gradient rows with the same arithmetic as K3 and applies the same Adam step. The
    sampler walk and the grouping of the global batch are computed on every rank
    (cheap, on the prep stream), so each rank's result is bit-identical to ONE GPU
    running the global batch (tables and Adam state are replicas: 288 GB per GPU).
    A ragged last batch is computed whole on every rank (no exchange)."""

    CHUNK = 64
    SLOTS = 3                     # chunk buffers in flight (walk, grouping, model)
    # chunk sizes after a (re)start of the prep pipeline. With the speculative walk and K36 a
    # chunk's preparation is ~45 us for 8 batches, and a preparation issued beside the model's
    # K35 steps mostly waits for CUs (K35 fills the chip): the C2 driver window (warm-up 5,
    # 20 timed steps) measured 21.7-21.9 M positives/s with chunks of 8 then 12 against
    # 20.8-21.2 M with 4, 8, 8 and 21.0-21.5 M with one chunk of 20
    RAMP = (8, 16, 32)
    # deferred schedule: steps between full-table flushes (every row complete;
    # parameters are also complete at every epoch end / sync_params()). Rarer
    # flushes let idle rows reach the cheap replay regime (adam.hip
    # p_update_vanishes) but lengthen the lags the per-step kernel replays when a
    # row is touched, and its slowest wave sets the step time: measured on C2 (64
    # warm-up + 256 steps) 18.0 M positives/s at 64, 12.4 M at 256, 12.3 M at 1,024.
    FLUSH_EVERY = 64
    # A chunk the model side waits for at once (pipeline (re)start: the epoch's first chunk,
    # or a timed region that holds its own preparation) is walked and grouped on the model's
    # stream — no hand-off between hardware queues (≈ 20 µs each) before the first step —
    # and the next chunks' walks are issued on the prep stream right behind its walk (they
    # run beside its grouping and steps). MIREC_MAIN_FIRST=0: the prep streams for it too.
    MAIN_FIRST = os.environ.get('MIREC_MAIN_FIRST', '1') != '0'
    _last_walked = None           # event after the latest issued walk (begin_epoch resets)
    _deferred_waits = ()          # cross-stream waits on a restart chunk, issued with the next walk
    _urgent = False               # the next chunk prepared is the one after a restart
    _late_top_up = None           # restart chunk whose next walks follow its model launch

    def __init__(self, model, optimizer, train_data, chunk=None, use_graph=True,
                 adam_mode='deferred', dist=None, fused_step=None):
        if adam_mode not in ADAM_MODES:
            raise ValueError(f'adam_mode must be one of {ADAM_MODES}, got {adam_mode!r}')
        self.model = model
        self.opt = optimizer
        self.data = train_data
        (self.pU, self.nU), (self.pI, self.nI) = model.fused_embedding_tables()
        self.device = self.pU.device
        self.B = train_data.step                   # positives per batch per rank
        self.times = train_data.times              # negatives per positive
        self.uid_field = train_data.uid_field
        self.iid_field = train_data.iid_field
        self.C = chunk or self.CHUNK
        self.use_graph = use_graph
        self.adam_mode = adam_mode
        self.group = dist
        if dist is not None:
            import torch.distributed as tdist
            self.G, self.rank = tdist.get_world_size(dist), tdist.get_rank(dist)
            self._backend = str(tdist.get_backend(dist))
            if self._backend != 'nccl':        # host-staged collectives cannot be captured
                self.use_graph = use_graph = False
        else:
            self.G, self.rank, self._backend = 1, 0, None
        B, T, G, d = self.B, self.times, self.G, self.pU.shape[1]
        self.Bg = G * B                            # positives per optimizer step
        self.d = d
        dev = self.device
        self.layout = ExchangeLayout(G, B, T, d)
        # gradient rows of the (global) batch: [user rows | item rows]
        self.xbuf = torch.empty(self.Bg * (2 + T) * d, dtype=torch.float32, device=dev)
        # data parallel: per-rank [losses | coefficients] blocks, all-gathered per step
        self.xchg = torch.empty(G * self.layout.W, dtype=torch.float32, device=dev)
        self.loss_k = torch.empty(self.C * self.Bg, dtype=torch.float32, device=dev)
        deferred = adam_mode == 'deferred'
        self.slots = [_Slot(self.C, B, T, G, dev, deferred) for _ in range(self.SLOTS)]
        self.samp_ws = torch.empty(lib().mirec_sample_walk_workspace_size(self.Bg, T),
                                   dtype=torch.uint8, device=dev)
        self.sort_ws = None
        # keys + K4 walk on one side stream, K2 grouping + look-ahead lists on a
        # second: chunk c+1 walks while chunk c is grouped; neither shares the main
        # stream's hardware queue (_prep_streams_for)
        self.prep_stream, self.group_stream = _prep_streams_for(dev)
        self.zero_i32 = torch.zeros(1, dtype=torch.int32, device=dev)
        self.loss_hist = torch.zeros(1, dtype=torch.float32, device=dev)
        self.consts = torch.zeros(4, dtype=torch.float32, device=dev)
        self.step_idx = torch.zeros(1, dtype=torch.int32, device=dev)
        self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)   # mirec_chunk_finish
        self.kernel_events = None   # list -> (name, start, end) HIP events (bench.py)
        self.kernel_uniq = []       # per eager step: [touched users, touched items]
        self._plan, self._plan_starts = [], None
        self._current = True        # no step enqueued since the last flush
        self.n_eager_steps = 0      # steps launched outside a captured chunk graph
        self.opt._ensure_state(self.pU)
        self.opt._ensure_state(self.pI)
        self._tables = (AdamTable * 2)()
        if deferred:
            self.lastU = torch.zeros(self.nU, dtype=torch.int32, device=dev)
            self.lastI = torch.zeros(self.nI, dtype=torch.int32, device=dev)
        # K35 (csrc/step.hip): the model side of a step in ONE launch (BPR + the touched
        # rows' Adam + look-ahead), bit-identical to K3 + K5. One GPU, deferred schedule;
        # needs the parity buffers of p (state after t steps in t & 1 ? alt : p)
        if fused_step is None:
            fused_step = deferred and G == 1 and d in (64, 128, 256)
        if fused_step and not (deferred and G == 1 and d in (64, 128, 256)):
            raise ValueError('fused_step needs adam_mode="deferred", one rank and d in '
                             '{64, 128, 256}')
        self.fused_step = bool(fused_step)
        self.pU_alt = torch.empty_like(self.pU.data) if self.fused_step else None
        self.pI_alt = torch.empty_like(self.pI.data) if self.fused_step else None
        self._rec_w = {}
        if self.fused_step:          # K35 records per slot (mirec_step_records, prep stream)
            for sl in self.slots:
                sl.records = [torch.empty(self.C * w, dtype=torch.int32, device=dev)
                              for w in self._rec_ints(self.Bg)]
            # split rows' hand-off scratch (one launch at a time on the compute stream)
            self._step_scratch = ops.step_scratch(self.Bg, T, d, dev)
        self._n_max = (ctypes.c_int64 * 2)(self.Bg, (1 + T) * self.Bg)
        g = self.opt.param_groups[0]
        self._adam_args = (g['betas'][0], g['betas'][1], g['eps'], g['weight_decay'])
        self._fill_tables()

    # ------------------------------------------------------------------ data side
    def _chunks(self, cuts=(), ramps=(0,)):
        """(first global batch, batches, global batch size) per chunk: chunks of at
        most C full batches, starting at 0 and at every batch index in `cuts`, then
        the ragged last batch on its own. From each batch index in `ramps` (where
        the prep pipeline starts empty) up to the next cut, the chunk sizes ramp up
        (RAMP, then C): the first steps wait for a 4-batch walk, not a C-batch one,
        and each next walk runs beside the previous chunk's steps."""
        n = self._users.numel()
        full = n // self.Bg
        bounds = sorted({0, full} | {int(c) for c in cuts if 0 < int(c) < full})
        ramp_at = {int(r) for r in ramps}
        out = []
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            ri = 0 if lo in ramp_at else len(self.RAMP)
            b0 = lo
            while b0 < hi:
                size = self.RAMP[ri] if ri < len(self.RAMP) else self.C
                ri += 1
                nb = min(size, self.C, hi - b0)
                out.append((b0, nb, self.Bg))
                b0 += nb
        if n % self.Bg:
            out.append((full, 1, n % self.Bg))
        return out

    def _chunk_flags(self, plan):
        """(entry, flush) per chunk of the deferred schedule: a chunk flushes every
        row at its end once FLUSH_EVERY or more steps have run since the last flush, or
        when the next chunk would take the count past 1.5 x FLUSH_EVERY (the ramp's
        4 + 8 + 16 + 32 steps flush before the first 64-step chunk instead of after it),
        and before a ragged batch / the end; a chunk after one that did not flush starts
        with an entry catch-up of the rows its first batch reads. `flush` is False or
        the flush's rows per wave per table (_flush_rows: a tuple, part of the chunk
        graph's key)."""
        flags, since = [], 0
        at = getattr(self, '_flush_at', set())
        for i, (b0, nb, Bc) in enumerate(plan):
            entry = since > 0
            since += nb
            nxt_full = i + 1 < len(plan) and plan[i + 1][2] == self.Bg
            nxt_nb = plan[i + 1][1] if i + 1 < len(plan) else 0
            flush = (since >= self.FLUSH_EVERY or since + nxt_nb > self.FLUSH_EVERY * 3 // 2
                     or not nxt_full or b0 + nb in at)
            if flush:
                since = 0
            flags.append((entry, self._flush_rows(b0 + nb) if flush else False))
        return flags

    # a flush of a table whose rows are mostly current (zero state) runs R rows per wave
    # (mirec_adam_flush_rows_f32) when about one row per R would lag
    FLUSH_SPARSE_MAX_ROWS = 8

    def _flush_rows(self, b_end):
        """Rows per wave of the flush after global batch b_end - 1, per table: an upper
        bound on the rows that can lag = the rows outside the zero state at the epoch
        start + every row the steps since then touched (B users, (1+T)B item slots per
        step); R = the largest power of two <= FLUSH_SPARSE_MAX_ROWS with R x that
        fraction <= 1 (one wave per row, R = 1, where most rows lag)."""
        if self.adam_mode != 'deferred' or self.d < 64:
            return (1, 1)
        out = []
        for q, per in enumerate((self.Bg, (1 + self.times) * self.Bg)):
            n_rows, busy0 = self._tables[q].n_rows, self._busy0[q]   # (a shard when sharded)
            frac = min(1.0, (busy0 + b_end * per) / max(n_rows, 1))
            r = 1
            while r * 2 <= self.FLUSH_SPARSE_MAX_ROWS and r * 2 * frac <= 1.0:
                r *= 2
            out.append(r)
        return tuple(out)

    def _sharded(self, Bc):
        return self.G > 1 and Bc == self.Bg

    def _prepare(self, slot, chunk, on=None):
        """Issue the walk half of a chunk's preparation on the prep stream, or — `on`, a
        pipeline (re)start whose chunk the model side waits for at once — the whole
        preparation on that stream (no cross-queue hand-off on the critical path; the
        prep and group streams order their next launches after it)."""
        b0, nb, Bc = chunk
        T = self.times
        KI = (1 + T) * Bc
        if slot.free_recorded and on is None and not slot.free.query():
            self.prep_stream.wait_event(slot.free)     # (a completed event needs no wait)
        if not self._sharded(Bc):
            # keys, K4 walk, K2 groupings and look-ahead lists: one native call
            # (mirec_prepare_chunk) on the prep stream
            cp = self._chunk_prep(slot)
            cp.users, cp.items = self._users.data_ptr(), self._items.data_ptr()
            cp.s0, cp.n_batches, cp.Bc = b0 * self.Bg, nb, Bc
            samp = self.data.sampler
            if samp.alias is not None:              # fast mode: draw ids of this chunk
                thr, idx, cp.alias_seed, cp.alias_counter = samp.alias_args(
                    self.device, nb * Bc * T)
                cp.alias_thr, cp.alias_idx, cp.n_alias = thr.data_ptr(), idx.data_ptr(), thr.numel()
            st = on if on is not None else self.prep_stream
            slot.ready_on_model = on is not None
            if on is None:
                self._apply_deferred_waits()
            lw = self._last_walked
            if on is not None and lw is not None and not lw.query():
                # the walk pointer and the speculative walk's workspace are sequential
                # state: a walk on the model's stream follows every walk issued before it
                on.wait_event(lw)
            check(lib().mirec_prepare_chunk_walk(ctypes.byref(cp), st.cuda_stream),
                  'mirec_prepare_chunk_walk')
            slot.walked.record(st)
            self._last_walked = slot.walked
            slot.chunk = chunk
            if on is None:
                if self._urgent:
                    # the chunk right after a restart: its grouping at once, on the same
                    # stream behind its walk (no hand-off between hardware queues)
                    self._urgent = False
                    check(lib().mirec_prepare_chunk_group(ctypes.byref(cp), st.cuda_stream),
                          'mirec_prepare_chunk_group')
                    slot.ready.record(st)
                    self.group_stream.wait_event(slot.ready)     # shared sort workspace
                    slot.group_pending = False
                    return
                slot.group_pending = True      # the grouping half: _issue_groups
                return
            check(lib().mirec_prepare_chunk_group(ctypes.byref(cp), st.cuda_stream),
                  'mirec_prepare_chunk_group')
            slot.ready.record(st)
            # the prep / group streams' waits on this chunk (the next walks continue its walk
            # pointer; the sort workspace is shared) go in with the next walk — after the
            # chunk's model launch, so the host's time first goes to what the GPU reaches first
            self._deferred_waits = [(self.prep_stream, slot.walked),
                                    (self.group_stream, slot.ready)]
            slot.group_pending = False
            return
        with torch.cuda.stream(self.prep_stream):
            s0 = b0 * self.Bg
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
            lay, g, B = self.layout, self.rank, self.B
            slot.lu[:nb * B].view(nb, B).copy_(lay.local_users(users, g))
            slot.li[:nb * (1 + T) * B].view(nb, 1 + T, B).copy_(
                lay.local_items(slot.item_keys[:nb * KI], g))
            if self.adam_mode == 'deferred':
                ops.uniq_ahead_diff(slot.u_uniq, slot.u_nu, Bc, nb, slot.u_ahead, slot.u_nah)
                ops.uniq_ahead_diff(slot.i_uniq, slot.i_nu, KI, nb, slot.i_ahead, slot.i_nah)
            slot.ready.record(self.prep_stream)
        slot.chunk = chunk

    def _apply_deferred_waits(self):
        for st, ev in self._deferred_waits:
            st.wait_event(ev)
        self._deferred_waits = []

    def _prepare_group(self, slot):
        """The grouping half of a chunk's preparation (K2 + look-ahead lists) on the
        group stream, after the chunk's walk."""
        self._apply_deferred_waits()
        self.group_stream.wait_event(slot.walked)
        check(lib().mirec_prepare_chunk_group(ctypes.byref(slot.prep),
                                              self.group_stream.cuda_stream),
              'mirec_prepare_chunk_group')
        slot.ready.record(self.group_stream)
        slot.group_pending = False

    def _chunk_prep(self, slot):
        """The slot's mirec_chunk_prep descriptor (pointers fixed per slot)."""
        cp = getattr(slot, 'prep', None)
        if cp is not None:
            return cp
        from recbole_amd._native import ChunkPrep
        dev = self.device
        with torch.cuda.stream(self.prep_stream):   # a first call builds the used-id bitmap:
            walk = self.data.sampler.walk_args(dev)   # stream-ordered before the walk reads it
        rl, pr, up, uc, bits, n_bits, reject, status = walk
        T = self.times
        nsort = lib().mirec_segment_sort_workspace_size(self.C * (1 + T) * self.Bg, self.nI)
        if self.sort_ws is None or self.sort_ws.numel() < nsort:
            self.sort_ws = torch.empty(nsort, dtype=torch.uint8, device=dev)
        p = lambda x: x.data_ptr() if x is not None else None
        cp = ChunkPrep()
        cp.T = T
        cp.user_keys, cp.item_keys = slot.user_keys.data_ptr(), slot.item_keys.data_ptr()
        cp.random_list, cp.L, cp.pr_dev = rl.data_ptr(), rl.numel(), pr.data_ptr()
        cp.used_ptr, cp.used_cols = (p(up), p(uc)) if bits is None else (None, None)
        cp.used_bits, cp.n_bits = p(bits), n_bits if bits is not None else 0
        cp.n_users, cp.n_items, cp.reject, cp.status = self.nU, self.nI, int(reject), p(status)
        cp.walk_ws, cp.walk_ws_bytes = self.samp_ws.data_ptr(), self.samp_ws.numel()
        cp.sort_ws, cp.sort_ws_bytes = self.sort_ws.data_ptr(), self.sort_ws.numel()
        for tag in ('u', 'i'):
            for f in ('perm', 'uniq', 'seg', 'nu'):
                setattr(cp, f'{tag}_{f}', getattr(slot, f'{tag}_{f}').data_ptr())
            if self.adam_mode == 'deferred':
                setattr(cp, f'{tag}_ahead', getattr(slot, f'{tag}_ahead').data_ptr())
                setattr(cp, f'{tag}_nah', getattr(slot, f'{tag}_nah').data_ptr())
        if slot.records is not None:
            cp.u_rec, cp.u_crec, cp.i_rec, cp.i_crec = (r.data_ptr() for r in slot.records)
        spec = self._spec_ws()
        if spec is not None:                        # K4s: the speculative walk
            cp.spec_ws, cp.spec_ws_bytes = spec.data_ptr(), spec.numel()
            cp.r_mean, cp.r_sd = self._spec_stats
        slot.prep = cp
        return cp

    # K4s (mirec_sample_walk_spec): the chunk's walk by speculation (exact; two launches
    # per 16 batches instead of a serial walk of ~10 us per batch)
    SPEC_WALK = os.environ.get('MIREC_SPEC_WALK', '1') != '0'

    def _spec_ws(self):
        """Workspace of the speculative walk (shared by the slots: the walks run in
        order on the walk stream), or None where it does not apply."""
        if not self.SPEC_WALK or self.data.sampler.alias is not None:
            return None
        T, Bc = self.times, self.Bg
        if Bc > 1024 or Bc * T > 4096:
            return None
        ws = getattr(self, '_spec_buf', None)
        if ws is None:
            counts = np.bincount(self._users.cpu().numpy(), minlength=self.nU)
            self._spec_stats = self.data.sampler.walk_stats(counts, Bc, T)
            n = lib().mirec_sample_walk_spec_workspace_size(Bc, T, min(self.C, 16),
                                                            *self._spec_stats)
            ws = self._spec_buf = torch.empty(n, dtype=torch.uint8, device=self.device)
        return ws

    # ------------------------------------------------------------------ model side
    def _rec_ints(self, Bc):
        """int32 per batch of the four K35 record buffers for batches of Bc positives."""
        w = self._rec_w.get(Bc)
        if w is None:
            KI = (1 + self.times) * Bc
            w = self._rec_w[Bc] = (ops.step_record_ints(Bc), Bc * REC_CONTRIB,
                                   ops.step_record_ints(KI), KI * REC_CONTRIB)
        return w

    def _fill_tables(self):
        """Per-table pointers that do not depend on the batch."""
        stU = self.opt.state[self.pU]
        stI = self.opt.state[self.pI]
        t = self._tables
        t[0].p, t[0].m, t[0].v, t[0].n_rows = (self.pU.data_ptr(), stU['exp_avg'].data_ptr(),
                                               stU['exp_avg_sq'].data_ptr(), self.nU)
        t[1].p, t[1].m, t[1].v, t[1].n_rows = (self.pI.data_ptr(), stI['exp_avg'].data_ptr(),
                                               stI['exp_avg_sq'].data_ptr(), self.nI)
        t[0].dense_grad = t[1].dense_grad = None
        if self.adam_mode == 'deferred':
            t[0].last, t[1].last = self.lastU.data_ptr(), self.lastI.data_ptr()
        else:
            t[0].last = t[1].last = None
        fs = getattr(self, 'fused_step', False)
        t[0].p_alt = self.pU_alt.data_ptr() if fs else None
        t[1].p_alt = self.pI_alt.data_ptr() if fs else None

    def _adam_state(self):
        """(m, v, deferred step counts) of each table."""
        stU, stI = self.opt.state[self.pU], self.opt.state[self.pI]
        return [(stU['exp_avg'], stU['exp_avg_sq'], self.lastU),
                (stI['exp_avg'], stI['exp_avg_sq'], self.lastI)]

    def _record(self, name, stream, fn):
        ev = self.kernel_events
        if ev is None:
            return fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        ev.append((name, e0, e1))

    def _step(self, slot, c, Bc, stream, step_off, ahead):
        """Model-side work of global batch c of `slot` (Bc positives) as optimizer
        step step_idx + step_off; every pointer is relative to the slot or a
        persistent buffer (graph-capturable). `ahead`: batch c+1 of the slot runs
        next, so the deferred Adam also completes the rows it reads."""
        T, d = self.times, self.d
        KI = (1 + T) * Bc
        L = lib()
        st = stream.cuda_stream
        sharded = self._sharded(Bc)
        x0 = self.xbuf.data_ptr()
        loss_p = self.loss_k.data_ptr() + 4 * c * self.Bg
        user_g = slot.user_keys.data_ptr() + 8 * c * Bc      # the (global) batch
        keys_g = slot.item_keys.data_ptr() + 8 * c * KI
        gU, gI = x0, x0 + 4 * Bc * d
        rowsU, rowsI = gU, gI
        if sharded:
            # K3 forward on the local slice -> [losses | coefficients] of this rank's
            # block; all-gather; every rank rebuilds the global batch's gradient rows
            lay, B = self.layout, self.B
            user_p = slot.lu.data_ptr() + 8 * c * B
            keys_p = slot.li.data_ptr() + 8 * c * (1 + T) * B
            mine = self.xchg.data_ptr() + 4 * self.rank * lay.W

            def bpr():
                check(L.mirec_bpr_fwd_coef_f32(self.pU.data_ptr(), self.nU, self.pI.data_ptr(),
                                               self.nI, d, user_p, keys_p, keys_p + 8 * B, B, T,
                                               1e-10, self._grad_scale(Bc), mine,
                                               mine + 4 * lay.coef0, st),
                      'mirec_bpr_fwd_coef_f32')
            self._record('bpr', stream, bpr)
            self._record('exchange', stream, lambda: self._exchange(c))

            def contrib():
                check(L.mirec_bpr_contrib_f32(self.pU.data_ptr(), self.nU, self.pI.data_ptr(),
                                              self.nI, d, user_g, keys_g, keys_g + 8 * Bc, Bc, T,
                                              self.xchg.data_ptr() + 4 * lay.coef0, B, lay.W,
                                              gU, gI, st), 'mirec_bpr_contrib_f32')
            self._record('contrib', stream, contrib)
        elif not self.fused_step:
            def bpr():
                check(L.mirec_bpr_fwd_bwd_f32(self.pU.data_ptr(), self.nU, self.pI.data_ptr(),
                                              self.nI, d, user_g, keys_g, keys_g + 8 * Bc, Bc,
                                              T, 1e-10, self._grad_scale(Bc), loss_p, None,
                                              None, gU, gI, st), 'mirec_bpr_fwd_bwd_f32')
            self._record('bpr', stream, bpr)
        t = self._tables
        t[0].rows, t[1].rows = rowsU, rowsI
        t[0].perm = slot.u_perm.data_ptr() + 4 * c * Bc
        t[0].uniq = slot.u_uniq.data_ptr() + 4 * c * Bc
        t[0].seg = slot.u_seg.data_ptr() + 4 * c * (Bc + 1)
        t[0].n_uniq = slot.u_nu.data_ptr() + 4 * c
        t[1].perm = slot.i_perm.data_ptr() + 4 * c * KI
        t[1].uniq = slot.i_uniq.data_ptr() + 4 * c * KI
        t[1].seg = slot.i_seg.data_ptr() + 4 * c * (KI + 1)
        t[1].n_uniq = slot.i_nu.data_ptr() + 4 * c
        if self.adam_mode == 'deferred' and ahead:
            t[0].ahead_uniq = slot.u_ahead.data_ptr() + 4 * c * Bc
            t[0].ahead_n_uniq = slot.u_nah.data_ptr() + 4 * c
            t[1].ahead_uniq = slot.i_ahead.data_ptr() + 4 * c * KI
            t[1].ahead_n_uniq = slot.i_nah.data_ptr() + 4 * c
        else:
            t[0].ahead_uniq = t[0].ahead_n_uniq = t[1].ahead_uniq = t[1].ahead_n_uniq = None

        if self.fused_step and not sharded:
            # K35: BPR + touched-row Adam + look-ahead in one launch (no gradient rows),
            # the touched rows from the chunk's records (built on the prep stream)
            rec = [r.data_ptr() + 4 * c * w for r, w in zip(slot.records, self._rec_ints(Bc))]
            rec += [x.data_ptr() for x in self._step_scratch]

            def fused():
                check(L.mirec_bpr_adam_step_f32(t, self._n_max, d, keys_g, Bc, T, 1e-10,
                                                self._grad_scale(Bc), loss_p, *rec,
                                                self.consts.data_ptr(),
                                                self.step_idx.data_ptr(), step_off,
                                                *self._adam_args, st), 'mirec_bpr_adam_step_f32')
            self._record('step', stream, fused)
            if self.kernel_events is not None:
                self.kernel_uniq.append(torch.stack([slot.u_nu[c], slot.i_nu[c]]))
            return
        if self.adam_mode == 'deferred':
            def adam():
                check(L.mirec_adam_deferred_f32(t, 2, self._n_max, d, self.consts.data_ptr(),
                                                self.step_idx.data_ptr(), step_off,
                                                *self._adam_args, st), 'mirec_adam_deferred_f32')
        else:
            def adam():
                check(L.mirec_adam_multi_f32(t, 2, d, self.consts.data_ptr(),
                                             self.step_idx.data_ptr(), step_off,
                                             *self._adam_args, st), 'mirec_adam_multi_f32')
        self._record('adam', stream, adam)
        if self.kernel_events is not None:       # rows touched, for the bench's byte count
            self.kernel_uniq.append(torch.stack([slot.u_nu[c], slot.i_nu[c]]))

    def _exchange(self, c):
        """All-gather every rank's [losses | coefficients] block (RCCL over xGMI: 10 KB
        per rank at C2), then lay the G*B losses out in global positive order for
        chunk_finish."""
        import torch.distributed as tdist
        lay = self.layout
        parts = list(self.xchg.view(self.G, lay.W).unbind(0))
        if self._backend == 'nccl':            # RCCL: in place, one collective
            tdist.all_gather_into_tensor(self.xchg, parts[self.rank], group=self.group)
        else:                                  # gloo (CPU-staged; tests): list form
            tdist.all_gather(parts, parts[self.rank].clone(), group=self.group)
        self.loss_k[c * self.Bg:(c + 1) * self.Bg].view(self.G, self.B).copy_(
            lay.gathered_losses(self.xchg))

    def _finish(self, c0, n_steps, Bc, stream):
        """Losses of batches c0..c0+n_steps of the slot -> loss_hist; step_idx += n."""
        rc = lib().mirec_chunk_finish(self.loss_k.data_ptr() + 4 * c0 * self.Bg, Bc, self.Bg,
                                      n_steps, float(Bc * self.times),
                                      self.loss_hist.data_ptr(), self.step_idx.data_ptr(),
                                      self.ticket.data_ptr(), stream.cuda_stream)
        check(rc, 'mirec_chunk_finish')

    def _flush(self, stream, rows=None):
        """Deferred schedule: bring every row to step_idx applied steps. rows: rows per
        wave per table (_flush_rows), or None / all ones for one wave per row."""
        if self.adam_mode != 'deferred':
            return
        if rows is not None and any(r > 1 for r in rows):
            rpw = (ctypes.c_int32 * 2)(*rows)

            def flush():
                check(lib().mirec_adam_flush_rows_f32(self._tables, 2, self.d, rpw,
                                                      self.consts.data_ptr(),
                                                      self.step_idx.data_ptr(), 0,
                                                      *self._adam_args, stream.cuda_stream),
                      'mirec_adam_flush_rows_f32')
        else:
            def flush():
                check(lib().mirec_adam_flush_f32(self._tables, 2, self.d, self.consts.data_ptr(),
                                                 self.step_idx.data_ptr(), 0, *self._adam_args,
                                                 stream.cuda_stream), 'mirec_adam_flush_f32')
        self._record('flush', stream, flush)

    def _entry_lists(self, slot):
        """(row list, device count) per table: the rows batch 0 of `slot` reads."""
        return [(slot.u_uniq, slot.u_nu), (slot.i_uniq, slot.i_nu)]

    def _entry(self, slot, stream):
        """Deferred schedule, chunk entered without a flush before it: bring the
        rows its first batch reads through the previous step (a look-ahead launch
        at step step_idx - 1: K5 with no touched rows)."""
        if self.adam_mode != 'deferred':
            return
        t = (AdamTable * 2)()                   # own descriptors: self._tables keeps its rows
        ctypes.memmove(t, self._tables, ctypes.sizeof(t))
        for q, (uniq, n) in enumerate(self._entry_lists(slot)):
            t[q].rows = self.xbuf.data_ptr()            # unused: no touched rows
            t[q].perm = t[q].uniq = t[q].seg = uniq.data_ptr()
            t[q].n_uniq = self.zero_i32.data_ptr()
            t[q].ahead_uniq = uniq.data_ptr()
            t[q].ahead_n_uniq = n.data_ptr()

        def entry():
            check(lib().mirec_adam_deferred_f32(t, 2, self._n_max, self.d, self.consts.data_ptr(),
                                                self.step_idx.data_ptr(), -1, *self._adam_args,
                                                stream.cuda_stream), 'mirec_adam_deferred_f32')
        self._record('ahead', stream, entry)

    def _grad_scale(self, Bc):
        """1 / (rows of the GLOBAL batch): the reference's .mean() over the batch."""
        R = Bc * self.times
        if getattr(self, '_gs_R', None) != R:
            self._gs_R = R
            self._gs = float(np.float32(1.0) / np.float32(R))
        return self._gs

    def _graph_for(self, slot, nb, entry, flush):
        """HIP graph of the model-side steps of an nb-batch chunk in `slot`, with
        the entry catch-up and / or the closing flush (captured once per (slot, nb,
        entry, flush); capture synchronizes, so begin_epoch captures every variant
        its plan uses before any batch runs)."""
        key = (nb, entry, flush)
        g = slot.graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(device=self.device)
            cap.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.graph(g, stream=cap):
                if entry:
                    self._entry(slot, cap)
                for c in range(nb):
                    self._step(slot, c, self.Bg, cap, c, c + 1 < nb)
                self._finish(0, nb, self.Bg, cap)
                if flush:
                    self._flush(cap, flush)
            torch.cuda.current_stream(self.device).wait_stream(cap)
            slot.graphs[key] = g
        return g

    def _capture_variants(self):
        """Capture the model-side graph of every (slot, size, entry, flush) variant the
        epoch's chunk plan uses."""
        S = len(self.slots)
        # flush flags are False, True or a tuple of row counts: sort by their repr
        variants = sorted({(k % S, n, e, f) for k, ((_, n, Bc), (e, f)) in
                           enumerate(zip(self._plan, self._flags)) if Bc == self.Bg},
                          key=lambda v: (v[0], v[1], v[2], repr(v[3])))
        for k, n, e, f in variants:
            self._graph_for(self.slots[k], n, e, f)

    # ------------------------------------------------------------------ epoch API
    def begin_epoch(self, cuts=(), hold_prep_from=None, flush_at=()):
        """Shuffle (reference order of RNG use), stage the epoch's Adam constants,
        and start preparing the first chunks; returns the number of (global) batches.

        cuts: batch indices at which a chunk must start (bench.py cuts at the
        warm-up / timed / measurement boundaries). flush_at: batch indices (chunk
        ends) where the deferred schedule also completes every row. hold_prep_from: batch index
        whose chunk (and every later one) is not prepared until release_prep() —
        so a timed region that starts there contains its own chunks' sampler walk
        and grouping."""
        data = self.data
        if data.shuffle:
            data._shuffle()                     # randperm (CPU RNG) + device reorder
        inter = data.dataset.inter_feat
        self._users = inter[self.uid_field]
        self._items = inter[self.iid_field]
        if not self._users.is_cuda:
            raise RuntimeError('fused train step needs the train table on the GPU')
        self.n_batches = nb = math.ceil(self._users.numel() / self.Bg)
        table = self.opt.step_constants(self.opt.n_steps + 1, max(nb, 1)).reshape(-1)
        if self.consts.numel() < table.size:   # persistent buffers (graph-captured pointers)
            self.consts = torch.zeros(table.size, dtype=torch.float32, device=self.device)
            self.loss_hist = torch.zeros(max(nb, 1), dtype=torch.float32, device=self.device)
            for s in self.slots:
                s.graphs = {}
        ptrs = [(t.p, t.m, t.v) for t in self._tables]
        self._fill_tables()                    # optimizer state may have been reloaded
        if ptrs != [(t.p, t.m, t.v) for t in self._tables]:
            for s in self.slots:
                s.graphs = {}
        self.consts[:table.size].copy_(torch.from_numpy(table))
        self.loss_hist.zero_()
        self.step_idx.zero_()
        self._busy0 = [t.n_rows for t in self._tables]   # rows that may lag (flush rows per wave)
        self._batches_enqueued = 0
        if self.adam_mode == 'deferred':       # rows are all flushed: epoch-relative counts
            busy = []
            for m, v, last in self._adam_state():   # zero-state rows: marked (adam.hip)
                ops.zero_state_marks(m, v, last, self._adam_args[3])
                busy.append((last != ops.ADAM_ZERO_STATE).sum())
            # one host read per epoch (outside any timed step)
            self._busy0 = [int(x) for x in torch.stack(busy).cpu()]
        if self.fused_step:                    # parity buffers: state 0 (and every
            self.pU_alt.copy_(self.pU.data)    # zero-state row) valid in both
            self.pI_alt.copy_(self.pI.data)
        ramps = (0,) if hold_prep_from is None else (0, int(hold_prep_from))
        self._plan, self._plan_starts = self._chunks(cuts, ramps), None
        self._flush_at = set(int(b) for b in flush_at)
        self._flags = self._chunk_flags(self._plan)
        if self.use_graph:                      # capture up front: capture synchronizes
            self._capture_variants()
        self.prep_stream.wait_stream(torch.cuda.current_stream(self.device))
        self._last_walked = None               # event after the latest issued walk
        self._deferred_waits, self._urgent, self._late_top_up = [], False, None
        self._next_chunk = 0                   # chunks whose walk (or whole prep) is issued
        self._next_group = 0                   # chunks whose grouping is issued
        self._prep_limit = (len(self._plan) if hold_prep_from is None
                            else self._chunk_of(hold_prep_from))
        self._cur = None                       # chunk index being consumed
        for s in self.slots:
            s.free_recorded = False
            if not self._sharded(self.Bg):     # the native preparation's descriptors now,
                self._chunk_prep(s)            # not on a timed region's first launch
        for _ in range(len(self.slots)):
            self._issue_prep()
        self._issue_groups(len(self.slots))
        return nb

    def release_prep(self, upto=None):
        """Let the chunks held by begin_epoch(hold_prep_from=...) be prepared; the
        first one's walk is issued at once (the rest as run_batches reaches them).
        upto: prepare only the chunks
        that start before global batch `upto` (a later call releases the rest), so a
        timed region does not also run the sampler walk of the batches after it."""
        self._prep_limit = (len(self._plan) if upto is None
                            else self._chunk_of(max(int(upto) - 1, 0)) + 1)
        if self._next_chunk < min(len(self._plan), self._prep_limit):
            k = self._next_chunk               # the first released walk starts right away:
            if self.MAIN_FIRST and not self._sharded(self._plan[k][2]):
                # the whole preparation on the model's stream (no cross-queue hand-off
                # before the first step); the next chunks' walks after its model launch
                self._issue_prep(on=torch.cuda.current_stream(self.device))
                self._late_top_up = k
            else:
                self._issue_prep()

    def _issue_prep(self, on=None):
        k = self._next_chunk
        if k >= min(len(self._plan), self._prep_limit):
            return
        slot = self.slots[k % len(self.slots)]
        slot.group_pending = False
        self._prepare(slot, self._plan[k], on)
        self._next_chunk += 1

    def _issue_groups(self, upto):
        """Issue the grouping halves of the walked chunks below `upto`."""
        while self._next_group < min(self._next_chunk, upto):
            slot = self.slots[self._next_group % len(self.slots)]
            if slot.group_pending:
                self._prepare_group(slot)
            self._next_group += 1

    def _enter_chunk(self, k, stream):
        if self._cur == k:
            return
        S = len(self.slots)
        if self._cur is not None:              # previous chunk fully enqueued
            prev = self.slots[self._cur % S]
            prev.free.record(stream)
            prev.free_recorded = True
        if (self.MAIN_FIRST and self._next_chunk == k and k < min(len(self._plan), self._prep_limit)
                and not self._sharded(self._plan[k][2])):
            self._issue_prep(on=stream)        # pipeline (re)start: prepared on this stream
            self._late_top_up = k
        while self._next_chunk <= k and self._next_chunk < min(len(self._plan),
                                                               self._prep_limit):
            self._issue_prep()
        if self._next_chunk <= k:
            raise RuntimeError(f'chunk {k} is held (begin_epoch(hold_prep_from=...)): '
                               'call release_prep() first')
        # this chunk's grouping first (its stream waits for the walk on the GPU; issued
        # later, the host's enqueue of the next walks would delay it), then the walks of
        # the next chunks (the same walk stream: they start as this chunk's walk ends) —
        # unless this chunk was prepared on the model's stream: then they follow its model
        # launch (run_batches), which the GPU reaches first
        self._issue_groups(k + 1)
        slot = self.slots[k % S]
        if self._late_top_up != k:
            self._top_up_prep(k)
        if not getattr(slot, 'ready_on_model', False):
            stream.wait_event(slot.ready)
        self._cur = k

    def run_batches(self, b_start, b_end):
        """Enqueue global batches [b_start, b_end) in order (no host sync). Whole
        chunks replay their captured graph; a chunk entered mid-way (or timed with
        per-kernel events) launches eagerly, one step and one loss bookkeeping launch
        at a time. A chunk starts with the entry catch-up and ends with the flush
        when its plan flags say so (_chunk_flags)."""
        stream = torch.cuda.current_stream(self.device)
        b = b_start
        while b < b_end:
            k = self._chunk_of(b)
            b0, nb, Bc = self._plan[k]
            entry, flush = self._flags[k]
            self._enter_chunk(k, stream)
            slot = self.slots[k % len(self.slots)]
            c0, c1 = b - b0, min(nb, b_end - b0)
            key = (nb, entry, flush)
            if (self.use_graph and c0 == 0 and c1 == nb and Bc == self.Bg
                    and self.kernel_events is None and key in slot.graphs):
                slot.graphs[key].replay()
                self._current = flush
            else:
                self.n_eager_steps += c1 - c0
                if c0 == 0 and entry:
                    self._entry(slot, stream)
                for c in range(c0, c1):
                    self._step(slot, c, Bc, stream, 0, c + 1 < nb)
                    self._finish(c, 1, Bc, stream)
                self._current = False
                if c1 == nb and flush:
                    self._flush(stream, flush)
                    self._current = True
            if self._late_top_up == k:         # after a restart chunk's launch: the next
                self._late_top_up = None       # walks, the first one grouped at once
                self._urgent = True
                self._top_up_prep(k)
                self._urgent = False
            self._issue_groups(k + len(self.slots))   # later chunks' groupings, behind
            b = b0 + c1
            self._batches_enqueued = b

    def _top_up_prep(self, k):
        """Prepare chunks up to k + SLOTS - 1 (their slots are free once the chunks
        before them have run)."""
        lim = min(len(self._plan), self._prep_limit, k + len(self.slots))
        while self._next_chunk < lim:
            self._issue_prep()

    def launch_batch(self, b):
        self.run_batches(b, b + 1)

    def _chunk_of(self, b):
        """Index of the plan chunk holding global batch b."""
        starts = self._plan_starts
        if starts is None or len(starts) != len(self._plan):
            starts = self._plan_starts = np.array([c[0] for c in self._plan], dtype=np.int64)
        return max(int(np.searchsorted(starts, b, side='right')) - 1, 0)

    def sync_params(self):
        """Make the parameters current (deferred schedule: flush every row, unless
        the last enqueued work was a chunk's closing flush)."""
        if not self._current:
            self._flush(torch.cuda.current_stream(self.device),
                        self._flush_rows(self._batches_enqueued))
            self._current = True

    def end_epoch(self, n_done=None):
        """Complete the parameters, account the optimizer steps and read the
        per-batch losses back (one sync)."""
        n_done = self.n_batches if n_done is None else n_done
        stream = torch.cuda.current_stream(self.device)
        stream.wait_stream(self.prep_stream)
        stream.wait_stream(self.group_stream)
        self.sync_params()
        self.opt.advance(n_done)
        self.data.pr = 0
        self.data.sampler.check_status()
        return [float(x) for x in self.loss_hist[:n_done].cpu().numpy()]

    def run_epoch(self):
        """One epoch; returns the list of per-batch mean losses (host floats)."""
        nb = self.begin_epoch()
        self.run_batches(0, nb)
        return self.end_epoch()

    def close(self):
        """Drop the captured chunk graphs (they hold collectives of the process
        group: release them before torch.distributed.destroy_process_group)."""
        torch.cuda.synchronize(self.device)
        for s in self.slots:
            s.graphs = {}
        torch.cuda.synchronize(self.device)


class ShardedBPRTrainStep(FusedBPRTrainStep):
    """The fused pairwise step with ROW-SHARDED tables over G ranks:
    rank r owns rows id % G == r of both tables (parameters, Adam m / v and the
    deferred step counts) as a [S, d] shard, S = ceil(n / G).

    Per optimizer step over a global batch of G*B positives (csrc/shard.hip):
      prep (replicated on every rank, prep stream): walk + K2 grouping of the global
        batch over owner-major keys, the exchange plans and this rank's slice of the
        grouping (mirec_shard_plan / mirec_shard_own);
      forward exchange: each owner gathers the rows every slice needs from its shards
        (mirec_shard_gather_f32) and one all-to-all (RCCL over xGMI; equal blocks of
        `cap` rows per rank pair) delivers them;
      K3 on this rank's slice of positives, reading rows from the receive buffer;
      backward exchange: the slice's per-slot gradient rows go back to the owners
        in the same message positions (second all-to-all);
      K5 (deferred) on the owned rows only, summing each row's contributions in the
        global grouping order — the result is bit-identical to one GPU running the
        global batch;
      per chunk: one all-gather of the per-positive losses for the loss history.
    The dominant optimizer work (touched rows + flush) is 1/G per rank. The model's
    full parameter tensors are written back from the shards at end_epoch() (one
    all-gather of p, m, v per epoch) for evaluation and checkpoints, and re-read
    into the shards at begin_epoch(). With dist=None it runs the same protocol on
    one rank (G = 1; the all-to-alls are copies)."""

    CAP_SLACK = 1.25
    # the per-step row exchanges: 'rccl' (two all-to-alls of equal blocks) or 'ipc' (the
    # owners' gather stores into the readers' IPC-mapped windows, K3 stores the gradient
    # rows into the owners' windows, flags on the GPU: csrc/comm.hip, trainer/comm.py)
    EXCHANGE = os.environ.get('MIREC_EXCHANGE', 'rccl')

    def __init__(self, model, optimizer, train_data, chunk=None, use_graph=True,
                 adam_mode='deferred', dist=None, cap=None, exchange=None):
        if adam_mode != 'deferred':
            raise ValueError('the row-sharded step runs the deferred Adam schedule')
        exchange = exchange or self.EXCHANGE
        if exchange not in ('rccl', 'ipc'):
            raise ValueError(f"exchange must be 'rccl' or 'ipc', got {exchange!r}")
        super().__init__(model, optimizer, train_data, chunk=chunk, use_graph=use_graph,
                         adam_mode=adam_mode, dist=dist, fused_step=False)
        G, B, T, d, dev = self.G, self.B, self.times, self.d, self.device
        self.SU, self.SI = -(-self.nU // G), -(-self.nI // G)
        # rows per (slice, owner) message: the slice's (2+T)*B slots spread over G
        # owners (cyclic ownership); a chunk whose plan overflows is re-planned with a
        # larger cap before it runs (_enter_chunk), never run on a truncated plan
        self.cap = int(cap or min((2 + T) * B,
                                  math.ceil(self.CAP_SLACK * (2 + T) * B / G) + 64))
        self.shU = [torch.zeros(self.SU, d, device=dev) for _ in range(3)]   # p, m, v
        self.shI = [torch.zeros(self.SI, d, device=dev) for _ in range(3)]
        self.lastU = torch.zeros(self.SU, dtype=torch.int32, device=dev)
        self.lastI = torch.zeros(self.SI, dtype=torch.int32, device=dev)
        self._solo = dist is None            # one rank, no process group: no collectives
        self.exchange = 'rccl' if self._solo else exchange
        self.win = None
        if self.exchange == 'ipc':           # every rank's receive window, mapped everywhere
            from recbole_amd.trainer.comm import PeerWindows
            self.win = PeerWindows(dist, (2 + T) * B, d, dev)
        self.loss_g = torch.empty(G * self.C * B, dtype=torch.float32, device=dev)
        self.loss_mine = torch.zeros(self.C * B, dtype=torch.float32, device=dev)
        self.status = torch.zeros(2, dtype=torch.int32, device=dev)    # epoch backstop
        self.cap_growths = 0
        Bg, KI = self.Bg, (1 + T) * self.Bg
        C = self.C
        for sl in self.slots:
            sl.u_keyed = torch.empty(C * Bg, dtype=torch.int64, device=dev)
            sl.i_keyed = torch.empty(C * KI, dtype=torch.int64, device=dev)
            sl.map2 = torch.empty(C * (Bg + KI), dtype=torch.int32, device=dev)
            sl.pos = torch.empty(C * (2 + T) * B, dtype=torch.int64, device=dev)
            # this chunk's plan status ([overflow, largest message]), read by the host
            # before the chunk's model side is launched (_enter_chunk)
            sl.plan_status = torch.zeros(4, dtype=torch.int32, device=dev)
            sl.plan_status_host = torch.zeros(4, dtype=torch.int32).pin_memory()
            sl.planned = torch.cuda.Event()
            for tag, per in (('u', Bg), ('i', KI)):
                setattr(sl, f'own_{tag}', torch.empty(C * per, dtype=torch.int32, device=dev))
                setattr(sl, f'own_{tag}_seg', torch.empty(C * (per + 1), dtype=torch.int32,
                                                          device=dev))
                setattr(sl, f'own_{tag}_n', torch.zeros(C, dtype=torch.int32, device=dev))
                setattr(sl, f'perm2_{tag}', torch.empty(C * per, dtype=torch.int32, device=dev))
                setattr(sl, f'own_{tag}_ah', torch.empty(C * per, dtype=torch.int32, device=dev))
                setattr(sl, f'own_{tag}_nah', torch.zeros(C, dtype=torch.int32, device=dev))
                setattr(sl, f'sel_{tag}', torch.empty(C * per, dtype=torch.int32, device=dev))
                if self.win is not None:     # the owner's push lists (mirec_shard_next)
                    setattr(sl, f'next_{tag}_t', torch.empty(C * per, dtype=torch.int32,
                                                             device=dev))
                    setattr(sl, f'next_{tag}_a', torch.empty(C * per, dtype=torch.int32,
                                                             device=dev))
        # slots per (batch, table) a rank's owner-filtered grouping holds (its ~1/G share
        # of the global batch with slack; a batch over it is re-selected at the table's
        # full size before its chunk runs: _enter_chunk)
        self.cap_sel = {tag: min(per, math.ceil(self.CAP_SLACK * per / G) + 64)
                        for tag, per in (('u', Bg), ('i', KI))}
        self.sel_growths = 0
        self._alloc_exchange()
        self._n_max = (ctypes.c_int64 * 2)(min(Bg, self.SU), min(KI, self.SI))
        self._fill_tables()

    def _alloc_exchange(self):
        """Buffers sized by `cap`: the two all-to-all send / receive buffers (rccl; the
        ipc exchange receives in the windows, sized for the largest cap) and the per-slot
        message plans."""
        M, d, dev = self.G * self.cap, self.d, self.device
        if self.win is None:
            self.sendF = torch.empty(M, d, device=dev)
            self.recvF = self.sendF if self._solo else torch.empty(M, d, device=dev)
            self.sendB = torch.empty(M, d, device=dev)
            self.recvB = self.sendB if self._solo else torch.empty(M, d, device=dev)
        for sl in self.slots:
            sl.fwd_rows = torch.empty(self.C * M, dtype=torch.int64, device=dev)
            sl.bwd_src = torch.empty(self.C * M, dtype=torch.int32, device=dev)

    # ------------------------------------------------------------ shards <-> full tensors
    def _owned_ids(self, n, S):
        ids = torch.arange(S, device=self.device, dtype=torch.int64) * self.G + self.rank
        return ids[ids < n]

    def _load_shards(self):
        """Owned rows of the model's full p and the optimizer's m, v -> the shards."""
        full = [(self.pU, self.opt.state[self.pU]), (self.pI, self.opt.state[self.pI])]
        for (p, st), sh, n, S in zip(full, (self.shU, self.shI), (self.nU, self.nI),
                                     (self.SU, self.SI)):
            ids = self._owned_ids(n, S)
            for dst, src in zip(sh, (p.data, st['exp_avg'], st['exp_avg_sq'])):
                dst[:ids.numel()].copy_(src[ids])

    def _store_shards(self):
        """All shards -> the full p, m, v on every rank (one all-gather each)."""
        full = [(self.pU, self.opt.state[self.pU]), (self.pI, self.opt.state[self.pI])]
        for (p, st), sh, n, S in zip(full, (self.shU, self.shI), (self.nU, self.nI),
                                     (self.SU, self.SI)):
            for src, dst in zip(sh, (p.data, st['exp_avg'], st['exp_avg_sq'])):
                g = self._all_gather(src)                       # [G*S, d], owner-major
                dst.copy_(g.view(self.G, S, self.d).transpose(0, 1).reshape(-1, self.d)[:n])

    def _all_gather(self, x):
        if self.group is None:
            return x
        import torch.distributed as tdist
        out = torch.empty((self.G,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        if self._backend == 'nccl':
            tdist.all_gather_into_tensor(out, x.contiguous(), group=self.group)
        else:
            parts = list(out.unbind(0))
            tdist.all_gather(parts, x.contiguous(), group=self.group)
        return out.view((-1,) + tuple(x.shape[1:]))

    def _all_to_all(self, recv, send):
        if self.group is None:
            return                                              # recv is send
        import torch.distributed as tdist
        if self._backend == 'nccl':
            tdist.all_to_all_single(recv, send, group=self.group)
        else:                                                   # gloo: host-staged
            r = torch.empty(recv.shape, dtype=recv.dtype)
            tdist.all_to_all_single(r, send.cpu(), group=self.group)
            recv.copy_(r)

    # ------------------------------------------------------------ data side
    def _prepare(self, slot, chunk, on=None):     # on: the base class's diagnostic (unused)
        b0, nb, Bc = chunk
        T, G, r = self.times, self.G, self.rank
        KI = (1 + T) * Bc
        L = lib()
        if slot.free_recorded:
            self.prep_stream.wait_event(slot.free)
        with torch.cuda.stream(self.prep_stream):
            st = self.prep_stream.cuda_stream
            s0 = b0 * self.Bg
            users = slot.user_keys[:nb * Bc]
            users.copy_(self._users[s0:s0 + nb * Bc])
            keys = slot.item_keys[:nb * KI].view(nb, 1 + T, Bc)
            keys[:, 0, :].copy_(self._items[s0:s0 + nb * Bc].view(nb, Bc))
            neg = slot.item_keys[Bc:nb * KI]
            self.data.sampler.launch_batches(users, Bc, nb, T, neg, out_stride=KI,
                                             ws=self.samp_ws)
            self._plan_chunk(slot, chunk, st)
            slot.ready.record(self.prep_stream)
        slot.chunk = chunk

    def _plan_chunk(self, slot, chunk, st):
        """This rank's grouping of a walked chunk and its exchange plans (on the current
        stream, `st`): per table, the slots of the rows this rank owns (mirec_shard_select,
        ~1/G of the global batch), their K2 grouping over owner-major keys and look-ahead
        lists; the plans from the unsorted keys (mirec_shard_plan); the owned lists with the
        contributions' places in the backward messages (mirec_shard_own_sel). The plan
        status goes to pinned host memory."""
        _, nb, Bc = chunk
        T, G, r = self.times, self.G, self.rank
        KI = (1 + T) * Bc
        L = lib()
        users = slot.user_keys[:nb * Bc]
        items = slot.item_keys[:nb * KI]
        slot.plan_status.zero_()
        cs = {}
        for k, (tag, ids, per, S) in enumerate((('u', users, Bc, self.SU),
                                                ('i', items, KI, self.SI))):
            cs[tag] = c_ = min(self.cap_sel[tag], per)
            keyed = getattr(slot, f'{tag}_keyed')[:nb * c_]
            check(L.mirec_shard_select(ids.data_ptr(), nb, per, G, S, r, c_, keyed.data_ptr(),
                                       getattr(slot, f'sel_{tag}').data_ptr(),
                                       slot.plan_status.data_ptr() + 4 * (2 + k), st),
                  'mirec_shard_select')
            g_ = lambda n: getattr(slot, f'{tag}_{n}')
            self.sort_ws = ops.segment_sort_batched(keyed, c_, G * S + 1, g_('perm'), g_('uniq'),
                                                    g_('seg'), g_('nu'), ws=self.sort_ws)
            ops.uniq_ahead_diff(g_('uniq'), g_('nu'), c_, nb, g_('ahead'), g_('nah'))
        check(L.mirec_shard_plan(users.data_ptr(), items.data_ptr(), nb, Bc, self.B, T, G, r,
                                 self.cap, slot.fwd_rows.data_ptr(), slot.map2.data_ptr(),
                                 slot.pos.data_ptr(), slot.bwd_src.data_ptr(),
                                 slot.plan_status.data_ptr(), st), 'mirec_shard_plan')
        for tag, per, off, S in (('u', Bc, 0, self.SU), ('i', KI, Bc, self.SI)):
            g_ = lambda n: getattr(slot, n).data_ptr()
            check(L.mirec_shard_own_sel(g_(f'{tag}_uniq'), g_(f'{tag}_seg'), g_(f'{tag}_nu'),
                                        g_(f'{tag}_perm'), cs[tag], nb, g_(f'{tag}_ahead'),
                                        g_(f'{tag}_nah'), slot.map2.data_ptr(), Bc + KI, off,
                                        S, r, g_(f'sel_{tag}'), per, g_(f'own_{tag}'),
                                        g_(f'own_{tag}_seg'), g_(f'own_{tag}_n'),
                                        g_(f'perm2_{tag}'), g_(f'own_{tag}_ah'),
                                        g_(f'own_{tag}_nah'), st), 'mirec_shard_own_sel')
            if self.win is not None:
                check(L.mirec_shard_next(g_(f'own_{tag}'), g_(f'own_{tag}_n'),
                                         g_(f'own_{tag}_ah'), g_(f'own_{tag}_nah'), per, nb,
                                         g_(f'next_{tag}_t'), g_(f'next_{tag}_a'), st),
                      'mirec_shard_next')
        # epoch backstop: overflow flag (min: -4 < 0) and the largest message (max)
        torch.minimum(self.status[:1], slot.plan_status[:1], out=self.status[:1])
        torch.maximum(self.status[1:], slot.plan_status[1:2], out=self.status[1:])
        slot.plan_status_host.copy_(slot.plan_status, non_blocking=True)
        slot.planned.record(torch.cuda.current_stream(self.device))

    def _enter_chunk(self, k, stream):
        """Before chunk k's model side is enqueued: its plan must fit `cap`. Every rank
        counts every message, so all ranks see the same status and grow `cap` to the
        same value (no collective); the chunk and the prepared ones after it are
        re-planned. No step ever runs on an overflowed plan."""
        new = self._cur != k
        super()._enter_chunk(k, stream)
        if not new:
            return
        slot = self.slots[k % len(self.slots)]
        if not slot.planned.query():          # the plan status reaches pinned memory
            slot.planned.synchronize()
        over, most, sel_u, sel_i = (int(x) for x in slot.plan_status_host)
        _, _, Bc = self._plan[k]
        grow = {tag: n for tag, n, per in (('u', sel_u, Bc), ('i', sel_i, (1 + self.times) * Bc))
                if n > min(self.cap_sel[tag], per)}
        if grow:
            self._grow_sel(grow)
            over, most = (int(x) for x in slot.plan_status_host[:2])
        if over == -4:
            self._grow_cap(most)

    def _grow_sel(self, grow):
        """A batch owns more slots of a table than its owner-filtered grouping holds:
        re-select + re-plan every prepared chunk with that table's full batch size (no
        overflow possible). The graphs stay (they read the owned lists, whose strides do
        not change)."""
        T, Bg = self.times, self.Bg
        logging.getLogger().warning(f'owner-filtered grouping: {grow} owned slots exceed '
                                    f'cap_sel={self.cap_sel}; re-selecting at full size')
        torch.cuda.synchronize(self.device)
        for tag in grow:
            self.cap_sel[tag] = Bg if tag == 'u' else (1 + T) * Bg
        self.sel_growths += 1
        for q in range(self._cur if self._cur is not None else 0, self._next_chunk):
            slot = self.slots[q % len(self.slots)]
            with torch.cuda.stream(self.prep_stream):
                self._plan_chunk(slot, self._plan[q], self.prep_stream.cuda_stream)
        torch.cuda.synchronize(self.device)

    def _grow_cap(self, most):
        """Larger messages: reallocate the cap-sized buffers, re-plan every prepared
        chunk from its walked keys and recapture the chunk graphs."""
        T, B = self.times, self.B
        new_cap = min((2 + T) * B, max(most, math.ceil(self.CAP_SLACK * self.cap)))
        logger = logging.getLogger()
        logger.warning(f'row exchange: a (slice, owner) message of {most} rows exceeds '
                       f'cap={self.cap}; re-planning with cap={new_cap}')
        torch.cuda.synchronize(self.device)
        self.cap = new_cap
        self.cap_growths += 1
        self._alloc_exchange()
        self._fill_tables()
        self.status.zero_()
        for q in range(self._cur, self._next_chunk):           # prepared chunks, in order
            slot = self.slots[q % len(self.slots)]
            with torch.cuda.stream(self.prep_stream):
                self._plan_chunk(slot, self._plan[q], self.prep_stream.cuda_stream)
        torch.cuda.synchronize(self.device)
        if int(self.slots[self._cur % len(self.slots)].plan_status_host[0]) == -4:
            raise RuntimeError('row exchange plan still overflows after re-planning')
        for slot in self.slots:                                 # later chunks: checked on entry
            slot.graphs = {}
        if self.use_graph:
            self._capture_variants()

    # ------------------------------------------------------------ model side
    def _fill_tables(self):
        if not hasattr(self, 'shU'):
            return super()._fill_tables()
        t = self._tables
        for q, (sh, last, S) in enumerate(((self.shU, self.lastU, self.SU),
                                           (self.shI, self.lastI, self.SI))):
            t[q].p, t[q].m, t[q].v = (x.data_ptr() for x in sh)
            t[q].n_rows = S
            t[q].last = last.data_ptr()
            t[q].dense_grad = None
            t[q].rows = self.win.bwd if self.win is not None else self.recvB.data_ptr()

    def _adam_state(self):
        return [(self.shU[1], self.shU[2], self.lastU), (self.shI[1], self.shI[2], self.lastI)]

    def _entry_lists(self, slot):
        return [(slot.own_u, slot.own_u_n), (slot.own_i, slot.own_i_n)]

    def _n_local(self, Bc):
        return max(0, min(self.B, Bc - self.rank * self.B))

    def _step_ipc(self, slot, c, Bc, stream):
        """The forward half of a step through the peer windows (csrc/comm.hip). The chunk's
        first step pushes its rows with a gather launch (after the entry catch-up); later
        steps' rows were pushed by the step before's optimizer launch (_adam_ipc). K3's
        blocks wait for the owners' flags on the GPU (no separate wait launch), read the
        rows in the window and store each gradient row into its owner's window."""
        T, B = self.times, self.B
        L = lib()
        st = stream.cuda_stream
        n = self._n_local(Bc)
        w = self.win.comm
        if c == 0:
            def push():
                check(L.mirec_comm_push_rows_f32(w, self.shU[0].data_ptr(),
                                                 self.shI[0].data_ptr(), slot.fwd_rows.data_ptr(),
                                                 self.cap, st), 'mirec_comm_push_rows_f32')
            self._record('gather', stream, push)
        loss_p = self.loss_mine.data_ptr() + 4 * c * B
        pos_p = slot.pos.data_ptr() + 8 * c * (2 + T) * B

        def bpr():                      # every rank launches it: its last block raises the flags
            check(L.mirec_comm_bpr_f32(w, pos_p, pos_p + 8 * n, pos_p + 16 * n, n, T, 1e-10,
                                       self._grad_scale(Bc), loss_p, self.cap, st),
                  'mirec_comm_bpr_f32')
        self._record('bpr', stream, bpr)

    def _adam_ipc(self, slot, c, Bc, stream, step_off, ahead):
        """The owner's deferred Adam with the backward wait and, unless c is the chunk's
        last step, the next step's forward push folded in (mirec_comm_adam_deferred_f32):
        every row step c+1 reads is in this launch's touched or look-ahead list, and goes
        from registers to its readers' windows right after its update."""
        KI = (1 + self.times) * Bc
        t = self._tables
        nxt = seg = dst = None
        if ahead:
            g_ = lambda n, off: getattr(slot, n).data_ptr() + 4 * off
            nxt = (ctypes.c_void_p * 4)(g_('next_u_t', c * Bc), g_('next_u_a', c * Bc),
                                        g_('next_i_t', c * KI), g_('next_i_a', c * KI))
            seg = (ctypes.c_void_p * 2)(g_('own_u_seg', (c + 1) * (Bc + 1)),
                                        g_('own_i_seg', (c + 1) * (KI + 1)))
            dst = (ctypes.c_void_p * 2)(g_('perm2_u', (c + 1) * Bc), g_('perm2_i', (c + 1) * KI))
        st = stream.cuda_stream

        def adam():
            check(lib().mirec_comm_adam_deferred_f32(
                self.win.comm, t, 2, self._n_max, self.d, self.consts.data_ptr(),
                self.step_idx.data_ptr(), step_off, *self._adam_args, nxt, seg, dst, self.cap, st),
                'mirec_comm_adam_deferred_f32')
        self._record('adam', stream, adam)

    def _step(self, slot, c, Bc, stream, step_off, ahead):
        T, d, G, B, M = self.times, self.d, self.G, self.B, self.G * self.cap
        KI = (1 + T) * Bc
        L = lib()
        st = stream.cuda_stream
        n = self._n_local(Bc)
        if self.win is not None:
            self._step_ipc(slot, c, Bc, stream)
        else:
            self._step_rccl(slot, c, Bc, stream)
        t = self._tables
        for q, (tag, per) in enumerate((('u', Bc), ('i', KI))):
            t[q].perm = getattr(slot, f'perm2_{tag}').data_ptr() + 4 * c * per
            t[q].uniq = getattr(slot, f'own_{tag}').data_ptr() + 4 * c * per
            t[q].seg = getattr(slot, f'own_{tag}_seg').data_ptr() + 4 * c * (per + 1)
            t[q].n_uniq = getattr(slot, f'own_{tag}_n').data_ptr() + 4 * c
            if ahead:
                t[q].ahead_uniq = getattr(slot, f'own_{tag}_ah').data_ptr() + 4 * c * per
                t[q].ahead_n_uniq = getattr(slot, f'own_{tag}_nah').data_ptr() + 4 * c
            else:
                t[q].ahead_uniq = t[q].ahead_n_uniq = None

        if self.win is not None:
            self._adam_ipc(slot, c, Bc, stream, step_off, ahead)
        else:
            def adam():
                check(L.mirec_adam_deferred_f32(t, 2, self._n_max, d, self.consts.data_ptr(),
                                                self.step_idx.data_ptr(), step_off,
                                                *self._adam_args, st), 'mirec_adam_deferred_f32')
            self._record('adam', stream, adam)
        if self.kernel_events is not None:
            self.kernel_uniq.append(torch.stack([slot.own_u_n[c], slot.own_i_n[c]]))

    def _step_rccl(self, slot, c, Bc, stream):
        T, d, G, B, M = self.times, self.d, self.G, self.B, self.G * self.cap
        L = lib()
        st = stream.cuda_stream
        n = self._n_local(Bc)

        def fwd_gather():
            check(L.mirec_shard_gather_f32(self.shU[0].data_ptr(), self.shI[0].data_ptr(), d,
                                           slot.fwd_rows.data_ptr() + 8 * c * M, M,
                                           self.sendF.data_ptr(), st), 'mirec_shard_gather_f32')
        self._record('gather', stream, fwd_gather)
        self._record('exchange', stream, lambda: self._all_to_all(self.recvF, self.sendF))
        loss_p = self.loss_mine.data_ptr() + 4 * c * B
        pos_p = slot.pos.data_ptr() + 8 * c * (2 + T) * B

        def bpr():
            # K3 reading the received rows; each slot's gradient row goes straight into
            # its backward message position (the position its row came in): no separate
            # backward gather (sendB's padding rows are never read by the owners)
            if n == 0:
                return
            check(L.mirec_bpr_fwd_bwd_at_ids_f32(self.recvF.data_ptr(), M, d, pos_p,
                                                 pos_p + 8 * n, pos_p + 16 * n, n, T, 1e-10,
                                                 self._grad_scale(Bc), loss_p,
                                                 self.sendB.data_ptr(), st),
                  'mirec_bpr_fwd_bwd_at_ids_f32')
        self._record('bpr', stream, bpr)
        self._record('exchange_bwd', stream, lambda: self._all_to_all(self.recvB, self.sendB))

    def _finish(self, c0, n_steps, Bc, stream):
        """Losses of this rank's slices of steps c0..c0+n_steps -> all ranks (one
        all-gather), laid out in global positive order, then chunk_finish."""
        B, G = self.B, self.G
        mine = self.loss_mine[c0 * B:(c0 + n_steps) * B]
        gathered = self._all_gather(mine).view(G, n_steps, B)
        self.loss_k.view(self.C, self.Bg)[c0:c0 + n_steps].view(n_steps, G, B).copy_(
            gathered.transpose(0, 1))
        super()._finish(c0, n_steps, Bc, stream)

    # ------------------------------------------------------------ epoch API
    def begin_epoch(self, cuts=(), hold_prep_from=None, flush_at=()):
        self.status.zero_()
        self._load_shards()
        return super().begin_epoch(cuts=cuts, hold_prep_from=hold_prep_from, flush_at=flush_at)

    def close(self):
        super().close()
        if self.win is not None:             # after a barrier: no rank still stores into it
            self.win.close()
            self.win = None

    def end_epoch(self, n_done=None):
        losses = super().end_epoch(n_done)
        if self.win is not None and self.win.status() != 0:
            raise RuntimeError('row exchange: a wait for a peer\'s flags timed out (a rank '
                               'stopped or fell out of step)')
        if int(self.status[0].item()) == -4:                 # backstop: _enter_chunk re-plans
            raise RuntimeError(f'row exchange overflow: a (slice, owner) message exceeded '
                               f'cap={self.cap} rows')
        self._store_shards()
        return losses


def fused_full_sort_eval(model, eval_data, topk_evaluator, user_batch=1 << 20, dp=None,
                         round_users=None):
    """Trainer.evaluate for a FULL loader (trainer.py:355-412) on K6: scores,
    pad/history mask, top-K and positive flags in one kernel per user batch; only
    the [n_users, K] positive matrix returns to the host for the metric
    reduction (evaluators.py:122-141). With a DataParallelStep `dp` every rank ranks
    its contiguous block of users and one all-gather assembles the flags in user
    order (trainer/dist.py) — the metrics of one GPU."""
    dev = model.fused_item_table().device
    K = max(topk_evaluator.topk)
    uids, hist_ptr, hist_cols, pos_ptr, pos_cols = eval_data.device_csr(dev)
    EI = model.fused_item_table().contiguous()
    n = uids.numel()
    lo, hi, blk = dp.user_block(n) if dp is not None else (0, n, n)
    flags = torch.empty(max(hi - lo, 0), K, dtype=torch.uint8, device=dev)
    rnd = round_users or _fullsort_round_users(dev, EI.shape[1])
    if dp is None and n > rnd and user_batch >= n and round_users != 0 and K >= 2:
        return _fullsort_overlapped(model, eval_data, topk_evaluator, uids, hist_ptr, hist_cols,
                                    pos_ptr, pos_cols, EI, K, flags, rnd)
    for s in range(lo, hi, user_batch):
        e = min(hi, s + user_batch)
        Uq = model.fused_user_vectors(uids[s:e]).contiguous()
        o = {'pos_flags': flags[s - lo:e - lo]}
        ops.fullsort_topk(Uq, EI, K, hist_ptr=hist_ptr[s:e + 1], hist_cols=hist_cols,
                          pos_ptr=pos_ptr[s:e + 1], pos_cols=pos_cols, out=o)
    if dp is not None:
        flags = dp.gather_rows(flags, n, blk)
    pos_idx = flags.cpu().numpy().astype(bool)
    return topk_evaluator.evaluate_pos_idx(pos_idx, eval_data.get_pos_len_list())


def _fullsort_round_users(dev, d):
    """Users of one full round of K6 workgroups (128 users each; two resident per
    CU for d <= 128, one for d = 256): launches of this size fill the chip."""
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    return 128 * cus * (2 if d <= 128 else 1)


def _fullsort_overlapped(model, eval_data, topk_evaluator, uids, hist_ptr, hist_cols, pos_ptr,
                         pos_cols, EI, K, flags, chunk):
    """fused_full_sort_eval in round-sized K6 launches: each launch's flags go to the
    host on a copy stream and its metric rows are reduced while the next launches
    run (TopKEvaluator.evaluate_pos_idx_chunks: the same values as one block)."""
    dev = flags.device
    n = uids.numel()
    host = torch.empty(flags.shape, dtype=torch.uint8, pin_memory=True)
    copy_stream = torch.cuda.Stream(device=dev)
    done = []
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        Uq = model.fused_user_vectors(uids[s:e]).contiguous()
        # a launch far below a round (the last one) splits the item range instead,
        # so it does not take a full round's time for a few workgroups
        wgs, full = -(-(e - s) // 128), chunk // 128
        split = min(16, full // wgs) if 2 * wgs <= full else 1
        ops.fullsort_topk(Uq, EI, K, hist_ptr=hist_ptr[s:e + 1], hist_cols=hist_cols,
                          pos_ptr=pos_ptr[s:e + 1], pos_cols=pos_cols,
                          out={'pos_flags': flags[s:e]}, n_split=split)
        ready = torch.cuda.Event()
        ready.record()
        with torch.cuda.stream(copy_stream):
            copy_stream.wait_event(ready)
            host[s:e].copy_(flags[s:e], non_blocking=True)
            copied = torch.cuda.Event()
            copied.record(copy_stream)
        done.append((s, e, copied, Uq))
    pl = np.asarray(eval_data.get_pos_len_list())

    def blocks():
        for s, e, copied, _ in done:
            copied.synchronize()
            yield host[s:e].numpy().astype(bool), pl[s:e]
    out = topk_evaluator.evaluate_pos_idx_chunks(blocks(), n)
    torch.cuda.current_stream(dev).wait_stream(copy_stream)
    return out


def fused_seq_full_sort_eval(model, eval_data, topk_evaluator):
    """Trainer.evaluate for SequentialFullDataLoader (trainer.py:328-353 with
    sequential_dataloader.py:318-345: pad column masked, the target swapped to
    the front, no history mask) on K6: per batch, the sequence representations
    are ranked against every item with the target as the only positive."""
    dev = model.fused_item_table().device
    K = max(topk_evaluator.topk)
    EI = model.fused_item_table().contiguous()
    flags = []
    for interaction, _, _, _, _ in eval_data:
        inter = interaction.to(dev)
        Uq = model.fused_query_vectors(inter).detach().contiguous()
        n = Uq.shape[0]
        pos_ptr = torch.arange(n + 1, dtype=torch.int64, device=dev)
        pos_cols = inter[eval_data.iid_field].to(torch.int32).contiguous()
        o = ops.fullsort_topk(Uq, EI, K, pos_ptr=pos_ptr, pos_cols=pos_cols)
        flags.append(o['pos_flags'])
    pos_idx = torch.cat(flags).cpu().numpy().astype(bool)
    return topk_evaluator.evaluate_pos_idx(pos_idx, eval_data.get_pos_len_list())


def fused_seq_sampled_eval(model, eval_data, topk_evaluator):
    """Trainer.evaluate for SequentialNegSampleDataLoader in evaluation (uni-N, this
    fork's validation, data/utils.py:86-88): the reference repeats every sequence
    1+N times through the whole model (predict on each copy) and ranks the padded
    score rows with topk (trainer.py:384-409, abstract_evaluator.py:65-75). Here each
    sequence is encoded once and K9c counts the sampled items that beat the
    positive; pos_idx[q, r] = (rank[q] == r). The negatives are the ones the
    RepeatableSampler's per-row walk would draw (sample_by_user_ids(uid, N) for row
    after row, no rejection): the next N values of the walk, row by row, taken with
    one device gather; the walk pointer advances by rows x N exactly as it would."""
    from recbole_amd._native import check, lib, ptr, stream_handle
    sampler = eval_data.sampler
    dev = model.fused_item_table().device
    EI = model.fused_item_table().contiguous()
    K = max(topk_evaluator.topk)
    m = eval_data.neg_sample_by
    sampler.to_device(dev)
    L = sampler.random_list_length
    ranks = []
    for start in range(0, eval_data.pr_end, eval_data.step):
        inter = eval_data.augmentation(slice(start, start + eval_data.step)).to(dev)
        uids = inter[eval_data.uid_field]
        n = uids.numel()
        if n == 0:
            continue
        mn, mx = int(uids.min()), int(uids.max())
        if mn < 0 or mx >= sampler.n_users:
            raise ValueError(f'user_id [{mn if mn < 0 else mx}] not exist.')
        idx = (sampler._pr_dev + torch.arange(n * m, device=dev)) % L
        neg = sampler._rl_dev[idx].to(torch.int64)
        sampler._pr_dev.copy_((sampler._pr_dev + n * m) % L)
        S = model.fused_query_vectors(inter).detach().contiguous()
        pos = inter[eval_data.iid_field].to(torch.int64).contiguous()
        rank = torch.empty(n, dtype=torch.int32, device=dev)
        rc = lib().mirec_rank_of_pos_f32(ptr(S), ptr(EI), EI.shape[0], EI.shape[1], ptr(pos),
                                         ptr(neg), n, m, ptr(rank), stream_handle())
        check(rc, 'mirec_rank_of_pos_f32')
        ranks.append(rank)
    rank = torch.cat(ranks) if ranks else torch.zeros(0, dtype=torch.int32, device=dev)
    pos_idx = (rank.unsqueeze(1) == torch.arange(K, device=dev).unsqueeze(0)).cpu().numpy()
    return topk_evaluator.evaluate_pos_idx(pos_idx, eval_data.get_pos_len_list())


def fused_general_sampled_eval(model, eval_data, evaluator):
    """Trainer.evaluate for a GeneralNegSampleDataLoader in evaluation (uni-N /
    pop-N, point-wise, one batch = whole users: this fork's uni1000 validation,
    data/utils.py:86-88) with every batch built on the device.

    The reference builds each batch on the host (general_dataloader.py:210-221):
    per user, slice its rows, sample_by_user_ids(uids, N) (one sampler call per
    user), repeat them 1+N times with the negatives written after the positives
    (_neg_sample_by_point_wise_sampling, :243-251), join every user/item feature
    (unused by the general models' predict), concatenate the users, then
    predict + evaluator.collect (trainer.py:384-409). Here one K4 launch walks the
    batch's per-user calls in order (mirec_sample_walk_segments: the same walk,
    the same values, the pointer advanced exactly as the calls would), the
    [pos | negs] layout is assembled with two device scatters, and the model's
    own predict and the evaluator's collect run on the same layout — so the
    collected matrices are the ones the reference sequence produces on this
    device, without the per-user host loop and the feature joins."""
    sampler = eval_data.sampler
    dev = model.fused_item_table().device
    sampler.to_device(dev)
    ds = eval_data.dataset
    uid_f, iid_f = eval_data.uid_field, eval_data.iid_field
    items_all = ds.inter_feat[iid_f].to(dev)
    N = int(eval_data.neg_sample_by)
    times = eval_data.times
    test_bs = eval_data.config['eval_batch_size']
    out = []
    for start in range(0, eval_data.pr_end, eval_data.step):
        ul = eval_data.uid_list[start:start + eval_data.step]
        n_u = eval_data.uid2items_num[ul].astype(np.int64)
        s_u = eval_data.uid2start[ul].astype(np.int64)
        P = int(n_u.sum())
        if P == 0:
            continue
        seg = np.r_[0, np.cumsum(n_u)]
        # positive rows of the batch's users, user after user (dataset sorted by user)
        rows = np.repeat(s_u - seg[:-1], n_u) + np.arange(P)
        keys = torch.as_tensor(np.repeat(ul, n_u), dtype=torch.int64).to(dev)
        negs = sampler.launch_segments(keys, torch.as_tensor(seg).to(dev), int(n_u.max()), N)
        # block of user b: [its n_b positives | its n_b * N negatives], blocks in order
        blk = np.repeat(seg[:-1] * times, n_u)                  # block start per positive
        within = np.arange(P) - np.repeat(seg[:-1], n_u)        # positive's index in its block
        pos_at = torch.as_tensor(blk + within).to(dev)
        neg_blk = np.repeat(seg[:-1] * times + n_u, n_u * N)    # negatives' region start
        neg_at = torch.as_tensor(neg_blk + np.arange(P * N) - np.repeat(seg[:-1] * N, n_u * N))
        items = torch.empty(P * times, dtype=torch.int64, device=dev)
        items[pos_at] = items_all[torch.as_tensor(rows).to(dev)]
        items[neg_at.to(dev)] = negs
        users = torch.as_tensor(np.repeat(ul, n_u * times), dtype=torch.int64).to(dev)
        from recbole_amd.data.interaction import Interaction
        inter = Interaction({uid_f: users, iid_f: items})
        inter.set_additional_info(list(n_u), list(n_u * times))
        bs = inter.length
        if bs <= test_bs:
            scores = model.predict(inter)
        else:                                   # trainer.py _spilt_predict
            scores = torch.cat([model.predict(Interaction({uid_f: users[i:i + test_bs],
                                                           iid_f: items[i:i + test_bs]}))
                                for i in range(0, bs, test_bs)])
        out.append(evaluator.collect(inter, scores))
    sampler.check_status()
    return evaluator.evaluate(out, eval_data)
