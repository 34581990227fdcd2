"""Fused train step and full-sort evaluation for embedding models (BPR-MF).

One training step of Trainer._train_epoch (trainer.py:157-174) for a pairwise
model with learner 'adam', as a fixed sequence of gfx950 kernels on one HIP
stream, with no host synchronisation inside the epoch:

  K4 sampler walk  (sampler.py:103-154)      neg ids for the batch's users
  K3 fused BPR     (bpr.py:74-83)            loss rows + per-row gradients
  K2 segment sort  (embedding backward)      group gradient rows by table row
  K5 dense Adam    (optim.Adam.step)         every row of both tables, compact grads
  step_finish                                per-step mean loss kept on device

The batch is a contiguous slice of the train table resident in HBM, shuffled
once per epoch with torch.randperm on the CPU generator (interaction.py:272-276)
and re-ordered on the device with the K1 gather. Per-batch losses are read
back once per epoch (the reference reads `losses.item()` every batch).
Optionally the steps of an epoch are captured once into a HIP graph and
replayed (config `train_graph`), which removes the per-launch host overhead.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from recbole_amd import ops


class FusedBPRTrainStep(object):
    """Device buffers and launch sequence of the fused pairwise train step."""

    def __init__(self, model, optimizer, train_data):
        self.model = model
        self.opt = optimizer
        self.data = train_data
        (self.pU, self.nU), (self.pI, self.nI) = model.fused_embedding_tables()
        self.device = self.pU.device
        self.B = train_data.step                   # positives per batch
        self.times = train_data.times              # negatives per positive
        self.uid_field = train_data.uid_field
        self.iid_field = train_data.iid_field
        B, T, d = self.B, self.times, self.pU.shape[1]
        dev = self.device
        self.item_keys = torch.empty((1 + T) * B, dtype=torch.int64, device=dev)
        self.bpr_out = {
            'loss_k': torch.empty(B, dtype=torch.float32, device=dev),
            'gU': torch.empty(B, d, dtype=torch.float32, device=dev),
            'gI': torch.empty((1 + T) * B, d, dtype=torch.float32, device=dev),
        }
        self.segU = ops.Segments(B, dev, 4 * 4 * B + 256)
        self.segI = ops.Segments((1 + T) * B, dev, 4 * 4 * (1 + T) * B + 256)
        self.loss_hist = None
        self.kernel_events = None   # list -> HIP events around the K5 launches (bench.py)

    # ------------------------------------------------------------------ one step
    def _launch_step(self, user, pos, consts, step_idx):
        Bb = user.numel()
        T = self.times
        neg = self.item_keys[Bb:(1 + T) * Bb]
        self.item_keys[:Bb].copy_(pos)
        self.data.sampler.launch_batches(user, Bb, 1, T, neg)
        o = {'loss_k': self.bpr_out['loss_k'][:Bb], 'gU': self.bpr_out['gU'][:Bb],
             'gI': self.bpr_out['gI'][:(1 + T) * Bb]}
        ops.bpr_fwd_bwd(self.pU.data, self.pI.data, user, pos, neg, T, grads=True, out=o)
        segU = ops.segment_sort(user, self.nU, self.segU)
        segI = ops.segment_sort(self.item_keys[:(1 + T) * Bb], self.nI, self.segI)
        ev = self.kernel_events
        if ev is not None:
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
        self.opt.step_compact(self.pU, o['gU'], segU, consts, step_idx)
        if ev is not None:
            e[1].record()
        self.opt.step_compact(self.pI, o['gI'], segI, consts, step_idx)
        if ev is not None:
            e[2].record()
            ev.append(e)
        ops.step_finish(o['loss_k'], float(Bb * T), self.loss_hist, step_idx)

    def begin_epoch(self):
        """Shuffle (reference order of RNG use) and stage the epoch's constants;
        returns the number of batches."""
        data = self.data
        if data.shuffle:
            data._shuffle()                     # randperm (CPU RNG) + device reorder
        inter = data.dataset.inter_feat
        self._users = inter[self.uid_field]
        self._items = inter[self.iid_field]
        if not self._users.is_cuda:
            raise RuntimeError('fused train step needs the train table on the GPU')
        self.n_batches = math.ceil(self._users.numel() / self.B)
        self._consts, self._step_idx = self.opt.prepare_window(self.n_batches, self.device)
        self.loss_hist = torch.zeros(max(self.n_batches, 1), dtype=torch.float32,
                                     device=self.device)
        return self.n_batches

    def launch_batch(self, b):
        """Enqueue the kernels of batch b (no host synchronisation)."""
        s = b * self.B
        self._launch_step(self._users[s:s + self.B], self._items[s:s + self.B], self._consts,
                          self._step_idx)

    def end_epoch(self, n_done=None):
        """Account the optimizer steps and read the per-batch losses back (one sync)."""
        n_done = self.n_batches if n_done is None else n_done
        self.opt.advance(n_done)
        self.data.pr = 0
        return [float(x) for x in self.loss_hist[:n_done].cpu().numpy()]

    def run_epoch(self, use_graph=False):
        """One epoch; returns the list of per-batch mean losses (host floats)."""
        nb = self.begin_epoch()
        for b in range(nb):
            self.launch_batch(b)
        return self.end_epoch()


def fused_full_sort_eval(model, eval_data, topk_evaluator, user_batch=4096):
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
