"""oracle/cpu_baseline.py — TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).

Times the reference's training step as the reference runs it on a CPU, from
the oracle's restatement (the reference itself may not be executed here,
SURVEY.md §8c):
  GeneralNegSampleDataLoader batch  — slice of the shuffled train table
  Sampler.sample_by_user_ids        — NumpyWalk: the reference's Python
                                      rejection loop (sampler.py:144-153) over
                                      Python sets of used items
  _neg_sample_by_pair_wise_sampling — Interaction.repeat(times)
  BPR.calculate_loss + backward     — torch CPU nn.Embedding (dense grads)
  optimizer.step                    — torch.optim.Adam over every row
Used-item sets are materialised only for the users the timed batches touch
(membership semantics unchanged; the reference builds them for all users at
setup, which is not part of a step).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from oracle import cpu_ref


class _LazySets(object):
    def __init__(self, ptr, cols):
        self.ptr, self.cols, self.cache = ptr, cols, {}

    def __getitem__(self, k):
        k = int(k)
        s = self.cache.get(k)
        if s is None:
            s = self.cache[k] = set(self.cols[self.ptr[k]:self.ptr[k + 1]].tolist())
        return s


def time_bpr_steps(users, items, used_ptr, used_cols, random_list, n_users, n_items, d, B, T,
                   steps=20, warmup=3, lr=1e-3, threads=None, seed=0):
    """Returns (positives_per_second, seconds_timed, threads_used)."""
    if threads:
        torch.set_num_threads(threads)
    torch.manual_seed(seed)
    model = cpu_ref.BPRCPU(n_users, n_items, d)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    walk = cpu_ref.NumpyWalk(random_list, _LazySets(used_ptr, used_cols))
    users = torch.as_tensor(users)
    items = torch.as_tensor(items)

    def one(b):
        ub, ib = users[b * B:(b + 1) * B], items[b * B:(b + 1) * B]
        neg = torch.as_tensor(walk.sample_by_key_ids(ub.numpy(), T))
        ur, pr_, nr = cpu_ref.pairwise_rows(ub, ib, neg, T)
        opt.zero_grad()
        loss = model.calculate_loss(ur, pr_, nr)
        loss.item()
        loss.backward()
        opt.step()

    for b in range(warmup):
        one(b)
    t0 = time.perf_counter()
    for b in range(warmup, warmup + steps):
        one(b)
    dt = time.perf_counter() - t0
    return steps * B / dt, dt, torch.get_num_threads()
