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


def host_threads():
    """Threads for the CPU baseline: the CPUs this process may run on (sched_getaffinity),
    capped by the cgroup CPU quota when one is set (cgroup v2 cpu.max, v1 cfs quota) — the
    host share a job on the GPU box actually gets, not the machine's core count. Returns
    (threads, record) with how the number was derived (written into the bench JSON)."""
    import math
    import os
    aff = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else os.cpu_count()
    quota = None
    for path, parse in (('/sys/fs/cgroup/cpu.max', lambda t: t.split()),
                        ('/sys/fs/cgroup/cpu/cpu.cfs_quota_us', None)):
        try:
            txt = open(path).read().strip()
        except OSError:
            continue
        if parse is not None:
            q, per = parse(txt)
            if q != 'max':
                quota = int(q) / int(per)
        else:
            q = int(txt)
            per = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
            if q > 0:
                quota = q / per
        break
    threads = aff if quota is None else max(1, min(aff, math.floor(quota)))
    return threads, {'sched_getaffinity': aff, 'cgroup_cpu_quota': quota,
                     'os_cpu_count': os.cpu_count(), 'threads': threads,
                     'derivation': 'min(len(sched_getaffinity(0)), floor(cgroup CPU quota))'}


def time_bpr_steps(users, items, used_ptr, used_cols, random_list, n_users, n_items, d, B, T,
                   steps=20, warmup=3, lr=1e-3, threads=None, seed=0, split=None):
    """Returns (positives_per_second, seconds_timed, threads_used). `split` (a dict, if
    given) receives the timed seconds by cost centre: 'pipeline_s' = the
    batch slice + the sampler walk with its Python rejection loop (sampler.py:144-153) +
    the pairwise layout (general_dataloader.py:233-241), 'model_s' = zero_grad +
    calculate_loss + backward + Adam step (trainer.py:160-173)."""
    if threads:
        torch.set_num_threads(threads)
    torch.manual_seed(seed)
    model = cpu_ref.BPRCPU(n_users, n_items, d)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    walk = cpu_ref.NumpyWalk(random_list, _LazySets(used_ptr, used_cols))
    users = torch.as_tensor(users)
    items = torch.as_tensor(items)

    acc = [0.0, 0.0]

    def one(b):
        ta = time.perf_counter()
        ub, ib = users[b * B:(b + 1) * B], items[b * B:(b + 1) * B]
        neg = torch.as_tensor(walk.sample_by_key_ids(ub.numpy(), T))
        ur, pr_, nr = cpu_ref.pairwise_rows(ub, ib, neg, T)
        tb = time.perf_counter()
        opt.zero_grad()
        loss = model.calculate_loss(ur, pr_, nr)
        loss.item()
        loss.backward()
        opt.step()
        acc[0] += tb - ta
        acc[1] += time.perf_counter() - tb

    for b in range(warmup):
        one(b)
    acc[0] = acc[1] = 0.0
    t0 = time.perf_counter()
    for b in range(warmup, warmup + steps):
        one(b)
    dt = time.perf_counter() - t0
    if split is not None:
        split['pipeline_s'], split['model_s'] = acc[0], acc[1]
    return steps * B / dt, dt, torch.get_num_threads()


class _EmptySets(object):
    def __getitem__(self, k):
        return set()


def _cpu_batch(inter):
    return {k: v.cpu() for k, v in inter.interaction.items()}


def time_deepfm_steps(batches, tok, tok_dims, flt, d, hidden, steps=3, warmup=1, lr=1e-3,
                      threads=None, dropout=0.2):
    """C4: DeepFM.calculate_loss + backward + optim.Adam on torch CPU (dense
    gradients of every table, as the reference). Returns (samples/s, s, threads)."""
    if threads:
        torch.set_num_threads(threads)
    model = cpu_ref.DeepFMCPU(tok, tok_dims, [], [], flt, d, hidden, dropout)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    cb = [_cpu_batch(b) for b in batches[:steps + warmup]]   # cycled when fewer

    def one(b):
        opt.zero_grad()
        loss = model.calculate_loss(b, b['label'])
        loss.item()
        loss.backward()
        opt.step()

    for i in range(warmup):
        one(cb[i % len(cb)])
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        one(cb[i % len(cb)])
    dt = time.perf_counter() - t0
    B = len(cb[0]['label'])
    return steps * B / dt, dt, torch.get_num_threads()


def time_sasrec_steps(batches, random_list, n_items, L, d, n_neg, steps=3, warmup=1, lr=1e-3,
                      threads=None):
    """C3: RepeatableSampler walk (numpy restatement, no rejection) + SASRec forward
    + sampled softmax + backward + optim.Adam on torch CPU. Returns (seq/s, s, threads)."""
    if threads:
        torch.set_num_threads(threads)
    model = cpu_ref.SASRecCPU(n_items, L, d, 2, 2, 256, 1e-12)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    walk = cpu_ref.NumpyWalk(random_list, _EmptySets())     # RepeatableSampler: no rejection
    cb = [_cpu_batch(b) for b in batches[:steps + warmup]]   # cycled when fewer

    def one(b):
        neg = torch.as_tensor(walk.sample_by_key_ids(b['user_id'].numpy(), n_neg))
        opt.zero_grad()
        loss = model.calculate_loss(b['item_id_list'], b['item_length'], b['item_id'], neg,
                                    'SSM')
        loss.item()
        loss.backward()
        opt.step()

    for i in range(warmup):
        one(cb[i % len(cb)])
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        one(cb[i % len(cb)])
    dt = time.perf_counter() - t0
    return steps * len(cb[0]['item_id']) / dt, dt, torch.get_num_threads()


def time_full_sort_users(user_e, item_e, n_users, K=10, batch=256, threads=None):
    """C5 scorer as the reference runs it on the CPU (trainer.py:328-353 +
    evaluators.py:53-76): scores = U[u] @ I^T, pad column -inf, topk, for
    n_users users in batches. Returns (users/s, s, threads)."""
    if threads:
        torch.set_num_threads(threads)
    t0 = time.perf_counter()
    for s in range(0, n_users, batch):
        sc = torch.matmul(user_e[s:s + batch], item_e.T)
        sc[:, 0] = -np.inf
        torch.topk(torch.flip(sc, dims=[-1]), K, dim=-1)
    dt = time.perf_counter() - t0
    return n_users / dt, dt, torch.get_num_threads()
