"""Standalone K6 full-sort timing on C2-shaped random data (for profiling)."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recbole_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--users', type=int, default=138493)
ap.add_argument('--items', type=int, default=26745)
ap.add_argument('--d', type=int, default=128)
ap.add_argument('--k', type=int, default=10)
ap.add_argument('--hist', type=int, default=115)
ap.add_argument('--reps', type=int, default=3)
a = ap.parse_args()
dev = torch.device('cuda', 0)
rng = np.random.default_rng(0)
U = torch.randn(a.users, a.d, device=dev) * 0.1
E = torch.randn(a.items, a.d, device=dev) * 0.1
deg = rng.integers(1, 2 * a.hist, a.users)
hp = np.r_[0, np.cumsum(deg)].astype(np.int64)
hc = np.concatenate([np.sort(rng.choice(np.arange(1, a.items), min(k, a.items - 2), replace=False))
                     for k in deg[:2000]] * (a.users // 2000 + 1))[:hp[-1]].astype(np.int32)
pp = np.arange(a.users + 1, dtype=np.int64)
pc = rng.integers(1, a.items, a.users).astype(np.int32)
T = lambda x: torch.as_tensor(x, device=dev)
args = dict(hist_ptr=T(hp), hist_cols=T(hc), pos_ptr=T(pp), pos_cols=T(pc))
ops.fullsort_topk(U, E, a.k, **args)
torch.cuda.synchronize()
for r in range(a.reps):
    t0 = time.perf_counter()
    ops.fullsort_topk(U, E, a.k, **args)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f'fullsort users={a.users} items={a.items} d={a.d}: {dt*1e3:.2f} ms '
          f'{a.users/dt:.0f} users/s {2*a.users*a.items*a.d/dt/1e12:.2f} TFLOP/s')
