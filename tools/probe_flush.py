"""The C2 closing flush in isolation (diagnostic): tables of the C2 shape (138,494 users and
26,745 items x d = 128, p / p_alt parity buffers) with the `last` marks a 20-step driver
window leaves — about 10 K users touched since the previous flush (lags 1..20), every item
lagging by a geometric number of steps, the rest of the users in the zero state — flushed
with mirec_adam_flush_rows_f32 at several rows-per-wave settings and with the one-wave-per-row
form. HIP events around each launch; the buffers are restored between launches.

usage: python tools/probe_flush.py [--reps 5] [--target 25]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--target', type=int, default=25)
    ap.add_argument('--users', type=int, default=10000)
    args = ap.parse_args()
    from recbole_amd import ops
    from recbole_amd.trainer.optim import FusedAdam
    dev = torch.device('cuda', 0)
    d, T = 128, args.target
    rng = np.random.default_rng(0)
    opt = FusedAdam([torch.nn.Parameter(torch.zeros(1))], lr=1e-3)
    consts = torch.from_numpy(opt.step_constants(1, 256).reshape(-1)).to(dev)
    base = torch.full((1,), T, dtype=torch.int32, device=dev)
    state = []
    for n, kind in ((138494, 'users'), (26745, 'items')):
        last = np.full(n, ops.ADAM_ZERO_STATE, np.int64)
        if kind == 'users':
            rows = rng.choice(n, args.users, replace=False)
            last[rows] = rng.integers(T - 20, T, args.users)
        else:
            last[:] = np.maximum(T - rng.geometric(0.09, n), T - 25)
        busy = last != ops.ADAM_ZERO_STATE
        P = torch.randn(n, d) * 0.05
        M = torch.zeros(n, d)
        V = torch.zeros(n, d)
        M[busy] = torch.randn(int(busy.sum()), d) * 1e-3
        V[busy] = torch.rand(int(busy.sum()), d) * 1e-6
        state.append([P.to(dev), P.clone().to(dev), M.to(dev), V.to(dev),
                      torch.as_tensor(last.astype(np.int32), device=dev)])
    work = [[x.clone() for x in s] for s in state]
    tabs = ops.adam_tables([dict(p=P, p_alt=A, m=M, v=V, last=L) for P, A, M, V, L in work])
    out = {'lagging_rows': [int((s[4] < T).sum()) for s in state]}

    def restore():
        for w, s in zip(work, state):
            for a, b in zip(w, s):
                a.copy_(b)

    for name, fr in (('one_wave_per_row', None), ('R=1,1', (1, 1)), ('R=8,1', (8, 1)),
                     ('R=8,4', (8, 4)), ('R=8,8', (8, 8)), ('R=16,8', (16, 8)),
                     ('R=32,8', (32, 8)), ('R=32,16', (32, 16)), ('R=64,16', (64, 16))):
        ts = []
        for _ in range(args.reps):
            restore()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            ops.adam_multi(tabs, d, consts, base, 0, 'flush', flush_rows=fr)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        out[name] = round(float(np.median(ts)), 1)
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
