"""K5 probe for PMC passes (GPU): the C2 tables in a steady-training state
(m, v random, non-vanishing updates) or a fresh one (m = v = 0 on most user
rows), then `--reps` launches each of the deferred per-step kernel (one batch's
touched + look-ahead rows lagging `--gap` steps) and the flush of every row
lagging `--gap` steps. HIP-event medians are printed; run under
`rocprofv3 --pmc ...` for the counters.

usage: python tools/probe_adam.py [--gap 64] [--reps 5] [--state steady|fresh]
"""
import argparse
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from recbole_amd import ops  # noqa: E402
from recbole_amd.trainer.optim import FusedAdam  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gap', type=int, default=64)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--state', default='steady', choices=['steady', 'fresh'])
    ap.add_argument('--only', default='both', choices=['both', 'deferred', 'flush'])
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    d, nU, nI, B, KI = 128, 138494, 26745, 512, 2560
    rng = np.random.default_rng(0)
    g = torch.Generator(device='cpu').manual_seed(0)
    P = [(torch.randn(n, d, generator=g) * 0.1).to(dev) for n in (nU, nI)]
    M = [(torch.randn(n, d, generator=g) * 1e-3).to(dev) for n in (nU, nI)]
    V = [(torch.rand(n, d, generator=g) * 1e-6).to(dev) for n in (nU, nI)]
    if args.state == 'fresh':                  # rows never touched: m = v = +0
        M[0][13000:].zero_()
        V[0][13000:].zero_()
    last = [torch.zeros(n, dtype=torch.int32, device=dev) for n in (nU, nI)]
    opt = FusedAdam([torch.nn.Parameter(torch.zeros(4))])
    consts = torch.from_numpy(opt.step_constants(1, 4096).reshape(-1)).to(dev)
    base = torch.zeros(1, dtype=torch.int32, device=dev)
    keys = [torch.as_tensor(rng.integers(0, nU, B), device=dev),
            torch.as_tensor(rng.integers(0, nI, KI), device=dev)]
    segs = [ops.segment_sort(k, n) for k, n in zip(keys, (nU, nI))]
    rows = [torch.randn(k.numel(), d, device=dev) * 1e-2 for k in keys]
    ahead = []
    for q, n in enumerate((nU, nI)):
        nu = int(segs[q].n_uniq.item())
        touched = set(segs[q].uniq[:nu].cpu().tolist())
        cand = rng.choice(n, size=nu * 2, replace=False)
        a = np.array(sorted(x for x in cand if x not in touched)[:nu], np.int32)
        ahead.append((torch.as_tensor(a, device=dev),
                      torch.tensor([len(a)], dtype=torch.int32, device=dev)))
    specs = [dict(p=P[q], m=M[q], v=V[q], rows=rows[q], segs=segs[q], last=last[q],
                  ahead=ahead[q]) for q in range(2)]
    tabs = ops.adam_tables(specs)
    nmax = [B, KI]
    snap = [(p.clone(), m.clone(), v.clone()) for p, m, v in zip(P, M, V)]

    def prep():
        base.fill_(1000)
        for x in last:
            x.fill_(1000 - args.gap)
        for (p, m, v), (p0, m0, v0) in zip(zip(P, M, V), snap):
            p.copy_(p0); m.copy_(m0); v.copy_(v0)

    def timeit(fn):
        ts = []
        for _ in range(args.reps):
            prep()
            torch.cuda._sleep(100000)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return float(np.median(ts))
    if args.only in ('both', 'deferred'):
        t = timeit(lambda: ops.adam_multi(tabs, d, consts, base, 0, 'deferred', n_max_uniq=nmax))
        print(f'deferred gap {args.gap}: {t:.2f} us', flush=True)
    if args.only in ('both', 'flush'):
        f = timeit(lambda: ops.adam_multi(tabs, d, consts, base, 0, 'flush'))
        rows_ = nU + nI
        print(f'flush gap {args.gap}: {f:.2f} us = {rows_ * d * args.gap / f * 1e-6:.3f} '
              f'T element-steps/s', flush=True)


if __name__ == '__main__':
    main()
