"""Micro-benchmark of the K5 schedules on the C2 table shapes (GPU).

Times (HIP events, 50 launches each): streamed dense Adam over both tables; the
deferred kernel for one batch's touched rows (512 users, ~2.5k items, plus as
many look-ahead rows) with every row lagging `gap` steps; and the flush of all
rows lagging `gap` steps.
"""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from recbole_amd import ops  # noqa: E402
from recbole_amd.trainer.optim import FusedAdam  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    d, nU, nI, B, KI = 128, 138494, 26745, 512, 2560
    rng = np.random.default_rng(0)
    P = [torch.randn(n, d, device=dev) * 0.1 for n in (nU, nI)]
    M = [torch.randn(n, d, device=dev) * 1e-3 for n in (nU, nI)]
    V = [torch.rand(n, d, device=dev) * 1e-6 for n in (nU, nI)]
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

    def timeit(fn, reps=50, prep=None):
        ts = []
        for _ in range(reps):
            if prep:
                prep()
            torch.cuda._sleep(100000)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return float(np.median(ts))

    print(f"streamed      : {timeit(lambda: ops.adam_multi(tabs, d, consts, base, 0)):8.2f} us")
    for gap in (0, 1, 8, 32, 63, 127, 511):
        def prep(gap=gap):
            base.fill_(1000)
            for x in last:
                x.fill_(1000 - gap)
        t = timeit(lambda: ops.adam_multi(tabs, d, consts, base, 0, 'deferred', n_max_uniq=nmax),
                   prep=prep)
        f = timeit(lambda: ops.adam_multi(tabs, d, consts, base, 0, 'flush'), reps=10, prep=prep)
        print(f"gap {gap:4d}: deferred {t:8.2f} us   flush(all rows) {f:9.2f} us")


if __name__ == '__main__':
    main()
