"""north_star's gather roofline on counters: K3 (bpr_fwd_bwd) at
the throughput setting of SURVEY.md §8d (B = 65,536 positives, 4 negatives, d = 128)
on two table sizes:
  c2   the C2 tables (138,494 + 26,745 rows = 84.6 MB: they fit the 256 MiB Infinity
       cache, so repeated gathers may never reach HBM);
  big  2,000,000 + 2,000,000 rows (2.05 GB: past the LLC; uniform ids, so almost
       every row gather misses it).
HIP events per launch (median of `reps`); algorithmic bytes per launch =
2*(B + (1+T)B)*d*4 (rows read + gradient rows written) + 8*(B + (1+T)B) + 4*B. Run
under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` (separate passes) for the HBM
bytes of the same launches (tools/gpu_r3_gather.sh).

usage: python tools/gather_probe.py [--reps 20] [--out gpurun_out/gather.json]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def probe(nU, nI, B, T, d, reps, dev, tag):
    from recbole_amd import ops
    g = torch.Generator(device='cpu').manual_seed(7)
    EU = torch.randn(nU, d, device=dev) * 0.1
    EI = torch.randn(nI, d, device=dev) * 0.1
    user = torch.randint(0, nU, (B,), generator=g).to(dev)
    pos = torch.randint(1, nI, (B,), generator=g).to(dev)
    negs = torch.randint(1, nI, (T * B,), generator=g).to(dev)
    out = {}
    ops.bpr_fwd_bwd(EU, EI, user, pos, negs, T, out=out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ops.bpr_fwd_bwd(EU, EI, user, pos, negs, T, out=out)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    t = float(np.median(ts))
    rows = B + (1 + T) * B
    nbytes = 2 * rows * d * 4 + rows * 8 + B * 4
    return {'tables': tag, 'table_rows': [nU, nI], 'table_mb': round((nU + nI) * d * 4 / 2**20, 1),
            'kernel': f'K3 bpr_fwd_bwd<{d}> at B={B}', 'launches': reps + 1,
            'bytes_per_launch': nbytes, 'launch_us': round(t * 1e6, 1),
            'achieved': round(nbytes / t / 1e9, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(nbytes / t / 1e9 / HBM_PEAK_GBS, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    res = [probe(138494, 26745, 65536, 4, 128, args.reps, dev, 'c2'),
           probe(2_000_000, 2_000_000, 65536, 4, 128, args.reps, dev, 'big')]
    for r in res:
        print(json.dumps(r), flush=True)
    if args.out:
        json.dump(res, open(args.out, 'w'), indent=1)


if __name__ == '__main__':
    main()
