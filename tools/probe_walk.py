"""Phase profile of the K4 walk on the C2 workload (GPU; needs the profiling build
MIREC_LIB=recbole_amd/_lib/alt/walkprof.so from
`tools/build_variant.sh walkprof -DMIREC_WALK_PROF`): shader-clock totals per
phase (setup, round 0, refills) per batch, refill-round counts.

usage: MIREC_LIB=... python tools/probe_walk.py [--keys 512] [--batches 64]
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--keys', type=int, default=512)
    ap.add_argument('--batches', type=int, default=64)
    args = ap.parse_args()
    import bench
    from recbole_amd._native import lib
    dev = torch.device('cuda:0')
    _, train, _, _, _, _ = bench.build_workload(dev)
    samp = train.sampler
    uid = train.dataset.inter_feat[train.uid_field]
    T, K, nb = train.times, args.keys, args.batches
    g = torch.Generator().manual_seed(7)
    idx = torch.randint(0, len(uid), (K * nb,), generator=g)
    keys = uid[idx.to(uid.device)].to(dev, torch.int64).contiguous()
    out = torch.empty(K * nb * T, dtype=torch.int64, device=dev)
    ws = torch.empty(lib().mirec_sample_walk_workspace_size(K, T), dtype=torch.uint8, device=dev)
    f = lib().mirec_walk_prof
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 16)()
    for rep in range(3):
        torch.cuda.synchronize()
        f(buf, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        samp.launch_batches(keys, K, nb, T, out, ws=ws)
        e1.record()
        torch.cuda.synchronize()
        f(buf, 0)
        us = e0.elapsed_time(e1) * 1e3 / nb
        v = list(buf)
        tot = (sum(v[:5]) or 1)
        ck = us / (tot / nb)                  # us per clock (the batch time covers every phase)
        print(f'   us/batch: setup {v[0] / nb * ck:.2f}, round-0 values+membership '
              f'{v[3] / nb * ck:.2f}, round-0 scan {v[4] / nb * ck:.2f}, round-0 tail '
              f'{v[1] / nb * ck:.2f}, refills {v[2] / nb * ck:.2f}', flush=True)
        print(f'rep {rep}: {us:.2f} us/batch; clocks/batch setup {v[0]/nb:.0f} round0 {v[1]/nb:.0f} '
              f'refill {v[2]/nb:.0f} (frac {v[0]/tot:.2f}/{v[1]/tot:.2f}/{v[2]/tot:.2f}); per batch: '
              f'pending after round 0 {v[8]/nb:.1f}, wide rounds {v[9]/nb:.2f}, tail entry '
              f'{v[10]/nb:.1f}, tail rounds {v[11]/nb:.2f}', flush=True)


if __name__ == '__main__':
    main()
