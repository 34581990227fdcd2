"""Diagnostic (GPU): is the K4 walk's round 0 bound by the used-id bitmap's address
locality? Times one-batch walks (512 keys x 4 negatives, the C2 batch) on the C2
bitmap (463 MB) for (a) random users over all 138 K, (b) users confined to a
1.7 MB slice of the bitmap (users 1..512), and (c) the same keys with rejection
off (no bitmap loads at all).

usage: python tools/probe_walk_locality.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from recbole_amd import ops
    dev = torch.device('cuda', 0)
    config, train, test, model, opt, step = bench.build_workload(dev)
    samp = train.sampler
    rl, pr, up, uc, bits, n_bits, reject, status = samp.walk_args(dev)
    nU = step.nU
    B, T, reps = 512, 4, 200
    g = torch.Generator(device='cpu').manual_seed(0)
    cases = {
        'random users': torch.randint(1, nU, (reps, B), generator=g),
        'users 1..512': torch.randint(1, 513, (reps, B), generator=g),
    }
    out = torch.empty(B * T, dtype=torch.int64, device=dev)
    ws = torch.empty(lib_ws(B, T), dtype=torch.uint8, device=dev)
    for name, keys in cases.items():
        for rej in (True, False):
            keys_d = keys.to(dev)
            for r in range(10):            # warm
                ops.sample_walk(rl, pr, keys_d[r], T, up, uc, nU, rej, out=out, ws=ws,
                                used_bits=bits, n_bits=n_bits)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for r in range(reps):
                ops.sample_walk(rl, pr, keys_d[r], T, up, uc, nU, rej, out=out, ws=ws,
                                used_bits=bits, n_bits=n_bits)
            b.record()
            torch.cuda.synchronize()
            print(f'{name:14s} reject={rej!s:5s}: {a.elapsed_time(b) * 1e3 / reps:6.2f} us per '
                  f'batch launch', flush=True)


def lib_ws(B, T):
    from recbole_amd._native import lib
    return lib().mirec_sample_walk_workspace_size(B, T)


if __name__ == '__main__':
    main()
