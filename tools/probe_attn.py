"""K9e at C3's shapes (B = 2,048, L = 50, H = 2, dh = 64, SASRec mask) in isolation
(diagnostic): forward and backward launch times by HIP events (median of 20), with and
without dropout.

usage: python tools/probe_attn.py [--B 2048] [--L 50]
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
    ap.add_argument('--B', type=int, default=2048)
    ap.add_argument('--L', type=int, default=50)
    ap.add_argument('--H', type=int, default=2)
    args = ap.parse_args()
    from recbole_amd._native import check, lib, ptr
    dev = torch.device('cuda', 0)
    B, L, H = args.B, args.L, args.H
    g = torch.Generator().manual_seed(0)
    q, k, v, go = (torch.randn(B, L, H * 64, generator=g).to(dev) for _ in range(4))
    lens = torch.randint(4, L + 1, (B,), generator=g)
    seq = (torch.arange(L)[None, :] < lens[:, None]).long()
    ext = seq[:, None, None, :] * (torch.triu(torch.ones(L, L), 1) == 0).long()[None, None]
    mask = ((1.0 - ext.float()) * -10000.0).to(dev).contiguous()
    out, dq, dk, dv = (torch.empty_like(q) for _ in range(4))
    lse = torch.empty(B * H, 64, device=dev)
    keep = torch.empty(B * H, 64, dtype=torch.int64, device=dev)
    counter = torch.zeros(1, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    L_ = lib()
    res = {}
    for p in (0.0, 0.5):
        def fwd():
            check(L_.mirec_attn_fwd_f32(ptr(q), ptr(k), ptr(v), ptr(mask), B, L, H, p, 7,
                                        ptr(counter) if p else None, ptr(out), ptr(lse),
                                        ptr(keep) if p else None, st), 'fwd')

        def bwd():
            check(L_.mirec_attn_bwd_f32(ptr(q), ptr(k), ptr(v), ptr(mask), ptr(go), ptr(lse),
                                        ptr(keep) if p else None, ptr(counter) if p else None,
                                        B, L, H, p, ptr(dq), ptr(dk), ptr(dv), st), 'bwd')
        for name, fn in (('fwd', fwd), ('bwd', bwd)):
            ts = []
            for _ in range(22):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                fn()
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            res[f'{name}_p{p}'] = round(float(np.median(ts[2:])), 1)
    flops_b = 5 * 2 * B * H * L * L * 64
    res['bwd_frac_p0.5'] = round(flops_b / (res['bwd_p0.5'] * 1e-6) / 157.3e12, 3)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
