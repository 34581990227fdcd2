"""K11 at C3's shapes (M = 102,400 rows) in isolation (diagnostic): forward and data-gradient
launch times by HIP events (median of 20) per width pair, and the fp32 MFMA fraction.

usage: python tools/probe_linear.py [--M 102400]
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
    ap.add_argument('--M', type=int, default=102400)
    args = ap.parse_args()
    from recbole_amd.model import layers
    dev = torch.device('cuda', 0)
    M = args.M
    res = {}
    for K, N in ((128, 128), (128, 256), (256, 128)):
        x = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev)
        b = torch.randn(N, device=dev)
        gy = torch.randn(M, N, device=dev)
        for name, fn in (('fwd', lambda: layers.linear_rows(x, W, b)),
                         ('dx', lambda: layers.linear_rows_grad(gy, W)),
                         ('torch_fwd', lambda: torch.nn.functional.linear(x, W, b))):
            ts = []
            for _ in range(22):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            us = float(np.median(ts[2:]))
            res[f'{K}x{N}_{name}_us'] = round(us, 1)
            res[f'{K}x{N}_{name}_frac'] = round(2 * M * K * N / (us * 1e-6) / 157.3e12, 3)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
