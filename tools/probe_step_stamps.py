"""Where a K35 launch (csrc/step.hip) spends its time: the diagnostic build with
per-block real-time stamps (MIREC_LIB=recbole_amd/_lib/alt/step_stamps.so, built by
`tools/build_variant.sh step_stamps -DMIREC_STEP_STAMPS`), one eager step at a time on
the C2 workload. Per launch: the spread of block start times (dispatch), and per block
class (look-ahead rows, touched user rows, touched item rows) the time from entry to
the first load levels, to the end of the contributions / loads, and to the end (shares of
split rows: the end of the last arriver only) — as
quantiles over the blocks, in microseconds (100 MHz stamps: 10 ns resolution). The
stamp build's own run time is not quoted anywhere: its shares are what count.

usage: MIREC_LIB=recbole_amd/_lib/alt/step_stamps.so python tools/probe_step_stamps.py
       [--warmup 96] [--steps 24]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TICK_US = 0.01          # s_memrealtime: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--warmup', type=int, default=96)
    ap.add_argument('--steps', type=int, default=24)
    args = ap.parse_args()
    import bench
    from recbole_amd._native import lib
    L = lib()
    L.mirec_step_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device('cuda', 0)
    _, _, _, _, _, step = bench.build_workload(dev, source='memory')
    nb = step.begin_epoch(cuts=(args.warmup,))
    step.run_batches(0, args.warmup)
    torch.cuda.synchronize()
    nU_max, nI_max = step._n_max[0], step._n_max[1]
    cap = 256                                        # shares per (table, batch): step.hip kSplitCap
    rpb = 4                                          # rows (waves) per workgroup: MIREC_STEP_RPB
    halves = 2 if step.d >= 128 else 1               # look-ahead slots per row
    # segments (stamps per wave, each segment padded to whole workgroups): shares U, I,
    # look-ahead U, I (halves x rows), touched U, I
    starts = [0]
    for n in (cap, cap, halves * nU_max, halves * nI_max, nU_max, nI_max):
        starts.append(starts[-1] + -(-n // rpb) * rpb)
    buf = np.zeros(32768 * 4, dtype=np.uint64)
    out = []
    for b in range(args.warmup, args.warmup + args.steps):
        L.mirec_step_stamps_clear()
        torch.cuda.synchronize()
        step.run_batches(b, b + 1)                 # mid-chunk: eager, one K35 launch
        torch.cuda.synchronize()
        L.mirec_step_stamps(buf.ctypes.data, buf.nbytes)
        st = buf.reshape(-1, 4).astype(np.int64)[:starts[-1]]
        live = (st[:, 3] > 0) & (st[:, 1] > 0)     # blocks that did work (stamp 3 written)
        t0 = st[st[:, 0] > 0, 0].min()
        rec = {'batch': b, 'makespan_us': round((st[live, 3].max() - t0) * TICK_US, 2),
               'dispatch_spread_us': np.round(np.quantile(
                   (st[st[:, 0] > 0, 0] - t0) * TICK_US, [0.5, 0.9, 1.0]), 2).tolist()}
        names = ('share_users', 'share_items', 'ahead_users', 'ahead_items', 'touched_users',
                 'touched_items')
        for q, name in enumerate(names):
            a, e = starts[q], starts[q + 1]
            s = st[a:e][live[a:e]]
            if len(s) == 0:
                rec[name] = None
                continue
            q = lambda x: np.round(np.quantile(x * TICK_US, [0.5, 0.9, 1.0]), 2).tolist()
            rec[name] = {'blocks': int(len(s)), 'start': q(s[:, 0] - t0),
                         'to_loads': q(s[:, 1] - s[:, 0]), 'loads_or_contrib': q(s[:, 2] - s[:, 1]),
                         'tail': q(s[:, 3] - s[:, 2]), 'end': q(s[:, 3] - t0)}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    step.end_epoch(args.warmup + args.steps)


if __name__ == '__main__':
    main()
