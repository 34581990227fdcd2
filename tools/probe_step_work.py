"""Executed work of K35 (and of the flush / entry catch-ups) in bench.py's windows, from
the diagnostic build's counters (MIREC_LIB=recbole_amd/_lib/alt/work.so, built by
`tools/build_variant.sh work -DMIREC_STEP_COUNT`; csrc/adam_core.h MIREC_WORK): the
element-steps actually executed by kind (full zero-gradient steps, vanishing steps that
move only m and v, gradient steps; zero-state rows and rows already current are never
touched and so never counted), the rows stepped / replayed and the contributions formed.
Runs bench.py's sequence (--warmup W --steps K, then the 64-step measurement window one
eager launch at a time + its flush) and writes per-window totals and per-launch means.

Flop model of the executed work (per element): gradient step 13 (torch's formula, sqrt and
each division one op), zero-gradient step with the p update 9, vanishing step 3 (m: fma,
v: mul); BPR per contribution: user row (1+T) dots of 2d + T*4d (contrib_u) + d (the sum),
item as positive (1+T)*2d + T*2d + d, item as negative 2*2d + d + d.
Bytes: algorithmic = (touched rows + look-ahead rows) x (p, m, v) x d x 4 read and written;
gathered = the partner rows every contribution reads ((2+T) rows for a user / positive
contribution, 3 for a negative) x d x 4.

usage: MIREC_LIB=recbole_amd/_lib/alt/work.so python tools/probe_step_work.py [--warmup 5]
       [--steps 20] [--out profiles/r04_k35_work.json]
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

NAMES = ['zero_full', 'zero_vanish', 'grad_steps', 'ahead_own_step', 'touched_rows',
         'ahead_halves', 'contrib_user', 'contrib_pos', 'contrib_neg', 'split_parts',
         'flush_rows']


def read(L, clear=True):
    a = (ctypes.c_ulonglong * 16)()
    b = (ctypes.c_ulonglong * 16)()
    torch.cuda.synchronize()
    assert L.mirec_work_counters(a, 1 if clear else 0) == 0
    assert L.mirec_work_counters_adam(b, 1 if clear else 0) == 0
    return {n: int(a[i]) + int(b[i]) for i, n in enumerate(NAMES)}


def model(c, d, T):
    fl = {'adam': 13 * c['grad_steps'] + 9 * (c['zero_full'] + c['ahead_own_step'])
                  + 3 * c['zero_vanish'],
          'bpr': c['contrib_user'] * ((1 + T) * 2 * d + T * 4 * d + d)
                 + c['contrib_pos'] * ((1 + T) * 2 * d + T * 2 * d + d)
                 + c['contrib_neg'] * (2 * 2 * d + 2 * d)}
    rows = c['touched_rows'] + c['ahead_halves'] / 2.0
    return {'flops': fl['adam'] + fl['bpr'], 'flops_adam': fl['adam'], 'flops_bpr': fl['bpr'],
            'algorithmic_bytes': rows * 3 * d * 4 * 2,
            'gathered_bytes': ((c['contrib_user'] + c['contrib_pos']) * (2 + T)
                               + c['contrib_neg'] * 3) * d * 4,
            'element_steps': c['grad_steps'] + c['zero_full'] + c['zero_vanish']
                             + c['ahead_own_step']}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    import bench
    from recbole_amd._native import lib
    L = lib()
    for f in (L.mirec_work_counters, L.mirec_work_counters_adam):
        f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        f.restype = ctypes.c_int
    dev = torch.device('cuda', 0)
    _, _, _, _, _, step = bench.build_workload(dev, d=128, neg=4)
    W, K, M, d, T = args.warmup, args.steps, step.C, 128, step.times
    step.begin_epoch(cuts=(W, W + K, W + K + M), hold_prep_from=W, flush_at=(W + K, W + K + M))
    step.run_batches(0, W)
    read(L)
    step.release_prep(upto=W + K)
    step.run_batches(W, W + K)
    timed = read(L)
    step.sync_params()
    timed_flush = read(L)
    out = {'config': {'warmup': W, 'steps': K, 'd': d, 'T': T, 'B': step.B,
                      'lib': os.environ.get('MIREC_LIB')},
           'timed_region': {'counts': timed, 'flush_counts': timed_flush,
                            **model({k: timed[k] + timed_flush[k] for k in NAMES}, d, T)}}
    step.release_prep()
    per = []
    for b in range(W + K, W + K + M):
        step.run_batches(b, b + 1)       # eager mid-chunk launches (step + loss bookkeeping)
        per.append(read(L))
    # the chunk ends at W+K+M with its flush (enqueued by the last run_batches)
    fl = per[-1]
    mean = {k: float(np.mean([p[k] for p in per[:-1]])) for k in NAMES}
    out['measurement_window'] = {'steps': M, 'per_launch_mean': mean,
                                 'per_launch': model(mean, d, T),
                                 'last_step_plus_flush': fl,
                                 'window_total': model({k: sum(p[k] for p in per) for k in NAMES},
                                                       d, T)}
    step.end_epoch(W + K + M)
    print(json.dumps(out, indent=1))
    if args.out:
        json.dump(out, open(args.out, 'w'), indent=1)


if __name__ == '__main__':
    main()
