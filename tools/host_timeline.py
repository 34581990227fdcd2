"""Host-side timeline of bench.py's timed region (diagnostic): wall time of each
host call between t0 and the closing synchronize for the driver's --warmup/--steps
window, without a profiler attached.

usage: python tools/host_timeline.py [--warmup 5] [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    import bench
    from recbole_amd.trainer import fused as F
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    _, _, _, _, _, step = bench.build_workload(dev, source='memory')
    W, K = args.warmup, args.steps
    marks = []
    t_ref = [0.0]

    def mark(name):
        marks.append((name, (time.perf_counter() - t_ref[0]) * 1e6))

    # wrap the host entry points of the timed region
    orig_prepare, orig_step = step._prepare, step._step

    def prepare(slot, chunk, *a):
        mark(f'prepare{chunk[:2]} in')
        orig_prepare(slot, chunk, *a)
        mark('prepare out')
    step._prepare = prepare

    def wrap(name):
        orig = getattr(step, name)

        def f(*a, **kw):
            mark(f'{name} in')
            r = orig(*a, **kw)
            mark(f'{name} out')
            return r
        setattr(step, name, f)
    for name in ('_enter_chunk', '_prepare_group', '_issue_groups', '_top_up_prep', '_entry',
                 '_flush', '_finish'):
        wrap(name)
    orig_replay = torch.cuda.CUDAGraph.replay

    def replay(self):
        mark('graph replay in')
        orig_replay(self)
        mark('graph replay out')
    torch.cuda.CUDAGraph.replay = replay
    for rep in range(args.reps):
        M = step.C
        nb = step.begin_epoch(cuts=(W, W + K, W + K + M), hold_prep_from=W)
        step.run_batches(0, W)
        torch.cuda.synchronize()
        marks.clear()
        t_ref[0] = t0 = time.perf_counter()
        torch.cuda._sleep(1)
        mark('marker')
        step.release_prep(upto=W + K)
        mark('released')
        step.run_batches(W, W + K)
        mark('run_batches out')
        step.sync_params()
        mark('sync_params out')
        torch.cuda.synchronize()
        mark('synchronized')
        el = time.perf_counter() - t0
        print(f'rep {rep}: {el * 1e6:.1f} us  = {K * step.Bg / el / 1e6:.2f} M pos/s')
        for n, t in marks:
            print(f'   {t:9.1f}  {n}')
        step.end_epoch(W + K)
    del F


if __name__ == '__main__':
    main()
