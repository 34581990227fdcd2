"""Device-side timeline of bench.py's driver window WITHOUT a profiler attached
(diagnostic): timing events recorded on the walk, group and model streams around
each chunk's walk half, grouping half and model launch, plus host timestamps of
the same calls, all relative to an event/host mark at t0.

usage: python tools/event_timeline.py [--warmup 5] [--steps 20] [--reps 3]
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
    ap.add_argument('--ramp', default=None)
    ap.add_argument('--eager', action='store_true', help='no graphs: events around every launch')
    args = ap.parse_args()
    import bench
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    _, _, _, _, _, step = bench.build_workload(dev)
    if args.ramp:
        step.RAMP = tuple(int(x) for x in args.ramp.split(','))
    if args.eager:
        step.use_graph = False
    W, K = args.warmup, args.steps
    evs = []           # (name, event, host us)
    t_ref = [0.0]

    def mark(name, stream):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        evs.append((name, e, (time.perf_counter() - t_ref[0]) * 1e6))

    orig_prepare, orig_group = step._prepare, step._prepare_group
    slot_chunk = {}

    def prepare(slot, chunk, on=None):
        st = on if on is not None else step.prep_stream
        mark(f'walk{chunk[:2]} issue' + (' (model stream)' if on is not None else ''), st)
        orig_prepare(slot, chunk, on)
        slot_chunk[id(slot)] = chunk
        mark(f'walk{chunk[:2]} done', st)

    def group(slot):
        c = slot_chunk.get(id(slot), ('?', '?'))[:2]
        mark(f'group{c} issue(after walk wait)', step.group_stream)
        orig_group(slot)
        mark(f'group{c} done', step.group_stream)

    step._prepare, step._prepare_group = prepare, group
    for rep in range(args.reps):
        M = step.C
        step.begin_epoch(cuts=(W, W + K, W + K + M), hold_prep_from=W)
        step.run_batches(0, W)
        torch.cuda.synchronize()
        evs.clear()
        main_s = torch.cuda.current_stream(dev)
        t_ref[0] = t0 = time.perf_counter()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        if args.eager:
            step.kernel_events = []
        step.release_prep(upto=W + K)
        b = W
        while b < W + K:                       # chunk by chunk, marks around each launch
            k = step._chunk_of(b)
            b0, nb, _ = step._plan[k]
            nxt = min(b0 + nb, W + K)
            mark(f'model{(b0, nb)} enter', main_s)
            step.run_batches(b, nxt)
            mark(f'model{(b0, nb)} end', main_s)
            b = nxt
        step.sync_params()
        mark('flush end', main_s)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f'rep {rep}: {el * 1e6:.1f} us = {K * step.Bg / el / 1e6:.2f} M pos/s')
        for name, e, h in evs:
            print(f'   gpu {e0.elapsed_time(e) * 1e3:8.1f}  host {h:8.1f}  {name}')
        if args.eager:
            for name, a, b_ in step.kernel_events:
                print(f'   kernel {name:8s} {e0.elapsed_time(a) * 1e3:8.1f} -> '
                      f'{e0.elapsed_time(b_) * 1e3:8.1f}  ({a.elapsed_time(b_) * 1e3:6.1f})')
            step.kernel_events = None
        step.release_prep()
        step.end_epoch(W + K)


if __name__ == '__main__':
    main()
