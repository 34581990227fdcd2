"""Do the parallel branches of a captured HIP graph run concurrently? (diagnostic)

Captures [fork -> stream A: spin ~T | stream B: spin ~T -> join] and [A: spin T; then
spin T] and times replays with events: equal times mean the branches were serialized.
Also times the host cost of hipGraphLaunch for graphs of 1..64 kernel nodes.

usage: python tools/probe_graph_fork.py
"""
import time

import torch


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    cyc = int(2.4e3 * 100)                     # ~100 us of spinning at 2.4 GHz
    main_s = torch.cuda.current_stream()

    def graph_of(fn):
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        cap.wait_stream(main_s)
        with torch.cuda.graph(g, stream=cap):
            fn(cap)
        main_s.wait_stream(cap)
        return g

    def forked(cap):
        side = torch.cuda.Stream()
        side.wait_stream(cap)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        cap.wait_stream(side)

    def serial(cap):
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)

    for name, fn in (('forked', forked), ('serial', serial)):
        g = graph_of(fn)
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        print(f'{name}: replay {min(ts):.1f} us (two ~100 us spins)', flush=True)

    for n in (1, 8, 16, 64):
        def many(cap, n=n):
            for _ in range(n):
                torch.cuda._sleep(10)
        g = graph_of(many)
        g.replay()
        torch.cuda.synchronize()
        hs = []
        for _ in range(10):
            torch.cuda._sleep(int(2.4e3 * 300))     # keep the queue busy: pure host cost
            t = time.perf_counter()
            g.replay()
            hs.append((time.perf_counter() - t) * 1e6)
            torch.cuda.synchronize()
        print(f'graph of {n} nodes: hipGraphLaunch host {min(hs):.1f} us (median '
              f'{sorted(hs)[5]:.1f})', flush=True)


if __name__ == '__main__':
    main()
