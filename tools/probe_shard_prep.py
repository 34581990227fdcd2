"""The row-sharded C2 step's per-chunk preparation at N ranks, timed on ONE GPU (the prep
is replicated or per-rank work that needs no peer): rank 0's grouping + plans for a chunk
of global batches of N x 512 positives (4 negatives), the global grouping every rank
repeated (rounds <= 5) against the owner-filtered one (each rank groups its ~1/N of the
slots: mirec_shard_select + K2 + mirec_shard_own_sel). HIP events around each call.

usage: python tools/probe_shard_prep.py [--ranks 8] [--batches 16] [--reps 5]
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
    ap.add_argument('--ranks', type=int, default=8)
    ap.add_argument('--batches', type=int, default=16)
    ap.add_argument('--reps', type=int, default=5)
    args = ap.parse_args()
    import bench
    from recbole_amd import ops
    from recbole_amd._native import check, lib
    dev = torch.device('cuda', 0)
    G, nb, B, T = args.ranks, args.batches, 512, 4
    Bc = G * B
    KI = (1 + T) * Bc
    u, i, nU, nI = bench.make_c2(2020)
    rng = np.random.default_rng(0)
    pick = rng.integers(0, len(u), nb * Bc)
    users = torch.as_tensor(u[pick], device=dev)
    items = torch.empty(nb, 1 + T, Bc, dtype=torch.int64)
    items[:, 0] = torch.as_tensor(i[pick]).view(nb, Bc)
    items[:, 1:] = torch.as_tensor(rng.integers(1, nI, (nb, T, Bc)))
    items = items.view(-1).to(dev)
    SU, SI = -(-nU // G), -(-nI // G)
    cap = min((2 + T) * B, -(-5 * (2 + T) * B // (4 * G)) + 64)
    r = 0
    L = lib()
    st = torch.cuda.current_stream(dev).cuda_stream
    z = lambda n, dt=torch.int32: torch.zeros(n, dtype=dt, device=dev)
    tabs = {'u': (users, Bc, SU, 0), 'i': (items, KI, SI, Bc)}
    bufs = {t: dict(keyed=z(nb * per, torch.int64), perm=z(nb * per), uniq=z(nb * per),
                    seg=z(nb * (per + 1)), nu=z(nb), ah=z(nb * per), nah=z(nb), sel=z(nb * per),
                    own=z(nb * per), oseg=z(nb * (per + 1)), on=z(nb), p2=z(nb * per),
                    oa=z(nb * per), ona=z(nb), nt=z(nb * per), na=z(nb * per))
            for t, (_, per, _, _) in tabs.items()}
    M = G * cap
    plan = [z(nb * M, torch.int64), z(nb * (Bc + KI)), z(nb * (2 + T) * B, torch.int64),
            z(nb * M), z(4)]
    ws = [None]
    times = {}

    def timed(name, fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        times.setdefault(name, []).append((a, b))

    def run(filtered):
        for t, (ids, per, S, off) in tabs.items():
            bb = bufs[t]
            cs = min(per, -(-5 * per // (4 * G)) + 64) if filtered else per
            if filtered:
                timed(f'{t} select', lambda: check(L.mirec_shard_select(
                    ids.data_ptr(), nb, per, G, S, r, cs, bb['keyed'].data_ptr(),
                    bb['sel'].data_ptr(), plan[4].data_ptr() + 8, st), 'select'))
            else:
                timed(f'{t} keys', lambda: check(L.mirec_shard_keys(
                    ids.data_ptr(), nb * per, G, S, bb['keyed'].data_ptr(), st), 'keys'))
            kk = bb['keyed'][:nb * cs]

            def sort():
                ws[0] = ops.segment_sort_batched(kk, cs, G * S + (1 if filtered else 0),
                                                 bb['perm'], bb['uniq'], bb['seg'], bb['nu'],
                                                 ws=ws[0])
            timed(f'{t} sort', sort)
            timed(f'{t} ahead', lambda: ops.uniq_ahead_diff(bb['uniq'], bb['nu'], cs, nb,
                                                            bb['ah'], bb['nah']))
            bb['cs'] = cs
        timed('plan', lambda: check(L.mirec_shard_plan(
            users.data_ptr(), items.data_ptr(), nb, Bc, B, T, G, r, cap,
            *[x.data_ptr() for x in plan], st), 'plan'))
        for t, (ids, per, S, off) in tabs.items():
            bb = bufs[t]
            a = [bb['uniq'].data_ptr(), bb['seg'].data_ptr(), bb['nu'].data_ptr(),
                 bb['perm'].data_ptr(), bb['cs'], nb, bb['ah'].data_ptr(), bb['nah'].data_ptr(),
                 plan[1].data_ptr(), Bc + KI, off, S, r]
            o = [bb['own'].data_ptr(), bb['oseg'].data_ptr(), bb['on'].data_ptr(),
                 bb['p2'].data_ptr(), bb['oa'].data_ptr(), bb['ona'].data_ptr(), st]
            if filtered:
                timed(f'{t} own', lambda: check(L.mirec_shard_own_sel(
                    *a, bb['sel'].data_ptr(), per, *o), 'own_sel'))
            else:
                timed(f'{t} own', lambda: check(L.mirec_shard_own(*a, *o), 'own'))
            timed(f'{t} next', lambda: check(L.mirec_shard_next(
                bb['own'].data_ptr(), bb['on'].data_ptr(), bb['oa'].data_ptr(),
                bb['ona'].data_ptr(), per, nb, bb['nt'].data_ptr(), bb['na'].data_ptr(), st),
                'next'))

    out = {'ranks': G, 'batches': nb, 'global_batch_positives': Bc}
    for filtered in (False, True):
        times.clear()
        for _ in range(args.reps):
            run(filtered)
        torch.cuda.synchronize()
        us = {k: round(float(np.median([a.elapsed_time(b) * 1e3 for a, b in v[1:]])), 1)
              for k, v in times.items()}
        tot = sum(us.values())
        key = 'owner_filtered' if filtered else 'global'
        out[key] = {'us_per_chunk': us, 'total_us_per_chunk': round(tot, 1),
                    'us_per_step': round(tot / nb, 2)}
        print(key, json.dumps(out[key]))
    print(json.dumps(out))


if __name__ == '__main__':
    main()
