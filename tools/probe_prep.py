"""Launch latency of the chunk preparation's kernels on the C2 workload (diagnostic):
the K4 walk (serial, one workgroup) against K4s (speculative, two launches per 16
batches), and the grouping side — K36 (mirec_chunk_group, one launch) against the
launches it replaces (K2 LDS sorts + mirec_step_records + look-ahead lists) — for
chunks of 1..64 batches. HIP events over back-to-back launches on one stream (the
walk restarts from the same pointer every repetition). Prints one JSON line per case.

usage: python tools/probe_prep.py [--reps 50]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=50)
    args = ap.parse_args()
    import bench
    from recbole_amd import ops
    from types import SimpleNamespace
    dev = torch.device('cuda', 0)
    _, train, _, _, _, step = bench.build_workload(dev, source='memory')
    step.begin_epoch()
    torch.cuda.synchronize()
    samp = train.sampler
    rl, pr, up, uc, bits, n_bits, reject, status = samp.walk_args(dev)
    users = step._users
    items = step._items
    Bc, T, nU, nI = step.Bg, step.times, step.nU, step.nI
    KI = (1 + T) * Bc
    counts = np.bincount(users.cpu().numpy(), minlength=nU)
    stats = samp.walk_stats(counts, Bc, T)
    print(json.dumps({'walk_stats': {'r_mean': round(stats[0], 2), 'r_sd': round(stats[1], 2)}}),
          flush=True)
    mem = dict(used_bits=bits, n_bits=n_bits)
    for nb in (1, 4, 8, 16, 64):
        out = torch.empty(nb * KI, dtype=torch.int64, device=dev)
        uk = torch.empty(nb * Bc, dtype=torch.int64, device=dev)
        p0 = int(pr.item())
        res = {'batches': nb}

        def serial():
            pr.fill_(p0)
            ops.sample_walk(rl, pr, users, T, up, uc, nU, True, batch_keys=Bc, n_batches=nb,
                            out=out[Bc:], out_stride=KI, status=status, **mem)

        def spec():
            pr.fill_(p0)
            ops.sample_walk_spec(rl, pr, users, Bc, nb, T, up, uc, nU, True, *stats, out=out[Bc:],
                                 out_stride=KI, status=status, items=items, user_keys=uk,
                                 item_keys=out, key_stride=KI, **mem)
        res['walk_serial_us'] = round(timed(serial, args.reps), 1)
        serial()
        ref = out.clone()
        res['walk_spec_us'] = round(timed(spec, args.reps), 1)
        spec()
        torch.cuda.synchronize()
        res['spec_equal'] = bool(torch.equal(out.view(nb, KI)[:, Bc:], ref.view(nb, KI)[:, Bc:]))
        # grouping side on the walked keys
        z = lambda n: torch.zeros(n, dtype=torch.int32, device=dev)
        o = {}
        for tag, per in (('u', Bc), ('i', KI)):
            o[f'{tag}_perm'], o[f'{tag}_uniq'] = z(nb * per), z(nb * per)
            o[f'{tag}_seg'], o[f'{tag}_nu'] = z(nb * (per + 1)), z(nb)
            o[f'{tag}_rec'], o[f'{tag}_crec'] = z(nb * ops.step_record_ints(per)), z(nb * per * 8)
            o[f'{tag}_ahead'], o[f'{tag}_nah'] = z(nb * per), z(nb)
        res['k36_us'] = round(timed(lambda: ops.chunk_group(uk, out, nb, Bc, T, nU, nI, o),
                                    args.reps), 1)
        ws = [None]

        def old():
            for tag, keys, per, space in (('u', uk, Bc, nU), ('i', out, KI, nI)):
                ws[0] = ops.segment_sort_batched(keys, per, space, o[f'{tag}_perm'],
                                                 o[f'{tag}_uniq'], o[f'{tag}_seg'],
                                                 o[f'{tag}_nu'], ws=ws[0])
            g = {t: SimpleNamespace(perm=o[f'{t}_perm'], uniq=o[f'{t}_uniq'], seg=o[f'{t}_seg'],
                                    n_uniq=o[f'{t}_nu']) for t in 'ui'}
            ops.step_records(uk, out, nb, Bc, T, nU, nI, g['u'], g['i'],
                             out=[o[k] for k in ('u_rec', 'u_crec', 'i_rec', 'i_crec')])
        res['sort_records_us'] = round(timed(old, args.reps), 1)
        print(json.dumps(res), flush=True)
    step.end_epoch(0)


if __name__ == '__main__':
    main()
