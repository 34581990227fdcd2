"""K4 walk micro-benchmark on the C2 workload: one launch walks `--batches`
consecutive batches of `--keys` users (drawn like training positives: users of
random training interactions) x 4 negatives; prints us per batch and the
rejection rate (extra walk positions per slot).

    python tools/bench_walk.py --keys 512 4096
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--keys', type=int, nargs='+', default=[512, 4096])
    ap.add_argument('--batches', type=int, default=64)
    ap.add_argument('--reps', type=int, default=5)
    args = ap.parse_args()
    import bench
    dev = torch.device('cuda:0')
    config, train, test, model, opt, step = bench.build_workload(dev)
    samp = train.sampler
    uid = train.dataset.inter_feat[train.uid_field]
    T = train.times
    g = torch.Generator().manual_seed(7)
    res = {}
    for K in args.keys:
        n = K * args.batches
        idx = torch.randint(0, len(uid), (n,), generator=g)
        keys = uid[idx.to(uid.device)].to(dev, torch.int64).contiguous()
        out = torch.empty(n * T, dtype=torch.int64, device=dev)
        from recbole_amd._native import lib
        ws = torch.empty(lib().mirec_sample_walk_workspace_size(K, T), dtype=torch.uint8,
                         device=dev)
        times, adv = [], []
        for r in range(args.reps):
            if samp._rl_dev is None:
                samp.to_device(dev)
            pr0 = int(samp._pr_dev.item())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            samp.launch_batches(keys, K, args.batches, T, out, ws=ws)
            e1.record()
            torch.cuda.synchronize()
            pr1 = int(samp._pr_dev.item())
            L = samp._rl_dev.numel()
            adv.append(((pr1 - pr0) % L) / float(n * T))
            times.append(e0.elapsed_time(e1) * 1e3 / args.batches)
        res[K] = {'us_per_batch': round(min(times[1:] or times), 2),
                  'walk_positions_per_slot': round(sum(adv) / len(adv), 4),
                  'status': int(samp._status.item())}
        print(K, res[K], flush=True)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
