"""Latency of one K2 LDS sort workgroup (segment_sort_batched, one batch) against n and
key space: the serial part of the chunk pipeline's fill. HIP events over
200 back-to-back launches on the current stream; prints one JSON line per case."""
import json
import sys
import torch

sys.path.insert(0, '.')
from recbole_amd import ops  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    g = torch.Generator(device='cpu').manual_seed(0)
    for n, space in ((64, 138494), (512, 138494), (512, 26745), (2560, 26745), (2560, 138494),
                     (2560, 16), (8192, 26745)):
        for nb in (1, 4, 64):
            keys = torch.randint(0, space, (nb * n,), generator=g).to(dev)
            perm = torch.empty(nb * n, dtype=torch.int32, device=dev)
            uniq = torch.empty(nb * n, dtype=torch.int32, device=dev)
            seg = torch.empty(nb * (n + 1), dtype=torch.int32, device=dev)
            nu = torch.empty(nb, dtype=torch.int32, device=dev)
            ws = ops.segment_sort_batched(keys, n, space, perm, uniq, seg, nu)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 200
            a.record()
            for _ in range(reps):
                ops.segment_sort_batched(keys, n, space, perm, uniq, seg, nu, ws)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3 / reps
            # check one batch against a stable argsort
            k0 = keys[:n].cpu()
            ok = torch.equal(perm[:n].cpu().long(), torch.sort(k0, stable=True).indices)
            print(json.dumps({'n': n, 'space': space, 'batches': nb, 'us_per_launch': round(us, 2),
                              'perm_ok': bool(ok)}), flush=True)


if __name__ == '__main__':
    main()
