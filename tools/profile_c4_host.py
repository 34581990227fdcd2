"""Host-side profile (cProfile) of the C4 DeepFM step: the generic trainer step is
bound by host work, not by the GPU (tools/bench_models.py C4 trace: GPU busy ~50 %)."""
import cProfile
import io
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import bench_models as bm  # noqa: E402


def _timed(step, steps, warmup, opt):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    for key in ('tottime', 'cumulative'):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(35)
        print(s.getvalue())
    return 1.0


bm._timed = _timed
bm.CPU_BASELINE = False
bm.bench_c4(torch.device('cuda', 0), 100, 10)
