"""Phase timing of the per-block 8-bit sort (segsort_radix8_kernel) on C4's token keys:
26 field blocks of 2,048 Zipf(1.1) ids at their table offsets. With MIREC_LIB pointing at
a -DMIREC_R8_PROBE build, block 0 stamps wall_clock64 (100 MHz) at its phase ends.
usage: [MIREC_LIB=recbole_amd/_lib/alt/r8probe.so] python tools/probe_r8.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_models import _zipf_ids, c4_vocab          # noqa: E402
from recbole_amd import ops                           # noqa: E402
from recbole_amd._native import lib                  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    rng = np.random.default_rng(2020)
    vocab = [v + 1 for v in c4_vocab()]
    off = np.concatenate([[0], np.cumsum(vocab)[:-1]])
    B = 2048
    keys = np.concatenate([off[j] + _zipf_ids(rng, 1.1, B, vocab[j] - 1) for j in range(26)])
    space = int(sum(vocab))
    kd = torch.as_tensor(keys, device=dev)
    for _ in range(5):
        ops.segment_sort_blocks(kd, B, space)
    torch.cuda.synchronize()
    out = {}
    L = lib()
    if hasattr(L, 'mirec_r8_probe_read'):
        buf = (ctypes.c_uint64 * 16)()
        assert L.mirec_r8_probe_read(buf) == 0
        t = list(buf)
        out['block0_phase_us'] = {f'{k}': round((t[k] - t[0]) / 100.0, 2) for k in range(1, 11)
                                  if t[k] >= t[0] and t[k] - t[0] < 10 ** 7}
        out['shader_mhz'] = round((t[13] - t[12]) / max(1, t[7] - t[0]) * 100.0, 1)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(200):
        ops.segment_sort_blocks(kd, B, space)
    e.record()
    torch.cuda.synchronize()
    out['us_per_call_2launch'] = round(s.elapsed_time(e) / 200 * 1000, 2)
    spans = [int(np.ptp(keys[j * B:(j + 1) * B])).bit_length() for j in range(26)]
    out['span_bits'] = spans
    out['n_uniq_per_block'] = [int(len(np.unique(keys[j * B:(j + 1) * B]))) for j in range(26)]
    print(json.dumps(out))


if __name__ == '__main__':
    main()
