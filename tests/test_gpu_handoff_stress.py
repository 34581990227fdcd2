"""The in-launch hand-offs under UNEVEN load with L1-warm consumers
(MI355X_MICROARCH.md, inter-workgroup visibility: "test every hand-off under uneven load,
consumer L1-warm").

K35's split rows (csrc/step.hip part_store / join: write-through contribution vectors,
a per-wave drain, one agent-scope add per participant, an acquire on the last adder) and
the chained / onesweep sorts' status words (csrc/segsort.hip: relaxed agent-scope
tickets and counts) are each run REPS times back to back, while a streaming copy of
512 MB runs on another stream and occupies the CUs the launch does not get first (the
blocks of one launch then start and finish at very different times). The launches
reuse the same scratch addresses, so a consumer's L1 can hold lines of the previous
launch's vectors / words. Every output word is compared bitwise with the reference
(K3 + K5 for K35; numpy's stable sort for the sorts) after every launch.

Reference behaviour these kernels must reproduce: trainer.py:173 (the Adam step every
split row applies once, with ALL its contributions), the embedding backward's
per-row sums (bpr.py:74-83)."""
import numpy as np
import pytest
import torch

from test_gpu_step import build_case, check_k35, run_k35

pytestmark = pytest.mark.gpu

REPS = 12


def _load(dev):
    """A streaming copy on its own stream (≈ 60 us per call at HBM speed), issued in a
    burst so it overlaps the launches under test."""
    src = torch.empty(128 * 2 ** 20, dtype=torch.float32, device=dev).uniform_()
    dst = torch.empty_like(src)
    side = torch.cuda.Stream(device=dev)
    return src, dst, side


@pytest.mark.parametrize('d,T,s,Bc,few', [(128, 4, 12, 640, 5), (256, 3, 9, 96, 0),
                                          (256, 4, 10, 640, 3)])
def test_k35_split_rows_under_load(dev, d, T, s, Bc, few):
    c = build_case(dev, d, T, s, Bc, few)
    src, dst, side = _load(dev)
    main = torch.cuda.current_stream(dev)
    results = []
    for rep in range(REPS):
        side.wait_stream(main)
        with torch.cuda.stream(side):                 # the load first: it takes the CUs
            for _ in range(2 + rep % 3):
                dst.copy_(src)
        results.append(run_k35(c))
    torch.cuda.synchronize()
    for r in results:
        check_k35(c, r)


@pytest.mark.parametrize('kind', ['blocks', 'onesweep'])
def test_sort_status_words_under_load(dev, kind):
    from recbole_amd import ops
    rng = np.random.default_rng(3)
    if kind == 'blocks':               # 26 field blocks of 2,048 keys (C4's token fields)
        bn, nb = 2048, 26
        offs = np.cumsum([0] + [int(x) for x in rng.integers(1000, 1 << 20, nb - 1)])
        keys = np.concatenate([o + (np.minimum(rng.zipf(1.2, bn), 999) - 1)
                               for o in offs]).astype(np.int64)
        space = int(offs[-1]) + 1000
    else:                              # > ONESWEEP_MIN: the device-wide sort
        keys = (np.minimum(rng.zipf(1.1, 300_000), 3_000_000) - 1).astype(np.int64)
        space = 3_000_000
    n = len(keys)
    order = np.argsort(keys, kind='stable')
    u, first = np.unique(keys[order], return_index=True)
    kd = torch.as_tensor(keys, device=dev)
    status = torch.zeros(64, dtype=torch.int32, device=dev)
    src, dst, side = _load(dev)
    main = torch.cuda.current_stream(dev)
    outs = []
    for rep in range(REPS):
        side.wait_stream(main)
        with torch.cuda.stream(side):
            for _ in range(1 + rep % 3):
                dst.copy_(src)
        if kind == 'blocks':
            outs.append(ops.segment_sort_blocks(kd, bn, space, status=status))
        else:
            outs.append(ops.segment_sort(kd, space))
    torch.cuda.synchronize()
    for segs in outs:
        nu = int(segs.n_uniq.item())
        assert nu == len(u)
        assert np.array_equal(segs.perm[:n].cpu().numpy(), order)
        assert np.array_equal(segs.uniq[:nu].cpu().numpy(), u)
        assert np.array_equal(segs.seg[:nu + 1].cpu().numpy(), np.r_[first, n])
    assert int(status.abs().sum().item()) == 0
    for buf in ops._SORT_STATUS.values():
        assert int(buf.abs().sum().item()) == 0
