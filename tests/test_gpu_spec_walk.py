"""K4s (csrc/sampler.hip walk_spec_kernel + walk_commit_kernel, mirec_sample_walk_spec):
the walk of a chunk of batches by speculation equals the serial walk (K4,
mirec_sample_walk, itself pinned to the oracle's C and numpy restatements of
sampler.py:82-154) bit for bit — every value, the walk pointer after it, the status —
whatever the windows: statistics that fit the data, windows of one candidate (every
batch after the first falls back to the serial walk), a mean far off (all miss),
batches whose round-0 rejections exceed what a candidate resolves (n0 > 256), a random
list shorter than a batch (wrap-around inside round 0), the CSR and the bitmap
membership, more than 16 batches (two launch pairs), one batch, a ragged last batch is
not walked here (fixed-size batches only), bad keys (status -2) and a walk that
cannot terminate (status -3). Also the chunk preparation's key rows."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _setup(dev, n_users, n_items, deg_hi, seed, n_inter=60000):
    rng = np.random.default_rng(seed)
    deg = np.minimum(rng.integers(1, deg_hi + 1, n_users), n_items - 2)
    u = np.repeat(np.arange(n_users), deg)
    i = rng.integers(1, n_items, len(u))
    ptr, cols = cpu_ref.used_csr(n_users, u, i)
    rl = rng.permutation(np.arange(1, n_items))
    # keys drawn like train interactions (heavy users appear more often)
    inter_u = np.repeat(np.arange(n_users), np.diff(ptr))
    return rng, rl, ptr, cols, inter_u


def _stats(rl, ptr, cols, key_counts, Kb, num):
    """The sampler's window statistics (Sampler.walk_stats)."""
    L = len(rl)
    mult = np.bincount(rl, minlength=int(rl.max()) + 1)
    cs = np.concatenate([[0], np.cumsum(mult[cols])])
    p = np.minimum((cs[ptr[1:]] - cs[ptr[:-1]]) / L, 0.999)
    w = key_counts / key_counts.sum()
    q = p / (1 - p)
    eq, eq2 = (w * q).sum(), (w * q / (1 - p)).sum()
    var = Kb * num * eq2 + Kb * num * num * max((w * q * q).sum() - eq * eq, 0)
    return Kb * num * eq, float(np.sqrt(var))


def _dev_walk(dev, rl, ptr, cols, bits):
    from recbole_amd import ops
    drl = torch.as_tensor(rl.astype(np.int32), device=dev)
    dup = torch.as_tensor(ptr.astype(np.int64), device=dev)
    duc = torch.as_tensor(cols.astype(np.int32) if len(cols) else np.zeros(1, np.int32),
                          device=dev)
    n_users, n_bits = len(ptr) - 1, int(rl.max()) + 1
    mem = dict(used_bits=ops.used_bitmap(dup, duc, n_users, n_bits), n_bits=n_bits) if bits else {}
    return drl, dup, duc, mem


def _both(dev, rl, ptr, cols, keys, Kb, nb, num, stats, bits, pr0=0, n_key_space=None):
    from recbole_amd import ops
    drl, dup, duc, mem = _dev_walk(dev, rl, ptr, cols, bits)
    n_key_space = n_key_space or len(ptr) - 1
    dk = torch.as_tensor(keys, dtype=torch.int64, device=dev)
    res = []
    for spec in (False, True):
        pr = torch.tensor([pr0], dtype=torch.int64, device=dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        if spec:
            out = ops.sample_walk_spec(drl, pr, dk, Kb, nb, num, dup, duc, n_key_space, True,
                                       *stats, status=st, **mem)
        else:
            out = ops.sample_walk(drl, pr, dk, num, dup, duc, n_key_space, True, batch_keys=Kb,
                                  n_batches=nb, status=st, **mem)
        res.append((out.cpu().numpy(), int(pr.item()), int(st.item())))
    return res


@pytest.mark.parametrize('bits', [False, True])
@pytest.mark.parametrize('nb', [1, 4, 16, 21])
@pytest.mark.parametrize('windows', ['fit', 'one', 'off'])
def test_spec_walk_equals_serial(dev, bits, nb, windows):
    Kb, num = 512, 4
    rng, rl, ptr, cols, inter_u = _setup(dev, 3000, 6000, 120, 7 + nb)
    keys = inter_u[rng.integers(0, len(inter_u), Kb * nb)]
    stats = {'fit': _stats(rl, ptr, cols, np.bincount(inter_u, minlength=3000), Kb, num),
             'one': (0.0, 0.0), 'off': (400.0, 1.0)}[windows]
    (a, pa, sa), (b, pb, sb) = _both(dev, rl, ptr, cols, keys, Kb, nb, num, stats, bits,
                                     pr0=int(rng.integers(0, len(rl))))
    assert np.array_equal(a, b) and pa == pb and sa == sb == 0


def test_spec_walk_heavy_rejection_and_short_list(dev):
    """~40 % of the items used per key (n0 ~ 800 > 256: every candidate left to the
    serial walk), and a random list of 1,499 values under 2,048-slot batches."""
    Kb, num, nb = 1024, 2, 5
    rng, rl, ptr, cols, inter_u = _setup(dev, 200, 1500, 600, 3)
    keys = inter_u[rng.integers(0, len(inter_u), Kb * nb)]
    stats = _stats(rl, ptr, cols, np.bincount(inter_u, minlength=200), Kb, num)
    (a, pa, sa), (b, pb, sb) = _both(dev, rl, ptr, cols, keys, Kb, nb, num, stats, True)
    assert np.array_equal(a, b) and pa == pb and sa == sb == 0


def test_spec_walk_moderate_rejection_short_list(dev):
    """ml-100k-like: 1,682 items, ~6 % used per key, batches wrap the list."""
    Kb, num, nb = 1024, 2, 9
    rng, rl, ptr, cols, inter_u = _setup(dev, 943, 1683, 200, 4)
    keys = inter_u[rng.integers(0, len(inter_u), Kb * nb)]
    stats = _stats(rl, ptr, cols, np.bincount(inter_u, minlength=943), Kb, num)
    (a, pa, sa), (b, pb, sb) = _both(dev, rl, ptr, cols, keys, Kb, nb, num, stats, True)
    assert np.array_equal(a, b) and pa == pb and sa == sb == 0


def test_spec_walk_bad_key_status(dev):
    Kb, num, nb = 512, 4, 3
    rng, rl, ptr, cols, inter_u = _setup(dev, 300, 2000, 50, 5)
    keys = inter_u[rng.integers(0, len(inter_u), Kb * nb)]
    keys[Kb + 17] = 300 + 5                                   # outside [0, n_users)
    stats = _stats(rl, ptr, cols, np.bincount(inter_u, minlength=300), Kb, num)
    (a, pa, sa), (b, pb, sb) = _both(dev, rl, ptr, cols, keys, Kb, nb, num, stats, False)
    assert np.array_equal(a, b) and pa == pb and sa == sb == -2


def test_spec_walk_livelock_status(dev):
    """User 0 may take only item 2, user 1 only item 1; the list alternates so that the
    walk cannot terminate: status -3 from both walks, the same values up to it."""
    rl = np.array([1, 2, 3, 4])
    ptr, cols = cpu_ref.used_csr(2, np.array([0, 0, 0, 1, 1, 1]), np.array([1, 3, 4, 2, 3, 4]))
    keys = np.array([0, 1] * 4)
    res = _both(dev, rl, ptr, cols, keys, 2, 4, 1, (0.5, 0.5), False)
    (a, pa, sa), (b, pb, sb) = res
    assert sa == sb == -3


def test_spec_walk_key_rows(dev):
    """With user_keys / item_keys: the chunk preparation's key rows (users; positives at
    the head of each (1+T)*Kb item row), and the values at out + Kb of each row."""
    from recbole_amd import ops
    Kb, num, nb = 512, 4, 6
    rng, rl, ptr, cols, inter_u = _setup(dev, 3000, 6000, 120, 9)
    keys = inter_u[rng.integers(0, len(inter_u), Kb * nb)]
    items = rng.integers(1, 6000, Kb * nb)
    stats = _stats(rl, ptr, cols, np.bincount(inter_u, minlength=3000), Kb, num)
    drl, dup, duc, mem = _dev_walk(dev, rl, ptr, cols, True)
    KI = (1 + num) * Kb
    dk = torch.as_tensor(keys, device=dev)
    di = torch.as_tensor(items, device=dev)
    uk = torch.zeros(nb * Kb, dtype=torch.int64, device=dev)
    ik = torch.zeros(nb * KI, dtype=torch.int64, device=dev)
    pr = torch.zeros(1, dtype=torch.int64, device=dev)
    ops.sample_walk_spec(drl, pr, dk, Kb, nb, num, dup, duc, 3000, True, *stats,
                         out=ik[Kb:], out_stride=KI, items=di, user_keys=uk, item_keys=ik,
                         key_stride=KI, **mem)
    pr2 = torch.zeros(1, dtype=torch.int64, device=dev)
    ref = ops.sample_walk(drl, pr2, dk, num, dup, duc, 3000, True, batch_keys=Kb, n_batches=nb,
                          **mem).cpu().numpy().reshape(nb, num * Kb)
    ikh = ik.cpu().numpy().reshape(nb, KI)
    assert np.array_equal(uk.cpu().numpy(), keys)
    assert np.array_equal(ikh[:, :Kb], items.reshape(nb, Kb))
    assert np.array_equal(ikh[:, Kb:], ref)
    assert int(pr.item()) == int(pr2.item())
