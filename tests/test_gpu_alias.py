"""Alias-table fast mode on the GPU (labelled NON-PARITY, north_star (c)).

The reference has no alias sampler, so these tests pin the kernel to its own
spec (tests/alias_spec.py: same values for the same seed and counter, exactly)
and check the statistics the mode promises: draws follow the random_list's
value frequencies (chi-square), used ids are never returned, and each user's
draws follow the frequencies restricted to its unused ids."""
import numpy as np
import pytest
import torch
from scipy.stats import chisquare

from tests.alias_spec import sample, table_mass

pytestmark = pytest.mark.gpu


def _table(counts, dev):
    from recbole_amd import ops
    thr, alias = ops.alias_build(np.asarray(counts, dtype=np.int64))
    return thr, alias, torch.as_tensor(thr.view(np.int32), device=dev), torch.as_tensor(alias, device=dev)


def test_alias_kernel_matches_spec(dev):
    from recbole_amd import ops
    from recbole_amd.sampler.sampler import _csr_from_pairs
    rng = np.random.default_rng(1)
    n_items, n_users = 300, 40
    counts = rng.integers(0, 50, n_items)
    counts[0] = 0
    thr, alias, thr_d, al_d = _table(counts, dev)
    ku = rng.integers(0, n_users, 3000)
    kv = rng.integers(1, n_items, 3000)
    ptr, cols = _csr_from_pairs(n_users, ku, kv)
    used = [set(cols[ptr[u]:ptr[u + 1]].tolist()) for u in range(n_users)]
    up, uc = torch.as_tensor(ptr, device=dev), torch.as_tensor(cols, device=dev)
    bits = ops.used_bitmap(up, uc, n_users, n_items)
    keys = rng.integers(0, n_users, 333)
    kd = torch.as_tensor(keys, device=dev)
    for seed, counter, num, bk in ((7, 0, 3, None), (2 ** 63 + 5, 123456789, 4, 100)):
        exp = sample(thr, alias, seed, counter, keys, num, used, batch_keys=bk)
        got_csr = ops.sample_alias(thr_d, al_d, seed, counter, kd, num, up, uc, n_users, True,
                                   batch_keys=bk).cpu().numpy()
        got_bits = ops.sample_alias(thr_d, al_d, seed, counter, kd, num, up, uc, n_users, True,
                                    batch_keys=bk, used_bits=bits, n_bits=n_items).cpu().numpy()
        assert np.array_equal(got_csr, exp)
        assert np.array_equal(got_bits, exp)
        g = np.arange(len(exp))
        bk_ = bk or len(keys)
        owner = keys[(g // (bk_ * num)) * bk_ + (g % (bk_ * num)) % np.minimum(
            bk_, len(keys) - (g // (bk_ * num)) * bk_)]
        assert not any(int(v) in used[int(u)] for v, u in zip(got_csr, owner))
    # no rejection: plain table draws
    exp = sample(thr, alias, 9, 77, keys, 5)
    got = ops.sample_alias(thr_d, al_d, 9, 77, kd, 5, None, None, n_users, False).cpu().numpy()
    assert np.array_equal(got, exp)


def test_alias_distribution_chi_square(dev):
    """4M draws over a Zipf popularity table of 2,000 items follow the counts."""
    from recbole_amd import ops
    n = 2000
    counts = (1e5 / np.arange(1, n + 1) ** 1.0).astype(np.int64)
    counts[0] = 0
    thr, alias, thr_d, al_d = _table(counts, dev)
    keys = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
    v = torch.cat([ops.sample_alias(thr_d, al_d, 3, c << 22, keys, 1, None, None, 1, False)
                   for c in range(4)]).cpu().numpy()
    obs = np.bincount(v, minlength=n)
    assert obs[0] == 0
    p = table_mass(thr, alias)
    p = p / p.sum()
    nz = counts > 0
    assert chisquare(obs[nz], p[nz] * len(v)).pvalue > 1e-4
    # and the table is the counts' distribution (to 2^-32 per column)
    np.testing.assert_allclose(p, counts / counts.sum(), atol=1e-8)


def test_alias_rejection_conditional_distribution(dev):
    """One user owning the 20 most popular of 200 items: its draws avoid them
    and follow the counts renormalised over the rest."""
    from recbole_amd import ops
    n = 200
    counts = np.arange(n, 0, -1, dtype=np.int64) * 10
    counts[0] = 0
    thr, alias, thr_d, al_d = _table(counts, dev)
    used_items = np.arange(1, 21)
    up = torch.tensor([0, len(used_items)], dtype=torch.int64, device=dev)
    uc = torch.as_tensor(used_items.astype(np.int32), device=dev)
    keys = torch.zeros(1 << 19, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    v = ops.sample_alias(thr_d, al_d, 11, 0, keys, 2, up, uc, 1, True, status=status).cpu().numpy()
    assert int(status.item()) == 0
    obs = np.bincount(v, minlength=n)
    assert obs[:21].sum() == 0
    p = counts.astype(np.float64)
    p[:21] = 0
    p /= p.sum()
    assert chisquare(obs[21:], p[21:] * len(v)).pvalue > 1e-4


def test_alias_status_codes(dev):
    from recbole_amd import ops
    counts = np.array([0, 1, 1], dtype=np.int64)
    thr, alias, thr_d, al_d = _table(counts, dev)
    up = torch.tensor([0, 2], dtype=torch.int64, device=dev)
    uc = torch.tensor([1, 2], dtype=torch.int32, device=dev)       # every item used
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.sample_alias(thr_d, al_d, 1, 0, torch.zeros(4, dtype=torch.int64, device=dev), 1, up, uc,
                     1, True, status=st)
    assert int(st.item()) == -3
    st.zero_()
    ops.sample_alias(thr_d, al_d, 1, 0, torch.tensor([5], dtype=torch.int64, device=dev), 1,
                     up, uc, 1, True, status=st)
    assert int(st.item()) == -2


def test_alias_sampler_and_fused_training(tmp_path, dev):
    """neg_sampling_alias through the data pipeline: Sampler draws avoid each
    user's used items, the fused BPR step trains on alias negatives, and the
    evaluation loader's per-user calls work in the fast mode."""
    from tests.test_gpu_e2e import _pipeline
    from recbole_amd.trainer import Trainer
    config, train, valid, test, model = _pipeline(tmp_path, epochs=2, neg_sampling_alias=True)
    samp = train.sampler
    assert samp.alias is not None
    ptr, cols = samp.used_csr['train']
    users = torch.arange(1, samp.n_users, device=dev)
    v = samp.sample_by_user_ids(users, 4).view(4, -1).cpu().numpy()
    for k, u in enumerate(users.cpu().numpy()):
        assert not set(v[:, k].tolist()) & set(cols[ptr[u]:ptr[u + 1]].tolist())
    tr = Trainer(config, model)
    l0 = tr._train_epoch(train, 0)
    l1 = tr._train_epoch(train, 1)
    assert np.isfinite(l0) and np.isfinite(l1) and l1 < l0
    samp.check_status()
    # sampled validation (uniform 1000, one sampler call per user) in the fast mode
    score, res = tr._valid_epoch(valid)
    assert np.isfinite(score)
    valid.sampler.check_status()
    # the bench's fast-mode line: the same step with the alias draws (it must not
    # consume the walk pointer)
    assert samp.random_pr == 0
