"""LightGCN host logic on the CPU: the normalised adjacency (bit-identical to the
oracle's scipy restatement of lightgcn.py:71-104) and the K7 unit plan."""
import numpy as np
import pytest

from oracle import cpu_ref


@pytest.mark.parametrize('seed', [0, 1])
def test_norm_adj_bitwise(seed):
    from recbole_amd.model.general_recommender.lightgcn import norm_adj_csr
    rng = np.random.default_rng(seed)
    U, I = 60, 90
    r, c = rng.integers(1, U, 800), rng.integers(1, I, 800)
    A = cpu_ref.lightgcn_norm_adj(r, c, U, I).coalesce()
    rp, cols, vals = norm_adj_csr(r, c, U, I)
    rows = np.repeat(np.arange(U + I), np.diff(rp))
    idx = A.indices().numpy()
    assert np.array_equal(idx[0], rows) and np.array_equal(idx[1], cols)
    assert np.array_equal(A.values().numpy(), vals)      # same float32 bits


def test_spmm_plan_covers_every_nonzero_once():
    from recbole_amd import ops
    rng = np.random.default_rng(3)
    deg = np.r_[0, 1, 5, 17, 0, 300, 2, 64, 65]
    rp = np.r_[0, np.cumsum(deg)]
    cols = rng.integers(0, len(deg), rp[-1])
    plan = ops.SpmmPlan(rp, cols, np.ones(rp[-1], np.float32), device='cpu', piece=16)
    ur, ub, us = plan.unit_row.numpy(), plan.unit_beg.numpy(), plan.unit_slot.numpy()
    assert len(ub) == len(ur) + 1 and ub[-1] == rp[-1]
    seen = np.zeros(rp[-1], dtype=int)
    for u, r in enumerate(ur):
        assert rp[r] <= ub[u] <= ub[u + 1] <= rp[r + 1] and ub[u + 1] - ub[u] <= 16
        seen[ub[u]:ub[u + 1]] += 1
    assert (seen == 1).all()
    assert set(ur.tolist()) == set(range(len(deg)))       # empty rows still get a unit
    fr, fp = plan.fix_row.numpy(), plan.fix_ptr.numpy()
    assert fr.tolist() == [r for r in range(len(deg)) if deg[r] > 16]
    for k, r in enumerate(fr):
        assert sorted(us[ur == r].tolist()) == list(range(fp[k], fp[k + 1]))
    assert (us[~np.isin(ur, fr)] == -1).all()


def test_spmm_plan_caps_units_of_hub_rows():
    from recbole_amd import ops
    deg = np.r_[3, 100_000, 5]
    rp = np.r_[0, np.cumsum(deg)]
    plan = ops.SpmmPlan(rp, np.zeros(rp[-1], np.int64), np.ones(rp[-1], np.float32),
                        device='cpu', piece=16, max_units=64)
    ur, ub = plan.unit_row.numpy(), plan.unit_beg.numpy()
    assert (ur == 1).sum() == 64 and plan.n_fix == 1
    sizes = np.diff(ub)[ur == 1]
    assert sizes.sum() == 100_000 and sizes.max() - sizes.min() <= 1
