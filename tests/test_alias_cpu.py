"""Alias-table fast mode, host side (no GPU): mirec_alias_build's integer Vose table
encodes the count distribution to within one 2^-32 unit per column it touches,
for uniform, popularity (Zipf), sparse (zero counts) and single-item counts."""
import numpy as np
import pytest

from tests.alias_spec import draw, table_mass


def _check(counts):
    from recbole_amd import ops
    counts = np.asarray(counts, dtype=np.int64)
    thr, alias = ops.alias_build(counts)
    n = len(counts)
    assert thr.dtype == np.uint32 and alias.dtype == np.int32
    assert ((alias >= 0) & (alias < n)).all()
    mass = table_mass(thr, alias)
    exp = counts.astype(np.float64) * n * 2.0 ** 32 / counts.sum()
    touched = np.bincount(alias, minlength=n) + 1
    assert np.all(np.abs(mass - exp) <= touched + 1), np.abs(mass - exp).max()
    # zero-count values are never drawn: no column keeps mass for them
    z = counts == 0
    assert (mass[z] <= 1).all() and not np.isin(np.flatnonzero(z), alias[thr < 2 ** 32 - 1]).any()
    return thr, alias


def test_alias_uniform():
    c = np.ones(1000, dtype=np.int64)
    c[0] = 0                                   # item 0 is [PAD]: the walk never yields it
    _check(c)


def test_alias_zipf():
    rng = np.random.default_rng(0)
    c = (1e6 / np.arange(1, 5001) ** 1.1).astype(np.int64)
    rng.shuffle(c)
    c[0] = 0
    _check(c)


def test_alias_sparse_and_single():
    c = np.zeros(64, dtype=np.int64)
    c[[3, 17, 60]] = [5, 1, 1000]
    _check(c)
    one = np.zeros(10, dtype=np.int64)
    one[7] = 3
    thr, alias = _check(one)
    v = draw(thr, alias, 5, np.arange(1000, dtype=np.uint64), 0)
    assert (v == 7).all()


def test_alias_rejects_bad_counts():
    from recbole_amd import ops
    from recbole_amd._native import NativeError
    with pytest.raises(NativeError):
        ops.alias_build(np.zeros(5, dtype=np.int64))
    with pytest.raises(NativeError):
        ops.alias_build(np.array([1, -1, 2], dtype=np.int64))


def test_alias_spec_distribution_cpu():
    """The spec's draws follow the table (chi-square, 200k draws, 50 values)."""
    from scipy.stats import chisquare
    c = np.arange(1, 51, dtype=np.int64) ** 2
    from recbole_amd import ops
    thr, alias = ops.alias_build(c)
    v = draw(thr, alias, 1234, np.arange(200000, dtype=np.uint64), 0)
    obs = np.bincount(v, minlength=50)
    p = c / c.sum()
    assert chisquare(obs, p * len(v)).pvalue > 1e-3
