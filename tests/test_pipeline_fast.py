"""The vectorised host pipeline pieces against the per-group /
per-pair restatements of the reference they replace: grouped ratio split
(dataset.py:1249-1315: groups in first-appearance order, _calcu_split_ids per
group), cumulative used-id CSRs (sampler.py:206-227), the atomic-file reader."""
import numpy as np
import pytest


def _calcu(tot, ratios):
    cnt = [int(ratios[i] * tot) for i in range(len(ratios))]
    cnt[0] = tot - sum(cnt[1:])
    for i in range(1, len(ratios)):
        if cnt[0] <= 1:
            break
        if 0 < ratios[-i] * tot < 1:
            cnt[-i] += 1
            cnt[0] -= 1
    return list(np.cumsum(cnt)[:-1])


def _loop_split(keys, ratios):
    groups, seen = {}, []
    for idx, k in enumerate(keys.tolist()):
        if k not in groups:
            groups[k] = []
            seen.append(k)
        groups[k].append(idx)
    parts = [[] for _ in ratios]
    for k in seen:
        g = groups[k]
        ids = _calcu(len(g), ratios)
        for p, s, e in zip(parts, [0] + ids, ids + [len(g)]):
            p.extend(g[s:e])
    return [np.asarray(p, dtype=np.int64) for p in parts]


@pytest.mark.parametrize('ratios', [[0.8, 0.1, 0.1], [0.5, 0.5], [1.0], [0.7, 0.2, 0.05, 0.05],
                                    [0.1, 0.1, 0.8]])
def test_grouped_ratio_split_matches_loop(ratios):
    from recbole_amd.data.dataset.dataset import _grouped_ratio_split
    rng = np.random.default_rng(len(ratios))
    sizes = np.r_[np.arange(1, 25), rng.integers(1, 200, 300)]
    keys = np.repeat(rng.permutation(len(sizes)) * 7 + 3, sizes)
    keys = keys[rng.permutation(len(keys))]
    tot = sum(ratios)
    r = [x / tot for x in ratios]
    got = _grouped_ratio_split(keys, r)
    exp = _loop_split(keys, r)
    assert len(got) == len(exp)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)


def test_cumulative_csr_matches_unique():
    from recbole_amd import ops
    rng = np.random.default_rng(0)
    n = 50
    phases = [(rng.integers(0, n, m), rng.integers(0, 300, m)) for m in (2000, 300, 300, 0)]
    ks, vs = [], []
    for u, i in phases:
        ks.append(u)
        vs.append(i)
        K, V = np.concatenate(ks), np.concatenate(vs)
        ptr, cols = ops.host_csr_build(K, V, n)
        assert ptr[0] == 0 and ptr[-1] == len(cols) and cols.dtype == np.int32
        for k in range(n):
            assert np.array_equal(cols[ptr[k]:ptr[k + 1]], np.unique(V[K == k]))
    with pytest.raises(Exception):
        ops.host_csr_build(np.array([0, n]), np.array([1, 2]), n)
    # large enough for the threaded row sort (rows split over threads)
    K = rng.integers(0, 97, 400_000)
    V = rng.integers(0, 5000, 400_000)
    ptr, cols = ops.host_csr_build(K, V, 97)
    order = np.lexsort((V, K))
    k2, v2 = K[order], V[order]
    keep = np.r_[True, (k2[1:] != k2[:-1]) | (v2[1:] != v2[:-1])]
    assert np.array_equal(cols, v2[keep])
    assert np.array_equal(np.diff(ptr), np.bincount(k2[keep], minlength=97))


def test_counting_order_is_stable_argsort():
    from recbole_amd import ops
    from recbole_amd.data.dataset.dataset import _stable_order
    rng = np.random.default_rng(1)
    for n, space in ((0, 5), (10, 3), (100000, 7000), (50000, 60)):
        k = rng.integers(0, space, n)
        assert np.array_equal(ops.host_counting_order(k, space), np.argsort(k, kind='stable'))
        assert np.array_equal(_stable_order(k), np.argsort(k, kind='stable'))
    with pytest.raises(Exception):
        ops.host_counting_order(np.array([0, 9]), 5)


def test_atomic_reader_matches_pandas(tmp_path):
    """_read_atomic == pd.read_csv (the reference's reader, dataset.py:342-408),
    missing-value tokens included (quoted or not), for the token, float and
    token_seq columns; also through the categorical (code) path."""
    import pandas as pd
    from recbole_amd.data.dataset.dataset import _read_atomic
    f = tmp_path / 'x.inter'
    f.write_text('user_id:token\titem_id:token\trating:float\tname:token_seq\tts:float\n'
                 '1\t007\t4.5\ta b\t878887116\n'
                 'x\t\t\t\t1.0000000000000002\n'
                 '"q"\t12\t3\tc\t-0\n'
                 # pandas' missing-value tokens (None, <NA>, a quoted empty field, NA)
                 'None\t<NA>\tNone\t""\tNA\n'
                 '""\tNA\t<NA>\tnull\t2\n'
                 '"NA"\tn/a\t1\tNone\t3\n')
    cols = ['user_id:token', 'item_id:token', 'rating:float', 'name:token_seq', 'ts:float']
    dt = {c: (np.float64 if c.endswith(':float') else str) for c in cols}
    got = _read_atomic(str(f), '\t', cols, dt)
    exp = pd.read_csv(str(f), delimiter='\t', usecols=cols, dtype=dt)
    assert list(got.columns) == list(exp.columns)
    for c in cols:
        g, e = got[c].values, exp[c].values
        assert len(g) == len(e)
        for a, b in zip(g, e):
            if isinstance(b, float) and np.isnan(b):
                assert isinstance(a, float) and np.isnan(a), (c, a)
            else:
                assert a == b and type(a) is type(b), (c, a, b)
    cat = _read_atomic(str(f), '\t', cols, dt, cat_cols=('user_id:token', 'item_id:token'))
    for c in ('user_id:token', 'item_id:token'):
        g = np.asarray(cat[c], dtype=object)
        e = exp[c].values
        assert [x if isinstance(x, str) else None for x in g] == \
            [x if isinstance(x, str) else None for x in e], c


def test_factorize_pieces_matches_pandas():
    import pandas as pd
    from recbole_amd.data.dataset.dataset import _factorize
    rng = np.random.default_rng(4)
    toks = np.array([f't{x}' for x in rng.integers(0, 40, 500)], dtype=object)
    toks[rng.integers(0, 500, 20)] = np.nan
    other = np.array([f't{x}' for x in rng.integers(20, 70, 200)], dtype=object)
    cat = pd.Categorical(toks[:300])
    pieces = [cat, toks[300:], other, pd.Categorical(other[::-1])]
    got_ids, got_u = _factorize(pieces)
    exp_ids, exp_u = pd.factorize(np.concatenate([np.asarray(cat, dtype=object), toks[300:],
                                                  other, other[::-1]]))
    assert np.array_equal(got_ids, exp_ids)
    assert list(got_u) == list(exp_u)


def _loop_loo(keys, leave_one_num):
    groups, seen = {}, []
    for idx, k in enumerate(keys.tolist()):
        if k not in groups:
            groups[k] = []
            seen.append(k)
        groups[k].append(idx)
    nxt = [[] for _ in range(leave_one_num + 1)]
    for k in seen:
        g = groups[k]
        tot = len(g)
        legal = min(leave_one_num, tot - 1)
        pr = tot - legal
        nxt[0].extend(g[:pr])
        for i in range(legal):
            nxt[-legal + i].append(g[pr])
            pr += 1
    return [np.asarray(x, dtype=np.int64) for x in nxt]


@pytest.mark.parametrize('leave_one_num', [1, 2, 3])
def test_grouped_leave_one_out_matches_loop(leave_one_num):
    from recbole_amd.data.dataset.dataset import _grouped_leave_one_out
    rng = np.random.default_rng(leave_one_num)
    sizes = np.r_[np.arange(1, 8), rng.integers(1, 60, 400)]
    keys = np.repeat(rng.permutation(len(sizes)) * 3 + 1, sizes)
    keys = keys[rng.permutation(len(keys))]
    got = _grouped_leave_one_out(keys, leave_one_num)
    exp = _loop_loo(keys, leave_one_num)
    assert len(got) == len(exp)
    for a, b in zip(got, exp):
        assert np.array_equal(a, b)
