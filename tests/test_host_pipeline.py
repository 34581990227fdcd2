"""Host plumbing pinned by the reference's own tests and fixtures:
metric formulas (tests/metrics/*), full-sort loader arrays
(tests/data/test_dataloader.py:115-235), train batch order
(test_dataloader.py:31-58) and the ml-100k split the survey derives."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT


def test_metrics_match_reference_known_answers():
    from recbole_amd.evaluator.metrics import metrics_dict
    g = json.load(open(os.path.join(GOLDEN, 'metrics_known_answers.json')))
    t = g['topk']
    pos_idx, pos_len = np.array(t['pos_idx']), np.array(t['pos_len'])
    for name, exp in t['expected'].items():
        assert metrics_dict[name](pos_idx, pos_len).tolist() == np.array(exp).tolist(), name
    for case in g['loss'].values():
        trues, preds = np.array(case['trues']), np.array(case['preds'])
        assert metrics_dict['auc'](trues, preds) == case['auc']
        assert metrics_dict['rmse'](trues, preds) == case['rmse']
        assert metrics_dict['mae'](trues, preds) == case['mae']
        assert metrics_dict['logloss'](trues, preds) == pytest.approx(case['logloss'])


def test_vectorised_metrics_bit_identical_to_reference_loops():
    from oracle import cpu_ref
    from recbole_amd.evaluator.metrics import metrics_dict
    rng = np.random.default_rng(1)
    for t in range(200):
        n, K = int(rng.integers(1, 20)), int(rng.integers(1, 12))
        pi = rng.random((n, K)) < rng.random()
        pl = rng.integers(0 if t % 7 == 0 else 1, 15, n)
        for name in ['hit', 'mrr', 'precision', 'map', 'recall', 'ndcg']:
            with np.errstate(all='ignore'):
                a, b = metrics_dict[name](pi, pl), cpu_ref.METRICS[name](pi, pl)
            assert np.array_equal(a, b, equal_nan=True), name


def _prep(config_dict):
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset, data_preparation
    from recbole_amd.utils import init_seed
    cd = dict(config_dict, data_path=os.path.join(GOLDEN, 'data'), use_gpu=False)
    config = Config(config_dict=cd)
    init_seed(config['seed'], config['reproducibility'])
    return config, data_preparation(config, create_dataset(config))


def test_full_dataloader_arrays_match_reference_fixture():
    exp = json.load(open(os.path.join(GOLDEN, 'full_dataloader_expected.json')))
    config, (train, valid, test) = _prep(exp['config'])
    batches = list(test)
    assert len(batches) == len(exp['test'])
    for b, e in zip(batches, exp['test']):
        user_df, (hr, hc), srow, after, before = b
        assert user_df['user_id'].tolist() == [e['user']]
        assert list(user_df.pos_len_list) == [e['pos_len']]
        assert list(user_df.user_len_list) == [e['user_len']]
        assert hc.tolist() == e['history_col'] and (hr == 0).all()
        assert after.tolist() == e['swap_col_after']
        assert before.tolist() == e['swap_col_before'] and (srow == 0).all()


def test_train_batch_order_without_shuffle():
    config, (train, valid, test) = _prep({
        'model': 'BPR', 'dataset': 'general_dataloader', 'load_col': None,
        'eval_setting': 'TO_RS', 'training_neg_sample_num': 0, 'split_ratio': [0.8, 0.1, 0.1],
        'train_batch_size': 6, 'eval_batch_size': 2})
    for data, items, bs in [(train, list(range(1, 41)), 6), (valid, list(range(41, 46)), 2),
                            (test, list(range(46, 51)), 2)]:
        data.shuffle = False
        pr = 0
        for batch in data:
            assert batch['item_id'].tolist() == items[pr:pr + bs]
            pr += bs


def test_ml100k_split_sizes():
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset, data_preparation
    from recbole_amd.utils import init_seed
    config = Config(model='BPR', dataset='ml-100k',
                    config_dict={'data_path': os.path.join(ROOT, 'dataset'), 'use_gpu': False})
    init_seed(config['seed'], config['reproducibility'])
    ds = create_dataset(config)
    assert (ds.user_num, ds.item_num, ds.inter_num) == (944, 1682, 99991)
    train, valid, test = data_preparation(config, ds)
    assert (len(train.dataset), len(valid.dataset), len(test.dataset)) == (80799, 9596, 9596)
    assert len(train) == 40 and train.step == 2048 and train.times == 1


def test_sampler_used_csr_matches_python_sets():
    from recbole_amd.sampler.sampler import _csr_from_pairs
    rng = np.random.default_rng(5)
    u, i = rng.integers(0, 30, 500), rng.integers(1, 80, 500)
    ptr, cols = _csr_from_pairs(30, u, i)
    sets = [set() for _ in range(30)]
    for a, b in zip(u, i):
        sets[a].add(int(b))
    for k in range(30):
        assert cols[ptr[k]:ptr[k + 1]].tolist() == sorted(sets[k])


def test_fused_adam_constants_follow_torch():
    from recbole_amd.trainer.optim import FusedAdam
    p = torch.nn.Parameter(torch.zeros(4, 4))
    opt = FusedAdam([p], lr=1e-3)
    c = opt.step_constants(1, 3)
    for j, t in enumerate([1.0, 2.0, 3.0]):
        assert c[j, 0] == np.float32(1e-3 / (1 - 0.9 ** t))
        assert c[j, 1] == np.float32((1 - 0.999 ** t) ** 0.5)
        assert c[j, 2] == np.float32(1.0 / float(c[j, 1]))      # RN(1 / bc2_sqrt)
    with pytest.raises(ValueError):
        FusedAdam([p], betas=(0.9, 1.0))


def test_reciprocal_division_is_correctly_rounded():
    """K5 evaluates x / bc2_sqrt as q = x*r; q + fma(-q, d, x)*r with r = RN(1/d).
    Check it against IEEE division on the actual divisors (numpy float32, the
    fma emulated in float64: the residual is exact there; the last fma can
    double-round only with probability ~2^-29 per case). The exhaustive check
    (two binades of x, ~13k divisors, hardware fmaf) was run once offline."""
    from recbole_amd.trainer.optim import FusedAdam
    opt = FusedAdam([torch.nn.Parameter(torch.zeros(4))])
    c = opt.step_constants(1, 3000)
    rng = np.random.default_rng(0)
    x = np.sqrt(rng.random(20000).astype(np.float32) * np.float32(1e-6))
    for d, r in zip(c[::37, 1], c[::37, 2]):
        q = x * r
        e = (x.astype(np.float64) - q.astype(np.float64) * np.float64(d)).astype(np.float32)
        q2 = (q.astype(np.float64) + e.astype(np.float64) * np.float64(r)).astype(np.float32)
        assert np.array_equal(q2, x / d)


def test_metric_pattern_tables_equal_direct_formulas():
    """The pattern-table path of the top-K metrics (many users, small K) gives the
    same float64 rows as the direct vectorised formulas, incl. empty positive sets."""
    from recbole_amd.evaluator import metrics as M
    rng = np.random.default_rng(5)
    for K in (1, 3, 10):
        pos_idx = rng.random((20000, K)) < 0.3
        pos_len = rng.integers(0, 3 * K, 20000)
        for name in ('hit', 'mrr', 'precision', 'recall', 'ndcg', 'map'):
            with np.errstate(all='ignore'):
                a = M.metrics_dict[name](pos_idx, pos_len)
                b = M.topk_metric_rows(name, pos_idx, pos_len)
            assert np.array_equal(a, b, equal_nan=True), (K, name)
