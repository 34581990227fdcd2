"""Writes tests/golden/*.json — the reference's known-answer vectors as data.

Sources (transcribed, not executed — the reference may not be run here,
SURVEY.md §8c):
  metrics_known_answers.json   tests/metrics/test_topk_metrics.py:15-79 and
                               tests/metrics/test_loss_metrics.py:16-52
  full_dataloader_expected.json tests/data/test_dataloader.py:115-235
                               (test half; the valid half is superseded by the
                               fork's uni1000 validation, data/utils.py:86-88)
  data/general_*                the atomic-file fixtures of tests/data/ (copied)
Also writes sampler_walk.json: self-generated vectors of the sampler walk from
the oracle's C restatement (parity pinned by restatement only).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', '..'))


def log2(x):
    return float(np.log2(x))


def metrics():
    pos_idx = [[0, 0, 0], [1, 1, 1], [1, 0, 1], [0, 0, 1]]
    pos_len = [1, 3, 4, 2]
    e = {
        'hit': [[0, 0, 0], [1, 1, 1], [1, 1, 1], [0, 0, 1]],
        'ndcg': [[0, 0, 0], [1, 1, 1],
                 [1, 1 / log2(2) / (1 / log2(2) + 1 / log2(3)),
                  (1 / log2(2) + 1 / log2(4)) / (1 / log2(2) + 1 / log2(3) + 1 / log2(4))],
                 [0, 0, 1 / log2(4) / (1 / log2(2) + 1 / log2(3))]],
        'mrr': [[0, 0, 0], [1, 1, 1], [1, 1, 1], [0, 0, 1 / 3]],
        'map': [[0, 0, 0], [1, 1, 1], [1, 1 / 2, (1 / 3) * ((1 / 1) + (2 / 3))],
                [0, 0, (1 / 3) * (1 / 2)]],
        'recall': [[0, 0, 0], [1 / 3, 2 / 3, 3 / 3], [1 / 4, 1 / 4, 2 / 4], [0, 0, 1 / 2]],
        'precision': [[0, 0, 0], [1 / 1, 2 / 2, 3 / 3], [1 / 1, 1 / 2, 2 / 3], [0, 0, 1 / 3]],
    }
    loss = {
        'case0': {'preds': [0.1, 0.9, 0.2, 0.3], 'trues': [1, 0, 1, 1],
                  'auc': 0.0,
                  'rmse': float(np.sqrt((0.9 ** 2 + 0.9 ** 2 + 0.8 ** 2 + 0.7 ** 2) / 4)),
                  'logloss': float((-np.log(0.1) - np.log(0.2) - np.log(0.3) - np.log(0.1)) / 4),
                  'mae': (0.9 + 0.9 + 0.8 + 0.7) / 4},
        'case1': {'preds': [0.7, 0.5, 0.6, 0.2], 'trues': [0, 1, 1, 0],
                  'auc': 2 / (2 * 2),
                  'rmse': float(np.sqrt((0.7 ** 2 + 0.5 ** 2 + 0.4 ** 2 + 0.2 ** 2) / 4)),
                  'logloss': float((-np.log(0.5) - np.log(0.6) - np.log(0.3) - np.log(0.8)) / 4),
                  'mae': (0.7 + 0.5 + 0.4 + 0.2) / 4},
    }
    return {'topk': {'pos_idx': pos_idx, 'pos_len': pos_len, 'expected': e}, 'loss': loss}


def full_dataloader():
    test = [
        {'user': 1, 'pos_len': 5, 'user_len': 101, 'history_col': list(range(1, 46)),
         'swap_col_after': [0, 1, 2, 3, 4, 46, 47, 48, 49, 50],
         'swap_col_before': [50, 49, 48, 47, 46, 4, 3, 2, 1, 0]},
        {'user': 2, 'pos_len': 5, 'user_len': 101,
         'history_col': list(range(1, 36)) + [41, 42],
         'swap_col_after': [0, 1, 2, 3, 4, 36, 37, 38, 39, 40],
         'swap_col_before': [40, 39, 38, 37, 36, 4, 3, 2, 1, 0]},
        {'user': 3, 'pos_len': 1, 'user_len': 101, 'history_col': [],
         'swap_col_after': [0, 1], 'swap_col_before': [1, 0]},
    ]
    return {'config': {'model': 'BPR', 'dataset': 'general_full_dataloader', 'load_col': None,
                       'eval_setting': 'TO_RS,full', 'training_neg_sample_num': 1,
                       'split_ratio': [0.8, 0.1, 0.1], 'train_batch_size': 6,
                       'eval_batch_size': 100},
            'test': test}


def sampler_walk():
    from oracle import cpu_ref
    rng = np.random.default_rng(2020)
    cases = []
    for c in range(6):
        n_users, n_items = int(rng.integers(3, 40)), int(rng.integers(10, 300))
        nnz = int(rng.integers(1, n_users * n_items // 3))
        u = rng.integers(0, n_users, nnz)
        i = rng.integers(1, n_items, nnz)
        ptr, cols = cpu_ref.used_csr(n_users, u, i)
        if (np.diff(ptr) + 1 >= n_items).any():
            continue
        np.random.seed(2020 + c)
        rl = cpu_ref.random_list_uniform(n_items)
        pr = 0
        batches = []
        for b in range(4):
            K, num = int(rng.integers(1, 64)), int(rng.integers(1, 6))
            keys = rng.integers(0, n_users, K)
            out, pr = cpu_ref.c_sample_walk(rl, pr, keys, num, ptr, cols, n_users, True)
            batches.append({'keys': keys.tolist(), 'num': num, 'out': out.tolist(), 'pr': pr})
        cases.append({'n_users': n_users, 'n_items': n_items, 'used_ptr': ptr.tolist(),
                      'used_cols': cols.tolist(), 'random_list': rl.tolist(),
                      'batches': batches})
    return cases


if __name__ == '__main__':
    for name, fn in [('metrics_known_answers.json', metrics),
                     ('full_dataloader_expected.json', full_dataloader),
                     ('sampler_walk.json', sampler_walk)]:
        with open(os.path.join(HERE, name), 'w') as f:
            json.dump(fn(), f)
        print('wrote', name)
