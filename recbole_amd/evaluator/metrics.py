"""Metric formulas (mirror of recbole/evaluator/metrics.py:27-322), vectorised
numpy in float64 — the per-user rows are bit-identical to the reference's
loops (checked against its known-answer tests, tests/test_metrics.py)."""
from logging import getLogger

import numpy as np
from sklearn.metrics import auc as sk_auc
from sklearn.metrics import mean_absolute_error, mean_squared_error


def _ranks(pos_index):
    return np.broadcast_to(np.arange(1, pos_index.shape[1] + 1), pos_index.shape)


def _capped_ranks(pos_index, pos_len):
    """The reference's `ranges[lens:] = ranges[lens - 1]` (map_/ndcg_): rank
    capped at L = min(pos_len, K); L == 0 indexes ranges[-1], i.e. K everywhere."""
    K = pos_index.shape[1]
    L = np.where(pos_len > K, K, pos_len)
    r = np.minimum(_ranks(pos_index), L[:, None])
    return np.where((L == 0)[:, None], K, r)


def hit_(pos_index, pos_len):
    return (np.cumsum(pos_index, axis=1) > 0).astype(int)


def mrr_(pos_index, pos_len):
    idxs = pos_index.argmax(axis=1)
    hit = pos_index[np.arange(len(idxs)), idxs] > 0
    val = np.where(hit, 1 / (idxs + 1), 0.0)
    col = np.arange(pos_index.shape[1])[None, :]
    return np.where(col >= idxs[:, None], val[:, None], 0.0).astype(np.float64)


def precision_(pos_index, pos_len):
    return pos_index.cumsum(axis=1) / np.arange(1, pos_index.shape[1] + 1)


def map_(pos_index, pos_len):
    pre = precision_(pos_index, pos_len)
    sum_pre = np.cumsum(pre * pos_index.astype(np.float64), axis=1)
    return sum_pre / _capped_ranks(pos_index, np.asarray(pos_len))


def recall_(pos_index, pos_len):
    return np.cumsum(pos_index, axis=1) / np.asarray(pos_len).reshape(-1, 1)


def ndcg_(pos_index, pos_len):
    # every row of the reference's idcg / discount matrices is the same vector:
    # compute it once (same float64 ops, same values) and index / broadcast it
    K = pos_index.shape[1]
    w = 1.0 / np.log2(np.arange(1, K + 1, dtype=np.float64) + 1)
    idcg = np.cumsum(w)[_capped_ranks(pos_index, np.asarray(pos_len)) - 1]
    dcg = np.cumsum(np.where(pos_index, w[None, :], 0.0), axis=1)
    return dcg / idcg


def _binary_clf_curve(trues, preds):
    """evaluator/utils.py:87-116."""
    trues = (trues == 1)
    desc = np.argsort(preds)[::-1]
    preds = preds[desc]
    trues = trues[desc]
    uniq = np.where(np.diff(preds))[0]
    thr = np.r_[uniq, trues.size - 1]
    tps = np.cumsum(trues)[thr]
    fps = 1 + thr - tps
    return fps, tps


def auc_(trues, preds):
    fps, tps = _binary_clf_curve(trues, preds)
    if len(fps) > 2:
        keep = np.where(np.r_[True, np.logical_or(np.diff(fps, 2), np.diff(tps, 2)), True])[0]
        fps, tps = fps[keep], tps[keep]
    tps = np.r_[0, tps]
    fps = np.r_[0, fps]
    if fps[-1] <= 0:
        getLogger().warning('No negative samples in y_true, false positive value should be meaningless')
        fpr = np.repeat(np.nan, fps.shape)
    else:
        fpr = fps / fps[-1]
    if tps[-1] <= 0:
        getLogger().warning('No positive samples in y_true, true positive value should be meaningless')
        tpr = np.repeat(np.nan, tps.shape)
    else:
        tpr = tps / tps[-1]
    return sk_auc(fpr, tpr)


def mae_(trues, preds):
    return mean_absolute_error(trues, preds)


def rmse_(trues, preds):
    return np.sqrt(mean_squared_error(trues, preds))


def log_loss_(trues, preds):
    eps = 1e-15
    preds = np.clip(np.float64(preds), eps, 1 - eps)
    return np.sum(-trues * np.log(preds) - (1 - trues) * np.log(1 - preds)) / len(preds)


metrics_dict = {
    'ndcg': ndcg_, 'hit': hit_, 'precision': precision_, 'map': map_, 'recall': recall_,
    'mrr': mrr_, 'rmse': rmse_, 'mae': mae_, 'logloss': log_loss_, 'auc': auc_,
}

# ---------------------------------------------------------------------------
# Pattern tables. A top-K metric row depends only on the row's K hit bits and,
# for map/ndcg, on min(pos_len, K) (recall divides by pos_len itself). For small
# K every distinct row is computed ONCE by the functions above — the same float64
# operations, hence the same values — and gathered per user: the [n_users, K]
# matrices are bit-identical, at a fraction of the host time for 10^5+ users.
_PATTERN_MAX_K = 12
_LEN_DEPENDENT = ('map', 'ndcg')


def _all_patterns(K):
    codes = np.arange(1 << K, dtype=np.int64)
    return ((codes[:, None] >> np.arange(K)) & 1).astype(bool)


def uses_patterns(pos_index):
    K, n = pos_index.shape[1], pos_index.shape[0]
    return K <= _PATTERN_MAX_K and n >= (1 << K) * 4


def pattern_codes(pos_index):
    """Row codes sum_k hit[k] << k of a [n, K] hit matrix (the pattern-table index)."""
    K = pos_index.shape[1]
    return np.asarray(pos_index, dtype=np.int64) @ (np.int64(1) << np.arange(K, dtype=np.int64))


def topk_metric_rows(name, pos_index, pos_len, codes=None):
    """metrics_dict[name](pos_index, pos_len) through the pattern table when
    max(topk) is small; identical values either way. `codes`: pattern_codes of
    pos_index when the caller evaluates several metrics of the same matrix."""
    fn = metrics_dict[name]
    K = pos_index.shape[1]
    if not uses_patterns(pos_index):
        return fn(pos_index, pos_len)
    pos_len = np.asarray(pos_len)
    if codes is None:
        codes = pattern_codes(pos_index)
    pats = _all_patterns(K)
    if name == 'recall':
        # cumsum of hits / pos_len: the same integer cumsum and the same division
        return np.cumsum(pats, axis=1)[codes] / pos_len.reshape(-1, 1)
    if name in _LEN_DEPENDENT:
        L = np.where(pos_len > K, K, pos_len)                 # 0..K (0 = empty positive set)
        rows = np.repeat(pats, K + 1, axis=0)
        lens = np.tile(np.arange(K + 1), 1 << K)
        table = fn(rows, lens)
        return table[codes * (K + 1) + L]
    return fn(pats, np.ones(1 << K, dtype=np.int64))[codes]
