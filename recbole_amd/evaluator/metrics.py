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
    ranks = _ranks(pos_index).astype(np.float64)
    idcg_full = np.cumsum(1.0 / np.log2(ranks + 1), axis=1)
    idcg = np.take_along_axis(idcg_full, _capped_ranks(pos_index, np.asarray(pos_len)) - 1,
                              axis=1)
    dcg = np.cumsum(np.where(pos_index, 1.0 / np.log2(ranks + 1), 0), axis=1)
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
