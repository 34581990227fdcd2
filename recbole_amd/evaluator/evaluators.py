"""Evaluators (mirror of recbole/evaluator/evaluators.py:37-370,
abstract_evaluator.py:18-120 — the base classes live in
abstract_evaluator.py). TopKEvaluator.collect keeps the reference's
score-matrix contract for models without a fused scorer; the fused full-sort
path feeds `evaluate_pos_idx` with the K6 kernel's positive flags directly."""
from collections import ChainMap

import numpy as np
import torch

from recbole_amd.evaluator.abstract_evaluator import GroupedEvaluator, IndividualEvaluator
from recbole_amd.evaluator.metrics import (metrics_dict, pattern_codes, topk_metric_rows,
                                           uses_patterns)

topk_metrics = {m.lower(): m for m in ['Hit', 'Recall', 'MRR', 'Precision', 'NDCG', 'MAP']}
loss_metrics = {m.lower(): m for m in ['AUC', 'RMSE', 'MAE', 'LOGLOSS']}
rank_metrics = {m.lower(): m for m in ['GAUC']}
group_metrics = ChainMap(topk_metrics, rank_metrics)
individual_metrics = ChainMap(loss_metrics)


class TopKEvaluator(GroupedEvaluator):

    def __init__(self, config, metrics):
        super().__init__(config, metrics)
        self.topk = config['topk']
        self._check_args()

    def _check_args(self):
        if isinstance(self.topk, (int, list)):
            if isinstance(self.topk, int):
                self.topk = [self.topk]
            for k in self.topk:
                if k <= 0:
                    raise ValueError(f'topk must be a positive integer or a list of positive '
                                     f'integers, but get `{k}`')
        else:
            raise TypeError('The topk must be a integer, list')

    # the score-matrix contract (get_score_matrix) is GroupedEvaluator's
    # (abstract_evaluator.py:65-95); collect = evaluators.py:53-76
    def collect(self, interaction, scores_tensor):
        user_len_list = interaction.user_len_list
        scores = torch.flip(self.get_score_matrix(scores_tensor, user_len_list), dims=[-1])
        shape = torch.full((len(user_len_list), 1), scores.shape[1], device=scores.device)
        _, topk_idx = torch.topk(scores, max(self.topk), dim=-1)
        return torch.cat((topk_idx, shape), dim=1)

    def evaluate(self, batch_matrix_list, eval_data):
        pos_len_list = eval_data.get_pos_len_list()
        res = torch.cat(batch_matrix_list, dim=0).cpu().numpy()
        topk_idx, shapes = res[:, :-1], res[:, -1]
        assert len(pos_len_list) == len(topk_idx)
        pos_idx = topk_idx >= (shapes - pos_len_list).reshape(-1, 1)
        return self.evaluate_pos_idx(pos_idx, pos_len_list)

    def evaluate_pos_idx(self, pos_idx, pos_len_list):
        """Metric reduction from the [n_users, max(topk)] positive matrix
        (evaluators.py:78-141)."""
        out = {}
        # one pattern-code pass for all metrics; each metric's mean over users is
        # the same ordered reduction as the stacked [metrics, users, K] mean
        # (axis 0 of a [users, K] matrix), without the stacked copy
        codes = pattern_codes(pos_idx) if uses_patterns(pos_idx) else None

        def one(m):
            return topk_metric_rows(m.lower(), pos_idx, pos_len_list, codes).mean(axis=0)
        if len(self.metrics) > 1 and pos_idx.shape[0] >= 1 << 16:
            # 10^5+ users: the metrics are independent numpy passes (GIL released in
            # the gathers / ufuncs), one thread each — the same values
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(min(len(self.metrics), 8)) as ex:
                vals = list(ex.map(one, self.metrics))
        else:
            vals = [one(m) for m in self.metrics]
        for m, v in zip(self.metrics, vals):
            for k in self.topk:
                out[f'{m}@{k}'] = round(v[k - 1], self.precision)
        return out

    def evaluate_pos_idx_chunks(self, chunks, n_users):
        """evaluate_pos_idx over (pos_idx, pos_len) row blocks arriving in user order
        (the fused evaluator hands over each K6 launch's block while the next runs).
        Each metric keeps a running [1, K] sum continued block by block — the same
        sequential over-users reduction as the mean of the whole matrix (numpy's
        axis-0 reduce of a [users, K] block) for K >= 2, so the values are identical;
        with K = 1 numpy reduces the [users, 1] matrix pairwise instead, so callers
        take this path only for max(topk) >= 2."""
        from concurrent.futures import ThreadPoolExecutor
        acc = {m: None for m in self.metrics}

        def one(m, pos_idx, pos_len, codes):
            rows = topk_metric_rows(m.lower(), pos_idx, pos_len, codes)
            a = acc[m]
            if a is not None:
                rows = np.concatenate([a, rows])
            acc[m] = np.add.reduce(rows, axis=0, keepdims=True)
        with ThreadPoolExecutor(min(len(self.metrics), 8)) as ex:
            for pos_idx, pos_len in chunks:
                codes = pattern_codes(pos_idx) if uses_patterns(pos_idx) else None
                list(ex.map(lambda m: one(m, pos_idx, pos_len, codes), self.metrics))
        if n_users == 0 or any(acc[m] is None for m in self.metrics):
            return self.evaluate_pos_idx(np.zeros((0, max(self.topk)), dtype=bool),
                                         np.zeros(0, dtype=np.int64))
        out = {}
        for m in self.metrics:
            v = acc[m][0] / n_users
            for k in self.topk:
                out[f'{m}@{k}'] = round(v[k - 1], self.precision)
        return out


class LossEvaluator(IndividualEvaluator):

    def __init__(self, config, metrics):
        super().__init__(config, metrics)
        self.label_field = config['LABEL_FIELD']

    def collect(self, interaction, pred_scores):
        trues = interaction[self.label_field].to(pred_scores.device)
        assert len(trues) == len(pred_scores)
        return self.get_score_matrix(trues.float(), pred_scores.float())

    def evaluate(self, batch_matrix_list, *args):
        concat = torch.cat(batch_matrix_list, dim=0).cpu().numpy()
        trues, preds = concat[:, 0], concat[:, 1]
        return {m: round(metrics_dict[m.lower()](trues, preds), self.precision)
                for m in self.metrics}


metric_eval_bind = [(topk_metrics, TopKEvaluator), (loss_metrics, LossEvaluator)]
