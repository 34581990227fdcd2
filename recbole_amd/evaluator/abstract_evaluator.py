"""Evaluator base classes (mirror of recbole/evaluator/abstract_evaluator.py:21-140).

`BaseEvaluator` holds the metric list, whether the eval setting is `full`, and the
rounding precision; the `collect` / `evaluate` / `_calculate_metrics` protocol is
abstract. `GroupedEvaluator` turns a batch's flat score vector into a per-user score
matrix — a plain view for full ranking, per-user rows padded with -inf (to at least
max(topk) columns) for sampled ranking. `IndividualEvaluator` pairs labels with scores
for the loss metrics and refuses full ranking, as the reference does.
"""
import numpy as np
import torch


class BaseEvaluator(object):

    def __init__(self, config, metrics):
        self.metrics = metrics
        self.full = ('full' in config['eval_setting'])
        self.precision = config['metric_decimal_place']

    def collect(self, *args):
        raise NotImplementedError

    def evaluate(self, *args):
        raise NotImplementedError

    def _calculate_metrics(self, *args):
        raise NotImplementedError


class GroupedEvaluator(BaseEvaluator):
    """Metrics computed per user, then averaged (top-K). Subclasses set `self.topk`."""

    def sample_collect(self, scores_tensor, user_len_list):
        # one scatter into a -inf matrix: user u's j-th score lands at (u, j); the width
        # covers the longest user and at least max(topk) columns
        lens = torch.as_tensor(list(user_len_list), dtype=torch.long,
                               device=scores_tensor.device)
        width = max(int(lens.max()) if lens.numel() else 0, max(self.topk))
        out = scores_tensor.new_full((lens.numel(), width), -np.inf)
        owner = torch.repeat_interleave(torch.arange(lens.numel(), device=lens.device), lens)
        first = torch.cumsum(lens, 0) - lens
        col = torch.arange(owner.numel(), device=lens.device) - first[owner]
        out[owner, col] = scores_tensor.reshape(-1)
        return out

    def full_sort_collect(self, scores_tensor, user_len_list):
        return scores_tensor.view(len(user_len_list), -1)

    def get_score_matrix(self, scores_tensor, user_len_list):
        if self.full:
            return self.full_sort_collect(scores_tensor, user_len_list)
        return self.sample_collect(scores_tensor, user_len_list)


class IndividualEvaluator(BaseEvaluator):
    """Metrics over all (label, score) pairs regardless of user (AUC, LogLoss, ...)."""

    def __init__(self, config, metrics):
        super().__init__(config, metrics)
        self._check_args()

    def sample_collect(self, true_scores, pred_scores):
        return torch.stack((true_scores, pred_scores.detach()), dim=1)

    def full_sort_collect(self, true_scores, pred_scores):
        raise NotImplementedError('full sort can\'t use IndividualEvaluator')

    def get_score_matrix(self, true_scores, pred_scores):
        if self.full:
            return self.full_sort_collect(true_scores, pred_scores)
        return self.sample_collect(true_scores, pred_scores)

    def _check_args(self):
        if self.full:
            raise NotImplementedError('full sort can\'t use IndividualEvaluator')
