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
from torch.nn.utils.rnn import pad_sequence


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
        rows = torch.split(scores_tensor, list(user_len_list), dim=0)
        mat = pad_sequence(rows, batch_first=True, padding_value=-np.inf)
        width = max(self.topk)
        if mat.shape[1] < width:
            wide = torch.full((mat.shape[0], width), -np.inf, device=mat.device)
            wide[:, :mat.shape[1]] = mat
            mat = wide
        return mat

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
