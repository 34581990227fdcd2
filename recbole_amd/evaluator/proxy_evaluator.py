"""ProxyEvaluator (mirror of recbole/evaluator/proxy_evaluator.py:19-100)."""
from collections import ChainMap

from recbole_amd.evaluator.evaluators import (TopKEvaluator, group_metrics, individual_metrics,
                                              metric_eval_bind)


class ProxyEvaluator(object):

    def __init__(self, config):
        self.config = config
        self.valid_metrics = ChainMap(group_metrics, individual_metrics)
        self.metrics = config['metrics']
        self._check_args()
        self.evaluators = self.build()

    def build(self):
        out = []
        names = [m.lower() for m in self.metrics]
        for metrics, evaluator in metric_eval_bind:
            used = [m for m in names if m in metrics]
            if used:
                out.append(evaluator(self.config, used))
        return out

    @property
    def topk_evaluator(self):
        for e in self.evaluators:
            if isinstance(e, TopKEvaluator):
                return e
        return None

    def collect(self, interaction, scores):
        return [e.collect(interaction, scores) for e in self.evaluators]

    def merge_batch_result(self, batch_matrix_list):
        d = {}
        for lst in batch_matrix_list:
            for i, v in enumerate(lst):
                d.setdefault(i, []).append(v)
        return d

    def evaluate(self, batch_matrix_list, eval_data):
        md = self.merge_batch_result(batch_matrix_list)
        out = {}
        for i, e in enumerate(self.evaluators):
            out.update(e.evaluate(md[i], eval_data))
        return out

    def _check_args(self):
        if isinstance(self.metrics, (str, list)):
            if isinstance(self.metrics, str):
                if self.metrics[0] == '[':
                    self.metrics = self.metrics[1:]
                if self.metrics[-1] == ']':
                    self.metrics = self.metrics[:-1]
                self.metrics = self.metrics.strip().split(',')
            for m in self.metrics:
                if m.lower() not in self.valid_metrics:
                    raise ValueError(f'There is no metric named {m}!')
        else:
            raise TypeError('metrics must be str or list')
