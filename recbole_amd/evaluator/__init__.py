from recbole_amd.evaluator.abstract_evaluator import (BaseEvaluator, GroupedEvaluator,
                                                      IndividualEvaluator)
from recbole_amd.evaluator.evaluators import (LossEvaluator, TopKEvaluator, group_metrics,
                                              individual_metrics, loss_metrics, topk_metrics)
from recbole_amd.evaluator.metrics import metrics_dict
from recbole_amd.evaluator.proxy_evaluator import ProxyEvaluator

__all__ = ['BaseEvaluator', 'GroupedEvaluator', 'IndividualEvaluator', 'ProxyEvaluator',
           'TopKEvaluator', 'LossEvaluator', 'metrics_dict', 'group_metrics',
           'individual_metrics', 'topk_metrics', 'loss_metrics']
