"""Negative-sampling loader mixins (mirror of recbole/data/dataloader/neg_sample_mixin.py:19-140).

`NegSampleMixin` stores the sampler and its arguments and adapts the batch size at
setup; `NegSampleByMixin` fixes the batch layout of `by`-N sampling: `times` = N
(pairwise: one row per (positive, negative), the negatives under the `neg_` prefix of
every item feature) or 1 + N (pointwise: the positive row plus N labelled negative
rows). Subclasses supply the abstract hooks below, as in the reference.
"""
from recbole_amd.data.dataloader.abstract_dataloader import AbstractDataLoader
from recbole_amd.utils import DataLoaderType, EvaluatorType, FeatureSource, FeatureType, InputType


def _hook(name):
    """An abstract hook of the reference's mixins: raises until a loader supplies it."""
    def missing(self, *args):
        raise NotImplementedError(f'Method [{name}] should be implemented.')
    return missing


class NegSampleMixin(AbstractDataLoader):
    dl_type = DataLoaderType.NEGSAMPLE
    _STRATEGIES = ('by', 'full')

    def __init__(self, config, dataset, sampler, neg_sample_args, batch_size=1,
                 dl_format=InputType.POINTWISE, shuffle=False):
        strategy = neg_sample_args['strategy']
        if strategy not in self._STRATEGIES:
            raise ValueError(f"Neg_sample strategy [{strategy}] has not been implemented.")
        self.sampler, self.neg_sample_args = sampler, neg_sample_args
        super().__init__(config, dataset, batch_size=batch_size, dl_format=dl_format,
                         shuffle=shuffle)

    def setup(self):
        self._batch_size_adaptation()

    _batch_size_adaptation = _hook('batch_size_adaptation')
    _neg_sampling = _hook('neg_sampling')
    get_pos_len_list = _hook('get_pos_len_list')
    get_user_len_list = _hook('get_user_len_list')


class NegSampleByMixin(NegSampleMixin):
    """`by`-N sampling: the batch layout (times, label or neg_ fields) per dl_format."""

    def __init__(self, config, dataset, sampler, neg_sample_args, batch_size=1,
                 dl_format=InputType.POINTWISE, shuffle=False):
        if neg_sample_args['strategy'] != 'by':
            raise ValueError('neg_sample strategy in GeneralInteractionBasedDataLoader() should be `by`')
        evaluating = sampler.phase != 'train'
        self.user_inter_in_one_batch = evaluating and config['eval_type'] != EvaluatorType.INDIVIDUAL
        self.neg_sample_by = neg_sample_args['by']
        layouts = {InputType.POINTWISE: self._layout_point_wise,
                   InputType.PAIRWISE: self._layout_pair_wise}
        if dl_format not in layouts:
            raise ValueError(f'`neg sampling by` with dl_format [{dl_format}] not been implemented.')
        layouts[dl_format](config, dataset)
        super().__init__(config, dataset, sampler, neg_sample_args, batch_size=batch_size,
                         dl_format=dl_format, shuffle=shuffle)

    def _layout_point_wise(self, config, dataset):
        # the positive row and N negative rows, told apart by a float label field
        self.times = self.neg_sample_by + 1
        self.sampling_func = self._neg_sample_by_point_wise_sampling
        self.label_field = config['LABEL_FIELD']
        dataset.set_field_property(self.label_field, FeatureType.FLOAT, FeatureSource.INTERACTION, 1)

    def _layout_pair_wise(self, config, dataset):
        # one row per (positive, negative): every item feature again under the neg_ prefix
        self.times = self.neg_sample_by
        self.sampling_func = self._neg_sample_by_pair_wise_sampling
        self.neg_prefix = config['NEG_PREFIX']
        iid = config['ITEM_ID_FIELD']
        self.neg_item_id = self.neg_prefix + iid
        item_cols = [iid] if dataset.item_feat is None else list(dataset.item_feat.columns)
        for c in item_cols:
            dataset.copy_field_property(self.neg_prefix + c, c)

    _neg_sample_by_pair_wise_sampling = _hook('neg_sample_by_pair_wise_sampling')
    _neg_sample_by_point_wise_sampling = _hook('neg_sample_by_point_wise_sampling')
