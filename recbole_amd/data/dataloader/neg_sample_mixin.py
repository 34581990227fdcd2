"""Negative-sampling loader mixins (mirror of recbole/data/dataloader/neg_sample_mixin.py:19-140).

`NegSampleMixin` stores the sampler and its arguments and adapts the batch size at
setup; `NegSampleByMixin` fixes the batch layout of `by`-N sampling: `times` = N
(pairwise: one row per (positive, negative), the negatives under the `neg_` prefix of
every item feature) or 1 + N (pointwise: the positive row plus N labelled negative
rows). Subclasses supply the abstract hooks below, as in the reference.
"""
from recbole_amd.data.dataloader.abstract_dataloader import AbstractDataLoader
from recbole_amd.utils import DataLoaderType, EvaluatorType, FeatureSource, FeatureType, InputType


class NegSampleMixin(AbstractDataLoader):
    dl_type = DataLoaderType.NEGSAMPLE

    def __init__(self, config, dataset, sampler, neg_sample_args, batch_size=1,
                 dl_format=InputType.POINTWISE, shuffle=False):
        if neg_sample_args['strategy'] not in ['by', 'full']:
            raise ValueError(f"Neg_sample strategy [{neg_sample_args['strategy']}] has not been implemented.")
        self.sampler = sampler
        self.neg_sample_args = neg_sample_args
        super().__init__(config, dataset, batch_size=batch_size, dl_format=dl_format,
                         shuffle=shuffle)

    def setup(self):
        self._batch_size_adaptation()

    def _batch_size_adaptation(self):
        raise NotImplementedError('Method [batch_size_adaptation] should be implemented.')

    def _neg_sampling(self, inter_feat):
        raise NotImplementedError('Method [neg_sampling] should be implemented.')

    def get_pos_len_list(self):
        raise NotImplementedError('Method [get_pos_len_list] should be implemented.')

    def get_user_len_list(self):
        raise NotImplementedError('Method [get_user_len_list] should be implemented.')


class NegSampleByMixin(NegSampleMixin):

    def __init__(self, config, dataset, sampler, neg_sample_args, batch_size=1,
                 dl_format=InputType.POINTWISE, shuffle=False):
        if neg_sample_args['strategy'] != 'by':
            raise ValueError('neg_sample strategy in GeneralInteractionBasedDataLoader() should be `by`')
        self.user_inter_in_one_batch = (sampler.phase != 'train') and (
            config['eval_type'] != EvaluatorType.INDIVIDUAL)
        self.neg_sample_by = neg_sample_args['by']
        if dl_format == InputType.POINTWISE:
            self.times = 1 + self.neg_sample_by
            self.sampling_func = self._neg_sample_by_point_wise_sampling
            self.label_field = config['LABEL_FIELD']
            dataset.set_field_property(self.label_field, FeatureType.FLOAT,
                                       FeatureSource.INTERACTION, 1)
        elif dl_format == InputType.PAIRWISE:
            self.times = self.neg_sample_by
            self.sampling_func = self._neg_sample_by_pair_wise_sampling
            self.neg_prefix = config['NEG_PREFIX']
            iid_field = config['ITEM_ID_FIELD']
            self.neg_item_id = self.neg_prefix + iid_field
            cols = [iid_field] if dataset.item_feat is None else dataset.item_feat.columns
            for c in cols:
                dataset.copy_field_property(self.neg_prefix + c, c)
        else:
            raise ValueError(f'`neg sampling by` with dl_format [{dl_format}] not been implemented.')
        super().__init__(config, dataset, sampler, neg_sample_args, batch_size=batch_size,
                         dl_format=dl_format, shuffle=shuffle)

    def _neg_sample_by_pair_wise_sampling(self, *args):
        raise NotImplementedError('Method [neg_sample_by_pair_wise_sampling] should be implemented.')

    def _neg_sample_by_point_wise_sampling(self, *args):
        raise NotImplementedError('Method [neg_sample_by_point_wise_sampling] should be implemented.')
