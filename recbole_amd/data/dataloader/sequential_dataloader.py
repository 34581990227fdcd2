"""Sequential loaders (mirror of recbole/data/dataloader/sequential_dataloader.py:24-370).

A sample is (history window, target row) of SequentialDataset. Instead of
materialising every augmented sequence up front (the reference's
pre_processed_data, :73-127), the loader keeps the index arrays (target row,
window start, window length) — resident in HBM when the model runs on the GPU —
and builds each batch's `<field>_list` columns with the window-gather kernel and
its target-row columns with the K1 gather. The per-epoch shuffle draws the same
torch.randperm the reference's Interaction.shuffle draws (interaction.py:272-276).

Build extension: with loss_type 'SSM' (sampled softmax, SASRec on the C3
configuration) the pairwise loader attaches the `neg_sample_num` negatives of a
batch as neg_item_id [num * B] (the sampler's j*B + k layout) without repeating
the positive rows.
"""
from __future__ import annotations

import numpy as np
import torch

from recbole_amd.data.dataloader.abstract_dataloader import AbstractDataLoader
from recbole_amd.data.dataloader.general_dataloader import _loader_device
from recbole_amd.data.dataloader.neg_sample_mixin import NegSampleByMixin, NegSampleMixin
from recbole_amd.data.interaction import Interaction, cat_interactions
from recbole_amd.utils import DataLoaderType, FeatureSource, FeatureType, InputType


class SequentialDataLoader(AbstractDataLoader):
    dl_type = DataLoaderType.ORIGIN

    def __init__(self, config, dataset, batch_size=1, dl_format=InputType.POINTWISE,
                 shuffle=False):
        self.uid_field = dataset.uid_field
        self.iid_field = dataset.iid_field
        self.time_field = dataset.time_field
        self.max_item_list_len = config['MAX_ITEM_LIST_LENGTH']
        list_suffix = config['LIST_SUFFIX']
        self.list_fields = {}
        for field in dataset.inter_feat:
            if field == self.uid_field:
                continue
            list_field = field + list_suffix
            self.list_fields[field] = list_field
            setattr(self, f'{field}_list_field', list_field)
            ftype = dataset.field2type[field]
            if ftype in (FeatureType.TOKEN_SEQ, FeatureType.FLOAT_SEQ):
                raise NotImplementedError('sequence-valued fields inside item lists are not '
                                          'part of this build')
            list_ftype = FeatureType.TOKEN_SEQ if ftype == FeatureType.TOKEN else \
                FeatureType.FLOAT_SEQ
            dataset.set_field_property(list_field, list_ftype, FeatureSource.INTERACTION,
                                       self.max_item_list_len)
        self.item_list_length_field = config['ITEM_LIST_LENGTH_FIELD']
        dataset.set_field_property(self.item_list_length_field, FeatureType.TOKEN,
                                   FeatureSource.INTERACTION, 1)
        self.device = _loader_device(config)
        if self.device is not None:
            dataset.to_device(self.device)
        dev = self.device or 'cpu'
        T = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.int64), device=dev)
        self.uid_list = T(dataset.uid_list)
        self.item_list_start = T(dataset.item_list_start)
        self.item_list_length = T(dataset.item_list_length)
        self.target_index = T(dataset.target_index)
        self._list_cols = None
        super().__init__(config, dataset, batch_size=batch_size, dl_format=dl_format,
                         shuffle=shuffle)

    @property
    def pr_end(self):
        return len(self.uid_list)

    def _shuffle(self):
        perm = torch.randperm(self.pr_end)          # the reference's RNG draw
        idx = perm.to(self.uid_list.device)
        self.uid_list = self.uid_list[idx]
        self.item_list_start = self.item_list_start[idx]
        self.item_list_length = self.item_list_length[idx]
        self.target_index = self.target_index[idx]

    def _next_batch_data(self):
        cur = self.augmentation(slice(self.pr, self.pr + self.step))
        self.pr += self.step
        return cur

    def _columns(self):
        """Source columns of the list fields: int64 tokens, float64 floats (the
        reference allocates list fields as int64 / float64, :112-118)."""
        if self._list_cols is None:
            inter = self.dataset.inter_feat
            cols = {}
            for field in self.list_fields:
                t = inter[field]
                t = t.to(torch.int64) if not t.is_floating_point() else t.to(torch.float64)
                cols[field] = t.contiguous()
            self._list_cols = cols
        return self._list_cols

    def augmentation(self, index):
        """Batch of samples `index` (sequential_dataloader.py:95-127)."""
        start = self.item_list_start[index].contiguous()
        length = self.item_list_length[index].contiguous()
        target = self.target_index[index].contiguous()
        L = self.max_item_list_len
        new = self.dataset.inter_feat[target]
        cols = {self.item_list_length_field: length.clone()}
        for field, col in self._columns().items():
            lf = self.list_fields[field]
            if col.is_cuda:
                from recbole_amd import ops
                cols[lf] = ops.window_gather(col, start, length, L)
            else:
                pos = start.unsqueeze(1) + torch.arange(L).unsqueeze(0)
                valid = torch.arange(L).unsqueeze(0) < length.unsqueeze(1)
                vals = col[pos.clamp(max=max(len(col) - 1, 0))]
                cols[lf] = torch.where(valid, vals, torch.zeros((), dtype=col.dtype))
        new.update(Interaction(cols))
        return new


class SequentialNegSampleDataLoader(NegSampleByMixin, SequentialDataLoader):
    """sequential_dataloader.py:130-262."""

    def __init__(self, config, dataset, sampler, neg_sample_args, batch_size=1,
                 dl_format=InputType.POINTWISE, shuffle=False):
        self.no_repeat = (config['loss_type'] == 'SSM' and sampler.phase == 'train')
        super().__init__(config, dataset, sampler, neg_sample_args, batch_size=batch_size,
                         dl_format=dl_format, shuffle=shuffle)

    def _batch_size_adaptation(self):
        if self.no_repeat:
            self.step = self.batch_size
            return
        batch_num = max(self.batch_size // self.times, 1)
        self.step = batch_num
        self.upgrade_batch_size(batch_num * self.times)

    def _next_batch_data(self):
        cur = self.augmentation(slice(self.pr, self.pr + self.step))
        cur = self._neg_sampling(cur)
        self.pr += self.step
        if self.user_inter_in_one_batch:
            n = len(cur[self.uid_field]) // self.times
            pos_len_list = np.ones(n, dtype=np.int64)
            cur.set_additional_info(list(pos_len_list), list(pos_len_list * self.times))
        return cur

    def _neg_sampling(self, data):
        if self.user_inter_in_one_batch:
            parts = []
            for i in range(len(data[self.uid_field])):
                uids = data[self.uid_field][i:i + 1]
                neg_iids = self.sampler.sample_by_user_ids(uids, self.neg_sample_by)
                parts.append(self.sampling_func(data[i:i + 1], neg_iids))
            return cat_interactions(parts)
        uids = data[self.uid_field]
        neg_iids = self.sampler.sample_by_user_ids(uids, self.neg_sample_by)
        return self.sampling_func(data, neg_iids)

    def _neg_sample_by_pair_wise_sampling(self, data, neg_iids):
        new = data if self.no_repeat else data.repeat(self.times)
        new.update(Interaction({self.neg_item_id: neg_iids.to(new[self.iid_field].device)}))
        return new

    def _neg_sample_by_point_wise_sampling(self, data, neg_iids):
        n = len(data[self.uid_field])
        new = data.repeat(self.times)
        new[self.iid_field][n:] = neg_iids.to(new[self.iid_field].device)
        labels = torch.zeros(n * self.times, device=new[self.iid_field].device)
        labels[:n] = 1.0
        new.update(Interaction({self.label_field: labels}))
        return new

    def get_pos_len_list(self):
        return np.ones(self.pr_end, dtype=np.int64)

    def get_user_len_list(self):
        return np.full(self.pr_end, self.times)


class SequentialFullDataLoader(NegSampleMixin, SequentialDataLoader):
    """sequential_dataloader.py:265-370: every sample ranked against all items;
    no history mask, the target moved to column 0 by the swap arrays."""
    dl_type = DataLoaderType.FULL

    def _batch_size_adaptation(self):
        pass

    def _shuffle(self):
        self.logger.warning("SequentialFullDataLoader can't shuffle")

    def _next_batch_data(self):
        interaction = super()._next_batch_data()
        n = len(interaction[self.iid_field])
        item_num = self.dataset.item_num
        interaction.set_additional_info(np.ones(n, dtype=np.int64), np.full(n, item_num))
        scores_row = torch.arange(n).repeat(2)
        padding_idx = torch.zeros(n, dtype=torch.int64)
        positive_idx = interaction[self.iid_field].cpu()
        scores_col_after = torch.cat((padding_idx, positive_idx))
        scores_col_before = torch.cat((positive_idx, padding_idx))
        return interaction, None, scores_row, scores_col_after, scores_col_before

    def get_pos_len_list(self):
        return np.ones(self.pr_end, dtype=np.int64)

    def get_user_len_list(self):
        return np.full(self.pr_end, self.dataset.item_num)
