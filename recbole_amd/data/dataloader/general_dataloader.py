"""General-recommendation loaders (mirror of
recbole/data/dataloader/general_dataloader.py:24-378 and
neg_sample_mixin.py:19-140 — the mixins live in
neg_sample_mixin.py, as in the reference).

Train batches are slices of the (shuffled) train table kept resident in HBM;
negatives come from the device walk (K4). The full-sort loader builds, per
evaluated user, the positive and history item lists as CSR with vectorised
numpy (the reference walks every interaction in Python,
general_dataloader.py:300-313) and still yields the reference's 5-tuple
(user_df, (history_row, history_col), swap_row, swap_col_after,
swap_col_before) when iterated; the trainer's fused evaluator consumes the
CSR directly.
"""
from __future__ import annotations

import numpy as np
import torch

from recbole_amd.data.dataloader.abstract_dataloader import AbstractDataLoader
from recbole_amd.data.dataloader.neg_sample_mixin import NegSampleByMixin, NegSampleMixin
from recbole_amd.data.interaction import Interaction, cat_interactions
from recbole_amd.utils import DataLoaderType, InputType


def _loader_device(config):
    dev = config['device']
    return dev if dev is not None and torch.device(dev).type == 'cuda' else None


class GeneralDataLoader(AbstractDataLoader):
    dl_type = DataLoaderType.ORIGIN

    @property
    def pr_end(self):
        return len(self.dataset)

    def _shuffle(self):
        self.dataset.shuffle()

    def _next_batch_data(self):
        cur = self.dataset[self.pr:self.pr + self.step]
        self.pr += self.step
        return cur


class GeneralNegSampleDataLoader(NegSampleByMixin):
    """general_dataloader.py:132-265."""

    def __init__(self, config, dataset, sampler, neg_sample_args, batch_size=1,
                 dl_format=InputType.POINTWISE, shuffle=False):
        self.uid_field = dataset.uid_field
        self.iid_field = dataset.iid_field
        self.uid_list, self.uid2index, self.uid2items_num = None, None, None
        self.device = _loader_device(config)
        super().__init__(config, dataset, sampler, neg_sample_args, batch_size=batch_size,
                         dl_format=dl_format, shuffle=shuffle)
        if self.device is not None and not self.user_inter_in_one_batch:
            # train table resident in HBM; batches are device slices
            dataset.to_device(self.device)
            self.sampler.to_device(self.device)

    def setup(self):
        if self.user_inter_in_one_batch:
            self.dataset.sort(by=self.uid_field, ascending=True)
            uids = self.dataset.inter_feat[self.uid_field].cpu().numpy()
            n_users = self.dataset.user_num
            if len(uids):
                starts = np.flatnonzero(np.r_[True, uids[1:] != uids[:-1]])
                ends = np.r_[starts[1:], len(uids)]
                self.uid_list = uids[starts]
            else:
                starts = ends = self.uid_list = np.zeros(0, dtype=np.int64)
            self.uid2start = np.zeros(n_users, dtype=np.int64)
            self.uid2items_num = np.zeros(n_users, dtype=np.int64)
            self.uid2start[self.uid_list] = starts
            self.uid2items_num[self.uid_list] = ends - starts
        self._batch_size_adaptation()

    def _batch_size_adaptation(self):
        if self.user_inter_in_one_batch:
            inters_num = sorted(self.uid2items_num * self.times, reverse=True)
            batch_num = 1
            new_batch_size = inters_num[0]
            for i in range(1, len(inters_num)):
                if new_batch_size + inters_num[i] > self.batch_size:
                    break
                batch_num = i + 1
                new_batch_size += inters_num[i]
            self.step = batch_num
            self.upgrade_batch_size(new_batch_size)
        else:
            batch_num = max(self.batch_size // self.times, 1)
            self.step = batch_num
            self.upgrade_batch_size(batch_num * self.times)

    @property
    def pr_end(self):
        return len(self.uid_list) if self.user_inter_in_one_batch else len(self.dataset)

    def _shuffle(self):
        if self.user_inter_in_one_batch:
            np.random.shuffle(self.uid_list)
        else:
            self.dataset.shuffle()

    def _next_batch_data(self):
        if self.user_inter_in_one_batch:
            uid_list = self.uid_list[self.pr:self.pr + self.step]
            parts = []
            for uid in uid_list:
                s = int(self.uid2start[uid])
                parts.append(self._neg_sampling(self.dataset[s:s + int(self.uid2items_num[uid])]))
            cur = cat_interactions(parts)
            pos_len_list = self.uid2items_num[uid_list]
            cur.set_additional_info(list(pos_len_list), list(pos_len_list * self.times))
            self.pr += self.step
            return cur
        cur = self._neg_sampling(self.dataset[self.pr:self.pr + self.step])
        self.pr += self.step
        return cur

    def _neg_sampling(self, inter_feat):
        uids = inter_feat[self.uid_field]
        neg_iids = self.sampler.sample_by_user_ids(uids, self.neg_sample_by)
        return self.sampling_func(inter_feat, neg_iids)

    def _neg_sample_by_pair_wise_sampling(self, inter_feat, neg_iids):
        inter_feat = inter_feat.repeat(self.times)
        neg = Interaction({self.iid_field: neg_iids})
        neg = self.dataset.join(neg)
        neg.add_prefix(self.neg_prefix)
        inter_feat.update(neg)
        return inter_feat

    def _neg_sample_by_point_wise_sampling(self, inter_feat, neg_iids):
        n = len(inter_feat)
        new = inter_feat.repeat(self.times)
        new[self.iid_field][n:] = neg_iids.to(new[self.iid_field].device)
        new = self.dataset.join(new)
        labels = torch.zeros(n * self.times, device=new[self.iid_field].device)
        labels[:n] = 1.0
        new.update(Interaction({self.label_field: labels}))
        return new

    def get_pos_len_list(self):
        return self.uid2items_num[self.uid_list]

    def get_user_len_list(self):
        return self.uid2items_num[self.uid_list] * self.times


def _csr_difference(ptr_a, cols_a, ptr_b, cols_b):
    """Row-wise sorted set difference A - B of two CSRs over the same rows."""
    n = len(ptr_a) - 1
    ra = np.repeat(np.arange(n), np.diff(ptr_a))
    rb = np.repeat(np.arange(n), np.diff(ptr_b))
    mul = int(max(cols_a.max() if len(cols_a) else 0, cols_b.max() if len(cols_b) else 0)) + 1
    ka = ra.astype(np.int64) * mul + cols_a
    kb = rb.astype(np.int64) * mul + cols_b
    # rows ascending and each row's columns ascending: ka and kb are sorted, so
    # membership is one binary search per element of A
    if len(kb):
        at = np.minimum(np.searchsorted(kb, ka), len(kb) - 1)
        keep = kb[at] != ka
    else:
        keep = np.ones(len(ka), dtype=bool)
    rows, cols = ra[keep], cols_a[keep]
    ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(ptr, rows + 1, 1)
    return np.cumsum(ptr), cols.astype(np.int32)


class GeneralFullDataLoader(NegSampleMixin):
    """general_dataloader.py:268-378."""
    dl_type = DataLoaderType.FULL

    def __init__(self, config, dataset, sampler, neg_sample_args, batch_size=1,
                 dl_format=InputType.POINTWISE, shuffle=False):
        if neg_sample_args['strategy'] != 'full':
            raise ValueError('neg_sample strategy in GeneralFullDataLoader() should be `full`')
        uid_field, iid_field = dataset.uid_field, dataset.iid_field
        user_num = dataset.user_num
        dataset.sort(by=uid_field, ascending=True)
        uids = dataset.inter_feat[uid_field].cpu().numpy().astype(np.int64)
        iids = dataset.inter_feat[iid_field].cpu().numpy().astype(np.int64)
        # positives of this phase per user (sorted, unique)
        order = np.lexsort((iids, uids))
        u, i = uids[order], iids[order]
        if len(u):
            keep = np.r_[True, (u[1:] != u[:-1]) | (i[1:] != i[:-1])]
            u, i = u[keep], i[keep]
        self.uid_list = np.unique(uids)
        rows = np.searchsorted(self.uid_list, u)
        n = len(self.uid_list)
        pos_ptr = np.zeros(n + 1, dtype=np.int64)
        np.add.at(pos_ptr, rows + 1, 1)
        self.pos_ptr = np.cumsum(pos_ptr)
        self.pos_cols = i.astype(np.int32)
        # history = used(phase) - positives, per evaluated user
        up, uc = sampler.used_csr[sampler.phase]
        sel_len = up[self.uid_list + 1] - up[self.uid_list]
        used_ptr = np.r_[0, np.cumsum(sel_len)].astype(np.int64)
        gather = (np.repeat(up[self.uid_list] - used_ptr[:-1], sel_len) +
                  np.arange(used_ptr[-1])) if n else np.zeros(0, dtype=np.int64)
        used_cols = uc[gather] if len(gather) else np.zeros(0, dtype=np.int32)
        self.hist_ptr, self.hist_cols = _csr_difference(used_ptr, used_cols, self.pos_ptr,
                                                        self.pos_cols)
        self.uid2items_num = np.zeros(user_num, dtype=np.int64)
        self.uid2items_num[self.uid_list] = np.diff(self.pos_ptr)
        self.uid2row = np.full(user_num, -1, dtype=np.int64)
        self.uid2row[self.uid_list] = np.arange(n)
        self.user_df = dataset.join(Interaction({uid_field: torch.as_tensor(self.uid_list)}))
        super().__init__(config, dataset, sampler, neg_sample_args, batch_size=batch_size,
                         dl_format=dl_format, shuffle=shuffle)

    def _batch_size_adaptation(self):
        batch_num = max(self.batch_size // self.dataset.item_num, 1)
        self.step = batch_num
        self.upgrade_batch_size(batch_num * self.dataset.item_num)

    @property
    def pr_end(self):
        return len(self.uid_list)

    def _shuffle(self):
        self.logger.warning("GeneralFullDataLoader can't shuffle")

    def _next_batch_data(self):
        user_df = self.user_df[self.pr:self.pr + self.step]
        cur = self._neg_sampling(user_df, self.pr)
        self.pr += self.step
        return cur

    def _neg_sampling(self, user_df, row0):
        item_num = self.dataset.item_num
        rows = np.arange(row0, row0 + len(user_df))
        pos_len = np.diff(self.pos_ptr)[rows]
        user_df.set_additional_info(pos_len, np.full(len(rows), item_num))
        h_row, h_col, s_row, s_after, s_before = [], [], [], [], []
        for b, r in enumerate(rows):
            hc = self.hist_cols[self.hist_ptr[r]:self.hist_ptr[r + 1]]
            h_row.append(np.full(len(hc), b, dtype=np.int64))
            h_col.append(hc.astype(np.int64))
            pos = self.pos_cols[self.pos_ptr[r]:self.pos_ptr[r + 1]].astype(np.int64)
            pl = len(pos)
            # sorted(set(range(pl)) ^ positives)  (general_dataloader.py:325)
            swap = np.union1d(np.setdiff1d(np.arange(pl), pos), np.setdiff1d(pos, np.arange(pl)))
            s_row.append(np.full(len(swap), b, dtype=np.int64))
            s_after.append(swap)
            s_before.append(swap[::-1])
        cat = lambda xs: torch.as_tensor(np.concatenate(xs) if xs else np.zeros(0, np.int64))
        return (user_df, (cat(h_row), cat(h_col)), cat(s_row), cat(s_after), cat(s_before))

    def get_pos_len_list(self):
        return self.uid2items_num[self.uid_list]

    def get_user_len_list(self):
        return np.full(self.pr_end, self.dataset.item_num)

    def device_csr(self, device):
        """(uids, hist_ptr, hist_cols, pos_ptr, pos_cols) resident on `device`,
        uploaded once per loader (the fused evaluator's inputs; history and
        positives do not change between evaluations)."""
        key = str(device)
        cache = self.__dict__.setdefault('_device_csr', {})
        if key not in cache:
            up = lambda a: torch.as_tensor(a, device=device)
            hist_cols = self.hist_cols if len(self.hist_cols) else np.zeros(1, np.int32)
            cache[key] = (torch.as_tensor(self.uid_list, dtype=torch.int64, device=device),
                          up(self.hist_ptr), up(hist_cols), up(self.pos_ptr), up(self.pos_cols))
        return cache[key]
