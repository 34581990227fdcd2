"""SequentialDataset (mirror of recbole/data/dataset/sequential_dataset.py:19-140).

Same augmentation and leave-one-out split, vectorised: after sorting by
(user, time), every interaction i that is not its user's first becomes a
sample whose history is rows [max(user_start, i - L), i) (the reference's
running seq_start, :72-85) and whose target is row i. The history is kept as
(start, length) index pairs — the sequences themselves are materialised per
batch on the device by the loader (window gather kernel).
"""
import copy

import numpy as np

from recbole_amd.data.dataset.dataset import Dataset


class SequentialDataset(Dataset):

    def prepare_data_augmentation(self):
        """sequential_dataset.py:43-89."""
        if self.uid_field is None or self.time_field is None:
            raise ValueError('sequential datasets need uid_field and time_field')
        max_len = self.config['MAX_ITEM_LIST_LENGTH']
        self.sort(by=[self.uid_field, self.time_field], ascending=True)
        uids = self.inter_feat[self.uid_field].cpu().numpy()
        n = len(uids)
        first = np.r_[True, uids[1:] != uids[:-1]] if n else np.zeros(0, dtype=bool)
        user_start = np.maximum.accumulate(np.where(first, np.arange(n), 0)) if n else \
            np.zeros(0, dtype=np.int64)
        target = np.flatnonzero(~first).astype(np.int64)
        start = np.maximum(user_start[target], target - max_len).astype(np.int64)
        self.uid_list = uids[target]
        self.item_list_start = start
        self.target_index = target
        self.item_list_length = (target - start).astype(np.int64)
        self.mask = np.ones(n, dtype=bool)

    @property
    def item_list_index(self):
        """slice(start, target) per sample, as the reference stores them."""
        return np.array([slice(s, s + n) for s, n in zip(self.item_list_start,
                                                          self.item_list_length)])

    def leave_one_out(self, group_by, leave_one_num=1):
        """sequential_dataset.py:91-112 + dataset.py:1317-1337, vectorised."""
        if group_by is None:
            raise ValueError('Leave one out strategy require a group field.')
        if group_by != self.uid_field:
            raise ValueError('Sequential models require group by user.')
        self.prepare_data_augmentation()
        u = self.uid_list
        m = len(u)
        first = np.r_[True, u[1:] != u[:-1]] if m else np.zeros(0, dtype=bool)
        gid = np.cumsum(first) - 1
        gstart = np.flatnonzero(first)
        gsize = np.diff(np.r_[gstart, m])
        k = np.arange(m) - gstart[gid]                  # position inside the group
        tot = gsize[gid]
        legal = np.minimum(leave_one_num, tot - 1)
        pr = tot - legal
        part = np.where(k < pr, 0, leave_one_num + 1 - legal + (k - pr))
        next_index = [np.flatnonzero(part == p) for p in range(leave_one_num + 1)]
        self._drop_unused_col()
        out = []
        for index in next_index:
            ds = copy.copy(self)
            for field in ['uid_list', 'item_list_start', 'target_index', 'item_list_length']:
                setattr(ds, field, np.array(getattr(ds, field)[index]))
            ds.mask = np.ones(len(self.inter_feat), dtype=bool)
            out.append(ds)
        if leave_one_num >= 2:
            out[0].mask[self.target_index[np.r_[next_index[1], next_index[2]]]] = False
            out[1].mask[self.target_index[next_index[2]]] = False
        elif leave_one_num == 1:
            out[0].mask[self.target_index[next_index[1]]] = False
        return out

    def inter_matrix(self, form='coo', value_field=None):
        """Interactions of this phase only (sequential_dataset.py:114-136)."""
        import scipy.sparse as sp
        keep = np.flatnonzero(self.mask)
        src = self.inter_feat[self.uid_field].cpu().numpy()[keep]
        tgt = self.inter_feat[self.iid_field].cpu().numpy()[keep]
        data = np.ones(len(keep)) if value_field is None else \
            self.inter_feat[value_field].cpu().numpy()[keep]
        mat = sp.coo_matrix((data, (src, tgt)), shape=(self.user_num, self.item_num))
        return mat if form == 'coo' else mat.tocsr()

    def build(self, eval_setting):
        """sequential_dataset.py:138-160: TO ordering and LS split required."""
        self._change_feat_format()
        oa = eval_setting.ordering_args
        if oa['strategy'] == 'shuffle':
            raise ValueError('Ordering strategy `shuffle` is not supported in sequential models.')
        if oa['strategy'] == 'by':
            if oa['field'] != self.time_field:
                raise ValueError('Sequential models require `TO` (time ordering) strategy.')
            if oa['ascending'] is not True:
                raise ValueError('Sequential models require `time_field` to sort in ascending '
                                 'order.')
        sa = eval_setting.split_args
        if sa['strategy'] == 'loo':
            return self.leave_one_out(group_by=eval_setting.group_field,
                                      leave_one_num=sa['leave_one_num'])
        raise ValueError('Sequential models require `loo` (leave one out) split strategy.')
