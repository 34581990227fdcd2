"""Batch container (mirror of recbole/data/interaction.py:19-347).

A dict of equal-length tensors. When the tensors live on the GPU, row
selections (slicing is a view; fancy indexing / shuffle / sort reorders) run
through the K1 gather kernel (recbole_amd/csrc/gather.hip) instead of a host
copy, so the train loaders keep their columns resident in HBM.
"""
from __future__ import annotations

import numpy as np
import torch


def _take(t: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
    if t.is_cuda:
        from recbole_amd import ops
        idx = index.to(device=t.device, dtype=torch.int64)
        return ops.gather_rows(t.contiguous(), idx)
    return t[index]


class Interaction(object):

    def __init__(self, interaction, pos_len_list=None, user_len_list=None):
        self.interaction = interaction
        self.pos_len_list = self.user_len_list = None
        self.set_additional_info(pos_len_list, user_len_list)
        for k in self.interaction:
            if not isinstance(self.interaction[k], torch.Tensor):
                raise ValueError(f'Interaction [{interaction}] should only contains torch.Tensor')
        self.length = -1
        for k in self.interaction:
            self.length = max(self.length, self.interaction[k].shape[0])

    def set_additional_info(self, pos_len_list=None, user_len_list=None):
        self.pos_len_list = pos_len_list
        self.user_len_list = user_len_list
        if (self.pos_len_list is None) ^ (self.user_len_list is None):
            raise ValueError('pos_len_list and user_len_list should be both None or valued.')

    def __iter__(self):
        return self.interaction.__iter__()

    def __getitem__(self, index):
        if isinstance(index, str):
            return self.interaction[index]
        if isinstance(index, (np.ndarray, list)):
            index = torch.as_tensor(np.asarray(index))
        ret = {}
        for k in self.interaction:
            if isinstance(index, torch.Tensor) and index.dim() > 0:
                if index.dtype == torch.bool:
                    index = index.nonzero().view(-1)
                ret[k] = _take(self.interaction[k], index)
            else:
                ret[k] = self.interaction[k][index]
        return Interaction(ret)

    def __contains__(self, item):
        return item in self.interaction

    def __len__(self):
        return self.length

    def __str__(self):
        info = [f'The batch_size of interaction: {self.length}']
        for k in self.interaction:
            t = self.interaction[k]
            info.append(f'    {k}, {t.shape}, {t.device.type}, {t.dtype}')
        return '\n'.join(info) + '\n'

    __repr__ = __str__

    @property
    def columns(self):
        return list(self.interaction.keys())

    def to(self, device, selected_field=None):
        ret = {}
        keys = self.interaction.keys() if selected_field is None else (
            [selected_field] if isinstance(selected_field, str) else selected_field)
        keys = set(keys)
        for k in self.interaction:
            t = self.interaction[k]
            ret[k] = t.to(device, non_blocking=True) if k in keys else t
        return Interaction(ret, self.pos_len_list, self.user_len_list)

    def cpu(self):
        return Interaction({k: t.cpu() for k, t in self.interaction.items()},
                           self.pos_len_list, self.user_len_list)

    def numpy(self):
        return {k: t.cpu().numpy() for k, t in self.interaction.items()}

    def repeat(self, sizes):
        ret = {}
        for k, t in self.interaction.items():
            ret[k] = t.repeat(sizes) if t.dim() == 1 else t.repeat([sizes, 1])
        npl = self.pos_len_list * sizes if self.pos_len_list else None
        nul = self.user_len_list * sizes if self.user_len_list else None
        return Interaction(ret, npl, nul)

    def repeat_interleave(self, repeats, dim=0):
        ret = {k: t.repeat_interleave(repeats, dim=dim) for k, t in self.interaction.items()}
        npl = list(np.multiply(self.pos_len_list, repeats)) if self.pos_len_list else None
        nul = list(np.multiply(self.user_len_list, repeats)) if self.user_len_list else None
        return Interaction(ret, npl, nul)

    def update(self, new_inter):
        for k in new_inter.interaction:
            self.interaction[k] = new_inter.interaction[k]
        if new_inter.pos_len_list is not None:
            self.pos_len_list = new_inter.pos_len_list
        if new_inter.user_len_list is not None:
            self.user_len_list = new_inter.user_len_list

    def drop(self, column):
        if column not in self.interaction:
            raise ValueError(f'Column [{column}] is not in [{self}].')
        del self.interaction[column]

    def _reindex(self, index):
        for k in self.interaction:
            self.interaction[k] = _take(self.interaction[k], index)
        if self.pos_len_list is not None:
            self.pos_len_list = self.pos_len_list[index]
        if self.user_len_list is not None:
            self.user_len_list = self.user_len_list[index]

    def shuffle(self):
        """interaction.py:272-276: torch.randperm on the CPU generator (the RNG
        stream the reference consumes), applied to every column."""
        index = torch.randperm(self.length)
        self._reindex(index)
        return index

    def sort(self, by, ascending=True):
        if isinstance(by, str):
            if by not in self.interaction:
                raise ValueError(f'[{by}] is not exist in interaction [{self}].')
            by = [by]
        elif isinstance(by, (list, tuple)):
            for b in by:
                if b not in self.interaction:
                    raise ValueError(f'[{b}] is not exist in interaction [{self}].')
        else:
            raise TypeError(f'Wrong type of by [{by}].')
        if isinstance(ascending, bool):
            ascending = [ascending]
        elif isinstance(ascending, (list, tuple)):
            for a in ascending:
                if not isinstance(a, bool):
                    raise TypeError(f'Wrong type of ascending [{ascending}].')
        else:
            raise TypeError(f'Wrong type of ascending [{ascending}].')
        if len(by) != len(ascending):
            if len(ascending) == 1:
                ascending = ascending * len(by)
            else:
                raise ValueError(f'by [{by}] and ascending [{ascending}] should have same length.')
        for b, a in zip(by[::-1], ascending[::-1]):
            col = self.interaction[b].cpu().numpy()
            index = np.argsort(col, kind='stable')
            if not a:
                index = index[::-1].copy()
            self._reindex(torch.as_tensor(index))

    def add_prefix(self, prefix):
        self.interaction = {prefix + k: v for k, v in self.interaction.items()}


def cat_interactions(interactions):
    if not isinstance(interactions, (list, tuple)):
        raise TypeError(f'Interactions [{interactions}] should be list or tuple.')
    if len(interactions) == 0:
        raise ValueError(f'Interactions [{interactions}] should have some interactions.')
    cols = set(interactions[0].columns)
    for inter in interactions:
        if cols != set(inter.columns):
            raise ValueError(f'Interactions [{interactions}] should have some interactions.')
    return Interaction({c: torch.cat([inter[c] for inter in interactions]) for c in cols})
