"""Case study API (mirror of recbole/utils/case_study.py:22-88) on the K6 scorer.

full_sort_scores returns the reference's [n, n_items] score matrix (FP32 MFMA
score kernel, pad column and history set to -inf). full_sort_topk ranks the users
with K6 directly when the model exposes the fused scorer hooks — no score matrix is
formed — and otherwise takes torch.topk of full_sort_scores like the reference.
Users are taken in the loader's order (the reference selects them with np.isin over
the loader's user list). Tied scores may come back in a different order than
torch.topk's (which is unspecified).
"""
import numpy as np
import torch

from recbole_amd import ops
from recbole_amd.data.dataloader.general_dataloader import GeneralFullDataLoader
from recbole_amd.data.dataloader.sequential_dataloader import SequentialFullDataLoader


def _select(uid_series, test_data):
    """(kind, rows of the loader, input interaction)."""
    uid_field = test_data.dataset.uid_field
    if isinstance(test_data, GeneralFullDataLoader):
        rows = np.flatnonzero(np.isin(test_data.uid_list, np.asarray(uid_series)))
        return 'general', rows, test_data.user_df[torch.as_tensor(rows)]
    if isinstance(test_data, SequentialFullDataLoader):
        uids = test_data.uid_list.cpu().numpy()
        rows = np.flatnonzero(np.isin(uids, np.asarray(uid_series)))
        return 'sequential', rows, test_data.augmentation(
            torch.as_tensor(rows, device=test_data.uid_list.device))
    raise NotImplementedError(f'case study of {type(test_data).__name__}')


def _history(test_data, rows):
    hp, hc = test_data.hist_ptr, test_data.hist_cols
    r = np.concatenate([np.full(hp[x + 1] - hp[x], i) for i, x in enumerate(rows)]) \
        if len(rows) else np.zeros(0, np.int64)
    c = np.concatenate([hc[hp[x]:hp[x + 1]] for x in rows]) if len(rows) else \
        np.zeros(0, np.int64)
    return torch.as_tensor(r, dtype=torch.int64), torch.as_tensor(c, dtype=torch.int64)


@torch.no_grad()
def full_sort_scores(uid_series, model, test_data):
    """Scores of all items for each selected user; [pad] and history items -inf
    (case_study.py:22-70)."""
    model.eval()
    dataset = test_data.dataset
    kind, rows, inter = _select(uid_series, test_data)
    dev = next(model.parameters()).device
    inter = inter.to(dev)
    try:
        scores = model.full_sort_predict(inter)
    except NotImplementedError:
        inter = inter.repeat_interleave(dataset.item_num)
        inter.update(test_data.get_item_feature().to(dev).repeat(len(rows)))
        scores = model.predict(inter)
    scores = scores.view(-1, dataset.item_num)
    scores[:, 0] = -np.inf
    if kind == 'general':
        hr, hc = _history(test_data, rows)
        scores[hr.to(dev), hc.to(dev)] = -np.inf
    return scores


@torch.no_grad()
def full_sort_topk(uid_series, model, test_data, k):
    """(topk_scores, topk_index) of every selected user (case_study.py:73-88)."""
    fused = (hasattr(model, 'fused_user_vectors') or hasattr(model, 'fused_query_vectors'))
    if not fused or k > 50:
        return torch.topk(full_sort_scores(uid_series, model, test_data), k)
    model.eval()
    kind, rows, inter = _select(uid_series, test_data)
    EI = model.fused_item_table().contiguous()
    dev = EI.device
    if kind == 'general':
        if not hasattr(model, 'fused_user_vectors'):
            return torch.topk(full_sort_scores(uid_series, model, test_data), k)
        uids = torch.as_tensor(test_data.uid_list[rows], dtype=torch.int64, device=dev)
        Uq = model.fused_user_vectors(uids).contiguous()
        hp = test_data.hist_ptr
        ptr = np.r_[0, np.cumsum(hp[rows + 1] - hp[rows])].astype(np.int64)
        _, hc = _history(test_data, rows)
        hist_cols = hc.to(torch.int32) if len(hc) else torch.zeros(1, dtype=torch.int32)
        o = ops.fullsort_topk(Uq, EI, k, hist_ptr=torch.as_tensor(ptr, device=dev),
                              hist_cols=hist_cols.to(dev))
    else:
        if not hasattr(model, 'fused_query_vectors'):
            return torch.topk(full_sort_scores(uid_series, model, test_data), k)
        Uq = model.fused_query_vectors(inter.to(dev)).detach().contiguous()
        o = ops.fullsort_topk(Uq, EI, k)
    return o['scores'], o['ids'].to(torch.int64)
