"""case_study.full_sort_topk (reference case_study.py:73-88) on K6 against an fp64
CPU oracle of the reference sequence (case_study.py:22-70: full_sort_predict
scores, [pad] and history items set to -inf, torch.topk): scores within fp32
rounding of the fp64 ones, and ids identical wherever the oracle's consecutive
scores are separated by more than that rounding (exact ties may order either
way), for a general (BPR, history masked) and a sequential (SASRec) loader."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _oracle_topk(Q, E, hist_rows, k):
    """fp64 scores Q @ E^T, column 0 and (row, item) pairs in hist_rows -inf, top-k."""
    S = Q.double() @ E.double().T
    S[:, 0] = -np.inf
    for r, items in enumerate(hist_rows):
        if len(items):
            S[r, torch.as_tensor(np.asarray(items, dtype=np.int64))] = -np.inf
    return torch.topk(S, k)


def _check(got_s, got_i, ref_s, ref_i, tol=1e-5):
    got_s, got_i = got_s.cpu().double(), got_i.cpu()
    np.testing.assert_allclose(got_s.numpy(), ref_s.numpy(), rtol=tol, atol=tol)
    # ids must agree wherever rank r is separated from its neighbours by more than
    # fp32 rounding in the oracle's order
    sep = torch.ones_like(ref_s, dtype=torch.bool)
    gaps = (ref_s[:, :-1] - ref_s[:, 1:]).abs() > 4 * tol * ref_s[:, :-1].abs().clamp(min=1)
    sep[:, :-1] &= gaps
    sep[:, 1:] &= gaps
    assert sep.float().mean() > 0.9
    assert torch.equal(got_i[sep], ref_i[sep])


def test_case_study_bpr(tmp_path):
    from tests.test_gpu_e2e import _pipeline
    from recbole_amd.trainer import Trainer
    from recbole_amd.utils.case_study import full_sort_topk
    config, train, valid, test, model = _pipeline(tmp_path, epochs=1)
    Trainer(config, model)._train_epoch(train, 0)
    rows = np.arange(0, len(test.uid_list), 3)
    uids = test.uid_list[rows]
    got_s, got_i = full_sort_topk(uids, model, test, 10)
    U = model.user_embedding.weight.detach().cpu()[torch.as_tensor(np.asarray(uids))]
    E = model.item_embedding.weight.detach().cpu()
    hist = [test.hist_cols[test.hist_ptr[r]:test.hist_ptr[r + 1]] for r in rows]
    ref_s, ref_i = _oracle_topk(U, E, hist, 10)
    _check(got_s, got_i, ref_s, ref_i)
    # history items never appear in the top-K
    for r, h in enumerate(hist):
        assert not set(got_i[r].tolist()) & set(np.asarray(h).tolist())


def test_case_study_sasrec(tmp_path):
    from tests.test_gpu_sasrec import _oracle, _pipeline
    from recbole_amd.utils.case_study import _select, full_sort_topk
    config, train, valid, test, model = _pipeline(tmp_path)
    model.eval()
    uids = np.unique(test.uid_list.cpu().numpy())[::2]
    got_s, got_i = full_sort_topk(uids, model, test, 10)
    _, rows, inter = _select(uids, test)
    ref = _oracle(model).eval()
    with torch.no_grad():
        Q = ref.forward(inter[model.ITEM_SEQ].cpu(), inter[model.ITEM_SEQ_LEN].cpu())
    E = model.item_embedding.weight.detach().cpu()
    ref_s, ref_i = _oracle_topk(Q, E, [[] for _ in range(len(rows))], 10)
    _check(got_s, got_i, ref_s, ref_i, tol=2e-5)
