"""case_study.full_sort_scores / full_sort_topk (case_study.py:22-88): the K6 top-K
agrees with torch.topk of the masked score matrix (scores within fp32 rounding of
the two score kernels' accumulation orders; ids identical where scores are not
tied), for a general (BPR, history masked) and a sequential (SASRec) loader."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _check(model, test, uids, k=10):
    from recbole_amd.utils.case_study import full_sort_scores, full_sort_topk
    sc = full_sort_scores(uids, model, test)
    ref_s, ref_i = torch.topk(sc, k)
    got_s, got_i = full_sort_topk(uids, model, test, k)
    assert got_s.shape == ref_s.shape
    torch.testing.assert_close(got_s, ref_s, rtol=1e-5, atol=1e-6)
    gap = (ref_s[:, :-1] - ref_s[:, 1:]).abs().min(dim=1).values.cpu()
    clear = gap > 1e-5
    assert clear.float().mean() > 0.5
    assert torch.equal(got_i.cpu()[clear], ref_i.cpu()[clear])
    assert torch.isinf(sc[:, 0]).all()


def test_case_study_bpr(tmp_path):
    from tests.test_gpu_e2e import _pipeline
    from recbole_amd.trainer import Trainer
    config, train, valid, test, model = _pipeline(tmp_path, epochs=1)
    Trainer(config, model)._train_epoch(train, 0)
    uids = test.uid_list[::3]
    _check(model, test, uids)
    from recbole_amd.utils.case_study import full_sort_scores
    sc = full_sort_scores(uids, model, test)
    r = 0
    h = test.hist_cols[test.hist_ptr[r * 3 * 0]:test.hist_ptr[1]]
    assert torch.isinf(sc[0, torch.as_tensor(h.astype(np.int64))]).all()


def test_case_study_sasrec(tmp_path):
    from tests.test_gpu_sasrec import _pipeline
    config, train, valid, test, model = _pipeline(tmp_path)
    uids = np.unique(test.uid_list.cpu().numpy())[::2]
    _check(model, test, uids)
