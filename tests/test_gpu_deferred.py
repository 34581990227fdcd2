"""Deferred K5 schedule on the autograd path (FusedAdam.enable_deferred): the
embedding tables of DeepFM (token table) and SASRec (item table, BPR / SSM
losses) are updated only on the rows a batch touches, with skipped zero-gradient
steps replayed on the next read and at flushes. The result must be bit-identical
to the dense (streamed) Adam over every row — checked over several optimizer
windows, including a window roll-over and an evaluation in between."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(pipeline, tmp_path, mode, steps, window, **over):
    from recbole_amd.trainer import Trainer
    config, train, valid, test, model = pipeline(tmp_path, adam_mode=mode, **over)
    tr = Trainer(config, model)
    deferred = getattr(tr.optimizer, '_deferred', {})
    assert bool(deferred) == (mode == 'deferred')
    for ds in deferred.values():
        ds['window'] = window
    losses = []
    batches = list(train)
    for k in range(steps):
        b = batches[k % len(batches)]
        tr.optimizer.zero_grad()
        loss = model.calculate_loss(b.to(config['device']))
        loss.backward()
        tr.optimizer.step()
        losses.append(loss.item())
        if k == steps // 2:                   # an evaluation in the middle
            with torch.no_grad():
                model.eval()
                model.predict(batches[0].to(config['device']))
                model.train()
    tr.optimizer.flush()
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    st = tr.optimizer.state_dict()['state']
    mom = [(s['exp_avg'].cpu(), s['exp_avg_sq'].cpu()) for _, s in sorted(st.items())]
    return losses, sd, mom


def _compare(a, b):
    la, sa, ma = a
    lb, sb, mb = b
    assert la == lb
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    for (x1, y1), (x2, y2) in zip(ma, mb):
        assert torch.equal(x1, x2) and torch.equal(y1, y2)


def test_deepfm_deferred_bitwise(tmp_path):
    from tests.test_gpu_deepfm import _pipeline
    a = _train(_pipeline, tmp_path, 'deferred', 11, 4, train_batch_size=256)
    b = _train(_pipeline, tmp_path, 'streamed', 11, 4, train_batch_size=256)
    _compare(a, b)


@pytest.mark.parametrize('loss_type,neg', [('BPR', 1), ('SSM', 9)])
def test_sasrec_deferred_bitwise(tmp_path, loss_type, neg):
    from tests.test_gpu_sasrec import _pipeline
    kw = dict(loss_type=loss_type, training_neg_sample_num=neg, train_batch_size=128)
    a = _train(_pipeline, tmp_path, 'deferred', 9, 3, **kw)
    b = _train(_pipeline, tmp_path, 'streamed', 9, 3, **kw)
    _compare(a, b)
