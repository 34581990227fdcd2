"""The captured generic training step (trainer/graph_step.py GraphedTrainStep):
DeepFM (token + first-order tables on the deferred K5 schedule, MLP / biases
dense) replayed from one HIP graph per batch shape, against the eager step of the
ordinary FusedAdam (host step indices, separate windows) — losses, parameters and
Adam state bit-identical over several graph-mode window roll-overs, a ragged last
batch (eager) and a checkpoint-style flush in between."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(tmp_path, graphed, steps, window):
    from tests.test_gpu_deepfm import _pipeline
    from recbole_amd.trainer import Trainer
    from recbole_amd.trainer.graph_step import GraphedTrainStep
    config, train, valid, test, model = _pipeline(tmp_path, adam_mode='deferred',
                                                  train_batch_size=200)
    tr = Trainer(config, model)
    opt = tr.optimizer
    assert getattr(opt, '_deferred', {})
    from recbole_amd.data.interaction import Interaction
    batches = [b.to(config['device']) for b in train]
    batches = batches[:5] + [Interaction({k: v[:77] for k, v in batches[5].interaction.items()})]
    assert batches[-1].length != batches[0].length          # a ragged batch (runs eagerly)
    gs = GraphedTrainStep(model, opt, window=window) if graphed else None
    losses = []
    for k in range(steps):
        b = batches[k % len(batches)]
        if gs is not None:
            loss = gs.step(b).clone()
        else:
            opt.zero_grad()
            loss = model.calculate_loss(b)
            loss.backward()
            opt.step()
        losses.append(float(loss.item()))
        if k == steps // 2:
            opt.flush()                                   # e.g. a checkpoint / evaluation
    opt.flush()
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    st = opt.state_dict()['state']
    mom = [(s['exp_avg'].cpu(), s['exp_avg_sq'].cpu()) for _, s in sorted(st.items())]
    return losses, sd, mom, (gs.n_graphed if gs else 0), opt.n_steps


def test_graphed_deepfm_step_bitwise(tmp_path):
    steps, window = 40, 8
    la, sa, ma, ng, na = _run(tmp_path / 'g', True, steps, window)
    lb, sb, mb, _, nb = _run(tmp_path / 'e', False, steps, window)
    assert na == nb == steps
    assert ng >= steps // 2                               # most steps replayed the graph
    assert la == lb
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    for (x1, y1), (x2, y2) in zip(ma, mb):
        assert torch.equal(x1, x2) and torch.equal(y1, y2)
