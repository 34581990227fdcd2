"""The captured generic training step (trainer/graph_step.py GraphedTrainStep):
DeepFM (token + first-order tables on the deferred K5 schedule, MLP / biases
dense) replayed from one HIP graph per batch shape, against the eager step of the
ordinary FusedAdam (host step indices, separate windows) — losses, parameters and
Adam state bit-identical over several graph-mode window roll-overs, a ragged last
batch (eager) and a checkpoint-style flush in between."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(tmp_path, graphed, steps, window, model_name='DeepFM', **kw):
    from recbole_amd.trainer import Trainer
    from recbole_amd.trainer.graph_step import GraphedTrainStep
    if model_name == 'DeepFM':
        from tests.test_gpu_deepfm import _pipeline
        config, train, valid, test, model = _pipeline(tmp_path, adam_mode='deferred',
                                                      train_batch_size=200)
    else:
        from tests.test_gpu_sasrec import _pipeline
        config, train, valid, test, model = _pipeline(
            tmp_path, adam_mode='deferred', train_batch_size=96, hidden_dropout_prob=0.0,
            attn_dropout_prob=0.0, **kw)
    tr = Trainer(config, model)
    opt = tr.optimizer
    assert getattr(opt, '_deferred', {}) or kw.get('loss_type') == 'CE'
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


@pytest.mark.parametrize('loss', ['SSM', 'BPR', 'CE'])
def test_graphed_sasrec_step_bitwise(tmp_path, loss):
    """SASRec (K9a embedding + LayerNorm, torch transformer blocks, K9b sampled softmax /
    K3 BPR over the sequence outputs with the item table deferred; CE with a dense item
    table), dropout 0: the captured step equals the eager step bit for bit."""
    kw = {'loss_type': loss}
    if loss != 'CE':
        kw['training_neg_sample_num'] = 4 if loss == 'SSM' else 1
    steps, window = 24, 8
    la, sa, ma, ng, na = _run(tmp_path / 'g', True, steps, window, 'SASRec', **kw)
    lb, sb, mb, _, nb = _run(tmp_path / 'e', False, steps, window, 'SASRec', **kw)
    assert na == nb == steps
    assert ng >= steps // 2
    assert la == lb
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    for (x1, y1), (x2, y2) in zip(ma, mb):
        assert torch.equal(x1, x2) and torch.equal(y1, y2)


def test_copy_many(dev):
    """mirec_copy_many: mixed dtypes and sizes, unaligned views, > 96 copies (two
    launches) — every destination equals its source, nothing else is written."""
    from recbole_amd import ops
    g = torch.Generator(device='cpu').manual_seed(0)
    srcs, dsts, guards = [], [], []
    for i in range(130):
        n = [0, 1, 3, 17, 1000, 65537][i % 6]
        dt = [torch.float32, torch.int64, torch.int8, torch.float64][i % 4]
        base = torch.randint(-100, 100, (n + 3,), generator=g).to(dt).to(dev)
        s = base[i % 3:i % 3 + n]                       # unaligned views
        buf = torch.full((n + 5,), 7, dtype=dt, device=dev)
        d = buf[1:1 + n]
        srcs.append(s.contiguous() if not s.is_contiguous() else s)
        dsts.append(d)
        guards.append(buf)
    ops.copy_many(dsts, srcs)
    torch.cuda.synchronize()
    for s, d, buf in zip(srcs, dsts, guards):
        assert torch.equal(d, s)
        assert (buf[0] == 7).item() and bool((buf[1 + s.numel():] == 7).all())
