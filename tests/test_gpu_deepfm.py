"""DeepFM on the GPU (K8 field embedding + first order + FM, library-GEMM MLP,
fused sigmoid + BCE) against the oracle's torch-CPU restatement of
deepfm.py:26-73 / abstract_recommender.py:151-412 / layers.py (dropout 0 so
both sides are deterministic). Tolerances: fp32 1e-4 relative on loss and
predictions (north_star), gradients 1e-4 relative + 1e-6 absolute."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref
from tests.ctx_data import write_ctx_dataset

pytestmark = pytest.mark.gpu


def _pipeline(tmp_path, **over):
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset, data_preparation
    from recbole_amd.utils import get_model, init_seed
    root = write_ctx_dataset(str(tmp_path), seq=over.pop('seq', True))
    cd = {'model': 'DeepFM', 'dataset': 'ctx', 'data_path': root, 'embedding_size': 16,
          'dropout_prob': 0.0, 'load_col': None, 'epochs': 1, 'train_batch_size': 512,
          'checkpoint_dir': str(tmp_path / 'saved')}
    cd.update(over)
    config = Config(config_dict=cd)
    init_seed(config['seed'], config['reproducibility'])
    ds = create_dataset(config)
    train, valid, test = data_preparation(config, ds)
    model = get_model('DeepFM')(config, train).to(config['device'])
    return config, train, valid, test, model


def _oracle(model):
    ref = cpu_ref.DeepFMCPU(model.token_field_names, model.token_field_dims,
                            model.token_seq_field_names, model.token_seq_field_dims,
                            model.float_field_names, model.embedding_size,
                            model.mlp_hidden_size, 0.0)
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    return ref


def _cpu(inter):
    return {k: v.cpu() for k, v in inter.interaction.items()}


@pytest.mark.parametrize('seq', [True, False])
def test_loss_grads_predictions_match_oracle(tmp_path, seq):
    config, train, valid, test, model = _pipeline(tmp_path, seq=seq)
    ref = _oracle(model)
    b = next(iter(train)).to(config['device'])
    loss = model.calculate_loss(b)
    loss.backward()
    lr_ = ref.calculate_loss(_cpu(b), b['label'].cpu())
    lr_.backward()
    np.testing.assert_allclose(loss.item(), lr_.item(), rtol=1e-4)
    refp = dict(ref.named_parameters())
    for name, p in model.named_parameters():
        assert p.grad is not None, name
        torch.testing.assert_close(p.grad.cpu(), refp[name].grad, rtol=1e-4, atol=1e-6,
                                   msg=name)
    with torch.no_grad():
        pred = model.predict(b).cpu()
        exp = ref.forward(_cpu(b))
    torch.testing.assert_close(pred, exp, rtol=1e-4, atol=1e-6)


def test_train_steps_match_oracle(tmp_path):
    from recbole_amd.trainer import Trainer
    config, train, valid, test, model = _pipeline(tmp_path)
    ref = _oracle(model)
    opt = torch.optim.Adam(ref.parameters(), lr=config['learning_rate'])
    trainer = Trainer(config, model)
    for b in list(train)[:5]:
        bd = b.to(config['device'])
        trainer.optimizer.zero_grad()
        loss = model.calculate_loss(bd)
        loss.backward()
        trainer.optimizer.step()
        opt.zero_grad()
        lr_ = ref.calculate_loss(_cpu(b), b['label'].cpu())
        lr_.backward()
        opt.step()
        np.testing.assert_allclose(loss.item(), lr_.item(), rtol=1e-4)
    assert trainer.optimizer._deferred            # the token table ran deferred
    trainer.optimizer.flush()                     # complete the rows no batch touched last
    refp = dict(ref.named_parameters())
    for name, p in model.named_parameters():
        torch.testing.assert_close(p.detach().cpu(), refp[name].detach(), rtol=1e-3, atol=2e-5,
                                   msg=name)


def test_run_recbole_deepfm(tmp_path):
    from recbole_amd.quick_start import run_recbole
    root = write_ctx_dataset(str(tmp_path))
    res = run_recbole(model='DeepFM', dataset='ctx', config_dict={
        'data_path': root, 'epochs': 2, 'load_col': None, 'embedding_size': 16,
        'checkpoint_dir': str(tmp_path / 'saved'), 'show_progress': False})
    r = res['test_result']
    assert set(k.lower() for k in r) == {'auc', 'logloss'}
    assert 0.0 <= r[[k for k in r if k.lower() == 'auc'][0]] <= 1.0
