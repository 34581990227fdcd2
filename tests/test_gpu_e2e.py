"""End-to-end parity of the drop-in path on the GPU: Config -> dataset ->
data_preparation -> BPR -> Trainer.fit (fused kernels) against the oracle
replaying the reference's algorithm on the CPU with the same RNG streams:
torch.randperm epoch order (interaction.py:272-276), the sampler walk
(sampler.py:103-154, C restatement), nn.Embedding + BPRLoss + optim.Adam on
torch CPU (trainer.py:157-174)."""
import os

import numpy as np
import pytest
import torch

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _write_dataset(root, name, n_users=300, n_items=500, n_inter=12000, seed=0):
    rng = np.random.default_rng(seed)
    d = os.path.join(root, name)
    os.makedirs(d, exist_ok=True)
    u = rng.integers(1, n_users + 1, n_inter)
    pop = 1.0 / np.arange(1, n_items + 1)
    i = rng.choice(np.arange(1, n_items + 1), n_inter, p=pop / pop.sum())
    ts = rng.random(n_inter)
    with open(os.path.join(d, f'{name}.inter'), 'w') as f:
        f.write('user_id:token\titem_id:token\ttimestamp:float\n')
        for a, b, c in zip(u, i, ts):
            f.write(f'u{a}\ti{b}\t{c:.6f}\n')
    return root


def _pipeline(tmp_path, **over):
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset, data_preparation
    from recbole_amd.utils import get_model, init_seed
    root = _write_dataset(str(tmp_path), 'synth')
    cd = {'model': 'BPR', 'dataset': 'synth', 'data_path': root, 'epochs': 2,
          'train_batch_size': 512, 'training_neg_sample_num': 2, 'embedding_size': 64,
          'eval_setting': 'RO_RS,full', 'checkpoint_dir': str(tmp_path / 'saved'),
          'load_col': {'inter': ['user_id', 'item_id', 'timestamp']}}
    cd.update(over)
    config = Config(config_dict=cd)
    init_seed(config['seed'], config['reproducibility'])
    ds = create_dataset(config)
    train, valid, test = data_preparation(config, ds)
    model = get_model(cd['model'])(config, train).to(config['device'])
    return config, train, valid, test, model


def _oracle_train(init_u, init_i, users0, items0, rng_state, rl, used_ptr, used_cols, n_users,
                  B, T, epochs, lr):
    # nn.Embedding's constructor draws from the CPU generator: build first, then
    # restore the generator so the epoch permutations line up with the product's
    m = cpu_ref.BPRCPU(init_u.shape[0], init_i.shape[0], init_u.shape[1], init=False)
    m.user_embedding.weight.data.copy_(init_u)
    m.item_embedding.weight.data.copy_(init_i)
    opt = torch.optim.Adam(m.parameters(), lr=lr)
    torch.set_rng_state(rng_state)
    users, items = users0.clone(), items0.clone()
    pr = 0
    epoch_losses = []
    for _ in range(epochs):
        perm = torch.randperm(len(users))
        users, items = users[perm], items[perm]
        total = 0.0
        for s in range(0, len(users), B):
            ub, ib = users[s:s + B], items[s:s + B]
            neg, pr = cpu_ref.c_sample_walk(rl, pr, ub.numpy(), T, used_ptr, used_cols, n_users,
                                            True)
            ur, pr_, nr = cpu_ref.pairwise_rows(ub, ib, torch.as_tensor(neg), T)
            opt.zero_grad()
            loss = m.calculate_loss(ur, pr_, nr)
            total += loss.item()
            loss.backward()
            opt.step()
        epoch_losses.append(total)
    return m, epoch_losses, pr


@pytest.mark.parametrize('fused', [True, False])
def test_fit_matches_oracle(tmp_path, fused):
    from recbole_amd.trainer import Trainer
    config, train, valid, test, model = _pipeline(tmp_path, fused_train=fused)
    init_u = model.user_embedding.weight.detach().cpu().clone()
    init_i = model.item_embedding.weight.detach().cpu().clone()
    users0 = train.dataset.inter_feat['user_id'].cpu().clone()
    items0 = train.dataset.inter_feat['item_id'].cpu().clone()
    rng_state = torch.get_rng_state()
    rl = train.sampler.random_list.copy()
    ptr, cols = cpu_ref.used_csr(train.dataset.user_num, users0.numpy(), items0.numpy())
    trainer = Trainer(config, model)
    assert trainer._fused_applicable(train) == fused
    losses = []
    for e in range(config['epochs']):
        losses.append(trainer._train_epoch(train, e))
    m, ref_losses, ref_pr = _oracle_train(init_u, init_i, users0, items0, rng_state, rl, ptr,
                                          cols, train.dataset.user_num, train.step, train.times,
                                          config['epochs'], config['learning_rate'])
    assert train.sampler.random_pr == ref_pr                 # bit-exact walk
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-4)
    torch.testing.assert_close(model.user_embedding.weight.detach().cpu(),
                               m.user_embedding.weight.detach(), rtol=1e-3, atol=2e-5)
    torch.testing.assert_close(model.item_embedding.weight.detach().cpu(),
                               m.item_embedding.weight.detach(), rtol=1e-3, atol=2e-5)


@pytest.mark.parametrize('d', [64, 256])
def test_fused_adam_schedules_bitwise_identical(tmp_path, d):
    """Deferred and streamed dense Adam, graph-replayed chunks and eager steps, the
    one-launch K35 step (parity buffers) and the K3 + K5 launches: identical bits in the
    weights, the optimizer state and the losses."""
    from recbole_amd.trainer.fused import FusedBPRTrainStep
    from recbole_amd.trainer.optim import FusedAdam
    out = {}
    for mode, graph, k35 in (('streamed', True, False), ('deferred', True, True),
                             ('deferred', False, True), ('deferred', True, False)):
        config, train, valid, test, model = _pipeline(tmp_path, embedding_size=d)
        opt = FusedAdam(model.parameters(), lr=config['learning_rate'])
        fs = FusedBPRTrainStep(model, opt, train, chunk=8, use_graph=graph, adam_mode=mode,
                               fused_step=k35)
        assert fs.fused_step == k35
        losses = []
        for _ in range(2):
            nb = fs.begin_epoch()
            fs.run_batches(0, 11)                 # a graph chunk, then eager partial chunks
            fs.run_batches(11, nb)
            losses += fs.end_epoch()
        st = [opt.state[p][k].cpu() for p in (fs.pU, fs.pI) for k in ('exp_avg', 'exp_avg_sq')]
        out[(mode, graph, k35)] = ([fs.pU.detach().cpu(), fs.pI.detach().cpu()] + st, losses)
    ref_t, ref_l = out[('streamed', True, False)]
    for key, (ts, ls) in out.items():
        assert ls == ref_l, key
        for a, b in zip(ref_t, ts):
            assert torch.equal(a, b), key


def test_fused_full_sort_eval_matches_generic(tmp_path):
    """The fused K6 evaluator and the reference's full_sort_predict + mask + swap +
    TopKEvaluator.collect sequence give identical metrics."""
    from recbole_amd.trainer import Trainer
    config, train, valid, test, model = _pipeline(tmp_path, epochs=1)
    trainer = Trainer(config, model)
    trainer._train_epoch(train, 0)
    fused = trainer.evaluate(test, load_best_model=False)
    config['fused_eval'] = False                      # reference sequence on the same model
    generic = trainer.evaluate(test, load_best_model=False)
    assert fused.keys() == generic.keys()
    for k in fused:
        assert fused[k] == pytest.approx(generic[k], abs=2e-4), k


def test_fused_full_sort_eval_overlapped_identical(tmp_path):
    """Round-sized K6 launches with the host metric reduction of each launch's block
    overlapping the next (the path C2's 138 K users take) give exactly the metrics
    of one launch and one block (round_users=0 disables the split)."""
    from recbole_amd.evaluator import TopKEvaluator
    from recbole_amd.trainer import Trainer
    from recbole_amd.trainer.fused import fused_full_sort_eval
    config, train, valid, test, model = _pipeline(tmp_path, epochs=1)
    Trainer(config, model)._train_epoch(train, 0)
    ev = TopKEvaluator(config, ['recall', 'mrr', 'ndcg', 'hit', 'precision', 'map'])
    one = fused_full_sort_eval(model, test, ev, round_users=0)
    for r in (128, 300, 4096):
        assert fused_full_sort_eval(model, test, ev, round_users=r) == one, r


def test_run_recbole_end_to_end(tmp_path):
    from recbole_amd.quick_start import run_recbole
    root = _write_dataset(str(tmp_path), 'synth')
    res = run_recbole(model='BPR', dataset='synth', config_dict={
        'data_path': root, 'epochs': 2, 'checkpoint_dir': str(tmp_path / 'saved'),
        'load_col': {'inter': ['user_id', 'item_id', 'timestamp']}, 'show_progress': False})
    assert set(res['test_result']) == {'recall@10', 'mrr@10', 'ndcg@10', 'hit@10',
                                       'precision@10'}
    assert 0.0 <= res['test_result']['hit@10'] <= 1.0


def test_checkpoint_roundtrip(tmp_path):
    from recbole_amd.trainer import Trainer
    config, train, valid, test, model = _pipeline(tmp_path, epochs=1)
    tr = Trainer(config, model)
    tr._train_epoch(train, 0)
    tr._save_checkpoint(0)
    sd = torch.load(tr.saved_model_file, weights_only=True)   # plain checkpoint: no unpickling
    assert set(sd['state_dict']) == {'user_embedding.weight', 'item_embedding.weight'}
    assert set(sd['optimizer']['state'][0]) == {'step', 'exp_avg', 'exp_avg_sq'}
    config2, train2, _, _, model2 = _pipeline(tmp_path, epochs=1)
    tr2 = Trainer(config2, model2)
    tr2.resume_checkpoint(tr.saved_model_file)
    assert tr2.start_epoch == 1 and tr2.optimizer.n_steps == tr.optimizer.n_steps
    torch.testing.assert_close(model2.user_embedding.weight, model.user_embedding.weight)
