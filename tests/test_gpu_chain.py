"""End-to-end parity of the drop-in chain FROM THE SEED at the BASELINE configs'
real sizes, against the oracle replayed independently (nothing is copied from
the product: the oracle re-derives the split, the sampler's random_list, the
initial weights and every epoch permutation from init_seed(2020)):

  C2  BPR-MF ml-20m-shape (bench.py's workload: 138,494 x 26,745 tables, d=128,
      4 negatives, 512 positives per step): one full 64-step chunk through the
      fused path (graph replay, deferred Adam) — every sampled negative id
      bit-exact, walk pointer exact, per-step losses and the tables after the
      chunk within 1e-4; then the streamed dense-Adam schedule over the same chunk
      bit-identical to the deferred one at full table size.
  C1  BPR on the bundled ml-100k atomic files through Trainer (3 epochs):
      epoch losses 1e-5, walk pointer exact, tables 1e-4; and the reference's
      own entry line (`from recbole.quick_start import run_recbole`) runs it.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _train_arrays(train):
    f = train.dataset.inter_feat
    return f['user_id'].cpu().numpy().copy(), f['item_id'].cpu().numpy().copy()


def test_c2_chunk_chain_from_seed(dev):
    import bench
    config, train, test, model, opt, step = bench.build_workload(dev, source='memory')
    tu, ti = _train_arrays(train)
    rl = np.asarray(train.sampler.random_list).copy()
    init = [p.detach().cpu().clone() for p in (step.pU, step.pI)]
    saved_table = {k: v.clone() for k, v in train.dataset.inter_feat.interaction.items()}
    rng_before_epoch = torch.get_rng_state()
    C = step.C
    step.RAMP = ()              # one chunk of C batches: its keys stay in slot 0 (read below)
    step.begin_epoch(cuts=(C,), hold_prep_from=C)      # no look-ahead walk past the chunk
    step.run_batches(0, C)
    losses = step.end_epoch(C)
    pr = train.sampler.random_pr
    KI = (1 + step.times) * step.B
    keys = step.slots[0].item_keys[:C * KI].view(C, KI).cpu().numpy()
    got = [p.detach().cpu().clone() for p in (step.pU, step.pI)]

    # ---- oracle, from the seed
    u, i, nU, nI = bench.make_c2(2020)
    torch.manual_seed(2020)
    np.random.seed(2020)
    parts = cpu_ref.ro_rs_split(u, (0.8, 0.1, 0.1))
    ref_rl = cpu_ref.random_list_uniform(nI)
    ref = cpu_ref.BPRCPU(nU, nI, 128)
    assert torch.equal(torch.get_rng_state(), rng_before_epoch)
    assert np.array_equal(tu, u[parts[0]]) and np.array_equal(ti, i[parts[0]])
    assert np.array_equal(rl, ref_rl)
    assert torch.equal(init[0], ref.user_embedding.weight.detach())
    assert torch.equal(init[1], ref.item_embedding.weight.detach())
    ptr, cols = cpu_ref.used_csr(nU, tu, ti)
    ref_losses, ref_negs, ref_pr = cpu_ref.bpr_replay(ref, tu, ti, ref_rl, ptr, cols, nU,
                                                       step.B, step.times, C)
    for s in range(C):
        bad = np.flatnonzero(keys[s, step.B:] != ref_negs[s])
        assert bad.size == 0, (f'negatives of step {s}: {bad.size} differ, first at '
                               f'{bad[:8].tolist()}: {keys[s, step.B:][bad[:8]].tolist()} vs '
                               f'{np.asarray(ref_negs[s])[bad[:8]].tolist()}')
    assert pr == ref_pr
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-4)
    torch.testing.assert_close(got[0], ref.user_embedding.weight.detach(), rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(got[1], ref.item_embedding.weight.detach(), rtol=1e-4, atol=1e-6)

    # ---- streamed dense Adam over the same chunk: identical bits
    from recbole_amd.model.general_recommender import BPR
    from recbole_amd.trainer.fused import FusedBPRTrainStep
    from recbole_amd.trainer.optim import FusedAdam
    train.dataset.inter_feat.interaction = {k: v.clone() for k, v in saved_table.items()}
    train.sampler.random_pr = 0
    model2 = BPR(config, train).to(dev)
    model2.user_embedding.weight.data.copy_(init[0])
    model2.item_embedding.weight.data.copy_(init[1])
    opt2 = FusedAdam(model2.parameters(), lr=config['learning_rate'])
    step2 = FusedBPRTrainStep(model2, opt2, train, adam_mode='streamed')
    torch.set_rng_state(rng_before_epoch)
    step2.begin_epoch(cuts=(C,), hold_prep_from=C)     # ramped chunks (2, 4, .., 32, 2)
    step2.run_batches(0, C)
    losses2 = step2.end_epoch(C)
    assert losses2 == losses
    assert torch.equal(step2.pU.detach().cpu(), got[0])
    assert torch.equal(step2.pI.detach().cpu(), got[1])
    for p, q in ((step.pU, step2.pU), (step.pI, step2.pI)):
        for k in ('exp_avg', 'exp_avg_sq'):
            assert torch.equal(opt.state[p][k], opt2.state[q][k]), k


def test_c1_ml100k_trainer_chain_from_seed(dev, tmp_path):
    from recbole.config import Config
    from recbole.data import create_dataset, data_preparation
    from recbole.trainer import Trainer
    from recbole.utils import get_model, init_seed
    config = Config(model='BPR', dataset='ml-100k', config_dict={
        'data_path': os.path.join(ROOT, 'dataset'), 'checkpoint_dir': str(tmp_path),
        'state': 'ERROR'})
    init_seed(config['seed'], config['reproducibility'])
    train, valid, test = data_preparation(config, create_dataset(config))
    model = get_model('BPR')(config, train).to(config['device'])
    trainer = Trainer(config, model)
    assert trainer._fused_applicable(train)
    epochs = [trainer._train_epoch(train, e) for e in range(3)]

    u, i, nU, nI = cpu_ref.load_ml100k(os.path.join(ROOT, 'dataset', 'ml-100k'))
    torch.manual_seed(2020)
    np.random.seed(2020)
    parts = cpu_ref.ro_rs_split(u, (0.8, 0.1, 0.1))
    rl = cpu_ref.random_list_uniform(nI)
    ref = cpu_ref.BPRCPU(nU, nI, 64)
    tu, ti = u[parts[0]], i[parts[0]]
    ptr, cols = cpu_ref.used_csr(nU, tu, ti)
    steps_per_epoch = -(-len(tu) // 2048)
    ref_losses, _, ref_pr = cpu_ref.bpr_replay(ref, tu, ti, rl, ptr, cols, nU, 2048, 1,
                                               3 * steps_per_epoch)
    ref_epochs = [sum(ref_losses[e * steps_per_epoch:(e + 1) * steps_per_epoch])
                  for e in range(3)]
    assert train.sampler.random_pr == ref_pr
    np.testing.assert_allclose(epochs, ref_epochs, rtol=1e-5)
    torch.testing.assert_close(model.user_embedding.weight.detach().cpu(),
                               ref.user_embedding.weight.detach(), rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(model.item_embedding.weight.detach().cpu(),
                               ref.item_embedding.weight.detach(), rtol=1e-4, atol=1e-6)


def test_reference_entry_line_runs_c1(tmp_path):
    """A script written against the reference (its run_recbole.py import line)
    runs BPR on ml-100k through this build, with --alpha -> config_dict."""
    script = tmp_path / 'user_script.py'
    script.write_text(
        'from recbole.quick_start import run_recbole\n'
        'import sys, json\n'
        "r = run_recbole(model='BPR', dataset='ml-100k', config_dict={'epochs': 2, "
        "'data_path': sys.argv[1], 'checkpoint_dir': sys.argv[2], 'show_progress': False, "
        "'state': 'ERROR'})\n"
        "print('RESULT', json.dumps(r['test_result']))\n")
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, str(script), os.path.join(ROOT, 'dataset'),
                          str(tmp_path / 'saved')], cwd=str(tmp_path), env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [x for x in out.stdout.splitlines() if x.startswith('RESULT')][-1]
    import json
    res = json.loads(line[len('RESULT '):])
    assert set(res) == {'recall@10', 'mrr@10', 'ndcg@10', 'hit@10', 'precision@10'}
    assert 0.0 < res['hit@10'] <= 1.0
    cli = subprocess.run([sys.executable, os.path.join(ROOT, 'run_recbole.py'), '--model', 'BPR',
                          '--dataset', 'ml-100k', '--alpha', '0.5', '--epochs=1',
                          f'--data_path={os.path.join(ROOT, "dataset")}',
                          f'--checkpoint_dir={tmp_path / "saved2"}', '--show_progress=False'],
                         cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert cli.returncode == 0, cli.stderr[-3000:]
