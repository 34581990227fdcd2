"""LightGCN on the GPU (K7 graph propagation + K3 BPR + EmbLoss kernels) against
the oracle's torch-CPU restatement of lightgcn.py:32-180 (torch.sparse.mm,
BPRLoss, EmbLoss, optim.Adam). Tolerances: fp32 1e-4 relative on losses and
propagated embeddings (north_star), gradients 1e-4 relative + 1e-7 absolute."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _graph(U, I, nnz, seed, hub=True):
    rng = np.random.default_rng(seed)
    u = rng.integers(1, U, nnz)
    pop = 1.0 / np.arange(1, I) ** 1.2
    i = rng.choice(np.arange(1, I), nnz, p=pop / pop.sum())
    if hub:                                  # one user with a very long row (split units)
        u[: nnz // 4] = 1
    return u, i


@pytest.mark.parametrize('d', [32, 64, 128, 256])
@pytest.mark.parametrize('piece', [3, 256])
def test_spmm_epilogues_match_torch_sparse(dev, d, piece):
    from recbole_amd import ops
    from recbole_amd.model.general_recommender.lightgcn import norm_adj_csr
    U, I = 70, 120
    u, i = _graph(U, I, 1500, d + piece)
    A = cpu_ref.lightgcn_norm_adj(u, i, U, I)
    plan = ops.SpmmPlan(*norm_adj_csr(u, i, U, I), device=dev, piece=piece)
    assert (plan.n_fix > 0) == (piece == 3)
    g = torch.Generator().manual_seed(d)
    X = torch.randn(U + I, d, generator=g)
    Add = torch.randn(U + I, d, generator=g)
    Acc = torch.randn(U + I, d, generator=g)
    ref = torch.sparse.mm(A, X)
    Xd, Ad, Cd = X.to(dev), Add.to(dev), Acc.to(dev)
    Y = torch.empty_like(Xd)
    ops.spmm_csr(plan, Xd, y=Y)
    torch.testing.assert_close(Y.cpu(), ref, rtol=1e-5, atol=1e-6)
    # split operands (lo, hi) + add + running accumulator, all in one launch
    Yl, Yh = torch.empty(U, d, device=dev), torch.empty(I, d, device=dev)
    Ol, Oh = torch.empty(U, d, device=dev), torch.empty(I, d, device=dev)
    ops.spmm_csr(plan, (Xd[:U].contiguous(), Xd[U:].contiguous()), y=(Yl, Yh), add=Ad,
                 add_scale=0.25, acc_in=(Cd[:U].contiguous(), Cd[U:].contiguous()),
                 acc_out=(Ol, Oh), acc_scale=0.5)
    y2 = ref + 0.25 * Add
    torch.testing.assert_close(torch.cat([Yl, Yh]).cpu(), y2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(torch.cat([Ol, Oh]).cpu(), (Acc + y2) * 0.5, rtol=1e-5, atol=1e-6)


def _models(dev, U, I, d, n_layers, u, i, reg=1e-5):
    from recbole_amd.model.general_recommender import lightgcn as L
    from recbole_amd import ops
    A = cpu_ref.lightgcn_norm_adj(u, i, U, I)
    ref = cpu_ref.LightGCNCPU(U, I, d, n_layers, reg, A)
    plan = ops.SpmmPlan(*L.norm_adj_csr(u, i, U, I), device=dev, piece=16)
    EU = torch.nn.Parameter(ref.user_embedding.weight.detach().clone().to(dev))
    EI = torch.nn.Parameter(ref.item_embedding.weight.detach().clone().to(dev))
    return ref, plan, EU, EI


@pytest.mark.parametrize('n_layers', [0, 1, 2, 3])
def test_propagation_and_loss_grads(dev, n_layers):
    from recbole_amd.model.general_recommender import lightgcn as L
    from recbole_amd.model.general_recommender.bpr import _BPRLossFn
    U, I, d, R = 90, 160, 64, 256
    u, i = _graph(U, I, 2000, n_layers)
    ref, plan, EU, EI = _models(dev, U, I, d, n_layers, u, i, reg=1e-2)
    rng = np.random.default_rng(7)
    user = torch.as_tensor(rng.integers(0, U, R))
    pos = torch.as_tensor(rng.integers(1, I, R))
    neg = torch.as_tensor(rng.integers(1, I, R))
    ua, ia = ref.forward()
    gua, gia = L._PropagateFn.apply(EU, EI, plan, n_layers)
    torch.testing.assert_close(gua.detach().cpu(), ua.detach(), rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(gia.detach().cpu(), ia.detach(), rtol=1e-4, atol=1e-6)
    loss_ref = ref.calculate_loss(user, pos, neg)
    loss_ref.backward()
    ud, pd, nd = user.to(dev), pos.to(dev), neg.to(dev)
    mf = _BPRLossFn.apply(gua, gia, ud, pd, nd)
    loss = mf + 1e-2 * L._EmbRegFn.apply(EU, EI, ud, pd, nd)
    loss.backward()
    assert loss.shape == loss_ref.shape == (1,)
    np.testing.assert_allclose(loss.item(), loss_ref.item(), rtol=1e-4)
    torch.testing.assert_close(EU.grad.cpu(), ref.user_embedding.weight.grad, rtol=1e-4,
                               atol=1e-7)
    torch.testing.assert_close(EI.grad.cpu(), ref.item_embedding.weight.grad, rtol=1e-4,
                               atol=1e-7)


def test_fit_and_full_sort_match_oracle(tmp_path):
    """Config -> Dataset -> LightGCN -> Trainer (generic loop, FusedAdam on dense
    grads) vs the oracle on the same batches; then full-sort top-K (fused K6)
    vs the generic reference sequence."""
    from tests.test_gpu_e2e import _pipeline
    from recbole_amd.trainer import Trainer
    config, train, valid, test, model = _pipeline(
        tmp_path, model='LightGCN', training_neg_sample_num=1, epochs=1, embedding_size=64)
    U, I = model.n_users, model.n_items
    m = model.interaction_matrix
    ref = cpu_ref.LightGCNCPU(U, I, 64, model.n_layers, model.reg_weight,
                              cpu_ref.lightgcn_norm_adj(m.row, m.col, U, I), init=False)
    ref.user_embedding.weight.data.copy_(model.user_embedding.weight.detach().cpu())
    ref.item_embedding.weight.data.copy_(model.item_embedding.weight.detach().cpu())
    opt = torch.optim.Adam(ref.parameters(), lr=config['learning_rate'])
    trainer = Trainer(config, model)
    assert not trainer._fused_applicable(train)
    batches = [b for b in train]                       # fixed batches for both sides
    for b in batches[:6]:
        bd = b.to(config['device'])
        trainer.optimizer.zero_grad()
        loss = model.calculate_loss(bd)
        loss.backward()
        trainer.optimizer.step()
        opt.zero_grad()
        lr_ = ref.calculate_loss(b['user_id'].cpu(), b['item_id'].cpu(), b['neg_item_id'].cpu())
        lr_.backward()
        opt.step()
        np.testing.assert_allclose(loss.item(), lr_.item(), rtol=1e-4)
    torch.testing.assert_close(model.user_embedding.weight.detach().cpu(),
                               ref.user_embedding.weight.detach(), rtol=1e-3, atol=2e-5)
    torch.testing.assert_close(model.item_embedding.weight.detach().cpu(),
                               ref.item_embedding.weight.detach(), rtol=1e-3, atol=2e-5)
    model.restore_user_e = model.restore_item_e = None
    fused = trainer.evaluate(test, load_best_model=False)
    config['fused_eval'] = False
    generic = trainer.evaluate(test, load_best_model=False)
    for k in fused:
        assert fused[k] == pytest.approx(generic[k], abs=2e-4), k
    uid = torch.arange(1, 9)
    exp = ref.full_sort_predict(uid).detach()
    from recbole_amd.data.interaction import Interaction
    got = model.full_sort_predict(Interaction({'user_id': uid}).to(config['device'])).cpu()
    torch.testing.assert_close(got, exp, rtol=1e-4, atol=1e-5)


def test_run_recbole_lightgcn(tmp_path):
    from tests.test_gpu_e2e import _write_dataset
    from recbole_amd.quick_start import run_recbole
    root = _write_dataset(str(tmp_path), 'synth')
    res = run_recbole(model='LightGCN', dataset='synth', config_dict={
        'data_path': root, 'epochs': 1, 'checkpoint_dir': str(tmp_path / 'saved'),
        'load_col': {'inter': ['user_id', 'item_id', 'timestamp']}, 'show_progress': False})
    assert 0.0 <= res['test_result']['hit@10'] <= 1.0
