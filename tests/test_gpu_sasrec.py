"""SASRec on the GPU (K9a embedding+LayerNorm, K3 BPR / K9b sampled softmax /
library-GEMM CE, window-gather loaders, K6 sequential full-sort) against the
oracle's torch-CPU restatement (sasrec.py:25-158, layers.py:338-552), dropout 0.
Tolerances: fp32 1e-4 relative on losses and outputs (north_star); gradients
1e-4 relative + 1e-6 absolute (the transformer in between is the same op
sequence on both sides)."""
import math

import numpy as np
import pytest
import torch

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _pipeline(tmp_path, **over):
    from tests.test_gpu_e2e import _write_dataset
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset, data_preparation
    from recbole_amd.utils import get_model, init_seed
    root = _write_dataset(str(tmp_path), 'synth', n_users=80, n_items=120, n_inter=3000)
    cd = {'model': 'SASRec', 'dataset': 'synth', 'data_path': root, 'epochs': 1,
          'load_col': {'inter': ['user_id', 'item_id', 'timestamp']}, 'MAX_ITEM_LIST_LENGTH': 12,
          'hidden_dropout_prob': 0.0, 'attn_dropout_prob': 0.0, 'train_batch_size': 256,
          'checkpoint_dir': str(tmp_path / 'saved'), 'loss_type': 'CE',
          'training_neg_sample_num': 0}
    cd.update(over)
    config = Config(config_dict=cd)
    init_seed(config['seed'], config['reproducibility'])
    ds = create_dataset(config)
    train, valid, test = data_preparation(config, ds)
    model = get_model('SASRec')(config, train).to(config['device'])
    return config, train, valid, test, model


def _oracle(model):
    ref = cpu_ref.SASRecCPU(model.n_items, model.max_seq_length, model.hidden_size,
                            model.n_layers, model.n_heads, model.inner_size, model.layer_norm_eps)
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    return ref


@pytest.mark.parametrize('d', [32, 64, 128, 256])
def test_seq_embed_layernorm_fwd_bwd(dev, d):
    from recbole_amd.model.sequential_recommender.sasrec import _SeqEmbedLNFn
    g = torch.Generator().manual_seed(d)
    nI, L, B = 300, 17, 37
    E = torch.randn(nI, d, generator=g)
    P = torch.randn(L, d, generator=g)
    gam, bet = torch.randn(d, generator=g), torch.randn(d, generator=g)
    seq = torch.randint(0, nI, (B, L), generator=g)
    seq[:, -5:] = 0
    gout = torch.randn(B, L, d, generator=g)
    ref_e = torch.nn.Embedding(nI, d, padding_idx=0)
    ref_e.weight.data.copy_(E)
    params = [torch.nn.Parameter(t.clone()) for t in (P, gam, bet)]
    x = ref_e(seq) + params[0][torch.arange(L)].unsqueeze(0)
    y = torch.nn.functional.layer_norm(x, (d,), params[1], params[2], 1e-12)
    (y * gout).sum().backward()
    dp = [torch.nn.Parameter(t.clone().to(dev)) for t in (E, P, gam, bet)]
    yd = _SeqEmbedLNFn.apply(*dp, seq.to(dev), 1e-12)
    (yd * gout.to(dev)).sum().backward()
    torch.testing.assert_close(yd.detach().cpu(), y.detach(), rtol=1e-4, atol=1e-5)
    for a, b in zip(dp, [ref_e.weight] + params):
        torch.testing.assert_close(a.grad.cpu(), b.grad, rtol=1e-4, atol=1e-4)
    assert (dp[0].grad[0] == 0).all()                   # padding_idx row


@pytest.mark.parametrize('d,N', [(64, 1), (128, 100), (256, 7)])
def test_sampled_softmax_matches_torch(dev, d, N):
    from recbole_amd.model.sequential_recommender.sasrec import _SampledSoftmaxFn
    g = torch.Generator().manual_seed(N)
    nI, B = 500, 61
    S = torch.randn(B, d, generator=g) * 0.3
    E = torch.randn(nI, d, generator=g) * 0.3
    pos = torch.randint(1, nI, (B,), generator=g)
    neg = torch.randint(1, nI, (N * B,), generator=g)
    Sp, Ep = torch.nn.Parameter(S.clone()), torch.nn.Parameter(E.clone())
    items = torch.cat([pos.view(1, B), neg.view(N, B)], 0).T
    logits = (Sp.unsqueeze(1) * Ep[items]).sum(-1)
    loss = torch.nn.functional.cross_entropy(logits, torch.zeros(B, dtype=torch.long))
    loss.backward()
    Sd, Ed = torch.nn.Parameter(S.to(dev)), torch.nn.Parameter(E.to(dev))
    ld = _SampledSoftmaxFn.apply(Sd, Ed, pos.to(dev), neg.to(dev))
    ld.backward()
    np.testing.assert_allclose(ld.item(), loss.item(), rtol=1e-5)
    torch.testing.assert_close(Sd.grad.cpu(), Sp.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(Ed.grad.cpu(), Ep.grad, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('loss_type,neg', [('CE', 0), ('BPR', 1), ('SSM', 20)])
def test_sasrec_loss_grads_match_oracle(tmp_path, loss_type, neg):
    config, train, valid, test, model = _pipeline(tmp_path, loss_type=loss_type,
                                                  training_neg_sample_num=neg)
    ref = _oracle(model)
    b = next(iter(train))
    loss = model.calculate_loss(b)
    loss.backward()
    c = {k: v.cpu() for k, v in b.interaction.items()}
    lr_ = ref.calculate_loss(c['item_id_list'], c['item_length'], c['item_id'],
                             c.get('neg_item_id'), loss_type)
    lr_.backward()
    np.testing.assert_allclose(loss.item(), lr_.item(), rtol=1e-4)
    refp = dict(ref.named_parameters())
    for name, p in model.named_parameters():
        torch.testing.assert_close(p.grad.cpu(), refp[name].grad, rtol=1e-4, atol=1e-6,
                                   msg=name)


def test_sasrec_train_and_eval(tmp_path):
    """Adam steps vs torch Adam on the oracle; fused K6 sequential full-sort eval
    vs the generic full_sort_predict + mask + swap + topk sequence; sampled
    (uni1000) validation runs."""
    from recbole_amd.trainer import Trainer
    config, train, valid, test, model = _pipeline(tmp_path)
    ref = _oracle(model)
    opt = torch.optim.Adam(ref.parameters(), lr=config['learning_rate'])
    trainer = Trainer(config, model)
    for b in list(train)[:4]:
        trainer.optimizer.zero_grad()
        loss = model.calculate_loss(b)
        loss.backward()
        trainer.optimizer.step()
        c = {k: v.cpu() for k, v in b.interaction.items()}
        opt.zero_grad()
        lr_ = ref.calculate_loss(c['item_id_list'], c['item_length'], c['item_id'])
        lr_.backward()
        opt.step()
        np.testing.assert_allclose(loss.item(), lr_.item(), rtol=1e-4)
    trainer.optimizer.flush()
    refp = dict(ref.named_parameters())
    for name, p in model.named_parameters():
        torch.testing.assert_close(p.detach().cpu(), refp[name].detach(), rtol=1e-3, atol=2e-5,
                                   msg=name)
    fused = trainer.evaluate(test, load_best_model=False)
    config['fused_eval'] = False
    generic = trainer.evaluate(test, load_best_model=False)
    for k in fused:
        assert fused[k] == pytest.approx(generic[k], abs=2e-4), k
    res = trainer.evaluate(valid, load_best_model=False)
    assert 0.0 <= res['hit@10'] <= 1.0


def test_run_recbole_sasrec(tmp_path):
    from tests.test_gpu_e2e import _write_dataset
    from recbole_amd.quick_start import run_recbole
    root = _write_dataset(str(tmp_path), 'synth', n_users=80, n_items=120, n_inter=3000)
    res = run_recbole(model='SASRec', dataset='synth', config_dict={
        'data_path': root, 'epochs': 1, 'checkpoint_dir': str(tmp_path / 'saved'),
        'load_col': {'inter': ['user_id', 'item_id', 'timestamp']}, 'show_progress': False,
        'MAX_ITEM_LIST_LENGTH': 12, 'training_neg_sample_num': 0})
    assert 0.0 <= res['test_result']['hit@10'] <= 1.0


def test_fused_sampled_eval_matches_generic(tmp_path):
    """uni1000 validation (the fork's switch): K9c rank-of-positive on one encoding
    per sequence vs the reference sequence (1+N copies through predict, flip + topk)
    row by row: the same negatives (the per-row walk), and the positive's top-K
    position equal where no sampled item ties it; where copies of the positive item
    tie it exactly (torch.topk leaves their order unspecified) the generic position
    lies in [#greater, #greater-or-equal] and K9c reports #greater-or-equal. Then
    the full fused evaluation leaves the walk pointer where the generic one does."""
    from recbole_amd._native import lib, ptr, stream_handle
    from recbole_amd.trainer import Trainer
    config, train, valid, test, model = _pipeline(tmp_path)
    tr = Trainer(config, model)
    for b in list(train)[:3]:
        tr.optimizer.zero_grad()
        model.calculate_loss(b).backward()
        tr.optimizer.step()
    model.eval()
    dev = config['device']
    sm = valid.sampler
    sm.to_device(dev)
    L, m, K = sm.random_list_length, valid.neg_sample_by, 10
    pr_start = sm.random_pr
    ties = 0
    with torch.no_grad():
        for start in range(0, valid.pr_end, valid.step):
            pr0 = sm.random_pr
            valid.pr = start
            b = valid._next_batch_data()
            items = b['item_id'].view(-1, 1 + m)
            sc = model.predict(b.to(dev)).view(-1, 1 + m)
            _, ti = torch.topk(torch.flip(sc, dims=[-1]), K)
            sm.random_pr = pr0
            inter = valid.augmentation(slice(start, start + valid.step)).to(dev)
            n = inter['user_id'].numel()
            idx = (sm._pr_dev + torch.arange(n * m, device=dev)) % L
            neg = sm._rl_dev[idx].to(torch.int64)
            sm._pr_dev.copy_((sm._pr_dev + n * m) % L)
            assert torch.equal(neg.view(n, m).cpu(), items[:, 1:].cpu())
            S = model.fused_query_vectors(inter).contiguous()
            E = model.item_embedding.weight.detach()
            rank = torch.empty(n, dtype=torch.int32, device=dev)
            lib().mirec_rank_of_pos_f32(ptr(S), ptr(E), E.shape[0], E.shape[1],
                                        ptr(inter['item_id'].contiguous()), ptr(neg), n, m,
                                        ptr(rank), stream_handle())
            for r in range(n):
                g = sc[r]
                gt, ge = int((g[1:] > g[0]).sum()), int((g[1:] >= g[0]).sum())
                hit = (ti[r] >= m).nonzero()
                gpos = int(hit[0]) if len(hit) else None
                # the two paths encode the sequence in different batches: scores may
                # differ by rounding, so near-ties of OTHER items may fall either way
                other = items[r, 1:] != items[r, 0]
                near = int((((g[1:] - g[0]).abs() <= 1e-5 * g[0].abs() + 1e-6) & other).sum())
                assert abs(int(rank[r]) - ge) <= near, (int(rank[r]), gt, ge, near)
                if gt == ge and near == 0:
                    assert gpos == (ge if ge < K else None)
                else:
                    ties += 1
                    assert gpos is None or gt <= gpos <= ge
    pr_generic = sm.random_pr
    sm.random_pr = pr_start
    valid.pr = 0
    tr.evaluate(valid, load_best_model=False)           # the fused path end to end
    assert sm.random_pr == pr_generic


@pytest.mark.parametrize('d', [32, 64, 128, 256])
def test_add_layernorm_and_gelu_match_torch(dev, d):
    """K9d LayerNorm(a + b) forward / backward and the GELU kernels against torch
    fp32 (nn.LayerNorm over the materialised sum; the erf formula of layers.py)."""
    from recbole_amd.model.layers import _AddLNFn, _GeluFn
    g = torch.Generator(device='cpu').manual_seed(d)
    n = 3000
    a = torch.randn(n, d, generator=g).to(dev).requires_grad_()
    b = torch.randn(n, d, generator=g).to(dev).requires_grad_()
    ln = torch.nn.LayerNorm(d, eps=1e-12).to(dev)
    with torch.no_grad():
        ln.weight.copy_(torch.randn(d, generator=g))
        ln.bias.copy_(torch.randn(d, generator=g))
    gy = torch.randn(n, d, generator=g).to(dev)
    y = _AddLNFn.apply(a, b, ln.weight, ln.bias, 1e-12)
    ga, gb, gw, gbias = torch.autograd.grad(y, (a, b, ln.weight, ln.bias), gy)
    a2, b2 = a.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    y2 = ln(a2 + b2)
    ra, rb, rw, rbias = torch.autograd.grad(y2, (a2, b2, ln.weight, ln.bias), gy)
    for got, ref in ((y, y2), (ga, ra), (gb, rb), (gw, rw), (gbias, rbias)):
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
    x = (torch.randn(n, d, generator=g) * 3).to(dev).requires_grad_()
    yg = _GeluFn.apply(x)
    (gx,) = torch.autograd.grad(yg, x, gy)
    x2 = x.detach().clone().requires_grad_()
    yr = x2 * 0.5 * (1.0 + torch.erf(x2 / math.sqrt(2.0)))
    (rx,) = torch.autograd.grad(yr, x2, gy)
    torch.testing.assert_close(yg, yr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(gx, rx, rtol=1e-4, atol=1e-5)
    # the float4 kernels (n % 4 == 0, aligned) and the one-element kernels (an odd
    # count) compute the same bits per element
    from recbole_amd._native import check, lib, ptr
    xs, gs = x.detach().reshape(-1), gy.reshape(-1).contiguous()
    m = xs.numel() - 1
    y1, d1 = torch.empty(m, device=dev), torch.empty(m, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    check(lib().mirec_gelu_fwd_f32(ptr(xs), m, ptr(y1), st), 'gelu_fwd')
    check(lib().mirec_gelu_bwd_f32(ptr(xs), ptr(gs), m, ptr(d1), st), 'gelu_bwd')
    assert torch.equal(y1, yg.detach().reshape(-1)[:m])
    assert torch.equal(d1, gx.reshape(-1)[:m])


def test_scale_by_in_place(dev):
    """mirec_scale_by_f32 (the SSM backward's gI * g in place): bit for bit torch's
    multiply, and an untouched buffer when g == 1."""
    from recbole_amd._native import check, lib, ptr
    g = torch.Generator().manual_seed(3)
    x = torch.randn(3001, 128, generator=g).to(dev)
    x[0, :4] = torch.tensor([0.0, -0.0, float('inf'), -float('inf')])
    st = torch.cuda.current_stream(dev).cuda_stream
    for s in (1.0, 0.37, -2.0):
        y = x.clone()
        sv = torch.tensor([s], device=dev)
        check(lib().mirec_scale_by_f32(ptr(y), y.numel(), ptr(sv), st), 'scale_by')
        torch.cuda.synchronize(dev)
        assert torch.equal(y.view(torch.int32), (x * sv).view(torch.int32))
