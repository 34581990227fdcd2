"""BASELINE.json configurations at their real sizes (beyond C1 / C2, which
tests/test_gpu_chain.py covers end to end from the seed):

  C3  K9b sampled softmax over the full 3,000,001-row item table (d = 128,
      B = 2,048 sequences, 100 negatives, hot and duplicated ids) against fp64 torch.
  C4  DeepFM over the full Criteo-shape vocabulary (26 token fields summing to
      33,000,026 rows incl. PADs, 13 float fields, d = 16, B = 2,048): K8 forward,
      fused BCE, backward (K8 + K2 grouping of 53,248 contributions over 33 M
      rows), against the oracle's torch-CPU DeepFM (dropout 0).
  C5  K6 full-sort top-10 against all 5,000,001 items at d = 256 for a user
      sample with history masks, against torch-CPU scores + the reference's
      mask/flip/topk; K7 propagation over the C5 graph (10 M x 5 M, ~94 M edges,
      d = 256) checked by size-independent properties: sampled rows against an
      fp64 restatement (incl. the hub rows) and the symmetry <Ax, y> = <x, Ay>.
Tolerances: fp32 1e-4 relative (north_star), gradients 1e-4 relative + small
absolute; top-K ids identical except at exact score ties."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _bench_models():
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import bench_models
    return bench_models


def test_c3_sampled_softmax_full_item_table(dev):
    from recbole_amd.model.sequential_recommender.sasrec import _SampledSoftmaxFn
    I, d, B, N = 3_000_001, 128, 2048, 100
    g = torch.Generator(device=dev).manual_seed(3)
    W = torch.nn.Parameter(torch.randn(I, d, device=dev, generator=g) * 0.05)
    S = torch.nn.Parameter(torch.randn(B, d, device=dev, generator=g) * 0.5)
    pos = torch.randint(1, I, (B,), device=dev, generator=g)
    neg = torch.randint(1, I, (N * B,), device=dev, generator=g)
    neg[:3000] = 7                                   # a hot row (Zipf head)
    neg[5000:5100] = pos[:100]                       # sampled copies of the positive
    pos[-1] = I - 1                                  # last row of the table
    loss = _SampledSoftmaxFn.apply(S, W, pos, neg)
    loss.backward()

    items = torch.cat([pos.view(1, B), neg.view(N, B)], 0).T.cpu()        # [B, 1+N]
    rows = W.detach()[items.to(dev)].cpu().double().requires_grad_(True)
    Sd = S.detach().cpu().double().requires_grad_(True)
    logits = (Sd.unsqueeze(1) * rows).sum(-1)
    ref = torch.nn.functional.cross_entropy(logits, torch.zeros(B, dtype=torch.long))
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item())
    torch.testing.assert_close(S.grad.cpu().double(), Sd.grad, rtol=1e-4, atol=1e-8)
    touched = torch.unique(items)
    dW = torch.zeros(I, d, dtype=torch.float64).index_add_(0, items.reshape(-1),
                                                           rows.grad.reshape(-1, d))
    got = W.grad.cpu()
    torch.testing.assert_close(got[touched].double(), dW[touched], rtol=1e-4, atol=1e-8)
    mask = torch.ones(I, dtype=torch.bool)
    mask[touched] = False
    assert not got[mask].any()                       # untouched rows: exactly zero


def test_c4_deepfm_full_vocabulary(dev):
    bm = _bench_models()
    from recbole_amd.config import Config
    from recbole_amd.data.interaction import Interaction
    from recbole_amd.model.context_aware_recommender import DeepFM
    from recbole_amd.utils import FeatureType
    vocab = bm.c4_vocab()
    assert sum(vocab) == 33_000_000
    B, d = 2048, 16
    types, nums = {'label': FeatureType.FLOAT}, {'label': 1}
    for j in range(13):
        types[f'I{j}'], nums[f'I{j}'] = FeatureType.FLOAT, 1
    for j, v in enumerate(vocab):
        types[f'C{j}'], nums[f'C{j}'] = FeatureType.TOKEN, v + 1
    config = Config(model='DeepFM', dataset='criteo-synth', config_dict={
        'embedding_size': d, 'load_col': None, 'state': 'ERROR', 'data_path': ROOT,
        'dropout_prob': 0.0})
    config['device'] = dev
    torch.manual_seed(2020)
    model = DeepFM(config, bm.StubDataset(types, nums)).to(dev)
    rng = np.random.default_rng(2020)
    cols = {'label': torch.as_tensor((rng.random(B) < 0.256).astype(np.float32))}
    for j in range(13):
        x = rng.lognormal(0.0, 2.0, B)
        cols[f'I{j}'] = torch.as_tensor(((x - x.min()) / (x.max() - x.min())).astype(np.float32))
    for j, v in enumerate(vocab):
        ids = bm._zipf_ids(rng, 1.1, B, v)
        ids[:3] = [v, 1, v]                          # last row of each field + repeats
        cols[f'C{j}'] = torch.as_tensor(ids)
    inter = Interaction(cols).to(dev)
    assert model.token_embedding_table.embedding.weight.shape[0] == 33_000_026
    loss = model.calculate_loss(inter)
    loss.backward()
    with torch.no_grad():
        pred = model.predict(inter).cpu()

    ref = cpu_ref.DeepFMCPU(model.token_field_names, model.token_field_dims, [], [],
                            model.float_field_names, d, model.mlp_hidden_size, 0.0)
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    cb = {k: v.cpu() for k, v in inter.interaction.items()}
    lr_ = ref.calculate_loss(cb, cb['label'])
    lr_.backward()
    np.testing.assert_allclose(loss.item(), lr_.item(), rtol=1e-4)
    with torch.no_grad():
        torch.testing.assert_close(pred, ref.forward(cb), rtol=1e-4, atol=1e-6)
    refp = dict(ref.named_parameters())
    offs = np.r_[0, np.cumsum([v + 1 for v in vocab])[:-1]]
    rows = torch.as_tensor(np.unique(np.concatenate(
        [cols[f'C{j}'].numpy() + offs[j] for j in range(26)])))
    for name, p in model.named_parameters():
        gp, gr = p.grad, refp[name].grad
        if gp.shape[0] >= 33_000_026:                # token tables: touched rows + zeros
            gp = gp.cpu()
            torch.testing.assert_close(gp[rows], gr[rows], rtol=1e-4, atol=1e-6, msg=name)
            keep = torch.ones(gp.shape[0], dtype=torch.bool)
            keep[rows] = False
            assert not gp[keep].any(), name
        else:
            torch.testing.assert_close(gp.cpu(), gr, rtol=1e-4, atol=1e-6, msg=name)


def test_c5_fullsort_all_items_d256(dev):
    from recbole_amd import ops
    I, d, n, K = 5_000_001, 256, 48, 10
    g = torch.Generator(device=dev).manual_seed(5)
    EI = torch.randn(I, d, device=dev, generator=g) * 0.05
    Uq = torch.randn(n, d, device=dev, generator=g) * 0.05
    rng = np.random.default_rng(5)
    hist = [np.unique(rng.integers(1, I, rng.integers(0, 3000))) for _ in range(n)]
    scores = (Uq.cpu().double() @ EI.cpu().double().T)               # [n, I] fp64
    top_cand = torch.topk(scores, 40, dim=1).indices.numpy()
    for r in range(0, n, 3):                                          # mask some true top items
        hist[r] = np.union1d(hist[r], top_cand[r, :5])
    posl = [np.setdiff1d(np.r_[top_cand[r, 10:12], rng.integers(1, I, 2)], hist[r])
            for r in range(n)]
    T_ = lambda x, dt: torch.as_tensor(np.asarray(x, dtype=dt), device=dev)
    hp = np.r_[0, np.cumsum([len(h) for h in hist])]
    pp = np.r_[0, np.cumsum([len(p) for p in posl])]
    out = ops.fullsort_topk(Uq, EI, K, hist_ptr=T_(hp, np.int64),
                            hist_cols=T_(np.concatenate(hist), np.int32),
                            pos_ptr=T_(pp, np.int64), pos_cols=T_(np.concatenate(posl), np.int32))
    exp_flags, exp_ids = cpu_ref.full_sort_pos_idx(scores.float(), [h.tolist() for h in hist],
                                                   [p.tolist() for p in posl], K)
    got = out['ids'].cpu().numpy()
    assert np.array_equal(got, exp_ids)
    assert np.array_equal(out['pos_flags'].cpu().numpy().astype(bool), exp_flags)


def test_c5_propagation_properties(dev):
    bm = _bench_models()
    from recbole_amd import ops
    from recbole_amd.model.general_recommender.lightgcn import norm_adj_csr, propagate
    U, I, d = 10_000_001, 5_000_001, 256
    u, i = bm.make_c5_graph(U - 1, I - 1, 100_000_000)
    print(f'C5 graph: {len(u):,} edges', flush=True)
    rp, cols, vals = norm_adj_csr(u, i, U, I)
    print('C5 normalised adjacency built', flush=True)
    del u, i
    plan = ops.SpmmPlan(rp, cols, vals, device=dev)
    g = torch.Generator(device=dev).manual_seed(11)
    XU = torch.randn(U, d, device=dev, generator=g)
    XI = torch.randn(I, d, device=dev, generator=g)
    yu, yi = propagate(plan, XU, XI, 1)             # mean of [X, A X] (layer-mean epilogue)
    # rows: a random sample + the hub rows (largest degrees: split into many units)
    deg = np.diff(rp)
    rng = np.random.default_rng(0)
    sample = np.unique(np.r_[rng.integers(0, U + I, 3000), np.argsort(deg)[-4:]])
    colsd = torch.as_tensor(cols.astype(np.int64), device=dev)
    valsd = torch.as_tensor(vals, device=dev).double()
    X = lambda idx: torch.where((idx < U).unsqueeze(1), XU[idx.clamp(max=U - 1)],
                                XI[(idx - U).clamp(min=0)]).double()
    for r in sample:
        a, b = int(rp[r]), int(rp[r + 1])
        acc = torch.zeros(d, dtype=torch.float64, device=dev)
        for s in range(a, b, 1 << 20):                                # hub rows in pieces
            e = min(b, s + (1 << 20))
            acc += (valsd[s:e].unsqueeze(1) * X(colsd[s:e])).sum(0)
        ref = (X(torch.tensor([r], device=dev))[0] + acc) / 2
        got = (yu[r] if r < U else yi[r - U]).double()
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-5)
    # symmetry of the normalised adjacency: <A x, y> = <x, A y> (one column each)
    del XU, XI, yu, yi
    x = torch.randn(U + I, 1, device=dev, generator=g)
    y = torch.randn(U + I, 1, device=dev, generator=g)
    Ax = 2 * torch.cat(propagate(plan, x[:U].expand(U, 32).contiguous(),
                                 x[U:].expand(I, 32).contiguous(), 1))[:, 0] - x[:, 0]
    Ay = 2 * torch.cat(propagate(plan, y[:U].expand(U, 32).contiguous(),
                                 y[U:].expand(I, 32).contiguous(), 1))[:, 0] - y[:, 0]
    lhs = float((Ax.double() * y[:, 0].double()).sum())
    rhs = float((x[:, 0].double() * Ay.double()).sum())
    assert abs(lhs - rhs) <= 1e-4 * (abs(lhs) + abs(rhs) + 1.0)
