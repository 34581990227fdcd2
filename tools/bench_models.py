"""Per-configuration measurements of the model rows of SURVEY.md §8 beyond the
C2 headline (bench.py): one JSON line per configuration, 1 GPU.

  C3  SASRec, Amazon-Books shape: I = 3,000,000 (+PAD), L = 50, d = 128, 2 layers,
      2 heads, inner 256, 100 uniform negatives per sequence from the device walk
      (RepeatableSampler, K4), sampled-softmax loss (K9b), dense Adam over every
      parameter (the reference's optim.Adam on nn.Embedding(sparse=False)).
      Unit: sequences/s; dominant-kernel rooflines from HIP events.
  C4  DeepFM, Criteo shape: 13 float + 26 token fields, vocabularies summing to
      33,000,000 (10M, 8M, 5M, 4M, 3M, then geometric down to 3), Zipf(1.1) ids,
      d = 16, MLP 624-128-128-128-1 (dropout 0.2), BCE, B = 2,048, dense Adam.
      Unit: samples/s.
  C5  LightGCN, 10M users x 5M items, 100M edges (Zipf items, Zipf-like user
      degrees), d = 256, 2 layers: propagation (K7) once, then full-sort top-10
      (K6) of a bounded sample of users against all 5M items. Unit: users/s.

Synthetic data (seeded numpy PCG64 / torch generators), random init. Each step is
the Trainer's generic step: zero_grad -> calculate_loss -> backward -> FusedAdam.
Usage: python tools/bench_models.py [--configs C3,C4,C5] [--steps K] [--warmup W]
       [--scale S] (S < 1 shrinks the tables / graph for a quick run).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MFMA_F32_PEAK_TFLOPS = 157.3   # fp32 matrix peak (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md
FP32_PEAK_TFLOPS = 157.3   # fp32 MFMA / vector peak
CPU_BASELINE = True
ADAM_MODE = 'deferred'
GRAPH_STEP = True


class StubDataset:
    """The dataset surface a model constructor reads (fields / field2type / num)."""

    def __init__(self, types, nums, uid=None, iid=None):
        self.field2type = dict(types)
        self._num = dict(nums)
        self.uid_field, self.iid_field = uid, iid

    def fields(self, ftype=None, source=None):
        return [f for f in self.field2type if ftype is None or self.field2type[f] in ftype]

    def num(self, field):
        return self._num[field]


MARKERS = os.environ.get('MODELS_MARKERS') == '1'   # trace markers (tools/step_breakdown.py)


def _timed(fn, steps, warmup, opt=None):
    """Mean wall time per step over `steps` steps; with a deferred optimizer the
    flush that completes every row is inside the timed region (no work skipped).
    MODELS_MARKERS=1: two 1-cycle spin kernels bracket the timed region in a kernel
    trace (tools/step_breakdown.py)."""
    for _ in range(warmup):
        fn()
    if opt is not None:
        opt.flush()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if MARKERS:
        torch.cuda._sleep(1)
    for _ in range(steps):
        fn()
    if opt is not None:
        opt.flush()
    if MARKERS:
        torch.cuda._sleep(1)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def _window_events(step, names, steps=8):
    """HIP events around the named native launches (ops.timed_launch) over `steps`
    eager steps enqueued behind a spin kernel (the host enqueues the whole window
    before the GPU reaches it, so an event pair brackets its kernel only). Returns
    {name: (launches per step, mean launch us)}."""
    from recbole_amd import ops
    ops.KERNEL_EVENTS = {n: [] for n in names}
    try:
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2.4e3 * 1500 * steps))
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ev = ops.KERNEL_EVENTS
    finally:
        ops.KERNEL_EVENTS = None
    return {n: (len(v) / steps, float(np.mean([a.elapsed_time(b) * 1e3 for a, b in v])))
            for n, v in ev.items() if v}


def _pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` (a name, or a tuple of names whose per-launch
    traffic is summed: one call's launches) from the newest committed models PMC summary
    (profiles/r*_models_pmc.json, tools/models_pmc.py), or None when that summary did not
    trace every one of them (never an older file's entry for a kernel the step no longer
    runs)."""
    import glob
    import json
    paths = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_models_pmc.json')))
    if not paths:
        return None, None
    recs = json.load(open(paths[-1]))
    names = (kernel,) if isinstance(kernel, str) else tuple(kernel)
    got = [recs.get(k) for k in names]
    if any(r is None for r in got):
        return None, None
    return sum(r['traffic'] for r in got), os.path.basename(paths[-1])


def _step_breakdown(config):
    """The committed per-step kernel breakdown of the timed step (rocprofv3 kernel
    trace, tools/step_breakdown.py): profiles/r*_<config>_step.json, newest."""
    import glob
    import json
    paths = sorted(glob.glob(os.path.join(ROOT, 'profiles', f'r*_{config}_step.json')))
    if not paths:
        return None
    r = json.load(open(paths[-1]))
    return {'source': os.path.basename(paths[-1]), 'wall_us_per_step': r['wall_us_per_step'],
            'kernel_us_per_step': r['kernel_us_per_step'],
            'launches_per_step': r['launches_per_step'], 'dominant': r['dominant'],
            'top5': [{k: x[k] for k in ('kernel', 'us_per_step', 'launches_per_step')}
                     for x in r['kernels'][:5]]}


def _event_time(fn, reps=10):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    return float(np.median(ts))


def _zipf_ids(rng, a, n, vmax):
    """Zipf(a) ranks clipped to [1, vmax] (id 0 is [PAD])."""
    return np.minimum(rng.zipf(a, n), vmax).astype(np.int64)


# ----------------------------------------------------------------------------- C4
def c4_vocab(total=33_000_000):
    big = [10_000_000, 8_000_000, 5_000_000, 4_000_000, 3_000_000]
    rest = total - sum(big)
    r = 0.55
    w = r ** np.arange(21)
    sizes = np.maximum(np.round(w / w.sum() * rest).astype(np.int64), 3)
    sizes[0] += rest - sizes.sum()
    return big + sizes.tolist()


def bench_c4(dev, steps, warmup, scale=1.0, B=2048, d=16, n_batches=16):
    from recbole_amd.config import Config
    from recbole_amd.model.context_aware_recommender import DeepFM
    from recbole_amd.model.context import _CtxFMFn
    from recbole_amd.trainer.optim import FusedAdam
    from recbole_amd.data.interaction import Interaction
    from recbole_amd.utils import FeatureType
    vocab = [max(3, int(v * scale)) for v in c4_vocab()]
    types = {'label': FeatureType.FLOAT}
    nums = {'label': 1}
    for j in range(13):
        types[f'I{j}'], nums[f'I{j}'] = FeatureType.FLOAT, 1
    for j, v in enumerate(vocab):
        types[f'C{j}'], nums[f'C{j}'] = FeatureType.TOKEN, v + 1      # + [PAD]
    config = Config(model='DeepFM', dataset='criteo-synth', config_dict={
        'embedding_size': d, 'load_col': None, 'state': 'ERROR', 'data_path': ROOT})
    config['device'] = dev
    torch.manual_seed(2020)
    model = DeepFM(config, StubDataset(types, nums)).to(dev)
    rng = np.random.default_rng(2020)
    batches = []
    for _ in range(n_batches):
        cols = {'label': torch.as_tensor((rng.random(B) < 0.256).astype(np.float32))}
        for j in range(13):
            x = rng.lognormal(0.0, 2.0, B)
            cols[f'I{j}'] = torch.as_tensor(((x - x.min()) / (x.max() - x.min())).astype(
                np.float32))
        for j, v in enumerate(vocab):
            cols[f'C{j}'] = torch.as_tensor(_zipf_ids(rng, 1.1, B, v))
        batches.append(Interaction(cols).to(dev))
    opt = FusedAdam(model.parameters(), lr=1e-3)
    if ADAM_MODE == 'deferred':
        opt.enable_deferred(model.deferred_tables())
    it = [0]
    gs = None
    if GRAPH_STEP:                 # the Trainer's captured step (trainer/graph_step.py)
        from recbole_amd.trainer.graph_step import GraphedTrainStep
        gs = GraphedTrainStep(model, opt)

    def step():
        b = batches[it[0] % n_batches]
        it[0] += 1
        if gs is not None:
            gs.step(b)
            return
        opt.zero_grad()
        loss = model.calculate_loss(b)
        loss.backward()
        opt.step()

    t = _timed(step, steps, warmup, opt)
    V = sum(nums[f'C{j}'] for j in range(26))
    # the timed step's dominant kernel (profiles/r03_C4_step.json: ctx_fm_bwd_kernel, K8
    # backward), timed live on its stream over eager steps of the same batches.
    # Algorithmic bytes per launch: concat + g_concat read (39 fields x d floats per
    # sample), g_fm read, gradient rows written (26 token + 13 float fields x d floats)
    # and the first-order gradients (39 floats) per sample.
    def eager():
        b = batches[it[0] % n_batches]
        it[0] += 1
        opt.zero_grad()
        model.calculate_loss(b).backward()
        opt.step()
    ev = _window_events(eager, ('ctx_fm_bwd', 'ctx_fm_fwd', 'mlp_fwd', 'mlp_bwd', 'k2_blocks'))
    opt.flush()
    bwd_n, bwd_us = ev['ctx_fm_bwd']
    fwd_n, fwd_us = ev['ctx_fm_fwd']
    # K10 (the MLP on fp32 MFMA): 2 FLOPs per multiply-add of every layer, per launch
    dims = [39 * d, 128, 128, 128, 1]
    mlp_flops = 2 * B * sum(a * b_ for a, b_ in zip(dims[:-1], dims[1:]))
    mf_n, mf_us = ev['mlp_fwd']
    mb_n, mb_us = ev['mlp_bwd']
    k2_n, k2_us = ev['k2_blocks']
    nk = 26 * B                                 # token keys of a step
    k2_bytes = nk * (8 + 4 + 4 + 4)             # keys read; perm, uniq, seg written
    bwd_bytes = B * (2 * 39 * d * 4 + 4 + 39 * d * 4 + 39 * 4)
    fwd_bytes = B * (26 * (d * 4 + 4 + 8) + 13 * 4 + 39 * d * 4 + 4 + 26 * 8)
    traffic, tsrc = _pmc_traffic('ctx_fm_bwd_kernel')
    cpu = None
    if CPU_BASELINE:
        from oracle import cpu_baseline as cb
        thr, how = cb.host_threads()
        runs = [cb.time_deepfm_steps(batches, [f'C{j}' for j in range(26)],
                                     [nums[f'C{j}'] for j in range(26)],
                                     [f'I{j}' for j in range(13)], d, [128, 128, 128],
                                     steps=20, warmup=2, threads=thr) for _ in range(3)]
        sps, used = float(np.median([r[0] for r in runs])), runs[0][2]
        vals = np.array([r[0] for r in runs])
        cpu = {'value': round(sps, 1), 'unit': 'samples/s', 'cores': used, 'kind': 'port',
               'threads_derivation': how, 'runs': [round(r[0], 1) for r in runs],
               'cv': round(float(vals.std() / vals.mean()), 4),
               'sample': f'median of 3 runs of 2 warm-up + 20 timed C4 steps of the oracle '
                         f'restatement on torch CPU (DeepFMCPU + dense optim.Adam over every '
                         f'table), {sum(r[1] for r in runs):.1f} s timed in all; bounded below '
                         f'the 20 + 200 of SURVEY.md 8d: a CPU step moves the 2.1 GB tables '
                         f'several times (~1 s), and the run-to-run spread (cv) is reported'}
    fwd_k = ('mlp_l0_fwd_kernel', 'mlp_fwd_kernel')
    wide = os.environ.get('MIREC_MLP_WIDE_FWD') == '1'       # csrc/mlp.hip wide_fwd_on
    k10 = {'kernel': ('mlp_l0_fwd_kernel + mlp_fwd_kernel (K10 forward: the wide layer 0 over '
                      'the whole chip, then layers 1.. + deep_predict_layer; dropout, ReLU; '
                      'one event pair around both launches)') if wide else
                     ('mlp_fwd_kernel (K10 forward: every layer + deep_predict_layer in one '
                      'launch, one 16-row block per CU; dropout, ReLU)'), 'bound': 'mfma',
           'achieved': round(mlp_flops / (mf_us * 1e-6) / 1e12, 2),
           'peak': MFMA_F32_PEAK_TFLOPS, 'unit': 'TFLOP/s',
           'frac': round(mlp_flops / (mf_us * 1e-6) / 1e12 / MFMA_F32_PEAK_TFLOPS, 4),
           'traffic': _pmc_traffic(fwd_k)[0],
           'traffic_source': _pmc_traffic(fwd_k)[1],
           'flops_per_launch': mlp_flops, 'launch_us': round(mf_us, 2),
           'launches_per_step': mf_n,
           'timing': 'HIP events around each launch on its stream, 8 eager steps'}
    k2 = {'kernel': 'segsort_radix8_kernel (K2 grouping of the 26 token fields: one chained '
                    'launch, keys formed from the field columns; latency-bound)',
          'bound': 'hbm', 'achieved': round(k2_bytes / (k2_us * 1e-6) / 1e9, 1),
          'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
          'frac': round(k2_bytes / (k2_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5),
          'traffic': _pmc_traffic('segsort_radix8_kernel')[0],
          'traffic_source': _pmc_traffic('segsort_radix8_kernel')[1],
          'bytes_per_launch': k2_bytes, 'launch_us': round(k2_us, 2), 'launches_per_step': k2_n,
          'timing': 'HIP events around each call on its stream, 8 eager steps'}
    # the roofline of the timed step's dominant kernel (committed trace breakdown)
    sb = _step_breakdown('C4')
    dom = (sb or {}).get('dominant', {}).get('kernel', '') if sb else ''
    roof = k2 if 'segsort' in dom else k10
    return {
        'cpu_baseline': cpu,
        'adam_mode': ADAM_MODE, 'graph_step': bool(GRAPH_STEP),
        'config': 'C4', 'metric': 'train samples/s', 'value': round(B / t, 1),
        'unit': 'samples/s', 'ms_per_step': round(t * 1e3, 3), 'batch': B, 'steps': steps,
        'workload': f'DeepFM Criteo-shape: 13 float + 26 token fields, vocab {V:,} '
                    f'(incl. PADs), d={d}, MLP 624-128-128-128-1, dropout 0.2, BCE, dense Adam',
        'dtype': 'fp32', 'data': 'synthetic (Zipf(1.1) ids, log-normal floats, seeded)',
        'step_breakdown': _step_breakdown('C4'),
        'roofline': roof,
        'k10_fwd': k10,
        'k2_grouping': k2,
        'k10_bwd': {'kernel': 'mlp_bwd_data_kernel + mlp_bwd_wide_kernel (K10 backward: layers '
                              'L-1..1 in row blocks, then layer 0\'s data gradient and every '
                              'weight gradient over the whole chip; one event pair around both '
                              'launches)', 'bound': 'mfma',
                    'traffic': _pmc_traffic(('mlp_bwd_data_kernel', 'mlp_bwd_wide_kernel'))[0],
                    'achieved': round(2 * mlp_flops / (mb_us * 1e-6) / 1e12, 2),
                    'peak': MFMA_F32_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                    'frac': round(2 * mlp_flops / (mb_us * 1e-6) / 1e12 / MFMA_F32_PEAK_TFLOPS, 4),
                    'flops_per_call': 2 * mlp_flops, 'call_us': round(mb_us, 2)},
        'k8_bwd': {'kernel': 'ctx_fm_bwd_kernel<16> (K8 backward)', 'bound': 'hbm',
                     'achieved': round(bwd_bytes / (bwd_us * 1e-6) / 1e9, 1),
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(bwd_bytes / (bwd_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                     'traffic': traffic, 'traffic_source': tsrc,
                     'bytes_per_launch': bwd_bytes, 'launch_us': round(bwd_us, 2),
                     'launches_per_step': bwd_n,
                     'timing': 'HIP events around each launch on its stream, 8 eager steps'},
        'k8_fwd': {'kernel': 'ctx_fm_fwd_kernel<16> (K8 forward: field gather + first order + '
                             'FM)', 'bound': 'hbm',
                   'achieved': round(fwd_bytes / (fwd_us * 1e-6) / 1e9, 1),
                   'unit': 'GB/s', 'bytes_per_launch': fwd_bytes, 'launch_us': round(fwd_us, 2),
                   'launches_per_step': fwd_n},
    }


# ----------------------------------------------------------------------------- C3
def bench_c3(dev, steps, warmup, scale=1.0, B=2048, L=50, d=128, n_neg=100, n_batches=8):
    from recbole_amd import ops
    from recbole_amd.config import Config
    from recbole_amd.data.interaction import Interaction
    from recbole_amd.model.sequential_recommender import SASRec
    from recbole_amd.trainer.optim import FusedAdam
    from recbole_amd.utils import FeatureType
    n_items = max(1000, int(3_000_000 * scale)) + 1
    config = Config(model='SASRec', dataset='books-synth', config_dict={
        'hidden_size': d, 'inner_size': 256, 'n_layers': 2, 'n_heads': 2,
        'MAX_ITEM_LIST_LENGTH': L, 'loss_type': 'SSM', 'training_neg_sample_num': n_neg,
        'state': 'ERROR', 'data_path': ROOT})
    config['device'] = dev
    torch.manual_seed(2020)
    model = SASRec(config, StubDataset({'item_id': FeatureType.TOKEN},
                                       {'item_id': n_items})).to(dev)
    rng = np.random.default_rng(2020)
    batches = []
    for _ in range(n_batches):
        lens = np.minimum(rng.poisson(20, B) + 4, L).astype(np.int64)
        seq = np.zeros((B, L), dtype=np.int64)
        ids = _zipf_ids(rng, 1.1, int(lens.sum()), n_items - 1)
        mask = np.arange(L)[None, :] < lens[:, None]
        seq[mask] = ids
        batches.append(Interaction({
            'item_id_list': torch.as_tensor(seq), 'item_length': torch.as_tensor(lens),
            'item_id': torch.as_tensor(_zipf_ids(rng, 1.1, B, n_items - 1)),
            'user_id': torch.as_tensor(rng.integers(1, 1_000_000, B))}).to(dev))
    random_list = torch.as_tensor(rng.permutation(np.arange(1, n_items)).astype(np.int32),
                                  device=dev)
    pr = torch.zeros(1, dtype=torch.int64, device=dev)
    opt = FusedAdam(model.parameters(), lr=1e-3)
    if ADAM_MODE == 'deferred':
        opt.enable_deferred(model.deferred_tables())
    it = [0]
    gs = None
    if GRAPH_STEP:                 # the Trainer's captured step (trainer/graph_step.py)
        from recbole_amd.trainer.graph_step import GraphedTrainStep
        gs = GraphedTrainStep(model, opt)

    def step():
        b = batches[it[0] % n_batches]
        it[0] += 1
        # the data side (the loader's K4 walk of 100 negatives per sequence) stays eager
        neg = ops.sample_walk(random_list, pr, b['user_id'], n_neg, None, None, 1_000_000, False)
        b.interaction['neg_item_id'] = neg
        if gs is not None:
            gs.step(b)
            return
        opt.zero_grad()
        loss = model.calculate_loss(b)
        loss.backward()
        opt.step()

    t = _timed(step, steps, warmup, opt)
    from recbole_amd.model.sequential_recommender.sasrec import _SampledSoftmaxFn
    b0 = batches[0]
    S = torch.randn(B, d, device=dev)
    W = model.item_embedding.weight
    neg = ops.sample_walk(random_list, pr, b0['user_id'], n_neg, None, None, 1_000_000, False)
    tk = _event_time(lambda: _SampledSoftmaxFn.apply(S, W, b0['item_id'], neg))
    k9_bytes = B * (1 + n_neg) * (d * 4 + 8 + d * 4) + B * d * 4 * 2
    # the timed step's dominant kernel (profiles/r03_C3_step.json): the attention backward
    # of torch's fused scaled_dot_product_attention (a library kernel, 2 launches per step:
    # one per layer), timed live with HIP events at the step's shapes (B x heads x L x
    # d/heads, the model's additive mask, its attention dropout). FLOPs per launch: the
    # flash backward's five L x L x dh matmuls (S recomputed, dV, dP, dQ, dK).
    H = config['n_heads']
    dh = d // H
    seq0 = b0['item_id_list']
    mask = model.get_attention_mask(seq0)
    mha = model.trm_encoder.layer[0].multi_head_attention
    p_drop = mha.attn_dropout.p
    from recbole_amd.model import layers as _layers
    k9e = _layers.attn_k9e_applies(torch.empty(B, L, d, device=dev), mask, H, dh)
    if k9e:   # K9e (csrc/attn.hip), the step's own attention: forward, then backward
        q, k, v = (torch.randn(B, L, d, device=dev, requires_grad=True) for _ in range(3))
        rng = mha._k9e_rng(q.device) if p_drop > 0 else None
        o = _layers._AttnFn.apply(q, k, v, mask, H, p_drop, rng)
        ta_fwd = _event_time(lambda: _layers._AttnFn.apply(q.detach(), k.detach(), v.detach(),
                                                           mask, H, p_drop, rng))
    else:
        q, k, v = (torch.randn(B, H, L, dh, device=dev, requires_grad=True) for _ in range(3))
        o = torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=mask,
                                                             dropout_p=p_drop)
        ta_fwd = None
    go = torch.randn_like(o)
    ta = _event_time(lambda: torch.autograd.grad(o, (q, k, v), go, retain_graph=True))
    attn_flops = 5 * 2 * B * H * L * L * dh
    flops = 86.3e6 * B    # transformer fwd+bwd per sequence
    cpu = None
    if CPU_BASELINE:
        from oracle import cpu_baseline as cb
        thr, how = cb.host_threads()
        runs = [cb.time_sasrec_steps(batches, random_list.cpu().numpy(), n_items, L, d, n_neg,
                                     steps=8, warmup=1, threads=thr) for _ in range(3)]
        sps, used = float(np.median([r[0] for r in runs])), runs[0][2]
        vals = np.array([r[0] for r in runs])
        cpu = {'value': round(sps, 1), 'unit': 'sequences/s', 'cores': used, 'kind': 'port',
               'threads_derivation': how, 'runs': [round(r[0], 1) for r in runs],
               'cv': round(float(vals.std() / vals.mean()), 4),
               'sample': f'median of 3 runs of 1 warm-up + 8 timed C3 steps of the oracle '
                         f'restatement on torch CPU (numpy walk, SASRecCPU + sampled softmax, '
                         f'dense optim.Adam over the 1.5 GB item table), '
                         f'{sum(r[1] for r in runs):.1f} s timed in all; bounded below the '
                         f'20 + 200 of SURVEY.md 8d (~3 s per CPU step), the run-to-run spread '
                         f'(cv) is reported'}
    return {
        'cpu_baseline': cpu,
        'adam_mode': ADAM_MODE,
        'config': 'C3', 'metric': 'train sequences/s', 'value': round(B / t, 1),
        'unit': 'sequences/s', 'ms_per_step': round(t * 1e3, 3), 'batch': B, 'steps': steps,
        'workload': f'SASRec Amazon-Books-shape: {n_items:,} items (incl. PAD), L={L}, d={d}, '
                    f'2 layers x 2 heads, inner 256, sampled softmax over {n_neg} walk '
                    f'negatives, dense Adam',
        'dtype': 'fp32', 'data': 'synthetic (Zipf(1.1) items, Poisson(20)+4 lengths, seeded)',
        'transformer_tflops_at_step_rate': round(flops / t / 1e12, 2),
        'step_breakdown': _step_breakdown('C3'),
        'roofline': {'kernel': ('K9e attn_bwd_kernel (csrc/attn.hip: the attention backward, '
                                'one workgroup per sequence x head; P recomputed, dP, dS, dQ, '
                                'dK, dV on fp32 MFMA)') if k9e else
                               ('attention backward of torch scaled_dot_product_attention '
                                '(bwd_kernel_fuse, library)'),
                     'bound': 'mfma', 'achieved': round(attn_flops / ta / 1e12, 2),
                     'peak': 157.3, 'unit': 'TFLOP/s',
                     'frac': round(attn_flops / ta / 1e12 / 157.3, 4),
                     'flops_per_launch': attn_flops, 'launch_us': round(ta * 1e6, 1),
                     'fwd_us': round(ta_fwd * 1e6, 1) if ta_fwd else None,
                     'fwd_tflops': (round(2 * 2 * B * H * L * L * dh / ta_fwd / 1e12, 2)
                                    if ta_fwd else None),
                     'timing': 'HIP events around the backward (torch.autograd.grad) of one '
                               'attention at the step shapes, and around one forward (median '
                               'of 10, host-inclusive)',
                     'note': 'fp32 dense MFMA peak; FLOPs of the five L x L x dh products of '
                             'the backward (S recomputed, dV, dP, dQ, dK)'},
        'k9b': _k9b_line(d, n_neg, k9_bytes, tk),
    }


def _k9b_line(d, n_neg, k9_bytes, tk):
    """K9b's roofline on its kernel time in the committed C3 step trace (rocprofv3,
    profiles/r*_C3_step.json: the launch inside the captured step), the host-inclusive
    HIP-event time of an eager launch beside it."""
    import glob
    import json
    t_trace, src = None, None
    for path in sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_C3_step.json')))[::-1]:
        ks = [k for k in json.load(open(path))['kernels'] if 'sampled_softmax' in k['kernel']]
        if ks:
            t_trace, src = ks[0]['avg_us'] * 1e-6, os.path.basename(path)
            break
    t = t_trace if t_trace is not None else tk
    return {'kernel': f'K9b sampled_softmax<{d}> ({n_neg} negatives)', 'bound': 'hbm',
            'achieved': round(k9_bytes / t / 1e9, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(k9_bytes / t / 1e9 / HBM_PEAK_GBS, 4), 'bytes_per_launch': k9_bytes,
            'launch_us': round(t * 1e6, 1), 'timing_source': src or 'HIP events (eager)',
            'launch_us_incl_host': round(tk * 1e6, 1)}


# ----------------------------------------------------------------------------- C5
def make_c5_graph(n_users, n_items, nnz, seed=2020):
    """Distinct (user, item) edges: user degrees Zipf-like (min 1), items Zipf(1.0)."""
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, n_users + 1) ** 0.6
    deg = np.maximum(1, np.round(w / w.sum() * nnz)).astype(np.int64)
    deg = np.minimum(deg, n_items // 2)
    u = np.repeat(rng.permutation(np.arange(1, n_users + 1)), deg[rng.permutation(n_users)])
    p = 1.0 / np.arange(1, n_items + 1)
    cdf = np.cumsum(p / p.sum())
    i = np.searchsorted(cdf, rng.random(len(u))).astype(np.int64) + 1
    i = np.minimum(i, n_items)
    key = np.unique(u * (n_items + 1) + i)
    return key // (n_items + 1), key % (n_items + 1)


def bench_c5(dev, scale=1.0, d=256, n_layers=2, K=10, sample_users=131072):
    from recbole_amd import ops
    from recbole_amd.model.general_recommender.lightgcn import norm_adj_csr, propagate
    U = int(10_000_000 * scale) + 1
    I = int(5_000_000 * scale) + 1
    t0 = time.perf_counter()
    u, i = make_c5_graph(U - 1, I - 1, int(100_000_000 * scale))
    print(f'C5: {len(u):,} edges generated ({time.perf_counter() - t0:.0f} s)', file=sys.stderr,
          flush=True)
    rp, cols, vals = norm_adj_csr(u, i, U, I)
    print(f'C5: normalised adjacency built ({time.perf_counter() - t0:.0f} s)', file=sys.stderr,
          flush=True)
    plan = ops.SpmmPlan(rp, cols, vals, device=dev)
    setup = time.perf_counter() - t0
    g = torch.Generator(device=dev).manual_seed(2020)
    EU = torch.randn(U, d, generator=g, device=dev) * 0.01
    EI = torch.randn(I, d, generator=g, device=dev) * 0.01
    out_u, out_i = torch.empty_like(EU), torch.empty_like(EI)
    tmp = [torch.empty(U + I, d, device=dev)]
    propagate(plan, EU, EI, n_layers, out_u, out_i, tmp)      # warm-up
    torch.cuda.synchronize()
    tp = _event_time(lambda: propagate(plan, EU, EI, n_layers, out_u, out_i, tmp), reps=3)
    # K7 algorithmic bytes per layer: per nonzero col+val (8 B) + the gathered row
    # (d*4 B); per row the output write (d*4) and the accumulator read/write
    nnz2 = int(rp[-1])
    per_layer = nnz2 * (8 + d * 4) + (U + I) * (d * 4 * 3) + (U + I + 1) * 8
    # full-sort sample: users 1..n, history = their training edges, 1 positive each
    n = min(sample_users, U - 1)
    users = torch.arange(1, n + 1, device=dev)
    up = rp[:U + 1]
    hist_ptr = torch.as_tensor((up[1:n + 2] - up[1]).astype(np.int64), device=dev)
    hist_cols = torch.as_tensor((cols[up[1]:up[n + 1]].astype(np.int64) - U).astype(np.int32),
                                device=dev)
    rng = np.random.default_rng(7)
    pos_cols = torch.as_tensor(rng.integers(1, I, n).astype(np.int32), device=dev)
    pos_ptr = torch.arange(n + 1, dtype=torch.int64, device=dev)
    Uq = ops.gather_rows(out_u, users)
    o = {}
    run = lambda: ops.fullsort_topk(Uq, out_i, K, hist_ptr=hist_ptr, hist_cols=hist_cols,
                                    pos_ptr=pos_ptr, pos_cols=pos_cols, out=o)
    run()
    torch.cuda.synchronize()
    tf = _event_time(run, reps=3)
    flops = 2.0 * n * I * d
    cpu = None
    if CPU_BASELINE:
        from oracle import cpu_baseline as cb
        thr, how = cb.host_threads()
        nc = 512
        uq, it = Uq[:nc].cpu(), out_i.cpu()
        runs = [cb.time_full_sort_users(uq, it, nc, K=K, threads=thr) for _ in range(3)]
        ups, used = float(np.median([r[0] for r in runs])), runs[0][2]
        cpu = {'value': round(ups, 1), 'unit': 'users/s', 'cores': used, 'kind': 'port',
               'threads_derivation': how, 'runs': [round(r[0], 1) for r in runs],
               'sample': f'median of 3 runs of {nc} users ranked on torch CPU as the reference '
                         f'does (U[u] @ I^T, pad mask, flip + topk), '
                         f'{sum(r[1] for r in runs):.1f} s timed in all'}
    return {
        'cpu_baseline': cpu,
        'config': 'C5', 'metric': 'full-sort eval users/s', 'value': round(n / tf, 1),
        'unit': 'users/s', 'users_timed': n,
        'workload': f'LightGCN {U - 1:,} users x {I - 1:,} items, {len(u):,} edges, d={d}, '
                    f'{n_layers} layers; full-sort top-{K} vs all items with history mask',
        'dtype': 'fp32', 'data': 'synthetic (Zipf items, Zipf-like user degrees, seeded)',
        'setup_s': round(setup, 1),
        'roofline': {'kernel': f'K6 fullsort_topk<{d}> (fp32 MFMA 32x32x2)', 'bound': 'mfma',
                     'achieved': round(flops / tf / 1e12, 2), 'peak': FP32_PEAK_TFLOPS,
                     'unit': 'TFLOP/s', 'frac': round(flops / tf / 1e12 / FP32_PEAK_TFLOPS, 4),
                     'flops_per_launch': flops, 'launch_ms': round(tf * 1e3, 2)},
        'propagation': {'kernel': f'K7 spmm_units_kernel<{d}> x {n_layers} layers',
                        'bound': 'hbm', 'ms': round(tp * 1e3, 2),
                        'achieved': round(n_layers * per_layer / tp / 1e9, 1),
                        'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                        'frac': round(n_layers * per_layer / tp / 1e9 / HBM_PEAK_GBS, 4),
                        'bytes_per_layer': per_layer, 'nnz': nnz2},
        'full_pass_s_estimate': round((U - 1) / (n / tf) + tp, 1),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--configs', default='C3,C4,C5')
    ap.add_argument('--steps', type=int, default=64)
    ap.add_argument('--warmup', type=int, default=8)
    ap.add_argument('--scale', type=float, default=1.0)
    ap.add_argument('--out', default=None)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--adam-mode', default='deferred', choices=['deferred', 'streamed'])
    ap.add_argument('--eager-step', action='store_true', help='C3 / C4 without the captured step')
    args = ap.parse_args()
    global CPU_BASELINE, ADAM_MODE, GRAPH_STEP
    CPU_BASELINE = not args.no_cpu_baseline
    GRAPH_STEP = not args.eager_step
    ADAM_MODE = args.adam_mode
    dev = torch.device('cuda', 0)
    res = []
    for c in args.configs.split(','):
        if c == 'C3':
            r = bench_c3(dev, args.steps, args.warmup, args.scale)
        elif c == 'C4':
            r = bench_c4(dev, args.steps, args.warmup, args.scale)
        elif c == 'C5':
            r = bench_c5(dev, args.scale)
        else:
            raise SystemExit(f'unknown config {c}')
        print(json.dumps(r), flush=True)
        res.append(r)
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
