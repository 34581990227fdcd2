"""Benchmark: train positives/s of BPR-MF on the ml-20m-shape workload (C2).

BASELINE.json metric: "train positives/sec (+neg) per node; full-sort eval
users/sec". Workload: 138,493 users x 26,744 items (+PAD),
~20 M synthetic interactions (item popularity Zipf(1.0), user activity
log-normal(sigma=1) rescaled to mean 144.4, min 20), RO_RS 0.8/0.1/0.1 split,
embedding_size 128, 4 uniform negatives per positive, train_batch_size 2,048
rows -> 512 positives per step, Adam lr 1e-3 — built and trained through the
product path (Dataset -> data_preparation -> BPR -> FusedBPRTrainStep).

A step = one batch: K4 sampler walk + K2 grouping + K35 step records (the data side,
on two prep streams, one chunk of batches per launch) -> K35, one launch per step: BPR
forward + backward + the touched rows' dense-Adam step (deferred schedule: every
zero-gradient step of every row is applied, bit-identically, when the row is next read
or at a flush) + the look-ahead replays of the rows the next step reads -> per-chunk
loss bookkeeping; the timed region ends with the flush that makes every row current.
Inputs are resident in HBM before the timed region; the walk and grouping of every
timed step run inside it.

Prints ONE JSON line (rank 0). With --gpus N>1 (torchrun, one rank per GPU) the
tables are ROW-SHARDED (cyclic ownership; --dp-mode replicated keeps
replicas): each optimizer step consumes a global batch of N x 512 positives, every
rank walks and groups the global batch, owners send the rows each rank's slice reads
and receive its gradient rows back (two RCCL all-to-alls over xGMI), and apply the
deferred Adam step to their rows only — bit-identical to one GPU running the global
batch (weak scaling: the per-GPU batch is fixed; value = global positives /
max-over-ranks time).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)


def make_c2(seed=2020, n_users=138493, n_items=26744, target=20_000_263):
    """Synthetic ml-20m-shape interactions (ids 1..n, 0 = PAD)."""
    rng = np.random.default_rng(seed)
    act = rng.lognormal(0.0, 1.0, n_users)
    p = 1.0 / np.arange(1, n_items + 1)
    cdf = np.cumsum(p / p.sum())
    scale = 144.4
    for _ in range(3):                                 # dedupe shrinks heavy users: rescale
        a = np.maximum(np.round(act / act.mean() * scale), 20).astype(np.int64)
        a = np.minimum(a, n_items // 2)
        u = np.repeat(np.arange(1, n_users + 1, dtype=np.int64), a)
        i = np.searchsorted(cdf, rng.random(len(u))).astype(np.int64) + 1
        key = np.unique(u * (n_items + 1) + i)
        if abs(len(key) - target) / target < 0.02:
            break
        scale *= target / len(key)
    u, i = key // (n_items + 1), key % (n_items + 1)
    order = rng.permutation(len(u))                    # file order: not grouped by user
    return u[order], i[order], n_users + 1, n_items + 1


# the generator's version: bump it whenever make_c2 / write_c2_inter change what they write
C2_GEN_VERSION = 1


def c2_name(seed=2020):
    """Dataset name (= directory and file stem) of the synthetic C2 atomic file: it carries
    the seed and the generator version, so a cached file from other generator arguments is
    never reused (build_workload regenerates when the name is absent)."""
    return f'c2-synth-s{seed}-g{C2_GEN_VERSION}'


C2_NAME = c2_name()


def write_c2_inter(path, u, i, seed=2020):
    """The synthetic interactions as an atomic `.inter` file in the ml-20m layout
    (user_id:token, item_id:token, rating:float, timestamp:float; tab separated), so the
    benchmark's dataset goes through the reference's loading path (dataset.py:342-408
    read, 908-928 factorize remap, 1281-1315 RO_RS split). Arrow's CSV writer; the
    header is written as the reference's atomic files spell it."""
    import pyarrow as pa
    import pyarrow.csv as pacsv
    rng = np.random.default_rng(seed + 1)
    rating = rng.integers(1, 11, len(u)) / 2.0
    ts = (789652009 + np.sort(rng.integers(0, 600_000_000, len(u)))).astype(np.float64)
    tb = pa.table({'u': u, 'i': i, 'r': rating, 't': ts})
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = f'{path}.part{os.getpid()}'          # one writer's temporary: rename is atomic
    with open(tmp, 'wb') as f:
        f.write(b'user_id:token\titem_id:token\trating:float\ttimestamp:float\n')
        pacsv.write_csv(tb, f, pacsv.WriteOptions(include_header=False, delimiter='\t'))
    os.replace(tmp, path)


def build_workload(dev, d=128, neg=4, batch_rows=2048, seed=2020, adam_mode='deferred',
                   dist=None, chunk=None, sharded=False, alias=False, fused_step=None,
                   source='file', shape=None, exchange=None):
    """C2 through the drop-in path. source='file' (default): the synthetic interactions
    are written as an atomic file (MIREC_BENCH_DATA, default /tmp/mirec_bench; reused
    when present) and built by create_dataset -> data_preparation, the reference's
    pipeline; source='memory': Dataset.from_interactions of the same arrays (no file).
    shape=(n_users, n_items, interactions): a smaller instance of the same generator
    (source='memory' only; the smoke test). The step object carries the setup timings
    (step.setup_info)."""
    if shape is not None and source != 'memory':
        raise ValueError('shape= needs source="memory"')
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset, data_preparation
    from recbole_amd.data.dataset import Dataset
    from recbole_amd.model.general_recommender import BPR
    from recbole_amd.trainer.fused import FusedBPRTrainStep, ShardedBPRTrainStep
    from recbole_amd.trainer.optim import FusedAdam
    from recbole_amd.utils import init_seed
    info = {'source': source}
    root = os.environ.get('MIREC_BENCH_DATA', '/tmp/mirec_bench')
    name = c2_name(seed)
    path = os.path.join(root, name, f'{name}.inter')
    cd = {'data_path': root if source == 'file' else ROOT, 'embedding_size': d,
          'training_neg_sample_num': neg, 'train_batch_size': batch_rows,
          'eval_setting': 'RO_RS,full', 'use_gpu': True, 'state': 'ERROR',
          'neg_sampling_alias': alias,
          'load_col': {'inter': ['user_id', 'item_id', 'rating', 'timestamp']}}
    t = time.perf_counter()
    # ranks of a job share the node's file: rank 0 writes it, the others wait at a barrier
    # (every rank writing the same temporary raced: one rename found it gone)
    writer = dist is None or torch.distributed.get_rank(dist) == 0
    if source == 'memory' or (writer and not os.path.exists(path)):
        u, i, nU, nI = make_c2(seed) if shape is None else make_c2(seed, *shape)
        info['generate_s'] = round(time.perf_counter() - t, 2)
        if source == 'file':
            t = time.perf_counter()
            write_c2_inter(path, u, i, seed)
            info['write_s'] = round(time.perf_counter() - t, 2)
    if source == 'file' and dist is not None:
        torch.distributed.barrier(group=dist)
    if source == 'file':
        info['file'] = path
        info['file_mb'] = round(os.path.getsize(path) / 2 ** 20, 1)
    config = Config(model='BPR', dataset=name if source == 'file' else 'synthetic-ml20m',
                    config_dict=cd)
    config['device'] = dev
    init_seed(config['seed'], config['reproducibility'])
    t = time.perf_counter()
    if source == 'file':
        ds = create_dataset(config)
    else:
        ds = Dataset.from_interactions(config, u, i, nU, nI)
    info['create_dataset_s'] = round(time.perf_counter() - t, 2)
    t = time.perf_counter()
    train, valid, test = data_preparation(config, ds)
    info['data_preparation_s'] = round(time.perf_counter() - t, 2)
    model = BPR(config, train).to(dev)
    opt = FusedAdam(model.parameters(), lr=config['learning_rate'])
    if sharded:
        step = ShardedBPRTrainStep(model, opt, train, adam_mode=adam_mode, dist=dist, chunk=chunk,
                                   exchange=exchange)
    else:
        step = FusedBPRTrainStep(model, opt, train, adam_mode=adam_mode, dist=dist, chunk=chunk,
                                 fused_step=fused_step)
    step.setup_info = info
    return config, train, test, model, opt, step


def pmc_bytes(substr):
    """HBM bytes per launch of the kernel whose name contains `substr`, from the
    newest committed PMC summary (profiles/*_pmc.json, tools/summarize_prof.py:
    FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction; the newest one that traced it: the
    driver-window run launches no flush_row / K3), or None."""
    import glob
    files = sorted(f for f in glob.glob(os.path.join(ROOT, 'profiles', '*_pmc.json'))
                   if 'models_pmc' not in f)
    for path in files[::-1]:          # newest summary that traced this kernel
        for k, v in json.load(open(path)).items():
            if substr in k:
                return v.get('hbm_bytes_per_launch'), os.path.basename(path)
    return None, None


def executed_work(W, K):
    """K35's executed work in bench's measurement window after --warmup W --steps K, from
    the newest committed counter run of the same window (profiles/r*_k35_work*.json,
    tools/probe_step_work.py on the diagnostic build: element-steps actually executed —
    zero-state rows and rows already current never run, vanishing steps count as the m / v
    work they do), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_k35_work*.json')))[::-1]:
        d = json.load(open(path))
        c = d.get('config', {})
        if c.get('warmup') == W and c.get('steps') == K:
            return d, os.path.basename(path)
    return None, None


def pmc_valu_insts(substr):
    """(VALU, transcendental f32) wave-instructions per launch of the kernel whose
    name contains `substr` (SQ_INSTS_VALU, SQ_INSTS_VALU_TRANS_F32 pass of
    tools/prof_pmc.sh), or (None, None)."""
    import glob
    for path in sorted(f for f in glob.glob(os.path.join(ROOT, 'profiles', '*_pmc.json'))
                       if 'models_pmc' not in f)[::-1]:
        for k, v in json.load(open(path)).items():
            if substr in k and 'sq_insts_valu_per_launch' in v:
                return (v['sq_insts_valu_per_launch'],
                        v.get('sq_insts_valu_trans_f32_per_launch', 0.0),
                        v.get('valu_busy_frac'), os.path.basename(path))
    return None, None, None, None


# VALU issue model (MI355X_MICROARCH.md, per-instruction cycle constants): a wave64
# f32 VALU instruction takes 2 cycles of its SIMD at full rate, a transcendental
# (v_sqrt / v_rcp) 8; 1,024 SIMDs at 2.4 GHz.
SIMDS, CLOCK_HZ = 1024, 2.4e9


ADAM_FLOPS = 13      # IEEE fp32 ops per element per Adam step in torch's formula
VALU_PEAK_TFLOPS = 157.3   # MI355X fp32 vector peak (MI355X_MICROARCH.md)


def roofline(step, events, uniq, d, M, W=None, K=None):
    """Rooflines from the per-launch HIP events of an eager window of M steps
    that starts right after a flush and ends with one (every row of both tables
    is advanced exactly M Adam steps by the window's K5 launches).

    K5 dense Adam (dominant; fp32 VALU-bound: sqrt and two divisions per element):
      FLOPs = (n_users + n_items) * d * M * 13 over the window's deferred + flush
      launches. 13 = lerp (sub + fma) 3, v (mul + mul + fma) 4, sqrt 1, / 1, + eps 1,
      step * m 1, / 1, + p 1 (sqrt and division counted as one op each).
    K3 BPR (HBM view): bytes per launch = 2*(B+(1+T)B)*d*4 (rows read + gradient
      rows written) + 8*(B+(1+T)B) (ids) + 4*B (losses).
    """
    per = {}
    for name, a, b in events:
        per.setdefault(name, []).append(a.elapsed_time(b) * 1e-3)
    kernels_us = {k: round(float(np.mean(v)) * 1e6, 2) for k, v in per.items()}
    R, B, T = d * 4, step.B, step.times
    rowsI = (1 + T) * B
    fused = 'step' in per                      # K35: BPR + Adam step + look-ahead, one launch
    bpr = None
    if 'bpr' in per:
        bpr_bytes = 2 * (B + rowsI) * R + (B + rowsI) * 8 + B * 4
        t_bpr = kernels_us['bpr'] * 1e-6
        tb, _ = pmc_bytes(f'bpr_fwd_bwd_kernel<{d}>')
        bpr = {'kernel': f'K3 bpr_fwd_bwd<{d}>', 'bound': 'hbm', 'traffic': tb,
               'achieved': round(bpr_bytes / t_bpr / 1e9, 1), 'peak': HBM_PEAK_GBS,
               'unit': 'GB/s', 'frac': round(bpr_bytes / t_bpr / 1e9 / HBM_PEAK_GBS, 4),
               'bytes_per_launch': bpr_bytes, 'avg_launch_us': kernels_us['bpr']}
    # kernel time of the window's dense-Adam work: the per-step launches (K5 touched rows +
    # look-ahead, or K35 which also holds the BPR forward/backward), entry catch-ups and
    # the closing flush
    step_key = 'step' if fused else 'adam'
    t_adam = sum(per.get(step_key, [])) + sum(per.get('ahead', [])) + sum(per.get('flush', []))
    rows = getattr(step, 'SU', step.nU) + getattr(step, 'SI', step.nI)   # this rank's table rows
    flops = rows * d * M * ADAM_FLOPS
    if fused:   # + the BPR arithmetic K35 also does: (1+T) dots of 2d and 8d per pair
        flops += M * B * ((1 + T) * 2 * d + T * 8 * d)
    tf = flops / t_adam / 1e12
    flush_k = 'adam_flush_row_kernel' if d >= 64 else 'adam_flush_list_kernel'
    per_k = f'bpr_adam_step_kernel<{d}>' if fused else f'adam_deferred_kernel<{d},'
    nd, nf = len(per.get(step_key, [])) + len(per.get('ahead', [])), len(per.get('flush', []))
    if fused:
        name = ('K35 bpr_adam_step_kernel<%d> x %d (BPR fwd/bwd + touched-row Adam + '
                'look-ahead, one launch per step) + %s<%d> x %d (+ entry catch-up x %d)'
                % (d, len(per['step']), flush_k, d, nf, len(per.get('ahead', []))))
    else:
        name = ('K5 deferred dense Adam: adam_deferred_kernel<%d, float> x %d + %s<%d> x %d'
                % (d, nd, flush_k, d, nf))
    if step.adam_mode == 'streamed':
        name = f'K5 adam_multi_kernel<{d}> x {len(per.get("adam", []))} (streamed dense Adam)'
    adam = {'kernel': name, 'bound': 'valu', 'achieved': round(tf, 2),
            'peak': VALU_PEAK_TFLOPS, 'unit': 'TFLOP/s', 'frac': round(tf / VALU_PEAK_TFLOPS, 4),
            'traffic': None, 'flops_per_window': flops, 'window_steps': M,
            'window_kernel_us': round(t_adam * 1e6, 1),
            'us_per_step': round(t_adam * 1e6 / M, 2),
            'flops_formula': '(table rows on this rank) * d * steps * 13'
                             + (' + steps * B * ((1+T)*2d + 8dT) (BPR)' if fused else '')}
    if step.adam_mode == 'deferred':
        bd, src = pmc_bytes(per_k)
        bf, _ = pmc_bytes(f'{flush_k}<{d}>')
        vd, td, bd_busy, vsrc = pmc_valu_insts(per_k)
        vf, tf_, bf_busy, _ = pmc_valu_insts(f'{flush_k}<{d}>')
        if bd_busy is not None and bf_busy is not None:
            # measured VALU pipe occupancy of the per-step kernel and the flush (PMC pass,
            # tools/prof_pmc.sh: 4 * SQ_ACTIVE_INST_VALU / (SIMDs * clock * duration))
            adam.update({'valu_busy_frac_' + ('step' if fused else 'deferred'): bd_busy,
                         'valu_busy_frac_flush': bf_busy, 'valu_source': vsrc})
        if vd is not None and vf is not None:
            insts = nd * vd + nf * vf
            trans = nd * td + nf * tf_
            t_issue = ((insts - trans) * 2 + trans * 8) / SIMDS / CLOCK_HZ
            adam.update({'valu_insts_per_window': int(insts),
                         'valu_insts_per_element_step': round(
                             insts * 64 / (rows * d * M), 2),
                         'valu_issue_bound_us': round(t_issue * 1e6, 1),
                         'valu_issue_frac': round(t_issue / t_adam, 4),
                         'valu_issue_model': 'PMC SQ_INSTS_VALU x 2 cyc (+6 per '
                                             'SQ_INSTS_VALU_TRANS_F32) / 1024 SIMDs / 2.4 GHz'})
        if bd is not None and bf is not None:
            adam.update({'traffic': int(nd * bd + nf * bf), 'traffic_unit': 'HBM bytes per window',
                         'traffic_source': src,
                         'traffic_note': 'PMC FETCH_SIZE x2 + WRITE_SIZE per launch x launches; '
                                         'streamed dense Adam moves 6*(nU+nI)*d*4 = %d per step'
                                         % (6 * (step.nU + step.nI) * R)})
    work, wsrc = executed_work(W, K) if fused else (None, None)
    if work is not None:
        # the roofline on the work the kernels execute (counter run of this same window):
        # the formula above credits every element-step of the dense update; here zero-state
        # rows, current rows and vanishing steps count only what they run
        mw = work['measurement_window']
        ex = mw['window_total']
        tf_ex = ex['flops'] / t_adam / 1e12
        t_step = kernels_us['step'] * 1e-6
        pl = mw['per_launch']
        alg_gbs = pl['algorithmic_bytes'] / t_step / 1e9
        tb_step, tsrc = pmc_bytes(per_k)
        adam.update({
            'dense_formula': {'achieved': adam['achieved'], 'frac': adam['frac'],
                              'flops_per_window': adam['flops_per_window']},
            'achieved': round(tf_ex, 3), 'frac': round(tf_ex / VALU_PEAK_TFLOPS, 4),
            'flops_per_window': int(ex['flops']), 'flops_source': wsrc,
            'flops_formula': 'executed (counters): 13 per gradient element-step, 9 per '
                             'zero-gradient step with its p update, 3 per vanishing step, BPR '
                             'dots + contribution vectors per contribution formed',
            'k35_per_launch': {
                'executed_flops': int(pl['flops']),
                'algorithmic_bytes': int(pl['algorithmic_bytes']),
                'algorithmic_bytes_formula': '(touched rows + look-ahead rows) x (p, m, v) x '
                                             'd x 4 B, read and written',
                'gathered_bytes': int(pl['gathered_bytes']),
                'avg_launch_us': kernels_us['step'],
                'hbm_frac_algorithmic': round(alg_gbs / HBM_PEAK_GBS, 4),
                'pmc_bytes_per_launch': tb_step, 'pmc_source': tsrc,
                'rows': {k: mw['per_launch_mean'][k] for k in
                         ('touched_rows', 'ahead_halves', 'contrib_user', 'contrib_pos',
                          'contrib_neg', 'split_parts')}}})
    if step.adam_mode == 'streamed':           # memory-bound: HBM view is the binding one
        by = 6 * (step.nU + step.nI) * R * M
        gbs = by / t_adam / 1e9
        adam.update({'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': round(gbs / HBM_PEAK_GBS, 4),
                     'bytes_formula': '6 * (n_users + n_items) * d * 4 per step'})
    if work is not None:
        # K35 is a memory-latency kernel (two dependent load levels per row, ~1.3 row waves
        # per wave slot): its binding resource is HBM, so the headline roofline is the HBM
        # one — the bytes it must move per launch (touched + look-ahead rows' p, m, v read
        # and written, plus the BPR partner rows it gathers) over its per-launch time. The
        # VALU view stays as a secondary field.
        pl = adam['k35_per_launch']
        by = pl['algorithmic_bytes'] + pl['gathered_bytes']
        t_step = kernels_us['step'] * 1e-6
        gbs = by / t_step / 1e9
        rp_us, rp_src = rocprof_avg_us(per_k)
        hbm = {'kernel': f'K35 bpr_adam_step_kernel<{d}> (BPR fwd/bwd + touched-row Adam + '
                         'look-ahead, one launch per step)',
               'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
               'frac': round(gbs / HBM_PEAK_GBS, 4), 'traffic': pl['pmc_bytes_per_launch'],
               'traffic_source': pl['pmc_source'],
               'bytes_per_launch': int(by),
               'bytes_formula': '(touched + look-ahead rows) x (p, m, v) x d x 4 B read and '
                                'written + the gathered BPR partner rows (counter run %s)' % wsrc,
               'avg_launch_us': kernels_us['step'], 'avg_launch_source': 'HIP events in bench',
               'rocprof_avg_us': rp_us, 'rocprof_source': rp_src,
               'frac_at_rocprof_avg': (round(by / (rp_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
                                       if rp_us else None),
               'valu': adam}
        return hbm, bpr, kernels_us
    return adam, bpr, kernels_us


def rocprof_avg_us(substr):
    """Average duration (µs) of the kernel whose name contains `substr` in the newest
    committed driver-window rocprofv3 --stats summary (profiles/r*_c2_driver_kernel_stats.csv),
    or (None, None)."""
    import csv
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_c2_driver_kernel_stats.csv')))[::-1]:
        with open(path) as f:
            for row in csv.DictReader(f):
                if substr in row.get('Name', ''):
                    return round(float(row['AverageNs']) / 1e3, 2), os.path.basename(path)
    return None, None


def gather_throughput(step, d, neg, B=65536, reps=20, big_rows=2_000_000):
    """north_star's gather roofline at the throughput setting of SURVEY.md §8d
    (B = 65,536 positives, 4 negatives): K3 alone — (2+T) row gathers per positive and
    the per-contribution gradient rows written — HIP events per launch, median of reps.
    Bytes per launch = 2*(B + (1+T)B)*d*4 (rows read + gradient rows written)
    + 8*(B + (1+T)B) (ids) + 4*B (losses).
    The HBM figure ('frac') is taken on tables past the 256 MiB Infinity Cache (big_rows
    users + big_rows items, uniform ids: almost every row gather misses the LLC); the
    C2-table figure is reported beside it as LLC-resident (84.6 MB of tables)."""
    from recbole_amd import ops
    dev = step.device

    def one(EU, EI, nU, nI):
        g = torch.Generator(device='cpu').manual_seed(7)
        user = torch.randint(0, nU, (B,), generator=g).to(dev)
        pos = torch.randint(1, nI, (B,), generator=g).to(dev)
        negs = torch.randint(1, nI, (neg * B,), generator=g).to(dev)
        out = {}
        ops.bpr_fwd_bwd(EU, EI, user, pos, negs, neg, out=out)
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ops.bpr_fwd_bwd(EU, EI, user, pos, negs, neg, out=out)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e-3)
        return float(np.median(ts))

    rows = B + (1 + neg) * B
    nbytes = 2 * rows * d * 4 + rows * 8 + B * 4
    t_llc = one(step.pU.detach(), step.pI.detach(), step.nU, step.nI)
    g = torch.Generator(device=dev).manual_seed(11)
    EU = torch.randn(big_rows, d, device=dev, generator=g) * 0.1
    EI = torch.randn(big_rows, d, device=dev, generator=g) * 0.1
    t = one(EU, EI, big_rows, big_rows)
    del EU, EI
    traffic, tsrc = None, None        # PMC HBM bytes of the same launch (tools/gather_pmc.py)
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_gather.json')))[::-1]:
        big = [e for e in json.load(open(path)) if e.get('tables') == 'big']
        if big and big[0].get('table_rows') == [big_rows, big_rows]:
            traffic, tsrc = big[0].get('traffic'), os.path.basename(path)
            break
    gbs = nbytes / t / 1e9
    return {'kernel': f'K3 bpr_fwd_bwd<{d}> at B={B} positives, tables {big_rows:,} + '
                      f'{big_rows:,} rows ({2 * big_rows * d * 4 / 2**30:.2f} GiB: past the LLC)',
            'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 4), 'bytes_per_launch': nbytes,
            'traffic': traffic, 'traffic_source': tsrc,
            'launch_us': round(t * 1e6, 1), 'positives_per_s': round(B / t, 1),
            'llc_resident': {'tables': 'C2 (84.6 MB, fits the 256 MiB Infinity Cache)',
                             'achieved': round(nbytes / t_llc / 1e9, 1),
                             'frac': round(nbytes / t_llc / 1e9 / HBM_PEAK_GBS, 4),
                             'launch_us': round(t_llc * 1e6, 1)}}


def _cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(train, step_obj, d, neg, steps, warmup=20, runs=3):
    """SURVEY.md §8d protocol: the oracle's faithful CPU restatement of the
    reference step, `warmup` untimed steps then `steps` timed steps, median of
    `runs` runs, torch threads = the CPUs this job may use (sched_getaffinity capped by
    the cgroup CPU quota, oracle.cpu_baseline.host_threads; recorded in the JSON)."""
    from oracle import cpu_baseline as cb
    users = train.dataset.inter_feat['user_id'].cpu().numpy()
    items = train.dataset.inter_feat['item_id'].cpu().numpy()
    ptr, cols = train.sampler.used_csr['train']
    threads, how = cb.host_threads()
    vals, dts, splits = [], [], []
    for r in range(runs):
        sp = {}
        pps, dt, used = cb.time_bpr_steps(users, items, ptr, cols, train.sampler.random_list,
                                          step_obj.nU, step_obj.nI, d, step_obj.B, neg,
                                          steps=steps, warmup=warmup, threads=threads, seed=r,
                                          split=sp)
        vals.append(pps)
        dts.append(dt)
        splits.append(sp)
    med = int(np.argsort(vals)[len(vals) // 2])         # the median run's cost centres
    sp = splits[med]
    return {'value': round(float(np.median(vals)), 1), 'unit': 'positives/s', 'cores': used,
            # data pipeline (slice + sampler walk with the Python rejection
            # loop + pairwise layout) vs model step (fwd + bwd + dense Adam), median run
            'pipeline_s': round(sp['pipeline_s'], 3), 'model_s': round(sp['model_s'], 3),
            'pipeline_frac': round(sp['pipeline_s'] / (sp['pipeline_s'] + sp['model_s']), 4),
            'kind': 'port', 'runs': [round(v, 1) for v in vals],
            'nproc': os.cpu_count(), 'cpu_model': _cpu_model(),
            'torch_threads': used, 'threads_derivation': how,
            'sample': f'median of {runs} runs of {warmup} warm-up + {steps} timed C2 steps '
                      f'({steps * step_obj.B} positives x {neg} negatives per run) of the oracle '
                      f'restatement: Python rejection sampler + torch-CPU nn.Embedding/BPRLoss/'
                      f'dense Adam; {sum(dts):.1f} s timed in all'}


def _spawn_ranks(n):
    """`--gpus N` without a torchrun environment: start N ranks (one process per
    GPU) with torch.distributed.run and exit with its status. This parent never
    touches the GPU (no exec after GPU init on this pool)."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(('127.0.0.1', 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    # timed steps / warm-up steps (any values: the timed region always holds the
    # sampler walk + grouping of every timed step, see below)
    ap.add_argument('--steps', type=int, default=256)
    ap.add_argument('--warmup', type=int, default=64)
    ap.add_argument('--cpu-steps', type=int, default=200)
    ap.add_argument('--cpu-warmup', type=int, default=20)
    ap.add_argument('--cpu-runs', type=int, default=3)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-eval', action='store_true')
    ap.add_argument('--adam-mode', default='deferred', choices=['deferred', 'streamed'])
    # diagnostic: rows per step (default 2,048 = 512 positives x 4 negatives, C2)
    ap.add_argument('--batch-rows', type=int, default=2048)
    # diagnostic: steps per captured chunk (= deferred-Adam flush period), default 64
    ap.add_argument('--chunk', type=int, default=None)
    # multi-GPU table layout: row-sharded (default) or replicated;
    # 'sharded' with --gpus 1 runs the sharded protocol on one rank (diagnostic)
    ap.add_argument('--dp-mode', default=None, choices=['sharded', 'replicated'])
    # the sharded step's row exchanges: RCCL all-to-alls (default) or the IPC peer windows
    # (csrc/comm.hip); with --gpus 1 and no torchrun environment a 1-rank process group is
    # made in-process (so rocprofv3 can trace it: no launcher in between)
    ap.add_argument('--exchange', default=None, choices=['rccl', 'ipc'])
    # negative sampler: the bit-exact walk (default, the headline) or the alias-table
    # fast mode (labelled NON-PARITY: i.i.d. draws of the same distribution)
    ap.add_argument('--sampler', default='walk', choices=['walk', 'alias'])
    # diagnostic: chunk sizes after a pipeline (re)start, e.g. 2,4,8,16,32
    ap.add_argument('--ramp', default=None)
    # diagnostic: steps between deferred-Adam full flushes (default FLUSH_EVERY)
    ap.add_argument('--flush-every', type=int, default=None)
    # diagnostic: the K3 + K5 launches per step instead of the one-launch K35 step
    ap.add_argument('--no-fused-step', action='store_true')
    # diagnostic: prepare a pipeline-restart chunk on the prep streams (default: on the
    # model's stream, FusedBPRTrainStep.MAIN_FIRST)
    ap.add_argument('--no-main-first', action='store_true')
    # diagnostic: the synthetic interactions in memory instead of the atomic-file path
    ap.add_argument('--in-memory', action='store_true')
    args = ap.parse_args()

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(_spawn_ranks(args.gpus))
    if args.exchange and args.dp_mode == 'sharded' and 'WORLD_SIZE' not in os.environ:
        import socket
        with socket.socket() as s_:
            s_.bind(('127.0.0.1', 0))
            port = s_.getsockname()[1]
        os.environ.update(WORLD_SIZE='1', RANK='0', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1',
                          MASTER_PORT=str(port))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU')
    # a process group also at one rank when asked for the sharded protocol under
    # torchrun (exercises the RCCL path on a 1-GPU box)
    dist = world > 1 or (args.dp_mode == 'sharded' and 'WORLD_SIZE' in os.environ)
    # rehearsal of the multi-rank flow on a one-GPU box (diagnostic, never the driver's
    # run): every rank on cuda:0 and a gloo group (RCCL refuses two ranks on one device)
    one_dev = os.environ.get('MIREC_BENCH_ONE_DEVICE') == '1'
    if one_dev:
        local = 0
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        if one_dev:
            tdist.init_process_group('gloo')
        else:
            tdist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)

    d, neg = 128, 4
    t_setup = time.time()
    dp_mode = args.dp_mode or ('sharded' if dist else 'single')
    if dp_mode == 'replicated' and not dist:
        dp_mode = 'single'
    config, train, test, model, opt, step = build_workload(
        dev, d=d, neg=neg, batch_rows=args.batch_rows, adam_mode=args.adam_mode, chunk=args.chunk,
        dist=tdist.group.WORLD if dist else None, sharded=dp_mode == 'sharded',
        alias=args.sampler == 'alias', fused_step=False if args.no_fused_step else None,
        source='memory' if args.in_memory else 'file', exchange=args.exchange)
    if args.ramp:
        step.RAMP = tuple(int(x) for x in args.ramp.split(','))
    if args.flush_every:
        step.FLUSH_EVERY = args.flush_every
    if args.no_main_first:
        step.MAIN_FIRST = False

    setup_s = time.time() - t_setup
    K, W = args.steps, args.warmup
    if K < 1 or W < 0:
        raise SystemExit('--steps must be >= 1 and --warmup >= 0')
    # Chunks (one sampler-walk + grouping launch each, C steps) are cut at W, W+K and
    # W+K+C, and the preparation of the chunk at W and of every later chunk is held
    # until the timed region has started: the timed region holds the K4 walk and the
    # K2 grouping of every timed step (the first timed chunk's serially, the rest on
    # the prep stream beside the model side, as in steady state).
    M = step.C                                 # per-kernel measurement window after it
    # every row complete at the end of the timed region and of the measurement window
    nb = step.begin_epoch(cuts=(W, W + K, W + K + M), hold_prep_from=W,
                          flush_at=(W + K, W + K + M))
    if W + K + M > nb:
        raise SystemExit(f'steps+warmup exceed one epoch ({nb} batches)')
    step.run_batches(0, W)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    marks = os.environ.get('BENCH_MARKERS') == '1'   # trace markers (tools/check_timed_window.py)
    t0 = time.perf_counter()
    if marks:
        torch.cuda._sleep(1)
    step.release_prep(upto=W + K)              # the timed steps' chunks only
    eager0 = step.n_eager_steps
    step.run_batches(W, W + K)
    eager_timed = step.n_eager_steps - eager0
    step.sync_params()          # deferred schedule: every row complete inside the timed region
    if marks:
        torch.cuda._sleep(1)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    local_elapsed = elapsed
    if dist:
        t = torch.tensor([elapsed], device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())

    # Per-kernel HIP events around each model-side launch, on the stream it runs
    # on, over M further steps launched eagerly behind a spin kernel so the
    # events bracket kernel time only (not host enqueue gaps).
    # spin long enough (~2.4k cycles/us) to cover the host's enqueue of the whole
    # window (~5 eager launches per step), so the events bracket kernel time only
    step.release_prep()
    torch.cuda._sleep(int(2.4e3 * 400 * M))
    step.kernel_events, step.kernel_uniq = [], []
    step.run_batches(W + K, W + K + M)
    torch.cuda.synchronize()
    events, uniq = step.kernel_events, step.kernel_uniq
    step.kernel_events = None
    losses = step.end_epoch(W + K + M)
    assert all(np.isfinite(losses)), 'non-finite loss'
    roof, roof_bpr, kernels_us = roofline(step, events, uniq, d, M, W, K)
    mine = {'rank': rank, 'timed_s': round(local_elapsed, 6), 'kernels_us': kernels_us,
            'k5_us_per_step': roof.get('us_per_step', roof.get('valu', {}).get('us_per_step')),
            'table_rows': int(getattr(step, 'SU', step.nU) + getattr(step, 'SI', step.nI))}
    per_rank = [mine]
    if dist:
        per_rank = [None] * world
        tdist.all_gather_object(per_rank, mine)
    positives = K * step.Bg                    # global batch = world x 512 positives
    result = {
        'metric': 'train positives/sec (+neg) per node',
        'value': round(positives / elapsed, 1),
        'unit': 'positives/s',
        'n_gpus': world,
        'steps': K,
        'warmup': W,
        'timed_region': 'K steps incl. the sampler walk + grouping of every timed step '
                        '(chunk prep held until t0) and the closing deferred-Adam flush',
        'ms_per_step': round(elapsed / K * 1e3, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'fp32',
        'data': 'synthetic (ml-20m-shape, seeded), random xavier-normal init',
        'config': {'workload': 'C2 BPR-MF ml-20m-shape: 138,494 users x 26,745 items (incl. '
                               'PAD), ~20M interactions RO_RS 0.8/0.1/0.1, embedding 128, '
                               '4 uniform negatives, 512 positives (2,048 rows) per step, '
                               'dense Adam',
                   'global_batch': step.Bg, 'per_gpu_batch': step.B, 'train_interactions': int(
                       train.dataset.inter_num), 'parallelism': {
                           'single': 'single',
                           'sharded': f'dp{world} x row-sharded tables (cyclic ownership; ' + (
                               'rows through the IPC peer windows: owner push + K3 + owner Adam'
                               if getattr(step, 'exchange', 'rccl') == 'ipc' else
                               '2 RCCL all-to-alls of rows per step') +
                               f', cap {getattr(step, "cap", 0)} rows per rank pair)',
                           'replicated': f'dp{world} (replicated tables, RCCL all-gather of '
                                         f'per-row loss coefficients)'}[dp_mode],
                   'exchange_graph': bool(step.use_graph),
                   'sampler': ('walk (bit-exact)' if args.sampler == 'walk' else
                               'alias table (NON-PARITY fast mode)'),
                   'chunk_plan_timed': [n for b0, n, _ in step._plan if W <= b0 < W + K],
                   'eager_steps_timed': eager_timed},
        'roofline': roof,
        'roofline_bpr': roof_bpr,
        'kernels_us': kernels_us,
        'ranks': per_rank,
        'adam_mode': step.adam_mode,
        'fused_step': bool(getattr(step, 'fused_step', False)),
        'flush_every': int(getattr(step, 'FLUSH_EVERY', 0)),
        'setup_s': round(setup_s, 1),
        'setup': step.setup_info,
    }
    if not args.no_eval and rank == 0:
        from recbole_amd.trainer.fused import fused_full_sort_eval
        from recbole_amd.evaluator import TopKEvaluator
        ev = TopKEvaluator(config, ['recall', 'mrr', 'ndcg', 'hit', 'precision'])
        fused_full_sort_eval(model, test, ev)   # warm
        torch.cuda.synchronize()
        e0 = time.perf_counter()
        fused_full_sort_eval(model, test, ev)
        torch.cuda.synchronize()
        e_dt = time.perf_counter() - e0
        n_users = len(test.uid_list)
        # K6's own time: HIP events around each launch (on its stream) of one more pass
        from recbole_amd import ops
        ops.KERNEL_EVENTS = {'fullsort': []}
        fused_full_sort_eval(model, test, ev)
        torch.cuda.synchronize()
        k6 = [a.elapsed_time(b) * 1e-3 for a, b in ops.KERNEL_EVENTS['fullsort']]
        ops.KERNEL_EVENTS = None
        k6_s = float(sum(k6))
        flops = 2.0 * step.nI * d * n_users
        result['eval'] = {'metric': 'full-sort eval users/sec', 'value': round(n_users / e_dt, 1),
                          'users': n_users, 'seconds': round(e_dt, 4),
                          'flops_per_user': 2 * step.nI * d,
                          'roofline': {
                              'kernel': f'K6 fullsort_topk<{d}> (fp32 MFMA scores + mask + '
                                        f'top-{max(ev.topk)} + positive flags) x {len(k6)}',
                              'bound': 'mfma', 'achieved': round(flops / k6_s / 1e12, 2),
                              'peak': VALU_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                              'frac': round(flops / k6_s / 1e12 / VALU_PEAK_TFLOPS, 4),
                              'kernel_s': round(k6_s, 5), 'launches': len(k6),
                              'end_to_end_frac': round(flops / e_dt / 1e12 / VALU_PEAK_TFLOPS, 4),
                              'flops_formula': '2 * n_items * d per user (the score matmul)',
                              'timing': 'HIP events around each K6 launch on its stream'}}
    if rank == 0 and not args.no_eval:
        result['gather_throughput'] = gather_throughput(step, d, neg)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline(train, step, d, neg, args.cpu_steps,
                                              args.cpu_warmup, args.cpu_runs)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        step.close()             # captured collectives go before destroy_process_group
        del step
        tdist.destroy_process_group()


if __name__ == '__main__':
    main()
