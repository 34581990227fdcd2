"""Host data pipeline at C2 scale: write the synthetic
ml-20m-shape interactions as an atomic `.inter` file (user_id:token,
item_id:token, rating:float, timestamp:float — the ml-20m layout), then time the
drop-in path stage by stage: create_dataset (read + filter + factorize remap) and
data_preparation (RO_RS 0.8/0.1/0.1 grouped split, per-phase used-id CSRs,
random_list, the train / sampled-valid / full-sort-test loaders with their history
arrays). Writes one JSON line.

usage: python tools/bench_pipeline.py [--dir /tmp/c2_inter] [--out profiles/r02_pipeline.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_inter(path, u, i, seed=2020):
    rng = np.random.default_rng(seed + 1)
    rating = rng.integers(1, 11, len(u)) / 2.0
    ts = 789652009 + np.sort(rng.integers(0, 600_000_000, len(u)))
    import pandas as pd
    df = pd.DataFrame({'user_id:token': u, 'item_id:token': i, 'rating:float': rating,
                       'timestamp:float': ts})
    df.to_csv(path, sep='\t', index=False)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dir', default='/tmp/c2_inter')
    ap.add_argument('--out', default=None)
    ap.add_argument('--device', default='cpu')
    args = ap.parse_args()
    import bench
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset, data_preparation
    from recbole_amd.utils import init_seed
    name = bench.c2_name()
    d = os.path.join(args.dir, name)
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f'{name}.inter')
    t = time.perf_counter()
    if not os.path.exists(path):
        u, i, _, _ = bench.make_c2()
        write_inter(path, u, i)
    t_write = time.perf_counter() - t
    res = {'metric': 'C2 host data pipeline seconds', 'file_mb': round(os.path.getsize(path) / 2**20, 1),
           'write_s': round(t_write, 2)}
    config = Config(model='BPR', dataset=name, config_dict={
        'data_path': args.dir, 'embedding_size': 128, 'training_neg_sample_num': 4,
        'train_batch_size': 2048, 'eval_setting': 'RO_RS,full', 'state': 'ERROR',
        'load_col': {'inter': ['user_id', 'item_id', 'rating', 'timestamp']},
        'use_gpu': args.device != 'cpu'})
    init_seed(config['seed'], config['reproducibility'])
    t = time.perf_counter()
    ds = create_dataset(config)
    res['create_dataset_s'] = round(time.perf_counter() - t, 2)
    res['inters'], res['users'], res['items'] = int(ds.inter_num), int(ds.user_num), int(ds.item_num)
    t = time.perf_counter()
    train, valid, test = data_preparation(config, ds)
    res['data_preparation_s'] = round(time.perf_counter() - t, 2)
    res['train_inters'] = int(train.dataset.inter_num)
    res['value'] = round(res['create_dataset_s'] + res['data_preparation_s'], 2)
    res['unit'] = 's'
    res['higher_is_better'] = False
    res['cores'] = os.cpu_count()
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        open(args.out, 'w').write(line + '\n')


if __name__ == '__main__':
    main()
