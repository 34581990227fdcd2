"""SURVEY.md §8(f) row 1 at full C2 scale: the synthetic ml-20m-shape interactions
(~20 M) written as an atomic `.inter` file and built through the drop-in path the
benchmark uses (bench.build_workload source='file': create_dataset -> data_preparation,
reference dataset.py:342-408 read, 908-928 factorize remap, 1281-1315 RO_RS split)
give the train / valid / test tables the oracle derives from the same file on its own:
tokens by numpy's text reader, ids by first appearance (pd.factorize order), the RO
torch.randperm after init_seed and the per-user ratio split (oracle/cpu_ref.py
ro_rs_split). The written tokens are canonical decimal integers, so factorizing their
integer values is factorizing the strings."""
import os
import sys
import time

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import cpu_ref

# (n_users, n_items, interactions): the C2 shape (full-scale, slow) and a small
# instance of the same generator and file path that runs in the default CPU suite
SHAPES = {'c2': (138493, 26744, 20_000_263), 'small': (4000, 1500, 120_000)}


@pytest.mark.parametrize('shape', ['small', pytest.param('c2', marks=pytest.mark.slow)])
def test_c2_atomic_file_path_matches_oracle(tmp_path, shape):
    sys.path.insert(0, ROOT)
    import bench
    from recbole.config import Config
    from recbole.data import create_dataset, data_preparation
    from recbole.utils import init_seed
    nU, nI, target = SHAPES[shape]
    u, i, _, _ = bench.make_c2(n_users=nU, n_items=nI, target=target)
    name = bench.c2_name()
    path = tmp_path / name / f'{name}.inter'
    bench.write_c2_inter(str(path), u, i)
    del u, i
    config = Config(model='BPR', dataset=name, config_dict={
        'data_path': str(tmp_path), 'embedding_size': 128, 'training_neg_sample_num': 4,
        'train_batch_size': 2048, 'eval_setting': 'RO_RS,full', 'use_gpu': False,
        'state': 'ERROR', 'load_col': {'inter': ['user_id', 'item_id', 'rating', 'timestamp']}})
    init_seed(config['seed'], config['reproducibility'])
    t = time.perf_counter()
    ds = create_dataset(config)
    train, valid, test = data_preparation(config, ds)
    t_product = time.perf_counter() - t

    # ---- oracle, from the file alone
    t = time.perf_counter()
    cols = np.loadtxt(str(path), dtype=np.int64, delimiter='\t', skiprows=1, usecols=(0, 1))
    users, n_users = cpu_ref.factorize(cols[:, 0])
    items, n_items = cpu_ref.factorize(cols[:, 1])
    del cols
    assert (ds.user_num, ds.item_num) == (n_users, n_items)
    torch.manual_seed(config['seed'])         # init_seed: the RO randperm is the first draw
    parts = cpu_ref.ro_rs_split(users)
    t_oracle = time.perf_counter() - t
    assert len(users) > 0.95 * target
    for loader, rows in zip((train, valid, test), parts):
        inter = loader.dataset.inter_feat
        got_u = inter['user_id'].cpu().numpy()
        got_i = inter['item_id'].cpu().numpy()
        if loader is not train:                  # eval loaders sort their split by user
            order = np.argsort(users[rows], kind='stable')
            rows = rows[order]
        assert np.array_equal(got_u, users[rows])
        assert np.array_equal(got_i, items[rows])
    print(f'product {t_product:.1f} s, oracle {t_oracle:.1f} s')
