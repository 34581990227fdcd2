"""Sequential data host logic on the CPU: the vectorised augmentation and
leave-one-out split against the oracle's as-written loops of
sequential_dataset.py:43-112 / dataset.py:1317-1337, and the CPU batch
materialisation of the item lists."""
import numpy as np
import torch

from oracle import cpu_ref


def test_augmentation_and_split_match_reference_loops(tmp_path):
    from tests.test_gpu_e2e import _write_dataset
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset, data_preparation
    from recbole_amd.utils import init_seed
    root = _write_dataset(str(tmp_path), 'synth', n_users=40, n_items=60, n_inter=900)
    config = Config(config_dict={'model': 'SASRec', 'dataset': 'synth', 'data_path': root,
                                 'use_gpu': False, 'MAX_ITEM_LIST_LENGTH': 7,
                                 'training_neg_sample_num': 0,
                                 'load_col': {'inter': ['user_id', 'item_id', 'timestamp']}})
    init_seed(config['seed'], config['reproducibility'])
    ds = create_dataset(config)
    train, valid, test = data_preparation(config, ds)
    inter = train.dataset.inter_feat
    uids = inter['user_id'].numpy()
    u_list, index, target = cpu_ref.seq_augmentation(uids, 7)
    parts = cpu_ref.leave_one_out_index(u_list, 2)
    for loader, part in zip((train, valid, test), parts):
        assert np.array_equal(loader.dataset.target_index, np.asarray(target)[part])
        st = np.asarray([index[j][0] for j in part])
        ln = np.asarray([index[j][1] - index[j][0] for j in part])
        assert np.array_equal(loader.dataset.item_list_start, st)
        assert np.array_equal(loader.dataset.item_list_length, ln)
    b = test.augmentation(slice(0, 5))
    items = inter['item_id'].numpy()
    for r in range(5):
        s, n = test.dataset.item_list_start[r], test.dataset.item_list_length[r]
        exp = np.zeros(7, dtype=np.int64)
        exp[:n] = items[s:s + n]
        assert np.array_equal(b['item_id_list'][r].numpy(), exp)
        assert b['item_id'][r].item() == items[test.dataset.target_index[r]]
    assert b['timestamp_list'].dtype == torch.float64
