"""Popularity negative sampling (reference sampler.py:197-201 get_random_list
'popularity', the RepeatableSampler's :309-314, the walk :82-154): the random
list is every phase dataset's item column concatenated and shuffled by the global
numpy RNG; the GPU walk over it (K4, rejection of used ids for Sampler, none for
RepeatableSampler) returns bit-exactly the oracle's values (C walk and the numpy
line-by-line restatement), walk pointer included."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


def _built(tmp_path):
    from tests.test_gpu_e2e import _write_dataset
    from recbole_amd.config import Config
    from recbole_amd.config.eval_setting import EvalSetting
    from recbole_amd.data import create_dataset
    from recbole_amd.utils import init_seed
    root = _write_dataset(str(tmp_path), 'pop', n_users=120, n_items=300, n_inter=4000)
    config = Config(config_dict={'model': 'BPR', 'dataset': 'pop', 'data_path': root,
                                 'eval_setting': 'RO_RS,pop100', 'state': 'ERROR',
                                 'load_col': {'inter': ['user_id', 'item_id', 'timestamp']}})
    init_seed(config['seed'], config['reproducibility'])
    ds = create_dataset(config)
    es = EvalSetting(config)
    es.set_ordering_and_splitting('RO_RS')
    return ds, ds.build(es)


def _cols(datasets, field):
    return [np.asarray(d.inter_feat[field].cpu() if torch.is_tensor(d.inter_feat[field])
                       else d.inter_feat[field]) for d in datasets]


def test_popularity_sampler_walk_bit_exact(tmp_path, dev):
    from recbole_amd.sampler import Sampler
    ds, built = _built(tmp_path)
    np.random.seed(11)
    s = Sampler(['train', 'valid', 'test'], built, 'popularity')
    ref_rl = cpu_ref.random_list_popularity(_cols(built, ds.iid_field), seed=11)
    assert np.array_equal(np.asarray(s.random_list), ref_rl)
    tr = s.set_phase('train')
    tu, ti = _cols(built[:1], ds.uid_field)[0], _cols(built[:1], ds.iid_field)[0]
    ptr, cols = cpu_ref.used_csr(ds.user_num, tu, ti)
    used = np.array([set(cols[ptr[u]:ptr[u + 1]].tolist()) for u in range(ds.user_num)],
                    dtype=object)
    walk = cpu_ref.NumpyWalk(ref_rl, used)
    rng = np.random.default_rng(3)
    pr = 0
    for call in range(6):
        keys = rng.integers(1, ds.user_num, 57 if call != 2 else 1)   # one single-key call
        num = (1, 4, 9, 2, 3, 1)[call]
        exp_c, pr = cpu_ref.c_sample_walk(ref_rl, pr, keys, num, ptr, cols, ds.user_num, True)
        exp_np = walk.sample_by_key_ids(keys, num)
        got = tr.sample_by_user_ids(torch.as_tensor(keys), num)
        assert np.array_equal(np.asarray(exp_np), exp_c)
        assert np.array_equal(got.cpu().numpy(), exp_c), call
        assert tr.random_pr == pr


def test_popularity_repeatable_sampler_bit_exact(tmp_path, dev):
    from recbole_amd.sampler import RepeatableSampler
    ds, built = _built(tmp_path)
    col = [c.copy() for c in _cols([ds], ds.iid_field)]
    np.random.seed(5)
    s = RepeatableSampler(['train', 'valid', 'test'], ds, 'popularity')
    ref_rl = cpu_ref.random_list_popularity(col, seed=5)
    assert np.array_equal(np.asarray(s.random_list), ref_rl)
    # reference quirk (sampler.py:374 + :54): the list is a .numpy() view of the
    # dataset's item column, so the shuffle reorders that column in place too
    assert np.array_equal(_cols([ds], ds.iid_field)[0], ref_rl)
    ph = s.set_phase('test')
    rng = np.random.default_rng(9)
    pr = 0
    for num in (100, 7, 1000):
        keys = rng.integers(1, ds.user_num, 33)
        exp, pr = cpu_ref.c_sample_walk(ref_rl, pr, keys, num, None, None, ds.user_num, False)
        got = ph.sample_by_user_ids(torch.as_tensor(keys), num)
        assert np.array_equal(got.cpu().numpy(), exp)
        assert ph.random_pr == pr
