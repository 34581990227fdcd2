"""The reference's own dataset fixtures, transcribed (reference
tests/data/test_dataset.py; data files copied under tests/golden/data): id remap
order with and without fields_in_same_space (:354-399) and the TO_RS / TO_LS /
RO_RS split contents (:470-578) through the product's atomic-file Dataset."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _dataset(cfg):
    import logging
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset
    from recbole_amd.utils import init_seed
    base = {'model': 'BPR', 'data_path': os.path.join(GOLDEN, 'data'), 'load_col': None,
            'use_gpu': False, 'state': 'ERROR'}
    base.update(cfg)
    config = Config(config_dict=base)
    init_seed(config['seed'], config['reproducibility'])
    logging.basicConfig(level=logging.ERROR)
    return create_dataset(config)


def _split(cfg):
    from recbole_amd.config.eval_setting import EvalSetting
    ds = _dataset(cfg)
    es = EvalSetting(ds.config)
    es.set_ordering_and_splitting([x.strip() for x in ds.config['eval_setting'].split(',')][0])
    return ds.build(es)


def _seq(col):
    return [list(np.asarray(x).tolist()) for x in col]


def test_remap_id():
    ds = _dataset({'dataset': 'remap_id', 'fields_in_same_space': None})
    assert ds.token2id('user_id', ['ua', 'ub', 'uc', 'ud']).tolist() == [1, 2, 3, 4]
    assert ds.token2id('item_id', ['ia', 'ib', 'ic', 'id']).tolist() == [1, 2, 3, 4]
    f = ds.inter_feat
    assert np.asarray(f['user_id']).tolist() == [1, 2, 3, 4]
    assert np.asarray(f['item_id']).tolist() == [1, 2, 3, 4]
    assert np.asarray(f['add_user']).tolist() == [1, 2, 3, 4]
    assert np.asarray(f['add_item']).tolist() == [1, 2, 3, 4]
    assert _seq(f['user_list']) == [[1, 2], [], [3, 4, 1], [5]]
    with pytest.raises(ValueError):
        ds.token2id('user_id', 'nope')


def test_remap_id_with_fields_in_same_space():
    ds = _dataset({'dataset': 'remap_id', 'fields_in_same_space': [
        ['user_id', 'add_user', 'user_list'], ['item_id', 'add_item']]})
    assert ds.token2id('user_id', ['ua', 'ub', 'uc', 'ud', 'ue', 'uf']).tolist() == [1, 2, 3, 4, 5, 6]
    assert ds.token2id('item_id', ['ia', 'ib', 'ic', 'id', 'ie', 'if']).tolist() == [1, 2, 3, 4, 5, 6]
    f = ds.inter_feat
    assert np.asarray(f['user_id']).tolist() == [1, 2, 3, 4]
    assert np.asarray(f['item_id']).tolist() == [1, 2, 3, 4]
    assert np.asarray(f['add_user']).tolist() == [2, 5, 4, 6]
    assert np.asarray(f['add_item']).tolist() == [5, 3, 6, 1]
    assert _seq(f['user_list']) == [[3, 5], [], [1, 2, 3], [6]]


def _items(d):
    return np.asarray(d.inter_feat['item_id']).tolist()


R = lambda a, b: list(range(a, b))


def test_TO_RS_811():
    tr, va, te = _split({'dataset': 'build_dataset', 'eval_setting': 'TO_RS',
                         'split_ratio': [0.8, 0.1, 0.1]})
    assert _items(tr) == R(1, 17) + [1] + [1] + [1] + [1, 2, 3] + R(1, 8) + R(1, 9) + R(1, 10)
    assert _items(va) == R(17, 19) + [2] + [4] + [8] + [9] + [10]
    assert _items(te) == R(19, 21) + [2] + [3] + [5] + [9] + [10] + [11]


def test_TO_RS_820():
    tr, va, te = _split({'dataset': 'build_dataset', 'eval_setting': 'TO_RS',
                         'split_ratio': [0.8, 0.2, 0.0]})
    assert _items(tr) == R(1, 17) + [1] + [1] + [1, 2] + [1, 2, 3, 4] + R(1, 9) + R(1, 9) + R(1, 10)
    assert _items(va) == R(17, 21) + [2] + [3] + [5] + [9] + [9, 10] + [10, 11]
    assert len(te.inter_feat) == 0


def test_TO_RS_802():
    tr, va, te = _split({'dataset': 'build_dataset', 'eval_setting': 'TO_RS',
                         'split_ratio': [0.8, 0.0, 0.2]})
    assert _items(tr) == R(1, 17) + [1] + [1] + [1, 2] + [1, 2, 3, 4] + R(1, 9) + R(1, 9) + R(1, 10)
    assert len(va.inter_feat) == 0
    assert _items(te) == R(17, 21) + [2] + [3] + [5] + [9] + [9, 10] + [10, 11]


def test_TO_LS():
    tr, va, te = _split({'dataset': 'build_dataset', 'eval_setting': 'TO_LS', 'leave_one_num': 2})
    assert _items(tr) == R(1, 19) + [1] + [1] + [1] + [1, 2, 3] + R(1, 8) + R(1, 9) + R(1, 10)
    assert _items(va) == R(19, 20) + [2] + [4] + [8] + [9] + [10]
    assert _items(te) == R(20, 21) + [2] + [3] + [5] + [9] + [10] + [11]


@pytest.mark.parametrize('ratios,sizes', [
    ([0.8, 0.1, 0.1], (16 + 1 + 1 + 1 + 3 + 7 + 8 + 9, 2 + 0 + 0 + 1 + 1 + 1 + 1 + 1,
                       2 + 0 + 1 + 1 + 1 + 1 + 1 + 1)),
    ([0.8, 0.2, 0.0], (16 + 1 + 1 + 2 + 4 + 8 + 8 + 9, 4 + 0 + 1 + 1 + 1 + 1 + 2 + 2, 0)),
    ([0.8, 0.0, 0.2], (16 + 1 + 1 + 2 + 4 + 8 + 8 + 9, 0, 4 + 0 + 1 + 1 + 1 + 1 + 2 + 2))])
def test_RO_RS(ratios, sizes):
    tr, va, te = _split({'dataset': 'build_dataset', 'eval_setting': 'RO_RS', 'split_ratio': ratios})
    assert (len(tr.inter_feat), len(va.inter_feat), len(te.inter_feat)) == sizes
