"""The reference's negative-sampling dataloader fixtures, transcribed (reference
tests/data/test_dataloader.py; data files under tests/golden/data), run through
the product's loaders and the GPU sampler (K4):
  * pairwise training batches: positives in file order, item features joined
    (item_id == price), negatives in (40, 100] with their features joined under
    the NEG_PREFIX (neg_item_id == neg_price) (:60-85);
  * point-wise training batches: positives then negatives, labels, features
    joined on both halves (:87-113);
  * uni100 evaluation batches: batch size adaptation (101 -> 202, 303 kept),
    positives first, sampled ids outside the user's history, pos_len / user_len
    lists (:235-368)."""
import logging
import os

import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _loaders(cfg, pointwise=False):
    from recbole_amd.config import Config
    from recbole_amd.data import create_dataset, data_preparation
    from recbole_amd.utils import InputType, init_seed
    base = {'model': 'BPR', 'data_path': os.path.join(GOLDEN, 'data'), 'load_col': None,
            'state': 'ERROR'}
    base.update(cfg)
    config = Config(config_dict=base)
    if pointwise:                 # the reference runs DMF here (a point-wise model)
        config['MODEL_INPUT_TYPE'] = InputType.POINTWISE
    init_seed(config['seed'], config['reproducibility'])
    logging.basicConfig(level=logging.ERROR)
    return data_preparation(config, create_dataset(config))


def _np(x):
    return x.cpu().numpy()


def test_neg_sample_dataloader_pairwise():
    train, _, _ = _loaders({'dataset': 'general_dataloader', 'eval_setting': 'TO_RS,full',
                            'training_neg_sample_num': 1, 'split_ratio': [0.8, 0.1, 0.1],
                            'train_batch_size': 6, 'eval_batch_size': 100})
    train.shuffle = False
    items, pr, n = list(range(1, 41)), 0, 0
    for b in train:
        assert _np(b['item_id']).tolist() == items[pr:pr + 6]
        assert (b['item_id'] == b['price']).all()
        assert (40 < b['neg_item_id']).all() and (b['neg_item_id'] <= 100).all()
        assert (b['neg_item_id'] == b['neg_price']).all()
        pr += 6
        n += 1
    assert pr >= 40 and n == 7


def test_neg_sample_dataloader_pointwise():
    train, _, _ = _loaders({'dataset': 'general_dataloader', 'eval_setting': 'TO_RS,full',
                            'training_neg_sample_num': 1, 'split_ratio': [0.8, 0.1, 0.1],
                            'train_batch_size': 6, 'eval_batch_size': 100}, pointwise=True)
    train.shuffle = False
    items, pr = list(range(1, 41)), 0
    for b in train:
        step = len(b) // 2
        assert _np(b['item_id'][:step]).tolist() == items[pr:pr + step]
        assert (40 < b['item_id'][step:]).all() and (b['item_id'][step:] <= 100).all()
        assert (b['item_id'] == b['price']).all()
        lab = _np(b[train.label_field])
        assert (lab[:step] == 1).all() and (lab[step:] == 0).all()
        pr += step
    assert pr == 40


def _check_uni100(data, batch_size, result):
    assert data.batch_size == batch_size
    assert len(data) == len(result)
    for b, (check, pos_len, user_len) in zip(data, result):
        assert check(b['item_id'].cpu())
        assert list(b.pos_len_list) == pos_len
        assert list(b.user_len_list) == user_len


def test_uni100_dataloader_batch_size_101():
    _, valid, test = _loaders({'dataset': 'general_uni100_dataloader', 'eval_setting': 'TO_RS,uni100',
                               'training_neg_sample_num': 1, 'split_ratio': [0.8, 0.1, 0.1],
                               'train_batch_size': 6, 'eval_batch_size': 101})
    _check_uni100(valid, 202, [
        (lambda d: d[0] == 9 and (8 < d[1:]).all() and (d[1:] <= 100).all(), [1], [101]),
        (lambda d: d[0] == 1 and (d[1:] != 1).all(), [1], [101]),
        (lambda d: (d[0:2].numpy() == [17, 18]).all() and (16 < d[2:]).all()
         and (d[2:] <= 100).all(), [2], [202])])
    _check_uni100(test, 202, [
        (lambda d: d[0] == 10 and (9 < d[1:]).all() and (d[1:] <= 100).all(), [1], [101]),
        (lambda d: d[0] == 1 and (d[1:] != 1).all(), [1], [101]),
        (lambda d: (d[0:2].numpy() == [19, 20]).all() and (18 < d[2:]).all()
         and (d[2:] <= 100).all(), [2], [202])])


def test_uni100_dataloader_batch_size_303():
    _, valid, test = _loaders({'dataset': 'general_uni100_dataloader', 'eval_setting': 'TO_RS,uni100',
                               'training_neg_sample_num': 1, 'split_ratio': [0.8, 0.1, 0.1],
                               'train_batch_size': 6, 'eval_batch_size': 303})
    _check_uni100(valid, 303, [
        (lambda d: d[0] == 9 and (8 < d[1:101]).all() and (d[1:101] <= 100).all()
         and d[101] == 1 and (d[102:202] != 1).all(), [1, 1], [101, 101]),
        (lambda d: (d[0:2].numpy() == [17, 18]).all() and (16 < d[2:]).all()
         and (d[2:] <= 100).all(), [2], [202])])
    _check_uni100(test, 303, [
        (lambda d: d[0] == 10 and (9 < d[1:101]).all() and (d[1:101] <= 100).all()
         and d[101] == 1 and (d[102:202] != 1).all(), [1, 1], [101, 101]),
        (lambda d: (d[0:2].numpy() == [19, 20]).all() and (18 < d[2:]).all()
         and (d[2:] <= 100).all(), [2], [202])])
