"""Plugin lookup and small helpers (mirror of recbole/utils/utils.py:24-215)."""
from __future__ import annotations

import datetime
import importlib
import os
import random

import numpy as np
import torch

from recbole_amd.utils.enum_type import ModelType

_MODEL_SUBMODULES = ['general_recommender', 'context_aware_recommender',
                     'sequential_recommender']


def get_local_time():
    return datetime.datetime.now().strftime('%b-%d-%Y_%H-%M-%S')


def ensure_dir(dir_path):
    os.makedirs(dir_path, exist_ok=True)


def get_model(model_name):
    """Resolve `recbole_amd.model.<family>.<name.lower()>.<name>` (utils.py:50-75)."""
    model_file_name = model_name.lower()
    for sub in _MODEL_SUBMODULES:
        path = f'recbole_amd.model.{sub}.{model_file_name}'
        if importlib.util.find_spec(f'recbole_amd.model.{sub}') is None:
            continue
        if importlib.util.find_spec(path) is not None:
            return getattr(importlib.import_module(path), model_name)
    raise ValueError(f'`model_name` [{model_name}] is not the name of an existing model.')


def get_trainer(model_type, model_name):
    """`<Model>Trainer` if defined, else the generic Trainer (utils.py:78-96)."""
    mod = importlib.import_module('recbole_amd.trainer')
    try:
        return getattr(mod, model_name + 'Trainer')
    except AttributeError:
        return getattr(mod, 'Trainer')


def early_stopping(value, best, cur_step, max_step, bigger=True):
    """Validation-based early stopping (utils.py:99-140)."""
    stop_flag = False
    update_flag = False
    better = value > best if bigger else value < best
    if better:
        cur_step = 0
        best = value
        update_flag = True
    else:
        cur_step += 1
        if cur_step > max_step:
            stop_flag = True
    return best, cur_step, stop_flag, update_flag


def calculate_valid_score(valid_result, valid_metric=None):
    if valid_metric:
        return valid_result[valid_metric]
    return valid_result['Recall@10']


def dict2str(result_dict):
    return ''.join(f'{k} : {v}    ' for k, v in result_dict.items())


def init_seed(seed, reproducibility):
    """Seed python/numpy/torch exactly as the reference does (utils.py:175-192):
    the numpy stream feeds the sampler's shuffle, the torch CPU stream feeds the
    RO ordering randperm, xavier init and the per-epoch randperm."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.benchmark = not reproducibility
    torch.backends.cudnn.deterministic = bool(reproducibility)


def set_color(log, color, highlight=True):
    colors = ['black', 'red', 'green', 'yellow', 'blue', 'pink', 'cyan', 'white']
    idx = colors.index(color) if color in colors else len(colors) - 1
    prev = '\033[' + ('1;3' if highlight else '0;3') + str(idx) + 'm'
    return prev + log + '\033[0m'
