"""Layered configuration (mirror of recbole/config/configurator.py:28-363).

Precedence, lowest to highest (configurator.py:59-81, 229-257):
  package defaults < model defaults < dataset defaults < model-type preset
  < config files < config_dict < command line (``--key=value``).
Keys and values are the reference's; YAML is read with a SafeLoader (plus the
reference's float resolver) and command-line strings are parsed with
ast.literal_eval instead of eval() — same results for literal values.

New keys (MI355X build): ``n_gpus``, ``fused_train`` (use the fused HIP train
step, default True), ``train_graph`` (capture steps in a HIP graph),
``adam_mode`` ('deferred' | 'streamed': two bit-identical schedules of the dense
Adam, see trainer/fused.py).
"""
from __future__ import annotations

import ast
import os
import re
import sys
from logging import getLogger

import torch
import yaml

from recbole_amd.config.defaults import (DATASET_DEFAULTS, MODEL_DEFAULTS, OVERALL, SAMPLE,
                                         TYPE_DATASET_PRESETS, TYPE_PRESETS)
from recbole_amd.evaluator import group_metrics, individual_metrics
from recbole_amd.utils import (EvaluatorType, InputType, ModelType, dataset_arguments,
                               evaluation_arguments, general_arguments, get_model,
                               training_arguments)


def _yaml_loader():
    class Loader(yaml.SafeLoader):
        pass

    Loader.add_implicit_resolver(
        u'tag:yaml.org,2002:float',
        re.compile(u'''^(?:
             [-+]?(?:[0-9][0-9_]*)\\.[0-9_]*(?:[eE][-+]?[0-9]+)?
            |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
            |\\.[0-9_]+(?:[eE][-+][0-9]+)?
            |[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+\\.[0-9_]*
            |[-+]?\\.(?:inf|Inf|INF)
            |\\.(?:nan|NaN|NAN))$''', re.X), list(u'-+0123456789.'))
    return Loader


def _convert(value):
    """configurator.py:106-129: strings become literals when they parse as one."""
    if not isinstance(value, str):
        return value
    try:
        v = ast.literal_eval(value)
        if isinstance(v, (str, int, float, list, tuple, dict, bool)):
            return v
        return value
    except (ValueError, SyntaxError):
        if value.lower() == 'true':
            return True
        if value.lower() == 'false':
            return False
        return value


class Config(object):

    def __init__(self, model=None, dataset=None, config_file_list=None, config_dict=None):
        self.yaml_loader = _yaml_loader()
        # parameter categories of the printout (configurator.py:85-88)
        self.parameters = {'General': general_arguments, 'Training': training_arguments,
                           'Evaluation': evaluation_arguments, 'Dataset': dataset_arguments}
        self.file_config_dict = self._load_config_files(config_file_list)
        self.variable_config_dict = {k: _convert(v) for k, v in (config_dict or {}).items()}
        self.cmd_config_dict = self._load_cmd_line()
        ext = {}
        ext.update(self.file_config_dict)
        ext.update(self.variable_config_dict)
        ext.update(self.cmd_config_dict)
        self.external_config_dict = ext
        self.model, self.model_class, self.dataset = self._get_model_and_dataset(model, dataset)
        self.internal_config_dict = self._internal(self.model, self.model_class, self.dataset)
        self.final_config_dict = dict(self.internal_config_dict)
        self.final_config_dict.update(self.external_config_dict)
        self._set_default_parameters()
        self._init_device()
        self._set_train_neg_sample_args()

    # ------------------------------------------------------------------ loading
    def _load_config_files(self, files):
        out = {}
        for f in files or []:
            with open(f, 'r', encoding='utf-8') as fh:
                d = yaml.load(fh.read(), Loader=self.yaml_loader)
                if d:
                    out.update(d)
        return out

    def _load_cmd_line(self):
        out = {}
        if 'ipykernel_launcher' in sys.argv[0] or 'pytest' in sys.argv[0]:
            return out
        for arg in sys.argv[1:]:
            if not arg.startswith('--') or len(arg[2:].split('=')) != 2:
                continue
            k, v = arg[2:].split('=')
            if k in out and v != out[k]:
                raise SyntaxError(f"There are duplicate commend arg '{arg}' with different value.")
            out[k] = v
        return {k: _convert(v) for k, v in out.items()}

    def _get_model_and_dataset(self, model, dataset):
        if model is None:
            try:
                model = self.external_config_dict['model']
            except KeyError:
                raise KeyError('model need to be specified in at least one of the these ways: '
                               '[model variable, config file, config dict, command line] ')
        if not isinstance(model, str):
            model_class, model = model, model.__name__
        else:
            model_class = get_model(model)
        if dataset is None:
            try:
                dataset = self.external_config_dict['dataset']
            except KeyError:
                raise KeyError('dataset need to be specified in at least one of the these ways: '
                               '[dataset variable, config file, config dict, command line] ')
        return model, model_class, dataset

    def _internal(self, model, model_class, dataset):
        d = dict(OVERALL)
        d.update(MODEL_DEFAULTS.get(model, {}))
        d.update(SAMPLE)
        d.update(DATASET_DEFAULTS.get(dataset, {}))
        d['MODEL_TYPE'] = model_class.type
        preset = TYPE_PRESETS.get(model_class.type)
        if preset:
            d.update(preset)
        d.update(TYPE_DATASET_PRESETS.get((model_class.type, dataset), {}))
        return d

    # ------------------------------------------------------------------ derived
    def _set_default_parameters(self):
        c = self.final_config_dict
        c['dataset'] = self.dataset
        c['model'] = self.model
        if c.get('data_path') is None:
            c['data_path'] = os.path.join('dataset', self.dataset)
        else:
            c['data_path'] = os.path.join(c['data_path'], self.dataset)
        if hasattr(self.model_class, 'input_type'):
            c['MODEL_INPUT_TYPE'] = self.model_class.input_type
        elif 'loss_type' in c:
            if c['loss_type'] in ['CE']:
                if c['MODEL_TYPE'] == ModelType.SEQUENTIAL and c['training_neg_sample_num'] > 0:
                    raise ValueError('training_neg_sample_num should be 0 when the loss_type is CE')
                c['MODEL_INPUT_TYPE'] = InputType.POINTWISE
            elif c['loss_type'] in ['BPR', 'SSM']:
                # SSM: sampled softmax over neg_sample_num negatives (build extension)
                c['MODEL_INPUT_TYPE'] = InputType.PAIRWISE
        else:
            raise ValueError("Either Model has attr 'input_type',or arg 'loss_type' should exist in config.")
        eval_type = None
        for metric in c['metrics']:
            if metric.lower() in individual_metrics:
                if eval_type == EvaluatorType.RANKING:
                    raise RuntimeError('Ranking metrics and other metrics can not be used at the same time.')
                eval_type = EvaluatorType.INDIVIDUAL
            if metric.lower() in group_metrics:
                if eval_type == EvaluatorType.INDIVIDUAL:
                    raise RuntimeError('Ranking metrics and other metrics can not be used at the same time.')
                eval_type = EvaluatorType.RANKING
        c['eval_type'] = eval_type
        valid_metric = c['valid_metric'].split('@')[0]
        c['valid_metric_bigger'] = valid_metric.lower() not in ['rmse', 'mae', 'logloss']
        if isinstance(c.get('additional_feat_suffix'), str):
            c['additional_feat_suffix'] = [c['additional_feat_suffix']]

    def _init_device(self):
        c = self.final_config_dict
        use_gpu = c['use_gpu']
        # one process per GPU under torchrun (WORLD_SIZE > 1) picks its own device
        if (use_gpu and 'CUDA_VISIBLE_DEVICES' not in os.environ
                and int(os.environ.get('WORLD_SIZE', '1')) == 1):
            os.environ['CUDA_VISIBLE_DEVICES'] = str(c['gpu_id'])
        c['device'] = torch.device('cuda' if torch.cuda.is_available() and use_gpu else 'cpu')

    def _set_train_neg_sample_args(self):
        c = self.final_config_dict
        if c['training_neg_sample_num']:
            c['train_neg_sample_args'] = {
                'strategy': 'by', 'by': c['training_neg_sample_num'],
                'distribution': c['training_neg_sample_distribution'] or 'uniform'}
        else:
            c['train_neg_sample_args'] = {'strategy': 'none'}

    # ------------------------------------------------------------------ mapping API
    def __setitem__(self, key, value):
        if not isinstance(key, str):
            raise TypeError('index must be a str.')
        self.final_config_dict[key] = value

    def __getitem__(self, item):
        return self.final_config_dict.get(item)

    def __contains__(self, key):
        if not isinstance(key, str):
            raise TypeError('index must be a str.')
        return key in self.final_config_dict

    def __getstate__(self):            # the YAML loader class is local: rebuilt on load
        state = dict(self.__dict__)
        state.pop('yaml_loader', None)
        return state

    def __setstate__(self, state):
        self.__dict__.update(state)
        self.yaml_loader = _yaml_loader()

    def __str__(self):
        # one block per category, then everything uncategorised (configurator.py:342-360)
        listed = {k for keys in self.parameters.values() for k in keys}
        blocks = []
        for category, keys in self.parameters.items():
            lines = [f'{k} = {v}' for k, v in self.final_config_dict.items() if k in keys]
            blocks.append(f'{category} Hyper Parameters:\n' + '\n'.join(lines))
        rest = [f'{k} = {v}' for k, v in self.final_config_dict.items()
                if k not in listed and k not in ('model', 'dataset', 'config_files')]
        blocks.append('Other Hyper Parameters: \n' + '\n'.join(rest))
        return '\n' + '\n\n'.join(blocks) + '\n\n'

    def __repr__(self):
        return self.__str__()


def get_logger():
    return getLogger()
