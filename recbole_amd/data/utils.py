"""Dataset / loader construction (mirror of recbole/data/utils.py:27-286),
including the fork's hard-coded switch of a `full` VALIDATION to uni1000
(data/utils.py:86-88) — only the test phase is ranked against all items."""
import importlib
import os
import pickle
from logging import getLogger

from recbole_amd.config import EvalSetting
from recbole_amd.data.dataset import Dataset, SequentialDataset
from recbole_amd.data.dlapi import dlapi  # noqa: F401  (recbole.data.utils.dlapi)
from recbole_amd.sampler import RepeatableSampler, Sampler
from recbole_amd.utils import ModelType, ensure_dir


def create_dataset(config):
    model_type = config['MODEL_TYPE']
    if model_type == ModelType.SEQUENTIAL:
        return SequentialDataset(config)
    if model_type in (ModelType.GENERAL, ModelType.TRADITIONAL, ModelType.CONTEXT):
        return Dataset(config)
    raise NotImplementedError(f'model type {model_type} datasets are not part of this build yet')


# model family / negative-sampling strategy -> loader class name, resolved from
# recbole_amd.data.dataloader (reference data/utils.py:254-272)
_LOADER_FAMILY = {ModelType.GENERAL: 'General', ModelType.TRADITIONAL: 'General',
                  ModelType.CONTEXT: 'Context', ModelType.SEQUENTIAL: 'Sequential'}
_LOADER_KIND = {'none': 'DataLoader', 'by': 'NegSampleDataLoader', 'full': 'FullDataLoader'}


def get_data_loader(name, config, neg_sample_args):
    """Loader class for phase `name` ('train' / 'evaluation'): the class named
    `<family><kind>` in the dataloader package, as the reference looks it up. The
    reference's per-model table (DIN, DIEN, the autoencoders) and the fork's
    dataset-negative / both-way loaders belong to model families outside this build."""
    model_type = config['MODEL_TYPE']
    strategy = neg_sample_args['strategy']
    if model_type not in _LOADER_FAMILY:
        raise NotImplementedError(f'Model_type [{model_type}] has not been implemented.')
    if strategy not in _LOADER_KIND:
        raise NotImplementedError(f'neg_sample strategy [{strategy}] is not implemented')
    loaders = importlib.import_module('recbole_amd.data.dataloader')
    return getattr(loaders, _LOADER_FAMILY[model_type] + _LOADER_KIND[strategy])


def data_preparation(config, dataset, save=False):
    model_type = config['MODEL_TYPE']
    es = EvalSetting(config)
    built = dataset.build(es)
    train_dataset, valid_dataset, test_dataset = built
    phases = ['train', 'valid', 'test']
    sampler = None
    logger = getLogger()
    train_args = config['train_neg_sample_args']
    eval_args = es.neg_sample_args
    valid_args = dict(eval_args)
    if eval_args['strategy'] == 'full' and config['benchmark_filename'] is None:
        logger.warning('validation strategy switched to uniform 1000 (fork behaviour, '
                       'data/utils.py:86-88)')
        valid_args = {'strategy': 'by', 'by': 1000, 'distribution': 'uniform'}

    train_kwargs = {'config': config, 'dataset': train_dataset,
                    'batch_size': config['train_batch_size'],
                    'dl_format': config['MODEL_INPUT_TYPE'], 'shuffle': True}
    if train_args['strategy'] != 'none':
        if dataset.label_field in dataset.inter_feat and not config['train_use_bothway_sampler']:
            raise ValueError(f'`training_neg_sample_num` should be 0 '
                             f'if inter_feat have label_field [{dataset.label_field}].')
        if model_type != ModelType.SEQUENTIAL:
            sampler = Sampler(phases, built, train_args['distribution'])
        else:
            sampler = RepeatableSampler(phases, dataset, train_args['distribution'])
        if config['neg_sampling_alias']:
            sampler.enable_alias(config['seed'])
        train_kwargs['sampler'] = sampler.set_phase('train')
        train_kwargs['neg_sample_args'] = train_args
    train_data = get_data_loader('train', config, train_args)(**train_kwargs)

    eval_kwargs = {'config': config, 'batch_size': config['eval_batch_size'],
                   'dl_format': config['MODEL_INPUT_TYPE'].__class__.POINTWISE, 'shuffle': False}
    valid_kwargs = dict(eval_kwargs, dataset=valid_dataset)
    test_kwargs = dict(eval_kwargs, dataset=test_dataset)
    if eval_args['strategy'] != 'none':
        if sampler is None:
            if model_type != ModelType.SEQUENTIAL:
                sampler = Sampler(phases, built, eval_args['distribution'])
            else:
                sampler = RepeatableSampler(phases, dataset, eval_args['distribution'])
            if config['neg_sampling_alias']:
                sampler.enable_alias(config['seed'])
        else:
            sampler.set_distribution(eval_args['distribution'])
        test_kwargs['neg_sample_args'] = eval_args
        valid_kwargs['neg_sample_args'] = valid_args
        valid_kwargs['sampler'] = sampler.set_phase('valid')
        test_kwargs['sampler'] = sampler.set_phase('test')
    valid_data = get_data_loader('evaluation', config, valid_args)(**valid_kwargs)
    test_data = get_data_loader('evaluation', config, eval_args)(**test_kwargs)
    if save:
        save_split_dataloaders(config, dataloaders=(train_data, valid_data, test_data))
    return train_data, valid_data, test_data


def save_split_dataloaders(config, dataloaders):
    """Write the (train, valid, test) loaders to
    `<checkpoint_dir>/<dataset>-for-<model>-dataloader.pth` (data/utils.py:188-200).
    Device tensors are written with their device; reload on a machine that has it."""
    ensure_dir(config['checkpoint_dir'])
    path = os.path.join(config['checkpoint_dir'],
                        f'{config["dataset"]}-for-{config["model"]}-dataloader.pth')
    getLogger().info(f'Saved split dataloaders: {path}')
    with open(path, 'wb') as f:
        pickle.dump(dataloaders, f)
    return path


def load_split_dataloaders(saved_dataloaders_file):
    """Read loaders written by save_split_dataloaders (data/utils.py:203-215). The file
    is a pickle: load only files this build wrote itself."""
    with open(saved_dataloaders_file, 'rb') as f:
        return pickle.load(f)
