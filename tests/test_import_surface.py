"""The drop-in import surface: every in-scope module path and public name of the
reference (SURVEY.md §2 rows marked ★A / ★H) resolves through `recbole.*`, and
`recbole.X` is the same module object as `recbole_amd.X`. Reference paths:
recbole/{quick_start,config,data,data/dataset,data/dataloader,sampler,model,trainer,
evaluator,utils}/__init__.py and the modules named below."""
import importlib

import pytest

SURFACE = {
    'recbole.quick_start': ['run_recbole', 'objective_function'],
    'recbole.quick_start.quick_start': ['run_recbole', 'objective_function'],
    'recbole.config': ['Config', 'EvalSetting'],
    'recbole.config.configurator': ['Config'],
    'recbole.config.eval_setting': ['EvalSetting'],
    'recbole.data': ['create_dataset', 'data_preparation', 'save_split_dataloaders',
                     'load_split_dataloaders'],
    'recbole.data.utils': ['create_dataset', 'data_preparation', 'get_data_loader',
                           'save_split_dataloaders', 'load_split_dataloaders', 'dlapi'],
    'recbole.data.interaction': ['Interaction', 'cat_interactions'],
    'recbole.data.dataset': ['Dataset', 'SequentialDataset'],
    'recbole.data.dataset.dataset': ['Dataset'],
    'recbole.data.dataset.sequential_dataset': ['SequentialDataset'],
    'recbole.data.dataloader': [
        'AbstractDataLoader', 'NegSampleMixin', 'NegSampleByMixin', 'GeneralDataLoader',
        'GeneralNegSampleDataLoader', 'GeneralFullDataLoader', 'ContextDataLoader',
        'ContextNegSampleDataLoader', 'ContextFullDataLoader', 'SequentialDataLoader',
        'SequentialNegSampleDataLoader', 'SequentialFullDataLoader'],
    'recbole.data.dataloader.abstract_dataloader': ['AbstractDataLoader'],
    'recbole.data.dataloader.neg_sample_mixin': ['NegSampleMixin', 'NegSampleByMixin'],
    'recbole.data.dataloader.general_dataloader': [
        'GeneralDataLoader', 'GeneralNegSampleDataLoader', 'GeneralFullDataLoader'],
    'recbole.data.dataloader.context_dataloader': [
        'ContextDataLoader', 'ContextNegSampleDataLoader', 'ContextFullDataLoader'],
    'recbole.data.dataloader.sequential_dataloader': [
        'SequentialDataLoader', 'SequentialNegSampleDataLoader', 'SequentialFullDataLoader'],
    'recbole.sampler': ['Sampler', 'RepeatableSampler'],
    'recbole.sampler.sampler': ['AbstractSampler', 'Sampler', 'RepeatableSampler'],
    'recbole.model.abstract_recommender': [
        'AbstractRecommender', 'GeneralRecommender', 'SequentialRecommender',
        'ContextRecommender'],
    'recbole.model.layers': [
        'MLPLayers', 'MultiHeadAttention', 'FeedForward', 'TransformerLayer',
        'TransformerEncoder', 'FMEmbedding', 'BaseFactorizationMachine', 'FMFirstOrderLinear'],
    'recbole.model.loss': ['BPRLoss', 'EmbLoss'],
    'recbole.model.init': ['xavier_normal_initialization', 'xavier_uniform_initialization'],
    'recbole.model.general_recommender': ['BPR', 'LightGCN'],
    'recbole.model.general_recommender.bpr': ['BPR'],
    'recbole.model.general_recommender.lightgcn': ['LightGCN'],
    'recbole.model.sequential_recommender': ['SASRec'],
    'recbole.model.sequential_recommender.sasrec': ['SASRec'],
    'recbole.model.context_aware_recommender': ['DeepFM'],
    'recbole.model.context_aware_recommender.deepfm': ['DeepFM'],
    'recbole.trainer': ['Trainer'],
    'recbole.trainer.trainer': ['AbstractTrainer', 'Trainer'],
    'recbole.evaluator': ['ProxyEvaluator', 'TopKEvaluator', 'LossEvaluator', 'BaseEvaluator',
                          'GroupedEvaluator', 'IndividualEvaluator', 'metrics_dict'],
    'recbole.evaluator.abstract_evaluator': [
        'BaseEvaluator', 'GroupedEvaluator', 'IndividualEvaluator'],
    'recbole.evaluator.evaluators': ['TopKEvaluator', 'LossEvaluator', 'metric_eval_bind'],
    'recbole.evaluator.proxy_evaluator': ['ProxyEvaluator'],
    'recbole.evaluator.metrics': ['hit_', 'mrr_', 'map_', 'recall_', 'ndcg_', 'precision_',
                                  'auc_', 'mae_', 'rmse_', 'log_loss_', 'metrics_dict'],
    'recbole.utils': [
        'init_logger', 'get_local_time', 'ensure_dir', 'get_model', 'get_trainer',
        'early_stopping', 'calculate_valid_score', 'dict2str', 'init_seed', 'ModelType',
        'DataLoaderType', 'KGDataLoaderState', 'EvaluatorType', 'InputType', 'FeatureType',
        'FeatureSource', 'general_arguments', 'training_arguments', 'evaluation_arguments',
        'dataset_arguments'],
    'recbole.utils.utils': ['get_model', 'get_trainer', 'init_seed'],
    'recbole.utils.logger': ['init_logger'],
    'recbole.utils.enum_type': ['ModelType', 'InputType', 'KGDataLoaderState'],
    'recbole.utils.argument_list': [
        'general_arguments', 'training_arguments', 'evaluation_arguments', 'dataset_arguments'],
    'recbole.utils.case_study': ['full_sort_scores', 'full_sort_topk'],
}


@pytest.mark.parametrize('path', sorted(SURFACE))
def test_module_and_names(path):
    mod = importlib.import_module(path)
    real = importlib.import_module('recbole_amd' + path[len('recbole'):])
    assert mod is real
    missing = [n for n in SURFACE[path] if not hasattr(mod, n)]
    assert not missing, f'{path}: {missing}'


def test_get_data_loader_by_name():
    """data/utils.py:254-272: <family><strategy> resolved from recbole.data.dataloader."""
    from recbole.data import dataloader as dl
    from recbole.data.utils import get_data_loader
    from recbole.utils import ModelType
    fam = {ModelType.GENERAL: 'General', ModelType.TRADITIONAL: 'General',
           ModelType.CONTEXT: 'Context', ModelType.SEQUENTIAL: 'Sequential'}
    kind = {'none': 'DataLoader', 'by': 'NegSampleDataLoader', 'full': 'FullDataLoader'}
    for mt, f in fam.items():
        for s, k in kind.items():
            cls = get_data_loader('train', {'MODEL_TYPE': mt}, {'strategy': s})
            assert cls is getattr(dl, f + k)
    with pytest.raises(NotImplementedError):
        get_data_loader('train', {'MODEL_TYPE': ModelType.KNOWLEDGE}, {'strategy': 'by'})
    assert issubclass(dl.ContextNegSampleDataLoader, dl.GeneralNegSampleDataLoader)
    assert issubclass(dl.SequentialNegSampleDataLoader, dl.NegSampleByMixin)


def test_abstract_protocols_raise():
    from recbole.evaluator.abstract_evaluator import BaseEvaluator, IndividualEvaluator
    cfg = {'eval_setting': 'RO_RS,full', 'metric_decimal_place': 4}
    with pytest.raises(NotImplementedError):
        BaseEvaluator(cfg, ['hit']).collect()
    with pytest.raises(NotImplementedError):
        IndividualEvaluator(cfg, ['auc'])


def test_grouped_sample_collect_pads():
    """GroupedEvaluator.sample_collect: per-user rows padded with -inf to the longest
    user and at least max(topk) columns (abstract_evaluator.py:58-76 of the reference)."""
    import numpy as np
    import torch
    from recbole.evaluator.abstract_evaluator import GroupedEvaluator
    ev = GroupedEvaluator({'eval_setting': 'RO_RS,uni100', 'metric_decimal_place': 4}, ['hit'])
    ev.topk = [3, 5]
    sc = torch.arange(1, 12, dtype=torch.float32)
    m = ev.sample_collect(sc, [3, 1, 7])
    assert m.shape == (3, 7)
    assert m[0, :3].tolist() == [1, 2, 3] and m[1, 0] == 4 and m[2].tolist() == list(range(5, 12))
    assert torch.isinf(m[0, 3:]).all() and torch.isinf(m[1, 1:]).all()
    assert ev.sample_collect(sc[:2], [1, 1]).shape == (2, 5)
    assert np.isneginf(ev.sample_collect(sc[:2], [1, 1])[:, 1:].numpy()).all()


def test_cli_flags():
    """run_recbole.py keeps the reference's flags (run_recbole.py:18-21)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import run_recbole
    o = run_recbole._options(['-m', 'BPR', '-d', 'ml-100k', '--config_files', 'a.yaml b.yaml',
                              '--alpha', '0.5', '--epochs=3'])
    assert (o.model, o.dataset, o.config_files, o.alpha) == ('BPR', 'ml-100k',
                                                             'a.yaml b.yaml', 0.5)


def test_split_dataloaders_round_trip(tmp_path):
    """data_preparation(save=True) -> load_split_dataloaders (data/utils.py:188-215) on the
    bundled C1 data: the reloaded test loader yields the same full-sort 5-tuples."""
    import os

    import torch

    from conftest import ROOT
    from recbole.config import Config
    from recbole.data import create_dataset, data_preparation, load_split_dataloaders
    from recbole.utils import init_seed
    config = Config(model='BPR', dataset='ml-100k',
                    config_dict={'data_path': os.path.join(ROOT, 'dataset'), 'use_gpu': False,
                                 'state': 'ERROR', 'checkpoint_dir': str(tmp_path)})
    init_seed(config['seed'], config['reproducibility'])
    train, valid, test = data_preparation(config, create_dataset(config), save=True)
    path = tmp_path / 'ml-100k-for-BPR-dataloader.pth'
    t2, v2, e2 = load_split_dataloaders(str(path))
    assert (len(t2), len(v2), len(e2)) == (len(train), len(valid), len(test))
    for a, b in zip(test, e2):
        user_a, (hr_a, hc_a), sr_a, sa_a, sb_a = a
        user_b, (hr_b, hc_b), sr_b, sa_b, sb_b = b
        for x, y in ((hr_a, hr_b), (hc_a, hc_b), (sr_a, sr_b), (sa_a, sa_b), (sb_a, sb_b)):
            assert torch.equal(x, y)
        assert torch.equal(user_a[config['USER_ID_FIELD']], user_b[config['USER_ID_FIELD']])
