"""Loader classes, exported under the reference's names (recbole/data/dataloader/__init__.py:1-5):
`get_data_loader` resolves `{General|Context|Sequential}{DataLoader|NegSampleDataLoader|
FullDataLoader}` from this module by name (data/utils.py:254-272)."""
from recbole_amd.data.dataloader.abstract_dataloader import AbstractDataLoader
from recbole_amd.data.dataloader.context_dataloader import (ContextDataLoader,
                                                            ContextFullDataLoader,
                                                            ContextNegSampleDataLoader)
from recbole_amd.data.dataloader.general_dataloader import (GeneralDataLoader,
                                                            GeneralFullDataLoader,
                                                            GeneralNegSampleDataLoader)
from recbole_amd.data.dataloader.neg_sample_mixin import NegSampleByMixin, NegSampleMixin
from recbole_amd.data.dataloader.sequential_dataloader import (SequentialDataLoader,
                                                               SequentialFullDataLoader,
                                                               SequentialNegSampleDataLoader)

__all__ = ['AbstractDataLoader', 'NegSampleMixin', 'NegSampleByMixin',
           'GeneralDataLoader', 'GeneralNegSampleDataLoader', 'GeneralFullDataLoader',
           'ContextDataLoader', 'ContextNegSampleDataLoader', 'ContextFullDataLoader',
           'SequentialDataLoader', 'SequentialNegSampleDataLoader', 'SequentialFullDataLoader']
