from recbole_amd.data.dataloader.abstract_dataloader import AbstractDataLoader
from recbole_amd.data.dataloader.general_dataloader import (GeneralDataLoader,
                                                            GeneralFullDataLoader,
                                                            GeneralNegSampleDataLoader)

__all__ = ['AbstractDataLoader', 'GeneralDataLoader', 'GeneralNegSampleDataLoader',
           'GeneralFullDataLoader']
