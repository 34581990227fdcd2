from recbole_amd.data.interaction import Interaction, cat_interactions
from recbole_amd.data.utils import (create_dataset, data_preparation, get_data_loader,
                                    load_split_dataloaders, save_split_dataloaders)

__all__ = ['Interaction', 'cat_interactions', 'create_dataset', 'data_preparation',
           'get_data_loader', 'save_split_dataloaders', 'load_split_dataloaders']
