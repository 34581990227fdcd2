from recbole_amd.data.interaction import Interaction, cat_interactions
from recbole_amd.data.utils import create_dataset, data_preparation, get_data_loader

__all__ = ['Interaction', 'cat_interactions', 'create_dataset', 'data_preparation',
           'get_data_loader']
