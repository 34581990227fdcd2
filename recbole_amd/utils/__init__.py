from recbole_amd.utils.argument_list import (dataset_arguments, evaluation_arguments,
                                             general_arguments, training_arguments)
from recbole_amd.utils.enum_type import (DataLoaderType, EvaluatorType, FeatureSource,
                                         FeatureType, InputType, KGDataLoaderState, ModelType)
from recbole_amd.utils.logger import init_logger
from recbole_amd.utils.utils import (calculate_valid_score, dict2str, early_stopping, ensure_dir,
                                     get_local_time, get_model, get_trainer, init_seed, set_color)

__all__ = ['ModelType', 'DataLoaderType', 'KGDataLoaderState', 'EvaluatorType', 'InputType',
           'FeatureType', 'FeatureSource', 'init_logger', 'get_local_time', 'ensure_dir', 'get_model',
           'get_trainer', 'early_stopping', 'calculate_valid_score', 'dict2str', 'init_seed',
           'set_color', 'general_arguments', 'training_arguments', 'evaluation_arguments',
           'dataset_arguments']
