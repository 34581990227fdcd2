from recbole_amd.config.configurator import Config
from recbole_amd.config.eval_setting import EvalSetting

__all__ = ['Config', 'EvalSetting']
