from recbole_amd.trainer.optim import FusedAdam
from recbole_amd.trainer.trainer import AbstractTrainer, Trainer

__all__ = ['AbstractTrainer', 'Trainer', 'FusedAdam']
