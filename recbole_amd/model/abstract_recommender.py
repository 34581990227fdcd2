"""Model base classes (mirror of recbole/model/abstract_recommender.py:26-95).

Besides the reference's plugin contract (calculate_loss / predict /
full_sort_predict), a model may expose the fused hooks the MI355X Trainer
uses when present:
  fused_embedding_tables() -> list of (nn.Parameter, key_space) updated by K5
  fused_full_sort_topk(user_ids, hist, pos, K) -> K6 result
"""
from logging import getLogger

import numpy as np
import torch.nn as nn

from recbole_amd.utils import ModelType


class AbstractRecommender(nn.Module):

    def __init__(self):
        self.logger = getLogger()
        super().__init__()

    def calculate_loss(self, interaction):
        raise NotImplementedError

    def predict(self, interaction):
        raise NotImplementedError

    def full_sort_predict(self, interaction):
        raise NotImplementedError

    def __str__(self):
        params = sum(int(np.prod(p.size())) for p in self.parameters() if p.requires_grad)
        return super().__str__() + f'\nTrainable parameters: {params}'


class GeneralRecommender(AbstractRecommender):
    type = ModelType.GENERAL

    def __init__(self, config, dataset):
        super().__init__()
        self.USER_ID = config['USER_ID_FIELD']
        self.ITEM_ID = config['ITEM_ID_FIELD']
        self.NEG_ITEM_ID = config['NEG_PREFIX'] + self.ITEM_ID
        self.n_users = dataset.num(self.USER_ID)
        self.n_items = dataset.num(self.ITEM_ID)
        self.device = config['device']
