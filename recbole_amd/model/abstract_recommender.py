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

from recbole_amd.utils import InputType, ModelType


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


class ContextRecommender(AbstractRecommender):
    """Context-aware base (abstract_recommender.py:151-412): one FMEmbedding over
    the token fields, one embedding per token_seq field, one [n_float, d] table
    for the float fields, and FMFirstOrderLinear — same modules, names and
    construction order as the reference. The embedding of a batch runs in the
    fused K8 kernel (csrc/context.hip) through `fm_fields(interaction)`, which
    returns both the concatenated field rows and y_fm = first order + FM."""
    type = ModelType.CONTEXT
    input_type = InputType.POINTWISE

    def __init__(self, config, dataset):
        super().__init__()
        from recbole_amd.model.layers import FMEmbedding, FMFirstOrderLinear, _split_fields
        self.field_names = dataset.fields()
        self.LABEL = config['LABEL_FIELD']
        self.embedding_size = config['embedding_size']
        self.device = config['device']
        self.double_tower = config['double_tower'] if 'double_tower' in config else None
        if self.double_tower:
            raise NotImplementedError('double_tower context models are not part of this build')
        self.double_tower = False
        (self.token_field_names, self.token_field_dims, self.token_seq_field_names,
         self.token_seq_field_dims, self.float_field_names,
         self.float_field_dims) = _split_fields(config, dataset)
        self.num_feature_field = (len(self.token_field_names) + len(self.token_seq_field_names)
                                  + len(self.float_field_names))
        self.token_field_offsets = np.zeros(0, dtype=np.int64)
        if len(self.token_field_dims) > 0:
            self.token_field_offsets = np.array((0, *np.cumsum(self.token_field_dims)[:-1]),
                                                dtype=np.int64)
            self.token_embedding_table = FMEmbedding(self.token_field_dims,
                                                     self.token_field_offsets,
                                                     self.embedding_size)
        if len(self.float_field_dims) > 0:
            self.float_embedding_table = nn.Embedding(int(np.sum(self.float_field_dims)),
                                                      self.embedding_size)
        if len(self.token_seq_field_dims) > 0:
            self.token_seq_embedding_table = nn.ModuleList()
            for dim in self.token_seq_field_dims:
                self.token_seq_embedding_table.append(nn.Embedding(dim, self.embedding_size))
        self.first_order_linear = FMFirstOrderLinear(config, dataset)
        from recbole_amd.model.context import FieldLayout
        self.field_layout = FieldLayout(self.token_field_names, self.token_seq_field_names,
                                        self.float_field_names, self.token_field_offsets)

    def _fm_params(self):
        fo = self.first_order_linear
        T = self.token_embedding_table.embedding.weight if self.token_field_names else None
        T1 = fo.token_embedding_table.embedding.weight if self.token_field_names else None
        Ef = self.float_embedding_table.weight if self.float_field_names else None
        Ef1 = fo.float_embedding_table.weight if self.float_field_names else None
        seq = [e.weight for e in self.token_seq_embedding_table] \
            if self.token_seq_field_names else []
        seq1 = [e.weight for e in fo.token_seq_embedding_table] \
            if self.token_seq_field_names else []
        return T, T1, Ef, Ef1, fo.bias, seq, seq1

    def fm_fields(self, interaction):
        """(concat [B, num_feature_field, d], y_fm [B]) via K8, differentiable."""
        from recbole_amd.model.context import _CtxFMFn
        T, T1, Ef, Ef1, bias, seq, seq1 = self._fm_params()
        return _CtxFMFn.apply(self.field_layout, interaction, T, T1, Ef, Ef1, bias, *seq, *seq1)

    def concat_embed_input_fields(self, interaction):
        """[B, num_feature_field, d] (abstract_recommender.py:356-363)."""
        return self.fm_fields(interaction)[0]


class SequentialRecommender(AbstractRecommender):
    """abstract_recommender.py:97-121."""
    type = ModelType.SEQUENTIAL

    def __init__(self, config, dataset):
        super().__init__()
        self.USER_ID = config['USER_ID_FIELD']
        self.ITEM_ID = config['ITEM_ID_FIELD']
        self.ITEM_SEQ = self.ITEM_ID + config['LIST_SUFFIX']
        self.ITEM_SEQ_LEN = config['ITEM_LIST_LENGTH_FIELD']
        self.POS_ITEM_ID = self.ITEM_ID
        self.NEG_ITEM_ID = config['NEG_PREFIX'] + self.ITEM_ID
        self.max_seq_length = config['MAX_ITEM_LIST_LENGTH']
        self.n_items = dataset.num(self.ITEM_ID)

    def gather_indexes(self, output, gather_index):
        """Vectors at the given positions over a minibatch (:117-121)."""
        gather_index = gather_index.view(-1, 1, 1).expand(-1, -1, output.shape[-1])
        return output.gather(dim=1, index=gather_index).squeeze(1)
