"""DeepFM (mirror of recbole/model/context_aware_recommender/deepfm.py:26-73).

y = sigmoid(first_order + FM + MLP(concat of field rows)), nn.BCELoss. The
field embedding, first-order term and FM term run in the fused K8 kernel
(ContextRecommender.fm_fields); MLPLayers + deep_predict_layer run in K10
(model/mlp.py: one forward, two backward launches on fp32 MFMA); the
sigmoid + BCE and its gradient run in mirec_sigmoid_bce_f32. Same modules and
init (xavier_normal_ weights, zero biases, apply order) as the reference.
"""
import torch.nn as nn
from torch.nn.init import constant_, xavier_normal_

from recbole_amd.model.abstract_recommender import ContextRecommender
from recbole_amd.model.context import _SigmoidBCEFn, sigmoid_prob
from recbole_amd.model.layers import BaseFactorizationMachine, MLPLayers
from recbole_amd.model.mlp import deep_forward


class DeepFM(ContextRecommender):

    # the training step has no host synchronisation or host-side branching on device
    # values: the trainer may capture it in a HIP graph (trainer/graph_step.py)
    graph_step_safe = True

    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.mlp_hidden_size = config['mlp_hidden_size']
        self.dropout_prob = config['dropout_prob']
        self.fm = BaseFactorizationMachine(reduce_sum=True)
        size_list = [self.embedding_size * self.num_feature_field] + self.mlp_hidden_size
        self.mlp_layers = MLPLayers(size_list, self.dropout_prob)
        self.deep_predict_layer = nn.Linear(self.mlp_hidden_size[-1], 1)
        self.sigmoid = nn.Sigmoid()
        self.loss = nn.BCELoss()
        self.apply(self._init_weights)

    def _init_weights(self, module):
        if isinstance(module, nn.Embedding):
            xavier_normal_(module.weight.data)
        elif isinstance(module, nn.Linear):
            xavier_normal_(module.weight.data)
            if module.bias is not None:
                constant_(module.bias.data, 0)

    def _logits(self, interaction):
        concat, y_fm = self.fm_fields(interaction)
        B = concat.shape[0]
        y_deep = deep_forward(self.mlp_layers, self.deep_predict_layer, concat.view(B, -1))
        return y_fm, y_deep

    def forward(self, interaction):
        y_fm, y_deep = self._logits(interaction)
        return sigmoid_prob(y_fm, y_deep).squeeze()

    def calculate_loss(self, interaction):
        y_fm, y_deep = self._logits(interaction)
        return _SigmoidBCEFn.apply(y_fm, y_deep, interaction[self.LABEL])

    def predict(self, interaction):
        return self.forward(interaction)

    def deferred_tables(self):
        """Tables the trainer may run on the deferred K5 schedule (only rows a
        batch reads are touched): the token table [V, d] and the first-order
        token weights [V, 1], read by the same rows."""
        if not self.token_field_names:
            return []
        return [self.token_embedding_table.embedding.weight,
                self.first_order_linear.token_embedding_table.embedding.weight]
