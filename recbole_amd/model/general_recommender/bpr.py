"""BPR-MF (mirror of recbole/model/general_recommender/bpr.py:27-96).

Same parameters (user_embedding.weight, item_embedding.weight), same init
(xavier_normal_ on the CPU generator, user then item), same plugin methods.
The arithmetic runs in hand-written gfx950 kernels:

* calculate_loss  -> K3 fused gather + dot + BPR loss + per-row gradients,
                     wrapped in an autograd Function whose backward groups the
                     row gradients by table row (K2) and scatters them into the
                     dense weight gradients nn.Embedding(sparse=False) yields;
* predict         -> fused gather + dot (mirec_dot_rows_f32);
* full_sort_predict -> FP32-MFMA score matrix (mirec_score_matrix_f32).

The Trainer's fused path (recbole_amd/trainer/fused.py) bypasses autograd and
the dense gradients entirely: it calls fused_embedding_tables() and runs
K3 -> K2 -> K5 (dense Adam with compact gradients) per step, and
fused_full_sort_topk() for evaluation.
"""
import torch
import torch.nn as nn

from recbole_amd import ops
from recbole_amd.model.abstract_recommender import GeneralRecommender
from recbole_amd.model.init import xavier_normal_initialization
from recbole_amd.model.loss import BPRLoss
from recbole_amd.utils import InputType


class _BPRLossFn(torch.autograd.Function):
    """loss = mean_r -log(1e-10 + sigmoid(<u,p> - <u,n>)) with the embedding
    backward (bpr.py:74-83, loss.py:47-49)."""

    @staticmethod
    def forward(ctx, EU, EI, user, pos, neg):
        R = user.numel()
        o = ops.bpr_fwd_bwd(EU.detach(), EI.detach(), user, pos, neg, times=1, grads=True)
        loss = ops.fixed_sum(o['loss_k']).view(()) / R
        ctx.nU, ctx.nI = EU.shape[0], EI.shape[0]
        ctx.save_for_backward(user, torch.cat([pos, neg]), o['gU'], o['gI'])
        return loss

    @staticmethod
    def backward(ctx, g):
        user, item_keys, gU, gI = ctx.saved_tensors
        dEU = torch.zeros((ctx.nU, gU.shape[1]), dtype=gU.dtype, device=gU.device)
        dEI = torch.zeros((ctx.nI, gI.shape[1]), dtype=gI.dtype, device=gI.device)
        ops.segment_scatter_add(gU, ops.segment_sort(user, ctx.nU), dEU)
        ops.segment_scatter_add(gI, ops.segment_sort(item_keys, ctx.nI), dEI)
        if not (isinstance(g, torch.Tensor) and g.numel() == 1 and bool((g == 1).all())):
            dEU.mul_(g)
            dEI.mul_(g)
        return dEU, dEI, None, None, None


class BPR(GeneralRecommender):
    input_type = InputType.PAIRWISE

    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.embedding_size = config['embedding_size']
        self.user_embedding = nn.Embedding(self.n_users, self.embedding_size)
        self.item_embedding = nn.Embedding(self.n_items, self.embedding_size)
        self.loss = BPRLoss()
        self.apply(xavier_normal_initialization)

    def get_user_embedding(self, user):
        return ops.gather_rows(self.user_embedding.weight.detach(), user)

    def get_item_embedding(self, item):
        return ops.gather_rows(self.item_embedding.weight.detach(), item)

    def forward(self, user, item):
        return self.get_user_embedding(user), self.get_item_embedding(item)

    def calculate_loss(self, interaction):
        user = interaction[self.USER_ID].contiguous()
        pos_item = interaction[self.ITEM_ID].contiguous()
        neg_item = interaction[self.NEG_ITEM_ID].contiguous()
        return _BPRLossFn.apply(self.user_embedding.weight, self.item_embedding.weight, user,
                                pos_item, neg_item)

    def predict(self, interaction):
        return ops.dot_rows(self.user_embedding.weight.detach(),
                            self.item_embedding.weight.detach(),
                            interaction[self.USER_ID], interaction[self.ITEM_ID])

    def full_sort_predict(self, interaction):
        u = self.get_user_embedding(interaction[self.USER_ID])
        return ops.score_matrix(u, self.item_embedding.weight.detach()).view(-1)

    # ------------------------------------------------------------------ fused hooks
    def fused_embedding_tables(self):
        """(parameter, key space) pairs the fused trainer updates with K5."""
        return [(self.user_embedding.weight, self.n_users),
                (self.item_embedding.weight, self.n_items)]

    def fused_user_vectors(self, user_ids):
        """User-side vectors ranked by the full-sort scorer (K6)."""
        return ops.gather_rows(self.user_embedding.weight.detach(), user_ids)

    def fused_item_table(self):
        return self.item_embedding.weight.detach()
