"""LightGCN (mirror of recbole/model/general_recommender/lightgcn.py:32-180).

Same parameters (user_embedding.weight, item_embedding.weight), same init
(xavier_uniform_ on the CPU generator, user then item), same plugin methods and
the same loss: BPR on the propagated embeddings + reg_weight * EmbLoss of the
ego embeddings (:128-152). The arithmetic runs in hand-written gfx950 kernels:

* the normalised adjacency A_hat = D^-1/2 (A + A^T) D^-1/2 (:71-104) is built
  on the host once (vectorised; the reference's dok_matrix._update at :89 is
  a private scipy API) and kept in HBM as a CSR + K7 load-balancing plan;
* forward() = L K7 SpMM launches with the layer mean fused into the last one
  (:115-127); the ego matrix cat(E_U, E_I) is never materialised;
* its backward = L K7 launches of the Horner form
  dE_0 = c G + A_hat (c G + A_hat (... c G)),  c = 1/(L+1), writing the two
  weight gradients directly (A_hat is symmetric);
* BPR on the propagated rows = K3 (bpr.py's _BPRLossFn), EmbLoss = gather +
  squared norm / scaled gather kernels.

Like the reference, the propagated tables cached for full-sort evaluation
(restore_user_e / restore_item_e) are cleared only by calculate_loss (:129-131).
"""
import numpy as np
import torch
import torch.nn as nn

from recbole_amd import ops
from recbole_amd.model.abstract_recommender import GeneralRecommender
from recbole_amd.model.general_recommender.bpr import _BPRLossFn
from recbole_amd.model.init import xavier_uniform_initialization
from recbole_amd.model.loss import BPRLoss, EmbLoss
from recbole_amd.utils import InputType


def norm_adj_csr(inter_rows, inter_cols, n_users, n_items):
    """CSR (row_ptr int64, cols int32, vals float32) of the reference's
    norm_adj_matrix (lightgcn.py:71-104) over n_users + n_items nodes.

    Entries: (u, U+i) and (U+i, u) for every distinct training pair (the dict of
    :86-88 deduplicates, value 1); deg = nonzeros per row + 1e-7 (float64,
    :91-93); value = float32(deg_r^-1/2 * deg_c^-1/2) computed in float64 as
    scipy's D * A * D does, then cast like torch.FloatTensor(L.data)."""
    U, N = n_users, n_users + n_items
    r = np.asarray(inter_rows, dtype=np.int64)
    c = np.asarray(inter_cols, dtype=np.int64) + U
    key = np.unique(np.concatenate([r * N + c, c * N + r]))   # sorted by (row, col)
    rows, cols = key // N, key % N
    deg = np.bincount(rows, minlength=N).astype(np.float64)
    dinv = np.power(deg + 1e-7, -0.5)
    vals = (dinv[rows] * dinv[cols]).astype(np.float32)
    row_ptr = np.zeros(N + 1, dtype=np.int64)
    np.cumsum(np.bincount(rows, minlength=N), out=row_ptr[1:])
    return row_ptr, cols.astype(np.int32), vals


def propagate(plan, EU, EI, n_layers, out_u=None, out_i=None, tmp=None):
    """Mean of [E_0, A E_0, ..., A^L E_0] with E_0 = cat(EU, EI), written to
    (out_u, out_i) — K7 launches only (lightgcn.py:115-127)."""
    U, d = EU.shape
    dev = EU.device
    out_u = torch.empty_like(EU) if out_u is None else out_u
    out_i = torch.empty_like(EI) if out_i is None else out_i
    ego, out = (EU, EI), (out_u, out_i)
    if n_layers == 0:
        out_u.copy_(EU)
        out_i.copy_(EI)
        return out_u, out_i
    c = 1.0 / (n_layers + 1)
    bufs = [torch.empty(plan.n_rows, d, dtype=torch.float32, device=dev)
            for _ in range(min(n_layers - 1, 2))] if tmp is None else tmp
    x = ego
    for layer in range(n_layers):
        last = layer == n_layers - 1
        y = None if last else bufs[layer % 2]
        ops.spmm_csr(plan, x, y=y, acc_in=ego if layer == 0 else out, acc_out=out,
                     acc_scale=c if last else 1.0)
        x = y
    return out_u, out_i


def propagate_backward(plan, GU, GI, n_layers, dEU=None, dEI=None):
    """Gradient of propagate() w.r.t. (EU, EI) given the output gradient
    (GU, GI): dE_0 = c G + A (c G + A (... + A (c G))) with c = 1/(L+1)."""
    dEU = torch.empty_like(GU) if dEU is None else dEU
    dEI = torch.empty_like(GI) if dEI is None else dEI
    G, out = (GU, GI), (dEU, dEI)
    if n_layers == 0:
        dEU.copy_(GU)
        dEI.copy_(GI)
        return dEU, dEI
    c = 1.0 / (n_layers + 1)
    d = GU.shape[1]
    bufs = [torch.empty(plan.n_rows, d, dtype=torch.float32, device=GU.device)
            for _ in range(min(n_layers - 1, 2))]
    # H_{L-1} = c (G + A G); H_l = c G + A H_{l+1}; dE_0 = H_0
    first_out = out if n_layers == 1 else bufs[0]
    ops.spmm_csr(plan, G, acc_in=G, acc_out=first_out, acc_scale=c)
    h = first_out
    for k in range(1, n_layers):
        y = out if k == n_layers - 1 else bufs[k % 2]
        ops.spmm_csr(plan, h, y=y, add=G, add_scale=c)
        h = y
    return dEU, dEI


class _PropagateFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, EU, EI, plan, n_layers):
        ctx.plan, ctx.n_layers = plan, n_layers
        return propagate(plan, EU.detach(), EI.detach(), n_layers)

    @staticmethod
    def backward(ctx, gU, gI):
        if gU is None:
            gU = torch.zeros((ctx.plan.n_rows - gI.shape[0], gI.shape[1]), device=gI.device)
        if gI is None:
            gI = torch.zeros((ctx.plan.n_rows - gU.shape[0], gU.shape[1]), device=gU.device)
        dEU, dEI = propagate_backward(ctx.plan, gU.contiguous(), gI.contiguous(), ctx.n_layers)
        return dEU, dEI, None, None


class _EmbRegFn(torch.autograd.Function):
    """EmbLoss(E_U[user], E_I[pos], E_I[neg]) = (sum of Frobenius norms) / R
    (loss.py:79-84), forward and backward on the device."""

    @staticmethod
    def forward(ctx, EU, EI, user, pos, neg):
        R = neg.numel()
        sq = torch.cat([ops.fixed_sum(ops.gather_sqnorm(EU.detach(), user)),
                        ops.fixed_sum(ops.gather_sqnorm(EI.detach(), pos)),
                        ops.fixed_sum(ops.gather_sqnorm(EI.detach(), neg))])
        norms = torch.sqrt(sq)
        ctx.save_for_backward(EU, EI, user, pos, neg, norms)
        ctx.R = R
        loss = torch.zeros(1, device=EU.device)
        loss += norms[0:1]
        loss += norms[1:2]
        loss += norms[2:3]
        return loss / R

    @staticmethod
    def backward(ctx, g):
        EU, EI, user, pos, neg, norms = ctx.saved_tensors
        scale = (g.reshape(1) / ctx.R) / norms          # d ||X|| / dX = X / ||X||
        dEU = torch.zeros_like(EU)
        dEI = torch.zeros_like(EI)
        ops.segment_scatter_add(ops.gather_scale_rows(EU.detach(), user, scale[0:1]),
                                ops.segment_sort(user, EU.shape[0]), dEU)
        items = torch.cat([pos, neg])
        rows = torch.cat([ops.gather_scale_rows(EI.detach(), pos, scale[1:2]),
                          ops.gather_scale_rows(EI.detach(), neg, scale[2:3])])
        ops.segment_scatter_add(rows, ops.segment_sort(items, EI.shape[0]), dEI)
        return dEU, dEI, None, None, None


class LightGCN(GeneralRecommender):
    input_type = InputType.PAIRWISE

    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.interaction_matrix = dataset.inter_matrix(form='coo').astype(np.float32)
        self.latent_dim = config['embedding_size']
        self.n_layers = config['n_layers']
        self.reg_weight = config['reg_weight']
        self.user_embedding = nn.Embedding(self.n_users, self.latent_dim)
        self.item_embedding = nn.Embedding(self.n_items, self.latent_dim)
        self.mf_loss = BPRLoss()
        self.reg_loss = EmbLoss()
        self.restore_user_e = None
        self.restore_item_e = None
        m = self.interaction_matrix
        self.norm_adj_csr = norm_adj_csr(m.row, m.col, self.n_users, self.n_items)
        self._plan = None
        self.apply(xavier_uniform_initialization)

    @property
    def norm_adj_plan(self):
        """Device CSR + K7 plan, built on first use on the parameters' device."""
        dev = self.user_embedding.weight.device
        if self._plan is None or self._plan.row_ptr.device != dev:
            self._plan = ops.SpmmPlan(*self.norm_adj_csr, device=dev)
        return self._plan

    def forward(self):
        return _PropagateFn.apply(self.user_embedding.weight, self.item_embedding.weight,
                                  self.norm_adj_plan, self.n_layers)

    def calculate_loss(self, interaction):
        if self.restore_user_e is not None or self.restore_item_e is not None:
            self.restore_user_e, self.restore_item_e = None, None
        user = interaction[self.USER_ID].contiguous()
        pos_item = interaction[self.ITEM_ID].contiguous()
        neg_item = interaction[self.NEG_ITEM_ID].contiguous()
        user_all, item_all = self.forward()
        mf_loss = _BPRLossFn.apply(user_all, item_all, user, pos_item, neg_item)
        reg_loss = _EmbRegFn.apply(self.user_embedding.weight, self.item_embedding.weight,
                                   user, pos_item, neg_item)
        return mf_loss + self.reg_weight * reg_loss

    def predict(self, interaction):
        with torch.no_grad():
            user_all, item_all = self.forward()
        return ops.dot_rows(user_all, item_all, interaction[self.USER_ID],
                            interaction[self.ITEM_ID])

    def _restore(self):
        if self.restore_user_e is None or self.restore_item_e is None:
            with torch.no_grad():
                self.restore_user_e, self.restore_item_e = self.forward()
        return self.restore_user_e, self.restore_item_e

    def full_sort_predict(self, interaction):
        user_e, item_e = self._restore()
        u = ops.gather_rows(user_e, interaction[self.USER_ID])
        return ops.score_matrix(u, item_e).view(-1)

    # ------------------------------------------------------------------ fused eval hooks
    def fused_user_vectors(self, user_ids):
        return ops.gather_rows(self._restore()[0], user_ids)

    def fused_item_table(self):
        return self._restore()[1]
