"""SASRec (mirror of recbole/model/sequential_recommender/sasrec.py:25-158).

Same modules, names and init as the reference. The embedding side and the
losses run in hand-written gfx950 kernels:

* item gather + position add + LayerNorm (:107-114) -> K9a seq_embed_ln, whose
  backward returns per-position item-row gradients for the K2 grouping
  (padding row 0 gets none) and the LayerNorm / position gradients;
* loss_type 'BPR' (:126-134)  -> K3 fused dot + BPR + gradients on seq_output;
* loss_type 'SSM' (build extension for the C3 configuration: sampled softmax
  over the positive and neg_sample_num sampled negatives) -> K9b;
* loss_type 'CE' (:135-141)   -> full-vocabulary logits on the library GEMM +
  cross entropy (the reference's op sequence);
* full_sort_predict            -> FP32-MFMA score matrix; the trainer's fused
  evaluator ranks seq_output against all items with K6 (no score matrix).
The transformer encoder between them is the reference's op sequence on torch
(library GEMMs, softmax, LayerNorm).
"""
import torch
import torch.nn as nn

from recbole_amd import ops
from recbole_amd._native import check, lib, ptr, stream_handle
from recbole_amd.model.abstract_recommender import SequentialRecommender
from recbole_amd.model.layers import TransformerEncoder, _drop_rng, colsums
from recbole_amd.model.loss import BPRLoss


class _SeqEmbedLNFn(torch.autograd.Function):
    """LayerNorm(item_embedding[item_seq] + position_embedding[t]) (K9a)."""

    @staticmethod
    def forward(ctx, E, P, gamma, beta, item_seq, eps, p=0.0, rng=None):
        B, L = item_seq.shape
        d = E.shape[1]
        dev = E.device
        seq = item_seq.contiguous()
        h = getattr(E, '_mirec_deferred', None)
        # item 0 is the padding_idx (reference sasrec.py: nn.Embedding(..., padding_idx=0)):
        # no gradient, so its positions are left out of the grouping
        ctx.segs = h.catch_up(E, seq.view(-1), drop_key=0) if h is not None else None
        ctx.deferred = h is not None
        out = torch.empty(B, L, d, dtype=torch.float32, device=dev)
        mean = torch.empty(B * L, dtype=torch.float32, device=dev)
        rstd = torch.empty(B * L, dtype=torch.float32, device=dev)
        drawn = None
        if p > 0:                             # the embedding dropout folded in
            drawn = torch.empty(1, dtype=torch.int64, device=dev)
            rc = lib().mirec_seq_embed_ln_drop_fwd_f32(
                ptr(E.detach()), E.shape[0], ptr(P.detach()), ptr(seq), B, L, d,
                ptr(gamma.detach()), ptr(beta.detach()), eps, float(p), rng[0], ptr(rng[1]),
                ptr(drawn), ptr(out), ptr(mean), ptr(rstd), stream_handle())
            check(rc, "mirec_seq_embed_ln_drop_fwd_f32")
        else:
            rc = lib().mirec_seq_embed_ln_fwd_f32(ptr(E.detach()), E.shape[0], ptr(P.detach()),
                                                  ptr(seq), B, L, d, ptr(gamma.detach()),
                                                  ptr(beta.detach()), eps, ptr(out), ptr(mean),
                                                  ptr(rstd), stream_handle())
            check(rc, "mirec_seq_embed_ln_fwd_f32")
        ctx.save_for_backward(E, P, gamma, seq, mean, rstd, drawn)
        ctx.p, ctx.rng = p, rng
        return out

    @staticmethod
    def backward(ctx, g):
        E, P, gamma, seq, mean, rstd, drawn = ctx.saved_tensors
        B, L = seq.shape
        d = E.shape[1]
        dev = E.device
        n = B * L
        nparts = lib().mirec_seq_embed_ln_partials(n)
        dx = torch.empty(n, d, dtype=torch.float32, device=dev)
        ditem = torch.empty(n, d, dtype=torch.float32, device=dev)
        pg = torch.empty(nparts, d, dtype=torch.float32, device=dev)
        pb = torch.empty(nparts, d, dtype=torch.float32, device=dev)
        if ctx.p > 0:
            rc = lib().mirec_seq_embed_ln_drop_bwd_f32(
                ptr(E.detach()), E.shape[0], ptr(P.detach()), ptr(seq), B, L, d,
                ptr(gamma.detach()), ptr(mean), ptr(rstd), ptr(g.contiguous()), float(ctx.p),
                ctx.rng[0], ptr(drawn), ptr(ctx.rng[1]), ptr(dx), ptr(ditem), ptr(pg), ptr(pb),
                stream_handle())
            check(rc, "mirec_seq_embed_ln_drop_bwd_f32")
        else:
            rc = lib().mirec_seq_embed_ln_bwd_f32(ptr(E.detach()), E.shape[0], ptr(P.detach()),
                                                  ptr(seq), B, L, d, ptr(gamma.detach()),
                                                  ptr(mean), ptr(rstd), ptr(g.contiguous()),
                                                  ptr(dx), ptr(ditem), ptr(pg), ptr(pb),
                                                  stream_handle())
            check(rc, "mirec_seq_embed_ln_bwd_f32")
        if ctx.deferred:
            E._mirec_deferred.stash(E, ditem, seq.view(-1), ctx.segs)
            dE = None
        else:
            dE = ops.segment_scatter_add(ditem, ops.segment_sort(seq.view(-1), E.shape[0]),
                                         torch.zeros_like(E))
        dP = torch.zeros_like(P)
        dgamma = torch.empty_like(gamma)
        dbeta = torch.empty_like(gamma)
        colsums([(dx, B, L * d, dP), (pg, nparts, d, dgamma), (pb, nparts, d, dbeta)])
        return dE, dP, dgamma, dbeta, None, None, None, None


def _catch_up(ctx, E, items):
    h = getattr(E, '_mirec_deferred', None)
    ctx.deferred_E = E if h is not None else None
    # deferred Adam: complete the rows read (grouping reused by the backward)
    ctx.segs = h.catch_up(E, items.contiguous()) if h is not None else None


def _item_grad(ctx, gI, items):
    """Dense item-table gradient, or the compact rows handed to the deferred
    optimizer (then autograd gets None)."""
    if ctx.deferred_E is not None:
        ctx.deferred_E._mirec_deferred.stash(ctx.deferred_E, gI, items, ctx.segs)
        return None
    return ops.segment_scatter_add(gI, ops.segment_sort(items, ctx.nI),
                                   torch.zeros((ctx.nI, gI.shape[1]), device=gI.device))


class _SeqBPRFn(torch.autograd.Function):
    """BPRLoss(<s_r, E[pos_r]>, <s_r, E[neg_r]>) over R rows (K3 with the
    sequence outputs as the 'user' table, row r = user r)."""

    @staticmethod
    def forward(ctx, S, E, pos, neg):
        R = S.shape[0]
        rows = torch.arange(R, dtype=torch.int64, device=S.device)
        _catch_up(ctx, E, torch.cat([pos, neg]))
        o = ops.bpr_fwd_bwd(S.detach().contiguous(), E.detach(), rows, pos.contiguous(),
                            neg.contiguous(), times=1, grads=True)
        ctx.save_for_backward(torch.cat([pos, neg]), o['gU'], o['gI'])
        ctx.nI = E.shape[0]
        return ops.fixed_sum(o['loss_k']).view(()) / R

    @staticmethod
    def backward(ctx, g):
        items, gS, gI = ctx.saved_tensors
        return gS * g, _item_grad(ctx, gI * g, items), None, None


class _SampledSoftmaxFn(torch.autograd.Function):
    """mean_b [logsumexp(logits_b) - logit_b0], logits over [pos_b | negs_b] (K9b)."""

    @staticmethod
    def forward(ctx, S, E, pos, neg):
        B, d = S.shape
        N = neg.numel() // max(B, 1)
        dev = S.device
        loss = torch.empty(B, dtype=torch.float32, device=dev)
        gS = torch.empty(B, d, dtype=torch.float32, device=dev)
        gI = torch.empty((1 + N) * B, d, dtype=torch.float32, device=dev)
        _catch_up(ctx, E, torch.cat([pos, neg]))
        scale = float(torch.tensor(1.0) / torch.tensor(float(B)))
        rc = lib().mirec_sampled_softmax_f32(ptr(S.detach().contiguous()), ptr(E.detach()),
                                             E.shape[0], d, ptr(pos.contiguous()),
                                             ptr(neg.contiguous()), B, N, scale, ptr(loss),
                                             ptr(gS), ptr(gI), stream_handle())
        check(rc, "mirec_sampled_softmax_f32")
        ctx.save_for_backward(torch.cat([pos, neg]), gS, gI)
        ctx.nI = E.shape[0]
        return ops.fixed_sum(loss).view(()) / B

    @staticmethod
    def backward(ctx, g):
        items, gS, gI = ctx.saved_tensors
        if (g.is_cuda and g.dtype == torch.float32 and g.numel() == 1 and gI.is_contiguous()
                and gI.numel() % 4 == 0 and gI.data_ptr() % 16 == 0):
            # gI * g in place, a no-op launch when g == 1 (mirec_scale_by_f32): the saved
            # rows are this Function's own and serve one backward
            if getattr(ctx, 'scaled', False):
                raise RuntimeError('_SampledSoftmaxFn: one backward per forward')
            ctx.scaled = True
            check(lib().mirec_scale_by_f32(ptr(gI), gI.numel(), ptr(g.contiguous()),
                                           stream_handle()), 'mirec_scale_by_f32')
            return gS * g, _item_grad(ctx, gI, items), None, None
        return gS * g, _item_grad(ctx, gI * g, items), None, None


class SASRec(SequentialRecommender):

    # the training step has no host synchronisation or host-side branching on device
    # values (K9a / K9b / K3 launches with host-known sizes, deferred catch-ups on the
    # device step counter, dropout through torch's capture-aware generator): the
    # trainer may capture it in a HIP graph (trainer/graph_step.py)
    graph_step_safe = True

    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.n_layers = config['n_layers']
        self.n_heads = config['n_heads']
        self.hidden_size = config['hidden_size']
        self.inner_size = config['inner_size']
        self.hidden_dropout_prob = config['hidden_dropout_prob']
        self.attn_dropout_prob = config['attn_dropout_prob']
        self.hidden_act = config['hidden_act']
        self.layer_norm_eps = config['layer_norm_eps']
        self.initializer_range = config['initializer_range']
        self.loss_type = config['loss_type']
        self.item_embedding = nn.Embedding(self.n_items, self.hidden_size, padding_idx=0)
        self.position_embedding = nn.Embedding(self.max_seq_length, self.hidden_size)
        self.trm_encoder = TransformerEncoder(
            n_layers=self.n_layers, n_heads=self.n_heads, hidden_size=self.hidden_size,
            inner_size=self.inner_size, hidden_dropout_prob=self.hidden_dropout_prob,
            attn_dropout_prob=self.attn_dropout_prob, hidden_act=self.hidden_act,
            layer_norm_eps=self.layer_norm_eps)
        self.LayerNorm = nn.LayerNorm(self.hidden_size, eps=self.layer_norm_eps)
        self.dropout = nn.Dropout(self.hidden_dropout_prob)
        if self.loss_type == 'BPR':
            self.loss_fct = BPRLoss()
        elif self.loss_type == 'CE':
            self.loss_fct = nn.CrossEntropyLoss()
        elif self.loss_type == 'SSM':
            self.loss_fct = None
        else:
            raise NotImplementedError("Make sure 'loss_type' in ['BPR', 'CE', 'SSM']!")
        self.apply(self._init_weights)

    def _init_weights(self, module):
        if isinstance(module, (nn.Linear, nn.Embedding)):
            module.weight.data.normal_(mean=0.0, std=self.initializer_range)
        elif isinstance(module, nn.LayerNorm):
            module.bias.data.zero_()
            module.weight.data.fill_(1.0)
        if isinstance(module, nn.Linear) and module.bias is not None:
            module.bias.data.zero_()

    def get_attention_mask(self, item_seq):
        """Left-to-right mask, (1 - m) * -10000 (sasrec.py:91-105); on the GPU one launch
        (mirec_seq_attn_mask_f32, the same values bit for bit) instead of seven torch ops."""
        if (item_seq.is_cuda and item_seq.dtype == torch.int64 and item_seq.dim() == 2
                and self.item_embedding.weight.dtype == torch.float32):
            B, L = item_seq.shape
            mask = torch.empty(B, 1, L, L, dtype=torch.float32, device=item_seq.device)
            check(lib().mirec_seq_attn_mask_f32(ptr(item_seq.contiguous()), B, L, ptr(mask),
                                                stream_handle()), 'mirec_seq_attn_mask_f32')
            return mask
        attention_mask = (item_seq > 0).long()
        extended = attention_mask.unsqueeze(1).unsqueeze(2)
        max_len = attention_mask.size(-1)
        subsequent = torch.triu(torch.ones((1, max_len, max_len), device=item_seq.device),
                                diagonal=1)
        subsequent = (subsequent == 0).unsqueeze(1).long()
        extended = (extended * subsequent).to(dtype=self.item_embedding.weight.dtype)
        return (1.0 - extended) * -10000.0

    def forward(self, item_seq, item_seq_len):
        # the embedding dropout folds into K9a while training (p > 0); the module otherwise
        p = self.dropout.p if (self.dropout.training and 0 < self.dropout.p < 1) else 0.0
        rng = _drop_rng(self.dropout, item_seq.device) if p > 0 else None
        input_emb = _SeqEmbedLNFn.apply(self.item_embedding.weight,
                                        self.position_embedding.weight, self.LayerNorm.weight,
                                        self.LayerNorm.bias, item_seq, self.layer_norm_eps, p,
                                        rng)
        if p == 0:
            input_emb = self.dropout(input_emb)
        elif not input_emb.requires_grad:     # no backward to advance the draw counter
            rng[1].add_(1)
        mask = self.get_attention_mask(item_seq)
        out = self.trm_encoder(input_emb, mask, output_all_encoded_layers=True)[-1]
        return self.gather_indexes(out, item_seq_len - 1)

    def calculate_loss(self, interaction):
        item_seq = interaction[self.ITEM_SEQ]
        item_seq_len = interaction[self.ITEM_SEQ_LEN]
        seq_output = self.forward(item_seq, item_seq_len)
        pos_items = interaction[self.POS_ITEM_ID]
        W = self.item_embedding.weight
        if self.loss_type == 'BPR':
            return _SeqBPRFn.apply(seq_output, W, pos_items, interaction[self.NEG_ITEM_ID])
        if self.loss_type == 'SSM':
            return _SampledSoftmaxFn.apply(seq_output, W, pos_items,
                                           interaction[self.NEG_ITEM_ID])
        logits = torch.matmul(seq_output, W.transpose(0, 1))
        return self.loss_fct(logits, pos_items)

    def predict(self, interaction):
        seq_output = self.forward(interaction[self.ITEM_SEQ], interaction[self.ITEM_SEQ_LEN])
        return ops.dot_rows(seq_output.contiguous(), self.item_embedding.weight.detach(),
                            torch.arange(seq_output.shape[0], device=seq_output.device),
                            interaction[self.ITEM_ID])

    def full_sort_predict(self, interaction):
        self._sync_items()
        seq_output = self.forward(interaction[self.ITEM_SEQ], interaction[self.ITEM_SEQ_LEN])
        return ops.score_matrix(seq_output.detach().contiguous(),
                                self.item_embedding.weight.detach())

    def deferred_tables(self):
        """The item table on the deferred K5 schedule when every read of it is a
        row gather (BPR / SSM losses); CE reads the whole table every step."""
        return [] if self.loss_type == 'CE' else [self.item_embedding.weight]

    def _sync_items(self):
        h = getattr(self.item_embedding.weight, '_mirec_deferred', None)
        if h is not None:
            h.flush()

    # ------------------------------------------------------------------ fused eval hooks
    def fused_query_vectors(self, interaction):
        """Query vectors ranked by K6 (the sequence representations)."""
        return self.forward(interaction[self.ITEM_SEQ], interaction[self.ITEM_SEQ_LEN])

    def fused_item_table(self):
        self._sync_items()
        return self.item_embedding.weight.detach()
