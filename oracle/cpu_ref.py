"""oracle/cpu_ref.py — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference (ghazalehnt/RecBole @ v0.2.1 fork) hot path,
written from reading its source. Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module, and only as the checker
or the timed CPU baseline — never as the thing measured or shipped. The
product (recbole_amd/*) never imports it.

The reference itself may not be executed in this environment (SURVEY.md §8c:
a recorded denial), so parity is anchored as follows:
  * metric formulas  — pinned by the reference's known-answer tests
    (tests/metrics/test_topk_metrics.py:15-79, test_loss_metrics.py:10-52),
    transcribed as fixtures in tests/golden/;
  * full-sort masks / swap layout / batch order / split / remap — pinned by the
    reference's dataloader & dataset tests (tests/data/test_dataloader.py,
    test_dataset.py) and their atomic-file fixtures, copied as data;
  * sampled negative VALUES, BPR loss/gradients, Adam numerics — the reference
    tests pin none of these (only id ranges); they follow the algorithm as
    written (cited per function) and the PyTorch-CPU ops the reference calls.
    These are marked "parity pinned by restatement only" in DESIGN.md.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


# --------------------------------------------------------------------------
# Sampler  (recbole/sampler/sampler.py)
# --------------------------------------------------------------------------
def random_list_uniform(n_items: int, seed: int | None = None) -> np.ndarray:
    """Sampler.get_random_list('uniform') + set_distribution's shuffle
    (sampler.py:45-57, 191-197): np.arange(1, n_items) shuffled by the GLOBAL
    numpy RNG (the first draw after init_seed's np.random.seed, utils.py:183)."""
    if seed is not None:
        np.random.seed(seed)
    rl = np.arange(1, n_items)
    np.random.shuffle(rl)
    return rl


def random_list_popularity(item_columns: list[np.ndarray], seed: int | None = None):
    """Sampler.get_random_list('popularity') (sampler.py:198-202): concatenation
    of the item column of every phase dataset, shuffled once."""
    if seed is not None:
        np.random.seed(seed)
    rl = []
    for col in item_columns:
        rl.extend(np.asarray(col).tolist())
    rl = np.array(rl, dtype=np.int64) if len(rl) else np.zeros(0, dtype=np.int64)
    np.random.shuffle(rl)
    return rl


class NumpyWalk:
    """Line-by-line restatement of AbstractSampler.random_num + sample_by_key_ids
    (sampler.py:82-154) with Python sets as used_ids. Small cases only."""

    def __init__(self, random_list, used_ids):
        self.random_list = np.asarray(random_list)
        self.random_list_length = len(self.random_list)
        self.random_pr = 0
        self.used_ids = used_ids  # array-like of sets, indexed by key

    def random_num(self, num):  # sampler.py:82-101
        value_id = []
        self.random_pr %= self.random_list_length
        while True:
            if self.random_pr + num <= self.random_list_length:
                value_id.append(self.random_list[self.random_pr:self.random_pr + num])
                self.random_pr += num
                break
            else:
                value_id.append(self.random_list[self.random_pr:])
                num -= self.random_list_length - self.random_pr
                self.random_pr = 0
        return np.concatenate(value_id)

    def sample_by_key_ids(self, key_ids, num):  # sampler.py:103-154
        key_ids = np.array(key_ids)
        key_num = len(key_ids)
        total_num = key_num * num
        if (key_ids == key_ids[0]).all():
            key_id = key_ids[0]
            used = np.array(list(self.used_ids[key_id]))
            value_ids = self.random_num(total_num)
            check_list = np.arange(total_num)[np.isin(value_ids, used)]
            while len(check_list) > 0:
                value_ids[check_list] = value = self.random_num(len(check_list))
                perm = value.argsort(kind='quicksort')
                aux = value[perm]
                mask = np.empty(aux.shape, dtype=np.bool_)
                mask[:1] = True
                mask[1:] = aux[1:] != aux[:-1]
                value = aux[mask]
                rev_idx = np.empty(mask.shape, dtype=np.intp)
                rev_idx[perm] = np.cumsum(mask) - 1
                ar = np.concatenate((value, used))
                order = ar.argsort(kind='mergesort')
                sar = ar[order]
                bool_ar = (sar[1:] == sar[:-1])
                flag = np.concatenate((bool_ar, [False]))
                ret = np.empty(ar.shape, dtype=bool)
                ret[order] = flag
                mask = ret[rev_idx]
                check_list = check_list[mask]
        else:
            value_ids = np.zeros(total_num, dtype=np.int64)
            check_list = np.arange(total_num)
            key_ids = np.tile(key_ids, num)
            while len(check_list) > 0:
                value_ids[check_list] = self.random_num(len(check_list))
                check_list = np.array([
                    i for i, used, v in zip(check_list, [self.used_ids[k] for k in
                                                         key_ids[check_list]],
                                            value_ids[check_list]) if v in used
                ], dtype=np.int64)
        return value_ids.astype(np.int64)


def used_csr(n_keys: int, keys: np.ndarray, values: np.ndarray):
    """CSR (row_ptr int64[n_keys+1], cols int32 sorted unique per row) of the
    used sets Sampler.get_used_ids builds with Python sets (sampler.py:206-227)."""
    keys = np.asarray(keys, dtype=np.int64)
    values = np.asarray(values, dtype=np.int64)
    order = np.lexsort((values, keys))
    k = keys[order]
    v = values[order]
    if len(k):
        keep = np.ones(len(k), dtype=bool)
        keep[1:] = (k[1:] != k[:-1]) | (v[1:] != v[:-1])
        k, v = k[keep], v[keep]
    ptr = np.zeros(n_keys + 1, dtype=np.int64)
    np.add.at(ptr, k + 1, 1)
    ptr = np.cumsum(ptr)
    return ptr, v.astype(np.int32)


def _oracle_lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        _LIB = ctypes.CDLL(path)
        _LIB.oracle_sample_walk.restype = ctypes.c_int
    return _LIB


def c_sample_walk(random_list, pr: int, keys, num: int, used_ptr, used_cols, key_space: int,
                  reject: bool):
    """C restatement (oracle/walk.c) of the same walk: returns (values, new_pr)."""
    rl = np.ascontiguousarray(random_list, dtype=np.int32)
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    K = len(keys)
    out = np.zeros(K * num, dtype=np.int64)
    pr_io = ctypes.c_int64(pr)
    up = np.ascontiguousarray(used_ptr if used_ptr is not None else np.zeros(1), dtype=np.int64)
    uc = np.ascontiguousarray(used_cols if used_cols is not None else np.zeros(1),
                              dtype=np.int32)
    P = ctypes.c_void_p
    rc = _oracle_lib().oracle_sample_walk(
        rl.ctypes.data_as(P), ctypes.c_int64(len(rl)), ctypes.byref(pr_io),
        keys.ctypes.data_as(P), ctypes.c_int64(K), ctypes.c_int64(num), up.ctypes.data_as(P),
        uc.ctypes.data_as(P), ctypes.c_int64(key_space), ctypes.c_int(1 if reject else 0),
        out.ctypes.data_as(P))
    if rc == -3:
        raise RuntimeError("sampler livelock: rejection rounds exceeded 4L+1024")
    if rc != 0:
        raise ValueError("user_id out of range")
    return out, pr_io.value


# --------------------------------------------------------------------------
# Dataset pipeline  (recbole/data/dataset/dataset.py, data/utils.py:59-112)
# --------------------------------------------------------------------------
def read_atomic_tokens(path, field):
    """The token column `field` of an atomic file as strings, file order
    (dataset.py:342-408: header `name:type`, tab separated)."""
    with open(path, encoding='utf-8') as f:
        header = f.readline().rstrip('\n').split('\t')
        col = [h.split(':')[0] for h in header].index(field)
        return [line.rstrip('\n').split('\t')[col] for line in f if line.strip()]


def factorize(tokens):
    """pd.factorize order (dataset.py:908-928): ids 1.. by first appearance, 0 = [PAD]."""
    tok = np.asarray(tokens)
    uniq, first, inv = np.unique(tok, return_index=True, return_inverse=True)
    rank = np.empty(len(uniq), dtype=np.int64)
    rank[np.argsort(first, kind='stable')] = np.arange(len(uniq))
    return rank[inv] + 1, len(uniq) + 1


def load_ml100k(data_dir):
    """ml-100k as the reference's Dataset builds it for BPR
    (properties/dataset/ml-100k.yaml): .inter + the item file's item_id;
    filter_inter_by_user_or_item drops interactions whose item is not in the item
    file (dataset.py:_filter_inter_by_user_or_item); no user file is loaded; then
    remap (dataset.py:844-928): users over the inter column, items over
    [inter column, item-file column] concatenated. Returns
    (user ids, item ids, n_users, n_items), file order."""
    inter = os.path.join(data_dir, 'ml-100k.inter')
    u_tok = read_atomic_tokens(inter, 'user_id')
    i_tok = read_atomic_tokens(inter, 'item_id')
    item_tok = read_atomic_tokens(os.path.join(data_dir, 'ml-100k.item'), 'item_id')
    known = set(item_tok)
    keep = [k for k, t in enumerate(i_tok) if t in known]
    u_tok = [u_tok[k] for k in keep]
    i_tok = [i_tok[k] for k in keep]
    users, n_users = factorize(u_tok)
    items_all, n_items = factorize(i_tok + item_tok)
    return users, items_all[:len(i_tok)], n_users, n_items


def calcu_split_ids(tot, ratios):
    """Dataset._calcu_split_ids (dataset.py:1258-1279): all parts but the first
    rounded down, a non-empty part of < 1 row bumped to 1 while the first part has
    more than one row."""
    cnt = [int(r * tot) for r in ratios]
    cnt[0] = tot - sum(cnt[1:])
    for k in range(1, len(ratios)):
        if cnt[0] <= 1:
            break
        if 0 < ratios[-k] * tot < 1:
            cnt[-k] += 1
            cnt[0] -= 1
    return np.cumsum(cnt)[:-1]


def ro_rs_split(users, ratios=(0.8, 0.1, 0.1)):
    """Dataset.build for eval_setting RO_RS (dataset.py:1377-1413): one
    torch.randperm over all rows (Interaction.shuffle, interaction.py:272-276; the
    FIRST torch CPU draw after init_seed), then split_by_ratio grouped by user
    (dataset.py:1281-1315): groups in first-appearance order of the shuffled table,
    each group's rows in table order cut by calcu_split_ids. Returns the row index
    (into the UNshuffled arrays) of each part, in part order."""
    users = np.asarray(users)
    n = len(users)
    perm = torch.randperm(n).numpy()
    ku = users[perm]
    tot_r = sum(ratios)
    ratios = [r / tot_r for r in ratios]
    order = np.argsort(ku, kind='stable')                 # rows of each user in table order
    su = ku[order]
    starts = np.flatnonzero(np.r_[True, su[1:] != su[:-1]]) if n else np.zeros(0, np.int64)
    sizes = np.diff(np.r_[starts, n])
    rank = np.arange(n) - np.repeat(starts, sizes)         # position within its user group
    first = order[starts]                                  # first table row of each group
    group_pos = np.empty(len(starts), dtype=np.int64)
    group_pos[np.argsort(first, kind='stable')] = np.arange(len(starts))
    cuts = {t: calcu_split_ids(t, ratios) for t in np.unique(sizes)}
    cut = np.stack([cuts[t] for t in sizes]) if len(sizes) else np.zeros((0, len(ratios) - 1))
    part = (rank[:, None] >= np.repeat(cut, sizes, axis=0)).sum(1)
    gp = np.repeat(group_pos, sizes)
    out = []
    for k in range(len(ratios)):
        sel = np.flatnonzero(part == k)
        sel = sel[np.lexsort((rank[sel], gp[sel]))]        # group order, then table order
        out.append(perm[order[sel]])
    return out


def bpr_replay(model, train_users, train_items, random_list, used_ptr, used_cols, n_users,
               B, T, n_steps, lr=1e-3, on_step=None):
    """Trainer.fit's epochs for BPR with a uniform Sampler, from the current torch /
    numpy RNG state: per epoch one torch.randperm of the train table
    (GeneralNegSampleDataLoader._shuffle -> Interaction.shuffle), batches of B
    positives (general_dataloader.py:194-197), the walk + rejection
    (sampler.py:103-154, C restatement) continuing across batches and epochs,
    pairwise rows (:235-241), BPR + BPRLoss + optim.Adam on torch CPU
    (trainer.py:157-174). Stops after n_steps optimizer steps. Returns (per-step
    losses, per-step negatives, final walk pointer)."""
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    users = torch.as_tensor(np.asarray(train_users, dtype=np.int64))
    items = torch.as_tensor(np.asarray(train_items, dtype=np.int64))
    pr, losses, negs, done = 0, [], [], 0
    while done < n_steps:
        perm = torch.randperm(len(users))              # in place: epochs compose
        users, items = users[perm], items[perm]
        for s in range(0, len(users), B):
            if done == n_steps:
                break
            ub, ib = users[s:s + B], items[s:s + B]
            neg, pr = c_sample_walk(random_list, pr, ub.numpy(), T, used_ptr, used_cols,
                                    n_users, True)
            ur, pr_, nr = pairwise_rows(ub, ib, torch.as_tensor(neg), T)
            opt.zero_grad()
            loss = model.calculate_loss(ur, pr_, nr)
            losses.append(loss.item())
            loss.backward()
            opt.step()
            negs.append(neg)
            done += 1
            if on_step is not None:
                on_step(done, model)
    return losses, negs, pr


# --------------------------------------------------------------------------
# BPR model + loss + Adam step, torch CPU fp32 (the reference's own ops)
# --------------------------------------------------------------------------
class BPRCPU(torch.nn.Module):
    """BPR (recbole/model/general_recommender/bpr.py:27-96) with BPRLoss
    (loss.py:23-49) and xavier_normal_ init (init.py:15-31), torch CPU."""

    def __init__(self, n_users, n_items, d, init=True):
        super().__init__()
        self.user_embedding = torch.nn.Embedding(n_users, d)
        self.item_embedding = torch.nn.Embedding(n_items, d)
        if init:
            torch.nn.init.xavier_normal_(self.user_embedding.weight.data)
            torch.nn.init.xavier_normal_(self.item_embedding.weight.data)

    def calculate_loss(self, user, pos, neg, gamma=1e-10):
        u = self.user_embedding(user)
        p = self.item_embedding(pos)
        n = self.item_embedding(neg)
        ps = torch.mul(u, p).sum(dim=1)
        ns = torch.mul(u, n).sum(dim=1)
        return -torch.log(gamma + torch.sigmoid(ps - ns)).mean()

    def full_sort_predict(self, user):
        return torch.matmul(self.user_embedding(user),
                            self.item_embedding.weight.transpose(0, 1)).view(-1)


def pairwise_rows(user_b, pos_b, neg_flat, times):
    """GeneralNegSampleDataLoader._neg_sample_by_pair_wise_sampling layout
    (general_dataloader.py:235-241; Interaction.repeat interaction.py:189-217):
    row r = j*B + k -> (user[k], pos[k], neg[r])."""
    user_r = user_b.repeat(times)
    pos_r = pos_b.repeat(times)
    return user_r, pos_r, neg_flat


def bpr_train_steps(model: BPRCPU, batches, lr=1e-3, weight_decay=0.0):
    """Trainer._train_epoch inner loop (trainer.py:157-174) with optim.Adam
    (trainer.py:115-116). Returns the per-step losses."""
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)
    losses = []
    for user, pos, neg in batches:
        opt.zero_grad()
        loss = model.calculate_loss(user, pos, neg)
        losses.append(loss.item())
        loss.backward()
        opt.step()
    return losses, opt


def general_sampled_eval(user_emb, item_emb, uid_list, uid2start, uid2items_num, items_by_user,
                         step, random_list, pr, used_ptr, used_cols, n_users, N, K, full=True):
    """Trainer.evaluate over a GeneralNegSampleDataLoader in evaluation for BPR
    (point-wise uni-N, whole users per batch), as written:
      per batch of `step` users (general_dataloader.py:210-221): per user, its rows
      (dataset sorted by user), sample_by_user_ids([u]*n_u, N) (the walk + rejection,
      C restatement), rows repeated 1+N times with the negatives after the positives
      (_neg_sample_by_point_wise_sampling :243-251); users concatenated;
      BPR.predict = sum(u * i) (bpr.py:85-89) on torch CPU;
      TopKEvaluator.collect (evaluators.py:53-76): get_score_matrix —
      full_sort_collect's view(n_users_in_batch, -1) when 'full' is in
      eval_setting (abstract_evaluator.py:77-95; this fork's uni1000 validation
      keeps 'full'), else sample_collect's -inf padding — then flip + topk(K);
      TopKEvaluator.evaluate: pos_idx = topk_idx >= shape - pos_len.
    Returns (per-batch list of (items, scores, score matrix after flip, topk idx),
    pos_idx [n_users, K], final walk pointer)."""
    batches = []
    pos_rows = []
    for b0 in range(0, len(uid_list), step):
        ul = uid_list[b0:b0 + step]
        users, items, lens = [], [], []
        for u in ul:
            n = int(uid2items_num[u])
            s0 = int(uid2start[u])
            pos = np.asarray(items_by_user[s0:s0 + n], dtype=np.int64)
            neg, pr = c_sample_walk(random_list, pr, np.full(n, u, dtype=np.int64), N,
                                    used_ptr, used_cols, n_users, True)
            items.append(np.concatenate([pos, neg]))
            users.append(np.full(n * (1 + N), u, dtype=np.int64))
            lens.append(n * (1 + N))
        it = torch.as_tensor(np.concatenate(items))
        us = torch.as_tensor(np.concatenate(users))
        scores = torch.mul(user_emb[us], item_emb[it]).sum(dim=1)
        if full:
            mat = scores.view(len(ul), -1)
        else:
            mat = torch.nn.utils.rnn.pad_sequence(torch.split(scores, lens), batch_first=True,
                                                  padding_value=-np.inf)
            if mat.shape[1] < K:
                m2 = torch.full((mat.shape[0], K), -np.inf)
                m2[:, :mat.shape[1]] = mat
                mat = m2
        mat = torch.flip(mat, dims=[-1])
        _, idx = torch.topk(mat, K, dim=-1)
        pos_len = np.asarray([uid2items_num[u] for u in ul])
        pos_rows.append(idx.numpy() >= (mat.shape[1] - pos_len).reshape(-1, 1))
        batches.append((it.numpy(), scores, mat, idx))
    pos_idx = np.concatenate(pos_rows) if pos_rows else np.zeros((0, K), dtype=bool)
    return batches, pos_idx, pr


# --------------------------------------------------------------------------
# LightGCN  (recbole/model/general_recommender/lightgcn.py:32-180)
# --------------------------------------------------------------------------
def lightgcn_norm_adj(inter_rows, inter_cols, n_users, n_items):
    """get_norm_adj_mat (lightgcn.py:71-104) with scipy + torch CPU. The
    reference fills a dok_matrix through the private dok._update (:89), which
    the container's scipy lacks; the same dict of (row, col) -> 1 is written
    here through a CSR with duplicates reset to 1. Then, as written:
    sumArr = (A > 0).sum(1); diag = sumArr + 1e-7; D^-1/2 * A * D^-1/2 (float64
    from the float64 diag), coo, torch.sparse FloatTensor."""
    import scipy.sparse as sp
    N = n_users + n_items
    r = np.asarray(inter_rows, dtype=np.int64)
    c = np.asarray(inter_cols, dtype=np.int64) + n_users
    rows = np.concatenate([r, c])
    cols = np.concatenate([c, r])
    A = sp.coo_matrix((np.ones(len(rows), dtype=np.float32), (rows, cols)), shape=(N, N)).tocsr()
    A.data[:] = 1.0
    sumArr = (A > 0).sum(axis=1)
    diag = np.array(sumArr.flatten())[0] + 1e-7
    diag = np.power(diag, -0.5)
    D = sp.diags(diag)
    L = sp.coo_matrix(D * A * D)
    i = torch.LongTensor(np.array([L.row, L.col]))
    return torch.sparse_coo_tensor(i, torch.FloatTensor(L.data), torch.Size(L.shape))


class LightGCNCPU(torch.nn.Module):
    """LightGCN forward / calculate_loss / full_sort_predict on torch CPU
    (lightgcn.py:106-180) with BPRLoss + EmbLoss (loss.py:23-84)."""

    def __init__(self, n_users, n_items, d, n_layers, reg_weight, norm_adj, init=True):
        super().__init__()
        self.n_users, self.n_items, self.n_layers = n_users, n_items, n_layers
        self.reg_weight = reg_weight
        self.user_embedding = torch.nn.Embedding(n_users, d)
        self.item_embedding = torch.nn.Embedding(n_items, d)
        self.norm_adj_matrix = norm_adj
        if init:
            torch.nn.init.xavier_uniform_(self.user_embedding.weight.data)
            torch.nn.init.xavier_uniform_(self.item_embedding.weight.data)

    def forward(self):
        all_e = torch.cat([self.user_embedding.weight, self.item_embedding.weight], dim=0)
        embs = [all_e]
        for _ in range(self.n_layers):
            all_e = torch.sparse.mm(self.norm_adj_matrix, all_e)
            embs.append(all_e)
        out = torch.mean(torch.stack(embs, dim=1), dim=1)
        return torch.split(out, [self.n_users, self.n_items])

    def calculate_loss(self, user, pos, neg, gamma=1e-10):
        ua, ia = self.forward()
        u, p, n = ua[user], ia[pos], ia[neg]
        ps = torch.mul(u, p).sum(dim=1)
        ns = torch.mul(u, n).sum(dim=1)
        mf = -torch.log(gamma + torch.sigmoid(ps - ns)).mean()
        emb = torch.zeros(1)
        for e in (self.user_embedding(user), self.item_embedding(pos), self.item_embedding(neg)):
            emb += torch.norm(e, p=2)
        emb /= neg.shape[0]
        return mf + self.reg_weight * emb

    def full_sort_predict(self, user):
        ua, ia = self.forward()
        return torch.matmul(ua[user], ia.transpose(0, 1)).view(-1)


# --------------------------------------------------------------------------
# DeepFM  (recbole/model/context_aware_recommender/deepfm.py:26-73 with
# ContextRecommender abstract_recommender.py:151-412, FMEmbedding /
# BaseFactorizationMachine / FMFirstOrderLinear / MLPLayers layers.py)
# --------------------------------------------------------------------------
class _FMEmb(torch.nn.Module):
    def __init__(self, n, d):
        super().__init__()
        self.embedding = torch.nn.Embedding(n, d)


class _FirstOrder(torch.nn.Module):
    def __init__(self, tok_dims, seq_dims, n_float):
        super().__init__()
        if tok_dims:
            self.token_embedding_table = _FMEmb(int(sum(tok_dims)), 1)
        if n_float:
            self.float_embedding_table = torch.nn.Embedding(n_float, 1)
        if seq_dims:
            self.token_seq_embedding_table = torch.nn.ModuleList(
                [torch.nn.Embedding(n, 1) for n in seq_dims])
        self.bias = torch.nn.Parameter(torch.zeros((1,)))


class DeepFMCPU(torch.nn.Module):
    """Same module tree (state_dict keys) as the reference DeepFM; forward as
    written there, on torch CPU. tok/seq/float = ordered field-name lists."""

    def __init__(self, tok, tok_dims, seq, seq_dims, flt, d, hidden, dropout):
        super().__init__()
        self.tok, self.seq, self.flt, self.d = tok, seq, flt, d
        self.offsets = np.array((0, *np.cumsum(tok_dims)[:-1]), dtype=np.int64) if tok else None
        if tok:
            self.token_embedding_table = _FMEmb(int(sum(tok_dims)), d)
        if flt:
            self.float_embedding_table = torch.nn.Embedding(len(flt), d)
        if seq:
            self.token_seq_embedding_table = torch.nn.ModuleList(
                [torch.nn.Embedding(n, d) for n in seq_dims])
        self.first_order_linear = _FirstOrder(tok_dims, seq_dims, len(flt))
        sizes = [d * (len(tok) + len(seq) + len(flt))] + list(hidden)
        mods = []
        for a, b in zip(sizes[:-1], sizes[1:]):
            mods += [torch.nn.Dropout(dropout), torch.nn.Linear(a, b), torch.nn.ReLU()]
        self.mlp_layers = torch.nn.Module()
        self.mlp_layers.mlp_layers = torch.nn.Sequential(*mods)
        self.deep_predict_layer = torch.nn.Linear(sizes[-1], 1)

    def _seq_mean(self, table, ids):
        mask = (ids != 0).float()
        cnt = torch.sum(mask, dim=1, keepdim=True)
        e = table(ids)
        s = torch.sum(e * mask.unsqueeze(2).expand_as(e), dim=1)
        return torch.div(s, cnt + torch.FloatTensor([1e-8])).unsqueeze(1)

    def forward(self, inter):
        parts = []
        if self.tok:
            ids = torch.cat([inter[n].unsqueeze(1) for n in self.tok], dim=1)
            parts.append(self.token_embedding_table.embedding(
                ids + ids.new_tensor(self.offsets).unsqueeze(0)))
        if self.seq:
            parts.append(torch.cat([self._seq_mean(t, inter[n]) for t, n in
                                    zip(self.token_seq_embedding_table, self.seq)], dim=1))
        xf = None
        if self.flt:
            xf = torch.cat([inter[n].float().unsqueeze(1) for n in self.flt], dim=1)
            idx = torch.arange(0, xf.shape[1]).unsqueeze(0).expand_as(xf).long()
            parts.append(torch.mul(self.float_embedding_table(idx), xf.unsqueeze(2)))
        allE = torch.cat(parts, dim=1)
        B = allE.shape[0]
        fo = self.first_order_linear
        tot = []
        if self.flt:
            idx = torch.arange(0, xf.shape[1]).unsqueeze(0).expand_as(xf).long()
            tot.append(torch.sum(torch.mul(fo.float_embedding_table(idx), xf.unsqueeze(2)),
                                 dim=1, keepdim=True))
        if self.tok:
            tot.append(torch.sum(fo.token_embedding_table.embedding(
                ids + ids.new_tensor(self.offsets).unsqueeze(0)), dim=1, keepdim=True))
        if self.seq:
            res = []
            for t, n in zip(fo.token_seq_embedding_table, self.seq):
                m = (inter[n] != 0).float()
                e = t(inter[n])
                res.append(torch.sum(e * m.unsqueeze(2).expand_as(e), dim=1, keepdim=True))
            tot.append(torch.sum(torch.cat(res, dim=1), dim=1, keepdim=True))
        first = torch.sum(torch.cat(tot, dim=1), dim=1) + fo.bias
        sq_sum = torch.sum(allE, dim=1) ** 2
        sum_sq = torch.sum(allE ** 2, dim=1)
        fm = 0.5 * torch.sum(sq_sum - sum_sq, dim=1, keepdim=True)
        y_deep = self.deep_predict_layer(self.mlp_layers.mlp_layers(allE.view(B, -1)))
        return torch.sigmoid(first + fm + y_deep).squeeze()

    def calculate_loss(self, inter, label):
        return torch.nn.BCELoss()(self.forward(inter), label)


# --------------------------------------------------------------------------
# Sequential data + SASRec  (recbole/data/dataset/sequential_dataset.py:43-112,
# data/dataloader/sequential_dataloader.py:95-127, model/sequential_recommender/
# sasrec.py:25-158, model/layers.py:338-552)
# --------------------------------------------------------------------------
def seq_augmentation(uids_sorted, max_len):
    """prepare_data_augmentation's loop as written (:72-85) over rows already
    sorted by (user, time): (uid_list, (start, stop) per sample, target_index)."""
    uid_list, index, target = [], [], []
    last_uid, seq_start = None, 0
    for i, uid in enumerate(uids_sorted):
        if last_uid != uid:
            last_uid = uid
            seq_start = i
        else:
            if i - seq_start > max_len:
                seq_start += 1
            uid_list.append(uid)
            index.append((seq_start, i))
            target.append(i)
    return uid_list, index, target


def leave_one_out_index(group_keys, leave_one_num):
    """dataset.py:1249-1256 (_grouped_index) + :1317-1337, as written."""
    groups = {}
    for i, k in enumerate(group_keys):
        groups.setdefault(k, []).append(i)
    nxt = [[] for _ in range(leave_one_num + 1)]
    for index in groups.values():
        tot = len(index)
        legal = min(leave_one_num, tot - 1)
        pr = tot - legal
        nxt[0].extend(index[:pr])
        for i in range(legal):
            nxt[-legal + i].append(index[pr])
            pr += 1
    return nxt


class _MHA(torch.nn.Module):
    def __init__(self, h, d, eps):
        super().__init__()
        self.h, self.hd = h, d // h
        self.query, self.key, self.value = (torch.nn.Linear(d, d), torch.nn.Linear(d, d),
                                            torch.nn.Linear(d, d))
        self.dense = torch.nn.Linear(d, d)
        self.LayerNorm = torch.nn.LayerNorm(d, eps=eps)

    def _t(self, x):
        return x.view(*(x.size()[:-1] + (self.h, self.hd))).permute(0, 2, 1, 3)

    def forward(self, x, mask):
        import math
        q, k, v = self._t(self.query(x)), self._t(self.key(x)), self._t(self.value(x))
        sc = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(self.hd) + mask
        p = torch.softmax(sc, dim=-1)
        c = torch.matmul(p, v).permute(0, 2, 1, 3).contiguous()
        c = c.view(*(c.size()[:-2] + (self.h * self.hd,)))
        return self.LayerNorm(self.dense(c) + x)


class _FF(torch.nn.Module):
    def __init__(self, d, inner, eps):
        super().__init__()
        self.dense_1, self.dense_2 = torch.nn.Linear(d, inner), torch.nn.Linear(inner, d)
        self.LayerNorm = torch.nn.LayerNorm(d, eps=eps)

    def forward(self, x):
        import math
        h = self.dense_1(x)
        h = h * 0.5 * (1.0 + torch.erf(h / math.sqrt(2.0)))
        return self.LayerNorm(self.dense_2(h) + x)


class _TL(torch.nn.Module):
    def __init__(self, h, d, inner, eps):
        super().__init__()
        self.multi_head_attention = _MHA(h, d, eps)
        self.feed_forward = _FF(d, inner, eps)


class SASRecCPU(torch.nn.Module):
    """SASRec with dropout 0 (the reference's module tree: state_dict keys match),
    forward / losses as written in sasrec.py:107-158 on torch CPU. loss 'SSM' is
    the build's sampled softmax: CE over logits [pos | negs] with target 0."""

    def __init__(self, n_items, L, d, n_layers, n_heads, inner, eps):
        super().__init__()
        self.item_embedding = torch.nn.Embedding(n_items, d, padding_idx=0)
        self.position_embedding = torch.nn.Embedding(L, d)
        self.trm_encoder = torch.nn.Module()
        self.trm_encoder.layer = torch.nn.ModuleList([_TL(n_heads, d, inner, eps)
                                                      for _ in range(n_layers)])
        self.LayerNorm = torch.nn.LayerNorm(d, eps=eps)

    def forward(self, item_seq, item_len):
        pos = torch.arange(item_seq.size(1)).unsqueeze(0).expand_as(item_seq)
        x = self.LayerNorm(self.item_embedding(item_seq) + self.position_embedding(pos))
        am = (item_seq > 0).long().unsqueeze(1).unsqueeze(2)
        n = item_seq.size(1)
        sub = (torch.triu(torch.ones((1, n, n)), diagonal=1) == 0).unsqueeze(1).long()
        mask = (1.0 - (am * sub).float()) * -10000.0
        for layer in self.trm_encoder.layer:
            x = layer.feed_forward(layer.multi_head_attention(x, mask))
        idx = (item_len - 1).view(-1, 1, 1).expand(-1, -1, x.shape[-1])
        return x.gather(dim=1, index=idx).squeeze(1)

    def calculate_loss(self, item_seq, item_len, pos, neg=None, loss_type='CE'):
        s = self.forward(item_seq, item_len)
        W = self.item_embedding.weight
        if loss_type == 'BPR':
            ps = torch.sum(s * self.item_embedding(pos), dim=-1)
            ns = torch.sum(s * self.item_embedding(neg), dim=-1)
            return -torch.log(1e-10 + torch.sigmoid(ps - ns)).mean()
        if loss_type == 'SSM':
            B = s.shape[0]
            items = torch.cat([pos.view(1, B), neg.view(-1, B)], dim=0).T     # [B, 1+N]
            logits = (s.unsqueeze(1) * self.item_embedding(items)).sum(-1)
            return torch.nn.functional.cross_entropy(logits, torch.zeros(B, dtype=torch.long))
        return torch.nn.functional.cross_entropy(torch.matmul(s, W.T), pos)


# --------------------------------------------------------------------------
# Full-sort evaluation (trainer.py:328-353, evaluators.py:53-141)
# --------------------------------------------------------------------------
def full_sort_pos_idx(scores: torch.Tensor, hist: list, pos: list, K: int):
    """scores [n_users, I] (already U @ E_I^T); hist/pos: per-user item lists.
    Applies the reference's mask + swap + flip + topk and returns
    (pos_idx bool [n,K], topk_item_ids [n,K]) where topk_item_ids maps the
    flipped/swapped columns back to item ids."""
    scores = scores.clone()
    n, I = scores.shape
    scores[:, 0] = -np.inf
    col_of = np.tile(np.arange(I), (n, 1))  # which item sits in each column
    for r in range(n):
        h = list(hist[r])
        if h:
            scores[r, h] = -np.inf
        positive = set(int(x) for x in pos[r])
        pl = len(positive)
        swap = sorted(set(range(pl)) ^ positive)  # general_dataloader.py:325
        after = torch.tensor(swap, dtype=torch.long)
        before = after.flip(0)
        scores[r, after] = scores[r, before].clone()
        col_of[r, after.numpy()] = col_of[r, before.numpy()].copy()
    flipped = torch.flip(scores, dims=[-1])
    _, topk_idx = torch.topk(flipped, K, dim=-1)
    topk_idx = topk_idx.numpy()
    pos_len = np.array([len(set(p)) for p in pos])
    pos_idx = topk_idx >= (I - pos_len).reshape(-1, 1)
    item_ids = np.take_along_axis(col_of[:, ::-1], topk_idx, axis=1)
    return pos_idx, item_ids


# --------------------------------------------------------------------------
# Metrics  (recbole/evaluator/metrics.py:27-165), float64 numpy
# --------------------------------------------------------------------------
def hit_(pos_index, pos_len):
    result = np.cumsum(pos_index, axis=1)
    return (result > 0).astype(int)


def mrr_(pos_index, pos_len):
    idxs = pos_index.argmax(axis=1)
    result = np.zeros_like(pos_index, dtype=np.float64)
    for row, idx in enumerate(idxs):
        if pos_index[row, idx] > 0:
            result[row, idx:] = 1 / (idx + 1)
        else:
            result[row, idx:] = 0
    return result


def precision_(pos_index, pos_len):
    return pos_index.cumsum(axis=1) / np.arange(1, pos_index.shape[1] + 1)


def map_(pos_index, pos_len):
    pre = precision_(pos_index, pos_len)
    sum_pre = np.cumsum(pre * pos_index.astype(np.float64), axis=1)
    len_rank = np.full_like(pos_len, pos_index.shape[1])
    actual_len = np.where(pos_len > len_rank, len_rank, pos_len)
    result = np.zeros_like(pos_index, dtype=np.float64)
    for row, lens in enumerate(actual_len):
        ranges = np.arange(1, pos_index.shape[1] + 1)
        ranges[lens:] = ranges[lens - 1]
        result[row] = sum_pre[row] / ranges
    return result


def recall_(pos_index, pos_len):
    return np.cumsum(pos_index, axis=1) / pos_len.reshape(-1, 1)


def ndcg_(pos_index, pos_len):
    len_rank = np.full_like(pos_len, pos_index.shape[1])
    idcg_len = np.where(pos_len > len_rank, len_rank, pos_len)
    iranks = np.zeros_like(pos_index, dtype=np.float64)
    iranks[:, :] = np.arange(1, pos_index.shape[1] + 1)
    idcg = np.cumsum(1.0 / np.log2(iranks + 1), axis=1)
    for row, idx in enumerate(idcg_len):
        idcg[row, idx:] = idcg[row, idx - 1]
    ranks = np.zeros_like(pos_index, dtype=np.float64)
    ranks[:, :] = np.arange(1, pos_index.shape[1] + 1)
    dcg = 1.0 / np.log2(ranks + 1)
    dcg = np.cumsum(np.where(pos_index, dcg, 0), axis=1)
    return dcg / idcg


METRICS = {"hit": hit_, "mrr": mrr_, "precision": precision_, "map": map_, "recall": recall_,
           "ndcg": ndcg_}


def topk_metrics(pos_idx, pos_len, metrics, topk, precision=4):
    """TopKEvaluator._calculate_metrics + evaluate (evaluators.py:78-141)."""
    res = {}
    for m in metrics:
        v = METRICS[m.lower()](pos_idx, pos_len).mean(axis=0)
        for k in topk:
            res[f"{m.lower()}@{k}"] = round(v[k - 1], precision)
    return res
