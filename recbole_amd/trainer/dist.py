"""Data parallelism for the generic (autograd) trainer path and the sharded full-sort
evaluation — SURVEY.md §8e for C3 (SASRec), C4 (DeepFM) and C5 (LightGCN eval).

Training: every rank draws the same GLOBAL batch (same seeds, same loader RNG), takes
its contiguous slice of the samples, and back-propagates its local mean loss scaled by
1/G (exact for power-of-two G), so the sum over ranks of every gradient equals the
gradient of the global-batch mean. The exchange per step is
  * one all-reduce (SUM) of a flat bucket of the dense gradients (MLP / transformer
    weights, dense tables) — RCCL over xGMI;
  * the deferred tables (DeepFM's token rows, SASRec's item rows) ROW-SHARDED by
    default (shard_tables; FusedAdam.shard_deferred): each contribution row goes to
    the owner of its table row (all-to-all, source-rank order = the global batch's
    contribution order) and only the owner updates it; forwards fetch the rows they
    read from their owners. With shard_tables: False, one all-gather per stashed
    source instead and every rank applies the identical deferred K5 step to its
    replica.
A ragged global batch (size not divisible by G) is computed whole on every rank: no
exchange (each owner keeps the contributions to its own rows).

Evaluation: the full-sort users are split into G contiguous blocks; rank g ranks its
block with K6 and one all-gather assembles the [n_users, K] positive flags in user
order, so the metrics are those of one GPU.
"""
from __future__ import annotations

import torch
import torch.distributed as tdist


def active_group(config=None):
    """The default process group when torch.distributed runs with > 1 rank
    (and config['n_gpus'] does not say 1), else None."""
    if not (tdist.is_available() and tdist.is_initialized()):
        return None
    if tdist.get_world_size() <= 1:
        return None
    if config is not None and config['n_gpus'] is not None and int(config['n_gpus']) == 1:
        return None
    return tdist.group.WORLD


def _gather_cat(t, group):
    """all-gather of equal-shaped tensors, concatenated along dim 0 in rank order."""
    G = tdist.get_world_size(group)
    t = t.contiguous()
    if str(tdist.get_backend(group)) == 'nccl':
        out = torch.empty((G * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        tdist.all_gather_into_tensor(out, t, group=group)
        return out
    parts = [torch.empty_like(t) for _ in range(G)]
    tdist.all_gather(parts, t, group=group)
    return torch.cat(parts)


def all_to_all_v(send, send_counts, group):
    """Variable-size all-to-all along dim 0: send[...] holds send_counts[g] rows for
    rank g, in rank order; returns (the rows received, in source-rank order, and
    the per-source counts). RCCL directly; gloo (CPU tests) host-staged."""
    nccl = str(tdist.get_backend(group)) == 'nccl'
    dev = send.device
    sc = send_counts.to(torch.int64)
    sc = sc.to(dev) if nccl else sc.cpu()
    rc = torch.empty_like(sc)
    tdist.all_to_all_single(rc, sc, group=group)
    sl, rl = sc.tolist(), rc.tolist()
    shape = tuple(send.shape[1:])
    if nccl:
        recv = torch.empty((sum(rl),) + shape, dtype=send.dtype, device=dev)
        tdist.all_to_all_single(recv, send.contiguous(), output_split_sizes=rl,
                                input_split_sizes=sl, group=group)
    else:
        recv = torch.empty((sum(rl),) + shape, dtype=send.dtype)
        tdist.all_to_all_single(recv, send.contiguous().cpu(), output_split_sizes=rl,
                                input_split_sizes=sl, group=group)
        recv = recv.to(dev)
    return recv, rc.to(dev)


class DataParallelStep(object):

    def __init__(self, group):
        self.group = group
        self.G = tdist.get_world_size(group)
        self.rank = tdist.get_rank(group)

    def local_slice(self, inter):
        """(rank's slice of the global batch, True) or (the whole batch, False) when
        the batch does not split evenly. Columns whose length is m x the batch
        length (the sampler's j*B + k layout of SSM negatives) are sliced per block."""
        from recbole_amd.data.interaction import Interaction
        # samples = the shortest column (SSM batches carry N*B negatives)
        n = min(t.shape[0] for t in inter.interaction.values())
        if n % self.G != 0 or n == 0:
            return inter, False
        b = n // self.G
        s, e = self.rank * b, (self.rank + 1) * b
        cols = {}
        for k, t in inter.interaction.items():
            if t.shape[0] == n:
                cols[k] = t[s:e]
            elif t.shape[0] % n == 0:
                m = t.shape[0] // n
                cols[k] = t.view((m, n) + tuple(t.shape[1:]))[:, s:e].reshape(
                    (m * b,) + tuple(t.shape[1:]))
            else:
                raise ValueError(f'column {k} of length {t.shape[0]} does not follow the '
                                 f'batch of {n}')
        return Interaction(cols), True

    def loss_scale(self):
        return 1.0 / self.G

    def exchange(self, model, optimizer):
        """Sum the dense gradients over ranks (one bucket) and gather the deferred
        tables' stashed contribution rows."""
        params = [p for p in model.parameters() if p.grad is not None]
        if params:
            flat = torch.cat([p.grad.reshape(-1) for p in params])
            tdist.all_reduce(flat, op=tdist.ReduceOp.SUM, group=self.group)
            o = 0
            for p in params:
                n = p.grad.numel()
                p.grad.copy_(flat[o:o + n].view_as(p.grad))
                o += n
        for p, ds in getattr(optimizer, '_deferred', {}).items():
            if 'shard' in ds:
                # row-sharded: every contribution row to the owner of its row, in
                # source-rank order (= the global batch's order); local row ids
                G = ds['shard']['G']
                out = []
                for rows, keys, _ in ds['stash']:
                    owner = keys % G
                    order = torch.argsort(owner, stable=True)
                    counts = torch.bincount(owner, minlength=G)
                    rr, _ = all_to_all_v(rows[order], counts, self.group)
                    kk, _ = all_to_all_v(keys[order], counts, self.group)
                    out.append((rr, kk // G, 'owned'))
                ds['stash'] = out
                continue
            ds['stash'] = [(_gather_cat(rows, self.group), _gather_cat(keys, self.group), None)
                           for rows, keys, _ in ds['stash']]

    def global_loss(self, loss):
        """Mean over ranks of the local mean losses (the global-batch mean)."""
        t = loss.detach().reshape(1).clone()
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=self.group)
        return t / self.G

    # ------------------------------------------------------------------ evaluation
    def user_block(self, n):
        """Rank's contiguous block [s, e) of n users (blocks of ceil(n / G))."""
        b = -(-n // self.G)
        s = min(n, self.rank * b)
        return s, min(n, s + b), b

    def gather_rows(self, local, n, b):
        """Rows of every rank's block (padded to b rows) -> [n, ...] in user order."""
        pad = torch.zeros((b,) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        pad[:local.shape[0]] = local
        return _gather_cat(pad, self.group)[:n]
