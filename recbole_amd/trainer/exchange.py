"""Layout of the per-step exchange of the data-parallel fused step.

One optimizer step over G ranks processes a GLOBAL batch of G*B positives: global
positive k = g*B + k' is rank g's local positive k'. The reference's pairwise layout of
the global batch (general_dataloader.py:235-241) numbers contribution rows
  users: k                 items: r = j*G*B + k   (j = 0: positive, j >= 1: negative j)
BPR's backward needs, per row r, only one scalar besides the embedding rows
themselves: coef_r = d loss / d (pos_score - neg_score). Every rank holds the full
tables (replicas kept identical by the replicated Adam), so the rows of the whole
global batch are on every rank already. Rank g runs K3's forward on its slice
(`mirec_bpr_fwd_coef_f32`) and writes into its block of a small exchange buffer
[G, W] floats (W = (1+T)*B):
  [0, B)              the B per-positive losses of its local positives k'
  [B, B + T*B)        coef of its local rows, local pairwise order j*B + k'
One all-gather (G*W*4 bytes: 10 KB per rank at C2, instead of the 1.6 MB of gradient
rows) makes the buffer identical on every rank; then every rank rebuilds the gradient
rows of the GLOBAL batch (`mirec_bpr_contrib_f32`, the same per-row arithmetic as K3)
in the single-GPU layout and applies the same K5 — bit for bit the update of one GPU
running the global batch.
"""
from __future__ import annotations

import torch


class ExchangeLayout(object):

    def __init__(self, G: int, B: int, T: int, d: int):
        self.G, self.B, self.T, self.d = G, B, T, d
        self.coef0 = B                          # first coefficient of a rank's block
        self.W = (1 + T) * B                    # floats per rank

    # ---------------------------------------------------------------- key slicing
    def local_users(self, users_g: torch.Tensor, g: int) -> torch.Tensor:
        """[nb, G*B] global batch users -> rank g's [nb, B] (a view)."""
        nb = users_g.numel() // (self.G * self.B)
        return users_g.view(nb, self.G, self.B)[:, g, :]

    def local_items(self, items_g: torch.Tensor, g: int) -> torch.Tensor:
        """[nb, (1+T)*G*B] global pairwise item keys -> rank g's [nb, 1+T, B] (a view)."""
        nb = items_g.numel() // ((1 + self.T) * self.G * self.B)
        return items_g.view(nb, 1 + self.T, self.G, self.B)[:, :, g, :]

    # ---------------------------------------------------------------- gathered buffer
    def gathered_losses(self, buf: torch.Tensor) -> torch.Tensor:
        """[G, W] exchange buffer -> the G*B losses in global positive order (a view)."""
        return buf.view(self.G, self.W)[:, :self.B]

    def coef_global(self, buf: torch.Tensor) -> torch.Tensor:
        """[G, W] exchange buffer -> coefficients of the global batch in its pairwise
        order j*G*B + g*B + k' (a copy; the kernels index the rank blocks directly)."""
        c = buf.view(self.G, self.W)[:, self.coef0:].reshape(self.G, self.T, self.B)
        return c.permute(1, 0, 2).reshape(-1)


class ShardLayout(object):
    """Specification (torch, any device) of the row-sharded exchange plans that
    csrc/shard.hip computes on the device (include/mirec.h, "Row-sharded tables"):
    cyclic ownership (row id on rank id % G, local row id // G), owner-major K2 keys,
    per-(slice, owner) messages of `cap` rows in ascending global slot order.
    Used by the tests to pin the kernels bit for bit and to run the protocol on
    gloo CPU ranks."""

    def __init__(self, G: int, B: int, T: int, nU: int, nI: int, cap: int):
        self.G, self.B, self.T, self.cap = G, B, T, cap
        self.SU, self.SI = -(-nU // G), -(-nI // G)

    def keys(self, ids: torch.Tensor, S: int) -> torch.Tensor:
        return (ids % self.G) * S + ids // self.G

    def slots(self, users: torch.Tensor, items: torch.Tensor):
        """Global slots of one batch: (t, row id, is_user, slice, local slot index in
        its slice) — users t = k, items t = Bc + j*Bc + k."""
        Bc, T, B = users.numel(), self.T, self.B
        k = torch.arange(Bc)
        j = torch.arange(1 + T).repeat_interleave(Bc)
        kk = torch.arange(Bc).repeat(1 + T)
        t = torch.cat([k, Bc + j * Bc + kk])
        ids = torch.cat([users.cpu(), items.cpu()])
        is_user = torch.cat([torch.ones(Bc, dtype=torch.bool), torch.zeros((1 + T) * Bc,
                                                                          dtype=torch.bool)])
        kall = torch.cat([k, kk])
        g = kall // B
        n_g = torch.clamp(Bc - g * B, 0, B)
        jall = torch.cat([torch.zeros(Bc, dtype=torch.long), j])
        ls = torch.where(is_user, kall - g * B, n_g + jall * n_g + (kall - g * B))
        return t, ids, is_user, g, ls

    def plan(self, users: torch.Tensor, items: torch.Tensor, rank: int):
        """(fwd_rows [G*cap], map2 [Bc + (1+T)Bc] (-1 where not owned), pos
        [(2+T)*B] (-1 beyond the slice), bwd_src [G*cap], overflow) of one batch."""
        G, cap, T, B = self.G, self.cap, self.T, self.B
        t, ids, is_user, g, ls = self.slots(users, items)
        o = ids % G
        order = torch.argsort(t)
        t, ids, is_user, g, ls, o = (x[order] for x in (t, ids, is_user, g, ls, o))
        idx = torch.zeros_like(t)
        cnt = {}
        for q in range(len(t)):                     # ascending t within each (g, o)
            key = (int(g[q]), int(o[q]))
            idx[q] = cnt.get(key, 0)
            cnt[key] = idx[q] + 1
        over = bool((idx >= cap).any())
        fwd = torch.zeros(G * cap, dtype=torch.int64)
        bwd = torch.zeros(G * cap, dtype=torch.int32)
        Bc = users.numel()
        map2 = torch.full((Bc + (1 + T) * Bc,), -1, dtype=torch.int32)
        pos = torch.full(((2 + T) * B,), -1, dtype=torch.int64)
        ok = idx < cap
        local = ids // G
        mine = ok & (o == rank)
        fwd[(g * cap + idx)[mine]] = torch.where(is_user, local, -(local + 1))[mine]
        map2[t[mine]] = (g * cap + idx)[mine].to(torch.int32)
        req = ok & (g == rank)
        pos[ls[req]] = (o * cap + idx)[req]
        bwd[(o * cap + idx)[req]] = ls[req].to(torch.int32)
        return fwd, map2, pos, bwd, over

    def largest_message(self, users: torch.Tensor, items: torch.Tensor) -> int:
        """Rows of the largest (slice, owner) message of one batch (plan status[1])."""
        _, ids, _, g, _ = self.slots(users, items)
        msg = g * self.G + ids % self.G
        return int(torch.bincount(msg).max())

    def own(self, uniq: torch.Tensor, seg: torch.Tensor, perm: torch.Tensor,
            map2: torch.Tensor, map_off: int, S: int, rank: int):
        """Rank `rank`'s slice of one batch's sorted keyed uniq list: (local rows,
        segment offsets, {p: perm2[p]} for the positions of those segments)."""
        lo = int(torch.searchsorted(uniq, torch.tensor(rank * S, dtype=uniq.dtype)))
        hi = int(torch.searchsorted(uniq, torch.tensor((rank + 1) * S, dtype=uniq.dtype)))
        own = uniq[lo:hi] - rank * S
        oseg = seg[lo:hi + 1]
        p = torch.arange(int(seg[lo]), int(seg[hi]))
        return own, oseg, p, map2[map_off + perm[p]]
