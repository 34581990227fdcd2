"""Layout of the per-step gradient exchange of the data-parallel fused step.

One optimizer step over G ranks processes a GLOBAL batch of G*B positives: global
positive k = g*B + k' is rank g's local positive k'. The reference's pairwise layout of
the global batch (general_dataloader.py:235-241) numbers contribution rows
  users: k                 items: r = j*G*B + k   (j = 0: positive, j >= 1: negative j)
Rank g runs K3 on its local slice and writes its contribution rows into its slice of a
packed exchange buffer [G, R, d] (R = B + (1+T)*B + loss rows):
  rows [0, B)            user gradient rows of local positives k'
  rows [B, B + (1+T)B)   item gradient rows, local pairwise order j*B + k'
  rows [B + (1+T)B, R)   the B per-positive losses (flat floats)
One all-gather makes the whole buffer identical on every rank. The K2 grouping of the
GLOBAL batch keys (computed on every rank) refers to global contribution numbers; the
maps below turn them into packed rows, so every rank's Adam sums each row's
contributions in the global order — the same sums, bit for bit, as one GPU running the
global batch.
"""
from __future__ import annotations

import math

import torch


class ExchangeLayout(object):

    def __init__(self, G: int, B: int, T: int, d: int):
        self.G, self.B, self.T, self.d = G, B, T, d
        self.loss_rows = math.ceil(B / d)
        self.item0 = B                          # first item row of a rank's slice
        self.loss0 = B + (1 + T) * B            # first loss row
        self.R = self.loss0 + self.loss_rows    # rows per rank

    # ---------------------------------------------------------------- key slicing
    def local_users(self, users_g: torch.Tensor, g: int) -> torch.Tensor:
        """[nb, G*B] global batch users -> rank g's [nb, B] (a view)."""
        nb = users_g.numel() // (self.G * self.B)
        return users_g.view(nb, self.G, self.B)[:, g, :]

    def local_items(self, items_g: torch.Tensor, g: int) -> torch.Tensor:
        """[nb, (1+T)*G*B] global pairwise item keys -> rank g's [nb, 1+T, B] (a view)."""
        nb = items_g.numel() // ((1 + self.T) * self.G * self.B)
        return items_g.view(nb, 1 + self.T, self.G, self.B)[:, :, g, :]

    # ---------------------------------------------------------------- perm remaps
    def user_rows(self, perm: torch.Tensor) -> torch.Tensor:
        """Global user contribution numbers k -> packed rows g*R + k'."""
        g = torch.div(perm, self.B, rounding_mode='floor')
        return g * self.R + (perm - g * self.B)

    def item_rows(self, perm: torch.Tensor) -> torch.Tensor:
        """Global item contribution numbers j*G*B + k -> packed rows g*R + B + j*B + k'."""
        Bg = self.G * self.B
        j = torch.div(perm, Bg, rounding_mode='floor')
        k = perm - j * Bg
        g = torch.div(k, self.B, rounding_mode='floor')
        return g * self.R + self.item0 + j * self.B + (k - g * self.B)

    def gathered_losses(self, xbuf: torch.Tensor) -> torch.Tensor:
        """[G, R, d] exchange buffer -> the G*B losses in global positive order (a view)."""
        flat = xbuf.view(self.G, self.R * self.d)
        o = self.loss0 * self.d
        return flat[:, o:o + self.B]
