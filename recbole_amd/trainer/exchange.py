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
