"""A captured training step for the generic (autograd) trainer path.

Trainer._train_epoch (reference trainer.py:157-174) runs, per batch,
zero_grad -> calculate_loss -> backward -> optimizer.step. With hand-written
kernels behind the model's autograd Functions, a step of DeepFM at C4 is about
130 small launches and the host's launch rate, not the GPU, set the step time
(GPU busy ~50 %). GraphedTrainStep captures the whole step once — forward,
backward and FusedAdam in graph mode (device step counter, one constant window
for every parameter, trainer/optim.py) — and replays it per batch: one host
launch per step plus ONE copy launch of the batch's columns into the captured input
tensors (mirec_copy_many; torch's _foreach_copy_ issued one copy kernel per column,
≈ 4.4 µs each, ≈ 170 µs per DeepFM step).

The replayed step runs exactly the kernels of the eager step on the same
operands, so parameters, optimizer state and losses are bit-identical to the
eager graph-mode step (tests/test_gpu_graph_step.py). Batches of another shape
(the ragged last batch) run eagerly. Per-batch losses stay on the device
(read once per epoch); the NaN check is per epoch, as on the fused BPR path.
"""
from __future__ import annotations

import torch

from recbole_amd import ops
from recbole_amd.data.interaction import Interaction


class GraphedTrainStep(object):

    def __init__(self, model, optimizer, loss_func=None, warmup=3, window=256):
        self.model, self.opt = model, optimizer
        self.loss_func = loss_func or model.calculate_loss
        self.dev = next(model.parameters()).device
        self.warmup = warmup
        optimizer.graph_mode(self.dev, window)
        self.graph = None
        self.static = None
        self.keys = None
        self.static_loss = None
        self.n_warm = 0
        self.n_graphed = 0
        self.side = torch.cuda.Stream(device=self.dev)
        from recbole_amd.model.context import unit_grad
        self.unit = unit_grad(self.dev)      # the backward seed, allocated before any capture

    def _backward(self, loss):
        # seeded with the persistent unit (no fill launch; the loss Functions skip the
        # multiply by the seed) — the same gradient as loss.backward()
        if loss.dim() == 0:
            loss.backward(self.unit)
        else:
            loss.backward()

    def _eager(self, inter):
        self.opt.zero_grad(set_to_none=True)
        loss = self.loss_func(inter)
        self._backward(loss)
        self.opt.step()
        return loss.detach()

    def _fits(self, inter):
        return (self.static is not None and set(inter.interaction) == set(self.keys) and
                all(inter[k].shape == self.static[k].shape and inter[k].dtype == self.static[k].dtype
                    for k in self.keys))

    def step(self, inter):
        """One optimizer step on `inter` (device tensors); returns the device loss."""
        self.opt.graph_window()
        if self.static is None:
            self.keys = sorted(inter.interaction)
            self.static = Interaction({k: inter[k].clone() for k in self.keys})
            self._dst = [self.static[k] for k in self.keys]
        elif not self._fits(inter):
            return self._eager(inter)
        else:                                       # every column in ONE copy launch
            ops.copy_many(self._dst, [inter[k].contiguous() for k in self.keys])
        if self.graph is not None:
            self.graph.replay()
            self.opt.n_steps += 1
            self.n_graphed += 1
            return self.static_loss
        if self.n_warm < self.warmup:              # torch's recipe: warm up on a side stream
            cur = torch.cuda.current_stream(self.dev)
            self.side.wait_stream(cur)
            with torch.cuda.stream(self.side):
                loss = self._eager(self.static)
            cur.wait_stream(self.side)
            self.n_warm += 1
            return loss
        self.opt.zero_grad(set_to_none=True)
        n0 = self.opt.n_steps
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = self.loss_func(self.static)
            self._backward(loss)
            self.opt.step()
            self.static_loss = loss.detach()
        self.opt.n_steps = n0                      # capturing did not run the step
        self.graph = g
        g.replay()
        self.opt.n_steps += 1
        self.n_graphed += 1
        return self.static_loss

    def close(self):
        self.graph = None
