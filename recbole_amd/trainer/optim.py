"""FusedAdam: torch.optim.Adam semantics (the reference's learner 'adam',
trainer.py:115-116; torch optim/adam.py _single_tensor_adam) executed by the
K5 kernel, with two entry points:

* step()              — dense gradients in p.grad (drop-in for optim.Adam);
* step_compact(i, ..) — table i's gradient given as grouped compact rows
                        (the fused BPR path: no dense gradient ever exists).

Either way every row of every parameter is updated every step, exactly like
the reference's dense Adam over nn.Embedding(sparse=False) weights.

Bias corrections are computed on the host in double precision, like torch
(step_size = lr / (1 - b1^t), bc2_sqrt = sqrt(1 - b2^t)), cast to float and
kept in a device table indexed by a device step counter, so a captured HIP
graph can replay many steps. state_dict() has torch.optim.Adam's layout
(state[i] = {'step', 'exp_avg', 'exp_avg_sq'}), so checkpoints interoperate.
"""
from __future__ import annotations

import numpy as np
import torch

from recbole_amd import ops


class FusedAdam(torch.optim.Optimizer):

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        # torch.optim.Adam's argument checks (optim/adam.py __init__)
        if not 0.0 <= lr:
            raise ValueError(f'Invalid learning rate: {lr}')
        if not 0.0 <= eps:
            raise ValueError(f'Invalid epsilon value: {eps}')
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f'Invalid beta parameter at index 0: {betas[0]}')
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f'Invalid beta parameter at index 1: {betas[1]}')
        if not 0.0 <= weight_decay:
            raise ValueError(f'Invalid weight_decay value: {weight_decay}')
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False,
                        fused=None)
        super().__init__(params, defaults)
        self.n_steps = 0            # optimizer steps taken (torch's state['step'])
        self._consts = None         # device table [window, 4]: step_size, bc2_sqrt, 1/bc2_sqrt
        self._window_start = 0      # n_steps value at index 0 of the table
        self._step_idx = None       # device int32 cursor into the table

    # ------------------------------------------------------------------ state
    def _params(self):
        return [p for g in self.param_groups for p in g['params']]

    def _ensure_state(self, p):
        st = self.state[p]
        if 'exp_avg' not in st:
            st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    def step_constants(self, first_step: int, count: int):
        """float32 [count, 4] of (lr/(1-b1^t), sqrt(1-b2^t), RN(1/that), 0) for
        t = first_step..+count-1 (the K5 constant table, include/mirec.h)."""
        g = self.param_groups[0]
        lr, (b1, b2) = g['lr'], g['betas']
        out = np.zeros((count, 4), dtype=np.float32)
        for j in range(count):            # Python float pow, exactly as torch's step code
            t = float(first_step + j)
            out[j, 0] = lr / (1 - b1 ** t)
            out[j, 1] = (1 - b2 ** t) ** 0.5
        # correctly rounded reciprocal: 1/x in double then one rounding to float
        out[:, 2] = 1.0 / out[:, 1].astype(np.float64)
        # bound of the zero-gradient skip test (adam.hip p_update_vanishes):
        # step_size * bc2_sqrt * (1 + 2^-20), rounded up to float
        kq = out[:, 0].astype(np.float64) * out[:, 1].astype(np.float64) * (1 + 2.0 ** -20)
        kq32 = kq.astype(np.float32)
        out[:, 3] = np.where(kq32.astype(np.float64) < kq,
                             np.nextafter(kq32, np.float32(np.inf)), kq32)
        if count and not (out[:, 1] > 0).all():
            raise ValueError(f'beta2={b2} too close to 1: sqrt(1 - beta2^t) rounds to 0 in fp32')
        return out

    def prepare_window(self, n_steps_ahead: int, device):
        """Upload the constants of the next `n_steps_ahead` steps and reset the
        device cursor; the fused epoch runner calls this once per epoch."""
        table = self.step_constants(self.n_steps + 1, max(n_steps_ahead, 1))
        self._consts = torch.as_tensor(table.reshape(-1), device=device)
        self._window_start = self.n_steps
        if self._step_idx is None or self._step_idx.device != torch.device(device):
            self._step_idx = torch.zeros(1, dtype=torch.int32, device=device)
        else:
            self._step_idx.zero_()
        return self._consts, self._step_idx

    @property
    def device_step_idx(self):
        return self._step_idx

    def _group_args(self):
        g = self.param_groups[0]
        return dict(beta1=g['betas'][0], beta2=g['betas'][1], eps=g['eps'],
                    weight_decay=g['weight_decay'])

    # ------------------------------------------------------------------ steps
    def step_compact(self, p, rows, segs, consts, step_idx):
        """Adam step of parameter p whose gradient is the grouped compact rows.
        Does not advance n_steps (the epoch runner accounts steps)."""
        st = self._ensure_state(p)
        ops.adam_step(p.data, st['exp_avg'], st['exp_avg_sq'], consts, step_idx, rows=rows,
                      segs=segs, **self._group_args())

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        params = [p for p in self._params() if p.grad is not None]
        if not params:
            return loss
        dev = params[0].device
        consts, idx = self.prepare_window(1, dev)
        for p in params:
            st = self._ensure_state(p)
            ops.adam_step(p.data, st['exp_avg'], st['exp_avg_sq'], consts, idx,
                          dense_grad=p.grad.contiguous(), **self._group_args())
        self.n_steps += 1
        return loss

    def advance(self, n: int):
        self.n_steps += n

    # ------------------------------------------------------------------ (de)serialise
    def state_dict(self):
        params = self._params()
        state = {}
        for i, p in enumerate(params):
            st = self.state.get(p, {})
            if 'exp_avg' in st:
                state[i] = {'step': torch.tensor(float(self.n_steps)),
                            'exp_avg': st['exp_avg'], 'exp_avg_sq': st['exp_avg_sq']}
        groups = []
        k = 0
        for g in self.param_groups:
            gd = {key: v for key, v in g.items() if key != 'params'}
            gd['params'] = list(range(k, k + len(g['params'])))
            k += len(g['params'])
            groups.append(gd)
        return {'state': state, 'param_groups': groups}

    def load_state_dict(self, state_dict):
        params = self._params()
        for g, sg in zip(self.param_groups, state_dict['param_groups']):
            for key, v in sg.items():
                if key != 'params':
                    g[key] = v
        steps = 0
        for i, st in state_dict['state'].items():
            p = params[int(i)]
            mine = self._ensure_state(p)
            mine['exp_avg'].copy_(st['exp_avg'].to(p.device))
            mine['exp_avg_sq'].copy_(st['exp_avg_sq'].to(p.device))
            steps = int(float(st['step']))
        self.n_steps = steps
