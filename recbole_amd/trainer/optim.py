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
        # the K5 replay tests its fast-path ranges at the ends of step groups only
        # (adam.hip incr_steps): |step_size| must not increase, bc2_sqrt not decrease
        if count > 1 and not ((np.diff(np.abs(out[:, 0])) <= 0).all()
                              and (np.diff(out[:, 1]) >= 0).all()):
            raise ValueError('Adam step constants are not monotone (beta1/beta2 outside [0, 1))')
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
        deferred = getattr(self, '_deferred', {})
        params = [p for p in self._params() if p.grad is not None and p not in deferred]
        done = set()
        for p, q in self._pair_reduce(deferred):
            if self._pair_step(p, q):
                done.update((p, q))
        for p in deferred:
            if p not in done:
                self._deferred_step(p)
        advanced = False
        if params:
            advanced = self._dense_step(params)
        if params or deferred:
            if self._g is not None and not advanced:
                self._g['step'].add_(1)       # the device step counter of graph mode
            self.n_steps += 1
        return loss

    # ------------------------------------------------------------------ graph mode
    # A training step whose kernels take no host-side step index, so the whole step
    # (forward, backward, optimizer) can be captured in a HIP graph and replayed:
    # every parameter — dense and deferred — reads its Adam constants from ONE
    # window table indexed by a device counter that the step itself advances. The
    # host only rolls the window over between steps (graph_window()), flushing the
    # deferred tables exactly where the eager schedule would.
    _g = None

    def graph_mode(self, device, window: int = 256):
        self.flush()
        for ds in getattr(self, '_deferred', {}).values():
            ds['t0'] = None
            ds['window'] = window
        self._g = {'W': window, 't0': None,
                   'consts': torch.zeros(window * 4, dtype=torch.float32, device=device),
                   'step': torch.zeros(1, dtype=torch.int32, device=device),
                   # the flat launch's ticket when it advances 'step' (zero between steps)
                   'ticket': torch.zeros(1, dtype=torch.int32, device=device)}
        self._graph_open_window()

    def _graph_open_window(self):
        g = self._g
        g['t0'] = self.n_steps
        g['consts'].copy_(torch.as_tensor(self.step_constants(self.n_steps + 1, g['W'])
                                          .reshape(-1)))
        g['step'].zero_()
        for p in getattr(self, '_deferred', {}):
            ds = self._deferred[p]
            ds['t0'], ds['consts'] = self.n_steps, g['consts']
            if ds['marked']:
                ops.reset_marks(ds['last'])
            else:
                st = self.state[p]
                ops.zero_state_marks(st['exp_avg'], st['exp_avg_sq'], ds['last'],
                                     self._group_args()['weight_decay'])
                ds['marked'] = True

    def graph_window(self):
        """Before a graph-mode step: when the window is full, complete every deferred
        row and start the next window (host side, outside any captured graph)."""
        g = self._g
        if g is not None and self.n_steps - g['t0'] >= g['W']:
            self.flush()
            self._graph_open_window()

    def _sref(self, r, off=0):
        """(step base tensor, offset) of step index r + off of the current window."""
        if self._g is not None:
            return self._g['step'], off
        return self._zero_i32 if hasattr(self, '_zero_i32') else self._dwin['zero'], r + off

    def _dense_step(self, params, window=256):
        """One Adam step of parameters with dense gradients: the step constants come
        from a window uploaded once per `window` steps and every parameter goes into
        one flat K5 launch (up to 16 per launch) — no per-step host-to-device copy."""
        dev = params[0].device
        if self._g is not None:               # graph mode: the shared window, device index
            w = {'consts': self._g['consts'], 'zero': self._g['step'], 't0': self.n_steps,
                 'idx': self._g['step']}
        else:
            w = getattr(self, '_dwin', None)
        if self._g is None and (w is None or w['dev'] != dev or
                                not 0 <= self.n_steps - w['t0'] < w['W']):
            w = self._dwin = {
                'dev': dev, 't0': self.n_steps, 'W': window,
                'consts': torch.as_tensor(
                    self.step_constants(self.n_steps + 1, window).reshape(-1), device=dev),
                'idx': torch.arange(window, dtype=torch.int32, device=dev),
                'zero': torch.zeros(1, dtype=torch.int32, device=dev)}
        r = self.n_steps - w['t0']
        # every dense parameter in one flat launch per 16 (the same per-element step as
        # the row-table kernels: bit-identical; DeepFM ran six launches here)
        specs = []
        for p in params:
            st = self._ensure_state(p)
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            specs.append({'p': p.data, 'm': st['exp_avg'], 'v': st['exp_avg_sq'], 'g': g})
        # graph mode: the step's last launch also advances the device step counter
        ops.adam_flat_multi(specs, w['consts'],
                            w['idx'] if self._g is not None else w['idx'][r:r + 1],
                            advance_ticket=self._g['ticket'] if self._g is not None else None,
                            **self._group_args())
        return self._g is not None

    def advance(self, n: int):
        self.n_steps += n

    # ------------------------------------------------------------------ deferred tables
    # Embedding tables read sparsely through the autograd path (DeepFM's token
    # table, SASRec's item table) can run the deferred schedule of K5 instead of a
    # dense update: the model's autograd Functions (a) call catch_up() on the rows
    # a forward pass reads, which replays their skipped zero-gradient steps, and
    # (b) stash() the per-contribution gradient rows + their keys instead of
    # returning a dense gradient. step() then groups the stashed contributions
    # (K2) and applies the deferred step to the touched rows only; untouched rows
    # lag and are completed by flush() (window end, epoch end, state_dict()). The
    # result is bit-identical to the dense Adam the reference runs over every row.
    def enable_deferred(self, params, window: int = 256):
        """Run the deferred schedule for these 2-D parameters (width 1, 4..256)."""
        params = list(params)
        if not params:
            return
        dev = params[0].device
        if not hasattr(self, '_deferred'):
            self._deferred = {}
            self._zero_i32 = torch.zeros(1, dtype=torch.int32, device=dev)
            self._dummy_i32 = torch.zeros(2, dtype=torch.int32, device=dev)
            self._dummy_f32 = torch.zeros(4, dtype=torch.float32, device=dev)
            # the chained block sort's hand-off words (zero between calls; the optimizer
            # issues its sorts one after another on one stream)
            self._sort_status = torch.zeros(ops.CHAIN_MAX_BLOCKS + 1, dtype=torch.int32,
                                            device=dev)
        for p in params:
            if p.dim() != 2 or p.shape[1] not in (1, 4, 16, 32, 64, 128, 256) or not p.is_cuda:
                continue
            self._ensure_state(p)
            self._deferred[p] = {'last': torch.zeros(p.shape[0], dtype=torch.int32,
                                                     device=p.device),
                                 'window': window, 't0': None, 'consts': None, 'stash': [],
                                 'marked': False}
            p._mirec_deferred = self

    def _dstate(self, p):
        ds = self._deferred[p]
        if ds['t0'] is None:                  # open a window at the current step
            ds['t0'] = self.n_steps
            ds['consts'] = torch.as_tensor(
                self.step_constants(self.n_steps + 1, ds['window']).reshape(-1),
                device=p.device)
            if ds['marked']:                  # marks kept: those rows are still +0
                ops.reset_marks(ds['last'])
            else:                             # rows whose m, v are +0 (adam.hip kZeroState)
                st = self.state[p]
                ops.zero_state_marks(st['exp_avg'], st['exp_avg_sq'], ds['last'],
                                     self._group_args()['weight_decay'])
                ds['marked'] = True
        return ds

    def _dspec(self, p, ds, **kw):
        st = self.state[p]
        pt = ds['shard']['p'] if 'shard' in ds else p.data
        spec = {'p': pt, 'm': st['exp_avg'], 'v': st['exp_avg_sq'], 'last': ds['last']}
        spec.update(kw)
        return spec

    def _dtable(self, p, ds, **kw):
        return ops.adam_tables([self._dspec(p, ds, **kw)])

    def _pair_state(self, p, q):
        """The deferred state of q when p ([V, d], d > 1) and q ([V, 1]) can share one
        launch (mirec_adam_deferred_pair_f32): neither sharded, windows opened at the
        same step (the same step constants), else None."""
        dq = self._deferred.get(q) if q is not None else None
        ds = self._deferred[p]
        if (dq is None or 'shard' in dq or 'shard' in ds or q.shape[1] != 1 or p.shape[1] < 4
                or p.shape[0] != q.shape[0]):
            return None
        ds, dq = self._dstate(p), self._dstate(q)
        return dq if (dq['t0'] == ds['t0'] and dq['window'] == ds['window']) else None

    def catch_up(self, p, keys, segs=None, blocks=None, drop_key=None, pair=None):
        """Make the rows `keys` (int64, any order / duplicates) current before a
        forward pass reads them; returns their K2 grouping (`segs`: the grouping
        when the caller already has it, e.g. another table read by the same keys;
        `blocks`: the keys come in blocks of this size with increasing key ranges,
        which K2 then sorts block by block in LDS). drop_key: a padding_idx row —
        nn.Embedding gives it no gradient, so its contributions are left out of the
        grouping (they sort last under a sentinel key and n_uniq excludes them): the row
        stays untouched, which the deferred schedule makes bit-identical to a step with a
        zero gradient, and the reduction skips what can be half of a padded sequence
        batch's positions. Only with weight_decay 0: the row then never moves (a zero-
        gradient step keeps m = v = 0 and p), so the forward may read it un-caught-up.
        pair: a [V, 1] table of this optimizer read by the same keys (DeepFM's first-order
        weights): caught up too, in the same launch when _pair_state allows."""
        if (segs is None and drop_key is not None and 'shard' not in self._deferred[p]
                and self._group_args()['weight_decay'] == 0):
            n_rows = p.shape[0]
            k = keys.contiguous()
            k = torch.where(k == int(drop_key), torch.full_like(k, n_rows), k)
            segs = ops.segment_sort(k, n_rows + 1)
            last = segs.uniq.gather(0, (segs.n_uniq.long() - 1).clamp(min=0))
            segs.n_uniq.sub_((last == n_rows).to(torch.int32))
        elif segs is None and blocks:
            segs = ops.segment_sort_blocks(keys.contiguous(), int(blocks), p.shape[0],
                                           status=self._sort_status)
        elif segs is None:
            segs = ops.segment_sort(keys.contiguous(), p.shape[0])
        if 'shard' in self._deferred[p]:
            self._catch_up_sharded(p, keys)
            if pair is not None:
                self.catch_up(pair, keys, segs)
            return segs
        dq = self._pair_state(p, pair)
        ds = self._dstate(p)
        r = self.n_steps - ds['t0']
        if r > 0 or self._g is not None:      # (graph mode at r = 0: a no-op launch)
            class _Z:
                perm = uniq = seg = self._dummy_i32
                n_uniq = self._zero_i32
            kw = dict(rows=self._dummy_f32, segs=_Z, ahead=(segs.uniq, segs.n_uniq))
            specs = [self._dspec(p, ds, **kw)] + ([self._dspec(pair, dq, **kw)] if dq else [])
            base, off = self._sref(r, -1)
            ops.adam_multi(ops.adam_tables(specs), p.shape[1], ds['consts'], base, off,
                           schedule='deferred_pair' if dq else 'deferred',
                           n_max_uniq=[keys.numel()] * len(specs), **self._group_args())
        if pair is not None and dq is None:
            self.catch_up(pair, keys, segs)
        return segs

    def stash(self, p, rows, keys, segs=None):
        """Per-contribution gradient rows [n, d] for the table rows `keys` [n]
        (segs: their K2 grouping when the caller already has it)."""
        self._deferred[p]['stash'].append((rows, keys, segs))

    def _flush_table(self, p, ds, target, device_step=False):
        """Every row of p through step index `target` of the window (device_step:
        through the graph-mode device counter instead)."""
        if ds['t0'] is None or (target <= 0 and not device_step):
            return
        tab = self._dtable(p, ds)
        base, off = (self._g['step'], 0) if device_step else (self._zero_i32, target)
        ops.adam_multi(tab, p.shape[1], ds['consts'], base, off,
                       schedule='flush', **self._group_args())

    def flush(self):
        """Complete every row of every deferred table (after it, p / m / v equal
        the dense schedule's). Row-sharded tables: every owner completes its shard
        and one all-gather refreshes the full parameter on every rank (a collective:
        every rank calls flush at the same points)."""
        for p, ds in getattr(self, '_deferred', {}).items():
            if ds['t0'] is not None:
                self._flush_table(p, ds, self.n_steps - ds['t0'])
            if 'shard' in ds and ds['shard']['synced'] != self.n_steps:
                p.data.copy_(self._gather_shard(ds, ds['shard']['p'], p.shape[0]))
                ds['shard']['synced'] = self.n_steps

    def _pair_reduce(self, deferred):
        """Tables stashed with the same single grouping — a [V, d] table (d <= 16) and a
        [V, 1] one, DeepFM's token rows and first-order weights — are reduced in one pass
        (ops.segment_reduce2, bit for bit the two reductions); the results wait in
        ds['pre'] for _deferred_step."""
        one = [(p, ds) for p, ds in deferred.items()
               if len(ds['stash']) == 1 and ds['stash'][0][2] is not None and 'shard' not in ds
               and p.grad is None]
        wide = [(p, ds) for p, ds in one if 2 <= p.shape[1] <= 16]
        narrow = [(p, ds) for p, ds in one if p.shape[1] == 1]
        pairs = []
        for p, ds in wide:
            rows, keys, segs = ds['stash'][0]
            for q, dq in narrow:
                r1, k1, s1 = dq['stash'][0]
                if s1 is segs and 'pre' not in dq and r1.shape[0] == rows.shape[0]:
                    out, out1, ident = ops.segment_reduce2(rows.contiguous(),
                                                           r1.contiguous().view(-1, 1), segs)
                    ds['pre'] = (out, ident, ident.n)
                    dq['pre'] = (out1, ident, ident.n)
                    pairs.append((p, q))
                    break
        return pairs

    def _pair_step(self, p, q):
        """The deferred steps of a pair reduced together (_pair_reduce) in one launch
        (mirec_adam_deferred_pair_f32) when _pair_state allows; False: not taken (each
        table then takes _deferred_step)."""
        dq = self._pair_state(p, q)
        if dq is None or p.grad is not None or q.grad is not None:
            return False
        ds = self._deferred[p]
        ds['stash'], dq['stash'] = [], []
        rows, segs, n_keys = ds.pop('pre')
        rows1, segs1, n1 = dq.pop('pre')
        r = self.n_steps - ds['t0']
        tabs = ops.adam_tables([self._dspec(p, ds, rows=rows.contiguous(), segs=segs),
                                self._dspec(q, dq, rows=rows1.contiguous(), segs=segs1)])
        base, off = self._sref(r, 0)
        ops.adam_multi(tabs, p.shape[1], ds['consts'], base, off, schedule='deferred_pair',
                       n_max_uniq=[n_keys, n1], **self._group_args())
        if self._g is None and r + 1 >= ds['window']:   # window full: complete every row
            for t, dt in ((p, ds), (q, dq)):
                self._flush_table(t, dt, r + 1)
                dt['t0'] = None
        return True

    def _combine_stash(self, p, stash):
        """One summed gradient row per touched table row. Each source (one autograd
        Function's contributions) is grouped and reduced on its own, in chunked
        fixed order; several sources are then added row-wise in source order —
        the same sums the dense path forms (a dense gradient per Function, added
        by autograd), so both schedules stay bit-identical."""
        ds = self._deferred[p]
        n_rows = ds['shard']['n_own'] if 'shard' in ds else p.shape[0]
        parts = []
        for rows, keys, segs in stash:
            if segs is None:
                segs = ops.segment_sort(keys.contiguous(), n_rows)
            parts.append(ops.segment_reduce(rows.contiguous(), segs))
        if len(parts) == 1:
            rows, segs = parts[0]
            return rows, segs, segs.n
        if all(cr.shape[0] >= cs.n for cr, cs in parts):
            # second level as merges of the sources' row lists (ops.segment_merge2): the
            # sums of the sort + reduce below, bit for bit, in two launches per merge
            acc = parts[0]
            for k, part in enumerate(parts[1:]):
                acc = ops.segment_merge2(acc, part, a_pre=k > 0)
            rows, segs = acc
            return rows, segs, segs.n
        # second level: key = the table row of each compact row, sentinel n_rows
        # beyond a source's n_uniq (dropped after the sort: it is the last group)
        keys, rows = [], []
        for cr, cs in parts:
            idx = torch.arange(cs.n, device=p.device)
            keys.append(torch.where(idx < cs.n_uniq.long(), cs.uniq[:cs.n].long(),
                                    torch.full_like(idx, n_rows)))
            rows.append(cr[:cs.n])
        keys, rows = torch.cat(keys), torch.cat(rows)
        segs = ops.segment_sort(keys, n_rows + 1)
        last = segs.uniq.gather(0, (segs.n_uniq.long() - 1).clamp(min=0))
        segs.n_uniq.sub_((last == n_rows).to(torch.int32))
        rows, segs = ops.segment_reduce(rows, segs)
        return rows, segs, segs.n

    def _deferred_step(self, p):
        ds = self._deferred[p]
        stash, ds['stash'] = ds['stash'], []
        if 'shard' in ds:
            # contributions exchanged to their owners carry local row ids ('owned');
            # a batch computed whole on every rank (ragged: no exchange) keeps this
            # rank's rows only
            sh = ds['shard']
            out = []
            for rows, keys, tag in stash:
                if tag != 'owned':
                    mine = (keys % sh['G']) == sh['r']
                    rows, keys = rows[mine], keys[mine] // sh['G']
                out.append((rows, keys, None))
            stash = [x for x in out if x[1].numel()]
        if not stash and p.grad is None:      # table not in this step's graph: skipped
            if ds['t0'] is not None:
                self._flush_table(p, ds, self.n_steps - ds['t0'])
                ds['t0'] = None
            return
        ds = self._dstate(p)
        r = self.n_steps - ds['t0']
        pre = ds.pop('pre', None)
        if pre is not None:                   # reduced together with its pair table
            rows, segs, n_keys = pre
        elif stash:
            rows, segs, n_keys = self._combine_stash(p, stash)
        graph = self._g is not None
        if p.grad is not None and 'shard' in ds:
            raise NotImplementedError('a row-sharded deferred table takes stashed gradient '
                                      'rows only (no dense gradient)')
        if p.grad is not None:                # a dense contribution too: stream every row
            self._flush_table(p, ds, r, device_step=graph)
            st = self.state[p]
            kw = {'rows': rows.contiguous(), 'segs': segs} if stash else {}
            ops.adam_step(p.data, st['exp_avg'], st['exp_avg_sq'], ds['consts'],
                          self._g['step'] if graph else self._zero_i32 + r,
                          dense_grad=p.grad.contiguous(), **kw, **self._group_args())
            if graph:
                ds['last'].copy_((self._g['step'] + 1).expand_as(ds['last']))
            else:
                ds['last'].fill_(r + 1)
        else:
            tab = self._dtable(p, ds, rows=rows.contiguous(), segs=segs)
            base, off = self._sref(r, 0)
            ops.adam_multi(tab, p.shape[1], ds['consts'], base, off,
                           schedule='deferred', n_max_uniq=[n_keys],
                           **self._group_args())
        if not graph and r + 1 >= ds['window']:   # window full: complete every row
            self._flush_table(p, ds, r + 1)
            ds['t0'] = None

    # ------------------------------------------------------------------ row sharding
    # SURVEY.md §8e for the autograd path (C4 DeepFM's token tables, C3 SASRec's item
    # table): rank r of G owns the rows id % G == r of every deferred table — their
    # p, m, v and step counts as [n_own, d] shards (local row id // G), and runs the
    # deferred K5 (touched rows, catch-ups, flushes) on them only. The full parameter
    # stays on every rank as the forward's read cache: before a forward reads rows,
    # catch_up fetches them from their owners (all-to-all of ids, owner-side catch-up
    # of exactly those rows, all-to-all of the rows back into the cache); after the
    # backward, DataParallelStep.exchange sends every contribution row to its owner
    # (all-to-all, in source-rank order = the global batch's order), so each owner
    # applies the same sums and the same Adam step as one GPU on the global batch.
    def shard_deferred(self, group):
        """Row-shard the deferred tables over the ranks of `group`."""
        import torch.distributed as tdist
        G, r = tdist.get_world_size(group), tdist.get_rank(group)
        if G <= 1 or not getattr(self, '_deferred', None):
            return
        self.flush()
        for p, ds in self._deferred.items():
            if 'shard' in ds:
                continue
            st = self.state[p]
            own = torch.arange(r, p.shape[0], G, device=p.device)
            ds['shard'] = {'G': G, 'r': r, 'group': group, 'own': own, 'n_own': len(own),
                           'S': -(-p.shape[0] // G), 'p': p.data[own].contiguous(),
                           'synced': self.n_steps}
            st['exp_avg'] = st['exp_avg'][own].contiguous()       # this rank's moments only
            st['exp_avg_sq'] = st['exp_avg_sq'][own].contiguous()
            ds['last'] = torch.zeros(len(own), dtype=torch.int32, device=p.device)
            ds['t0'], ds['marked'] = None, False

    @staticmethod
    def _gather_shard(ds, t, n_rows):
        """The full [n_rows, ...] tensor of every rank's shard t (row id = l*G + g)."""
        from recbole_amd.trainer.dist import _gather_cat
        sh = ds['shard']
        G, S = sh['G'], sh['S']
        pad = torch.zeros((S,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[:t.shape[0]] = t
        full = _gather_cat(pad, sh['group']).view((G, S) + tuple(t.shape[1:]))
        return full.transpose(0, 1).reshape((G * S,) + tuple(t.shape[1:]))[:n_rows]

    def _catch_up_sharded(self, p, keys):
        """Make the rows `keys` of the cache p current: owners catch them up on their
        shards and send them back (two all-to-alls)."""
        from recbole_amd.trainer.dist import all_to_all_v
        ds = self._deferred[p]
        sh = ds['shard']
        if sh['synced'] == self.n_steps:      # the cache is complete (after a flush): no
            return                            # exchange (evaluation reads stay rank-local)
        G = sh['G']
        uniq = torch.unique(keys)
        owner = uniq % G
        send = uniq[torch.argsort(owner, stable=True)]
        counts = torch.bincount(owner, minlength=G)
        req, rcounts = all_to_all_v(send, counts, sh['group'])
        local = req // G
        ds = self._dstate(p)
        r = self.n_steps - ds['t0']
        if r > 0 and local.numel():
            lsegs = ops.segment_sort(local.contiguous(), sh['n_own'])

            class _Z:
                perm = uniq = seg = self._dummy_i32
                n_uniq = self._zero_i32
            tab = self._dtable(p, ds, rows=self._dummy_f32, segs=_Z,
                               ahead=(lsegs.uniq, lsegs.n_uniq))
            base, off = self._sref(r, -1)
            ops.adam_multi(tab, p.shape[1], ds['consts'], base, off,
                           schedule='deferred', n_max_uniq=[local.numel()],
                           **self._group_args())
        rows = sh['p'][local]
        back, _ = all_to_all_v(rows, rcounts, sh['group'])
        p.data[send] = back

    # ------------------------------------------------------------------ (de)serialise
    def state_dict(self):
        self.flush()
        params = self._params()
        state = {}
        for i, p in enumerate(params):
            st = self.state.get(p, {})
            if 'exp_avg' in st:
                m, v = st['exp_avg'], st['exp_avg_sq']
                ds = getattr(self, '_deferred', {}).get(p)
                if ds is not None and 'shard' in ds:   # row-sharded: the full moments
                    m = self._gather_shard(ds, m, p.shape[0])
                    v = self._gather_shard(ds, v, p.shape[0])
                state[i] = {'step': torch.tensor(float(self.n_steps)),
                            'exp_avg': m, 'exp_avg_sq': v}
        groups = []
        k = 0
        for g in self.param_groups:
            gd = {key: v for key, v in g.items() if key != 'params'}
            gd['params'] = list(range(k, k + len(g['params'])))
            k += len(g['params'])
            groups.append(gd)
        return {'state': state, 'param_groups': groups}

    def load_state_dict(self, state_dict):
        self._dwin = None
        for ds in getattr(self, '_deferred', {}).values():
            ds['t0'] = None                   # loaded rows are complete: new window
            ds['stash'] = []
            ds['marked'] = False              # zero-state marks recomputed from the state
        params = self._params()
        for g, sg in zip(self.param_groups, state_dict['param_groups']):
            for key, v in sg.items():
                if key != 'params':
                    g[key] = v
        steps = 0
        for i, st in state_dict['state'].items():
            p = params[int(i)]
            mine = self._ensure_state(p)
            steps = int(float(st['step']))     # every entry, row-sharded tables included
            ds = getattr(self, '_deferred', {}).get(p)
            if ds is not None and 'shard' in ds:       # this rank's rows of the full moments
                sh = ds['shard']
                own = sh['own'].to(st['exp_avg'].device)
                mine['exp_avg'].copy_(st['exp_avg'][own].to(p.device))
                mine['exp_avg_sq'].copy_(st['exp_avg_sq'][own].to(p.device))
                sh['p'].copy_(p.data[sh['own']])
                sh['synced'] = None
                continue
            mine['exp_avg'].copy_(st['exp_avg'].to(p.device))
            mine['exp_avg_sq'].copy_(st['exp_avg_sq'].to(p.device))
        self.n_steps = steps
        for p, ds in getattr(self, '_deferred', {}).items():
            if 'shard' in ds:
                ds['shard']['synced'] = self.n_steps      # the loaded p is complete
        if self._g is not None:               # graph mode: a new window at the loaded step
            self._graph_open_window()
