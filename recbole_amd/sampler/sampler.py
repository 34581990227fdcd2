"""Negative samplers (mirror of recbole/sampler/sampler.py:22-265, 341-420).

Same public API — Sampler(phases, datasets, distribution), set_phase(),
set_distribution(), sample_by_user_ids(user_ids, num), RepeatableSampler —
and the same bit-exact output, but the walk runs on the GPU (K4,
recbole_amd/csrc/sampler.hip):

* random_list: built and shuffled on the host with the GLOBAL numpy RNG exactly
  as the reference (sampler.py:45-57: first numpy draw after init_seed), then
  kept resident in HBM as int32;
* random_pr: one int64 in HBM per phase copy (set_phase returns a shallow copy
  with its own pointer, like the reference's copy.copy of an int attribute);
* used_ids: per phase a CSR (row_ptr int64[U+1], sorted int32 cols) built with
  vectorised numpy instead of the reference's per-interaction Python
  set.add loop (sampler.py:206-227); the `used_ids` attribute is still
  available as an array of Python sets, built lazily, for API compatibility.

Differences, documented: sample_by_user_ids returns a tensor on the sampler's
device (the reference returns a CPU tensor), and an out-of-range user id
raises ValueError before the walk advances (the reference advances
random_pr by one round first; ids < 0 wrap around there).
"""
from __future__ import annotations

import copy
import os

import numpy as np
import torch

from recbole_amd import ops
from recbole_amd._native import lib


class AbstractSampler(object):

    def __init__(self, distribution):
        self.distribution = ''
        self.random_list = np.zeros(0, dtype=np.int64)
        self.random_list_length = 0
        self.device = None
        self._rl_dev = None
        self._pr_dev = None
        self._pr_host = 0
        self.set_distribution(distribution)
        self.used_csr = self.get_used_csr()

    # ------------------------------------------------------------ distribution
    def set_distribution(self, distribution):
        """sampler.py:45-57."""
        if self.distribution == distribution:
            return
        self.distribution = distribution
        rl = np.asarray(self.get_random_list())
        np.random.shuffle(rl)
        self.random_list = rl
        self.random_list_length = len(rl)
        self._rl_dev = None
        self._pr_dev = None
        self._pr_host = 0
        if getattr(self, 'alias', None) is not None:
            self._build_alias()

    # ------------------------------------------------------------ alias fast mode
    def enable_alias(self, seed=0):
        """Switch to the alias-table FAST MODE (labelled NON-PARITY, north_star
        (c); config `neg_sampling_alias`): i.i.d. draws from the distribution the
        walk follows — p(v) proportional to the number of times v appears in
        random_list — with the same rejection of used ids, but not the reference's
        value sequence. Every draw is independent, so a chunk of batches is one
        wide launch instead of a serial walk (mirec_sample_alias). Deterministic
        for a seed; random_pr is left untouched."""
        self.alias_seed = int(seed) & (2 ** 64 - 1)
        self._alias_ctr = 0
        self._build_alias()
        return self

    def _build_alias(self):
        counts = np.bincount(np.asarray(self.random_list, dtype=np.int64),
                             minlength=self.n_items)
        self.alias = ops.alias_build(counts)
        self._alias_dev = None

    def alias_args(self, device, n_draws):
        """(thr, alias, seed, counter) for n_draws draws; advances the counter."""
        if self._alias_dev is None or self._alias_dev[0].device != torch.device(device):
            thr, idx = self.alias
            self._alias_dev = (torch.as_tensor(thr.view(np.int32), device=device),
                               torch.as_tensor(idx, device=device))
        c = self._alias_ctr
        self._alias_ctr += int(n_draws)
        return self._alias_dev[0], self._alias_dev[1], self.alias_seed, c

    def _alias_draw(self, keys, num, batch_keys=None, out=None, out_stride=0):
        up, uc = self._used_dev()
        bits, n_bits = self._used_bits()
        thr, idx, seed, c = self.alias_args(self.device, keys.numel() * int(num))
        return ops.sample_alias(thr, idx, seed, c, keys, int(num), up, uc, self.n_users,
                                up is not None, batch_keys=batch_keys, out=out,
                                out_stride=out_stride, status=self._status, used_bits=bits,
                                n_bits=n_bits)

    def _phase_alias(self, phase):
        # a phase copy draws its own stream (seed mixed with the phase index)
        if self.alias is not None:
            self.alias_seed = (self.alias_seed * 0x9E3779B97F4A7C15 +
                               1 + self.phases.index(phase)) & (2 ** 64 - 1)

    def get_random_list(self):
        raise NotImplementedError('method [get_random_list] should be implemented')

    def get_used_csr(self):
        raise NotImplementedError('method [get_used_csr] should be implemented')

    # ------------------------------------------------------------ device state
    def to_device(self, device):
        device = torch.device(device)
        if device.type != 'cuda':
            raise RuntimeError('recbole_amd samplers run on the GPU only (no CPU fallback)')
        if self.device != device or self._rl_dev is None:
            self.device = device
            self._rl_dev = torch.as_tensor(self.random_list.astype(np.int32), device=device)
            self._pr_dev = torch.tensor([self._pr_host], dtype=torch.int64, device=device)
            self._status = torch.zeros(1, dtype=torch.int32, device=device)
            self._ws = None
        return self

    alias = None

    @property
    def random_pr(self):
        if self._pr_dev is not None:
            return int(self._pr_dev.item())
        return self._pr_host

    @random_pr.setter
    def random_pr(self, value):
        self._pr_host = int(value)
        if self._pr_dev is not None:
            self._pr_dev.fill_(int(value))

    def _used_dev(self):
        return None, None

    def _used_bits(self):
        return None, 0

    def check_status(self):
        """Raise what the walk reported since the last check (one host sync):
        -2 a key outside [0, n_users) (the reference raises ValueError), -3 a walk
        that did not terminate (the reference would loop forever)."""
        if self._pr_dev is None:
            return
        s = int(self._status.item())
        if s == 0:
            return
        self._status.zero_()
        if s == -2:
            raise ValueError('user_id out of range in negative sampling')
        if self.alias is not None:
            raise RuntimeError('alias negative sampling found no free item for a user within '
                               '4096 draws')
        raise RuntimeError('negative sampling did not terminate: a user has no free item the '
                           'walk over random_list can reach')

    def _default_device(self):
        if self.device is not None:
            return self.device
        if not torch.cuda.is_available():
            raise RuntimeError('recbole_amd samplers run on the GPU only (no CPU fallback)')
        return torch.device('cuda', torch.cuda.current_device())

    # ------------------------------------------------------------ sampling
    def sample_by_key_ids(self, key_ids, num):
        """sampler.py:103-154 (both branches), on the device."""
        if self.random_list_length == 0:
            raise ValueError('the random list is empty; nothing to sample from')
        if self._rl_dev is None:
            self.to_device(self._default_device())
        keys = torch.as_tensor(key_ids)
        if keys.dim() == 0:
            keys = keys.view(1)
        keys = keys.to(device=self.device, dtype=torch.int64).contiguous()
        if self.alias is not None:
            out = self._alias_draw(keys, num)
            self.check_status()
            return out
        up, uc = self._used_dev()
        bits, n_bits = self._used_bits()
        reject = up is not None
        out = ops.sample_walk(self._rl_dev, self._pr_dev, keys, int(num), up, uc,
                              self.n_users, reject, status=self._status, used_bits=bits,
                              n_bits=n_bits)
        self.check_status()
        return out

    def launch_batches(self, keys_dev, batch_keys, n_batches, num, out, out_stride=0, ws=None):
        """Walk `n_batches` consecutive batches in ONE kernel launch (the trainer's
        ahead-of-time path); keys_dev are device user ids, batch b's values land at
        out[b*out_stride:] (default stride batch_keys*num) in the j*Kb + k layout."""
        if self._rl_dev is None:
            self.to_device(keys_dev.device)
        if self.alias is not None:
            return self._alias_draw(keys_dev, num, batch_keys=batch_keys, out=out,
                                    out_stride=out_stride)
        up, uc = self._used_dev()
        bits, n_bits = self._used_bits()
        return ops.sample_walk(self._rl_dev, self._pr_dev, keys_dev, int(num), up, uc,
                               self.n_users, up is not None, batch_keys=batch_keys,
                               n_batches=n_batches, out=out, status=self._status, ws=ws,
                               out_stride=out_stride, used_bits=bits, n_bits=n_bits)

    def walk_args(self, device):
        """Device operands of the walk for the native chunk preparation
        (mirec_prepare_chunk): (random_list, pr, used_ptr, used_cols, used_bits,
        n_bits, reject, status)."""
        if self._rl_dev is None:
            self.to_device(device)
        up, uc = self._used_dev()
        bits, n_bits = self._used_bits()
        return self._rl_dev, self._pr_dev, up, uc, bits, n_bits, up is not None, self._status

    def walk_stats(self, key_counts, batch_keys, num):
        """(mean, sd) of the refill draws one walk batch of `batch_keys` keys x `num`
        takes beyond its round-0 slots, when its keys are drawn like `key_counts` (host
        per-key weights, e.g. the train users' interaction counts): a key u rejects a
        draw with p_u = (occurrences in random_list of u's used ids) / L, so a slot takes
        Geometric(1 - p_u) - 1 extra draws (mean p/(1-p), variance p/(1-p)^2) and the
        num slots of a key share its p_u. Sizes the speculative walk's windows
        (mirec_sample_walk_spec) — a statistic, never a parity assumption."""
        key = (self.phase, int(batch_keys), int(num))
        cache = self.__dict__.setdefault('_walk_stats', {})
        if key in cache:
            return cache[key]
        try:
            reject = self._used_dev()[0] is not None       # RepeatableSampler: no rejection
        except ValueError:                                  # no phase set
            reject = False
        if not reject or self.random_list_length == 0:
            cache[key] = (0.0, 0.0)
            return cache[key]
        ptr, cols = self.used_csr[self.phase]
        rl = np.asarray(self.random_list, dtype=np.int64)
        mult = np.bincount(rl, minlength=int(max(self.n_items, rl.max() + 1 if len(rl) else 1)))
        cs = np.concatenate([[0], np.cumsum(mult[np.asarray(cols, dtype=np.int64)])])
        ptr = np.asarray(ptr, dtype=np.int64)
        p = np.minimum((cs[ptr[1:]] - cs[ptr[:-1]]) / float(len(rl)), 0.999)
        w = np.asarray(key_counts, dtype=np.float64)[:len(p)]
        w = np.pad(w, (0, len(p) - len(w)))
        w = w / max(w.sum(), 1.0)
        q = p / (1.0 - p)
        eq, eq2 = float((w * q).sum()), float((w * q / (1.0 - p)).sum())
        var_q = max(float((w * q * q).sum()) - eq * eq, 0.0)
        mean = batch_keys * num * eq
        var = batch_keys * num * eq2 + batch_keys * num * num * var_q
        cache[key] = (mean, float(np.sqrt(var)))
        return cache[key]

    def launch_segments(self, keys_dev, seg_ptr_dev, max_seg_keys, num):
        """Successive sample_by_key_ids calls (call s over keys_dev[seg_ptr[s]:
        seg_ptr[s+1]]) in ONE launch, the walk continuing from call to call; call
        s's values at [seg_ptr[s]*num, seg_ptr[s+1]*num) in the j*K_s + k layout."""
        if self._rl_dev is None:
            self.to_device(keys_dev.device)
        if self.alias is not None:
            # every draw is independent: expand the keys to the output layout
            # (call s, slot j*K_s + k -> key seg_ptr[s] + k) and draw one value each
            sp = seg_ptr_dev.to(torch.int64)
            K = sp[1:] - sp[:-1]
            seg = torch.repeat_interleave(torch.arange(len(K), device=sp.device), K * int(num))
            q = torch.arange(seg.numel(), device=sp.device) - sp[seg] * int(num)
            ekeys = keys_dev[sp[seg] + q % K[seg]].contiguous()
            return self._alias_draw(ekeys, 1)
        up, uc = self._used_dev()
        bits, n_bits = self._used_bits()
        return ops.sample_walk_segments(self._rl_dev, self._pr_dev, keys_dev, seg_ptr_dev,
                                        int(max_seg_keys), int(num), up, uc, self.n_users,
                                        up is not None, used_bits=bits, n_bits=n_bits,
                                        status=self._status)

    def sample_by_user_ids(self, user_ids, num):
        """sampler.py:246-265: empty input returns None (the reference's IndexError
        path); ids outside [0, n_users) raise ValueError."""
        ids = torch.as_tensor(user_ids)
        if ids.numel() == 0:
            return None
        mn, mx = int(ids.min()), int(ids.max())
        if mn < 0 or mx >= self.n_users:
            bad = mn if mn < 0 else mx
            raise ValueError(f'user_id [{bad}] not exist.')
        return self.sample_by_key_ids(ids, num)


def _csr_from_pairs(n_keys, keys, values):
    """CSR of the distinct (key, value) pairs, each row's values ascending
    (mirec_host_csr_build: one counting pass + a sort per row)."""
    return ops.host_csr_build(keys, values, n_keys)


class Sampler(AbstractSampler):
    """sampler.py:157-265: per-phase used sets are cumulative (train ⊂ valid ⊂ test)."""

    def __init__(self, phases, datasets, distribution='uniform'):
        if not isinstance(phases, list):
            phases = [phases]
        if not isinstance(datasets, list):
            datasets = [datasets]
        if len(phases) != len(datasets):
            raise ValueError(f'Phases {phases} and datasets {datasets} should have the same length.')
        self.phases = phases
        self.datasets = datasets
        self.uid_field = datasets[0].uid_field
        self.iid_field = datasets[0].iid_field
        self.n_users = datasets[0].user_num
        self.n_items = datasets[0].item_num
        self.phase = None
        self._used_dev_cache = {}
        super().__init__(distribution=distribution)

    def get_random_list(self):
        if self.distribution == 'uniform':
            return np.arange(1, self.n_items)
        if self.distribution == 'popularity':
            return np.concatenate([d.inter_feat[self.iid_field].numpy() for d in self.datasets])
        raise NotImplementedError(f'Distribution [{self.distribution}] has not been implemented.')

    def get_used_csr(self):
        """Cumulative per-phase used item sets as CSR (sampler.py:206-227)."""
        out = {}
        ks, vs = [], []
        for phase, ds in zip(self.phases, self.datasets):
            # cumulative sets (train, train+valid, all): counting pass + per-row sort
            ks.append(ds.inter_feat[self.uid_field].numpy())
            vs.append(ds.inter_feat[self.iid_field].numpy())
            out[phase] = ops.host_csr_build(np.concatenate(ks), np.concatenate(vs), self.n_users)
        last_ptr = out[self.phases[-1]][0]
        if (np.diff(last_ptr) + 1 == self.n_items).any():
            raise ValueError('Some users have interacted with all items, '
                             'which we can not sample negative items for them. '
                             'Please set `max_user_inter_num` to filter those users.')
        return out

    def set_phase(self, phase):
        if phase not in self.phases:
            raise ValueError(f'Phase [{phase}] not exist.')
        new = copy.copy(self)
        new.phase = phase
        new._phase_alias(phase)
        new._used_dev_cache = self._used_dev_cache
        new._pr_host = self.random_pr
        if self._pr_dev is not None:
            new._pr_dev = self._pr_dev.clone()
        return new

    def _used_dev(self):
        if self.phase is None:
            raise ValueError('call set_phase() before sampling')
        key = (self.phase, self.device)
        if key not in self._used_dev_cache:
            ptr, cols = self.used_csr[self.phase]
            self._used_dev_cache[key] = (
                torch.as_tensor(ptr, device=self.device),
                torch.as_tensor(cols if len(cols) else np.zeros(1, np.int32), device=self.device))
        return self._used_dev_cache[key]

    # the used sets as a [n_users, ceil(n_items/32)] bitmap when it fits this many
    # bytes of HBM (one load per membership test); else the CSR binary search
    BITMAP_BUDGET = int(os.environ.get('MIREC_SAMPLER_BITMAP_MB', '4096')) << 20

    def _used_bits(self):
        if lib().mirec_used_bitmap_bytes(self.n_users, self.n_items) > self.BITMAP_BUDGET:
            return None, 0
        key = (self.phase, self.device, 'bits')
        if key not in self._used_dev_cache:
            up, uc = self._used_dev()
            self._used_dev_cache[key] = ops.used_bitmap(up, uc, self.n_users, self.n_items)
        return self._used_dev_cache[key], self.n_items

    @property
    def used_ids(self):
        """The reference's array of Python sets for the current phase (slow; API only)."""
        src = self.used_csr[self.phase] if self.phase is not None else None
        if src is None:
            return {p: _sets(*self.used_csr[p]) for p in self.phases}
        return _sets(*src)


def _sets(ptr, cols):
    return np.array([set(cols[ptr[u]:ptr[u + 1]].tolist()) for u in range(len(ptr) - 1)],
                    dtype=object)


class RepeatableSampler(AbstractSampler):
    """sampler.py:341-420: no rejection (used sets are empty)."""

    def __init__(self, phases, dataset, distribution='uniform'):
        if not isinstance(phases, list):
            phases = [phases]
        self.phases = phases
        self.dataset = dataset
        self.iid_field = dataset.iid_field
        self.n_users = dataset.user_num
        self.n_items = dataset.item_num
        self.phase = None
        super().__init__(distribution=distribution)

    def get_random_list(self):
        if self.distribution == 'uniform':
            return np.arange(1, self.n_items)
        if self.distribution == 'popularity':
            return self.dataset.inter_feat[self.iid_field].numpy()
        raise NotImplementedError(f'Distribution [{self.distribution}] has not been implemented.')

    def get_used_csr(self):
        return None

    @property
    def used_ids(self):
        return np.array([set() for _ in range(self.n_users)], dtype=object)

    def set_phase(self, phase):
        if phase not in self.phases:
            raise ValueError(f'Phase [{phase}] not exist.')
        new = copy.copy(self)
        new.phase = phase
        new._phase_alias(phase)
        new._pr_host = self.random_pr
        if self._pr_dev is not None:
            new._pr_dev = self._pr_dev.clone()
        return new
