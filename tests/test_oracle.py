"""The oracle (test infrastructure) against the reference's own known-answer
tests and fixtures, and its C restatement against a line-by-line numpy
restatement of both reference sampler branches."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import cpu_ref


def test_oracle_metrics_match_reference_known_answers():
    g = json.load(open(os.path.join(GOLDEN, 'metrics_known_answers.json')))['topk']
    pos_idx, pos_len = np.array(g['pos_idx']), np.array(g['pos_len'])
    for name, exp in g['expected'].items():
        assert cpu_ref.METRICS[name](pos_idx, pos_len).tolist() == np.array(exp).tolist(), name


def test_c_walk_equals_numpy_restatement_random():
    rng = np.random.default_rng(0)
    for trial in range(150):
        n_users, n_items = int(rng.integers(2, 9)), int(rng.integers(5, 50))
        nnz = int(rng.integers(0, n_users * n_items // 2))
        ku, ki = rng.integers(0, n_users, nnz), rng.integers(1, n_items, nnz)
        sets = [set() for _ in range(n_users)]
        for a, b in zip(ku, ki):
            sets[a].add(int(b))
        # the reference's walk can cycle forever when a user has almost no free
        # item (sampler.py:148-153); keep every user at least half free
        if any(2 * len(s) + 1 >= n_items for s in sets):
            continue
        rl = rng.permutation(np.arange(1, n_items))
        ptr, cols = cpu_ref.used_csr(n_users, ku, ki)
        walk = cpu_ref.NumpyWalk(rl, sets)
        pr = 0
        for _ in range(4):
            K, num = int(rng.integers(1, 7)), int(rng.integers(1, 5))
            single = rng.random() < 0.3
            keys = np.full(K, int(rng.integers(0, n_users))) if single else \
                rng.integers(0, n_users, K)
            a = walk.sample_by_key_ids(keys, num)
            c, pr = cpu_ref.c_sample_walk(rl, pr, keys, num, ptr, cols, n_users, True)
            assert (a == c).all()
            assert pr == walk.random_pr % len(rl)
            for t, v in enumerate(a):
                assert v not in sets[keys[t % K]]


def test_walk_golden_vectors():
    cases = json.load(open(os.path.join(GOLDEN, 'sampler_walk.json')))
    assert cases
    for c in cases:
        pr = 0
        for b in c['batches']:
            out, pr = cpu_ref.c_sample_walk(np.array(c['random_list']), pr, np.array(b['keys']),
                                            b['num'], np.array(c['used_ptr']),
                                            np.array(c['used_cols']), c['n_users'], True)
            assert out.tolist() == b['out'] and pr == b['pr']


def test_walk_livelock_is_bounded():
    # Two rejected slots advance the walk by 2 per round: slot 0 only ever sees
    # even positions, slot 1 odd ones. User 0's only free item (2) sits at an odd
    # position, user 1's (1) at an even one -> the reference loops forever.
    rl = np.array([1, 2, 3, 4])
    ptr, cols = cpu_ref.used_csr(2, np.array([0, 0, 0, 1, 1, 1]), np.array([1, 3, 4, 2, 3, 4]))
    with pytest.raises(RuntimeError):
        cpu_ref.c_sample_walk(rl, 0, np.array([0, 1]), 1, ptr, cols, 2, True)


def test_walk_wraps_around_list():
    rl = np.array([3, 1, 2])
    out, pr = cpu_ref.c_sample_walk(rl, 2, np.array([0]), 7, None, None, 1, False)
    assert out.tolist() == [2, 3, 1, 2, 3, 1, 2] and pr == 0


def test_random_list_is_first_numpy_draw():
    np.random.seed(2020)
    expect = np.arange(1, 10)
    np.random.shuffle(expect)
    assert cpu_ref.random_list_uniform(10, seed=2020).tolist() == expect.tolist()


def test_full_sort_oracle_swap_semantics():
    """The mask/swap/flip/topk restatement ranks exactly the unmasked items and
    flags positives (trainer.py:328-353, evaluators.py:53-76, 134)."""
    rng = np.random.default_rng(3)
    for _ in range(30):
        n, I, K = 4, int(rng.integers(12, 40)), 5
        scores = torch.tensor(rng.standard_normal((n, I)), dtype=torch.float32)
        hist, pos = [], []
        for r in range(n):
            perm = rng.permutation(np.arange(1, I))
            pos.append(sorted(perm[:int(rng.integers(1, 5))].tolist()))
            hist.append(sorted(perm[5:5 + int(rng.integers(0, 5))].tolist()))
        pos_idx, ids = cpu_ref.full_sort_pos_idx(scores, hist, pos, K)
        for r in range(n):
            allowed = [i for i in range(1, I) if i not in hist[r]]
            best = sorted(allowed, key=lambda i: -float(scores[r, i]))[:K]
            assert ids[r].tolist() == best
            assert pos_idx[r].tolist() == [i in pos[r] for i in best]
