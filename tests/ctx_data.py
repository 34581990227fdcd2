"""Synthetic context-aware (Criteo-like) atomic files for the DeepFM tests:
label:float, user_id / item_id tokens, float fields, token fields with Zipf ids,
and a token_seq field."""
import os

import numpy as np


def write_ctx_dataset(root, name='ctx', n=3000, n_float=3, n_tok=4, seed=0, seq=True):
    rng = np.random.default_rng(seed)
    d = os.path.join(root, name)
    os.makedirs(d, exist_ok=True)
    cols = ['label:float', 'user_id:token', 'item_id:token']
    cols += [f'I{j}:float' for j in range(n_float)]
    cols += [f'C{j}:token' for j in range(n_tok)]
    if seq:
        cols.append('tags:token_seq')
    vocab = [5, 40, 300, 7, 1000, 3][:n_tok]
    with open(os.path.join(d, f'{name}.inter'), 'w') as f:
        f.write('\t'.join(cols) + '\n')
        for r in range(n):
            row = [str(int(rng.random() < 0.3)), f'u{rng.integers(0, 60)}',
                   f'i{rng.integers(0, 90)}']
            row += [f'{rng.lognormal(0, 1):.5f}' for _ in range(n_float)]
            for v in vocab:
                z = min(int(rng.zipf(1.3)), v)
                row.append(f'c{z}')
            if seq:
                k = int(rng.integers(0, 4))
                row.append(' '.join(f't{int(t)}' for t in rng.integers(0, 12, k)))
            f.write('\t'.join(row) + '\n')
    return root
