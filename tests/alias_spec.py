"""Numpy restatement of the alias-table fast mode's own specification
(include/mirec.h mirec_alias_build / mirec_sample_alias) — test infrastructure.

The fast mode is labelled NON-PARITY: the reference has no alias sampler, so
there is no reference sequence to match. These functions pin the GPU kernel to
the spec it documents (same draws for the same seed and counter), and give the
exact distribution the table encodes for the statistical tests."""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
TRIES = 4096


def mix64(z):
    """splitmix64 finaliser on a uint64 array (wrapping arithmetic)."""
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over='ignore'):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def draw(thr, alias, seed, ids, attempt):
    """Value of draw `ids` at `attempt` (arrays)."""
    with np.errstate(over='ignore'):
        key = np.asarray(ids, dtype=np.uint64) * np.uint64(TRIES) + np.uint64(attempt)
    r = mix64(np.uint64(seed) ^ mix64(key))
    n = np.uint64(len(thr))
    col = (((r >> np.uint64(32)) * n) >> np.uint64(32)).astype(np.int64)
    low = (r & np.uint64(0xFFFFFFFF)).astype(np.uint64)
    return np.where(low < thr[col].astype(np.uint64), col, alias[col].astype(np.int64))


def sample(thr, alias, seed, counter, keys, num, used=None, batch_keys=None):
    """mirec_sample_alias for one call: values in the walk's layout (batch b at
    b*batch_keys*num, slot j*Kb + k)."""
    keys = np.asarray(keys, dtype=np.int64)
    n_keys = len(keys)
    bk = batch_keys or max(n_keys, 1)
    out = np.empty(n_keys * num, dtype=np.int64)
    g = np.arange(n_keys * num)
    b = g // (bk * num)
    k0 = b * bk
    Kb = np.minimum(bk, n_keys - k0)
    s = g - k0 * num
    kk = keys[k0 + s % Kb]
    ids = np.uint64(counter) + g.astype(np.uint64)
    v = draw(thr, alias, seed, ids, 0)
    if used is not None:
        for a in range(1, TRIES):
            bad = np.array([int(x) in used[int(u)] for x, u in zip(v, kk)], dtype=bool)
            if not bad.any():
                break
            v[bad] = draw(thr, alias, seed, ids[bad], a)
    out[:] = v
    return out


def table_mass(thr, alias):
    """Exact probability mass (in units of 2^-32 / n) each value gets from the
    table: column c gives thr[c] units to c and 2^32 - thr[c] to alias[c]."""
    n = len(thr)
    mass = np.zeros(n, dtype=np.float64)
    t = thr.astype(np.float64)
    np.add.at(mass, np.arange(n), t)
    np.add.at(mass, alias.astype(np.int64), 2.0 ** 32 - t)
    return mass
