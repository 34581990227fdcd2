"""numpy restatement of K10's dropout draws (csrc/mlp.hip header) — the
specification the GPU masks are checked against. Test infrastructure only.

Element e (row-major index into layer l's input [B, dims[l]]) of layer l in the
training forward that read counter value c is kept iff
    splitmix64(splitmix64(seed + c) ^ (e * 8 + l)) >> 32  <  keep_threshold
"""
import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over='ignore'):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def keep_mask(seed, counter, layer, B, width, threshold):
    """[B, width] bool keep flags of layer `layer`'s input."""
    with np.errstate(over='ignore'):
        key = splitmix64(np.uint64(seed) + np.uint64(counter))
    e = np.arange(B * width, dtype=np.uint64)
    with np.errstate(over='ignore'):
        u = splitmix64(key ^ (e * np.uint64(8) + np.uint64(layer))) >> np.uint64(32)
    return (u < np.uint64(threshold)).reshape(B, width)
