"""recbole_amd — MI355X (gfx950) native drop-in for ghazalehnt/RecBole's
embedding-lookup + negative-sampling train loop and full-sort evaluator.

Module layout mirrors the reference's public API (config, data, sampler,
model, trainer, evaluator, utils, quick_start); the arithmetic of the hot path
lives in libmirec.so (recbole_amd/csrc, C-ABI in include/mirec.h).
"""
__version__ = '0.1.0'
