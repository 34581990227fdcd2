from recbole_amd.sampler.sampler import AbstractSampler, RepeatableSampler, Sampler

__all__ = ['AbstractSampler', 'Sampler', 'RepeatableSampler']
