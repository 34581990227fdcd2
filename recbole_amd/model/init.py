"""Parameter initialisation (mirror of recbole/model/init.py:15-50). Runs on the
CPU generator at model construction, in module-registration order, so the
torch RNG stream matches the reference before the weights move to HBM."""
import torch.nn as nn
from torch.nn.init import constant_, xavier_normal_, xavier_uniform_


def xavier_normal_initialization(module):
    if isinstance(module, nn.Embedding):
        xavier_normal_(module.weight.data)
    elif isinstance(module, nn.Linear):
        xavier_normal_(module.weight.data)
        if module.bias is not None:
            constant_(module.bias.data, 0)


def xavier_uniform_initialization(module):
    if isinstance(module, nn.Embedding):
        xavier_uniform_(module.weight.data)
    elif isinstance(module, nn.Linear):
        xavier_uniform_(module.weight.data)
        if module.bias is not None:
            constant_(module.bias.data, 0)
