import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def free_port():
    """A TCP port the OS reports free on 127.0.0.1 (rendezvous of multi-rank tests;
    pid-derived ports collided with sockets left in TIME_WAIT by earlier tests)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP kernels)')


@pytest.fixture(scope='session')
def dev():
    import torch
    assert torch.cuda.is_available(), 'gpu tests need a GPU'
    return torch.device('cuda', 0)
