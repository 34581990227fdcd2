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
    config.addinivalue_line('markers', 'slow: full-scale CPU test (minutes, GBs of memory); '
                                       'runs only with MIREC_SLOW_TESTS=1')


def pytest_collection_modifyitems(config, items):
    if os.environ.get('MIREC_SLOW_TESTS') == '1':
        return
    skip = pytest.mark.skip(reason='full-scale test: set MIREC_SLOW_TESTS=1 to run it')
    for item in items:
        if 'slow' in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope='session')
def dev():
    import torch
    assert torch.cuda.is_available(), 'gpu tests need a GPU'
    return torch.device('cuda', 0)
