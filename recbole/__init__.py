"""`recbole` — the drop-in import name.

The reference's entry points import `recbole.*` (run_recbole.py:13
`from recbole.quick_start import run_recbole`, and user code such as
`from recbole.config import Config`, `from recbole.data import create_dataset,
data_preparation`, `from recbole.utils import get_model, get_trainer, init_seed`,
`from recbole.model.general_recommender import BPR`, `from recbole.trainer import
Trainer`, `from recbole.sampler import Sampler`). This package makes every
`recbole.<path>` the SAME module object as `recbole_amd.<path>` (one class per
name: isinstance checks, plugin lookup by name and pickled enum values agree
between the two spellings), so scripts written against the reference run
unchanged on the MI355X path.
"""
import importlib
import importlib.abc
import importlib.util
import sys

_TARGET = 'recbole_amd'
__version__ = '0.2.1'      # the reference's version (recbole/__init__.py); product: recbole_amd


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target):
        self.target = target

    def create_module(self, spec):
        return importlib.import_module(self.target)

    def exec_module(self, module):       # the target module is already executed
        pass


class _AliasFinder(importlib.abc.MetaPathFinder):
    """recbole.<x> -> recbole_amd.<x> (only names recbole_amd defines)."""

    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(__name__ + '.'):
            return None
        real = _TARGET + fullname[len(__name__):]
        if importlib.util.find_spec(real) is None:
            return None
        mod = importlib.import_module(real)
        is_pkg = hasattr(mod, '__path__')
        return importlib.util.spec_from_loader(fullname, _AliasLoader(real), is_package=is_pkg)


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())
