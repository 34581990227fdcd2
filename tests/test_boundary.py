"""The C-ABI boundary: libmirec.so loads and exports every symbol that
include/mirec.h declares (no compute calls — runs without a GPU); the product
package never imports the oracle."""
import ast
import os
import re
import subprocess

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, 'include', 'mirec.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(mirec_[a-z0-9_]+)\s*\(', src)))


def test_header_declares_entry_points():
    names = _declared()
    assert 'mirec_sample_walk' in names and 'mirec_fullsort_topk_f32' in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    from recbole_amd import _native
    lib = _native.lib()                      # loads; raises if missing
    out = subprocess.check_output(['nm', '-D', '--defined-only', _native.LIB_PATH]).decode()
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for name in _declared():
        assert name in exported, name
        assert hasattr(lib, name)
    assert set(_native.SIGNATURES) == set(_declared())
    assert lib.mirec_abi_version() == _native.ABI_VERSION


def test_library_is_gfx950_code():
    from recbole_amd import _native
    blob = open(_native.LIB_PATH, 'rb').read()
    assert b'amdgcn-amd-amdhsa--gfx950' in blob
    # no other GPU target is bundled (gfx950 only, no multi-arch fallbacks)
    import re as _re
    targets = set(_re.findall(rb'amdgcn-amd-amdhsa--(gfx[0-9a-z]+)', blob))
    assert targets == {b'gfx950'}


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, 'recbole_amd')
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if not f.endswith('.py'):
                continue
            tree = ast.parse(open(os.path.join(dirpath, f)).read())
            for node in ast.walk(tree):
                if isinstance(node, ast.Import):
                    assert not any(a.name.split('.')[0] == 'oracle' for a in node.names), f
                elif isinstance(node, ast.ImportFrom):
                    assert (node.module or '').split('.')[0] != 'oracle', f


def test_ops_refuse_cpu_tensors():
    import pytest
    import torch
    from recbole_amd import ops
    from recbole_amd._native import NativeError
    with pytest.raises(NativeError):
        ops.gather_rows(torch.zeros(4, 4), torch.zeros(2, dtype=torch.int64))
    with pytest.raises(NativeError):
        ops.dot_rows(torch.zeros(4, 64), torch.zeros(4, 64), torch.zeros(2, dtype=torch.int64),
                     torch.zeros(2, dtype=torch.int64))
