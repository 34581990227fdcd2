"""Tree guards (CPU): every tracked Python source byte-compiles, no tracked source file is
larger than 1 MB, and the GPU suite collects without errors. A round-end snapshot once
committed a 218 MiB corrupt `recbole_amd/trainer/fused.py` that no check caught; these
run in the CPU suite and before every GPU call (tools/gpu_run.sh)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_SOURCE_BYTES = 1 << 20
SOURCE_EXT = ('.py', '.hip', '.h', '.c', '.cpp', '.sh')      # code (records may be any size)


def _tracked():
    try:
        out = subprocess.run(['git', 'ls-files', '-z'], cwd=ROOT, capture_output=True,
                             check=True).stdout
    except (OSError, subprocess.CalledProcessError):
        pytest.skip('not a git checkout')
    return [p for p in out.decode().split('\0') if p]


def test_tracked_python_compiles():
    bad = []
    for p in _tracked():
        if not p.endswith('.py'):
            continue
        path = os.path.join(ROOT, p)
        if not os.path.exists(path):            # deleted in the work tree, not yet staged
            continue
        with open(path, 'rb') as f:
            src = f.read()
        try:
            compile(src, p, 'exec', dont_inherit=True)
        except SyntaxError as e:
            bad.append(f'{p}:{e.lineno}: {e.msg}')
    assert not bad, 'sources that do not compile:\n' + '\n'.join(bad)


def test_tracked_sources_small():
    big = []
    for p in _tracked():
        path = os.path.join(ROOT, p)
        if p.endswith(SOURCE_EXT) and os.path.exists(path):
            n = os.path.getsize(path)
            if n > MAX_SOURCE_BYTES:
                big.append(f'{p}: {n} bytes')
    assert not big, 'tracked sources over 1 MB:\n' + '\n'.join(big)


def test_product_modules_import():
    """The drop-in surface imports (no GPU needed): trainer, quick start, bench."""
    code = ('import recbole_amd.trainer, recbole_amd.trainer.fused, recbole_amd.quick_start, '
            'recbole.trainer, recbole.quick_start, bench')
    subprocess.run([sys.executable, '-c', code], cwd=ROOT, check=True, timeout=300)


def test_gpu_suite_collects():
    r = subprocess.run([sys.executable, '-m', 'pytest', '--collect-only', '-q', '-m', 'gpu',
                        'tests'], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and 'error' not in r.stdout.lower().splitlines()[-1], \
        r.stdout[-3000:] + r.stderr[-3000:]
