"""Where the IPC owner-Adam time goes (one rank under torchrun, exchange='ipc', the bench's
driver window): variants of ShardedBPRTrainStep._adam_ipc, timed by bench.py's per-launch
HIP events.
  ipc      the product launch (adam_xchg: backward wait + deferred Adam + next-step push)
  nopush   the same launch without the push lists
  plain    mirec_adam_deferred_f32 reading the contribution rows in the (uncached) window
  cached   the window's backward region copied to a cached buffer first ('copyB'), then
           mirec_adam_deferred_f32 on the copy
One rank: no peer waits; the variants other than 'ipc' leave the next step's rows stale
(timing only).

usage: torchrun --nproc-per-node 1 tools/probe_ipc_adam.py VARIANT [bench args]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ['MIREC_EXCHANGE'] = 'ipc'

import torch  # noqa: E402

import bench  # noqa: E402
from recbole_amd._native import check, lib  # noqa: E402
from recbole_amd.trainer import fused  # noqa: E402

variant = sys.argv[1]
S = fused.ShardedBPRTrainStep
orig = S._adam_ipc
hip = ctypes.CDLL('libamdhip64.so')
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_void_p]


def patched(self, slot, c, Bc, stream, step_off, ahead):
    if variant == 'ipc':
        return orig(self, slot, c, Bc, stream, step_off, ahead)
    if variant == 'nopush':
        return orig(self, slot, c, Bc, stream, step_off, False)
    t = self._tables
    st = stream.cuda_stream
    if variant == 'cached':
        if not hasattr(self, '_probe_buf'):
            self._probe_buf = torch.empty(self.G * self.cap, self.d, device=self.device)
        n = self._probe_buf.numel() * 4
        self._record('copyB', stream, lambda: hip.hipMemcpyAsync(
            self._probe_buf.data_ptr(), self.win.bwd, n, 3, st))
        for q in range(2):
            t[q].rows = self._probe_buf.data_ptr()

    def adam():
        check(lib().mirec_adam_deferred_f32(t, 2, self._n_max, self.d, self.consts.data_ptr(),
                                            self.step_idx.data_ptr(), step_off,
                                            *self._adam_args, st), 'mirec_adam_deferred_f32')
    self._record('adam', stream, adam)


S._adam_ipc = patched
sys.argv = ['bench.py', '--gpus', '1', '--dp-mode', 'sharded'] + sys.argv[2:]
bench.main()
