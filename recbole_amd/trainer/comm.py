"""Host side of the cross-GPU exchange (csrc/comm.hip, include/mirec.h mirec_comm_*):
every rank's receive window mapped into every other rank through HIP IPC over xGMI,
the row-sharded step's two exchanges per step done by kernels storing into the peers'
windows (flag hand-off on the GPU) instead of RCCL all-to-alls.

PeerWindows(group, wcap, d) builds the communicator: this rank's window, its IPC handle
shared with the other ranks through the process group (all_gather_object: host
bytes, any backend), the peers' windows opened. Every rank of the group must construct
it at the same point (the handle exchange is a collective). close() frees the window
after a barrier (no rank may still store into it)."""
from __future__ import annotations

import ctypes
import os

import torch

from recbole_amd._native import NativeError, check, lib


def _device_id(device):
    """A physical identity of the device (its UUID; the PCI location as a fallback)."""
    p = torch.cuda.get_device_properties(device)
    u = getattr(p, 'uuid', None)
    if u is not None:
        return str(u)
    return f"{getattr(p, 'pci_domain_id', 0)}:{getattr(p, 'pci_bus_id', 0)}:" \
           f"{getattr(p, 'pci_device_id', 0)}"


class PeerWindows(object):

    def __init__(self, group, wcap, d, device):
        import torch.distributed as tdist
        self.group = group
        self.rank = tdist.get_rank(group)
        self.world = tdist.get_world_size(group)
        self.wcap, self.d, self.device = int(wcap), int(d), device
        L = lib()
        # the job's token: the same bytes on every rank (from rank 0)
        tok = [os.urandom(64) if self.rank == 0 else None]
        tdist.broadcast_object_list(tok, src=0, group=group)
        token = ctypes.create_string_buffer(tok[0], 64)
        self._comm = ctypes.c_void_p()
        check(L.mirec_comm_init(self.rank, self.world, token, ctypes.byref(self._comm)),
              'mirec_comm_init')
        hb = int(L.mirec_comm_handle_bytes())
        handle = ctypes.create_string_buffer(hb)
        local = ctypes.c_void_p()
        with torch.cuda.device(device):
            check(L.mirec_comm_window(self._comm, self.wcap, self.d, ctypes.byref(local), handle),
                  'mirec_comm_window')
        handles = [None] * self.world
        tdist.all_gather_object(handles, handle.raw, group=group)
        allh = ctypes.create_string_buffer(b''.join(handles), hb * self.world)
        with torch.cuda.device(device):
            check(L.mirec_comm_connect(self._comm, allh), 'mirec_comm_connect')
        # ranks sharing a device (tests on one GPU): a one-block wait ahead of each step
        # launch, so the launch's blocks never spin on compute units a peer needs
        ids = [None] * self.world
        tdist.all_gather_object(ids, _device_id(device), group=group)
        self.shared_device = ids.count(ids[self.rank]) > 1
        check(L.mirec_comm_config(self._comm, 1 if self.shared_device else 0),
              'mirec_comm_config')
        fo, bo = ctypes.c_int64(), ctypes.c_int64()
        status = ctypes.c_void_p()
        check(L.mirec_comm_layout(self._comm, ctypes.byref(fo), ctypes.byref(bo),
                                  ctypes.byref(status)), 'mirec_comm_layout')
        self.base = local.value
        self.fwd = self.base + fo.value           # this rank's forward region (device ptr)
        self.bwd = self.base + bo.value           # this rank's backward region
        self._status = status.value

    @property
    def comm(self):
        return self._comm

    def status(self):
        """0, or -5 when a wait gave up on a peer since the last read (a host read after
        the device's work; the library clears the word)."""
        torch.cuda.synchronize(self.device)
        out = ctypes.c_int32(0)
        check(lib().mirec_comm_status(self._comm, ctypes.byref(out)), 'mirec_comm_status')
        return int(out.value)

    def close(self):
        if self._comm is None:
            return
        import torch.distributed as tdist
        torch.cuda.synchronize(self.device)
        tdist.barrier(group=self.group)          # no rank stores into a freed window
        lib().mirec_comm_destroy(self._comm)
        self._comm = None

    def __del__(self):
        if getattr(self, '_comm', None) is not None:
            try:
                lib().mirec_comm_destroy(self._comm)
            except (NativeError, OSError):
                pass
            self._comm = None
