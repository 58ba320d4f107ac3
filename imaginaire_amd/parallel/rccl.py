"""Native RCCL communicators (``csrc/rccl_comm.hip``) for the collectives of a captured step.

:class:`NativeComm` mirrors a torch.distributed group with its own RCCL communicator
(bootstrapped once through the group) and runs all-reduce / all-gather directly on the
caller's HIP stream — no torch ``Work`` objects, so nothing for ProcessGroupNCCL's watchdog to
poll, which is what makes a step holding collectives capturable into a hipGraph on this stack
(see the C++ file). Overlap with compute uses a side stream joined by stream waits; under
capture those become graph dependencies.

Enabled by ``IMAGINAIRE_AMD_NATIVE_COMM``: ``1`` always (RCCL groups), ``0`` never, ``auto``
(default) whenever hipGraph capture is not switched off (``IMAGINAIRE_AMD_GRAPH`` != ``0``):
multi-rank training steps are captured by default (utils/cuda_graph.py). A new communicator is
checked once with a rank-sum all-reduce; if that fails on any rank (agreed over the torch
group), every rank falls back to the torch.distributed collectives together.
"""
import os

import torch
import torch.distributed as dist

from imaginaire_amd.ops import _ext

_COMMS = {}


def native_comm_wanted():
    mode = os.environ.get('IMAGINAIRE_AMD_NATIVE_COMM', 'auto')
    if mode == 'auto':
        return os.environ.get('IMAGINAIRE_AMD_GRAPH', '1') != '0'
    return mode == '1'


class _Pending(object):
    """Handle of an async native collective: ``wait()`` joins it into the current stream."""
    __slots__ = ('event',)

    def __init__(self, event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)


class NativeComm(object):
    """A native RCCL communicator over the ranks of ``group`` (None: the world)."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        X = _ext.ext()
        uid = [X.rccl_unique_id().tolist() if self.rank == 0 else None]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(uid, src=src, group=group)
        self.handle = X.rccl_comm_init(torch.tensor(uid[0], dtype=torch.uint8), self.rank,
                                       self.world)
        self._side = None

    def _stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream()
        return self._side

    def all_reduce(self, t, op='sum', async_op=False):
        """In place. ``op``: 'sum' | 'avg' | 'max'. ``async_op``: run on a side stream after
        the work queued so far; returns a handle whose ``wait()`` joins it."""
        if op == 'avg' and self.world == 1:
            # the average over one rank is the sum: RCCL's one-rank PreMulSum path rewrites the
            # whole buffer (~0.3 ms per 256 MB bucket), the in-place sum does not
            op = 'sum'
        code = {'sum': 0, 'avg': 1, 'max': 2}[op]
        if not async_op:
            _ext.ext().rccl_all_reduce(t, self.handle, code)
            return None
        side = self._stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            _ext.ext().rccl_all_reduce(t, self.handle, code)
            ev = torch.cuda.Event()
            ev.record(side)
        t.record_stream(side)
        return _Pending(ev)

    def all_gather(self, out, inp, async_op=False):
        """``out`` [world, *inp.shape] (contiguous) <- every rank's ``inp``."""
        if not async_op:
            _ext.ext().rccl_all_gather(out, inp.contiguous(), self.handle)
            return None
        side = self._stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            _ext.ext().rccl_all_gather(out, inp.contiguous(), self.handle)
            ev = torch.cuda.Event()
            ev.record(side)
        out.record_stream(side)
        inp.record_stream(side)
        return _Pending(ev)


def _verified(group):
    """A new :class:`NativeComm` of ``group`` after a rank-sum all-reduce check, or None on
    every rank if it failed on any (the outcome is agreed over the torch group, so all ranks
    take the same collective path)."""
    comm, ok = None, 1
    try:
        comm = NativeComm(group)
        t = torch.full((4,), float(comm.rank + 1), device='cuda')
        comm.all_reduce(t, 'sum')
        want = comm.world * (comm.world + 1) / 2.0
        ok = int(bool(torch.all(t == want).item()))
    except RuntimeError:
        ok = 0
    flag = torch.tensor([ok], dtype=torch.int32, device='cuda')
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    if int(flag.item()) == 1:
        return comm
    if dist.get_rank() == 0:
        print('[rccl] native communicator check failed; using torch.distributed collectives')
    return None


def native_comm_for(group=None, tag=None):
    """The cached :class:`NativeComm` of ``group`` (one per ``tag``: the DDP wrappers of G and
    D each get their own communicator and side stream) when native collectives are wanted and
    possible (RCCL backend, HIP extension loaded), else None."""
    if not (native_comm_wanted() and dist.is_available() and dist.is_initialized()):
        return None
    if dist.get_backend(group) != 'nccl' or not _ext.available():
        return None
    key = (id(group) if group is not None else None, tag)
    if key not in _COMMS:
        _COMMS[key] = _verified(group)
    return _COMMS[key]
