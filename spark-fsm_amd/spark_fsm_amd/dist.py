"""Multi-rank plumbing for libfsm's sharded SPADE.

libfsm runs one rank per GPU.  Its collectives go either over RCCL (the
production path: rank 0 calls `comm_unique_id()`, the bytes are broadcast by
any channel, every rank passes them to `Engine(..., unique_id=...)`) or over
host callbacks (`TorchHostComm`: any torch.distributed process group, e.g.
gloo).  The host form runs several ranks on one GPU, which is how the sharded
path is tested on a one-GPU box, and drives the CPU tests of the plumbing.
"""
import ctypes
import uuid

import numpy as np

from . import _lib


def comm_unique_id():
    """RCCL unique id (128 bytes) for Engine(unique_id=...), on rank 0."""
    L = _lib.load()
    buf = (ctypes.c_uint8 * 128)()
    _lib.check(L.fsm_comm_unique_id(buf))
    return bytes(buf)


def shard_plan(volumes, nranks):
    """fsm_shard_plan: owner rank of each work unit (largest first, least loaded)."""
    L = _lib.load()
    v = np.ascontiguousarray(volumes, dtype=np.uint64)
    owner = np.zeros(len(v), dtype=np.int32)
    P = ctypes.POINTER
    _lib.check(L.fsm_shard_plan(v.ctypes.data_as(P(ctypes.c_uint64)), len(v), int(nranks),
                                owner.ctypes.data_as(P(ctypes.c_int32))))
    return owner


class TorchHostComm:
    """fsm_host_comm over a torch.distributed process group.

    With a gloo group the host buffers are reduced in place as CPU tensors.
    With an NCCL (= RCCL on ROCm) group they are staged through a tensor on
    `device`, so libfsm's few small collectives (F1 histogram, frequent pairs,
    failure flags, pattern CSRs) run over the same RCCL communicator torch
    already set up for the job."""

    def __init__(self, group=None, device=None, store=None, claims=True):
        """claims: give libfsm the work-stealing counter (fsm_host_comm.fetch_add) over
        `store` (default: the process group's default store, e.g. the TCPStore of an
        env:// rendezvous).  Construct collectively (every rank of `group`), and one
        per Engine: the counter keys are per communicator."""
        import torch.distributed as dist
        self._dist = dist
        self._group = group
        self._device = device
        self._ar = _lib.ALLREDUCE_FN(self._allreduce)
        self._ag = _lib.ALLGATHER_FN(self._allgather)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._store = None
        # a key prefix common to the ranks (rank 0's), so that counters never collide with
        # another communicator's on the same store (collective: every rank, claims or not)
        obj = [uuid.uuid4().hex if self.rank == 0 else None]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(obj, src=src, group=group)
        self._prefix = "fsm-claims/%s/" % obj[0]
        if claims:
            if store is None:
                try:
                    store = dist.distributed_c10d._get_default_store()
                except Exception:  # noqa: BLE001 - no default store: static plan
                    store = None
            self._store = store
        self._fa = _lib.FETCH_ADD_FN(self._fetch_add) if self._store is not None else _lib.FETCH_ADD_FN()
        self.struct = _lib.HostComm(None, self._ar, self._ag, self._fa)

    def _fetch_add(self, user, key, inc):
        try:
            return int(self._store.add(self._prefix + str(int(key)), int(inc))) - int(inc)
        except Exception:  # noqa: BLE001 - must not unwind through C
            return -1

    def _allreduce(self, user, buf, n):
        try:
            import torch
            if n > 0:
                a = np.ctypeslib.as_array(buf, shape=(n,)).view(np.int32)  # u32 sums mod 2^32 == i32 bits
                t = torch.from_numpy(a)  # shares the C buffer: reduced in place
                if self._device is not None:
                    d = t.to(self._device)
                    self._dist.all_reduce(d, group=self._group)
                    t.copy_(d.cpu())
                else:
                    self._dist.all_reduce(t, group=self._group)
            return 0
        except Exception:  # noqa: BLE001 - must not unwind through C
            return 1

    def _allgather(self, user, send, recv, nbytes):
        try:
            import torch
            if nbytes > 0:
                s = torch.from_numpy(np.ctypeslib.as_array(ctypes.cast(send, ctypes.POINTER(ctypes.c_uint8)),
                                                           shape=(nbytes,)).copy())
                dev = self._device if self._device is not None else "cpu"
                s = s.to(dev)
                out = torch.empty(nbytes * self.world, dtype=torch.uint8, device=dev)
                self._dist.all_gather_into_tensor(out, s, group=self._group)
                r = np.ctypeslib.as_array(ctypes.cast(recv, ctypes.POINTER(ctypes.c_uint8)),
                                          shape=(nbytes * self.world,))
                r[:] = out.cpu().numpy()
            return 0
        except Exception:  # noqa: BLE001
            return 1


def selftest(nranks, rank, host_comm=None, unique_id=None, device=0):
    """fsm_comm_selftest: all-reduce + ragged all-gather across the ranks."""
    L = _lib.load()
    o = _lib.Opts()
    o.device, o.nranks, o.rank = device, nranks, rank
    if unique_id is not None:
        ctypes.memmove(o.unique_id, unique_id, 128)
    if host_comm is not None:
        o.host_comm = ctypes.pointer(host_comm.struct)
    _lib.check(L.fsm_comm_selftest(ctypes.byref(o)))


def selftest_inproc(ndevices):
    """fsm_comm_selftest of the in-process transport (fsm_opts.ndevices ranks as host
    threads of this process, no GPU): all-reduce, ragged and root-only gathers, the
    work-stealing counter."""
    L = _lib.load()
    o = _lib.Opts()
    o.nranks = 1
    o.ndevices = int(ndevices)
    _lib.check(L.fsm_comm_selftest(ctypes.byref(o)))
