"""The per-half-step ln_prob exchange of the sharded sampler, issued straight
into RCCL on the caller's HIP stream.

The reference has no multi-process evaluation at all: emcee maps ln_prob over
a multiprocessing pool on one host (mcmcfit.py:273-288).  Here every rank
evaluates W/(2N) walkers of the half and the ensemble's new ln_prob is
assembled everywhere by one all-gather.  The message is tiny
(W/2 doubles), so the exchange costs its fixed overhead, not bandwidth:
torch's ProcessGroupNCCL runs the collective on its own stream with an event
hand-off each way, ~10 us per call on the device timeline over a plain copy;
ncclAllGather enqueued on the stream the kernels already run on costs ~4 us
(tools/gather_probe.py, one rank).  The communicator is built from the same
librccl torch loaded, from a unique id broadcast over the process group.
"""
import ctypes
import os

NCCL_FLOAT64 = 8  # ncclDouble (rccl.h)


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # NCCL_UNIQUE_ID_BYTES


def uid_bytes(uid):
    """All 128 bytes of an ncclUniqueId (the c_char field stops at a NUL)."""
    return ctypes.string_at(ctypes.addressof(uid), ctypes.sizeof(uid))


def uid_from(b):
    if len(b) != ctypes.sizeof(_UniqueId):
        raise ValueError("ncclUniqueId is %d bytes" % ctypes.sizeof(_UniqueId))
    uid = _UniqueId()
    ctypes.memmove(ctypes.byref(uid), b, len(b))
    return uid


def _load_rccl():
    import torch
    here = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    lib = ctypes.CDLL(here if os.path.exists(here) else "librccl.so")
    lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
    lib.ncclAllGather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p]
    lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
    lib.ncclCommCount.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    lib.ncclCommUserRank.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    return lib


class RcclAllGather:
    """all_gather_into_tensor(out, mine) of float64 device tensors on the
    current stream, over a communicator of the ranks of `group` (built
    collectively by the constructor: every rank must construct it)."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.lib = _load_rccl()
        uid = _UniqueId()
        if self.rank == 0:
            self._check(self.lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        box = [uid_bytes(uid) if self.rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(box, src=src, group=group)
        uid = uid_from(box[0])
        self.comm = ctypes.c_void_p()
        torch.cuda.current_device()  # the rank's device is current (bench/torchrun set it)
        self._check(self.lib.ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank),
                    "ncclCommInitRank")

    def _check(self, r, what):
        if r != 0:
            raise RuntimeError("%s failed: %s" % (what, self.lib.ncclGetErrorString(r).decode()))

    def __call__(self, out, mine):
        import torch
        if mine.dtype != torch.float64 or out.dtype != torch.float64:
            raise TypeError("ln_prob exchange is float64")
        if not (mine.is_contiguous() and out.is_contiguous()) or out.numel() != mine.numel() * self.world:
            raise ValueError("out must hold world x mine contiguous elements")
        self._check(self.lib.ncclAllGather(ctypes.c_void_p(mine.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                           mine.numel(), NCCL_FLOAT64, self.comm,
                                           ctypes.c_void_p(torch.cuda.current_stream(mine.device).cuda_stream)),
                    "ncclAllGather")

    def count(self):
        """(ranks in the communicator, this rank's index) as RCCL reports them
        (ncclCommCount, ncclCommUserRank): bench.py puts them on its line"""
        n, r = ctypes.c_int(), ctypes.c_int()
        self._check(self.lib.ncclCommCount(self.comm, ctypes.byref(n)), "ncclCommCount")
        self._check(self.lib.ncclCommUserRank(self.comm, ctypes.byref(r)), "ncclCommUserRank")
        return n.value, r.value

    def close(self):
        if self.comm:
            self.lib.ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()
