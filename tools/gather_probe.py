"""Diagnostic: cost of the per-half-step ln_prob exchange on the caller's
stream.  One rank (world 1, NCCL = RCCL), a dependent chain per iteration:
tiny kernel -> exchange -> tiny kernel, timed over many iterations for
  copy   : a device copy in place of the exchange (the one-rank shard path)
  torch  : dist.all_gather_into_tensor (ProcessGroupNCCL, its own stream hand-off)
  rccl   : ncclAllGather from librccl called directly on the current stream
The differences are the exchange's fixed cost per call (the multi-GPU
scaling loss per half-step, apart from the xGMI transfer itself)."""
import ctypes
import os
import time

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)

n = 512
x = torch.zeros(n, dtype=torch.float64, device=dev)
out = torch.zeros(n, dtype=torch.float64, device=dev)
big = torch.zeros(1 << 22, dtype=torch.float64, device=dev)  # ~10 us of HBM work: GPU-bound loop

R = ctypes.CDLL("librccl.so")


class UID(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


uid = UID()
assert R.ncclGetUniqueId(ctypes.byref(uid)) == 0
comm = ctypes.c_void_p()
R.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, UID, ctypes.c_int]
assert R.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0
R.ncclAllGather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                            ctypes.c_void_p]


def ex_copy():
    out.copy_(x)


def ex_torch():
    dist.all_gather_into_tensor(out, x)


def ex_rccl():
    r = R.ncclAllGather(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()), n, 8, comm,
                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert r == 0


def run(fn, iters, work):
    for _ in range(20):
        x.add_(1.0)
        fn()
        out.add_(1.0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        for _ in range(work):
            big.add_(1.0)
        x.add_(1.0)
        fn()
        out.add_(1.0)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


# work = 0: host-bound (launch cost); work = 4: GPU-bound (the exchange's
# cost on the device timeline)
for work in (0, 4, 4):
    for name, fn in (("copy", ex_copy), ("torch", ex_torch), ("rccl", ex_rccl)):
        print("work %d %-6s %7.2f us / iteration" % (work, name, run(fn, 1000, work)), flush=True)
ex_rccl()
torch.cuda.synchronize()
assert torch.equal(out, x)  # the exchange delivered
R.ncclCommDestroy(comm)
dist.destroy_process_group()
