"""Diagnostic: do hipEvents recorded inside a captured HIP graph give
elapsed times after replay?  Prints the raw HIP status codes."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda", 0)
x = torch.zeros(1 << 20, device=dev)


def ev(flags=0):
    h = ctypes.c_void_p()
    rc = hip.hipEventCreateWithFlags(ctypes.byref(h), flags)
    assert rc == 0, rc
    return h


for flags in (0, 2):  # hipEventDefault, hipEventBlockingSync
    e0, e1 = ev(flags), ev(flags)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        print("record e0 during capture:", hip.hipEventRecord(e0, s))
        x.mul_(1.0001)
        x.add_(1.0)
        print("record e1 during capture:", hip.hipEventRecord(e1, s))
    g.replay()
    torch.cuda.synchronize()
    ms = ctypes.c_float()
    print("flags", flags, "query e0", hip.hipEventQuery(e0), "query e1", hip.hipEventQuery(e1),
          "elapsed rc", hip.hipEventElapsedTime(ctypes.byref(ms), e0, e1), "ms", ms.value)
    # events recorded on the stream around the replay, for comparison
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    a, b = ev(0), ev(0)
    hip.hipEventRecord(a, s)
    g.replay()
    hip.hipEventRecord(b, s)
    torch.cuda.synchronize()
    print("around replay elapsed rc", hip.hipEventElapsedTime(ctypes.byref(ms), a, b), "ms", ms.value)
