"""GPU: the sharded sampler's ln_prob exchange issued directly into RCCL on
the compute stream (lfit_python_amd.comm), on a one-rank communicator (the
box has one GPU; the multi-rank logic is covered by the gloo tests and runs
at N > 1 in the driver's scaling bench)."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def nccl_world1():
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        yield dev
    finally:
        dist.destroy_process_group()


def test_rccl_allgather_on_current_stream(nccl_world1):
    import torch
    from lfit_python_amd.comm import RcclAllGather
    g = RcclAllGather()
    try:
        mine = torch.arange(512, dtype=torch.float64, device=nccl_world1) * 0.5 - 3.0
        out = torch.full((512,), float("nan"), dtype=torch.float64, device=nccl_world1)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):  # enqueued on whatever stream is current
            mine.mul_(2.0)
            g(out, mine)
        s.synchronize()
        assert torch.equal(out, mine)
        with pytest.raises(ValueError):
            g(out[:100], mine)
        with pytest.raises(TypeError):
            g(out.float(), mine.float())
    finally:
        g.close()


def test_sampler_exchange_uses_direct_rccl(nccl_world1):
    import torch
    from lfit_python_amd.comm import RcclAllGather
    from lfit_python_amd.sampler import EnsembleSampler

    class Ev:
        device = nccl_world1

        def __call__(self, x, out=None):
            return -0.5 * (x * x).sum(1)

    S = EnsembleSampler(8, 2, Ev())
    mine = torch.linspace(-1, 1, 4, dtype=torch.float64, device=nccl_world1)
    out = torch.empty(4, dtype=torch.float64, device=nccl_world1)
    S._gather(out, mine)
    torch.cuda.synchronize()
    assert isinstance(S._rccl, RcclAllGather)
    assert torch.equal(out, mine)
    S.close()
    assert S._rccl is None
