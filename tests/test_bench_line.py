"""bench.py's multi-rank fields on CPU: two gloo ranks build the line's
"ranks" object (rank_block): the world size, every rank's own step and
exchange time, the communicator count slot; and the emulation value counts
only the walkers a rank evaluates."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, out):
    import sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blk = bench.rank_block(dist, world, "gloo", 1.0 + rank, 0.01 * (rank + 1), (world, rank) if rank == 0 else None,
                           torch.device("cpu"))
    out[rank] = blk
    dist.destroy_process_group()


def test_rank_block_two_gloo_ranks():
    with mp.Manager() as m:
        out = m.dict()
        mp.start_processes(_rank, args=(2, _port(), out), nprocs=2, join=True, start_method="spawn")
        b0, b1 = dict(out[0]), dict(out[1])
    assert b0["world_size"] == 2 and b0["backend"] == "gloo"
    assert b0["rccl_comm_count"] == 2 and b0["rccl_user_rank"] == 0
    assert b0["ms_per_step_per_rank"] == [1.0, 2.0] == b1["ms_per_step_per_rank"]
    assert b0["ms_per_step_min"] == 1.0 and b0["ms_per_step_max"] == 2.0
    np.testing.assert_allclose(b0["exchange_ms_per_half_step"], [0.01, 0.02])


def test_emulation_counts_evaluated_walkers():
    """--emulate-rank K/N holds the whole ensemble but evaluates W / N walkers
    per step: the line's value must count those"""
    import ast
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "value = (W // args.emu[1] if args.emu else W) * args.steps / elapsed" in src
    ast.parse(src)
