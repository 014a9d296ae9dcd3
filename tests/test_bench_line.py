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
    import sys
    sys.path.insert(0, ROOT)
    import bench
    # config 4 rehearsed as rank 0 of 8: 16 384 walkers held, 2 048 evaluated per step
    assert bench.line_value(16384, 20, 0.5, (0, 8)) == pytest.approx(2048 * 20 / 0.5)
    assert bench.line_value(16384, 20, 0.5, (7, 8)) == pytest.approx(2048 * 20 / 0.5)
    # no emulation: every walker of the ensemble, once per step
    assert bench.line_value(1024, 100, 0.01) == pytest.approx(1024 * 100 / 0.01)
    assert bench.line_value(2048, 10, 1.0, (1, 2)) == pytest.approx(1024 * 10)
    # the CLI parses K/N into the tuple line_value takes
    args = bench.parse(["--config", "4", "--emulate-rank", "3/8", "--steps", "7"])
    assert args.emu == (3, 8) and args.exchange_path
    assert bench.walker_count(args, 1) == 16384      # the whole ensemble is held
    assert bench.line_value(bench.walker_count(args, 1), args.steps, 2.0, args.emu) == pytest.approx(2048 * 7 / 2.0)
