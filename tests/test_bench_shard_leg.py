"""bench.py's sharded-window leg (the N > 1 runs' check of the in-library RCCL exchange, SURVEY.md
§8e) driven with one rank: the leg's phases, timing and parity code run end to end over a
world-1 RCCL communicator, and its reduced system must match the unsharded window's.  With
more ranks on one GPU RCCL refuses the communicator ("duplicate GPU"), which the leg reports
as an error instead of hanging (rehearsed with LDSO_BENCH_SHARE_GPU=1)."""
import os
import socket
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(200)
def test_sharded_window_leg_world1(built):
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import bench

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        out = bench.sharded_window_leg(dist, 0, 1, 0, "cpu", steps=3)
    finally:
        dist.destroy_process_group()
    assert "error" not in out, out
    assert out["points_total"] == 8000
    assert out["ms_per_pass"] > 0 and out["ms_per_pass_unsharded_one_gpu"] > 0
    p = out["parity"]
    assert p["ok"], p
    assert p["max_block_rel_err"] == 0.0  # one rank: the reduced system is the window's own
