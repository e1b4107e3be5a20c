"""Multi-GPU sharding of one window's points.

Points are ordered by host frame and dealt round-robin to ranks (ldso_ba_load with
shard_rank / shard_count), so every rank sees every host frame and any number of ranks stays
balanced (including more ranks than keyframes).  Images and frame-pair tables are replicated.
Every H/b term is a sum over points, so the only exchange per GN iteration is ONE all-reduce
(sum, fp64) of the packed upper triangles {HA, bA, Hsc, bsc} of every window
(2 * ((8N+4)(8N+5)/2 + 8N+4) doubles: 30 KB at N=7, 70 KB at N=11).  Priors (HL, bL) are added
once, by rank 0 (the host builds them from the window's priors).  Each rank then solves the
small system redundantly; resubstitution is shard-local.
"""
from __future__ import annotations

import numpy as np


def shard_points(point_host, n_frames, rank, world):
    """Caller point indices owned by `rank` (mirror of ldso_ba_load's rule)."""
    order = [p for f in range(n_frames) for p in np.flatnonzero(np.asarray(point_host) == f)]
    return np.array([p for q, p in enumerate(order) if q % world == rank], dtype=np.int64)


def allreduce_packed(tensor, dist):
    """Sum-reduce a packed-system tensor across ranks (RCCL over xGMI on GPUs, gloo on CPU)."""
    dist.all_reduce(tensor, op=dist.ReduceOp.SUM)
    return tensor


class PackedSystem:
    """Device-side exchange buffer for a BAContext: copy out, all-reduce, copy back."""

    def __init__(self, ctx):
        import torch

        self.ctx = ctx
        _, n, _ = ctx.packed_system()
        self.n = n
        self.buf = torch.empty(n, dtype=torch.float64, device=torch.device("cuda", torch.cuda.current_device()))

    def allreduce(self, dist):
        import torch

        from . import _lib as L

        L.check(self.ctx._lib.ldso_ba_copy_packed(self.ctx._h, self.buf.data_ptr(), self.n, 0))
        allreduce_packed(self.buf, dist)
        torch.cuda.current_stream().synchronize()
        L.check(self.ctx._lib.ldso_ba_copy_packed(self.ctx._h, self.buf.data_ptr(), self.n, 1))
