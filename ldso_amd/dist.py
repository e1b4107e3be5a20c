"""Multi-GPU sharding of one window's points.

Points are ordered by host frame and dealt round-robin to ranks (ldso_ba_load with
shard_rank / shard_count), so every rank sees every host frame and any number of ranks stays
balanced (including more ranks than keyframes).  Images and frame-pair tables are replicated.
Every H/b term is a sum over points, so the only exchange per GN iteration is ONE all-reduce
(sum, fp64) of the packed upper triangles {HA, bA, Hsc, bsc} of every window
(2 * ((8N+4)(8N+5)/2 + 8N+4) doubles: 30 KB at N=7, 70 KB at N=11).  Priors (HL, bL) are added
once, by rank 0 (the host builds them from the window's priors).  Each rank then solves the
small system redundantly; resubstitution is shard-local.

The newest frame's energy threshold (setNewFrameEnergyTH, an nth_element over all residuals
into the newest frame) is the one non-additive quantity: each rank exports its newest-frame
NewEnergyWithOutlier segment, one all-gather (fixed slot size, set at load) brings every
rank's values everywhere, and every rank re-selects the same exact threshold on the device.
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


def subset_window(window, points):
    """A Window holding only `points` (caller indices, any order) and their residuals; frame
    data is shared.  Used to restate a rank's shard on the CPU in tests."""
    import copy

    points = np.asarray(points, dtype=np.int64)
    b, e = window.point_res_begin[points], window.point_res_begin[points + 1]
    res = np.concatenate([np.arange(x, y) for x, y in zip(b, e)]) if len(points) else np.zeros(0, np.int64)
    w = copy.copy(window)
    w.point_host = window.point_host[points].copy()
    w.point_data = window.point_data[points].copy()
    w.point_res_begin = np.concatenate([[0], np.cumsum(e - b)]).astype(np.int32)
    for k in ("res_target", "res_state", "res_energy", "res_flags"):
        setattr(w, k, getattr(window, k)[res].copy())
    w._keep = []
    return w


def packed_upper(sysm):
    """{HA, bA, Hsc, bsc} of one window as ldso_ba's packed layout (upper triangles, row-major)."""
    iu = np.triu_indices(sysm["HA"].shape[0])
    return np.concatenate([sysm["HA"][iu], sysm["bA"], sysm["Hsc"][iu], sysm["bsc"]])


def frame_threshold(values):
    """setNewFrameEnergyTH (FullSystem.cc:2078-2109) over NewEnergyWithOutlier values (host
    restatement for tests; the product selects on the device, ldso_ba_frame_threshold_gathered)."""
    v = np.asarray(values, np.float32)
    v = v[v >= 0]
    if v.size == 0:
        return np.float32(12 * 12 * 8)
    nth = int(np.float32(0.7) * np.float32(v.size))
    x = np.float32(np.sqrt(np.partition(v, nth)[nth]))
    th = np.float32(26.0 * 0.5) + (x * np.float32(1.5)) * np.float32(0.5)
    return np.float32(th * th)


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


class NewestThreshold:
    """All-gather of the newest-frame energies + device re-selection of the frame threshold."""

    def __init__(self, ctx, dist):
        import ctypes as C

        import torch

        from . import _lib as L

        self.ctx, self.dist = ctx, dist
        s = C.c_int64()
        L.check(ctx._lib.ldso_ba_newest_stride(ctx._h, C.byref(s)))
        dev = torch.device("cuda", torch.cuda.current_device())
        t = torch.tensor([max(1, s.value)], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        self.stride = int(t.item())
        self.world = dist.get_world_size()
        nw = len(ctx.windows)
        self.local = torch.empty(nw * self.stride, dtype=torch.float32, device=dev)
        self.gathered = torch.empty(self.world * nw * self.stride, dtype=torch.float32, device=dev)

    def exchange(self):
        import torch

        from . import _lib as L

        L.check(self.ctx._lib.ldso_ba_export_newest(self.ctx._h, self.local.data_ptr(), self.stride))
        self.dist.all_gather_into_tensor(self.gathered, self.local)
        torch.cuda.current_stream().synchronize()
        L.check(self.ctx._lib.ldso_ba_frame_threshold_gathered(self.ctx._h, self.gathered.data_ptr(), self.world,
                                                               self.stride))


class ShardExchange:
    """Per-GN-iteration exchange of a point-sharded context: one fp64 all-reduce of the
    packed systems and one all-gather of the newest-frame energies."""

    def __init__(self, ctx, dist):
        self.packed = PackedSystem(ctx)
        self.th = NewestThreshold(ctx, dist)
        self.dist = dist

    def __call__(self):
        self.packed.allreduce(self.dist)
        self.th.exchange()
