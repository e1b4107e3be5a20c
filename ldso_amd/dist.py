"""Multi-GPU sharding of one window's points.

Points are sharded by host frame (ldso_ba_load(rank, world) / ldso_ba_shard_points): in
host-frame order the points are cut into `world` contiguous runs of equal residual counts, so a
rank holds whole host frames except where a cut falls inside one.  Images and frame-pair tables
are replicated.  Every H/b term is a sum over points, so the exchange per GN iteration is ONE
fp64 sum all-reduce of the packed upper triangles {HA, bA, Hsc, bsc} of every window
(2 * ((8N+4)(8N+5)/2 + 8N+4) doubles: 30 KB at N=7, 70 KB at N=11), one of the energy / #IN
pairs, and one all-gather of the newest frame's NewEnergyWithOutlier slots after which every
rank re-selects the exact setNewFrameEnergyTH threshold (nth_element is not additive).  The
priors (HL, bL) are not part of the reduced system: every rank adds them in its own solve, which
it runs redundantly on the reduced system; resubstitution is shard-local.

The product runs this exchange itself over RCCL, stream-ordered inside ldso_ba_linearize, once
the context is attached to a communicator (attach_rccl: ldso_ba_comm_unique_id on rank 0, the
id handed to the other ranks, ldso_ba_comm_init).  torch.distributed only carries the 128-byte
id.  The gloo test (tests/test_multigpu_gloo.py) rehearses the same contract on CPU through the
library's host entry points (shard_points, pack_upper / unpack_upper, frame_threshold).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def shard_points(window, rank, world):
    """Caller point indices ldso_ba_load keeps on `rank` (the library's own partition)."""
    s = window.c_struct(with_images=False)
    out = np.zeros(window.n_points, np.int32)
    n = C.c_int32()
    L.check(L.lib().ldso_ba_shard_points(C.byref(s), int(rank), int(world), L.ptr(out, L.i32p), C.byref(n)))
    window._keep = []
    return out[: n.value].astype(np.int64)


def pack_upper(sysm):
    """{HA, bA, Hsc, bsc} of one window in the packed layout the ranks reduce (ldso_ba_pack_upper)."""
    d = sysm["HA"].shape[0]
    out = np.zeros(d * (d + 1) + 2 * d, np.float64)
    a = {k: np.ascontiguousarray(sysm[k], np.float64) for k in ("HA", "bA", "Hsc", "bsc")}
    L.check(L.lib().ldso_ba_pack_upper(d, L.ptr(a["HA"], L.f64p), L.ptr(a["bA"], L.f64p), L.ptr(a["Hsc"], L.f64p),
                                       L.ptr(a["bsc"], L.f64p), L.ptr(out, L.f64p)))
    return out


def unpack_upper(packed, dim):
    o = {"HA": np.zeros((dim, dim)), "bA": np.zeros(dim), "Hsc": np.zeros((dim, dim)), "bsc": np.zeros(dim)}
    p = np.ascontiguousarray(packed, np.float64)
    L.check(L.lib().ldso_ba_unpack_upper(dim, L.ptr(p, L.f64p), L.ptr(o["HA"], L.f64p), L.ptr(o["bA"], L.f64p),
                                         L.ptr(o["Hsc"], L.f64p), L.ptr(o["bsc"], L.f64p)))
    return o


def frame_threshold(values):
    """setNewFrameEnergyTH over gathered NewEnergyWithOutlier values (ldso_ba_frame_threshold)."""
    v = np.ascontiguousarray(values, np.float32)
    out = np.zeros(1, np.float32)
    L.check(L.lib().ldso_ba_frame_threshold(L.ptr(v, L.f32p), v.size, L.ptr(out, L.f32p)))
    return out[0]


def attach_rccl(ctx, dist):
    """Attach `ctx` to an RCCL communicator over the torch.distributed group's ranks (which only
    carry the 128-byte id); from then on ldso_ba_linearize ends with the in-library exchange."""
    rank, world = dist.get_rank(), dist.get_world_size()
    uid = np.zeros(128, np.uint8)
    if rank == 0:
        L.check(L.lib().ldso_ba_comm_unique_id(uid.ctypes.data))
    box = [bytes(uid)]
    dist.broadcast_object_list(box, src=0)
    uid = np.frombuffer(box[0], np.uint8).copy()
    L.check(L.lib().ldso_ba_comm_init(ctx._h, uid.ctypes.data, rank, world))
    return ctx


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
    # each kept point keeps its features rank (the library orders a host's points by rank, so the
    # subset's order is the original's restricted to it)
    w.point_rank = None if window.point_rank is None else np.asarray(window.point_rank)[points].copy()
    w._keep = []
    return w
