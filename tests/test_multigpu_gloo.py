"""World-size-2 / 3 rehearsal of the point-sharded path on CPU (gloo, 127.0.0.1), through the
library's own multi-GPU contract:

* each rank takes ITS shard from the library (ldso_ba_shard_points, the host-frame partition
  ldso_ba_load applies), restates it with the CPU oracle and packs its partial {HA, bA, Hsc, bsc}
  with the library's packer (ldso_ba_pack_upper: the layout the device reduces);
* the ranks exchange exactly what the in-library RCCL exchange does after k_stitch: one sum
  all-reduce of the packed systems, one of [E, #IN], one all-gather of the newest-frame
  NewEnergyWithOutlier slots (stride = max over ranks, -1 padding), then the library's
  setNewFrameEnergyTH over the gathered values (ldso_ba_frame_threshold, k_frame_th's rule);
* rank 0 unpacks with ldso_ba_unpack_upper; system, energy and threshold must equal the
  unsharded window's.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):  # noqa: C901
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from ldso_amd import dist as ldist
        from ldso_amd import synth

        w = synth.make_window(n_frames=5, n_points=240, width=320, height=240, seed=31)
        mine = ldist.shard_points(w, rank, world)
        sub = ldist.subset_window(w, mine)
        ow = oracle.OracleWindow(sub, threads=0)
        e, s = ow.iteration()
        packed = torch.from_numpy(ldist.pack_upper(s))
        ldist.allreduce_packed(packed, dist)
        energy = torch.tensor([e[0], e[2]], dtype=torch.float64)
        dist.all_reduce(energy)
        # newest-frame slot: this rank's NewEnergyWithOutlier into frame N-1, padded with -1
        r = ow.residuals()
        seg = r["new_energy_wo"][sub.res_target == w.n_frames - 1]
        stride = torch.tensor([len(seg)], dtype=torch.int64)
        dist.all_reduce(stride, op=dist.ReduceOp.MAX)
        slot = torch.full((int(stride),), -1.0, dtype=torch.float32)
        slot[:len(seg)] = torch.from_numpy(seg)
        gathered = [torch.empty_like(slot) for _ in range(world)]
        dist.all_gather(gathered, slot)
        th = ldist.frame_threshold(torch.cat(gathered).numpy())
        if rank == 0:
            full = ldist.unpack_upper(packed.numpy(), 8 * w.n_frames + 4)
            q.put(dict(full=full, energy=energy.numpy(), th=th, n_mine=len(mine), hosts=np.unique(sub.point_host)))
        else:
            q.put(dict(n_mine=len(mine), hosts=np.unique(sub.point_host)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3, 4])
def test_shards_reduce_to_full_window(built, world):
    import oracle
    from ldso_amd import dist as ldist
    from ldso_amd import synth

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    r0 = next(o for o in outs if "full" in o)
    assert sum(o["n_mine"] for o in outs) == 240
    assert sum(len(o["hosts"]) for o in outs) <= 5 + world - 1  # host frames split only at the cuts

    w = synth.make_window(n_frames=5, n_points=240, width=320, height=240, seed=31)
    full = oracle.OracleWindow(w, threads=0)
    e, s = full.iteration()
    for k in ("HA", "bA", "Hsc", "bsc"):
        ref = np.triu(s[k]) + np.triu(s[k], 1).T if s[k].ndim == 2 else s[k]
        assert np.linalg.norm(r0["full"][k] - ref) <= 1e-6 * np.linalg.norm(ref), k
    assert r0["energy"][1] == e[2]
    assert abs(r0["energy"][0] - e[0]) <= 1e-9 * abs(e[0])
    assert r0["th"] == full.frame_energy_th()[-1]


def sharded_optimize(rank, world, cfg, n_its=6, th=1.2, min_its=1, dist_=None):
    """FullSystem::optimize's loop on ONE rank's shard of the window, with the exchange the
    in-library RCCL path does (ldso_ba.hip comm_exchange) and everything else through the library's
    host contract: the rank's run of points (ldso_ba_shard_points) restated by the oracle; per pass
    ONE fp64 sum all-reduce of [packed {HA, bA, Hsc, bsc} | E, #IN] and ONE all-gather of per-rank
    slots [newest-frame NewEnergyWithOutlier values | the rank's |idepth| run, zero-padded] ->
    setNewFrameEnergyTH (ldso_ba_frame_threshold) and doStepFromBackup's sumNID as one float chain
    over the runs in rank order (the unsharded order); every rank solves the reduced system
    redundantly (ldso_ba_solve_system, its own priors), resubstitutes its own points, steps the
    frames (ldso_ba_frame_step) and evaluates canbreak on that sumNID (ldso_ba_step_canbreak).
    world == 1 (dist_ None) is the unsharded loop of the same code.
    -> (energies per pass, iterations entered, status, frame states, sumNID per pass)."""
    import ctypes as C

    import oracle
    from ldso_amd import _lib as L
    from ldso_amd import dist as ldist
    from ldso_amd import synth

    lib = L.lib()
    w = synth.make_window(**cfg)
    N, dim = w.n_frames, w.dim
    ns = w.nullspaces()
    mine = ldist.shard_points(w, rank, world) if world > 1 else np.arange(w.n_points)
    sub = ldist.subset_window(w, mine)
    dev_order = np.argsort(sub.point_host, kind="stable")  # the device's point order: host frame, then caller
    ow = oracle.OracleWindow(sub, threads=0)
    ow.reset_oob()

    def chain(v):  # FullSystem.cc:1899-1909: one float chain, + 0 for padding leaves it as is
        return np.float32(np.cumsum(v, dtype=np.float32)[-1]) if len(v) else np.float32(0)

    def exchange():
        e, sysm = ow.iteration()
        idep = np.abs(sub.point_data[dev_order, 2].astype(np.float32))
        buf = np.concatenate([ldist.pack_upper(sysm), [e[0], e[2]]])
        r = ow.residuals()
        seg = r["new_energy_wo"][sub.res_target == N - 1]
        if dist_ is not None:
            t = torch.from_numpy(buf)
            dist_.all_reduce(t)  # the one all-reduce
            buf = t.numpy()
            m = torch.tensor([len(seg), len(idep)], dtype=torch.int64)
            dist_.all_reduce(m, op=dist_.ReduceOp.MAX)  # once per load in the library
            stride, prun = int(m[0]), (int(m[1]) + 3) // 4 * 4
            slot = torch.full((stride + prun,), -1.0, dtype=torch.float32)
            slot[:len(seg)] = torch.from_numpy(seg)
            slot[stride:] = 0.0
            slot[stride:stride + len(idep)] = torch.from_numpy(idep)
            gathered = [torch.empty_like(slot) for _ in range(world)]
            dist_.all_gather(gathered, slot)  # the one all-gather
            th_new = ldist.frame_threshold(torch.cat([g[:stride] for g in gathered]).numpy())
            nid = chain(torch.cat([g[stride:] for g in gathered]).numpy())
        else:
            th_new = ldist.frame_threshold(seg)
            nid = chain(idep)
        red = ldist.unpack_upper(buf[:-2], dim)
        red["HL"], red["bL"] = sysm["HL"], sysm["bL"]
        return red, buf[-2:], nid, np.float32(w.n_points), th_new

    red, en, snid, nnid, th_new = exchange()
    energies, snids = [en], [snid]
    frames = np.ascontiguousarray(sub.frames).copy()
    cval = sub.calib.astype(np.float64) * (1.0 / 50.0)
    czero = cval.copy()
    status, its = L.OPT_RAN_ALL, n_its
    for it in range(n_its):
        x = np.zeros(dim)
        p = lambda a: L.ptr(np.ascontiguousarray(a, np.float64), L.f64p)  # noqa: E731
        L.check(lib.ldso_ba_solve_system(None, N, it, 1e-5, p(red["HA"]), p(red["bA"]), p(red["HL"]), p(red["bL"]),
                                         L.ptr(None, L.f64p), L.ptr(None, L.f64p), p(red["Hsc"]), p(red["bsc"]),
                                         p(ns), 7, L.ptr(x, L.f64p)))
        if np.isnan(np.linalg.norm(x)):
            status, its = L.OPT_LOST, it + 1
            break
        step = ow.resubstitute(x, 1e-5)
        cb = C.c_int32()
        L.check(lib.ldso_ba_step_canbreak(N, L.ptr(x, L.f64p), float(snid), float(nnid), float(th), C.byref(cb)))
        out = np.zeros_like(frames)
        sf = np.zeros(4, np.float32)
        cd = np.zeros(4, np.float32)
        L.check(lib.ldso_ba_frame_step(N, frames.ctypes.data, L.ptr(x, L.f64p), out.ctypes.data, L.ptr(cval, L.f64p),
                                       L.ptr(czero, L.f64p), L.ptr(sf, L.f32p), L.ptr(cd, L.f32p)))
        frames = out
        idepth = (sub.point_data[:, 2] + step).astype(np.float32)
        sub.frames = frames
        sub.calib = sf.copy()
        sub.c_delta = cd.copy()
        sub.point_data = sub.point_data.copy()
        sub.point_data[:, 2] = idepth
        sub.point_data[:, 3] = idepth
        sub.point_data[:, 5] = 0
        sub.frame_energy_th = ow.frame_energy_th().copy()
        sub.frame_energy_th[N - 1] = th_new  # the exchanged setNewFrameEnergyTH
        sub.refresh_frame_terms()
        ow.update(sub)
        red, en, snid, nnid, th_new = exchange()
        energies.append(en)
        snids.append(snid)
        if cb.value and it >= min_its:
            status, its = L.OPT_CONVERGED, it + 1
            break
    return np.array(energies), its, status, frames, np.array(snids)


def _opt_worker(rank, world, port, q, cfgs):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = [sharded_optimize(rank, world, c, dist_=dist) for c in cfgs]
        q.put((rank, [(e, its, st, fr["state"], nid) for e, its, st, fr, nid in res]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_optimize_loop_matches_unsharded(built, world):
    """The whole sharded GN loop (shard, pass, one all-reduce + one all-gather, redundant solve,
    shard-local resubstitution, step, canbreak on the sumNID chain over the gathered runs) over gloo
    at world 2, 3 and 4: every rank leaves the loop at the same iteration with the same status as the
    unsharded loop, energies within 1e-5 (the ranks' float partials only reassociate), #IN equal,
    frame states within 5 % of the unsharded loop's total step; the first pass's sumNID (same
    idepths on both sides) bit-exact."""
    from ldso_amd import synth
    from test_optimize import CONVERGES, RUNS_ALL

    cfgs = [CONVERGES, RUNS_ALL]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_opt_worker, args=(r, world, port, q, cfgs)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=540) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for i, c in enumerate(cfgs):
        e1, its1, st1, fr1, nid1 = sharded_optimize(0, 1, c)
        print(f"{c}: unsharded {its1} its status {st1}; sharded {[outs[r][i][1:3] for r in range(world)]}")
        for r in range(world):
            e2, its2, st2, s2, nid2 = outs[r][i]
            assert nid2[0] == nid1[0]  # the unsharded chain, bit for bit
            # later passes chain idepths the (reassociated) solves moved apart
            np.testing.assert_allclose(nid2, nid1, rtol=1e-4)
            assert (its2, st2) == (its1, st1), (r, i)
            np.testing.assert_allclose(e2[:, 0], e1[:, 0], rtol=1e-5)
            np.testing.assert_array_equal(e2[:, 1], e1[:, 1])
            # the states: the solve amplifies the reassociation by the system's conditioning, so
            # (as tests/test_optimize.py's loop check) within 5 % of the whole step's norm
            s0 = synth.make_window(**c).frames["state"]
            assert np.linalg.norm(s2 - fr1["state"]) <= 0.05 * np.linalg.norm(fr1["state"] - s0)
    assert outs[0][0][2] == 1 and outs[0][1][2] == 0  # one window converges, the other runs all 6


def test_shard_rule_partitions_points(built):
    """ldso_ba_shard_points: every point exactly once, contiguous runs of the host-frame order,
    residual counts balanced to within one point's residuals, hosts split only at the cuts."""
    from ldso_amd import dist as ldist
    from ldso_amd import synth

    w = synth.make_window(n_frames=5, n_points=300, width=160, height=120, seed=9)
    nres = np.diff(w.point_res_begin)
    order = np.argsort(w.point_host, kind="stable")
    for world in (1, 2, 3, 5, 7, 16):
        parts = [ldist.shard_points(w, r, world) for r in range(world)]
        allp = np.sort(np.concatenate(parts))
        np.testing.assert_array_equal(allp, np.arange(w.n_points))
        pos = np.empty(w.n_points, np.int64)
        pos[order] = np.arange(w.n_points)
        for p in parts:  # a contiguous run of the host-frame order
            if len(p):
                q = np.sort(pos[p])
                assert q[-1] - q[0] == len(q) - 1
        loads = [int(nres[p].sum()) for p in parts]
        assert max(loads) - min(loads) <= 2 * nres.max()
        assert sum(len(np.unique(w.point_host[p])) for p in parts) <= 5 + world - 1


def test_library_frame_threshold_matches_oracle(built):
    import oracle
    from ldso_amd import dist as ldist
    from ldso_amd import synth

    w = synth.make_window(n_frames=4, n_points=150, width=320, height=240, seed=33)
    ow = oracle.OracleWindow(w, threads=0)
    ow.iteration()
    r = ow.residuals()
    assert ldist.frame_threshold(r["new_energy_wo"][w.res_target == 3]) == ow.frame_energy_th()[-1]
