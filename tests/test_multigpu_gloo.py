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
@pytest.mark.parametrize("world", [2, 3])
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
