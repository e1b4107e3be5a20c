"""World-size-2 rehearsal of the point-sharded path on CPU (gloo, 127.0.0.1).

Each rank restates its shard (ldso_amd.dist.shard_points: points ordered by host frame and
dealt round-robin, the rule ldso_ba_load applies) with the CPU oracle, packs its partial
{HA, bA, Hsc, bsc} the way the device does, and the ranks exchange exactly what the GPU path
exchanges: one all-reduce of the packed systems and one all-gather of the newest-frame energy
slots (fixed stride = max over ranks, -1 padding).  The reduced system and the re-selected
threshold must equal the unsharded window's.
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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from ldso_amd import dist as ldist
        from ldso_amd import synth

        w = synth.make_window(n_frames=5, n_points=240, width=320, height=240, seed=31)
        mine = ldist.shard_points(w.point_host, w.n_frames, rank, world)
        sub = ldist.subset_window(w, mine)
        ow = oracle.OracleWindow(sub, threads=0)
        e, s = ow.iteration()
        packed = torch.from_numpy(ldist.packed_upper(s))
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
            q.put(dict(packed=packed.numpy(), energy=energy.numpy(), th=th, n_mine=len(mine)))
        else:
            q.put(dict(n_mine=len(mine)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_shards_reduce_to_full_window(built):
    import oracle
    from ldso_amd import dist as ldist
    from ldso_amd import synth

    world = 2
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
    r0 = next(o for o in outs if "packed" in o)
    assert sum(o["n_mine"] for o in outs) == 240

    w = synth.make_window(n_frames=5, n_points=240, width=320, height=240, seed=31)
    full = oracle.OracleWindow(w, threads=0)
    e, s = full.iteration()
    ref = ldist.packed_upper(s)
    assert np.linalg.norm(r0["packed"] - ref) <= 1e-6 * np.linalg.norm(ref)
    assert r0["energy"][1] == e[2]
    assert abs(r0["energy"][0] - e[0]) <= 1e-9 * abs(e[0])
    assert r0["th"] == full.frame_energy_th()[-1]


def test_shard_rule_partitions_points(built):
    from ldso_amd import dist as ldist

    host = np.array([2, 0, 1, 0, 2, 1, 1, 0, 2, 2, 0])
    for world in (1, 2, 3, 5, 16):
        parts = [ldist.shard_points(host, 3, r, world) for r in range(world)]
        allp = np.sort(np.concatenate(parts))
        np.testing.assert_array_equal(allp, np.arange(len(host)))
        sizes = [len(p) for p in parts]
        assert max(sizes) - min(sizes) <= 1
        for p in parts:  # every shard sees hosts in frame order
            assert (np.diff(host[p]) >= 0).all()


def test_host_threshold_restatement_matches_oracle(built):
    import oracle
    from ldso_amd import dist as ldist
    from ldso_amd import synth

    w = synth.make_window(n_frames=4, n_points=150, width=320, height=240, seed=33)
    ow = oracle.OracleWindow(w, threads=0)
    ow.iteration()
    r = ow.residuals()
    assert ldist.frame_threshold(r["new_energy_wo"][w.res_target == 3]) == ow.frame_energy_th()[-1]
