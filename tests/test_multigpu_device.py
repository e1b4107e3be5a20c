"""World-2 exchange driven by the DEVICE's own buffers, on one GPU (two processes, two contexts on
cuda:0, gloo between them).  The pool gives this build one GPU, so the ranks share it and gloo
stands in for the in-library RCCL exchange over xGMI; everything else is the multi-GPU path
(SURVEY.md §8e):

* each rank loads its host-frame shard (ldso_ba_load(rank, world)), runs a pass, and hands its
  packed partial {HA, bA, Hsc, bsc} out of the context with ldso_ba_copy_packed;
* the ranks sum-reduce the packed systems and the [E, #IN] pairs, agree on the newest-frame slot
  stride (max) and all-gather the slots each context exported with ldso_ba_export_newest;
* every rank puts the reduced system back (ldso_ba_copy_packed, direction 1), re-selects the
  threshold on the device (ldso_ba_frame_threshold_gathered) and solves the reduced system on
  the device itself -- with the priors, which every shard keeps.

Checks: the reduced system equals the unsharded window's within BLOCK_TOL, energies and the
threshold exactly, x is bitwise identical on both ranks (same reduced system, same priors) and
within the float-rounding envelope of the unsharded solve.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CFG = dict(n_frames=7, n_points=900, seed=41)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(0)  # torch's HIP runtime first, as bench.py
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import ctypes as C

        from ldso_amd import BAContext, synth
        from ldso_amd import _lib as L

        w = synth.make_window(**CFG)
        ns = [w.nullspaces()]
        c = BAContext(0).load([w], shard_rank=rank, shard_count=world)
        c.linearize()
        _, n, _ = c.packed_system()
        dev = torch.empty(n, dtype=torch.float64, device="cuda")
        L.check(c._lib.ldso_ba_copy_packed(c._h, dev.data_ptr(), n, 0))
        host = dev.cpu()
        dist.all_reduce(host)
        dev.copy_(host.cuda())
        torch.cuda.synchronize()  # torch's stream wrote dev; the library reads it on its own stream
        L.check(c._lib.ldso_ba_copy_packed(c._h, dev.data_ptr(), n, 1))
        e = torch.tensor(c.energy(0), dtype=torch.float64)
        dist.all_reduce(e)
        st = C.c_int64()
        L.check(c._lib.ldso_ba_newest_stride(c._h, C.byref(st)))
        stride = torch.tensor([st.value], dtype=torch.int64)
        dist.all_reduce(stride, op=dist.ReduceOp.MAX)
        stride = int(stride.item())
        slot = torch.empty(stride, dtype=torch.float32, device="cuda")
        L.check(c._lib.ldso_ba_export_newest(c._h, slot.data_ptr(), stride))
        parts = [torch.empty(stride, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(parts, slot.cpu())
        gathered = torch.cat(parts).cuda()
        torch.cuda.synchronize()
        L.check(c._lib.ldso_ba_frame_threshold_gathered(c._h, gathered.data_ptr(), world, stride))
        x0 = c.solve_device(0, 1e-5, ns)[0]
        x2 = c.solve_device(2, 1e-5, ns)[0]
        out = dict(rank=rank, x0=x0, x2=x2, th=c.frame_energy_th(0), energy=e.numpy(), system=c.system(0),
                   n_points=c.stats()["points"])
        c.close()
        dist.destroy_process_group()
        q.put(out)
    except Exception as ex:  # report instead of hanging the parent
        q.put(dict(rank=rank, error=repr(ex)))


@pytest.mark.timeout(300)
def test_world2_exchange_of_device_buffers(built):
    import torch.multiprocessing as mp

    from ldso_amd import BAContext, synth
    from test_gpu_parity import BLOCK_TOL, block_errors, sensitivity, vec_block_errors

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=280) for _ in range(world)], key=lambda o: o["rank"])
    for p in procs:
        p.join(60)
    for o in outs:
        assert "error" not in o, o
    assert sum(o["n_points"] for o in outs) == CFG["n_points"]

    w = synth.make_window(**CFG)
    ns = w.nullspaces()
    full = BAContext(0).load([w])
    full.linearize()
    s_full, e_full, th_full = full.system(0), full.energy(0), full.frame_energy_th(0)
    x0_full = full.solve(0, 0, 1e-5, ns)
    x2_full = full.solve(0, 2, 1e-5, ns)
    full.close()
    N = CFG["n_frames"]
    for o in outs:
        s = o["system"]
        for k in ("HA", "Hsc"):
            assert block_errors(s[k], s_full[k], N) < BLOCK_TOL, k
        for k in ("bA", "bsc"):
            assert vec_block_errors(s[k], s_full[k], N) < BLOCK_TOL, k
        np.testing.assert_array_equal(s["HL"], s_full["HL"])  # every rank has the priors
        np.testing.assert_array_equal(s["bL"], s_full["bL"])
        assert o["energy"][2] == e_full[2]
        assert abs(o["energy"][0] - e_full[0]) <= 1e-9 * abs(e_full[0])
        np.testing.assert_array_equal(o["th"][-1], th_full[-1])
    # the redundant solve: bitwise the same on both ranks, and the unsharded solution up to the
    # system's float-rounding envelope (the shard sums reassociate H)
    np.testing.assert_array_equal(outs[0]["x0"], outs[1]["x0"])
    np.testing.assert_array_equal(outs[0]["x2"], outs[1]["x2"])
    for it, key, xf in ((0, "x0", x0_full), (2, "x2", x2_full)):
        env = sensitivity(N, it, s_full, ns, xf)
        rel = np.linalg.norm(outs[0][key] - xf) / np.linalg.norm(xf)
        print(f"it={it}: |x_world2 - x_full| / |x_full| = {rel:.3e} (envelope {env:.3e})")
        assert rel <= max(1e-6, 20 * env)
