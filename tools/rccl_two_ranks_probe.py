"""Probe: can two ranks on ONE GPU share an RCCL communicator (ldso_ba_comm_init)?  Each of two
processes loads its host-frame shard of one window on cuda:0, attaches the library's RCCL
communicator (the 128-byte id over a gloo group) and runs passes whose in-library exchange
reduces the packed systems; rank 0 compares the reduced system with an unsharded context's.
Prints one line per rank: OK with the worst block error, or the error RCCL gave."""
import os
import socket
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def block_worst(G, O, N):
    edges = [0, 4] + [4 + 8 * (f + 1) for f in range(N)]
    scale = np.linalg.norm(O)
    worst = 0.0
    for a in range(len(edges) - 1):
        for b in range(a, len(edges) - 1):
            g = G[edges[a]:edges[a + 1], edges[b]:edges[b + 1]]
            o = O[edges[a]:edges[a + 1], edges[b]:edges[b + 1]]
            den = max(np.linalg.norm(o), 1e-12 * scale, 1e-300)
            worst = max(worst, np.linalg.norm(g - o) / den)
    return worst


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ldso_amd import BAContext, synth
        from ldso_amd import dist as ldist

        cfg = dict(n_frames=7, n_points=900, seed=41)
        c = BAContext(0)
        ldist.attach_rccl(c, dist)
        c.load([synth.make_window(**cfg)], shard_rank=rank, shard_count=world)
        for _ in range(3):
            c.linearize()
        c.sync()
        s = c.system(0)
        out = dict(rank=rank)
        if rank == 0:
            f = BAContext(0).load([synth.make_window(**cfg)])
            for _ in range(3):
                f.linearize()
            sf = f.system(0)
            out["worst"] = max(block_worst(s[k], sf[k], cfg["n_frames"]) for k in ("HA", "Hsc"))
            out["th_equal"] = bool(np.array_equal(c.frame_energy_th(0), f.frame_energy_th(0)))
            f.close()
        c.close()
        dist.destroy_process_group()
        q.put(out)
    except Exception as ex:
        q.put(dict(rank=rank, error=repr(ex)[:500]))


def main():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for _ in range(2):
        print(q.get(timeout=100), flush=True)
    for p in ps:
        p.join(30)


if __name__ == "__main__":
    main()
