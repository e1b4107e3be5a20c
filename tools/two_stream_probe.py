"""Probe: do two window groups on two HIP streams overlap k_point_sc / the stitch of one group with
k_linearize of the other?  The bench workload (64 x S7 windows) as one context, as two contexts of 32
windows (each its own non-blocking stream; every step issues both passes back to back, no
cross-stream dependency inside the timed loop), and as four of 16.  Host wall time per step over
K steps after warm-up, min over rounds.
  python tools/two_stream_probe.py [--steps 50] [--rounds 3]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch

    torch.cuda.init()
    from ldso_amd import BAContext, synth

    ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(64)]
    res = {}
    for groups in (1, 2, 4):
        n = 64 // groups
        ctxs = [BAContext(0).load(ws[g * n:(g + 1) * n]) for g in range(groups)]
        best = 1e9
        for _ in range(a.rounds):
            for _ in range(5):
                for c in ctxs:
                    c.linearize()
            for c in ctxs:
                c.sync()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                for c in ctxs:
                    c.linearize()
            for c in ctxs:
                c.sync()
            best = min(best, (time.perf_counter() - t0) / a.steps * 1e6)
        res[groups] = best
        print(f"groups {groups} x {n} windows: {best:.1f} us per step of 64 windows", flush=True)
        for c in ctxs:
            c.close()
    print("RESULT", res)


if __name__ == "__main__":
    main()
