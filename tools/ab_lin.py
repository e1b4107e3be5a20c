"""A/B k_linearize variants on the bench workload (HIP-event timing, interleaved rounds).
  python tools/ab_lin.py [windows]"""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldso_amd import BAContext, synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(B)]
ctxs = {}
for tiled in (1, 2, 3):
    c = BAContext(0)
    c.set_tuning(2, tiled)
    c.load(ws)
    for _ in range(3):
        c.linearize()
    ctxs[tiled] = c
combos = [(1, 0, 1, 3, 1), (2, 0, 1, 3, 1), (3, 0, 1, 3, 1), (3, 0, 0, 3, 1)]
res = {k: [] for k in combos}
for rnd in range(3):
    for (tiled, load3, xcd, wv, cf) in combos:
        c = ctxs[tiled]
        c.set_tuning(3, load3)
        c.set_tuning(4, xcd)
        c.set_tuning(1, wv)
        c.set_tuning(5, cf)
        c.linearize()
        c.set_kernel_timing(True)
        for _ in range(20):
            c.linearize()
        ms, n = c.kernel_times()["k_linearize"]
        c.set_kernel_timing(False)
        res[(tiled, load3, xcd, wv, cf)].append(1e3 * ms / n)
for k in sorted(res, key=lambda k: min(res[k])):
    print(f"tiled={k[0]} load3={k[1]} xcd={k[2]} variant={k[3]} centre_first={k[4]}: best {min(res[k]):.1f} us  {['%.1f' % x for x in res[k]]}")

# cost split: the same pass without the accumulation (k_linearize skips the Top terms/reduction)
c = ctxs[1]
for v in (3,):
    c.set_tuning(1, v)
    c.set_tuning(4, 1)
    c.set_tuning(5, 1)
    c.set_tuning(3, 0)
    for acc in (True, False):
        c.linearize(accumulate=acc)
        c.set_kernel_timing(True)
        for _ in range(20):
            c.linearize(accumulate=acc)
        ms, n = c.kernel_times()["k_linearize"]
        c.set_kernel_timing(False)
        print(f"variant={v} accumulate={acc}: {1e3 * ms / n:.1f} us")
