"""Per-kernel times of the batched pass (64 x S7) with and without accumulation: with
accumulate=0 k_stitch runs only the per-window frame-threshold/energy blocks, which bounds
that block's share of the stitch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldso_amd import BAContext, synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(B)]
c = BAContext(0)
c.load(ws)
for acc in (True, False, True):
    for _ in range(3):
        c.linearize(accumulate=acc)
    c.sync()
    c.set_kernel_timing(True)
    for _ in range(20):
        c.linearize(accumulate=acc)
    c.sync()
    kt = c.kernel_times()
    c.set_kernel_timing(False)
    print(f"accumulate={acc}:", {k: round(1e3 * v[0] / v[1], 1) for k, v in kt.items() if v[1]})
c.close()
