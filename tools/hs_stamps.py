"""Diagnostic: run the batched pass (64 x S7) a few times on a LDSO_HS_STAMPS build of the library
(LDSO_BA_LIB=abl/hs/libldso_ba.so) so k_stitch_host prints its per-phase clocks."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldso_amd import BAContext, synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(B)]
c = BAContext(0)
c.load(ws)
for k in range(3):
    print(f"--- pass {k}", flush=True)
    c.linearize()
    c.sync()
c.close()
