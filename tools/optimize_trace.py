"""B windows' ldso_ba_optimize (6 GN iterations; argv: repeats, B), run a few times: the workload of the
kernel-trace timeline in profiles/ (rocprofv3 --kernel-trace -- python tools/optimize_trace.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.cuda.init()
from ldso_amd import BAContext, synth  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ws = [synth.make_window(**synth.S7, seed=1 + i) for i in range(B)]
ns = [w.nullspaces() for w in ws]
c = BAContext(0).load(ws)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    c.optimize(6, nullspaces=ns)
c.close()
