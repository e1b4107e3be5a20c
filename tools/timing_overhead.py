import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from ldso_amd import BAContext, synth
ws=[synth.make_window(**synth.S7, seed=1000+i) for i in range(64)]
c=BAContext(0); c.load(ws)
for _ in range(5): c.linearize()
c.sync()
for timing in (False, True, False, True):
    c.set_kernel_timing(timing)
    c.sync(); t=time.perf_counter()
    for _ in range(50): c.linearize()
    c.sync(); el=time.perf_counter()-t
    print("timing", timing, "ms/step %.4f" % (el/50*1e3))
