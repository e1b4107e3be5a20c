"""Stitched systems of two library builds on the same windows, compared bit for bit:
  python tools/sys_compare.py libA.so libB.so"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, hashlib
sys.path.insert(0, ROOT)
import torch
torch.cuda.init()
import numpy as np
from ldso_amd import BAContext, synth
import os
ws = [synth.make_window(**synth.S7, seed=900 + i) for i in range(3)]
if not os.environ.get("SYS_COMPARE_S7_ONLY"):
    ws.append(synth.make_window(n_frames=12, n_points=700, seed=950))
c = BAContext(0).load(ws)
c.linearize()
h = hashlib.sha256()
for i in range(len(ws)):
    s = c.system(i)
    for k in ("HA", "bA", "Hsc", "bsc"):
        h.update(np.ascontiguousarray(s[k]).tobytes())
print("RESULT", h.hexdigest())
'''
out = []
for lib in sys.argv[1:]:
    env = dict(os.environ, LDSO_BA_LIB=os.path.abspath(lib))
    p = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT))], env=env, capture_output=True,
                       text=True, timeout=300)
    line = [x for x in p.stdout.splitlines() if x.startswith("RESULT")]
    if p.returncode or not line:
        print(lib, "FAILED", p.stderr[-1500:])
        sys.exit(1)
    out.append(line[0].split()[1])
    print(lib, out[-1])
print("identical" if len(set(out)) == 1 else "DIFFERENT")
sys.exit(0 if len(set(out)) == 1 else 1)
