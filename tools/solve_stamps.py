"""Per-phase shader clocks of k_solve_fast (one S7 window, block 0, waves 0 and 1) from a diagnostic
build (-DLDSO_SOLVE_STAMPS, tools/build_ab.sh): assembly, each panel's next-panel update / barrier /
panel factorisation (wave 0) or trailing update (wave 1) / barrier, back substitution, projection,
xAd.  s_memtime ticks (shader clock, ~2.4 GHz).
  git apply tools/rejected/solve_fast_strips_and_stamps_r6.patch && bash tools/build_ab.sh stamps -DLDSO_SOLVE_STAMPS
  python tools/solve_stamps.py abl/stamps/libldso_ba.so [abl/strips/libldso_ba.so ...]"""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import ctypes as C, json, sys
import numpy as np
sys.path.insert(0, ROOT)
import torch
torch.cuda.init()
from ldso_amd import BAContext, synth
from ldso_amd import _lib as L
w = synth.make_window(**synth.S7, seed=1)
ns = [w.nullspaces()]
c = BAContext(0).load([w])
c.linearize()
f = L.lib().ldso_ba_diag_solve_stamps
out = {}
for it in (0, 2):
    runs = []
    for r in range(8):
        c.solve_device(it, 1e-5, ns)
        st = np.zeros((2, 48), np.uint64)
        assert f(st.ctypes.data_as(C.c_void_p)) == 0
        runs.append(st.astype(np.int64))
    s = runs[-1]
    w0, w1 = s[0], s[1]
    d = {"asm": int(w0[1] - w0[0]), "panel0": int(w0[2] - w0[1]), "bar0_w0": int(w0[3] - w0[2])}
    q = 0
    prev = w0[3]
    prev1 = w1[3]
    while q < 9 and w0[7 + 4 * q] > 0 and w0[7 + 4 * q] >= prev:
        d[f"p{q}"] = {"w0_next": int(w0[4 + 4 * q] - prev), "w0_barA": int(w0[5 + 4 * q] - w0[4 + 4 * q]),
                      "w0_panel": int(w0[6 + 4 * q] - w0[5 + 4 * q]), "w0_barB": int(w0[7 + 4 * q] - w0[6 + 4 * q]),
                      "w1_next": int(w1[4 + 4 * q] - prev1), "w1_barA": int(w1[5 + 4 * q] - w1[4 + 4 * q]),
                      "w1_trail": int(w1[6 + 4 * q] - w1[5 + 4 * q]), "w1_barB": int(w1[7 + 4 * q] - w1[6 + 4 * q])}
        prev, prev1 = w0[7 + 4 * q], w1[7 + 4 * q]
        q += 1
    d["fact_total"] = int(prev - w0[1])
    d["back"] = int(w0[40] - prev)
    d["bar_back"] = int(w0[41] - w0[40])
    d["apply"] = int(w0[42] - w0[41])
    d["xad"] = int(w0[43] - w0[42])
    d["total"] = int(w0[43] - w0[0])
    out[f"it{it}"] = d
    # stamps are only valid if every launch wrote them: clear between calls is not needed (overwritten)
print("RESULT " + json.dumps(out))
'''
for lib in sys.argv[1:]:
    env = dict(os.environ, LDSO_BA_LIB=os.path.abspath(lib))
    p = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT))], env=env, capture_output=True,
                       text=True, timeout=300)
    line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
    if p.returncode != 0 or not line:
        print(lib, "FAILED", p.returncode, p.stderr[-2000:])
        sys.exit(1)
    print(lib, json.dumps(json.loads(line[0][7:]), indent=1))
