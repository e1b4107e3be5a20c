"""Phase timing of k_solve_reg from its s_memtime stamps (diagnostic build, -DLDSO_EXP_STAMPS):
  LDSO_BA_LIB=abl/stamps/libldso_ba.so python tools/solve_stamps.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.cuda.init()
from ldso_amd import BAContext, synth  # noqa: E402
from ldso_amd import _lib as L  # noqa: E402

w = synth.make_window(**synth.S7, seed=1000)
ns = [w.nullspaces()]
c = BAContext(0).load([w])
c.linearize()
nsa = c._ns_all(ns)
names = ["start", "assembled", "rows loaded", "step 0", "step n/2", "forward done", "-", "substituted",
         "projected"]
for it in (0, 2):
    acc = []
    for rep in range(20):
        L.check(c._lib.ldso_ba_solve_device(c._h, it, 1e-5, L.ptr(nsa, L.f64p), 7, L.ptr(None, L.f64p)))
        c.sync()
        st = np.zeros(64, np.uint64)
        c._lib.ldso_ba_debug_stamps(ctypes.c_void_p(st.ctypes.data))
        acc.append(st.astype(np.int64) - int(st[0]))
    med = np.median(np.array(acc[5:]), axis=0)
    print(f"iteration {it}: " + ", ".join(f"{nm} {v:.0f}" for nm, v in zip(names, med[:9])))
    print("  assembly: window descriptor at %.0f, loads issued %.0f, index math %.0f, diag+barrier %.0f"
          % (med[14], med[9], med[10], med[11]))
    print("  projection: ntx at %.0f, coef at %.0f" % tuple(med[12:14]))
    for w in range(4):
        ph = med[16 + 8 * w:16 + 8 * w + 8]
        print(f"  step 10 wave {w}: top {ph[0]:.0f} +wait {ph[1]-ph[0]:.0f} +dg {ph[2]-ph[1]:.0f} "
              f"+pivot {ph[3]-ph[2]:.0f} +publish {ph[4]-ph[3]:.0f} (pub at {ph[7]-ph[3]:.0f}) "
              f"+rd {ph[5]-ph[4]:.0f} +update {ph[6]-ph[5]:.0f}")
c.close()
