"""Diagnostic: the batched pass (64 x S7) on a LDSO_LIN_STAMPS build of k_linearize
(git apply tools/diag/k_linearize_stamps.patch; bash tools/build_ab.sh linstamps -DLDSO_LIN_STAMPS=1;
LDSO_BA_LIB=abl/linstamps/libldso_ba.so): per-phase shader cycles of every 97th chunk --
prologue (loads, LDS staging), phase A (pattern pixels), phase B (per residual), Top (MFMA block)."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys
sys.path.insert(0, ROOT)
from ldso_amd import BAContext, synth
ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(64)]
c = BAContext(0)
c.load(ws)
for k in range(3):
    print(f"--- pass {k}", flush=True)
    c.linearize()
    c.sync()
c.close()
'''.replace("ROOT", repr(ROOT))
p = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=300)
passes, cur = [], None
for line in p.stdout.splitlines():
    if line.startswith("--- pass"):
        cur = []
        passes.append(cur)
    m = re.match(r"LINSTAMP (\d+) (\d+) (.*)", line)
    if m and cur is not None:
        cur.append((int(m.group(1)), int(m.group(2)), [int(x) for x in m.group(3).split()]))
for k, rows in enumerate(passes[1:], 1):
    full = [r for r in rows if r[1] == 64]
    ph = [[r[2][i + 1] - r[2][i] for r in full] for i in range(4)]
    med = [sorted(x)[len(x) // 2] for x in ph]
    avg = [sum(x) / len(x) for x in ph]
    tot = [r[2][4] - r[2][0] for r in full]
    print(f"pass {k}: {len(full)} full chunks; phase cycles (prologue, A, B, Top) median {med} mean "
          f"{[round(a) for a in avg]}; wave lifetime median {sorted(tot)[len(tot) // 2]}")
print(p.stderr[-500:] if p.returncode else "")
