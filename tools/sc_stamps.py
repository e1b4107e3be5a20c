"""Diagnostic: the batched pass (64 x S7) on a build with the LDSO_SC_STAMPS switch of
tools/rejected/k_linearize_k_point_sc_ab_switches_r4.patch (LDSO_BA_LIB=abl/scstamps/...):
k_point_sc prints per-phase s_memtime stamps of every 64th block; this summarises them per pass
(phase durations in shader cycles: zero U, gather, barrier, SYRK, final barrier; block start
offsets relative to the pass's first block)."""
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
for k in range(4):
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
    m = re.match(r"SCSTAMP (\d+) (.*)", line)
    if m and cur is not None:
        cur.append((int(m.group(1)), [int(x) for x in m.group(2).split()]))
for k, rows in enumerate(passes[1:], 1):
    t0 = min(r[1][0] for r in rows)
    tend = max(r[1][5] for r in rows)
    ph = [[r[1][i + 1] - r[1][i] for r in rows] for i in range(5)]
    med = [sorted(x)[len(x) // 2] for x in ph]
    mx = [max(x) for x in ph]
    starts = sorted(r[1][0] - t0 for r in rows)
    print(f"pass {k}: {len(rows)} blocks, span {tend - t0} cyc; phase medians (zero, gather, sync, syrk, sync) {med}, "
          f"max {mx}; block start offsets median {starts[len(starts) // 2]} max {starts[-1]}")
print(p.stderr[-500:] if p.returncode else "")
