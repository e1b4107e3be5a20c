import sys, time, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from ldso_amd import synth
from ldso_amd.tracker import CoarseTracker
w, h = 640, 480
calib = np.array([384.0, 432.0, 319.5, 239.5], np.float32)
color, make_pc = synth.make_tracker_scene(w, h, seed=0)
ct = CoarseTracker(w, h, 0)
ct.make_k(calib); ct.set_new_frame(color, 1.0)
pcs = make_pc([ct.frame_level(l)[0][:, 0] for l in range(ct.levels)])
ct.set_reference([(p["u"], p["v"], p["idepth"], p["color"]) for p in pcs], 1.0, (0.02, 3.0))
rng = np.random.default_rng(3)
Ts = np.stack([synth.se3_matrix(rng.normal(0, 2e-3, 3), rng.normal(0, 1e-2, 3)) for _ in range(32)])
ab = np.tile([0.05, 1.0], (32, 1))
for _ in range(20): ct.calc_res_gs(0, Ts[0], ab[0])
reps = 500
t0 = time.perf_counter()
for i in range(reps): ct.calc_res_gs(0, Ts[i % 32], ab[0])
print("lm_ms", 1e3 * (time.perf_counter() - t0) / reps)
ct.set_kernel_timing(True)
for i in range(reps): ct.calc_res_gs(0, Ts[i % 32], ab[0])
print({k: v[0] / max(1, v[1]) * 1e3 for k, v in ct.kernel_times().items() if v[1]})
