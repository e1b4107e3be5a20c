"""Generate the committed golden fixtures tests/golden/*.npz.

Inputs come from the seeded synthetic generator (small images so the files stay small; only
the intensity channel is stored, the gradient channels are rebuilt with FrameHessian::makeImages'
rule on load).  Expected outputs are the CPU restatement's (oracle/, single-thread path) for one
pass of linearizeAll(false) + applyRes + accumulate{AF,LF,SCF} and the solve.  The reference
itself cannot run here, so these fixtures pin regressions of the oracle and
of the GPU path; tests/test_oracle_kat.py pins the oracle against first principles.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle  # noqa: E402
from ldso_amd import synth  # noqa: E402

CASES = {
    "w3_p64": dict(n_frames=3, n_points=64, width=160, height=120, seed=101),
    "w5_p160": dict(n_frames=5, n_points=160, width=160, height=120, seed=102, baseline=0.08),
    "w7_p256": dict(n_frames=7, n_points=256, width=160, height=120, seed=103),  # SURVEY §7 step 2's N=7, P=256
}


def main(names=None):
    for name, cfg in CASES.items():
        if names and name not in names:
            continue
        w = synth.make_window(**cfg)
        ow = oracle.OracleWindow(synth.make_window(**cfg), threads=0)
        e, s = ow.iteration()
        r = ow.residuals()
        p = ow.points()
        ns = w.nullspaces()
        x = oracle.solve_system(w.n_frames, 2, 1e-5, s, nullspaces=ns)
        np.savez_compressed(
            os.path.join(HERE, f"{name}.npz"),
            cfg=np.array(repr(cfg)), n_frames=w.n_frames, width=w.width, height=w.height, calib=w.calib,
            frames=w.frames, I=w.dI[:, :, 0].copy(), frame_energy_th=w.frame_energy_th, point_host=w.point_host,
            point_data=w.point_data, point_res_begin=w.point_res_begin, res_target=w.res_target,
            res_state=w.res_state, res_energy=w.res_energy, res_flags=w.res_flags,
            out_energy=e, out_new_state=r["new_state"], out_state_energy=r["state_energy"],
            out_energy_wo=r["new_energy_wo"], out_center=r["center"], out_flags=r["flags"], out_jpjdf=r["jpjdf"],
            out_HdiF=p["HdiF"], out_bdSumF=p["bdSumF"], out_frame_th=ow.frame_energy_th(),
            out_HA=s["HA"], out_bA=s["bA"], out_HL=s["HL"], out_bL=s["bL"], out_Hsc=s["Hsc"], out_bsc=s["bsc"],
            out_x=x, nullspaces=ns)
        print(name, "residuals", w.n_residuals, "IN", int(e[2]), "E", e[0])


if __name__ == "__main__":
    main(sys.argv[1:])
