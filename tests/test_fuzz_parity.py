"""Randomised parity sweep: seeded random windows through one pass (linearizeAll + applyRes +
accumulate) on the GPU against the oracle, with everything the path branches on drawn at random --
keyframe count (2..16: the host stitch and, above 11, the per-pair records stitch), point count
(0..700), frame size (widths not a multiple of 8, heights not a multiple of 4), camera model,
forward or sideways motion (scale change, OOB pattern pixels), outlier fraction, points near the
border, the residuals per k_linearize wavefront (8..64 or automatic), both image layouts and the
affine-optimisation modes.  Bars as tests/test_gpu_parity.py's compare_pass: per residual and per
point bit-exact, the energy to 1e-12, the stitched blocks within 1e-4, the priors exact.
After the accumulating pass each case also runs the fix pass (linearizeAll(true) after resetOOB:
relBS of the new residuals) against the oracle's.  Each case prints its draw, so a failure names
the configuration to rerun."""
import numpy as np
import pytest

import oracle
from ldso_amd import BAContext, synth
from ldso_amd import _lib as L

pytestmark = pytest.mark.gpu

SIZES = [(160, 120), (317, 203), (640, 480), (1242, 375)]
AFFINE = [(1e12, 1e8), (0.0, 0.0), (-1.0, -1.0), (-1.0, 5.0)]


def draw(case):
    rng = np.random.default_rng(9000 + case)
    W, H = SIZES[rng.integers(len(SIZES))]
    n_win = int(rng.integers(1, 4))
    wins = []
    for k in range(n_win):
        N = int(rng.choice([2, 3, 4, 5, 6, 7, 8, 11, 13, 16], p=[.1, .12, .12, .12, .1, .14, .1, .1, .05, .05]))
        if case in (10, 11) and k == 0:  # two cases hold a window above 11 keyframes (k_stitch's records)
            N = 13 if case == 10 else 16
        P = int(rng.integers(0, 700 if N <= 8 else 300))
        calib = None
        if rng.random() < 0.5:
            f = float(rng.uniform(0.4, 1.2)) * W
            calib = [f, f * float(rng.uniform(0.95, 1.05)), W / 2 + float(rng.uniform(-0.1, 0.1)) * W,
                     H / 2 + float(rng.uniform(-0.1, 0.1)) * H]
        wins.append(dict(n_frames=N, n_points=P, width=W, height=H, seed=int(rng.integers(1 << 30)),
                         outlier_frac=float(rng.uniform(0.0, 0.3)), motion=str(rng.choice(["sideways", "forward"])),
                         edge_frac=float(rng.choice([0.0, 0.2])), calib=calib,
                         plane_depth=max(25.0, 2.5 * (N - 1))))  # the canyon's far facade beyond the travel
    chunk = int(rng.choice([0, 8, 24, 64]))
    layout = int(rng.choice([1, 3]))
    aff = AFFINE[rng.integers(len(AFFINE))]
    return wins, chunk, layout, aff


def window(cfg, s):
    w = synth.make_window(**cfg)
    w.settings = s
    return w.refresh_frame_terms()


@pytest.mark.parametrize("case", range(24))
def test_random_windows_match_oracle(built, case):
    from test_gpu_parity import compare_pass

    wins, chunk, layout, aff = draw(case)
    print(f"case {case}: chunk {chunk}, layout {layout}, affine {aff}")
    for c in wins:
        print("  ", c)
    s = L.OptSettings.default(affine_opt_mode_a=aff[0], affine_opt_mode_b=aff[1])
    ctx = BAContext(0)
    ctx.set_tuning(6, chunk)   # LDSO_BA_TUNE_TOP_CHUNK
    ctx.set_tuning(2, layout)  # LDSO_BA_TUNE_TILED_IMAGES
    ctx.set_settings(s).load([window(c, s) for c in wins])
    ctx.linearize(fix=False, accumulate=True)
    ows = []
    with oracle.affine_opt_modes(*aff):
        for i, c in enumerate(wins):
            ow = oracle.OracleWindow(window(c, s), threads=0)
            e_cpu, s_cpu = ow.iteration()
            compare_pass(ctx, ow, i, e_cpu, s_cpu)
            ows.append(ow)
        # then the fix pass (linearizeAll(true): relBS of the new residuals) after resetOOB
        ctx.reset_oob()
        ctx.linearize(fix=True, accumulate=False)
        for i, ow in enumerate(ows):
            ow.reset_oob()
            e_cpu = ow.linearize_all(True)
            compare_pass(ctx, ow, i, e_cpu, None, check_system=False)
            np.testing.assert_array_equal(ctx.residuals(i)["rel_bs"], ow.residuals()["rel_bs"])
            ow.close()
    ctx.close()


@pytest.mark.parametrize("case", range(8))
def test_random_point_marginalisation_matches_oracle(built, case):
    """flagPointsForRemoval -> fixLinearizationF -> marginalizePointsF on random windows (2-11
    keyframes, the sizes and motions above) with a random subset of points (host 0's and a random
    fraction of the rest) and random linearisation deltas: residual states, JpJdF and the point
    terms bit-exact against the oracle, H / b per 8x8 block within 1e-4 (test_marginalization's bars)."""
    from ldso_amd import dist as ldist
    from test_marginalization import ad_ht_delta, block_err, vec_err

    rng = np.random.default_rng(7000 + case)
    W, H = SIZES[rng.integers(len(SIZES))]
    cfg = dict(n_frames=int(rng.integers(2, 12)), n_points=int(rng.integers(50, 600)), width=W, height=H,
               seed=int(rng.integers(1 << 30)), motion=str(rng.choice(["sideways", "forward"])),
               outlier_frac=float(rng.uniform(0.0, 0.2)))
    frac, scale = float(rng.uniform(0.05, 0.5)), float(rng.choice([0.0, 1.0, 3.0]))
    print(f"case {case}: {cfg}, fraction {frac:.2f}, delta scale {scale}")
    w = synth.make_window(**cfg)
    N = w.n_frames
    S = np.array(sorted(set(np.flatnonzero(w.point_host == 0)) |
                        set(np.flatnonzero(rng.random(w.n_points) < frac))), np.int64)
    adh = ad_ht_delta(w, scale)
    parent = BAContext(0).load([w])
    parent.linearize()
    parent.sync()
    m = BAContext(0).load_marginalization(parent, 0, ldist.subset_window(w, S))
    Hm, bm = m.marginalize_points(adh)
    ow = oracle.OracleWindow(synth.make_window(**cfg), threads=0)
    Ho, bo = ow.marginalize_points(S.astype(np.int32), adh)
    assert block_err(Hm, Ho, N) <= 1e-4
    assert vec_err(bm, bo, N) <= 1e-4
    rg, ro = m.residuals(0), ow.residuals()
    rs = np.concatenate([np.arange(w.point_res_begin[p], w.point_res_begin[p + 1]) for p in S])
    for k in ("new_state", "state", "flags", "state_energy", "center"):
        np.testing.assert_array_equal(rg[k], ro[k][rs], err_msg=k)
    act = (ro["flags"][rs] & 1).astype(bool)
    np.testing.assert_array_equal(rg["jpjdf"][act], ro["jpjdf"][rs][act])
    pg, po = m.points(0), ow.points()
    for k in ("HdiF", "bdSumF", "idepth_hessian"):
        np.testing.assert_array_equal(pg[k], po[k][S], err_msg=k)
    m.close()
    parent.close()
    ow.close()
