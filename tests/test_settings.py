"""The reference settings that change this path's arithmetic or control flow (ldso_ba_opt_settings).

* setting_affineOptModeA / B (Setting.cc:65-66; the KITTI / EuRoC drivers set 0 / 0,
  run_dso_kitti.cc:299-300, run_dso_euroc.cc:291-292; TUM-Mono mode 2 sets -1 / -1,
  run_dso_tum_mono.cc:284-292) enter twice: FrameHessian::getPrior's affine priors
  (FrameHessian.h:154-165) and, when < 0, the zeroing of JabF after the pattern sums
  (Residuals.cc:186-187), which removes the affine parameter from Jab_r (the Top block's b rows of
  a / b) and from fixLinearizationF's res_toZeroF (Residuals.cc:239-240).
* setting_vi_enable (Setting.cc:152, true in the reference) and the solver modes other than
  FIX_LAMBDA | ORTHOGONALIZE_X_LATER are refused (< 0 with a message) at every entry point that
  takes settings, instead of being run as the default.

CPU: the checks, the priors against the oracle restatement at every mode, and a known answer that
pins the oracle's JabF zeroing to the reference text (HA unchanged, the a / b rows of bA exactly 0,
bsc unchanged).  GPU: the pass (per residual bit-exact, HA / bA / Hsc / bsc per block, HL / bL
exact), point marginalisation and the device GN loop at (1e12, 1e8), (0, 0), (-1, -1) and (-1, 5)
against the oracle run with the same settings.  Parity unpinned by the reference itself.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from ldso_amd import _lib as L
from ldso_amd import synth

MODES = {"default": (1e12, 1e8), "kitti_euroc": (0.0, 0.0), "fixed": (-1.0, -1.0), "fix_a": (-1.0, 5.0)}


def settings(mode="default", **kw):
    a, b = MODES[mode]
    return L.OptSettings.default(affine_opt_mode_a=a, affine_opt_mode_b=b, **kw)


def window(cfg, s):
    w = synth.make_window(**cfg)
    w.settings = s
    return w.refresh_frame_terms()


def ab_rows(N):
    return np.array([4 + 8 * f + k for f in range(N) for k in (6, 7)])


# ------------------------------------------------------------------------------------------
# CPU
# ------------------------------------------------------------------------------------------
def test_check_settings(built):
    lib = L.lib()
    d = L.OptSettings()
    lib.ldso_ba_default_settings(C.byref(d))
    assert (d.solver_mode, d.force_accept_step, d.min_opt_iterations, d.vi_enable) == (L.SOLVER_DEFAULT, 1, 1, 0)
    assert np.float32(d.th_opt_iterations) == np.float32(1.2)
    assert (d.affine_opt_mode_a, d.affine_opt_mode_b) == (np.float32(1e12), np.float32(1e8))
    assert lib.ldso_ba_check_settings(C.byref(d)) == 0
    assert lib.ldso_ba_check_settings(None) == 0
    for m in MODES:
        assert lib.ldso_ba_check_settings(C.byref(settings(m))) == 0
    s = settings(vi_enable=1)
    assert lib.ldso_ba_check_settings(C.byref(s)) < 0 and b"vi_enable" in lib.ldso_ba_last_error()
    s = L.OptSettings.default(affine_opt_mode_a=float("nan"))
    assert lib.ldso_ba_check_settings(C.byref(s)) < 0 and b"affineOptMode" in lib.ldso_ba_last_error()
    s = L.OptSettings.default(reserved_=1)
    assert lib.ldso_ba_check_settings(C.byref(s)) < 0


def _solve_rc(s):
    w = synth.make_window(n_frames=3, n_points=40, width=160, height=120, seed=5)
    n = w.dim
    H = np.eye(n)
    z = np.zeros((n, n))
    b = np.ones(n)
    x = np.zeros(n)
    ptrs = [L.ptr(a, L.f64p) for a in (H, b, z, np.zeros(n))] + [L.ptr(None, L.f64p)] * 2 + \
        [L.ptr(a, L.f64p) for a in (z, np.zeros(n))]
    sp = C.byref(s) if s is not None else None
    return L.lib().ldso_ba_solve_system(sp, 3, 0, 1e-5, *ptrs, L.ptr(None, L.f64p), 0, L.ptr(x, L.f64p)), x


def test_solve_system_refuses_unsupported_settings(built):
    """EnergyFunctional::solveSystemF's branches this library does not implement are refused on the
    host solver too (EnergyFunctional.cc:282-283, 307-376, 383-432), not run as the default."""
    rc, x = _solve_rc(None)
    assert rc == 0 and np.all(np.isfinite(x))
    assert _solve_rc(settings("kitti_euroc"))[0] == 0
    lib = L.lib()
    assert _solve_rc(settings(vi_enable=1))[0] < 0 and b"vi_enable" in lib.ldso_ba_last_error()
    assert _solve_rc(settings(solver_mode=L.SOLVER_DEFAULT | L.SOLVER_SVD))[0] < 0
    assert b"SOLVER_SVD" in lib.ldso_ba_last_error()
    assert _solve_rc(settings(solver_mode=L.SOLVER_DEFAULT | L.SOLVER_USE_GN))[0] < 0
    assert _solve_rc(settings(solver_mode=L.SOLVER_ORTHOGONALIZE_X_LATER))[0] < 0  # no FIX_LAMBDA


@pytest.mark.parametrize("mode", list(MODES))
def test_priors_follow_affine_modes(built, mode):
    """takeData's prior (getPrior, FrameHessian.h:142-170) through the product's host helper and the
    oracle restatement, at each mode: the first frame keeps the initial priors, every other frame
    gets the mode itself (>= 0) or setting_initialAffA/BPrior (< 0) on a and b."""
    s = settings(mode)
    w = window(dict(n_frames=5, n_points=40, width=160, height=120, seed=5), s)
    a, b = MODES[mode]
    with oracle.affine_opt_modes(a, b):
        ref = oracle.frame_terms(w)
    np.testing.assert_array_equal(w.frame_prior, ref["frame_prior"])
    fp = w.frame_prior
    assert fp[0, 6] == fp[0, 7] == np.float32(1e14)
    exp_a = np.float64(np.float32(1e14 if a < 0 else a))
    exp_b = np.float64(np.float32(1e14 if b < 0 else b))
    assert np.all(fp[1:, 6] == exp_a) and np.all(fp[1:, 7] == exp_b)
    assert np.all(fp[1:, :6] == 0)
    # the settings reach the helper: a refused set fails it
    bad = settings(mode, vi_enable=1)
    fr = np.ascontiguousarray(w.frames)
    out = np.zeros((5, 8))
    assert L.lib().ldso_ba_frame_take_data(5, fr.ctypes.data, C.byref(bad), L.ptr(out, L.f64p), L.ptr(None, L.f64p),
                                           L.ptr(None, L.f64p)) < 0


def test_oracle_affine_fixed_known_answer(built):
    """Residuals.cc:186-187 zero JabF only after the pattern sums: with a and b fixed the oracle's
    pass has the same residual states, energies, JpJdF, HA, Hsc and bsc as with them optimised, and
    the a / b rows of bA are exactly 0 (Jab_r = sum resF * 0); with only a fixed, only a's rows."""
    cfg = dict(n_frames=5, n_points=300, width=320, height=240, seed=41)
    out = {}
    for m in ("kitti_euroc", "fixed", "fix_a"):
        with oracle.affine_opt_modes(*MODES[m]):
            ow = oracle.OracleWindow(window(cfg, settings(m)), threads=0)
            e, s = ow.iteration()
            out[m] = (e, s, ow.residuals(), ow.points())
    N = cfg["n_frames"]
    e0, s0, r0, p0 = out["kitti_euroc"]
    rows = ab_rows(N)
    assert np.abs(s0["bA"][rows]).min() > 0
    for m in ("fixed", "fix_a"):
        e1, s1, r1, p1 = out[m]
        assert np.array_equal(e0, e1)
        for k in r0:
            np.testing.assert_array_equal(r0[k], r1[k], err_msg=k)
        for k in p0:
            np.testing.assert_array_equal(p0[k], p1[k], err_msg=k)
        for k in ("HA", "Hsc", "bsc"):
            np.testing.assert_array_equal(s0[k], s1[k], err_msg=k)
        zero = rows if m == "fixed" else rows[0::2]
        keep = np.setdiff1d(np.arange(s0["bA"].size), zero)
        assert np.all(s1["bA"][zero] == 0)
        np.testing.assert_array_equal(s1["bA"][keep], s0["bA"][keep])
        # the priors differ exactly where getPrior says
        assert not np.array_equal(s0["HL"], s1["HL"])


# ------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("mode", list(MODES))
def test_pass_parity_at_affine_modes(built, mode):
    """One pass (linearizeAll + applyRes + accumulate) with the context's settings against the oracle
    with the same globals: per-residual / per-point bit-exact, HL / bL exact, HA / bA / Hsc / bsc
    per 8x8 block within 1e-4; with a mode < 0 the a / b rows of bA are exactly 0 on both sides."""
    from ldso_amd import BAContext
    from test_gpu_parity import compare_pass

    cfgs = [dict(synth.S7, seed=1), dict(n_frames=11, n_points=900, seed=83)]
    s = settings(mode)
    ctx = BAContext(0).set_settings(s).load([window(c, s) for c in cfgs])
    assert ctx.settings().affine_opt_mode_a == np.float32(MODES[mode][0])
    ctx.linearize(fix=False, accumulate=True)
    a, b = MODES[mode]
    with oracle.affine_opt_modes(a, b):
        for i, c in enumerate(cfgs):
            ow = oracle.OracleWindow(window(c, s), threads=0)
            e_cpu, s_cpu = ow.iteration()
            sg = compare_pass(ctx, ow, i, e_cpu, s_cpu)
            rows = ab_rows(c["n_frames"])
            if a < 0:
                assert np.all(sg["bA"][rows[0::2]] == 0) and np.all(s_cpu["bA"][rows[0::2]] == 0)
            if b < 0:
                assert np.all(sg["bA"][rows[1::2]] == 0)
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["default", "fixed"])
def test_marginalization_parity_at_affine_modes(built, mode):
    """Point marginalisation on a marginalisation context (which takes its parent's settings):
    with a / b fixed, res_toZeroF loses the JabF delta terms (Residuals.cc:239-240)."""
    from ldso_amd import BAContext
    from ldso_amd import dist as ldist
    from test_marginalization import BLOCK_TOL, ad_ht_delta, block_err, marg_points, vec_err

    cfg = dict(n_frames=6, n_points=500, seed=35)
    s = settings(mode)
    w = window(cfg, s)
    S = marg_points(w)
    adh = ad_ht_delta(w)
    adh[:, 6:8] += np.float32(2e-3)  # explicit affine deltas: their res_toZeroF terms are visible
    parent = BAContext(0).set_settings(s).load([w])
    parent.linearize()
    m = BAContext(0).load_marginalization(parent, 0, ldist.subset_window(w, S))
    assert m.settings().affine_opt_mode_b == np.float32(MODES[mode][1])
    H, b = m.marginalize_points(adh)
    with oracle.affine_opt_modes(*MODES[mode]):
        Ho, bo = oracle.OracleWindow(window(cfg, s), threads=0).marginalize_points(S.astype(np.int32), adh)
    N = cfg["n_frames"]
    assert block_err(H, Ho, N) <= BLOCK_TOL
    assert vec_err(b, bo, N) <= BLOCK_TOL
    m.close()
    parent.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["kitti_euroc", "fixed"])
def test_optimize_at_affine_modes_matches_host_loop(built, mode):
    """ldso_ba_optimize with the KITTI / EuRoC modes (and a / b fixed) against FullSystem::optimize's
    loop stepped by the oracle under the same globals: iteration counts and exit status equal,
    energies within 1e-4, states within the loop's tolerance."""
    from ldso_amd import BAContext
    from test_optimize import CONVERGES, RUNS_ALL, check_against_host

    s = settings(mode)
    a, b = MODES[mode]
    for cfg in (CONVERGES, RUNS_ALL):
        w = window(cfg, s)
        ns = w.nullspaces()
        ctx = BAContext(0).load([w])
        e, fr, c, idep, its, st = ctx.optimize(6, nullspaces=[ns], settings=s)
        assert ctx.settings().affine_opt_mode_a == np.float32(a)  # installed by optimize
        with oracle.affine_opt_modes(a, b):
            check_against_host(cfg, e[:, 0], fr, c[0], idep[0], int(its[0]), int(st[0]), 6, ns, settings=s)
        ctx.close()


@pytest.mark.gpu
def test_context_refuses_unsupported_settings(built):
    """A refused set leaves the context's settings as they were; optimize with refused settings runs
    nothing."""
    from ldso_amd import BAContext

    w = window(dict(n_frames=4, n_points=100, width=320, height=240, seed=7), settings("kitti_euroc"))
    ctx = BAContext(0).set_settings(settings("kitti_euroc")).load([w])
    with pytest.raises(RuntimeError, match="vi_enable"):
        ctx.set_settings(settings("kitti_euroc", vi_enable=1))
    assert ctx.settings().affine_opt_mode_a == 0.0 and ctx.settings().vi_enable == 0
    with pytest.raises(RuntimeError, match="SOLVER_SVD"):
        ctx.optimize(3, settings=settings(solver_mode=L.SOLVER_DEFAULT | L.SOLVER_SVD))
    assert ctx.settings().solver_mode == L.SOLVER_DEFAULT
    ctx.linearize()
    x = ctx.solve(0, 0)
    assert np.all(np.isfinite(x))
    ctx.close()


@pytest.mark.gpu
def test_optimize_refuses_priors_from_other_affine_modes(built):
    """ldso_ba_optimize's first pass and solve use the loaded priors, its later steps recompute them
    from the settings (getPrior): a window whose loaded affine priors follow other modes than the
    loop's settings is refused (< 0), and a refused call leaves the context's settings as they were."""
    from ldso_amd import BAContext

    cfg = dict(n_frames=4, n_points=100, width=320, height=240, seed=7)
    w = window(cfg, settings("kitti_euroc"))  # priors with affineOptMode 0 / 0
    ctx = BAContext(0).load([w])
    assert ctx.settings().affine_opt_mode_a == np.float32(1e12)
    with pytest.raises(RuntimeError, match="affine priors"):
        ctx.optimize(2)  # the context's defaults (1e12 / 1e8)
    with pytest.raises(RuntimeError, match="affine priors"):
        ctx.optimize(2, settings=settings("fixed"))
    assert ctx.settings().affine_opt_mode_a == np.float32(1e12)  # not installed
    ctx.optimize(2, settings=settings("kitti_euroc"))
    assert ctx.settings().affine_opt_mode_a == 0.0
    ctx.close()
