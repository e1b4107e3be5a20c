"""Known-answer tests that pin the CPU restatement (oracle/) independently of its own code.

The reference ships no golden vectors for this path and cannot be built here, so these
first-principles checks are what pin the oracle:
  * geometric Jacobians (Residuals.cc:69-106) against central finite differences of the
    projection (ResidualProjections.h:57-84), in double;
  * the stitched active Hessian HA, bA (AccumulatedTopHessian.cc) against a dense J^T J, J^T r
    rebuilt in numpy from the per-residual Jacobians and the adjoints (setAdjointsF);
  * the Schur terms Hsc, bsc (AccumulatedSCHessian.cc) against sum_p h_pd h_pd^T / H_dd;
  * PSD-ness, symmetry, the gauge nullspaces (getNullspaces) of HA - Hsc;
  * setNewFrameEnergyTH against numpy's partition (nth_element);
  * the photometric residuals, weights, energies and states of linearize (Residuals.cc:48-208)
    against a float64 numpy restatement written from the reference text;
  * solveSystemF's LDLT, orthogonalize and resubstituteFPt against numpy.
"""
import numpy as np
import pytest

import oracle
from ldso_amd import synth

J_OFF = dict(resF=0, Jpdxi=8, Jpdc=20, Jpdd=28, JIdx=30, JabF=46, JIdx2=62, JabJIdx=66, Jab2=70)


def unpack_J(row):
    o = J_OFF
    return dict(resF=row[0:8], Jpdxi=row[8:20].reshape(2, 6), Jpdc=row[20:28].reshape(2, 4), Jpdd=row[28:30],
                JIdx=row[30:46].reshape(2, 8), JabF=row[46:62].reshape(2, 8))


WINDOWS = {
    "euroc_320x240": dict(n_frames=5, n_points=300, width=320, height=240, seed=13),
    # BASELINE config 3's geometry: KITTI 00's cropped 1232 x 368 output model and forward travel
    # (ldso_amd/synth.py KITTI00), a smaller window so the per-residual numpy checks stay fast
    "kitti00_forward": dict(synth.KITTI00, n_frames=5, n_points=300, seed=13),
}


@pytest.fixture(scope="module", params=list(WINDOWS))
def win(request):
    cfg = WINDOWS[request.param]
    w = synth.make_window(**cfg)
    ow = oracle.OracleWindow(w, threads=0)
    e, sysm = ow.iteration()
    return dict(w=w, ow=ow, e=e, sys=sysm, res=ow.residuals(), J=ow.jacobians().astype(np.float64), pts=ow.points(),
                cfg=cfg)


def se3_exp_small(xi):
    """exp of a twist [upsilon, omega] (double)"""
    w = xi[3:]
    th = np.linalg.norm(w)
    W = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-12:
        R, V = np.eye(3) + W, np.eye(3) + 0.5 * W
    else:
        R = np.eye(3) + np.sin(th) / th * W + (1 - np.cos(th)) / th ** 2 * W @ W
        V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * W + (th - np.sin(th)) / th ** 3 * W @ W
    return R, V @ xi[:3]


def project(R, t, calib, u, v, rho):
    fx, fy, cx, cy = calib
    klip = np.array([(u - cx) / fx, (v - cy) / fy, 1.0])
    p = R @ klip + t * rho
    return np.array([p[0] / p[2] * fx + cx, p[1] / p[2] * fy + cy])


def test_geometric_jacobians_match_finite_differences(win):
    w, J, res = win["w"], win["J"], win["res"]
    N = w.n_frames
    calib = w.calib.astype(np.float64)
    rng = np.random.default_rng(0)
    act = np.flatnonzero(res["flags"] & 1)
    checked = 0
    for k in rng.choice(act, 40, replace=False):
        p = np.searchsorted(w.point_res_begin, k, side="right") - 1
        h, t = w.point_host[p], w.res_target[k]
        pre = w.precalc[h + N * t].astype(np.float64)
        R0, t0 = pre[12:21].reshape(3, 3), pre[21:24]
        u, v, rho = (float(x) for x in w.point_data[p, [0, 1, 3]])
        Jk = unpack_J(J[k])
        eps = 1e-6
        for q in range(6):  # left perturbation of the host->target pose, tangent [t, w]
            xi = np.zeros(6)
            xi[q] = eps
            Rp, tp = se3_exp_small(xi)
            xi[q] = -eps
            Rm, tm = se3_exp_small(xi)
            d = (project(Rp @ R0, Rp @ t0 + tp, calib, u, v, rho) - project(Rm @ R0, Rm @ t0 + tm, calib, u, v, rho)) / (2 * eps)
            np.testing.assert_allclose(Jk["Jpdxi"][:, q], d, rtol=2e-3, atol=2e-3 * np.abs(Jk["Jpdxi"]).max())
        d = (project(R0, t0, calib, u, v, rho + 1e-7) - project(R0, t0, calib, u, v, rho - 1e-7)) / 2e-7
        np.testing.assert_allclose(Jk["Jpdd"], d, rtol=2e-3, atol=1e-3 * np.abs(d).max())
        for q in range(4):  # CalibHessian::value is value_scaled / SCALE_{F,C} (SCALE = 50)
            cp, cm = calib.copy(), calib.copy()
            cp[q] += 1e-4
            cm[q] -= 1e-4
            d = 50.0 * (project(R0, t0, cp, u, v, rho) - project(R0, t0, cm, u, v, rho)) / 2e-4
            np.testing.assert_allclose(Jk["Jpdc"][:, q], d, rtol=2e-3, atol=2e-3 * np.abs(Jk["Jpdc"]).max())
        checked += 1
    assert checked == 40


def dense_system(w, J, res, points=None):
    """J^T J, J^T r and the explicit Schur complement, rebuilt from per-residual Jacobians
    (optionally also each point's coupling row h_pd, H_dd and b_d into `points`)."""
    N, D = w.n_frames, w.dim
    HA = np.zeros((D, D))
    bA = np.zeros(D)
    Hsc = np.zeros((D, D))
    bsc = np.zeros(D)
    adH = w.ad_host.reshape(-1, 8, 8)
    adT = w.ad_target.reshape(-1, 8, 8)
    for p in range(w.n_points):
        hpd = np.zeros(D)
        hdd = 0.0
        bd = 0.0
        for k in range(w.point_res_begin[p], w.point_res_begin[p + 1]):
            if not res["flags"][k] & 1:
                continue
            h, t = w.point_host[p], w.res_target[k]
            Jk = unpack_J(J[k])
            for i in range(8):
                g = Jk["JIdx"][:, i]
                jrel = np.concatenate([g @ Jk["Jpdxi"], [Jk["JabF"][0, i], Jk["JabF"][1, i]]])
                row = np.zeros(D)
                row[:4] = g @ Jk["Jpdc"]
                row[4 + 8 * h:12 + 8 * h] += adH[h + N * t] @ jrel
                row[4 + 8 * t:12 + 8 * t] += adT[h + N * t] @ jrel
                jd = g @ Jk["Jpdd"]
                r = Jk["resF"][i]
                HA += np.outer(row, row)
                bA += row * r
                hpd += row * jd
                hdd += jd * jd
                bd += jd * r
        if hdd > 0:
            Hsc += np.outer(hpd, hpd) / hdd
            bsc += hpd * bd / hdd
        if points is not None:
            points.append((hpd, hdd, bd))
    return HA, bA, Hsc, bsc


def rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


def test_stitched_system_equals_dense_normal_equations(win):
    w, sysm = win["w"], win["sys"]
    HA, bA, Hsc, bsc = dense_system(w, win["J"], win["res"])
    # measured ~5e-8 (float accumulation in the restatement vs double here)
    assert rel(sysm["HA"], HA) < 1e-6
    assert rel(sysm["bA"], bA) < 1e-6
    assert rel(sysm["Hsc"], Hsc) < 1e-6
    assert rel(sysm["bsc"], bsc) < 1e-6
    # block-wise too (small blocks must not hide behind large ones)
    N = w.n_frames
    for a in range(N):
        sa = slice(4 + 8 * a, 12 + 8 * a)
        for b in range(N):
            sb = slice(4 + 8 * b, 12 + 8 * b)
            if np.linalg.norm(HA[sa, sb]) > 1e-9 * np.linalg.norm(HA):
                assert rel(sysm["HA"][sa, sb], HA[sa, sb]) < 1e-4
            if np.linalg.norm(Hsc[sa, sb]) > 1e-9 * np.linalg.norm(Hsc):
                assert rel(sysm["Hsc"][sa, sb], Hsc[sa, sb]) < 1e-4


def test_priors_only_in_HL(win):
    w, s = win["w"], win["sys"]
    D = w.dim
    assert np.count_nonzero(s["HL"] - np.diag(np.diag(s["HL"]))) == 0
    np.testing.assert_array_equal(np.diag(s["HL"])[:4], w.c_prior)
    np.testing.assert_array_equal(np.diag(s["HL"])[4:], w.frame_prior.ravel())
    np.testing.assert_allclose(s["bL"][4:], (w.frame_prior * w.frame_delta_prior).ravel())
    assert D == 8 * w.n_frames + 4


def test_psd_symmetry_and_gauge(win):
    w, s = win["w"], win["sys"]
    HA, Hsc = s["HA"], s["Hsc"]
    sym = lambda M: np.linalg.norm(M - M.T) / np.linalg.norm(M)
    assert sym(HA) < 1e-12 and sym(Hsc) < 1e-6
    # HA = J^T J is PSD, and HA - Hsc is the Schur complement of the full Hessian (PSD)
    sc = np.sqrt(np.clip(np.diag(HA), 1e-30, None))
    for M in (HA, HA - Hsc):
        Ms = M / np.outer(sc, sc)
        assert np.linalg.eigvalsh(0.5 * (Ms + Ms.T)).min() > -1e-6
    # the 6 pose + 1 scale gauge directions (FrameHessian::setStateZero, getNullspaces) are in
    # the kernel of the point-marginalised system (first order; FEJ makes it hold per residual)
    ns = w.nullspaces()
    M = HA - Hsc
    for n in ns:
        assert np.linalg.norm(M @ n) <= 1e-7 * np.linalg.norm(M, 2) * np.linalg.norm(n)  # measured <= 3e-9


def test_energy_and_frame_threshold(win):
    w, ow, e, res = win["w"], win["ow"], win["e"], win["res"]
    # linearizeAll returns the double sum of every residual's linearize() value
    assert e[2] == np.count_nonzero(res["new_state"] == 0)
    # after applyRes, state_energy is what linearize() returned (NewEnergy, or the kept energy if OOB)
    e_expect = res["state_energy"].astype(np.float64).sum()
    assert abs(e[0] - e_expect) <= 1e-9 * abs(e_expect)
    # setNewFrameEnergyTH: nth_element over NewEnergyWithOutlier >= 0 of residuals into the newest frame
    sel = (w.res_target == w.n_frames - 1) & (res["new_energy_wo"] >= 0)
    vals = res["new_energy_wo"][sel].astype(np.float32)
    nth = int(np.float32(0.7) * np.float32(len(vals)))
    v = np.float32(np.sqrt(np.partition(vals, nth)[nth]))
    th = np.float32(26.0 * 0.5) + (v * np.float32(1.5)) * np.float32(0.5)
    th = th * th
    assert ow.frame_energy_th()[-1] == th
    np.testing.assert_array_equal(ow.frame_energy_th()[:-1], w.frame_energy_th[:-1])


def test_single_and_multi_thread_paths_agree():
    """NUM_THREADS=6 IndexThreadReduce vs the multiThreading=false path (tid = -1 stitch)."""
    cfg = dict(n_frames=6, n_points=700, width=320, height=240, seed=19)
    o1 = oracle.OracleWindow(synth.make_window(**cfg), threads=0)
    e1, s1 = o1.iteration()
    o6 = oracle.OracleWindow(synth.make_window(**cfg), threads=6)
    e6, s6 = o6.iteration()
    oracle.set_threads(0)
    assert e1[2] == e6[2] and abs(e1[0] - e6[0]) <= 1e-12 * abs(e1[0])
    for k in ("HA", "bA", "Hsc", "bsc"):
        assert rel(s6[k], s1[k]) < 1e-6
    np.testing.assert_array_equal(o1.residuals()["new_state"], o6.residuals()["new_state"])


def _solve_inputs(H, b, n):
    Z = np.zeros((n, n))
    z = np.zeros(n)
    return dict(HA=H, bA=b, HL=Z, bL=z, Hsc=Z, bsc=z)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ldlt_solver_known_answer(seed):
    """solveSystemF's LDLT (Eigen::LDLT, symmetric pivoting) against numpy on SPD systems that
    need pivoting (diagonal spanning 1e-3..1e6): x = (H (1+lambda on diag))^-1 b."""
    rng = np.random.default_rng(seed)
    N = 4
    n = 8 * N + 4
    A = rng.standard_normal((n, n))
    D = np.diag(10.0 ** rng.uniform(-3, 6, n))
    H = D @ (A @ A.T + n * np.eye(n)) @ D
    b = rng.standard_normal(n)
    x = oracle.solve_system(N, 0, 1e-5, _solve_inputs(H, b, n))
    Hl = H.copy()
    Hl[np.diag_indices(n)] *= 1 + 1e-5
    xr = np.linalg.solve(Hl, b)
    assert np.linalg.norm(x - xr) <= 1e-9 * np.linalg.norm(xr)


def test_orthogonalize_known_answer():
    """orthogonalize (EnergyFunctional.cc:809-841): x minus its projection on span(N)."""
    rng = np.random.default_rng(5)
    N = 3
    n = 8 * N + 4
    A = rng.standard_normal((n, n))
    H = A @ A.T + n * np.eye(n)
    b = rng.standard_normal(n)
    ns = rng.standard_normal((7, n))
    x0 = oracle.solve_system(N, 0, 1e-5, _solve_inputs(H, b, n))
    x2 = oracle.solve_system(N, 2, 1e-5, _solve_inputs(H, b, n), nullspaces=ns)
    Q, _ = np.linalg.qr(ns.T)
    assert np.linalg.norm(x2 - (x0 - Q @ (Q.T @ x0))) <= 1e-10 * np.linalg.norm(x0)


def test_solver_backward_stable_on_ba_system(win):
    """On the (gauge-deficient) BA system itself: the Jacobi-scaled solve has a small backward
    error, ||H x - b|| <= 1e-12 ||H|| ||x||."""
    w, s = win["w"], win["sys"]
    n = w.dim
    x = oracle.solve_system(w.n_frames, 0, 1e-5, s)
    sym = lambda M: np.triu(M) + np.triu(M, 1).T  # the solve reads the upper triangles
    H = sym(s["HL"] + s["HA"])
    H[np.diag_indices(n)] *= 1 + 1e-5
    H -= sym(s["Hsc"]) * (1.0 / (1 + 1e-5))
    b = s["bL"] + s["bA"] - s["bsc"] / (1 + 1e-5)
    assert np.linalg.norm(H @ x - b) <= 1e-12 * np.linalg.norm(H, 2) * np.linalg.norm(x)


def test_resubstitute_known_answer(win):
    """resubstituteFPt (EnergyFunctional.cc:638-667): step_p = -(b_d - h_pd . x) / H_dd / (1 + lambda),
    with h_pd, H_dd, b_d rebuilt densely from the Jacobians (priorF = 0 in the synthetic set)."""
    w, J, res = win["w"], win["J"], win["res"]
    pts = []
    dense_system(w, J, res, pts)
    rng = np.random.default_rng(3)
    x = rng.standard_normal(w.dim) * 1e-3
    ow = oracle.OracleWindow(synth.make_window(**win["cfg"]), threads=0)
    ow.iteration()
    step = ow.resubstitute(x, 1e-5)
    exp = np.array([-(bd - hpd @ x) / hdd / (1 + 1e-5) if hdd > 0 else 0.0 for hpd, hdd, bd in pts])
    act = np.array([hdd > 0 for _, hdd, _ in pts])
    assert np.array_equal(step[~act], np.zeros((~act).sum()))
    assert np.linalg.norm(step[act] - exp[act]) <= 1e-5 * np.linalg.norm(exp[act])


# pattern 8 of staticPattern (Setting.cc:275); settings from Setting.cc:39-76
_PATTERN8 = np.array([[0, -2], [-1, -1], [1, -1], [-2, 0], [0, 0], [2, 0], [-1, 1], [0, 2]], np.float64)
_TH_SUM_COMPONENT, _HUBER_TH = 50.0 * 50.0, 9.0


def _photometric_residual(w, p, t):
    """PointFrameResidual::linearize's photometric part (Residuals.cc:48-208), restated in float64
    numpy from the reference text alone: the centre projection with the FEJ pose
    (ResidualProjections.h:57-84), the 8 pattern projections with PRE_KRKiTll / PRE_KtTll
    (ResidualProjections.h:24-33), bilinear dI (GlobalFuncs.h:90-103), the gradient weight, the
    Huber weight and the outlier test.  Returns (state, energy_wo, resF[8], JIdx[2,8], JabF[2,8],
    margin, tol): margin is how far the decisive quantity sits from a branch point (relative), so
    the caller can skip cases float32 rounding may legitimately flip; tol holds first-order error
    bounds of a float32 evaluation (energy, resF[8]): a pattern position carries ~1e-4 px of
    rounding (a few float32 ops at |K u| ~ 1e2), which the image gradient turns into an intensity
    error of 1e-4 (|dx| + |dy|), plus 1e-4 for I - (a c + b) cancelling two ~1e2 values; the position
    error grows with the coordinates' magnitude (x W / 320 for wider frames, e.g. KITTI's 1232)."""
    N, W, H = w.n_frames, w.width, w.height
    h = int(w.point_host[p])
    pre = w.precalc[h + N * t].astype(np.float64)
    pd = w.point_data[p].astype(np.float64)
    fx, fy, cx, cy = w.calib.astype(np.float64)
    wM3, hM3 = W - 3.0, H - 3.0
    margins = []

    klip = np.array([(pd[0] - cx) / fx, (pd[1] - cy) / fy, 1.0])
    ptp = pre[12:21].reshape(3, 3) @ klip + pre[21:24] * pd[3]
    Ku, Kv = ptp[0] / ptp[2] * fx + cx, ptp[1] / ptp[2] * fy + cy
    margins += [Ku - 1.1, Kv - 1.1, wM3 - Ku, hM3 - Kv]
    if not (ptp[2] > 0 and Ku > 1.1 and Kv > 1.1 and Ku < wM3 and Kv < hM3):
        return 1, -1.0, None, None, None, min(abs(m) for m in margins), None

    KRKi, Kt = pre[0:9].reshape(3, 3), pre[9:12]
    aff, b0 = pre[24:26], pre[26]
    dI = w.dI[t].astype(np.float64)
    e, wJI2 = 0.0, 0.0
    resF, JIdx, JabF = np.zeros(8), np.zeros((2, 8)), np.zeros((2, 8))
    tol_e, tol_r = 1e-5, np.zeros(8)
    pos_err = 1e-4 * max(1.0, max(W, H) / 320.0)  # float32 position rounding grows with |K u|
    for i, (dx, dy) in enumerate(_PATTERN8):
        q = KRKi @ np.array([pd[0] + dx, pd[1] + dy, 1.0]) + Kt * pd[2]
        Ku, Kv = q[0] / q[2], q[1] / q[2]
        margins += [Ku - 1.1, Kv - 1.1, wM3 - Ku, hM3 - Kv]
        if not (Ku > 1.1 and Kv > 1.1 and Ku < wM3 and Kv < hM3):
            return 1, -1.0, None, None, None, min(abs(m) for m in margins), None
        ix, iy = int(Ku), int(Kv)
        fxr, fyr = Ku - ix, Kv - iy
        b = ix + iy * W
        hit = (fxr * fyr * dI[b + 1 + W] + (fyr - fxr * fyr) * dI[b + W] + (fxr - fxr * fyr) * dI[b + 1]
               + (1 - fxr - fyr + fxr * fyr) * dI[b])
        color = pd[8 + i]
        r = hit[0] - (aff[0] * color + aff[1])
        wg = np.sqrt(_TH_SUM_COMPONENT / (_TH_SUM_COMPONENT + hit[1] ** 2 + hit[2] ** 2))
        wg = 0.5 * (wg + pd[16 + i])
        hw = 1.0 if abs(r) < _HUBER_TH else _HUBER_TH / abs(r)
        margins.append((abs(r) - _HUBER_TH) / _HUBER_TH)
        e += wg * wg * hw * r * r * (2 - hw)
        # the bilinear intensity's slope inside the cell is a convex combination of these differences
        sx = max(abs(dI[b + 1, 0] - dI[b, 0]), abs(dI[b + 1 + W, 0] - dI[b + W, 0]), abs(hit[1]))
        sy = max(abs(dI[b + W, 0] - dI[b, 0]), abs(dI[b + 1 + W, 0] - dI[b + 1, 0]), abs(hit[2]))
        dI_err = 1e-4 + pos_err * (sx + sy)
        tol_e += 4 * wg * wg * abs(r) * dI_err + 1e-5 * wg * wg * hw * r * r
        hw = (np.sqrt(hw) if hw < 1 else hw) * wg
        resF[i] = r * hw
        tol_r[i] = 2 * hw * dI_err + 1e-5 * abs(resF[i])
        JIdx[:, i] = hit[1:] * hw
        JabF[:, i] = ((color - b0) * hw, hw)
        wJI2 += hw * hw * (hit[1] ** 2 + hit[2] ** 2)
    th = max(float(w.frame_energy_th[h]), float(w.frame_energy_th[t]))
    margins += [(e - th) / th, (wJI2 - 2) / 2]
    state = 2 if (e > th or wJI2 < 2) else 0
    return state, e, resF, JIdx, JabF, min(abs(m) for m in margins), (tol_e, tol_r)


def test_photometric_residuals_known_answer(win):
    """The oracle's linearize (states, NewEnergyWithOutlier, resF, JIdx, JabF) against a float64
    numpy restatement of Residuals.cc:48-208 on every residual of the window (all three states;
    the largest error measured is 0.6 of the bound for resF, 0.14 for the energies).
    Tolerance: float32 arithmetic vs float64 — energies and resF within the first-order float32
    error bound _photometric_residual derives per residual, JIdx / JabF within 2e-4 of the row's
    largest entry (x W / 320 for frames wider than 320: position rounding); cases within 1e-4 of a
    branch point are skipped."""
    w, J, res = win["w"], win["J"], win["res"]
    seen = {0: 0, 1: 0, 2: 0}
    jtol = 2e-4 * max(1.0, max(w.width, w.height) / 320.0)  # the position rounding, as in _photometric_residual
    for k in range(w.n_residuals):
        p = int(np.searchsorted(w.point_res_begin, k, side="right") - 1)
        t = int(w.res_target[k])
        if w.res_state[k] == 1:  # linearize returns at once for a residual already OOB (Residuals.cc:18-22)
            assert res["new_state"][k] == 1 and res["new_energy_wo"][k] == -1
            seen[1] += 1
            continue
        state, e, resF, JIdx, JabF, margin, tol = _photometric_residual(w, p, t)
        if margin < 1e-4:
            continue
        assert res["new_state"][k] == state, (k, state)
        seen[state] += 1
        if state == 1:
            continue
        assert abs(res["new_energy_wo"][k] - e) <= tol[0], (k, res["new_energy_wo"][k], e, tol[0])
        Jk = unpack_J(J[k])
        assert np.all(np.abs(Jk["resF"] - resF) <= tol[1]), (k, Jk["resF"] - resF, tol[1])
        np.testing.assert_allclose(Jk["JIdx"], JIdx, rtol=0, atol=jtol * max(np.abs(JIdx).max(), 1e-3))
        np.testing.assert_allclose(Jk["JabF"], JabF, rtol=0, atol=jtol * max(np.abs(JabF).max(), 1e-3))
    assert seen[0] >= 1000 and seen[1] >= 10 and seen[2] >= 10, seen
