"""Marginalisation.

* EnergyFunctional::marginalizeFrame (EnergyFunctional.cc:109-191): ldso_ba_marginalize_frame is
  host C++; it is checked against a numpy Schur complement (the Jacobi scaling and the SVD
  pseudo-inverse of invertPosDef do not change the complement of a positive definite block).
* Point marginalisation (FullSystem::flagPointsForRemoval, FullSystem.cc:1384-1404, with
  PointFrameResidual::fixLinearizationF, Residuals.cc:219-245, and
  EnergyFunctional::marginalizePointsF, EnergyFunctional.cc:205-262): the oracle restatement is
  pinned by two known answers (with zero deltas res_toZeroF == resF, so M - Msc equals an ordinary
  pass over the same points; H does not depend on the deltas and b is affine in them); the GPU
  (ldso_ba_load_marginalization + ldso_ba_marginalize_points, images borrowed from the parent
  context) matches the oracle: residual states, JpJdF, HdiF, bdSumF bit for bit, H and b per
  8x8 block within 1e-4 (float accumulation order, as test_gpu_parity).  Parity unpinned by the
  reference itself (no golden vectors; unbuildable here).
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from ldso_amd import _lib as L
from ldso_amd import dist as ldist
from ldso_amd import synth

BLOCK_TOL = 1e-4


def ad_ht_delta(w, scale=1.0):
    """EnergyFunctional::setDeltaF's adHTdeltaF [h + N t] = delta_h^T adHostF + delta_t^T adTargetF."""
    N = w.n_frames
    d = (np.asarray(w.frame_delta) * scale).astype(np.float32)
    adH = np.asarray(w.ad_host).astype(np.float32).reshape(N * N, 8, 8)
    adT = np.asarray(w.ad_target).astype(np.float32).reshape(N * N, 8, 8)
    out = np.zeros((N * N, 8), np.float32)
    for h in range(N):
        for t in range(N):
            i = h + N * t
            out[i] = d[h] @ adH[i] + d[t] @ adT[i]
    return out


def block_err(G, O, N):
    edges = [0, 4] + [4 + 8 * (f + 1) for f in range(N)]
    scale = np.linalg.norm(O)
    worst = 0.0
    for a in range(len(edges) - 1):
        for b in range(len(edges) - 1):
            g = G[edges[a]:edges[a + 1], edges[b]:edges[b + 1]]
            o = O[edges[a]:edges[a + 1], edges[b]:edges[b + 1]]
            worst = max(worst, np.linalg.norm(g - o) / max(np.linalg.norm(o), 1e-9 * scale, 1e-300))
    return worst


def vec_err(g, o, N):
    edges = [0, 4] + [4 + 8 * (f + 1) for f in range(N)]
    scale = np.linalg.norm(o)
    return max(np.linalg.norm(g[a:b] - o[a:b]) / max(np.linalg.norm(o[a:b]), 1e-9 * scale, 1e-300)
               for a, b in zip(edges[:-1], edges[1:]))


def marg_points(w, every=5):
    """host frame 0's points (the frame being marginalised) plus every `every`-th other point"""
    P = w.n_points
    return np.array(sorted(set(np.flatnonzero(w.point_host == 0)) | set(range(0, P, every))), np.int64)


# ------------------------------------------------------------------------------------------
# CPU
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("idx", [0, 2, 4])
def test_marginalize_frame_known_answer(built, idx):
    rng = np.random.default_rng(11 + idx)
    N = 5
    n = 8 * N + 4
    A = rng.standard_normal((n, n))
    Dg = np.diag(10.0 ** rng.uniform(-1, 4, n))
    HM = np.ascontiguousarray(Dg @ (A @ A.T + n * np.eye(n)) @ Dg)
    bM = rng.standard_normal(n) * 100
    prior = 10.0 ** rng.uniform(0, 6, 8)
    dprior = rng.standard_normal(8) * 1e-3
    Ho = np.zeros((n - 8, n - 8))
    bo = np.zeros(n - 8)
    lib = L.lib()
    rc = lib.ldso_ba_marginalize_frame(N, idx, L.ptr(HM, L.f64p), L.ptr(bM, L.f64p), L.ptr(prior, L.f64p),
                                       L.ptr(dprior, L.f64p), L.ptr(Ho, L.f64p), L.ptr(bo, L.f64p))
    assert rc == 0
    fr = np.arange(4 + 8 * idx, 4 + 8 * idx + 8)
    keep = np.setdiff1d(np.arange(n), fr)
    Hbb = HM[np.ix_(fr, fr)] + np.diag(prior)
    bb = bM[fr] + prior * dprior
    Hab = HM[np.ix_(keep, fr)]
    Hr = HM[np.ix_(keep, keep)] - Hab @ np.linalg.solve(Hbb, Hab.T)
    br = bM[keep] - Hab @ np.linalg.solve(Hbb, bb)
    assert np.abs(Ho - Hr).max() <= 1e-9 * np.abs(Hr).max()
    assert np.abs(bo - br).max() <= 1e-9 * np.abs(br).max()
    np.testing.assert_array_equal(Ho, Ho.T)
    assert lib.ldso_ba_marginalize_frame(N, N, L.ptr(HM, L.f64p), L.ptr(bM, L.f64p), L.ptr(prior, L.f64p),
                                         L.ptr(dprior, L.f64p), L.ptr(Ho, L.f64p), L.ptr(bo, L.f64p)) < 0


def _zero_deltas(w):
    w.c_delta = np.zeros(4, np.float32)
    w.point_data = w.point_data.copy()
    w.point_data[:, 5] = 0  # deltaF
    return w


def test_oracle_marginalization_zero_delta_is_a_pass(built):
    """With every delta zero fixLinearizationF leaves res_toZeroF == resF, so marginalizePointsF's
    M - Msc equals an ordinary pass over the same points (priorF scaled, no prior shift)."""
    w = _zero_deltas(synth.make_window(n_frames=5, n_points=200, width=320, height=240, seed=21))
    S = marg_points(w)
    ow = oracle.OracleWindow(w, threads=0)
    H, b = ow.marginalize_points(S.astype(np.int32), np.zeros((25, 8), np.float32))
    sub = ldist.subset_window(w, S)
    sub.point_data = sub.point_data.copy()
    sub.point_data[:, 4] *= np.float32(600.0 * 600.0)  # setting_idepthFixPriorMargFac
    os_ = oracle.OracleWindow(sub, threads=0)
    os_.reset_oob()
    _, sysm = os_.iteration()
    np.testing.assert_allclose(H, sysm["HA"] - sysm["Hsc"], rtol=0, atol=1e-9 * np.abs(H).max())
    np.testing.assert_allclose(b, sysm["bA"] - sysm["bsc"], rtol=0, atol=1e-9 * np.abs(b).max())


def test_oracle_marginalization_affine_in_delta(built):
    """H does not depend on the linearisation deltas; b is affine in them."""
    w = _zero_deltas(synth.make_window(n_frames=5, n_points=200, width=320, height=240, seed=22))
    S = marg_points(w).astype(np.int32)
    D1 = ad_ht_delta(w, 1.0)
    D1[:, :6] += np.float32(1e-3)  # an explicit frame delta so the b shift is well above rounding
    outs = [oracle.OracleWindow(w, threads=0).marginalize_points(S, D1 * np.float32(s)) for s in (0.0, 1.0, 2.0)]
    (H0, b0), (H1, b1), (H2, b2) = outs
    np.testing.assert_array_equal(H0, H1)
    np.testing.assert_array_equal(H0, H2)
    d1, d2 = b1 - b0, b2 - b1
    assert np.linalg.norm(d1) > 1e-6 * np.linalg.norm(b0)
    assert np.linalg.norm(d2 - d1) <= 1e-3 * np.linalg.norm(d1)


def test_marginalization_load_errors(built):
    lib = L.lib()
    w = synth.make_window(n_frames=3, n_points=10, width=160, height=120, seed=1)
    s = w.c_struct(with_images=False)
    assert lib.ldso_ba_load_marginalization(None, None, 0, C.byref(s)) < 0
    assert lib.ldso_ba_marginalize_points(None, None, None, None) < 0


# ------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [dict(n_frames=5, n_points=300, seed=31), dict(n_frames=7, n_points=600, seed=32)])
def test_gpu_marginalize_points_matches_oracle(built, cfg):
    from ldso_amd import BAContext

    w = synth.make_window(width=640, height=480, **cfg)
    N = w.n_frames
    S = marg_points(w)
    adh = ad_ht_delta(w)
    parent = BAContext(0).load([w])
    parent.linearize()  # an ordinary pass first, as optimize() precedes flagPointsForRemoval
    parent.sync()
    before = parent.system(0)
    sub = ldist.subset_window(w, S)
    m = BAContext(0).load_marginalization(parent, 0, sub)
    H, b = m.marginalize_points(adh)

    ow = oracle.OracleWindow(synth.make_window(width=640, height=480, **cfg), threads=0)
    Ho, bo = ow.marginalize_points(S.astype(np.int32), adh)
    assert block_err(H, Ho, N) <= BLOCK_TOL
    assert vec_err(b, bo, N) <= BLOCK_TOL
    assert np.abs(H - H.T).max() <= 1e-12 * np.abs(H).max()

    rg, ro = m.residuals(0), ow.residuals()
    rs = np.concatenate([np.arange(w.point_res_begin[p], w.point_res_begin[p + 1]) for p in S])
    for k in ("new_state", "state", "flags", "state_energy", "center"):
        np.testing.assert_array_equal(rg[k], ro[k][rs], err_msg=k)
    act = (ro["flags"][rs] & 1).astype(bool)
    assert act.sum() > 0.5 * len(rs)
    np.testing.assert_array_equal(rg["jpjdf"][act], ro["jpjdf"][rs][act])
    pg, po = m.points(0), ow.points()
    for k in ("HdiF", "bdSumF", "idepth_hessian"):
        np.testing.assert_array_equal(pg[k], po[k][S], err_msg=k)

    # the parent window is untouched: the same pass gives the same system
    parent.linearize()
    after = parent.system(0)
    for k in ("HA", "Hsc"):
        assert block_err(after[k], before[k], N) <= 1e-12
    m.close()
    parent.close()


@pytest.mark.gpu
def test_gpu_marginalization_window_must_match_parent(built):
    from ldso_amd import BAContext

    w = synth.make_window(n_frames=5, n_points=100, width=320, height=240, seed=33)
    parent = BAContext(0).load([w])
    other = synth.make_window(n_frames=4, n_points=50, width=320, height=240, seed=34)
    with pytest.raises(RuntimeError, match="parent"):
        BAContext(0).load_marginalization(parent, 0, other)
    with pytest.raises(RuntimeError, match="marginalisation context"):
        parent.marginalize_points(np.zeros((25, 8), np.float32))
    parent.close()
