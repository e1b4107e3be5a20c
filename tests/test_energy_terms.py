"""EnergyFunctional::setDeltaF (adHTdeltaF), calcMEnergyF and calcLEnergyF_MT (SURVEY.md §8 row
a18; EnergyFunctional.cc:473-498, 523-533, 751-806): the product's host helpers against the
oracle restatement (bit-exact: same statement order) and against numpy known answers."""
import numpy as np

import oracle
from ldso_amd import _lib as L
from ldso_amd import synth


def _frames(w):
    N = w.n_frames
    prior = np.zeros((N, 8))
    delta = np.zeros((N, 8))
    dprior = np.zeros((N, 8))
    fr = np.ascontiguousarray(w.frames)
    L.check(L.lib().ldso_ba_frame_take_data(N, fr.ctypes.data, None, L.ptr(prior, L.f64p), L.ptr(delta, L.f64p),
                                            L.ptr(dprior, L.f64p)))
    return prior, delta, dprior


def test_ad_ht_delta_matches_oracle_and_numpy(built):
    w = synth.make_window(n_frames=6, n_points=50, width=160, height=120, seed=5)
    N = w.n_frames
    _, delta, _ = _frames(w)
    delta[:, :6] += 1e-3 * np.arange(1, 7)  # every frame moved off its linearisation point
    out = np.zeros((N * N, 8), np.float32)
    L.check(L.lib().ldso_ba_ad_ht_delta(N, L.ptr(delta, L.f64p), L.ptr(w.ad_host, L.f64p),
                                        L.ptr(w.ad_target, L.f64p), L.ptr(out, L.f32p)))
    ref = np.zeros_like(out)
    oracle.lib().oracle_ad_ht_delta(N, oracle._p(delta, oracle.f64p), oracle._p(np.ascontiguousarray(w.ad_host),
                                    oracle.f64p), oracle._p(np.ascontiguousarray(w.ad_target), oracle.f64p),
                                    oracle._p(ref, oracle.f32p))
    np.testing.assert_array_equal(out, ref)
    adH = np.asarray(w.ad_host).reshape(N * N, 8, 8)
    adT = np.asarray(w.ad_target).reshape(N * N, 8, 8)
    for h in range(N):
        for t in range(N):
            i = h + N * t
            kat = delta[h] @ adH[i] + delta[t] @ adT[i]
            mag = np.abs(delta[h]) @ np.abs(adH[i]) + np.abs(delta[t]) @ np.abs(adT[i])  # float rounding scale
            assert np.all(np.abs(out[i] - kat) <= 1e-6 * mag + 1e-12)


def test_calc_m_energy(built):
    rng = np.random.default_rng(3)
    N = 5
    n = 8 * N + 4
    A = rng.standard_normal((n, n))
    HM = np.ascontiguousarray(A @ A.T)
    bM = rng.standard_normal(n)
    cd = rng.standard_normal(4).astype(np.float32)
    delta = rng.standard_normal((N, 8)) * 1e-2
    e = np.zeros(1)
    L.check(L.lib().ldso_ba_calc_m_energy(N, L.ptr(HM, L.f64p), L.ptr(bM, L.f64p), L.ptr(cd, L.f32p),
                                          L.ptr(delta, L.f64p), L.ptr(e, L.f64p)))
    eo = oracle.lib().oracle_calc_m_energy(N, oracle._p(HM, oracle.f64p), oracle._p(bM, oracle.f64p),
                                           oracle._p(cd, oracle.f32p), oracle._p(delta, oracle.f64p))
    assert e[0] == eo
    d = np.concatenate([cd.astype(np.float64), delta.ravel()])
    assert abs(e[0] - d @ (2 * bM + HM @ d)) <= 1e-12 * abs(d @ (HM @ d)) + 1e-12


def test_calc_l_energy(built):
    rng = np.random.default_rng(4)
    w = synth.make_window(n_frames=5, n_points=333, width=160, height=120, seed=6)
    N = w.n_frames
    prior, _, dprior = _frames(w)
    dprior[:, 6:] += 1e-3  # nonzero affine deltas so the frame priors contribute
    cp = np.full(4, 5e9)
    cd = (rng.standard_normal(4) * 1e-4).astype(np.float32)
    deltaF = (rng.standard_normal(w.n_points) * 1e-2).astype(np.float32)
    priorF = rng.uniform(0, 2500, w.n_points).astype(np.float32)
    e = np.zeros(1)
    L.check(L.lib().ldso_ba_calc_l_energy(N, L.ptr(prior, L.f64p), L.ptr(dprior, L.f64p), L.ptr(cp, L.f64p),
                                          L.ptr(cd, L.f32p), w.n_points, L.ptr(deltaF, L.f32p),
                                          L.ptr(priorF, L.f32p), L.ptr(e, L.f64p)))
    eo = oracle.lib().oracle_calc_l_energy(N, oracle._p(prior, oracle.f64p), oracle._p(dprior, oracle.f64p),
                                           oracle._p(cp, oracle.f64p), oracle._p(cd, oracle.f32p), w.n_points,
                                           oracle._p(deltaF, oracle.f32p), oracle._p(priorF, oracle.f32p))
    assert e[0] == eo
    kat = (dprior * prior * dprior).sum() + float((cd.astype(np.float64) ** 2 * cp).sum()) + \
        float((deltaF.astype(np.float64) ** 2 * priorF).sum())
    assert abs(e[0] - kat) <= 1e-5 * abs(kat)


def test_frame_delta_is_stable_for_small_rotations(built):
    """get_state_minus_stateZero (FrameHessian.h:59-64) through Sophus' atan-form SE3::log: finite
    and first-order exact for rotation increments down to 1e-12 (the 1 - cos form cancels to 0/0)."""
    w = synth.make_window(n_frames=3, n_points=10, width=160, height=120, seed=7)
    fr = np.ascontiguousarray(w.frames).copy()
    for mag in (1e-12, 1e-9, 1e-8, 1e-6, 1e-3):
        fr["state"][:] = fr["state_zero"]
        fr["state"][1, 3:6] += mag * np.array([1.0, -2.0, 0.5])
        fr["state"][1, 0:3] += mag * np.array([0.3, 0.1, -0.2])
        delta, pr, dp = np.zeros((3, 8)), np.zeros((3, 8)), np.zeros((3, 8))
        L.check(L.lib().ldso_ba_frame_take_data(3, fr.ctypes.data, None, L.ptr(pr, L.f64p), L.ptr(delta, L.f64p),
                                                L.ptr(dp, L.f64p)))
        od = np.zeros((3, 8))
        oracle.lib().oracle_frame_take_data(3, fr.ctypes.data, oracle._p(pr, oracle.f64p), oracle._p(od, oracle.f64p),
                                            oracle._p(dp, oracle.f64p))
        np.testing.assert_array_equal(delta, od)
        assert np.all(np.isfinite(delta))
        np.testing.assert_allclose(delta[1, 3:6], mag * np.array([1.0, -2.0, 0.5]), rtol=1e-3 if mag > 1e-10 else 0.2)
