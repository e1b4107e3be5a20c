"""Coarse tracker: FrameHessian::makeImages, CoarseTracker::makeK,
calcRes and calcGSSSE (src/frontend/CoarseTracker.cc:312-339, 540-741; FrameHessian.cc:59-115).

CPU tests pin the oracle restatement (oracle/ldso_oracle_tracker.cpp) with known answers that
do not share its code: a numpy makeImages, an identity-pose calcRes (zero residual), a float64
calcGSSSE from the warped buffers, and finite differences of the calcRes energy against the
calcGSSSE gradient b (the Jacobian's sign, order and SCALE_* factors).  Parity unpinned by the
reference itself (no golden vectors; unbuildable here).

GPU tests compare include/ldso_ct.h against the oracle: pyramid images, absSquaredGrad and the
warped buffers bit for bit; calcRes Vec6 within 1e-5 relative (the reference sums E in float in
point order, the GPU sums in double by blocks); calcGSSSE H and b within 1e-5 of their largest
entry (Accumulator9's SSE-lane float sums vs the GPU's double block sums)."""
import numpy as np
import pytest

import oracle
from ldso_amd import synth

CALIB_640 = np.array([384.0, 432.0, 319.5, 239.5], np.float32)  # EUROC.txt relative 0.6/0.9/0.5/0.5


def np_make_images(color, w, h):
    """FrameHessian::makeImages restated in numpy (no shared code with the oracle)."""
    L = oracle.ct_levels(w, h)
    out = []
    I = np.asarray(color, np.float32).reshape(h, w)
    for l in range(L):
        wl, hl = w >> l, h >> l
        if l > 0:
            P = out[-1][0][:, 0].reshape(hl * 2, wl * 2)
            I = (np.float32(0.25) * (((P[0::2, 0::2] + P[0::2, 1::2]) + P[1::2, 0::2]) + P[1::2, 1::2])).astype(np.float32)
        f = I.reshape(-1)
        dI = np.zeros((wl * hl, 3), np.float32)
        dI[:, 0] = f
        ag = np.zeros(wl * hl, np.float32)
        idx = np.arange(wl, wl * (hl - 1))
        dx = (np.float32(0.5) * (f[idx + 1] - f[idx - 1])).astype(np.float32)
        dy = (np.float32(0.5) * (f[idx + wl] - f[idx - wl])).astype(np.float32)
        dx[np.isnan(dx) | (np.abs(dx) > 255)] = 0
        dy[np.isnan(dy) | (np.abs(dy) > 255)] = 0
        dI[idx, 1] = dx
        dI[idx, 2] = dy
        ag[idx] = dx * dx + dy * dy
        out.append((dI, ag))
    return out


def scene(w=640, h=480, seed=0):
    color, make_pc = synth.make_tracker_scene(w, h, seed=seed)
    levels = oracle.make_images(color, w, h)
    pcs = make_pc([dI[:, 0] for dI, _ in levels])
    calib = CALIB_640 * np.float32(w / 640)
    calib[2], calib[3] = (w - 1) / 2, (h - 1) / 2
    K = oracle.ct_make_k(calib, w, h)
    return color, levels, pcs, calib, K


def pose(i=0, scale=1.0):
    rng = np.random.default_rng(100 + i)
    return synth.se3_matrix(rng.normal(0, 2e-3, 3) * scale, rng.normal(0, 1e-2, 3) * scale)


AFF6 = (1.0, 1.0, 0.02, 3.0, 0.05, 1.0)  # ref exposure, new exposure, ref (a, b), new (a, b)


def pc_tuple(pc):
    return (pc["u"], pc["v"], pc["idepth"], pc["color"])


# ------------------------------------------------------------------------------------------
# CPU: the oracle against independent known answers
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("wh", [(640, 480), (752, 480), (320, 240), (1232, 368)])
def test_oracle_make_images_known_answer(built, wh):
    w, h = wh
    color, _ = synth.make_tracker_scene(w, h, seed=3)
    color = color.copy()
    color[5, 7] = np.nan  # NaN and huge steps: the |d| > 255 / isnan guards
    color[100, 100] = 4000.0
    got = oracle.make_images(color, w, h)
    ref = np_make_images(color, w, h)
    assert len(got) == oracle.ct_levels(w, h)
    for (a, ag), (b, bg) in zip(got, ref):
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(ag, bg)


def test_levels_and_k_follow_global_calib():
    assert oracle.ct_levels(640, 480) == 4  # pyrLevelsUsed for 640x480 (GlobalCalib.cc:20-30)
    assert oracle.ct_levels(752, 480) == 5
    assert oracle.ct_levels(1232, 368) == 5  # KITTI's cropped output: 77 x 23 is odd at level 4
    assert oracle.ct_levels(1242, 375) == 1  # an odd height never halves
    K = oracle.ct_make_k(CALIB_640, 640, 480)
    for l in range(4):
        fx, fy, cx, cy = K[l, :4]
        assert fx == np.float32(384.0 / 2 ** l) and fy == np.float32(432.0 / 2 ** l)
        assert abs(cx - ((319.5 + 0.5) / 2 ** l - 0.5)) < 1e-5
        Km = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float64)
        np.testing.assert_allclose(K[l, 4:].reshape(3, 3) @ Km, np.eye(3), atol=1e-6)


def test_oracle_calc_res_identity_is_photo_consistent(built):
    color, levels, pcs, calib, K = scene(320, 240)
    T = np.hstack([np.eye(3), np.zeros((3, 1))])
    for l, (dI, _) in enumerate(levels):
        wl, hl = 320 >> l, 240 >> l
        rs, warped = oracle.ct_calc_res(l, wl, hl, K[l], dI, pc_tuple(pcs[l]), T, (1, 1, 0, 0, 0, 0), 20.0)
        u, v = pcs[l]["u"], pcs[l]["v"]
        lo = ((u > 2) & (v > 2) & (u < wl - 3) & (v < hl - 3)).sum()  # points on the bound line round
        hi = ((u >= 2) & (v >= 2) & (u <= wl - 3) & (v <= hl - 3)).sum()  # either way through K Ki
        assert lo <= rs[1] <= hi and rs[5] == 0
        assert rs[0] < 1e-6 * hi
        assert warped.shape[0] % 4 == 0 and np.abs(warped[:, 5]).max() < 1e-3
        if l == 0:
            assert rs[2] < 1e-8 and rs[4] < 1e-8  # no translation, no motion (float rounding only)


def test_oracle_calc_gs_matches_float64_sum(built):
    color, levels, pcs, calib, K = scene(320, 240)
    l = 1
    T = pose(0)
    rs, warped = oracle.ct_calc_res(l, 160, 120, K[l], levels[l][0], pc_tuple(pcs[l]), T, AFF6, 20.0)
    H, b = oracle.ct_calc_gs(warped, K[l, 0], K[l, 1], AFF6)
    a = np.float32(np.exp(np.float32(AFF6[4] - AFF6[2])))
    W = warped.astype(np.float64)
    idp, u, v, gx, gy, r, wt, rc = W.T
    dx, dy = gx * K[l, 0], gy * K[l, 1]
    J = np.stack([idp * dx, idp * dy, -idp * (u * dx + v * dy), -(u * v * dx + dy * (1 + v * v)),
                  u * v * dy + dx * (1 + u * u), u * dy - v * dx, a * (AFF6[3] - rc), -np.ones_like(u)], 1)
    n = W.shape[0]
    s = np.array([0.5, 0.5, 0.5, 1, 1, 1, 10, 1000])
    Hr = (J * wt[:, None]).T @ J / n * np.outer(s, s)
    br = (J * (wt * r)[:, None]).sum(0) / n * s
    assert np.abs(H - Hr).max() <= 1e-5 * np.abs(Hr).max()
    assert np.abs(b - br).max() <= 1e-5 * np.abs(br).max()
    np.testing.assert_array_equal(H, H.T)


def test_oracle_calc_gs_gradient_matches_finite_differences(built):
    """In the quadratic Huber regime, d E / d xi_k = 2 n b_k / scale_k for the left increment
    refToNew' = exp(xi) refToNew (Sophus order: translation, rotation) and the new frame's
    affine (a, b): pins the Jacobian's sign, ordering and SCALE_* factors."""
    color, levels, pcs, calib, K = scene(640, 480, seed=1)
    l = 0
    wl, hl = 640, 480
    T0 = pose(2, 0.1)
    aff = np.array([1.0, 1.0, 0.0, 0.5, 0.01, 0.5])
    rs, warped = oracle.ct_calc_res(l, wl, hl, K[l], levels[l][0], pc_tuple(pcs[l]), T0, aff, 1e6)
    assert np.abs(warped[:, 5]).max() < 9  # all inliers of the Huber kernel (hw = 1)
    H, b = oracle.ct_calc_gs(warped, K[l, 0], K[l, 1], aff)
    n = warped.shape[0]
    s = np.array([0.5, 0.5, 0.5, 1, 1, 1, 10, 1000])
    grad = 2 * n * b / s

    def E(xi, da=0.0, db=0.0):
        T = synth.se3_matrix(xi[3:], xi[:3])
        T4 = np.vstack([T, [0, 0, 0, 1]]) @ np.vstack([T0, [0, 0, 0, 1]])
        a6 = aff.copy()
        a6[4] += da
        a6[5] += db
        return oracle.ct_calc_res(l, wl, hl, K[l], levels[l][0], pc_tuple(pcs[l]), T4[:3], a6, 1e6)[0][0]

    fd = np.zeros(8)
    for k in range(6):
        eps = 1e-4 if k < 3 else 1e-4
        e = np.zeros(6)
        e[k] = eps
        fd[k] = (E(e) - E(-e)) / (2 * eps)
    fd[6] = (E(np.zeros(6), da=1e-4) - E(np.zeros(6), da=-1e-4)) / 2e-4
    fd[7] = (E(np.zeros(6), db=1e-3) - E(np.zeros(6), db=-1e-3)) / 2e-3
    # bilinear interpolation vs central-difference image gradients: a few % on smooth images
    rel = np.abs(fd - grad) / np.abs(grad).max()
    assert rel[:6].max() < 0.05, (fd, grad)
    assert abs(fd[6] - grad[6]) <= 1e-3 * abs(grad[6]) + 1e-6 * np.abs(grad).max()
    assert abs(fd[7] - grad[7]) <= 1e-3 * abs(grad[7]) + 1e-6 * np.abs(grad).max()


# ------------------------------------------------------------------------------------------
# GPU: include/ldso_ct.h against the oracle
# ------------------------------------------------------------------------------------------
def _tracker(w, h, color, pcs, calib, B=None):
    from ldso_amd.tracker import CoarseTracker

    ct = CoarseTracker(w, h)
    ct.make_k(calib)
    ct.set_new_frame(color, 1.0, B)
    ct.set_reference([pc_tuple(p) for p in pcs], 1.0, AFF6[2:4])
    return ct


@pytest.mark.gpu
@pytest.mark.parametrize("wh", [(640, 480), (752, 480), (1232, 368)])
@pytest.mark.parametrize("with_b", [False, True])
def test_gpu_make_images_bit_exact(built, wh, with_b):
    from ldso_amd.tracker import CoarseTracker

    w, h = wh
    color, _ = synth.make_tracker_scene(w, h, seed=4)
    B = (255 * (np.linspace(0, 1, 256) ** 0.8)).astype(np.float32) if with_b else None
    ref = oracle.make_images(color, w, h, B)
    ct = CoarseTracker(w, h)
    assert ct.levels == len(ref)
    K = ct.make_k(CALIB_640)
    np.testing.assert_array_equal(K, oracle.ct_make_k(CALIB_640, w, h))
    ct.set_new_frame(color, 1.0, B)
    for l, (dI, ag) in enumerate(ref):
        gdI, gag = ct.frame_level(l)
        np.testing.assert_array_equal(gdI, dI)
        np.testing.assert_array_equal(gag, ag)
    ct.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,wh", [(0, (640, 480)), (1, (640, 480)), (2, (1232, 368))])
def test_gpu_calc_res_and_gs_match_oracle(built, seed, wh):
    w, h = wh
    color, levels, pcs, calib, K = scene(w, h, seed)
    ct = _tracker(w, h, color, pcs, calib)
    for l in range(len(levels)):
        wl, hl = w >> l, h >> l
        for i, cutoff in ((seed, 20.0), (seed + 7, 8.0)):
            T = pose(i, 2.0 ** l)
            rs_o, warped_o = oracle.ct_calc_res(l, wl, hl, K[l], levels[l][0], pc_tuple(pcs[l]), T, AFF6, cutoff)
            rs = ct.calc_res(l, T, AFF6[4:6], cutoff)
            assert rs[1] == rs_o[1]
            assert abs(rs[0] - rs_o[0]) <= 1e-5 * abs(rs_o[0]) + 1e-6
            np.testing.assert_allclose(rs[[2, 4]], rs_o[[2, 4]], rtol=1e-5, atol=1e-9)
            assert rs[3] == 0 and abs(rs[5] - rs_o[5]) <= 1e-7
            warped = ct.warped()
            np.testing.assert_array_equal(warped, warped_o)
            H, b = ct.calc_gs(l, T, AFF6[4:6])
            Ho, bo = oracle.ct_calc_gs(warped_o, K[l, 0], K[l, 1], AFF6)
            assert np.abs(H - Ho).max() <= 1e-5 * np.abs(Ho).max(), l
            assert np.abs(b - bo).max() <= 1e-5 * np.abs(bo).max(), l
    ct.close()


@pytest.mark.gpu
def test_gpu_calc_res_batch_equals_single_calls(built):
    w, h = 640, 480
    color, levels, pcs, calib, K = scene(w, h, 2)
    ct = _tracker(w, h, color, pcs, calib)
    Ts = np.stack([pose(i) for i in range(40)])
    ab = np.array([[0.05 + 0.01 * i, 1.0 - 0.1 * i] for i in range(40)])
    for l in (0, 2):
        rb = ct.calc_res_batch(l, Ts, ab, 20.0)
        for i in range(40):
            np.testing.assert_array_equal(rb[i], ct.calc_res(l, Ts[i], ab[i], 20.0))
    ct.close()


@pytest.mark.gpu
def test_gpu_fused_res_gs_equals_separate_calls(built):
    w, h = 640, 480
    color, levels, pcs, calib, K = scene(w, h, 3)
    ct = _tracker(w, h, color, pcs, calib)
    for l in range(ct.levels):
        for i in range(3):
            T = pose(10 + i, 2.0 ** l)
            rs, H, b = ct.calc_res_gs(l, T, AFF6[4:6], 20.0)
            rs2 = ct.calc_res(l, T, AFF6[4:6], 20.0)
            H2, b2 = ct.calc_gs(l, T, AFF6[4:6])
            np.testing.assert_array_equal(rs, rs2)
            np.testing.assert_array_equal(H, H2)
            np.testing.assert_array_equal(b, b2)
    ct.close()


@pytest.mark.gpu
def test_gpu_tracker_edge_cases(built):
    from ldso_amd.tracker import CoarseTracker

    w, h = 640, 480
    color, levels, pcs, calib, K = scene(w, h, 5)
    ct = CoarseTracker(w, h)
    with pytest.raises(RuntimeError, match="make_k"):
        ct.calc_res(0, pose(0))
    ct.make_k(calib)
    ct.set_new_frame(color)
    # empty levels and a level whose points all leave the image
    far = dict(u=np.full(5, 1000.0, np.float32), v=np.full(5, 1000.0, np.float32),
               idepth=np.ones(5, np.float32), color=np.ones(5, np.float32))
    empty = dict(u=np.zeros(0, np.float32), v=np.zeros(0, np.float32), idepth=np.zeros(0, np.float32),
                 color=np.zeros(0, np.float32))
    ct.set_reference([far, empty] + [pc_tuple(p) for p in pcs[2:]], 1.0, AFF6[2:4])
    with pytest.raises(RuntimeError, match="calcRes"):
        ct.calc_gs(0, pose(0))
    T = pose(0)
    for l in (0, 1):
        rs = ct.calc_res(l, T, AFF6[4:6], 20.0)
        rs_o, wo = oracle.ct_calc_res(l, w >> l, h >> l, K[l], levels[l][0],
                                      pc_tuple([far, empty][l]), T, AFF6, 20.0)
        assert rs[1] == 0 == rs_o[1] and wo.shape[0] == 0 and ct.warped().shape[0] == 0
        np.testing.assert_array_equal(np.isnan(rs), np.isnan(rs_o))  # 0/0 saturation fraction
        H, b = ct.calc_gs(l, T, AFF6[4:6])
    with pytest.raises(RuntimeError, match="level"):
        ct.calc_res(ct.levels, T)
    ct.close()
