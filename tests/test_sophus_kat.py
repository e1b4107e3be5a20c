"""The SE(3) arithmetic of the path against Sophus (thirdparty/Sophus/sophus/se3.hpp, so3.hpp).

LDSO keeps every pose as a Sophus SE3: a unit quaternion plus a translation.  The product's
se3.h (host helpers and the device frame step) and the oracle's restatement both keep that
representation and follow Sophus's statements.  Here a third restatement, written in plain Python
floats from the Sophus text (IEEE double, no fused multiply-add, libm's sin / cos / atan through
the math module), pins both:
  * first principles: exp against the matrix exponential of the twist (scipy), log(exp(xi)) = xi,
    exp / log / product / inverse / Adj identities, the small-angle and w ~ 0 branches;
  * the product's host helpers through the C ABI -- ldso_ba_frame_step (doStepFromBackup's
    log(exp(step) exp(state))), ldso_ba_frame_take_data (get_state_minus_stateZero),
    ldso_ba_set_adjoints (-Adj^T of target * host^-1) and ldso_ba_frame_precalc (the float
    rotation matrices of leftToLeft_0 and leftToLeft) -- to at most 4 ulp (measured: 0);
  * the oracle's doStepFromBackup states equal the product's.
Parity unpinned by the reference binary itself (Eigen is absent here): the reference
build may fuse a multiply-add where Eigen's packet code uses pmadd.
"""
import ctypes as C
import math

import numpy as np
import pytest

import oracle
from ldso_amd import _lib as L
from ldso_amd import synth

EPS = 1e-10  # Sophus::Constants<double>::epsilon() (common.hpp:144)


# ------------------------------------------------------------------------------------------
# Sophus, restated in Python floats.  Quaternions in Eigen's coeffs() order (x, y, z, w).
# ------------------------------------------------------------------------------------------
def q_normalize(q):  # SO3Base::normalize (so3.hpp:289-295), Eigen's norm as its packets sum it
    x, y, z, w = q
    n = math.sqrt((x * x + z * z) + (y * y + w * w))
    return (x / n, y / n, z / n, w / n)


def cross(a, b):  # Eigen's cross (OrthoMethods.h)
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def q_rotate(q, p):  # SO3 * point (so3.hpp:341-347)
    uv = cross(q[:3], p)
    uv = tuple(u + u for u in uv)
    c = cross(q[:3], uv)
    return tuple((p[i] + q[3] * uv[i]) + c[i] for i in range(3))


def q_matrix(q):  # Eigen's Quaternion::toRotationMatrix
    x, y, z, w = q
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return [[1.0 - (tyy + tzz), txy - twz, txz + twy],
            [txy + twz, 1.0 - (txx + tzz), tyz - twx],
            [txz - twy, tyz + twx, 1.0 - (txx + tyy)]]


def q_from_matrix(R):  # Eigen's Quaternion(Matrix3) (quaternionbase_assign_impl)
    t = (R[0][0] + R[1][1]) + R[2][2]
    q = [0.0, 0.0, 0.0, 0.0]
    if t > 0:
        t = math.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (R[2][1] - R[1][2]) * t
        q[1] = (R[0][2] - R[2][0]) * t
        q[2] = (R[1][0] - R[0][1]) * t
    else:
        i = 0
        if R[1][1] > R[0][0]:
            i = 1
        if R[2][2] > R[i][i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = math.sqrt(((R[i][i] - R[j][j]) - R[k][k]) + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (R[k][j] - R[j][k]) * t
        q[j] = (R[j][i] + R[i][j]) * t
        q[k] = (R[k][i] + R[i][k]) * t
    return tuple(q)


def hat(w):
    return [[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]]


def mm(A, B):
    return [[(A[i][0] * B[0][j] + A[i][1] * B[1][j]) + A[i][2] * B[2][j] for j in range(3)] for i in range(3)]


def mv(A, v):
    return tuple((A[i][0] * v[0] + A[i][1] * v[1]) + A[i][2] * v[2] for i in range(3))


def se3_exp(a):  # SE3::exp (se3.hpp:765-786) with SO3::expAndTheta (so3.hpp:577-605)
    w = a[3:]
    theta_sq = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]
    theta = math.sqrt(theta_sq)
    if theta < EPS:
        po4 = theta_sq * theta_sq
        imag = (0.5 - (1.0 / 48.0) * theta_sq) + (1.0 / 3840.0) * po4
        real = (1.0 - (1.0 / 8.0) * theta_sq) + (1.0 / 384.0) * po4
    else:
        imag = math.sin(0.5 * theta) / theta
        real = math.cos(0.5 * theta)
    q = (imag * w[0], imag * w[1], imag * w[2], real)
    W = hat(w)
    W2 = mm(W, W)
    if theta < EPS:
        V = q_matrix(q)
    else:
        s1 = (1.0 - math.cos(theta)) / theta_sq
        s2 = (theta - math.sin(theta)) / (theta_sq * theta)
        V = [[((1.0 if i == j else 0.0) + s1 * W[i][j]) + s2 * W2[i][j] for j in range(3)] for i in range(3)]
    return q, mv(V, a[:3])


def se3_mul(A, B):  # SE3 * SE3 (se3.hpp:305-309; so3.hpp:320-326 + the normalising constructor)
    (ax, ay, az, aw), (bx, by, bz, bw) = A[0], B[0]
    q = q_normalize((((aw * bx + ax * bw) + ay * bz) - az * by, ((aw * by + ay * bw) + az * bx) - ax * bz,
                     ((aw * bz + az * bw) + ax * by) - ay * bx, ((aw * bw - ax * bx) - ay * by) - az * bz))
    r = q_rotate(A[0], B[1])
    return q, tuple(A[1][i] + r[i] for i in range(3))


def se3_inv(A):  # SE3::inverse (se3.hpp:205-208)
    q = q_normalize((-A[0][0], -A[0][1], -A[0][2], A[0][3]))
    return q, q_rotate(q, tuple(t * -1.0 for t in A[1]))


def se3_log(A):  # SE3::log (se3.hpp:220-253), SO3::logAndTheta (so3.hpp:239-283)
    q, t = A
    sq_n = (q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]
    n, w = math.sqrt(sq_n), q[3]
    if n < EPS:
        f = 2.0 / w - (2.0 * sq_n) / (w * (w * w))
    elif abs(w) < EPS:
        f = math.pi / n if w > 0 else -math.pi / n
    else:
        f = (2.0 * math.atan(n / w)) / n
    theta = f * n
    om = (f * q[0], f * q[1], f * q[2])
    W = hat(om)
    W2 = mm(W, W)
    if abs(theta) < EPS:
        c = 1.0 / 12.0
    else:
        c = (1.0 - (theta * math.cos(0.5 * theta)) / (2.0 * math.sin(0.5 * theta))) / (theta * theta)
    Vi = [[((1.0 if i == j else 0.0) - 0.5 * W[i][j]) + c * W2[i][j] for j in range(3)] for i in range(3)]
    return mv(Vi, t) + om


def se3_adj(A):  # SE3::Adj (se3.hpp:100-108)
    R = q_matrix(A[0])
    tR = mm(hat(A[1]), R)
    M = np.zeros((6, 6))
    M[:3, :3] = R
    M[3:, 3:] = R
    M[:3, 3:] = tR
    return M


def evalpt(fs):
    m = [float(v) for v in fs["world_to_cam_evalpt"]]
    return q_from_matrix([m[0:3], m[3:6], m[6:9]]), tuple(m[9:12])


def ulps(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    ia, ib = a.view(np.int64), b.view(np.int64)
    ia = np.where(ia < 0, np.int64(-2 ** 63) - ia, ia)
    ib = np.where(ib < 0, np.int64(-2 ** 63) - ib, ib)
    return int(np.abs(ia - ib).max()) if a.size else 0


def random_tangents(rng, n):
    out = []
    for k in range(n):
        scale = [1e-13, 1e-6, 1e-3, 0.1, 1.0, 3.0][k % 6]
        out.append(tuple(float(v) for v in rng.standard_normal(6) * scale))
    out.append((0.1, -0.2, 0.3, math.pi - 1e-12, 0.0, 0.0))  # w ~ 0 after exp: the log's pi / n branch
    out.append((0.0,) * 6)
    return out


# ------------------------------------------------------------------------------------------
# first principles
# ------------------------------------------------------------------------------------------
def test_python_sophus_first_principles():
    from scipy.linalg import expm

    rng = np.random.default_rng(0)
    for a in random_tangents(rng, 60):
        q, t = se3_exp(a)
        T = np.zeros((4, 4))
        T[:3, :3] = hat(a[3:])
        T[:3, 3] = a[:3]
        E = expm(T)
        np.testing.assert_allclose(q_matrix(q), E[:3, :3], rtol=0, atol=1e-13)
        np.testing.assert_allclose(t, E[:3, 3], rtol=0, atol=1e-13 * max(1.0, np.abs(a[:3]).max()))
        assert abs(math.sqrt(sum(c * c for c in q)) - 1) < 1e-15
        if np.linalg.norm(a[3:]) < 3.0:  # log is the inverse inside the principal branch
            np.testing.assert_allclose(se3_log((q, t)), a, rtol=0, atol=1e-12 * max(1.0, np.abs(a).max()))
    for _ in range(30):
        A = se3_exp(tuple(rng.standard_normal(6)))
        B = se3_exp(tuple(rng.standard_normal(6)))
        M = lambda X: np.vstack([np.hstack([q_matrix(X[0]), np.array(X[1])[:, None]]), [0, 0, 0, 1]])
        np.testing.assert_allclose(M(se3_mul(A, B)), M(A) @ M(B), atol=1e-13)
        np.testing.assert_allclose(M(se3_inv(A)), np.linalg.inv(M(A)), atol=1e-13)
        # Adj: exp(Adj_A xi) = A exp(xi) A^-1
        xi = tuple(rng.standard_normal(6) * 0.1)
        lhs = M(se3_exp(tuple(se3_adj(A) @ np.array(xi))))
        np.testing.assert_allclose(lhs, M(A) @ M(se3_exp(xi)) @ np.linalg.inv(M(A)), atol=1e-12)
        # the matrix round trip
        np.testing.assert_allclose(np.abs(q_from_matrix(q_matrix(A[0]))), np.abs(A[0]), atol=1e-15)


# ------------------------------------------------------------------------------------------
# the product's host helpers and the oracle against it
# ------------------------------------------------------------------------------------------
def frames_with_states(rng, N=5):
    w = synth.make_window(n_frames=N, n_points=10, width=160, height=120, seed=9)
    fr = np.ascontiguousarray(w.frames).copy()
    for f in range(N):
        q = q_normalize(tuple(rng.standard_normal(4)))
        fr["world_to_cam_evalpt"][f, :9] = np.array(q_matrix(q)).ravel()
        fr["world_to_cam_evalpt"][f, 9:] = rng.standard_normal(3)
        scale = [1e-12, 1e-4, 1e-2, 0.3, 1.0][f % 5]
        fr["state"][f, :6] = rng.standard_normal(6) * scale
        fr["state_zero"][f, :6] = rng.standard_normal(6) * scale * 0.5
    return w, fr


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_frame_step_follows_sophus(built, seed):
    """doStepFromBackup's head<6> = log(exp(step) exp(state_backup)) (FullSystem.cc:1889-1893)
    through ldso_ba_frame_step, and the oracle's restatement of the same step."""
    rng = np.random.default_rng(seed)
    w, fr = frames_with_states(rng)
    N = len(fr)
    x = rng.standard_normal(8 * N + 4) * [1e-6, 1e-3, 0.1][seed]
    out = np.zeros_like(fr)
    cval = w.calib.astype(np.float64) / 50
    sf, cd = np.zeros(4, np.float32), np.zeros(4, np.float32)
    L.check(L.lib().ldso_ba_frame_step(N, fr.ctypes.data, L.ptr(x, L.f64p), out.ctypes.data, L.ptr(cval, L.f64p),
                                       L.ptr(cval.copy(), L.f64p), L.ptr(sf, L.f32p), L.ptr(cd, L.f32p)))
    worst = 0
    for f in range(N):
        step = tuple(1.0 * -x[4 + 8 * f + i] for i in range(6))
        ref = se3_log(se3_mul(se3_exp(step), se3_exp(tuple(float(v) for v in fr["state"][f, :6]))))
        worst = max(worst, ulps(out["state"][f, :6], ref))
    print("frame step: max ulp vs the Python Sophus restatement", worst)
    assert worst <= 4
    o_fr = oracle.do_step_from_backup(fr, x, cval.copy(), cval.copy(), w.point_host, w.point_data[:, 2],
                                      np.zeros(w.n_points, np.float32))[0]
    np.testing.assert_array_equal(o_fr["state"], out["state"])


def test_take_data_adjoints_and_precalc_follow_sophus(built):
    rng = np.random.default_rng(5)
    w, fr = frames_with_states(rng)
    N = len(fr)
    lib = L.lib()
    # takeData: get_state_minus_stateZero / PriorZero (FrameHessian.h:59-70)
    prior, delta, dprior = (np.zeros((N, 8)) for _ in range(3))
    L.check(lib.ldso_ba_frame_take_data(N, fr.ctypes.data, None, L.ptr(prior, L.f64p), L.ptr(delta, L.f64p),
                                        L.ptr(dprior, L.f64p)))
    worst = 0
    for f in range(N):
        s = tuple(float(v) for v in fr["state"][f, :6])
        mz = tuple(-float(v) for v in fr["state_zero"][f, :6])
        worst = max(worst, ulps(delta[f, :6], se3_log(se3_mul(se3_exp(mz), se3_exp(s)))))
        worst = max(worst, ulps(dprior[f, :6], se3_log(se3_exp(s))))
    # setAdjointsF: AH = -Adj(target * host^-1)^T scaled (EnergyFunctional.cc:561-580)
    adH, adT = np.zeros((N * N, 64)), np.zeros((N * N, 64))
    L.check(lib.ldso_ba_set_adjoints(N, fr.ctypes.data, L.ptr(adH, L.f64p), L.ptr(adT, L.f64p), L.ptr(None, L.f64p)))
    rs = np.array([0.5, 0.5, 0.5, 1, 1, 1])
    for h in range(N):
        for t in range(N):
            A = se3_adj(se3_mul(evalpt(fr[t]), se3_inv(evalpt(fr[h]))))
            got = adH[h + N * t].reshape(8, 8)[:6, :6]
            worst = max(worst, ulps(got, (-A.T) * rs[:, None]))
    print("takeData / adjoints: max ulp", worst)
    assert worst <= 4
    # FrameFramePrecalc::Set's float rotations (FrameFramePrecalc.cc:12-18), PRE_worldToCam =
    # exp(w2c_leftEps) * evalPT (FrameHessian.h:95-114)
    pre = np.zeros((N * N, L.PRECALC_STRIDE), np.float32)
    L.check(lib.ldso_ba_frame_precalc(N, fr.ctypes.data, L.ptr(w.calib, L.f32p), L.ptr(pre, L.f32p)))

    def cur(f):
        eps = tuple(0.5 * float(v) for v in fr["state"][f, :3]) + tuple(1.0 * float(v) for v in fr["state"][f, 3:6])
        return se3_mul(se3_exp(eps), evalpt(fr[f]))

    for h in range(N):
        for t in range(N):
            l0 = se3_mul(evalpt(fr[t]), se3_inv(evalpt(fr[h])))
            l = se3_mul(cur(t), se3_inv(cur(h)))
            np.testing.assert_array_equal(pre[h + N * t, 12:21], np.float32(np.array(q_matrix(l0[0])).ravel()))
            np.testing.assert_array_equal(pre[h + N * t, 21:24], np.float32(l0[1]))
            np.testing.assert_array_equal(pre[h + N * t, 27:36], np.float32(np.array(q_matrix(l[0])).ravel()))
            np.testing.assert_array_equal(pre[h + N * t, 36:39], np.float32(l[1]))
    # the oracle's frame terms are the same numbers
    w.frames = fr
    t_or = oracle.frame_terms(w)
    np.testing.assert_array_equal(t_or["precalc"], pre)
    np.testing.assert_array_equal(t_or["ad_host"], adH)
    np.testing.assert_array_equal(t_or["frame_delta"], delta)
