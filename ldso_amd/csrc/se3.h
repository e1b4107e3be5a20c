// se3.h -- the double-precision SE(3) and FrameFramePrecalc arithmetic of the path, shared by the
// host helpers (host_math.cpp) and the device GN loop (ldso_ba.hip k_step_resub), FP contraction
// off.  Pose restates Sophus's SE3 (thirdparty/Sophus/sophus/se3.hpp, so3.hpp) in its own
// representation -- a unit quaternion (Eigen coeffs() order x, y, z, w) and a translation -- with
// Sophus's operations statement for statement: SO3::expAndTheta (half-angle factors,
// so3.hpp:577-605), SE3::exp (se3.hpp:765-786), the quaternion product followed by SO3's
// normalising constructor (so3.hpp:320-326, 475-481, 289-295), the quaternion point action
// (so3.hpp:341-347), inverse (se3.hpp:205-208), SO3::logAndTheta + SE3::log (so3.hpp:239-283,
// se3.hpp:220-253), rotationMatrix() (Eigen's Quaternion::toRotationMatrix) and Adj (se3.hpp:100-108).
// Eigen's fixed-size reductions are written in the order its SSE/AVX packet code sums them (the
// quaternion norm as (x^2 + z^2) + (y^2 + w^2)); where the reference build fuses a multiply-add
// through Eigen's pmadd the result differs by an ulp.  The ABI hands worldToCam_evalPT over as
// matrix3x4(); it becomes a quaternion again through Eigen's Quaternion(Matrix3) as SE3(R, t) does.
// Also here: FrameHessian::setState's PRE_worldToCam (FrameHessian.h:95-114),
// AffLight::fromToVecExposure (AffLight.h:27-35), the per-pair body of FrameFramePrecalc::Set
// (FrameFramePrecalc.cc:6-35) and FrameHessian::takeData (FrameHessian.cc:131-135, FrameHessian.h:
// 59-70, 142-174).
#pragma once
#include <math.h>

#include "ldso_ba_internal.h"

// sin and cos of one argument: on the device one shared range reduction (the device library's
// sincos gives the bits of its sin and cos); on the host the two libm calls
LDSO_HD inline void sin_cos(double x, double &s, double &c) {
#ifdef __HIP_DEVICE_COMPILE__
    sincos(x, &s, &c);
#else
    s = sin(x);
    c = cos(x);
#endif
}

namespace ldso_ba {

constexpr double kScaleXiTrans = 0.5, kScaleXiRot = 1.0, kScaleA = 10.0, kScaleB = 1000.0;
constexpr double kSophusEps = 1e-10;  // Sophus::Constants<double>::epsilon() (common.hpp:144)

struct Mat3 {
    double m[9];
    LDSO_HD double &operator()(int r, int c) { return m[r * 3 + c]; }
    LDSO_HD double operator()(int r, int c) const { return m[r * 3 + c]; }
    LDSO_HD static Mat3 eye() {
        Mat3 a{};
        a(0, 0) = a(1, 1) = a(2, 2) = 1;
        return a;
    }
};
// Eigen's 3x3 lazy product: each entry summed over k = 0, 1, 2 in order
LDSO_HD inline Mat3 operator*(const Mat3 &a, const Mat3 &b) {
#pragma clang fp contract(off)
    Mat3 c;
    for (int r = 0; r < 3; r++)
        for (int q = 0; q < 3; q++) c(r, q) = (a(r, 0) * b(0, q) + a(r, 1) * b(1, q)) + a(r, 2) * b(2, q);
    return c;
}
// SO3::hat (so3.hpp)
LDSO_HD inline Mat3 skew(const double v[3]) {
    Mat3 s{};
    s(0, 1) = -v[2];
    s(0, 2) = v[1];
    s(1, 0) = v[2];
    s(1, 2) = -v[0];
    s(2, 0) = -v[1];
    s(2, 1) = v[0];
    return s;
}
// matrix * vector (Eigen: per row, k = 0, 1, 2 in order)
LDSO_HD inline void mat_vec(const Mat3 &a, const double v[3], double out[3]) {
#pragma clang fp contract(off)
    for (int i = 0; i < 3; i++) out[i] = (a(i, 0) * v[0] + a(i, 1) * v[1]) + a(i, 2) * v[2];
}
// Eigen's cross (OrthoMethods.h, the scalar path for double)
LDSO_HD inline void cross3(const double a[3], const double b[3], double out[3]) {
#pragma clang fp contract(off)
    out[0] = a[1] * b[2] - a[2] * b[1];
    out[1] = a[2] * b[0] - a[0] * b[2];
    out[2] = a[0] * b[1] - a[1] * b[0];
}

struct Pose {  // Sophus SE3: x -> R(q) x + t
    double q[4];  // unit quaternion, Eigen coeffs() order: x, y, z, w
    double t[3];
    LDSO_HD static Pose identity() {
        Pose p;
        p.q[0] = p.q[1] = p.q[2] = 0;
        p.q[3] = 1;
        p.t[0] = p.t[1] = p.t[2] = 0;
        return p;
    }
    // SO3Base::normalize (so3.hpp:289-295): coeffs() /= coeffs().norm()
    LDSO_HD void normalize() {
#pragma clang fp contract(off)
        const double len = sqrt((q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]));
        for (int i = 0; i < 4; i++) q[i] = q[i] / len;
    }
    // SO3 point action (so3.hpp:341-347): uv = vec x p; uv += uv; p + w uv + vec x uv
    LDSO_HD void rotate(const double p[3], double out[3]) const {
#pragma clang fp contract(off)
        double uv[3], c[3];
        cross3(q, p, uv);
        for (int i = 0; i < 3; i++) uv[i] = uv[i] + uv[i];
        cross3(q, uv, c);
        for (int i = 0; i < 3; i++) out[i] = (p[i] + q[3] * uv[i]) + c[i];
    }
    // SE3 product (se3.hpp:305-309): SO3 product (quaternion product, so3.hpp:320-326, then the
    // normalising SO3(quaternion) constructor) and translation() + so3() * other.translation()
    LDSO_HD Pose operator*(const Pose &b) const {
#pragma clang fp contract(off)
        const double ax = q[0], ay = q[1], az = q[2], aw = q[3];
        const double bx = b.q[0], by = b.q[1], bz = b.q[2], bw = b.q[3];
        Pose c;
        c.q[3] = ((aw * bw - ax * bx) - ay * by) - az * bz;
        c.q[0] = ((aw * bx + ax * bw) + ay * bz) - az * by;
        c.q[1] = ((aw * by + ay * bw) + az * bx) - ax * bz;
        c.q[2] = ((aw * bz + az * bw) + ax * by) - ay * bx;
        c.normalize();
        double r[3];
        rotate(b.t, r);
        for (int i = 0; i < 3; i++) c.t[i] = t[i] + r[i];
        return c;
    }
    // SE3::inverse (se3.hpp:205-208): SO3(conjugate) (normalised) and invR * (t * -1)
    LDSO_HD Pose inverse() const {
#pragma clang fp contract(off)
        Pose c;
        c.q[0] = -q[0];
        c.q[1] = -q[1];
        c.q[2] = -q[2];
        c.q[3] = q[3];
        c.normalize();
        const double mt[3] = {t[0] * -1.0, t[1] * -1.0, t[2] * -1.0};
        c.rotate(mt, c.t);
        return c;
    }
    // Eigen's Quaternion::toRotationMatrix (SO3::matrix(), so3.hpp:302-304)
    LDSO_HD Mat3 rotation_matrix() const {
#pragma clang fp contract(off)
        const double x = q[0], y = q[1], z = q[2], w = q[3];
        const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
        const double twx = tx * w, twy = ty * w, twz = tz * w;
        const double txx = tx * x, txy = ty * x, txz = tz * x;
        const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
        Mat3 R;
        R(0, 0) = 1.0 - (tyy + tzz);
        R(0, 1) = txy - twz;
        R(0, 2) = txz + twy;
        R(1, 0) = txy + twz;
        R(1, 1) = 1.0 - (txx + tzz);
        R(1, 2) = tyz - twx;
        R(2, 0) = txz - twy;
        R(2, 1) = tyz + twx;
        R(2, 2) = 1.0 - (txx + tyy);
        return R;
    }
    // SE3(Matrix3 R, t): SO3(R) = Eigen's Quaternion(Matrix3) (quaternionbase_assign_impl; not
    // normalised by Sophus, which only asserts orthogonality)
    LDSO_HD static Pose from_matrix(const double R[9], const double tr[3]) {
#pragma clang fp contract(off)
        Pose p;
        double tt = (R[0] + R[4]) + R[8];
        if (tt > 0) {
            tt = sqrt(tt + 1.0);
            p.q[3] = 0.5 * tt;
            tt = 0.5 / tt;
            p.q[0] = (R[7] - R[5]) * tt;
            p.q[1] = (R[2] - R[6]) * tt;
            p.q[2] = (R[3] - R[1]) * tt;
        } else {
            int i = 0;
            if (R[4] > R[0]) i = 1;
            if (R[8] > R[i * 4]) i = 2;
            const int j = (i + 1) % 3, k = (j + 1) % 3;
            tt = sqrt(((R[i * 4] - R[j * 4]) - R[k * 4]) + 1.0);
            p.q[i] = 0.5 * tt;
            tt = 0.5 / tt;
            p.q[3] = (R[k * 3 + j] - R[j * 3 + k]) * tt;
            p.q[j] = (R[j * 3 + i] + R[i * 3 + j]) * tt;
            p.q[k] = (R[k * 3 + i] + R[i * 3 + k]) * tt;
        }
        for (int i = 0; i < 3; i++) p.t[i] = tr[i];
        return p;
    }
    // SE3::exp (se3.hpp:765-786) of the tangent [upsilon(3), omega(3)], with SO3::expAndTheta
    // (so3.hpp:577-605): the quaternion from the half-angle factors, not normalised
    LDSO_HD static Pose exp(const double a[6]) {
#pragma clang fp contract(off)
        const double *w = a + 3;
        const double theta_sq = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2];
        const double theta = sqrt(theta_sq);
        const double half_theta = 0.5 * theta;
        double imag, real;
        if (theta < kSophusEps) {
            const double theta_po4 = theta_sq * theta_sq;
            imag = (0.5 - (1.0 / 48.0) * theta_sq) + (1.0 / 3840.0) * theta_po4;
            real = (1.0 - (1.0 / 8.0) * theta_sq) + (1.0 / 384.0) * theta_po4;
        } else {
            double sh, ch;
            sin_cos(half_theta, sh, ch);
            imag = sh / theta;
            real = ch;
        }
        Pose p;
        p.q[0] = imag * w[0];
        p.q[1] = imag * w[1];
        p.q[2] = imag * w[2];
        p.q[3] = real;
        const Mat3 W = skew(w), W2 = W * W;
        Mat3 V;
        if (theta < kSophusEps) {
            V = p.rotation_matrix();
        } else {
            double st, ct;
            sin_cos(theta, st, ct);
            const double s1 = (1.0 - ct) / theta_sq, s2 = (theta - st) / (theta_sq * theta);
            for (int k = 0; k < 9; k++) V.m[k] = ((k % 4 == 0 ? 1.0 : 0.0) + s1 * W.m[k]) + s2 * W2.m[k];
        }
        mat_vec(V, a, p.t);
        return p;
    }
    // SE3::log (se3.hpp:220-253) with SO3::logAndTheta's atan form (so3.hpp:239-283)
    LDSO_HD void log(double xi[6]) const {
#pragma clang fp contract(off)
        const double squared_n = (q[0] * q[0] + q[1] * q[1]) + q[2] * q[2];
        const double n = sqrt(squared_n), w = q[3];
        double f;  // two_atan_nbyw_by_n
        if (n < kSophusEps) {
            const double squared_w = w * w;
            f = 2.0 / w - (2.0 * squared_n) / (w * squared_w);
        } else if (fabs(w) < kSophusEps) {
            f = w > 0 ? M_PI / n : -M_PI / n;
        } else {
            f = (2.0 * atan(n / w)) / n;
        }
        const double theta = f * n;
        const double om[3] = {f * q[0], f * q[1], f * q[2]};
        const Mat3 W = skew(om), W2 = W * W;
        Mat3 Vi;
        if (fabs(theta) < kSophusEps) {
            for (int k = 0; k < 9; k++) Vi.m[k] = ((k % 4 == 0 ? 1.0 : 0.0) - 0.5 * W.m[k]) + (1. / 12.) * W2.m[k];
        } else {
            const double half_theta = 0.5 * theta;
            double sh, ch;
            sin_cos(half_theta, sh, ch);
            const double c = (1.0 - (theta * ch) / (2.0 * sh)) / (theta * theta);
            for (int k = 0; k < 9; k++) Vi.m[k] = ((k % 4 == 0 ? 1.0 : 0.0) - 0.5 * W.m[k]) + c * W2.m[k];
        }
        mat_vec(Vi, t, xi);
        for (int i = 0; i < 3; i++) xi[3 + i] = om[i];
    }
    // SE3::Adj (se3.hpp:100-108) = [R, hat(t) R; 0, R], R = so3().matrix()
    LDSO_HD void adjoint(double A[36]) const {
#pragma clang fp contract(off)
        for (int k = 0; k < 36; k++) A[k] = 0;
        const Mat3 R = rotation_matrix();
        const Mat3 tR = skew(t) * R;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                A[i * 6 + j] = R(i, j);
                A[i * 6 + 3 + j] = tR(i, j);
                A[(i + 3) * 6 + 3 + j] = R(i, j);
            }
    }
};

LDSO_HD inline Pose eval_pose(const ldso_ba_frame_state &f) {
    return Pose::from_matrix(f.world_to_cam_evalpt, f.world_to_cam_evalpt + 9);
}
// FrameHessian::setState (FrameHessian.h:95-114): PRE_worldToCam = exp(state_scaled[0:6]) * evalPT
LDSO_HD inline Pose current_pose(const ldso_ba_frame_state &f) {
#pragma clang fp contract(off)
    double eps[6];
    for (int i = 0; i < 6; i++) eps[i] = (i < 3 ? kScaleXiTrans : kScaleXiRot) * f.state[i];
    return Pose::exp(eps) * eval_pose(f);
}
// AffLight::fromToVecExposure (include/AffLight.h:27-35), float arithmetic as in the reference
LDSO_HD inline void affine_from_to(float expF, float expT, float aF, float bF, float aT, float bT, float &a, float &b) {
#pragma clang fp contract(off)
    if (expF == 0 || expT == 0) expF = expT = 1;
    a = expf(aT - aF) * expT / expF;
    b = bT - a * bF;
}


// FrameFramePrecalc::Set for one (h, t): o = LDSO_BA_PRECALC_STRIDE floats (zeroed first);
// ev/cur = evaluation-point / current poses, *InvH = the host's inverses
LDSO_HD inline void pair_precalc(const Pose &ev_t, const Pose &evInvH, const Pose &cur_t, const Pose &curInvH,
                                 const float calib[4], const ldso_ba_frame_state &fh, const ldso_ba_frame_state &ft,
                                 float *o) {
#pragma clang fp contract(off)
    const float fx = calib[0], fy = calib[1], cx = calib[2], cy = calib[3];
    // K and Eigen's cofactor K.inverse() (InverseImpl.h, compute_inverse<.,.,3>)
    const float K[9] = {fx, 0, cx, 0, fy, cy, 0, 0, 1};
    const float invdet = 1.0f / (fy * fx);
    const float Ki[9] = {fy * invdet, 0 * invdet, (0 * cy - cx * fy) * invdet,
                         0 * invdet,  fx * invdet, (cx * 0 - fx * cy) * invdet,
                         0 * invdet,  0 * invdet, (fx * fy - 0 * 0) * invdet};
    for (int k = 0; k < LDSO_BA_PRECALC_STRIDE; k++) o[k] = 0.f;
    const Pose l0 = ev_t * evInvH;   // leftToLeft_0
    const Pose l = cur_t * curInvH;  // leftToLeft
    const Mat3 R0d = l0.rotation_matrix(), Rd = l.rotation_matrix();
    float R[9], tt[3];
    for (int k = 0; k < 9; k++) {
        o[12 + k] = (float)R0d.m[k];        // PRE_RTll_0
        o[27 + k] = R[k] = (float)Rd.m[k];  // PRE_RTll
    }
    for (int k = 0; k < 3; k++) {
        o[21 + k] = (float)l0.t[k];          // PRE_tTll_0
        o[36 + k] = tt[k] = (float)l.t[k];   // PRE_tTll
    }
    float KR[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) KR[r * 3 + c] = K[r * 3] * R[c] + K[r * 3 + 1] * R[3 + c] + K[r * 3 + 2] * R[6 + c];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) o[r * 3 + c] = KR[r * 3] * Ki[c] + KR[r * 3 + 1] * Ki[3 + c] + KR[r * 3 + 2] * Ki[6 + c];
    for (int r = 0; r < 3; r++) o[9 + r] = K[r * 3] * tt[0] + K[r * 3 + 1] * tt[1] + K[r * 3 + 2] * tt[2];
    float a, b;
    affine_from_to((float)fh.ab_exposure, (float)ft.ab_exposure, (float)(kScaleA * fh.state[6]),
                   (float)(kScaleB * fh.state[7]), (float)(kScaleA * ft.state[6]), (float)(kScaleB * ft.state[7]), a, b);
    o[24] = (float)(double)a;
    o[25] = (float)(double)b;
    o[26] = (float)(fh.state_zero[7] * kScaleB);  // PRE_b0_mode = aff_g2l_0().b
}

// FrameHessian::takeData / getPrior / get_state_minus_stateZero / get_state_minus_statePriorZero.
// mode_a / mode_b: setting_affineOptModeA / B (getPrior, FrameHessian.h:142-170: the prior on a / b
// is the mode itself when >= 0, setting_initialAffA/BPrior when < 0; the first frame always gets
// the initial priors).  The float settings widen to the double prior as in the reference.
LDSO_HD inline void frame_take_data_one(const ldso_ba_frame_state &F, float mode_a, float mode_b, double *prior,
                                        double *delta, double *delta_prior) {
#pragma clang fp contract(off)
    double p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (F.is_first_frame) {
        p[0] = p[1] = p[2] = kInitialTransPrior;
        p[3] = p[4] = p[5] = kInitialRotPrior;
        p[6] = kInitialAffAPrior;
        p[7] = kInitialAffBPrior;
    } else {
        p[6] = mode_a < 0 ? kInitialAffAPrior : mode_a;
        p[7] = mode_b < 0 ? kInitialAffBPrior : mode_b;
    }
    double mz[6], z[6], lg[6];
    for (int i = 0; i < 6; i++) {
        mz[i] = -F.state_zero[i];
        z[i] = F.state[i];
    }
    if (prior)
        for (int i = 0; i < 8; i++) prior[i] = p[i];
    if (delta) {
        (Pose::exp(mz) * Pose::exp(z)).log(lg);
        for (int i = 0; i < 8; i++) delta[i] = i < 6 ? lg[i] : F.state[i] - F.state_zero[i];
    }
    if (delta_prior) {
        Pose::exp(z).log(lg);
        for (int i = 0; i < 8; i++) delta_prior[i] = i < 6 ? lg[i] : F.state[i];
    }
}

// FullSystem::doStepFromBackup (FullSystem.cc:1843-1922), the branch without SOLVER_MOMENTUM
// (setting_solverMode = FIX_LAMBDA | ORTHOGONALIZE_X_LATER) at stepfac 1, for one frame:
// step = -x.segment<8>(CPARS + 8 idx) (resubstituteF_MT, EnergyFunctional.cc:618-623), then
// state = state_backup + step except head<6> = log(exp(step.head<6>) exp(state_backup.head<6>)).
// the step's tangent: pstepfac.head<6>().cwiseProduct(step.head<6>()), step = -x
LDSO_HD inline void frame_step_tangent(const double *x8, double a[6]) {
#pragma clang fp contract(off)
    for (int i = 0; i < 6; i++) a[i] = 1.0 * -x8[i];
}
// the rest of the step once exp(a) and exp(state) are formed
LDSO_HD inline void frame_step_finish(const ldso_ba_frame_state &in, const double *x8, const Pose &ea, const Pose &eb,
                                      ldso_ba_frame_state &out) {
#pragma clang fp contract(off)
    out = in;
    double st[10], lg[6];
    for (int i = 0; i < 10; i++) st[i] = i < 8 ? -x8[i] : 0.0;
    (ea * eb).log(lg);
    for (int i = 0; i < 10; i++) out.state[i] = i < 6 ? lg[i] : in.state[i] + 1.0 * st[i];
}
LDSO_HD inline void frame_step_one(const ldso_ba_frame_state &in, const double *x8, ldso_ba_frame_state &out) {
    double a[6];
    frame_step_tangent(x8, a);
    frame_step_finish(in, x8, Pose::exp(a), Pose::exp(in.state), out);
}

// ... and the calibration: HCalib->step = -x.head<CPARS>(), setValue(value_backup + step)
// (CalibHessian.h:71-85): value_scaledf = (float)(SCALE_F / SCALE_C * value), cDeltaF = value - value_zero
LDSO_HD inline void calib_step(double value[4], const double *x4, const double value_zero[4], float scaledf[4],
                               float c_delta[4]) {
#pragma clang fp contract(off)
    for (int i = 0; i < 4; i++) value[i] = value[i] + 1.0 * (-x4[i]);
    const double sc[4] = {kScaleF, kScaleF, kScaleC, kScaleC};
    for (int i = 0; i < 4; i++) {
        scaledf[i] = (float)(sc[i] * value[i]);
        c_delta[i] = (float)(value[i] - value_zero[i]);
    }
}

// doStepFromBackup's return value canbreak (FullSystem.cc:1836-1838, 1894-1897, 1914-1931) at
// stepfac 1 on the visual-only path (sumI = sumIH = 0): float accumulators fed double products
// (float += double rounds the double sum), averaged over the frames, against 5e-4 / 5e-5 x
// setting_thOptIterations in double.  sum_nid / num_id: the window's sum of |idepth_backup| and its
// point count (window_nid).  xw: the window's x [8N+4] (step = -x).
LDSO_HD inline bool step_canbreak(int N, const double *xw, float sum_nid, float num_id, float th_opt) {
#pragma clang fp contract(off)
    float sumA = 0, sumB = 0, sumT = 0, sumR = 0;
    for (int f = 0; f < N; f++) {
        double st[8];
        for (int i = 0; i < 8; i++) st[i] = -xw[4 + 8 * f + i];
        sumA = (float)((double)sumA + st[6] * st[6]);
        sumB = (float)((double)sumB + st[7] * st[7]);
        sumT = (float)((double)sumT + ((st[0] * st[0] + st[1] * st[1]) + st[2] * st[2]));
        sumR = (float)((double)sumR + ((st[3] * st[3] + st[4] * st[4]) + st[5] * st[5]));
    }
    const float n = (float)N;
    sumA /= n;
    sumB /= n;
    sumR /= n;
    sumT /= n;
    const float sumNID = sum_nid / num_id;
    const double th = (double)th_opt, sumI = 0.0, sumIH = 0.0;
    return (double)sqrtf(sumA) < 0.0005 * th && (double)sqrtf(sumB) < 0.00005 * th &&
           (double)sqrtf(sumR) < 0.00005 * th && (double)(sqrtf(sumT) * sumNID) < 0.00005 * th &&
           sqrt(sumI) < 0.00005 * th && sqrt(sumIH) < 0.00005 * th;
}

}  // namespace ldso_ba
