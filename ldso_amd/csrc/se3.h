// se3.h -- the double-precision SE(3) and FrameFramePrecalc arithmetic of the path, shared by the
// host helpers (host_math.cpp) and the device GN loop (ldso_ba.hip k_step_resub), statement for
// statement, FP contraction off: Sophus SE3 exp / log / product / inverse / Adj
// (thirdparty/Sophus/sophus/se3.hpp, so3.hpp), FrameHessian::setState's PRE_worldToCam
// (FrameHessian.h:95-114), AffLight::fromToVecExposure (AffLight.h:27-35), the per-pair body of
// FrameFramePrecalc::Set (FrameFramePrecalc.cc:6-35) and FrameHessian::takeData
// (FrameHessian.cc:131-135, FrameHessian.h:59-70, 142-174).
#pragma once
#include <math.h>

#include "ldso_ba_internal.h"

namespace ldso_ba {

constexpr double kScaleXiTrans = 0.5, kScaleXiRot = 1.0, kScaleA = 10.0, kScaleB = 1000.0;

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
LDSO_HD inline Mat3 operator*(const Mat3 &a, const Mat3 &b) {
#pragma clang fp contract(off)
    Mat3 c{};
    for (int r = 0; r < 3; r++)
        for (int k = 0; k < 3; k++)
            for (int q = 0; q < 3; q++) c(r, q) += a(r, k) * b(k, q);
    return c;
}
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

struct Pose {  // rigid transform x -> R x + t (Sophus SE3 convention)
    Mat3 R;
    double t[3];
    LDSO_HD static Pose identity() {
        Pose p;
        p.R = Mat3::eye();
        p.t[0] = p.t[1] = p.t[2] = 0;
        return p;
    }
    LDSO_HD Pose operator*(const Pose &b) const {
#pragma clang fp contract(off)
        Pose c;
        c.R = R * b.R;
        for (int i = 0; i < 3; i++) c.t[i] = R(i, 0) * b.t[0] + R(i, 1) * b.t[1] + R(i, 2) * b.t[2] + t[i];
        return c;
    }
    LDSO_HD Pose inverse() const {
#pragma clang fp contract(off)
        Pose c;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) c.R(i, j) = R(j, i);
        for (int i = 0; i < 3; i++) c.t[i] = -(c.R(i, 0) * t[0] + c.R(i, 1) * t[1] + c.R(i, 2) * t[2]);
        return c;
    }
    // exp of the tangent [upsilon(3), omega(3)] (thirdparty/Sophus/sophus/se3.hpp)
    LDSO_HD static Pose exp(const double xi[6]) {
#pragma clang fp contract(off)
        const double *w = xi + 3;
        double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2], th = sqrt(th2);
        double a, b, c;
        if (th < 1e-10) {
            a = 1 - th2 / 6;
            b = 0.5 - th2 / 24;
            c = 1.0 / 6 - th2 / 120;
        } else {
            a = sin(th) / th;
            b = (1 - cos(th)) / th2;
            c = (th - sin(th)) / (th2 * th);
        }
        Mat3 W = skew(w), W2 = W * W, I = Mat3::eye();
        Pose p;
        Mat3 V;
        for (int k = 0; k < 9; k++) {
            p.R.m[k] = I.m[k] + a * W.m[k] + b * W2.m[k];
            V.m[k] = I.m[k] + b * W.m[k] + c * W2.m[k];
        }
        for (int i = 0; i < 3; i++) p.t[i] = V(i, 0) * xi[0] + V(i, 1) * xi[1] + V(i, 2) * xi[2];
        return p;
    }
    // Sophus SE3::log (se3.hpp:220-253) on the rotation matrix: Eigen's matrix -> quaternion
    // (Quaternion.h, quaternionbase_assign_impl), SO3::logAndTheta's atan form (so3.hpp:239-283),
    // and V^-1 with the half-angle factor; epsilon 1e-10 (common.hpp:144).  Stable for every
    // angle (no 1 - cos(theta) cancellation).
    LDSO_HD void log(double xi[6]) const {
#pragma clang fp contract(off)
        double q[4];  // x, y, z, w
        double tr = R(0, 0) + R(1, 1) + R(2, 2);
        if (tr > 0) {
            double t = sqrt(tr + 1.0);
            q[3] = 0.5 * t;
            t = 0.5 / t;
            q[0] = (R(2, 1) - R(1, 2)) * t;
            q[1] = (R(0, 2) - R(2, 0)) * t;
            q[2] = (R(1, 0) - R(0, 1)) * t;
        } else {
            int i = 0;
            if (R(1, 1) > R(0, 0)) i = 1;
            if (R(2, 2) > R(i, i)) i = 2;
            const int j = (i + 1) % 3, k = (j + 1) % 3;
            double t = sqrt(R(i, i) - R(j, j) - R(k, k) + 1.0);
            q[i] = 0.5 * t;
            t = 0.5 / t;
            q[3] = (R(k, j) - R(j, k)) * t;
            q[j] = (R(j, i) + R(i, j)) * t;
            q[k] = (R(k, i) + R(i, k)) * t;
        }
        const double n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2], n = sqrt(n2), w = q[3];
        double f;
        if (n < 1e-10) f = 2.0 / w - 2.0 * n2 / (w * (w * w));
        else if (fabs(w) < 1e-10) f = (w > 0 ? M_PI : -M_PI) / n;
        else f = 2.0 * atan(n / w) / n;
        const double th = f * n;
        const double om[3] = {f * q[0], f * q[1], f * q[2]};
        Mat3 W = skew(om), W2 = W * W;
        const double d = fabs(th) < 1e-10 ? 1.0 / 12.0
                                               : (1.0 - th * cos(0.5 * th) / (2.0 * sin(0.5 * th))) / (th * th);
        for (int i = 0; i < 3; i++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += ((i == k ? 1.0 : 0.0) - 0.5 * W(i, k) + d * W2(i, k)) * t[k];
            xi[i] = s;
            xi[3 + i] = om[i];
        }
    }
    // Adj = [R, [t]x R; 0, R]
    LDSO_HD void adjoint(double A[36]) const {
#pragma clang fp contract(off)
        for (int k = 0; k < 36; k++) A[k] = 0;
        Mat3 tR = skew(t) * R;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                A[i * 6 + j] = R(i, j);
                A[i * 6 + 3 + j] = tR(i, j);
                A[(i + 3) * 6 + 3 + j] = R(i, j);
            }
    }
};

LDSO_HD inline Pose eval_pose(const ldso_ba_frame_state &f) {
    Pose p;
    for (int k = 0; k < 9; k++) p.R.m[k] = f.world_to_cam_evalpt[k];
    for (int k = 0; k < 3; k++) p.t[k] = f.world_to_cam_evalpt[9 + k];
    return p;
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
    float R[9], tt[3];
    for (int k = 0; k < 9; k++) {
        o[12 + k] = (float)l0.R.m[k];        // PRE_RTll_0
        o[27 + k] = R[k] = (float)l.R.m[k];  // PRE_RTll
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
LDSO_HD inline void frame_step_one(const ldso_ba_frame_state &in, const double *x8, ldso_ba_frame_state &out) {
#pragma clang fp contract(off)
    out = in;
    double st[10], a[6], b[6], lg[6];
    for (int i = 0; i < 10; i++) st[i] = i < 8 ? -x8[i] : 0.0;
    for (int i = 0; i < 6; i++) {
        a[i] = 1.0 * st[i];  // pstepfac.head<6>().cwiseProduct(step.head<6>())
        b[i] = in.state[i];
    }
    (Pose::exp(a) * Pose::exp(b)).log(lg);
    for (int i = 0; i < 10; i++) out.state[i] = i < 6 ? lg[i] : in.state[i] + 1.0 * st[i];
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
