// ldso_oracle_tracker.cpp -- CPU restatement of LDSO's coarse tracker inner loops.
//
// TEST INFRASTRUCTURE ONLY (see ldso_oracle.h): only tests/ and bench.py's cpu_baseline leg load
// it, as the checker.  Same conventions as ldso_oracle.cpp: compiled -ffp-contract=off, every
// float statement rounds in the reference's source order, 3-term dot products left to right.
//
//   oracle_make_images   FrameHessian::makeImages            src/internal/FrameHessian.cc:59-115
//   oracle_ct_levels     setGlobalCalib's level rule         src/internal/GlobalCalib.cc:20-30
//   oracle_ct_make_k     CoarseTracker::makeK                src/frontend/CoarseTracker.cc:312-339
//   oracle_ct_calc_res   CoarseTracker::calcRes              src/frontend/CoarseTracker.cc:540-673
//   oracle_ct_calc_gs    CoarseTracker::calcGSSSE            src/frontend/CoarseTracker.cc:675-741
//                        with Accumulator9 (4 SSE lanes, 1k/1M blocked flush, finish)
//                                                            MatrixAccumulators.h:1104-1643
//   affine               AffLight::fromToVecExposure         include/AffLight.h:27-35
//   oracle_ip_make       ImmaturePoint::ImmaturePoint        src/internal/ImmaturePoint.cc:14-39
//   oracle_ip_trace      traceNewCoarse -> traceOn           src/frontend/FullSystem.cc:1157-1194
//                                                            src/internal/ImmaturePoint.cc:47-317
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "ldso_oracle.h"

namespace {

constexpr float kHuberTH = 9.0f;  // setting_huberTH, Setting.cc:76
constexpr float SCALE_XI_ROT = 1.0f, SCALE_XI_TRANS = 0.5f, SCALE_A = 10.0f, SCALE_B = 1000.0f;  // Settings.h:29-35

void affine_from_to(float expF, float expT, float aF, float bF, float aT, float bT, float &a, float &b) {
    if (expF == 0 || expT == 0) expT = expF = 1;
    a = std::exp(aT - aF) * expT / expF;
    b = bT - a * bF;
}

// Eigen's cofactor 3x3 inverse (Eigen/src/LU/InverseImpl.h) of K = [fx 0 cx; 0 fy cy; 0 0 1]
void k_inverse(float fx, float fy, float cx, float cy, float Ki[9]) {
    const float invdet = 1.0f / (fy * fx);
    Ki[0] = fy * invdet;
    Ki[1] = 0 * invdet;
    Ki[2] = (0 * cy - cx * fy) * invdet;
    Ki[3] = 0 * invdet;
    Ki[4] = fx * invdet;
    Ki[5] = (cx * 0 - fx * cy) * invdet;
    Ki[6] = 0 * invdet;
    Ki[7] = 0 * invdet;
    Ki[8] = (fx * fy - 0 * 0) * invdet;
}

// Accumulator9 (MatrixAccumulators.h:1104-1643): 45 upper entries x 4 SSE lanes, updateSSE_eighted
// (:1250-1368), shiftUp (:1624-1642), finish (:1121-1135)
struct Acc9 {
    float d[45][4], d1k[45][4], d1m[45][4];
    size_t num = 0, n1 = 0, n1k = 0, n1m = 0;
    Acc9() {
        std::memset(d, 0, sizeof d);
        std::memset(d1k, 0, sizeof d1k);
        std::memset(d1m, 0, sizeof d1m);
    }
    void shift_up(bool force) {
        if (n1 > 1000 || force) {
            for (int i = 0; i < 45; i++)
                for (int l = 0; l < 4; l++) d1k[i][l] = d[i][l] + d1k[i][l];
            n1k += n1;
            n1 = 0;
            std::memset(d, 0, sizeof d);
        }
        if (n1k > 1000 || force) {
            for (int i = 0; i < 45; i++)
                for (int l = 0; l < 4; l++) d1m[i][l] = d1k[i][l] + d1m[i][l];
            n1m += n1k;
            n1k = 0;
            std::memset(d1k, 0, sizeof d1k);
        }
    }
    void update_weighted(const float J[9][4], const float w[4]) {
        int idx = 0;
        for (int r = 0; r < 9; r++) {
            float Jw[4];
            for (int l = 0; l < 4; l++) Jw[l] = J[r][l] * w[l];
            for (int c = r; c < 9; c++, idx++)
                for (int l = 0; l < 4; l++) d[idx][l] = d[idx][l] + Jw[l] * J[c][l];
        }
        num += 4;
        n1++;
        shift_up(false);
    }
    void finish(float H[9][9]) {
        shift_up(true);
        int idx = 0;
        for (int r = 0; r < 9; r++)
            for (int c = r; c < 9; c++, idx++) {
                const float s = d1m[idx][0] + d1m[idx][1] + d1m[idx][2] + d1m[idx][3];
                H[r][c] = H[c][r] = s;
            }
    }
};

}  // namespace

extern "C" {

int oracle_ct_levels(int w, int h) {
    int wl = w, hl = h, lv = 1;
    while (wl % 2 == 0 && hl % 2 == 0 && wl * hl > 5000 && lv < 6) {
        wl /= 2;
        hl /= 2;
        lv++;
    }
    return lv;
}

void oracle_ct_make_k(const float calib[4], int w, int h, int levels, float *out) {
    float fx[6], fy[6], cx[6], cy[6];
    fx[0] = calib[0];
    fy[0] = calib[1];
    cx[0] = calib[2];
    cy[0] = calib[3];
    for (int l = 1; l < levels; l++) {
        fx[l] = fx[l - 1] * 0.5;
        fy[l] = fy[l - 1] * 0.5;
        cx[l] = (cx[0] + 0.5) / ((int)1 << l) - 0.5;
        cy[l] = (cy[0] + 0.5) / ((int)1 << l) - 0.5;
    }
    (void)w;
    (void)h;
    for (int l = 0; l < levels; l++) {
        float *o = out + 13 * l;
        o[0] = fx[l];
        o[1] = fy[l];
        o[2] = cx[l];
        o[3] = cy[l];
        k_inverse(fx[l], fy[l], cx[l], cy[l], o + 4);
    }
}

void oracle_make_images(const float *color, int w, int h, int levels, const float *B, float *dIp, float *absg) {
    size_t off = 0;
    std::vector<size_t> offs(levels);
    for (int l = 0; l < levels; l++) {
        offs[l] = off;
        off += (size_t)(w >> l) * (h >> l);
    }
    std::memset(dIp, 0, off * 3 * sizeof(float));
    std::memset(absg, 0, off * sizeof(float));
    for (int i = 0; i < w * h; i++) dIp[3 * i] = color[i];
    for (int lvl = 0; lvl < levels; lvl++) {
        const int wl = w >> lvl, hl = h >> lvl;
        float *dI_l = dIp + 3 * offs[lvl];
        float *dabs_l = absg + offs[lvl];
        if (lvl > 0) {
            const int wlm1 = w >> (lvl - 1);
            const float *dI_lm = dIp + 3 * offs[lvl - 1];
            for (int y = 0; y < hl; y++)
                for (int x = 0; x < wl; x++)
                    dI_l[3 * (x + y * wl)] =
                        0.25f * (dI_lm[3 * (2 * x + 2 * y * wlm1)] + dI_lm[3 * (2 * x + 1 + 2 * y * wlm1)] +
                                 dI_lm[3 * (2 * x + 2 * y * wlm1 + wlm1)] + dI_lm[3 * (2 * x + 1 + 2 * y * wlm1 + wlm1)]);
        }
        for (int idx = wl; idx < wl * (hl - 1); idx++) {
            float dx = 0.5f * (dI_l[3 * (idx + 1)] - dI_l[3 * (idx - 1)]);
            float dy = 0.5f * (dI_l[3 * (idx + wl)] - dI_l[3 * (idx - wl)]);
            if (std::isnan(dx) || std::fabs(dx) > 255.0) dx = 0;
            if (std::isnan(dy) || std::fabs(dy) > 255.0) dy = 0;
            dI_l[3 * idx + 1] = dx;
            dI_l[3 * idx + 2] = dy;
            dabs_l[idx] = dx * dx + dy * dy;
            if (B) {  // CalibHessian::getBGradOnly (CalibHessian.h:102-111)
                int c = dI_l[3 * idx] + 0.5f;
                if (c < 5) c = 5;
                if (c > 250) c = 250;
                const float gw = B[c + 1] - B[c];
                dabs_l[idx] *= gw * gw;
            }
        }
    }
}

// calcRes for one level.  kl = {fx, fy, cx, cy, Ki[9]} of the level (oracle_ct_make_k),
// dI = the new frame's level (wl*hl*3), pc = the reference's level point cloud.
// aff6 = {ref exposure, new exposure, ref a, ref b, new a, new b}.
// warped_out [n][8] (compacted, zero padded to a multiple of 4), *n_warped = buf_warped_n.
int oracle_ct_calc_res(int lvl, int wl, int hl, const float *kl, const float *dI, int n, const float *pc_u,
                       const float *pc_v, const float *pc_idepth, const float *pc_color, const double *T,
                       const double *aff6, float cutoffTH, double *rs, float *warped_out, int *n_warped) {
#pragma GCC diagnostic ignored "-Wmaybe-uninitialized"
    float E = 0;
    int numTermsInE = 0, numTermsInWarped = 0, numSaturated = 0;
    const float fxl = kl[0], fyl = kl[1], cxl = kl[2], cyl = kl[3];
    const float *Ki = kl + 4;
    float R[9], t[3], RKi[9];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) R[3 * i + j] = (float)T[4 * i + j];
        t[i] = (float)T[4 * i + 3];
    }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) RKi[3 * i + j] = R[3 * i] * Ki[j] + R[3 * i + 1] * Ki[3 + j] + R[3 * i + 2] * Ki[6 + j];
    float aLL, bLL;
    affine_from_to((float)aff6[0], (float)aff6[1], (float)aff6[2], (float)aff6[3], (float)aff6[4], (float)aff6[5], aLL,
                   bLL);
    float sumSquaredShiftT = 0, sumSquaredShiftRT = 0, sumSquaredShiftNum = 0;
    const float maxEnergy = 2 * kHuberTH * cutoffTH - kHuberTH * kHuberTH;
    for (int i = 0; i < n; i++) {
        const float id = pc_idepth[i], x = pc_u[i], y = pc_v[i];
        float pt[3];
        for (int k = 0; k < 3; k++) pt[k] = (RKi[3 * k] * x + RKi[3 * k + 1] * y + RKi[3 * k + 2] * 1) + t[k] * id;
        const float u = pt[0] / pt[2], v = pt[1] / pt[2];
        const float Ku = fxl * u + cxl, Kv = fyl * v + cyl;
        const float new_idepth = id / pt[2];
        if (lvl == 0 && i % 32 == 0) {
            float ptT[3], ptT2[3], pt3[3];
            for (int k = 0; k < 3; k++) {
                const float kx = Ki[3 * k] * x + Ki[3 * k + 1] * y + Ki[3 * k + 2] * 1;
                ptT[k] = kx + t[k] * id;
                ptT2[k] = kx - t[k] * id;
                pt3[k] = (RKi[3 * k] * x + RKi[3 * k + 1] * y + RKi[3 * k + 2] * 1) - t[k] * id;
            }
            const float uT = ptT[0] / ptT[2], vT = ptT[1] / ptT[2];
            const float KuT = fxl * uT + cxl, KvT = fyl * vT + cyl;
            const float uT2 = ptT2[0] / ptT2[2], vT2 = ptT2[1] / ptT2[2];
            const float KuT2 = fxl * uT2 + cxl, KvT2 = fyl * vT2 + cyl;
            const float u3 = pt3[0] / pt3[2], v3 = pt3[1] / pt3[2];
            const float Ku3 = fxl * u3 + cxl, Kv3 = fyl * v3 + cyl;
            sumSquaredShiftT += (KuT - x) * (KuT - x) + (KvT - y) * (KvT - y);
            sumSquaredShiftT += (KuT2 - x) * (KuT2 - x) + (KvT2 - y) * (KvT2 - y);
            sumSquaredShiftRT += (Ku - x) * (Ku - x) + (Kv - y) * (Kv - y);
            sumSquaredShiftRT += (Ku3 - x) * (Ku3 - x) + (Kv3 - y) * (Kv3 - y);
            sumSquaredShiftNum += 2;
        }
        if (!(Ku > 2 && Kv > 2 && Ku < wl - 3 && Kv < hl - 3 && new_idepth > 0)) continue;
        const float refColor = pc_color[i];
        // getInterpolatedElement33 (GlobalFuncs.h:89-103)
        const int ix = (int)Ku, iy = (int)Kv;
        const float dx = Ku - ix, dy = Kv - iy, dxdy = dx * dy;
        const float *bp = dI + 3 * (ix + iy * wl);
        float hit[3];
        for (int c = 0; c < 3; c++)
            hit[c] = dxdy * bp[3 * (1 + wl) + c] + (dy - dxdy) * bp[3 * wl + c] + (dx - dxdy) * bp[3 + c] +
                     (1 - dx - dy + dxdy) * bp[c];
        if (!std::isfinite(hit[0])) continue;
        const float residual = hit[0] - (float)(aLL * refColor + bLL);
        const float hw = std::fabs(residual) < kHuberTH ? 1 : kHuberTH / std::fabs(residual);
        if (std::fabs(residual) > cutoffTH) {
            E += maxEnergy;
            numTermsInE++;
            numSaturated++;
        } else {
            E += hw * residual * residual * (2 - hw);
            numTermsInE++;
            float *o = warped_out + 8 * numTermsInWarped;
            o[0] = new_idepth;
            o[1] = u;
            o[2] = v;
            o[3] = hit[1];
            o[4] = hit[2];
            o[5] = residual;
            o[6] = hw;
            o[7] = refColor;
            numTermsInWarped++;
        }
    }
    while (numTermsInWarped % 4 != 0) {
        std::memset(warped_out + 8 * numTermsInWarped, 0, 8 * sizeof(float));
        numTermsInWarped++;
    }
    *n_warped = numTermsInWarped;
    rs[0] = E;
    rs[1] = numTermsInE;
    rs[2] = sumSquaredShiftT / (sumSquaredShiftNum + 0.1);
    rs[3] = 0;
    rs[4] = sumSquaredShiftRT / (sumSquaredShiftNum + 0.1);
    rs[5] = numSaturated / (float)numTermsInE;
    return 0;
}

// calcGSSSE over warped [n][8] (n % 4 == 0); aff6 as above (a from fromToVecExposure, b0 = ref b)
int oracle_ct_calc_gs(int n, const float *warped, float fxl_, float fyl_, const double *aff6, double *H_out,
                      double *b_out) {
    if (n % 4) return -1;
    float aLL, bLL;
    affine_from_to((float)aff6[0], (float)aff6[1], (float)aff6[2], (float)aff6[3], (float)aff6[4], (float)aff6[5], aLL,
                   bLL);
    const float a = (float)(double)aLL, b0 = (float)aff6[3];
    Acc9 acc;
    for (int i = 0; i < n; i += 4) {
        float J[9][4], w[4];
        for (int l = 0; l < 4; l++) {
            const float *q = warped + 8 * (i + l);
            const float id = q[0], u = q[1], v = q[2];
            const float dx = q[3] * fxl_, dy = q[4] * fyl_;
            J[0][l] = id * dx;
            J[1][l] = id * dy;
            J[2][l] = 0 - id * (u * dx + v * dy);
            J[3][l] = 0 - ((u * v) * dx + dy * (1 + v * v));
            J[4][l] = (u * v) * dy + dx * (1 + u * u);
            J[5][l] = u * dy - v * dx;
            J[6][l] = a * (b0 - q[7]);
            J[7][l] = -1;
            J[8][l] = q[5];
            w[l] = q[6];
        }
        acc.update_weighted(J, w);
    }
    float H[9][9];
    acc.finish(H);
    const float scale[8] = {SCALE_XI_TRANS, SCALE_XI_TRANS, SCALE_XI_TRANS, SCALE_XI_ROT,
                            SCALE_XI_ROT,   SCALE_XI_ROT,   SCALE_A,        SCALE_B};
    const double inv_n = (double)(1.0f / n);
    for (int r = 0; r < 8; r++) {
        for (int c = 0; c < 8; c++) H_out[8 * r + c] = (double)H[r][c] * inv_n;
        b_out[r] = (double)H[r][8] * inv_n;
    }
    // H_out.block<8,k>(0,c) *= col scales, then rows; b rows (CoarseTracker.cc:728-740)
    for (int r = 0; r < 8; r++)
        for (int c = 0; c < 8; c++) H_out[8 * r + c] *= scale[c];
    for (int r = 0; r < 8; r++)
        for (int c = 0; c < 8; c++) H_out[8 * r + c] *= scale[r];
    for (int r = 0; r < 8; r++) b_out[r] *= scale[r];
    return 0;
}

}  // extern "C"

// ============================================================================================
// Immature points: ImmaturePoint::ImmaturePoint and ImmaturePoint::traceOn
// (src/internal/ImmaturePoint.cc:14-39, 47-317) over FullSystem::traceNewCoarse's loop
// (src/frontend/FullSystem.cc:1157-1194).  dI: the traced / sampled frame's level-0 [w*h][3].
// Taps are clamped to the last interpolable texel (the reference reads past the image there).
// ============================================================================================
namespace {

constexpr int kPat[8][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0}, {0, 0}, {2, 0}, {-1, 1}, {0, 2}};  // Setting.cc:275
constexpr float kOutlierTHSumComponent = 50.0f * 50.0f;  // Setting.cc:41
constexpr float kOutlierTH = 12 * 12;                    // Setting.cc:39
constexpr float kOverallEnergyTHWeight = 1.0f;           // Setting.cc:82
constexpr float kMaxPixSearch = 0.027f;                  // Setting.cc:28
constexpr int kMinTraceTestRadius = 2;                   // Setting.cc:52
constexpr float kTraceStepsize = 1.0f;                   // Setting.cc:89
constexpr int kTraceGNIterations = 3;                    // Setting.cc:90
constexpr float kTraceGNThreshold = 0.1f;                // Setting.cc:91
constexpr float kTraceExtraSlackOnTH = 1.2f;             // Setting.cc:92
constexpr float kTraceSlackInterval = 1.5f;              // Setting.cc:93
constexpr float kTraceMinImprovementFactor = 2;          // Setting.cc:94

// index of the top-left texel of a bilinear tap, clamped into [0, w-2] x [0, h-2]
inline long ip_base(float x, float y, int w, int h, float &fx, float &fy) {
    long ix = (long)(int)x, iy = (long)(int)y;
    fx = x - (int)x;
    fy = y - (int)y;
    ix = ix < 0 ? 0 : ix > w - 2 ? w - 2 : ix;
    iy = iy < 0 ? 0 : iy > h - 2 ? h - 2 : iy;
    return ix + iy * (long)w;
}

// getInterpolatedElement31 (GlobalFuncs.h:146-159)
inline float interp31(const float *dI, float x, float y, int w, int h) {
    float dx, dy;
    const float *bp = dI + 3 * ip_base(x, y, w, h, dx, dy);
    const float dxdy = dx * dy;
    return dxdy * bp[3 * (1 + w)] + (dy - dxdy) * bp[3 * w] + (dx - dxdy) * bp[3] + (1 - dx - dy + dxdy) * bp[0];
}

// getInterpolatedElement33 (GlobalFuncs.h:90-103), component by component
inline void interp33(const float *dI, float x, float y, int w, int h, float out[3]) {
    float dx, dy;
    const float *bp = dI + 3 * ip_base(x, y, w, h, dx, dy);
    const float dxdy = dx * dy;
    for (int c = 0; c < 3; c++)
        out[c] = dxdy * bp[3 * (1 + w) + c] + (dy - dxdy) * bp[3 * w + c] + (dx - dxdy) * bp[3 + c] +
                 (1 - dx - dy + dxdy) * bp[c];
}

// getInterpolatedElement33BiLin (GlobalFuncs.h:186-207)
inline void interp33_bilin(const float *dI, float x, float y, int w, int h, float out[3]) {
    float dx, dy;
    const float *bp = dI + 3 * ip_base(x, y, w, h, dx, dy);
    const float tl = bp[0], tr = bp[3], bl = bp[3 * w], br = bp[3 * w + 3];
    const float topInt = dx * tr + (1 - dx) * tl;
    const float botInt = dx * br + (1 - dx) * bl;
    const float leftInt = dy * bl + (1 - dy) * tl;
    const float rightInt = dy * br + (1 - dy) * tr;
    out[0] = dx * rightInt + (1 - dx) * leftInt;
    out[1] = rightInt - leftInt;
    out[2] = botInt - topInt;
}

int set_status(ldso_ct_immature &p, int s, float u, float v, float interval) {
    p.last_uv[0] = u;
    p.last_uv[1] = v;
    p.last_interval = interval;
    return p.last_status = s;
}

// ImmaturePoint::traceOn (ImmaturePoint.cc:47-317)
int trace_on(ldso_ct_immature &p, const float *dI, int w, int h, const float *KRKi, const float *Kt,
             const float *aff) {
    if (p.last_status == LDSO_CT_IPS_OOB) return p.last_status;
    const float maxPixSearch = (w + h) * kMaxPixSearch;
    float pr[3];
    for (int i = 0; i < 3; i++) pr[i] = KRKi[3 * i] * p.u + KRKi[3 * i + 1] * p.v + KRKi[3 * i + 2] * 1.0f;
    float ptpMin[3];
    for (int i = 0; i < 3; i++) ptpMin[i] = pr[i] + Kt[i] * p.idepth_min;
    const float uMin = ptpMin[0] / ptpMin[2], vMin = ptpMin[1] / ptpMin[2];
    if (!(uMin > 4 && vMin > 4 && uMin < w - 5 && vMin < h - 5)) return set_status(p, LDSO_CT_IPS_OOB, -1, -1, 0);

    float dist, uMax, vMax, ptpMax[3];
    if (std::isfinite(p.idepth_max)) {
        for (int i = 0; i < 3; i++) ptpMax[i] = pr[i] + Kt[i] * p.idepth_max;
        uMax = ptpMax[0] / ptpMax[2];
        vMax = ptpMax[1] / ptpMax[2];
        if (!(uMax > 4 && vMax > 4 && uMax < w - 5 && vMax < h - 5)) return set_status(p, LDSO_CT_IPS_OOB, -1, -1, 0);
        dist = (uMin - uMax) * (uMin - uMax) + (vMin - vMax) * (vMin - vMax);
        dist = std::sqrt(dist);
        if (dist < kTraceSlackInterval)
            return set_status(p, LDSO_CT_IPS_SKIPPED, (uMax + uMin) * 0.5f, (vMax + vMin) * 0.5f, dist);
    } else {
        dist = maxPixSearch;
        for (int i = 0; i < 3; i++) ptpMax[i] = pr[i] + Kt[i] * 0.01f;  // Eigen casts the double 0.01 to float
        uMax = ptpMax[0] / ptpMax[2];
        vMax = ptpMax[1] / ptpMax[2];
        const float dx = uMax - uMin, dy = vMax - vMin;
        const float d = 1.0f / std::sqrt(dx * dx + dy * dy);
        uMax = uMin + dist * dx * d;
        vMax = vMin + dist * dy * d;
        if (!(uMax > 4 && vMax > 4 && uMax < w - 5 && vMax < h - 5)) return set_status(p, LDSO_CT_IPS_OOB, -1, -1, 0);
    }
    if (!(p.idepth_min < 0 || (ptpMin[2] > 0.75f && ptpMin[2] < 1.5f))) return set_status(p, LDSO_CT_IPS_OOB, -1, -1, 0);

    float dx = kTraceStepsize * (uMax - uMin);
    float dy = kTraceStepsize * (vMax - vMin);
    const float *G = p.grad_h;
    const float a = (dx * G[0] + dy * G[2]) * dx + (dx * G[1] + dy * G[3]) * dy;       // (v^T G) v
    const float b = (dy * G[0] + -dx * G[2]) * dy + (dy * G[1] + -dx * G[3]) * -dx;  // v = (dy, -dx)
    float errorInPixel = 0.2f + 0.2f * (a + b) / a;
    if (errorInPixel * kTraceMinImprovementFactor > dist && std::isfinite(p.idepth_max))
        return set_status(p, LDSO_CT_IPS_BADCONDITION, (uMax + uMin) * 0.5f, (vMax + vMin) * 0.5f, dist);
    if (errorInPixel > 10) errorInPixel = 10;

    dx /= dist;
    dy /= dist;
    if (dist > maxPixSearch) {
        uMax = uMin + maxPixSearch * dx;
        vMax = vMin + maxPixSearch * dy;
        dist = maxPixSearch;
    }
    int numSteps = 1.9999f + dist / kTraceStepsize;
    const float R00 = KRKi[0], R01 = KRKi[1], R10 = KRKi[3], R11 = KRKi[4];  // Rplane = topLeftCorner<2,2>
    const float randShift = uMin * 1000 - std::floor(uMin * 1000);
    float ptx = uMin - randShift * dx;
    float pty = vMin - randShift * dy;
    float rp[8][2];
    for (int i = 0; i < 8; i++) {
        rp[i][0] = R00 * (float)kPat[i][0] + R01 * (float)kPat[i][1];
        rp[i][1] = R10 * (float)kPat[i][0] + R11 * (float)kPat[i][1];
    }
    if (!std::isfinite(dx) || !std::isfinite(dy)) return set_status(p, LDSO_CT_IPS_OOB, -1, -1, 0);

    float errors[100];
    float bestU = 0, bestV = 0, bestEnergy = 1e10f;
    int bestIdx = -1;
    if (numSteps >= 100) numSteps = 99;
    for (int i = 0; i < numSteps; i++) {
        float energy = 0;
        for (int idx = 0; idx < 8; idx++) {
            const float hitColor = interp31(dI, (float)(ptx + rp[idx][0]), (float)(pty + rp[idx][1]), w, h);
            if (!std::isfinite(hitColor)) {
                energy += 1e5f;
                continue;
            }
            const float residual = hitColor - (float)(aff[0] * p.color[idx] + aff[1]);
            const float hw = std::fabs(residual) < kHuberTH ? 1 : kHuberTH / std::fabs(residual);
            energy += hw * residual * residual * (2 - hw);
        }
        errors[i] = energy;
        if (energy < bestEnergy) {
            bestU = ptx;
            bestV = pty;
            bestEnergy = energy;
            bestIdx = i;
        }
        ptx += dx;
        pty += dy;
    }
    float secondBest = 1e10f;
    for (int i = 0; i < numSteps; i++)
        if ((i < bestIdx - kMinTraceTestRadius || i > bestIdx + kMinTraceTestRadius) && errors[i] < secondBest)
            secondBest = errors[i];
    const float newQuality = secondBest / bestEnergy;
    if (newQuality < p.quality || numSteps > 10) p.quality = newQuality;

    float uBak = bestU, vBak = bestV, gnstepsize = 1, stepBack = 0;
    if (kTraceGNIterations > 0) bestEnergy = 1e5f;
    for (int it = 0; it < kTraceGNIterations; it++) {
        float H = 1, bb = 0, energy = 0;
        for (int idx = 0; idx < 8; idx++) {
            float hc[3];
            interp33(dI, (float)(bestU + rp[idx][0]), (float)(bestV + rp[idx][1]), w, h, hc);
            if (!std::isfinite(hc[0])) {
                energy += 1e5f;
                continue;
            }
            const float residual = hc[0] - (aff[0] * p.color[idx] + aff[1]);
            const float dResdDist = dx * hc[1] + dy * hc[2];
            const float hw = std::fabs(residual) < kHuberTH ? 1 : kHuberTH / std::fabs(residual);
            H += hw * dResdDist * dResdDist;
            bb += hw * residual * dResdDist;
            energy += p.weights[idx] * p.weights[idx] * hw * residual * residual * (2 - hw);
        }
        if (energy > bestEnergy) {
            stepBack *= 0.5f;
            bestU = uBak + stepBack * dx;
            bestV = vBak + stepBack * dy;
        } else {
            float step = -gnstepsize * bb / H;
            if (step < -0.5f) step = -0.5f;
            else if (step > 0.5f) step = 0.5f;
            if (!std::isfinite(step)) step = 0;
            uBak = bestU;
            vBak = bestV;
            stepBack = step;
            bestU += step * dx;
            bestV += step * dy;
            bestEnergy = energy;
        }
        if (std::fabs(stepBack) < kTraceGNThreshold) break;
    }

    if (!(bestEnergy < p.energy_th * kTraceExtraSlackOnTH))
        return set_status(p, p.last_status == LDSO_CT_IPS_OUTLIER ? LDSO_CT_IPS_OOB : LDSO_CT_IPS_OUTLIER, -1, -1, 0);

    if (dx * dx > dy * dy) {
        p.idepth_min = (pr[2] * (bestU - errorInPixel * dx) - pr[0]) / (Kt[0] - Kt[2] * (bestU - errorInPixel * dx));
        p.idepth_max = (pr[2] * (bestU + errorInPixel * dx) - pr[0]) / (Kt[0] - Kt[2] * (bestU + errorInPixel * dx));
    } else {
        p.idepth_min = (pr[2] * (bestV - errorInPixel * dy) - pr[1]) / (Kt[1] - Kt[2] * (bestV - errorInPixel * dy));
        p.idepth_max = (pr[2] * (bestV + errorInPixel * dy) - pr[1]) / (Kt[1] - Kt[2] * (bestV + errorInPixel * dy));
    }
    if (p.idepth_min > p.idepth_max) std::swap(p.idepth_min, p.idepth_max);
    if (!std::isfinite(p.idepth_min) || !std::isfinite(p.idepth_max) || (p.idepth_max < 0))
        return set_status(p, LDSO_CT_IPS_OUTLIER, -1, -1, 0);
    return set_status(p, LDSO_CT_IPS_GOOD, bestU, bestV, 2 * errorInPixel);
}

}  // namespace

extern "C" {

void oracle_ip_make(const float *dI, int w, int h, int n, const float *uv, float type, int host,
                    ldso_ct_immature *out) {
    for (int k = 0; k < n; k++) {
        ldso_ct_immature &p = out[k];
        std::memset(&p, 0, sizeof(p));
        p.u = uv[2 * k];
        p.v = uv[2 * k + 1];
        p.idepth_min = 0;
        p.idepth_max = NAN;
        p.quality = 10000;
        p.type = type;
        p.host = host;
        p.last_status = LDSO_CT_IPS_UNINITIALIZED;
        float G[4] = {0, 0, 0, 0};
        bool ok = true;
        for (int idx = 0; idx < 8; idx++) {
            float ptc[3];
            interp33_bilin(dI, p.u + kPat[idx][0], p.v + kPat[idx][1], w, h, ptc);
            p.color[idx] = ptc[0];
            if (!std::isfinite(p.color[idx])) {
                ok = false;
                break;
            }
            G[0] += ptc[1] * ptc[1];
            G[1] += ptc[1] * ptc[2];
            G[2] += ptc[2] * ptc[1];
            G[3] += ptc[2] * ptc[2];
            p.weights[idx] = std::sqrt(kOutlierTHSumComponent / (kOutlierTHSumComponent + (ptc[1] * ptc[1] + ptc[2] * ptc[2])));
        }
        for (int i = 0; i < 4; i++) p.grad_h[i] = G[i];
        if (!ok) {
            p.energy_th = NAN;
            continue;
        }
        float e = 8 * kOutlierTH;
        e *= kOverallEnergyTHWeight * kOverallEnergyTHWeight;
        p.energy_th = e;
    }
}

void oracle_ip_trace(const float *dI, int w, int h, const float *krki, const float *kt, const float *aff, int n,
                     ldso_ct_immature *pts, int *counts) {
    for (int s = 0; s < 6; s++) counts[s] = 0;
    for (int k = 0; k < n; k++) {
        const int hh = pts[k].host;
        trace_on(pts[k], dI, w, h, krki + 9 * hh, kt + 3 * hh, aff + 2 * hh);
        counts[pts[k].last_status]++;
    }
}

}  // extern "C"
