// ldso_ba.hip -- MI355X (gfx950) kernels and C ABI of LDSO's photometric-BA hot path.
//
// One Gauss-Newton pass over every loaded window is seven stream-ordered launches:
//
//   k_linearize   lane per PointFrameResidual, one wavefront per (host,target) bucket chunk.
//                 linearize (Residuals.cc:15-217) + applyRes (Residuals.h:70-88) + the
//                 per-residual AccumulatorApprox terms (AccumulatedTopHessian.cc:66-99,
//                 MatrixAccumulators.h:893-1045) reduced across the wavefront into a 96-float
//                 partial per chunk.  The pair precalc, frame thresholds and image base are
//                 wave-uniform (scalar loads); the only vector traffic is the point record and
//                 32 texel gathers per residual.
//   k_frame_th    FullSystem::setNewFrameEnergyTH (FullSystem.cc:2078-2109), radix select.
//   k_point_sc    per point: Hdd/bd/Hcd sums (AccumulatedTopHessian.cc:94-116), HdiF
//                 (AccumulatedSCHessian.cc:24-33); then the Schur terms of a 64-point chunk of one
//                 host as one symmetric rank-64 update G += U^T diag(HdiF) U staged in LDS (the
//                 accD/accE/accEB/accHcc/accbc sums of AccumulatedSCHessian.cc:35-50).
//   k_stitch_top  per (h,t): adjoint sandwiches of AccumulatedTopHessian.cc:213-239 in double.
//   k_sc_reduce   per host: chunk partials -> G_h (double).
//   k_stitch_sc   per (host i, target j): AccumulatedSCHessian.cc:80-114 in double.
//   k_final       per window: gathers the block records into HA, bA, Hsc, bsc (upper triangle,
//                 symmetrised as stitchDoubleMT does) and the linearizeAll energy.
//
// The per-residual arithmetic of k_linearize is compiled with contraction off and follows the
// reference's statement order, so states, energies, JpJdF and the per-point sums are
// bit-identical to the CPU restatement; the H/b sums are reassociated (tolerance-checked).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ldso_ba.h"
#include "ldso_ba_internal.h"

using namespace ldso_ba;

namespace {

constexpr int kWave = 64;
constexpr int kTopVals = 96;    // 55 + 30 + 6 AccumulatorApprox entries, padded to 96
constexpr int kMaxRes = LDSO_BA_MAX_FRAMES - 1;
constexpr int kNumKernels = 8;
const char *kKernelNames[kNumKernels] = {"k_linearize", "k_frame_th", "k_point_sc", "k_stitch_top",
                                         "k_sc_reduce", "k_stitch_sc", "k_final", "k_resubstitute"};

thread_local std::string g_err;
int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return fail(-2, std::string(#expr) + ": " + hipGetErrorString(e_));  \
    } while (0)

// Per-window device descriptor.
struct WinDev {
    int N, P, R, D;
    int frame_base, pair_base, point_base, res_base;
    int top_item_base, n_top_items;
    int sc_item_base, n_sc_items;
    int K, KP, ntiles, pad0;
    long long sc_slab_base;  // floats
    long long g_base;        // doubles: N * KP*KP
    long long sc_rec_base;   // doubles: N*N * sc_rec_len
    long long top_rec_base;  // doubles: N*N * kTopRecLen
    long long sys_base;      // doubles: packed system
    int newest_begin, newest_end;
    int width, height;
    float wM3, hM3;
    float calib[4];
};

constexpr int kTopRecLen = 64 * 3 + 32 * 2 + 16 + 8 * 2 + 4;  // Hhh Htt Hht Hhc Htc Hcc bh bt bc = 292
__host__ __device__ inline int sc_rec_len(int N) { return N * 64 + 64 + 64 + 32 + 32 + 8 + 8; }
__host__ __device__ inline long long packed_len(int D) { return (long long)D * (D + 1) / 2; }
__host__ __device__ inline long long sys_len(int D) { return 2 * (packed_len(D) + D); }

// ============================================================================================
// k_linearize
// ============================================================================================
struct LinParams {
    const int4 *__restrict__ items;  // {res_begin, count, pair_global, win}
    const WinDev *__restrict__ wins;
    const float4 *__restrict__ img;
    const float *__restrict__ precalc;
    const float *__restrict__ frame_th;
    const int *__restrict__ rs_point;
    const float *__restrict__ pt_data;
    int8_t *rs_state;
    int8_t *rs_newstate;
    uint8_t *rs_flags;
    float *rs_energy;      // state_energy
    float *rs_newenergy;   // state_NewEnergy (persists: applyRes copies it on a later OOB)
    float *rs_energy_wo;   // state_NewEnergyWithOutlier
    float4 *rs_center;     // centerProjectedTo, relBS
    float4 *rs_rec;        // [R][4]: JpJdF[8], Hcd_r[4], Hdd_r, bd_r, -, -
    float *top_slab;       // [items][96]
    double *item_energy;   // [items][2]
    int n_items;
    int npix;
    int fix;
    int accumulate;
};

struct Geo {
    float Ku, Kv, new_idepth;
    float d_xi_x[6], d_xi_y[6], d_C_x[4], d_C_y[4], d_d_x, d_d_y;
};

// projectPoint (full form), ResidualProjections.h:57-84 + Residuals.cc:69-106
__device__ inline bool centre_projection(const float *__restrict__ pre, float u, float v, float idz,
                                         float fxl, float fyl, float cxl, float cyl, float wM3, float hM3,
                                         Geo &g) {
#pragma clang fp contract(off)
    const float fxli = 1.0f / fxl, fyli = 1.0f / fyl;
    const float *R0 = pre + 12, *t0 = pre + 21;
    const float K0 = (u + 0 - cxl) * fxli, K1 = (v + 0 - cyl) * fyli;
    float ptp[3];
#pragma unroll
    for (int i = 0; i < 3; i++) ptp[i] = (R0[3 * i] * K0 + R0[3 * i + 1] * K1 + R0[3 * i + 2] * 1.0f) + t0[i] * idz;
    const float drescale = 1.0f / ptp[2];
    g.new_idepth = idz * drescale;
    if (!(drescale > 0)) return false;
    const float uu = ptp[0] * drescale, vv = ptp[1] * drescale;
    g.Ku = uu * fxl + cxl;
    g.Kv = vv * fyl + cyl;
    if (!(g.Ku > 1.1f && g.Kv > 1.1f && g.Ku < wM3 && g.Kv < hM3)) return false;
    g.d_d_x = drescale * (t0[0] - t0[2] * uu) * kScaleIdepth * fxl;
    g.d_d_y = drescale * (t0[1] - t0[2] * vv) * kScaleIdepth * fyl;
    g.d_C_x[2] = drescale * (R0[6] * uu - R0[0]);
    g.d_C_x[3] = fxl * drescale * (R0[7] * uu - R0[1]) * fyli;
    g.d_C_x[0] = K0 * g.d_C_x[2];
    g.d_C_x[1] = K1 * g.d_C_x[3];
    g.d_C_y[2] = fyl * drescale * (R0[6] * vv - R0[3]) * fxli;
    g.d_C_y[3] = drescale * (R0[7] * vv - R0[4]);
    g.d_C_y[0] = K0 * g.d_C_y[2];
    g.d_C_y[1] = K1 * g.d_C_y[3];
    g.d_C_x[0] = (g.d_C_x[0] + uu) * kScaleF;
    g.d_C_x[1] *= kScaleF;
    g.d_C_x[2] = (g.d_C_x[2] + 1) * kScaleC;
    g.d_C_x[3] *= kScaleC;
    g.d_C_y[0] *= kScaleF;
    g.d_C_y[1] = (g.d_C_y[1] + vv) * kScaleF;
    g.d_C_y[2] *= kScaleC;
    g.d_C_y[3] = (g.d_C_y[3] + 1) * kScaleC;
    const float ni = g.new_idepth;
    g.d_xi_x[0] = ni * fxl;
    g.d_xi_x[1] = 0;
    g.d_xi_x[2] = -ni * uu * fxl;
    g.d_xi_x[3] = -uu * vv * fxl;
    g.d_xi_x[4] = (1 + uu * uu) * fxl;
    g.d_xi_x[5] = -vv * fxl;
    g.d_xi_y[0] = 0;
    g.d_xi_y[1] = ni * fyl;
    g.d_xi_y[2] = -ni * vv * fyl;
    g.d_xi_y[3] = -(1 + vv * vv) * fyl;
    g.d_xi_y[4] = uu * vv * fyl;
    g.d_xi_y[5] = uu * fyl;
    return true;
}

struct PhotoSums {
    float energy, wJI2;
    float JIdx2_00, JIdx2_10, JIdx2_11;
    float JabJIdx_00, JabJIdx_01, JabJIdx_10, JabJIdx_11;
    float Jab2_00, Jab2_01, Jab2_11;
    float JI_r0, JI_r1, Jab_r0, Jab_r1, rr;  // AccumulatedTopHessian.cc:69-77 (mode 0: resApprox = resF)
};

// Pattern loop of Residuals.cc:128-190 with getInterpolatedElement33 (GlobalFuncs.h:89-103).
// The JI_r / Jab_r / rr sums of the Top accumulation are folded into the same loop (same
// order, so identical rounding to summing the stored J afterwards).
__device__ inline bool pattern_loop(const float *__restrict__ pre, const float4 *__restrict__ img, int w,
                                    float wM3, float hM3, float u, float v, float ids,
                                    const float *__restrict__ color, const float *__restrict__ weights,
                                    PhotoSums &s) {
#pragma clang fp contract(off)
    constexpr int pat[8][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0}, {0, 0}, {2, 0}, {-1, 1}, {0, 2}};
    const float aff0 = pre[24], aff1 = pre[25], b0 = pre[26];
    s.energy = s.wJI2 = 0;
    s.JIdx2_00 = s.JIdx2_10 = s.JIdx2_11 = 0;
    s.JabJIdx_00 = s.JabJIdx_01 = s.JabJIdx_10 = s.JabJIdx_11 = 0;
    s.Jab2_00 = s.Jab2_01 = s.Jab2_11 = 0;
    s.JI_r0 = s.JI_r1 = s.Jab_r0 = s.Jab_r1 = s.rr = 0;
    // issue all eight projections first so the 32 texel loads can be in flight together
    float Kus[8], Kvs[8];
    bool ok = true;
#pragma unroll
    for (int idx = 0; idx < 8; idx++) {
        const float up = u + pat[idx][0], vp = v + pat[idx][1];
        float ptp[3];
#pragma unroll
        for (int i = 0; i < 3; i++) ptp[i] = (pre[3 * i] * up + pre[3 * i + 1] * vp + pre[3 * i + 2] * 1.0f) + pre[9 + i] * ids;
        Kus[idx] = ptp[0] / ptp[2];
        Kvs[idx] = ptp[1] / ptp[2];
        ok = ok && (Kus[idx] > 1.1f && Kvs[idx] > 1.1f && Kus[idx] < wM3 && Kvs[idx] < hM3);
    }
    if (!ok) return false;
    float4 t00[8], t10[8], t01[8], t11[8];
    float dxs[8], dys[8];
#pragma unroll
    for (int idx = 0; idx < 8; idx++) {
        const int ix = (int)Kus[idx], iy = (int)Kvs[idx];
        dxs[idx] = Kus[idx] - ix;
        dys[idx] = Kvs[idx] - iy;
        const float4 *bp = img + ix + iy * w;
        t00[idx] = bp[0];
        t10[idx] = bp[1];
        t01[idx] = bp[w];
        t11[idx] = bp[w + 1];
    }
#pragma unroll
    for (int idx = 0; idx < 8; idx++) {
        const float dx = dxs[idx], dy = dys[idx], dxdy = dx * dy;
        const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
        const float I = w11 * t11[idx].x + w01 * t01[idx].x + w10 * t10[idx].x + w00 * t00[idx].x;
        float gx = w11 * t11[idx].y + w01 * t01[idx].y + w10 * t10[idx].y + w00 * t00[idx].y;
        float gy = w11 * t11[idx].z + w01 * t01[idx].z + w10 * t10[idx].z + w00 * t00[idx].z;
        const float residual = I - (float)(aff0 * color[idx] + aff1);
        const float drdA = (color[idx] - b0);
        if (!isfinite(I)) return false;
        float wg = sqrtf(kOutlierTHSumComponent / (kOutlierTHSumComponent + (gx * gx + gy * gy)));
        wg = 0.5f * (wg + weights[idx]);
        float hw = fabsf(residual) < kHuberTH ? 1 : kHuberTH / fabsf(residual);
        s.energy += wg * wg * hw * residual * residual * (2 - hw);
        if (hw < 1) hw = sqrtf(hw);
        hw = hw * wg;
        gx *= hw;
        gy *= hw;
        const float resF = residual * hw;
        const float jab0 = drdA * hw;
        s.JIdx2_00 += gx * gx;
        s.JIdx2_11 += gy * gy;
        s.JIdx2_10 += gx * gy;
        s.JabJIdx_00 += drdA * hw * gx;
        s.JabJIdx_01 += drdA * hw * gy;
        s.JabJIdx_10 += hw * gx;
        s.JabJIdx_11 += hw * gy;
        s.Jab2_00 += drdA * drdA * hw * hw;
        s.Jab2_01 += drdA * hw * hw;
        s.Jab2_11 += hw * hw;
        s.wJI2 += hw * hw * (gx * gx + gy * gy);
        // setting_affineOptModeA/B >= 0 (Setting.cc:65-66): JabF stays as computed
        s.JI_r0 += resF * gx;
        s.JI_r1 += resF * gy;
        s.Jab_r0 += resF * jab0;
        s.Jab_r1 += resF * hw;
        s.rr += resF * resF;
    }
    return true;
}

// Point-side terms of AccumulatedTopHessian.cc:94-97 and takeData (Residuals.h:120-129).
__device__ inline void point_terms(const Geo &g, const PhotoSums &s, float jpjdf[8], float hcd[4], float &hdd,
                                   float &bd) {
#pragma clang fp contract(off)
    const float j0 = s.JIdx2_00 * g.d_d_x + s.JIdx2_10 * g.d_d_y;  // JIdx2 * Jpdd
    const float j1 = s.JIdx2_10 * g.d_d_x + s.JIdx2_11 * g.d_d_y;
#pragma unroll
    for (int i = 0; i < 6; i++) jpjdf[i] = g.d_xi_x[i] * j0 + g.d_xi_y[i] * j1;
    jpjdf[6] = s.JabJIdx_00 * g.d_d_x + s.JabJIdx_01 * g.d_d_y;
    jpjdf[7] = s.JabJIdx_10 * g.d_d_x + s.JabJIdx_11 * g.d_d_y;
    bd = s.JI_r0 * g.d_d_x + s.JI_r1 * g.d_d_y;
    hdd = j0 * g.d_d_x + j1 * g.d_d_y;
#pragma unroll
    for (int i = 0; i < 4; i++) hcd[i] = g.d_C_x[i] * j0 + g.d_C_y[i] * j1;
}

// Recursive-halving wavefront reduction of 96 floats: 96 shuffles instead of 6*96.  On return
// lane l (all 64) holds the full sums of elements base(l) + {0,1,2}, base = 48 b0 + 24 b1 +
// 12 b2 + 6 b3 + 3 b4 (b = bits of the lane id).
template <int L, int M>
__device__ inline void halve(float *v, int lane) {
    constexpr int H = L / 2;
    const bool upper = (lane & M) != 0;
#pragma unroll
    for (int i = 0; i < H; i++) {
        const float send = upper ? v[i] : v[i + H];
        const float keep = upper ? v[i + H] : v[i];
        v[i] = keep + __shfl_xor(send, M, kWave);
    }
}

__global__ __launch_bounds__(256) void k_linearize(LinParams P) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int item = blockIdx.x * 4 + wave;
    if (item >= P.n_items) return;
    const int4 it = P.items[item];
    const WinDev &W = P.wins[it.w];
    const int N = W.N;
    const int aidx = it.z - W.pair_base;
    const int h = aidx % N, t = aidx / N;
    const float *pre = P.precalc + (size_t)it.z * LDSO_BA_PRECALC_STRIDE;
    const float4 *img = P.img + (size_t)(W.frame_base + t) * P.npix;
    const float th = fmaxf(P.frame_th[W.frame_base + h], P.frame_th[W.frame_base + t]);

    const bool valid = lane < it.y;
    const int r = it.x + lane;
    double energy = 0;
    bool isIN = false, active = false;
    Geo g;
    PhotoSums s;
    if (valid) {
        const int8_t old_state = P.rs_state[r];
        uint8_t flags = P.rs_flags[r];
        float state_energy = P.rs_energy[r];
        float new_energy = P.rs_newenergy[r];
        int8_t new_state = LDSO_BA_RES_OOB;
        float e_wo = -1;
        float4 centre = P.rs_center[r];
        if (old_state == LDSO_BA_RES_OOB) {
            energy = state_energy;  // linearize returns state_energy; applyRes returns early
        } else {
            const int p = P.rs_point[r];
            const float *pd = P.pt_data + (size_t)p * LDSO_BA_POINT_STRIDE;
            const float4 pd0 = *(const float4 *)pd;
            float color[8], weights[8];
            *(float4 *)&color[0] = *(const float4 *)(pd + 8);
            *(float4 *)&color[4] = *(const float4 *)(pd + 12);
            *(float4 *)&weights[0] = *(const float4 *)(pd + 16);
            *(float4 *)&weights[4] = *(const float4 *)(pd + 20);
            bool ok = centre_projection(pre, pd0.x, pd0.y, pd0.w, W.calib[0], W.calib[1], W.calib[2], W.calib[3],
                                        W.wM3, W.hM3, g);
            if (ok) {
                centre.x = g.Ku;
                centre.y = g.Kv;
                centre.z = g.new_idepth;
                ok = pattern_loop(pre, img, W.width, W.wM3, W.hM3, pd0.x, pd0.y, pd0.z, color, weights, s);
            }
            if (!ok) {
                energy = state_energy;  // OOB: return state_energy, NewEnergy untouched
            } else {
                e_wo = s.energy;
                float el = s.energy;
                if (el > th || s.wJI2 < 2) {
                    el = th;
                    new_state = LDSO_BA_RES_OUTLIER;
                } else {
                    new_state = LDSO_BA_RES_IN;
                }
                new_energy = el;
                energy = el;
            }
            // applyRes(true), Residuals.h:70-88 (state_state != OOB here)
            active = (new_state == LDSO_BA_RES_IN);
            flags = active ? (flags | LDSO_BA_FLAG_ACTIVE) : (flags & ~LDSO_BA_FLAG_ACTIVE);
            state_energy = new_energy;
            if (active) {
                float jp[8], hc[4], hdd, bd;
                point_terms(g, s, jp, hc, hdd, bd);
                float4 *rec = P.rs_rec + (size_t)r * 4;
                rec[0] = make_float4(jp[0], jp[1], jp[2], jp[3]);
                rec[1] = make_float4(jp[4], jp[5], jp[6], jp[7]);
                rec[2] = make_float4(hc[0], hc[1], hc[2], hc[3]);
                rec[3] = make_float4(hdd, bd, 0.f, 0.f);
            }
            if (P.fix && active && (flags & LDSO_BA_FLAG_NEW)) {
                // linearizeAll_Reductor relBS (FullSystem.cc:1800-1812)
#pragma clang fp contract(off)
                float pi[3], pr[3];
#pragma unroll
                for (int i = 0; i < 3; i++) {
                    pi[i] = pre[3 * i] * pd0.x + pre[3 * i + 1] * pd0.y + pre[3 * i + 2] * 1.0f;
                    pr[i] = pi[i] + pre[9 + i] * pd0.z;
                }
                const float dx = pi[0] / pi[2] - pr[0] / pr[2], dy = pi[1] / pi[2] - pr[1] / pr[2];
                centre.w = 0.01f * sqrtf(dx * dx + dy * dy);
            }
            P.rs_state[r] = new_state;
            P.rs_flags[r] = flags;
            P.rs_energy[r] = state_energy;
            P.rs_newenergy[r] = new_energy;
            P.rs_center[r] = centre;
        }
        isIN = (new_state == LDSO_BA_RES_IN);
        P.rs_newstate[r] = new_state;
        P.rs_energy_wo[r] = e_wo;
    }

    // linearizeAll stats: sum of returned energies (double) and #IN, per chunk
    double esum = energy;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) esum += __shfl_xor(esum, m, kWave);
    const unsigned long long inmask = __ballot(isIN);
    if (lane == 0) {
        P.item_energy[2 * item] = esum;
        P.item_energy[2 * item + 1] = (double)__popcll(inmask);
    }
    if (!P.accumulate) return;

    // AccumulatorApprox::update / updateTopRight / updateBotRight terms (mode 0)
    float v[kTopVals];
    if (active) {
        float x[10], y[10];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            x[i] = g.d_C_x[i];
            y[i] = g.d_C_y[i];
        }
#pragma unroll
        for (int i = 0; i < 6; i++) {
            x[4 + i] = g.d_xi_x[i];
            y[4 + i] = g.d_xi_y[i];
        }
        const float a = s.JIdx2_00, b = s.JIdx2_10, c = s.JIdx2_11;
        int q = 0;
#pragma unroll
        for (int rr = 0; rr < 10; rr++)
#pragma unroll
            for (int cc = rr; cc < 10; cc++) v[q++] = a * x[cc] * x[rr] + c * y[cc] * y[rr] + b * (x[cc] * y[rr] + y[cc] * x[rr]);
#pragma unroll
        for (int rr = 0; rr < 10; rr++) {
            v[55 + 3 * rr] = x[rr] * s.JabJIdx_00 + y[rr] * s.JabJIdx_01;
            v[56 + 3 * rr] = x[rr] * s.JabJIdx_10 + y[rr] * s.JabJIdx_11;
            v[57 + 3 * rr] = x[rr] * s.JI_r0 + y[rr] * s.JI_r1;
        }
        v[85] = s.Jab2_00;
        v[86] = s.Jab2_01;
        v[87] = s.Jab_r0;
        v[88] = s.Jab2_11;
        v[89] = s.Jab_r1;
        v[90] = s.rr;
#pragma unroll
        for (int i = 91; i < kTopVals; i++) v[i] = 0;
    } else {
#pragma unroll
        for (int i = 0; i < kTopVals; i++) v[i] = 0;
    }
    halve<96, 1>(v, lane);
    halve<48, 2>(v, lane);
    halve<24, 4>(v, lane);
    halve<12, 8>(v, lane);
    halve<6, 16>(v, lane);
#pragma unroll
    for (int i = 0; i < 3; i++) v[i] += __shfl_xor(v[i], 32, kWave);
    if (lane < 32) {
        const int base = 48 * (lane & 1) + 24 * ((lane >> 1) & 1) + 12 * ((lane >> 2) & 1) + 6 * ((lane >> 3) & 1) +
                         3 * ((lane >> 4) & 1);
        float *o = P.top_slab + (size_t)item * kTopVals + base;
        o[0] = v[0];
        o[1] = v[1];
        o[2] = v[2];
    }
}

// ============================================================================================
// k_frame_th: setNewFrameEnergyTH via an exact 4-pass radix select (nth_element semantics)
// ============================================================================================
__global__ __launch_bounds__(256) void k_frame_th(const WinDev *__restrict__ wins, const float *__restrict__ e_wo,
                                                 float *frame_th) {
    const WinDev &W = wins[blockIdx.x];
    __shared__ unsigned hist[256];
    __shared__ unsigned s_prefix, s_rank, s_count;
    const int b = W.newest_begin, e = W.newest_end;
    if (threadIdx.x == 0) s_count = 0;
    __syncthreads();
    unsigned cnt = 0;
    for (int i = b + threadIdx.x; i < e; i += blockDim.x) cnt += (e_wo[i] >= 0);
    atomicAdd(&s_count, cnt);
    __syncthreads();
    const unsigned n = s_count;
    if (n == 0) {
        if (threadIdx.x == 0) frame_th[W.frame_base + W.N - 1] = 12 * 12 * LDSO_BA_PATTERN_NUM;
        return;
    }
    if (threadIdx.x == 0) {
        s_prefix = 0;
        s_rank = (unsigned)(int)(kFrameEnergyTHN * (float)n);
    }
    for (int pass = 0; pass < 4; pass++) {
        const int shift = 24 - 8 * pass;
        for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
        __syncthreads();
        const unsigned prefix = s_prefix;
        const unsigned pmask = pass == 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * pass));
        for (int i = b + threadIdx.x; i < e; i += blockDim.x) {
            const float x = e_wo[i];
            if (!(x >= 0)) continue;
            const unsigned key = __float_as_uint(x) & 0x7FFFFFFFu;  // -0.0 -> 0
            if ((key & pmask) != (prefix & pmask)) continue;
            atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned rank = s_rank, acc = 0;
            int d = 0;
            for (; d < 256; d++) {
                if (acc + hist[d] > rank) break;
                acc += hist[d];
            }
            s_rank = rank - acc;
            s_prefix = prefix | ((unsigned)d << shift);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
#pragma clang fp contract(off)
        const float nth = sqrtf(__uint_as_float(s_prefix));
        float v = nth * kFrameEnergyTHFacMedian;
        v = 26.0f * kFrameEnergyTHConstWeight + v * (1 - kFrameEnergyTHConstWeight);
        v = v * v;
        v *= kOverallEnergyTHWeight * kOverallEnergyTHWeight;
        frame_th[W.frame_base + W.N - 1] = v;
    }
}

// ============================================================================================
// k_point_sc
// ============================================================================================
struct PointParams {
    const int4 *__restrict__ items;  // {pt_begin, count, host, win}
    const WinDev *__restrict__ wins;
    const float *__restrict__ pt_data;
    const int *__restrict__ pt_nres;
    const int *__restrict__ pt_res;   // [P][kMaxRes]
    const uint8_t *__restrict__ rs_tgt;
    const uint8_t *__restrict__ rs_flags;
    const float4 *__restrict__ rs_rec;
    float *pt_out;                     // [P][12]
    float *sc_slab;
    int n_items;
};

__global__ __launch_bounds__(256) void k_point_sc(PointParams P) {
    const int4 it = P.items[blockIdx.x];
    const WinDev &W = P.wins[it.w];
    const int host = it.z, KP = W.KP, nt = KP / 4, ntiles = W.ntiles;
    const int Kj = 8 * (W.N - 1);
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *U = smem;               // [64][KP]
    float *Wt = smem + 64 * KP;    // [64]
    const int tid = threadIdx.x;
    for (int i = tid; i < 64 * KP; i += blockDim.x) U[i] = 0;
    __syncthreads();
    if (tid < it.y) {
#pragma clang fp contract(off)
        const int p = it.x + tid;
        const int nres = P.pt_nres[p];
        float hdd = 0, bd = 0, hcd[4] = {0, 0, 0, 0};
        int ngood = 0;
        float *row = U + tid * KP;
        for (int k = 0; k < nres; k++) {
            const int r = P.pt_res[(size_t)p * kMaxRes + k];
            if (!(P.rs_flags[r] & LDSO_BA_FLAG_ACTIVE)) continue;
            ngood++;
            const float4 *rec = P.rs_rec + (size_t)r * 4;
            const float4 j0 = rec[0], j1 = rec[1], hc = rec[2], hb = rec[3];
            bd += hb.y;
            hdd += hb.x;
            hcd[0] += hc.x;
            hcd[1] += hc.y;
            hcd[2] += hc.z;
            hcd[3] += hc.w;
            const int tg = P.rs_tgt[r];
            const int slot = tg < host ? tg : tg - 1;
            *(float4 *)(row + 8 * slot) = j0;
            *(float4 *)(row + 8 * slot + 4) = j1;
        }
        const float *pd = P.pt_data + (size_t)p * LDSO_BA_POINT_STRIDE;
        const float priorF = pd[4], deltaF = pd[5];
        float HdiF = 0, bdSum = 0, ih = 0;
        if (ngood > 0) {
            // AccumulatedSCHessian.cc:24-33 (Hdd_accLF = bd_accLF = Hcd_accLF = 0 in the hot path)
            float H = hdd + 0.0f + priorF;
            if (H < 1e-10f) H = 1e-10f;
            ih = H;
            HdiF = (float)(1.0 / (double)H);
            bdSum = bd + 0.0f;
            bdSum += priorF * deltaF;
            row[Kj + 0] = hcd[0] + 0.0f;
            row[Kj + 1] = hcd[1] + 0.0f;
            row[Kj + 2] = hcd[2] + 0.0f;
            row[Kj + 3] = hcd[3] + 0.0f;
            row[Kj + 4] = bdSum;
        }
        Wt[tid] = HdiF;
        float *o = P.pt_out + (size_t)p * 12;
        o[0] = HdiF;
        o[1] = bdSum;
        o[2] = ih;
        o[3] = hdd;
        o[4] = bd;
        o[5] = hcd[0];
        o[6] = hcd[1];
        o[7] = hcd[2];
        o[8] = hcd[3];
        o[9] = (float)ngood;
    }
    __syncthreads();
    // symmetric rank-k update of the upper 4x4 tiles: G += U^T diag(HdiF) U
    const int cnt = it.y;
    float *slab = P.sc_slab + W.sc_slab_base + (size_t)(blockIdx.x - W.sc_item_base) * ntiles * 16;
    for (int tile = tid; tile < ntiles; tile += blockDim.x) {
        int a = 0, rem = tile;
        while (rem >= nt - a) {
            rem -= nt - a;
            a++;
        }
        const int bb = a + rem;
        float acc[16];
#pragma unroll
        for (int i = 0; i < 16; i++) acc[i] = 0;
        for (int p = 0; p < cnt; p++) {
            const float wgt = Wt[p];
            const float4 ua = *(const float4 *)(U + p * KP + 4 * a);
            const float4 ub = *(const float4 *)(U + p * KP + 4 * bb);
            const float wa[4] = {wgt * ua.x, wgt * ua.y, wgt * ua.z, wgt * ua.w};
            const float ubv[4] = {ub.x, ub.y, ub.z, ub.w};
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i * 4 + j] += wa[i] * ubv[j];
        }
        float4 *o = (float4 *)(slab + (size_t)tile * 16);
        o[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        o[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
        o[2] = make_float4(acc[8], acc[9], acc[10], acc[11]);
        o[3] = make_float4(acc[12], acc[13], acc[14], acc[15]);
    }
}

// ============================================================================================
// k_stitch_top: per (h,t) pair, AccumulatedTopHessian.cc:213-239 (double)
// ============================================================================================
struct TopStitchParams {
    const WinDev *__restrict__ wins;
    const int *__restrict__ pair_win;
    const int2 *__restrict__ pair_items;  // {first item, n items}
    const float *__restrict__ top_slab;
    const double *__restrict__ adH;
    const double *__restrict__ adT;
    double *top_rec;
};

__global__ __launch_bounds__(64) void k_stitch_top(TopStitchParams P) {
    const int pair = blockIdx.x;
    const WinDev &W = P.wins[P.pair_win[pair]];
    const int N = W.N, aidx = pair - W.pair_base, h = aidx % N, t = aidx / N;
    if (h == t) return;
    __shared__ double acc[kTopVals];
    __shared__ double A[13][13];
    __shared__ double AH[64], AT[64], TH[64], TT[64];
    const int tid = threadIdx.x;
    const int2 pi = P.pair_items[pair];
    for (int j = tid; j < kTopVals; j += 64) {
        double s = 0;
        for (int k = 0; k < pi.y; k++) s += (double)P.top_slab[(size_t)(pi.x + k) * kTopVals + j];
        acc[j] = s;
    }
    AH[tid] = P.adH[(size_t)pair * 64 + tid];
    AT[tid] = P.adT[(size_t)pair * 64 + tid];
    __syncthreads();
    if (tid == 0) {  // AccumulatorApprox::finish layout (MatrixAccumulators.h:771-800)
        int q = 0;
        for (int r = 0; r < 10; r++)
            for (int c = r; c < 10; c++) {
                A[r][c] = A[c][r] = acc[q];
                q++;
            }
        for (int r = 0; r < 10; r++)
            for (int c = 0; c < 3; c++) A[r][10 + c] = A[10 + c][r] = acc[55 + 3 * r + c];
        A[10][10] = acc[85];
        A[10][11] = A[11][10] = acc[86];
        A[10][12] = A[12][10] = acc[87];
        A[11][11] = acc[88];
        A[11][12] = A[12][11] = acc[89];
        A[12][12] = acc[90];
    }
    __syncthreads();
    const int r = tid >> 3, c = tid & 7;
    {
        double sh = 0, st = 0;
        for (int k = 0; k < 8; k++) {
            sh += AH[r * 8 + k] * A[4 + k][4 + c];
            st += AT[r * 8 + k] * A[4 + k][4 + c];
        }
        TH[tid] = sh;
        TT[tid] = st;
    }
    __syncthreads();
    double *rec = P.top_rec + W.top_rec_base + (size_t)aidx * kTopRecLen;
    {
        double hh = 0, tt = 0, ht = 0;
        for (int k = 0; k < 8; k++) {
            hh += TH[r * 8 + k] * AH[c * 8 + k];
            tt += TT[r * 8 + k] * AT[c * 8 + k];
            ht += TH[r * 8 + k] * AT[c * 8 + k];
        }
        rec[tid] = hh;
        rec[64 + tid] = tt;
        rec[128 + tid] = ht;
    }
    if (tid < 32) {  // H(h,c), H(t,c): 8x4
        const int rr = tid >> 2, cc = tid & 3;
        double sh = 0, st = 0;
        for (int k = 0; k < 8; k++) {
            sh += AH[rr * 8 + k] * A[4 + k][cc];
            st += AT[rr * 8 + k] * A[4 + k][cc];
        }
        rec[192 + tid] = sh;
        rec[224 + tid] = st;
    }
    if (tid < 16) rec[256 + tid] = A[tid >> 2][tid & 3];
    if (tid < 8) {
        double sh = 0, st = 0;
        for (int k = 0; k < 8; k++) {
            sh += AH[tid * 8 + k] * A[4 + k][12];
            st += AT[tid * 8 + k] * A[4 + k][12];
        }
        rec[272 + tid] = sh;
        rec[280 + tid] = st;
    }
    if (tid < 4) rec[288 + tid] = A[tid][12];
}

// ============================================================================================
// k_sc_reduce: per (window, host) sum of the chunk partials into G_h (double, full symmetric)
// ============================================================================================
struct ScReduceParams {
    const WinDev *__restrict__ wins;
    const int *__restrict__ frame_win;
    const int2 *__restrict__ host_items;  // per global frame: {first sc item, n items}
    const float *__restrict__ sc_slab;
    double *G;
};

__global__ __launch_bounds__(256) void k_sc_reduce(ScReduceParams P) {
    const int fg = blockIdx.x;
    const WinDev &W = P.wins[P.frame_win[fg]];
    const int host = fg - W.frame_base, KP = W.KP, nt = KP / 4, ntiles = W.ntiles;
    const int2 hi = P.host_items[fg];
    double *G = P.G + W.g_base + (size_t)host * KP * KP;
    for (int e = threadIdx.x; e < ntiles * 16; e += blockDim.x) {
        const int tile = e >> 4, ii = (e >> 2) & 3, jj = e & 3;
        double s = 0;
        for (int k = 0; k < hi.y; k++)
            s += (double)P.sc_slab[W.sc_slab_base + (size_t)(hi.x - W.sc_item_base + k) * ntiles * 16 + e];
        int a = 0, rem = tile;
        while (rem >= nt - a) {
            rem -= nt - a;
            a++;
        }
        const int bb = a + rem;
        const int row = 4 * a + ii, col = 4 * bb + jj;
        G[(size_t)row * KP + col] = s;
        G[(size_t)col * KP + row] = s;
    }
}

// ============================================================================================
// k_stitch_sc: per (host i, target j): AccumulatedSCHessian.cc:80-114 (double)
// record: Hjk[N][64] | Hji[64] | Hii[64] | Hic[32] | Hjc[32] | bi[8] | bj[8]
// ============================================================================================
struct ScStitchParams {
    const WinDev *__restrict__ wins;
    const int *__restrict__ pair_win;
    const double *__restrict__ G;
    const double *__restrict__ adH;
    const double *__restrict__ adT;
    double *sc_rec;
};

__global__ __launch_bounds__(64) void k_stitch_sc(ScStitchParams P) {
    const int pair = blockIdx.x;
    const WinDev &W = P.wins[P.pair_win[pair]];
    const int N = W.N, aidx = pair - W.pair_base, i = aidx % N, j = aidx / N;
    if (i == j) return;
    const int KP = W.KP, Kc = 8 * (N - 1), sj = j < i ? j : j - 1;
    const double *G = P.G + W.g_base + (size_t)i * KP * KP;
    __shared__ double AHij[64], ATij[64], AHik[64], ATik[64], Dm[64], X[64], S[64];
    const int tid = threadIdx.x, r = tid >> 3, c = tid & 7;
    AHij[tid] = P.adH[(size_t)pair * 64 + tid];
    ATij[tid] = P.adT[(size_t)pair * 64 + tid];
    double *rec = P.sc_rec + W.sc_rec_base + (size_t)aidx * sc_rec_len(N);
    double sacc = 0;  // S = sum_k D_jk * AH_ik^T
    for (int k = 0; k < N; k++) {
        if (k == i) continue;
        const int sk = k < i ? k : k - 1;
        const int pik = W.pair_base + i + N * k;
        __syncthreads();
        Dm[tid] = G[(size_t)(8 * sj + r) * KP + 8 * sk + c];
        AHik[tid] = P.adH[(size_t)pik * 64 + tid];
        ATik[tid] = P.adT[(size_t)pik * 64 + tid];
        __syncthreads();
        double x = 0, sv = 0;
        for (int q = 0; q < 8; q++) {
            x += ATij[r * 8 + q] * Dm[q * 8 + c];
            sv += Dm[r * 8 + q] * AHik[c * 8 + q];
        }
        X[tid] = x;
        sacc += sv;
        __syncthreads();
        double hjk = 0;
        for (int q = 0; q < 8; q++) hjk += X[r * 8 + q] * ATik[c * 8 + q];
        rec[k * 64 + tid] = hjk;  // H(j,k) += AT_ij D AT_ik^T
    }
    __syncthreads();
    S[tid] = sacc;
    __syncthreads();
    double hji = 0, hii = 0;
    for (int q = 0; q < 8; q++) {
        hji += ATij[r * 8 + q] * S[q * 8 + c];
        hii += AHij[r * 8 + q] * S[q * 8 + c];
    }
    rec[N * 64 + tid] = hji;       // H(j,i) += sum_k AT_ij D AH_ik^T
    rec[N * 64 + 64 + tid] = hii;  // H(i,i) += sum_k AH_ij D AH_ik^T
    if (tid < 32) {
        const int rr = tid >> 2, cc = tid & 3;
        double hi = 0, hj = 0;
        for (int q = 0; q < 8; q++) {
            const double e = G[(size_t)(8 * sj + q) * KP + Kc + cc];
            hi += AHij[rr * 8 + q] * e;
            hj += ATij[rr * 8 + q] * e;
        }
        rec[N * 64 + 128 + tid] = hi;
        rec[N * 64 + 160 + tid] = hj;
    }
    if (tid < 8) {
        double bi = 0, bj = 0;
        for (int q = 0; q < 8; q++) {
            const double e = G[(size_t)(8 * sj + q) * KP + Kc + 4];
            bi += AHij[tid * 8 + q] * e;
            bj += ATij[tid * 8 + q] * e;
        }
        rec[N * 64 + 192 + tid] = bi;
        rec[N * 64 + 200 + tid] = bj;
    }
}

// ============================================================================================
// k_final: per window, assemble the packed upper triangles of HA, Hsc and bA, bsc, and the
// linearizeAll energy; symmetrisation as in AccumulatedTopHessian.h:91-104 / SC.h:91-97
// ============================================================================================
struct FinalParams {
    const WinDev *__restrict__ wins;
    const double *__restrict__ top_rec;
    const double *__restrict__ sc_rec;
    const double *__restrict__ G;
    const double *__restrict__ item_energy;
    double *sys;
    double *win_energy;  // [win][2]
    int accumulate;
};

__device__ inline void decode(int x, int &f, int &k) {  // H index -> (frame or -1 for calib, k)
    if (x < 4) {
        f = -1;
        k = x;
    } else {
        f = (x - 4) >> 3;
        k = (x - 4) & 7;
    }
}

__global__ __launch_bounds__(256) void k_final(FinalParams P) {
    const int w = blockIdx.x;
    const WinDev &W = P.wins[w];
    if (threadIdx.x == 0) {
        double e = 0, n = 0;
        for (int k = 0; k < W.n_top_items; k++) {
            e += P.item_energy[2 * (W.top_item_base + k)];
            n += P.item_energy[2 * (W.top_item_base + k) + 1];
        }
        P.win_energy[2 * w] = e;
        P.win_energy[2 * w + 1] = n;
    }
    if (!P.accumulate) return;
    const int N = W.N, D = W.D, KP = W.KP, Kc = 8 * (N - 1);
    const int srl = sc_rec_len(N);
    const double *trec = P.top_rec + W.top_rec_base;
    const double *srec = P.sc_rec + W.sc_rec_base;
    const double *G = P.G + W.g_base;
    auto T = [&](int h, int t) { return trec + (size_t)(h + N * t) * kTopRecLen; };
    auto S = [&](int i, int j) { return srec + (size_t)(i + N * j) * srl; };
    double *sys = P.sys + W.sys_base;
    const long long pl = packed_len(D);
    for (long long q = threadIdx.x; q < pl + D; q += blockDim.x) {
        double ha = 0, hs = 0;
        long long out = q;
        if (q < pl) {
            // packed index -> (row, col >= row)
            int row = (int)((2.0 * D + 1 - sqrt((2.0 * D + 1) * (2.0 * D + 1) - 8.0 * (double)q)) / 2);
            while ((long long)row * D - (long long)row * (row - 1) / 2 > q) row--;
            while ((long long)(row + 1) * D - (long long)(row + 1) * row / 2 <= q) row++;
            const int col = row + (int)(q - ((long long)row * D - (long long)row * (row - 1) / 2));
            int fa, ra, fb, cb;
            decode(row, fa, ra);
            decode(col, fb, cb);
            if (fa < 0 && fb < 0) {
                for (int k = 0; k < N * N; k++) {
                    const int h = k % N, t = k / N;
                    if (h != t) ha += T(h, t)[256 + ra * 4 + cb];
                }
                for (int i = 0; i < N; i++) hs += G[(size_t)i * KP * KP + (size_t)(Kc + ra) * KP + Kc + cb];
            } else if (fa < 0) {  // H(c, frame b) = H(b, c)^T
                const int b = fb;
                for (int t = 0; t < N; t++)
                    if (t != b) ha += T(b, t)[192 + cb * 4 + ra];
                for (int h = 0; h < N; h++)
                    if (h != b) ha += T(h, b)[224 + cb * 4 + ra];
                for (int j = 0; j < N; j++)
                    if (j != b) hs += S(b, j)[N * 64 + 128 + cb * 4 + ra];
                for (int i = 0; i < N; i++)
                    if (i != b) hs += S(i, b)[N * 64 + 160 + cb * 4 + ra];
            } else if (fa == fb) {
                const int a = fa, e = ra * 8 + cb;
                for (int t = 0; t < N; t++)
                    if (t != a) ha += T(a, t)[e];
                for (int h = 0; h < N; h++)
                    if (h != a) ha += T(h, a)[64 + e];
                for (int i = 0; i < N; i++)
                    if (i != a) hs += S(i, a)[a * 64 + e];
                for (int j = 0; j < N; j++)
                    if (j != a) hs += S(a, j)[N * 64 + 64 + e];
            } else {  // a < b
                const int a = fa, b = fb;
                ha = T(a, b)[128 + ra * 8 + cb] + T(b, a)[128 + cb * 8 + ra];
                for (int i = 0; i < N; i++)
                    if (i != a && i != b) hs += S(i, a)[b * 64 + ra * 8 + cb];
                hs += S(b, a)[N * 64 + ra * 8 + cb];
                hs += S(a, b)[N * 64 + cb * 8 + ra];
            }
        } else {
            const int x = (int)(q - pl);
            int fa, ra;
            decode(x, fa, ra);
            if (fa < 0) {
                for (int k = 0; k < N * N; k++) {
                    const int h = k % N, t = k / N;
                    if (h != t) ha += T(h, t)[288 + ra];
                }
                for (int i = 0; i < N; i++) hs += G[(size_t)i * KP * KP + (size_t)(Kc + ra) * KP + Kc + 4];
            } else {
                const int a = fa;
                for (int t = 0; t < N; t++)
                    if (t != a) ha += T(a, t)[272 + ra];
                for (int h = 0; h < N; h++)
                    if (h != a) ha += T(h, a)[280 + ra];
                for (int j = 0; j < N; j++)
                    if (j != a) hs += S(a, j)[N * 64 + 192 + ra];
                for (int i = 0; i < N; i++)
                    if (i != a) hs += S(i, a)[N * 64 + 200 + ra];
            }
            out = pl + x;
        }
        sys[out] = ha;                 // {HA upper, bA}
        sys[pl + D + out] = hs;        // {Hsc upper, bsc}
    }
}

// ============================================================================================
// k_resubstitute: EnergyFunctional::resubstituteFPt (EnergyFunctional.cc:638-667)
// ============================================================================================
struct ResubParams {
    const float *__restrict__ xad;   // [N*N][8] for this window (index h*N + t)
    const float *__restrict__ xc;    // [4]
    const int *__restrict__ pt_nres;
    const int *__restrict__ pt_res;
    const uint8_t *__restrict__ rs_tgt;
    const uint8_t *__restrict__ rs_flags;
    const float4 *__restrict__ rs_rec;
    const float *__restrict__ pt_out;
    const int *__restrict__ pt_host;
    float *pt_step;
    int begin, count, N;
    float lambda;
};

__global__ __launch_bounds__(256) void k_resubstitute(ResubParams P) {
#pragma clang fp contract(off)
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P.count) return;
    const int p = P.begin + k;
    const float *po = P.pt_out + (size_t)p * 12;
    if (po[9] == 0) {
        P.pt_step[p] = 0;
        return;
    }
    float b = po[1];
    const float d = P.xc[0] * po[5] + P.xc[1] * po[6] + P.xc[2] * po[7] + P.xc[3] * po[8];
    b -= d;
    const int h = P.pt_host[p];
    for (int q = 0; q < P.pt_nres[p]; q++) {
        const int r = P.pt_res[(size_t)p * kMaxRes + q];
        if (!(P.rs_flags[r] & LDSO_BA_FLAG_ACTIVE)) continue;
        const float *xa = P.xad + (size_t)(h * P.N + P.rs_tgt[r]) * 8;
        const float4 j0 = P.rs_rec[(size_t)r * 4], j1 = P.rs_rec[(size_t)r * 4 + 1];
        const float dd = xa[0] * j0.x + xa[1] * j0.y + xa[2] * j0.z + xa[3] * j0.w + xa[4] * j1.x + xa[5] * j1.y +
                         xa[6] * j1.z + xa[7] * j1.w;
        b -= dd;
    }
    if (!isfinite(b)) return;  // reference returns from the chunk; the step is left unchanged
    P.pt_step[p] = -b * po[0] / (1 + P.lambda);
}

// image repack: FrameHessian::dI AoS float3 -> float4 (16-B aligned texel loads)
__global__ void k_repack(const float *__restrict__ src, float4 *dst, int npix) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < npix) dst[i] = make_float4(src[3 * i], src[3 * i + 1], src[3 * i + 2], 0.f);
}

// ============================================================================================
// host side
// ============================================================================================
template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    int alloc(size_t count) {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = count;
        if (count == 0) return 0;
        hipError_t e = hipMalloc(&p, count * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            return fail(-3, std::string("hipMalloc failed: ") + hipGetErrorString(e));
        }
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    size_t bytes() const { return n * sizeof(T); }
};

struct WinHost {
    int N, P, R;                    // this shard
    int P_all, R_all;               // caller's counts
    std::vector<int> pt_orig;       // sorted -> caller point index
    std::vector<int> rs_orig;       // sorted -> caller residual index
    std::vector<int> pt_host;       // sorted point host
    std::vector<double> c_prior, frame_prior, frame_delta_prior;
    std::vector<float> c_delta;
    std::vector<float> adHF, adTF;  // float adjoints (resubstitute)
    bool add_priors = true;
};

struct PendingEv {
    int slot;
    hipEvent_t a, b;
};

}  // namespace

struct ldso_ba_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int n_win = 0, width = 0, height = 0, npix = 0;
    std::vector<WinHost> wh;
    std::vector<WinDev> wd;
    int n_top_items = 0, n_sc_items = 0, n_pairs = 0, n_frames = 0, P_tot = 0, R_tot = 0;
    DevBuf<WinDev> d_wins;
    DevBuf<float4> d_img;
    DevBuf<float> d_precalc, d_frame_th, d_pt_data, d_pt_out, d_pt_step;
    DevBuf<double> d_adH, d_adT;
    DevBuf<int> d_rs_point, d_pt_nres, d_pt_res, d_pair_win, d_frame_win, d_pt_host;
    DevBuf<uint8_t> d_rs_tgt, d_rs_flags;
    DevBuf<int8_t> d_rs_state, d_rs_newstate;
    DevBuf<float> d_rs_energy, d_rs_newenergy, d_rs_energy_wo;
    DevBuf<float4> d_rs_center, d_rs_rec;
    DevBuf<int4> d_top_items, d_sc_items;
    DevBuf<int2> d_pair_items, d_host_items;
    DevBuf<float> d_top_slab, d_sc_slab;
    DevBuf<double> d_item_energy, d_top_rec, d_sc_rec, d_G, d_sys, d_win_energy;
    DevBuf<float> d_xad;
    size_t sc_smem_max = 0;
    bool timing = false;
    std::vector<PendingEv> pending;
    std::vector<hipEvent_t> ev_pool;
    double kms[kNumKernels] = {0};
    long long kcount[kNumKernels] = {0};
    std::vector<double> sys_host;  // last downloaded packed systems
    bool sys_host_valid = false;
    std::vector<double> energy_host;
    bool energy_valid = false;
};

namespace {

hipEvent_t get_event(ldso_ba_ctx *c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
}

void drain_events(ldso_ba_ctx *c) {
    for (auto &pe : c->pending) {
        (void)hipEventSynchronize(pe.b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, pe.a, pe.b);
        c->kms[pe.slot] += ms;
        c->kcount[pe.slot] += 1;
        c->ev_pool.push_back(pe.a);
        c->ev_pool.push_back(pe.b);
    }
    c->pending.clear();
}

template <typename F>
int timed_launch(ldso_ba_ctx *c, int slot, F &&launch) {
    hipEvent_t a = nullptr, b = nullptr;
    if (c->timing) {
        a = get_event(c);
        b = get_event(c);
        (void)hipEventRecord(a, c->stream);
    }
    launch();
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(-2, std::string("launch ") + kKernelNames[slot] + ": " + hipGetErrorString(e));
    if (c->timing) {
        (void)hipEventRecord(b, c->stream);
        c->pending.push_back({slot, a, b});
    }
    return 0;
}

int check_window(const ldso_ba_window &w) {
    if (w.n_frames < 2 || w.n_frames > LDSO_BA_MAX_FRAMES) return fail(-1, "n_frames out of range [2,16]");
    if (w.n_points < 0 || w.n_residuals < 0) return fail(-1, "negative counts");
    if (!w.dI || !w.frame_energy_th || !w.precalc || !w.ad_host || !w.ad_target || !w.c_prior || !w.c_delta ||
        !w.frame_prior || !w.frame_delta_prior)
        return fail(-1, "null frame-level pointer");
    if (w.n_points > 0 && (!w.point_host || !w.point_data || !w.point_res_begin))
        return fail(-1, "null point pointer");
    if (w.n_residuals > 0 && (!w.res_target || !w.res_state || !w.res_energy || !w.res_flags))
        return fail(-1, "null residual pointer");
    if (w.width < 8 || w.height < 8) return fail(-1, "image too small");
    if (w.point_res_begin && (w.point_res_begin[0] != 0 || w.point_res_begin[w.n_points] != w.n_residuals))
        return fail(-1, "point_res_begin must span [0, n_residuals]");
    for (int p = 0; p < w.n_points; p++) {
        const int h = w.point_host[p];
        if (h < 0 || h >= w.n_frames) return fail(-1, "point_host out of range");
        const int b = w.point_res_begin[p], e = w.point_res_begin[p + 1];
        if (e < b || e - b > kMaxRes) return fail(-1, "a point has more than N-1 residuals");
        unsigned seen = 0;
        for (int k = b; k < e; k++) {
            const int t = w.res_target[k];
            if (t < 0 || t >= w.n_frames || t == h) return fail(-1, "res_target out of range or equal to host");
            if (seen & (1u << t)) return fail(-1, "duplicate (point, target) residual");
            seen |= 1u << t;
        }
    }
    return 0;
}

size_t sc_smem_bytes(int KP) { return (size_t)(64 * KP + 64) * sizeof(float); }

}  // namespace

// =========================================================================================
// C ABI
// =========================================================================================
extern "C" {

int ldso_ba_abi_version(void) { return LDSO_BA_ABI_VERSION; }
const char *ldso_ba_last_error(void) { return g_err.c_str(); }

int ldso_ba_frame_precalc(int32_t n, const ldso_ba_frame_state *f, const float calib[4], float *out) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !f || !calib || !out) return fail(-1, "bad arguments");
    return frame_precalc(n, f, calib, out);
}
int ldso_ba_set_adjoints(int32_t n, const ldso_ba_frame_state *f, double *adH, double *adT, double *cp) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !f || !adH || !adT) return fail(-1, "bad arguments");
    return set_adjoints(n, f, adH, adT, cp);
}
int ldso_ba_frame_take_data(int32_t n, const ldso_ba_frame_state *f, double *prior, double *delta, double *dp) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !f) return fail(-1, "bad arguments");
    return frame_take_data(n, f, prior, delta, dp);
}
int ldso_ba_nullspaces(int32_t n, const ldso_ba_frame_state *f, double *out) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !f || !out) return fail(-1, "bad arguments");
    return nullspaces(n, f, out);
}
int ldso_ba_solve_system(int32_t n, int32_t it, double lambda, const double *HA, const double *bA, const double *HL,
                         const double *bL, const double *HM, const double *bM, const double *Hsc, const double *bsc,
                         const double *ns, int32_t nn, double *x) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !HA || !bA || !HL || !bL || !Hsc || !bsc || !x)
        return fail(-1, "bad arguments");
    return solve_system(n, it, lambda, HA, bA, HL, bL, HM, bM, Hsc, bsc, ns, nn, x);
}

int ldso_ba_create(int32_t device, ldso_ba_ctx **out) {
    if (!out) return fail(-1, "null out");
    *out = nullptr;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(-1, "no such HIP device");
    HIP_TRY(hipSetDevice(device));
    ldso_ba_ctx *c = new ldso_ba_ctx();
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(-2, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    *out = c;
    return 0;
}

void ldso_ba_destroy(ldso_ba_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    drain_events(c);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    c->d_wins.release();
    c->d_img.release();
    c->d_precalc.release();
    c->d_frame_th.release();
    c->d_pt_data.release();
    c->d_pt_out.release();
    c->d_pt_step.release();
    c->d_adH.release();
    c->d_adT.release();
    c->d_rs_point.release();
    c->d_pt_nres.release();
    c->d_pt_res.release();
    c->d_pair_win.release();
    c->d_frame_win.release();
    c->d_pt_host.release();
    c->d_rs_tgt.release();
    c->d_rs_flags.release();
    c->d_rs_state.release();
    c->d_rs_newstate.release();
    c->d_rs_energy.release();
    c->d_rs_newenergy.release();
    c->d_rs_energy_wo.release();
    c->d_rs_center.release();
    c->d_rs_rec.release();
    c->d_top_items.release();
    c->d_sc_items.release();
    c->d_pair_items.release();
    c->d_host_items.release();
    c->d_top_slab.release();
    c->d_sc_slab.release();
    c->d_item_energy.release();
    c->d_top_rec.release();
    c->d_sc_rec.release();
    c->d_G.release();
    c->d_sys.release();
    c->d_win_energy.release();
    c->d_xad.release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

void *ldso_ba_stream(ldso_ba_ctx *c) { return c ? (void *)c->stream : nullptr; }

int ldso_ba_load(ldso_ba_ctx *c, int32_t n_windows, const ldso_ba_window *ws, int32_t shard_rank,
                 int32_t shard_count) {
    if (!c || n_windows < 1 || !ws) return fail(-1, "bad arguments");
    if (shard_count < 1 || shard_rank < 0 || shard_rank >= shard_count) return fail(-1, "bad shard");
    for (int w = 0; w < n_windows; w++) {
        int rc = check_window(ws[w]);
        if (rc) return rc;
        if (ws[w].width != ws[0].width || ws[w].height != ws[0].height)
            return fail(-1, "all windows of a context must share the image size");
    }
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->n_win = n_windows;
    c->width = ws[0].width;
    c->height = ws[0].height;
    c->npix = c->width * c->height;
    c->wh.assign(n_windows, WinHost());
    c->wd.assign(n_windows, WinDev());
    c->sys_host_valid = false;
    c->energy_valid = false;

    // host-side layout
    std::vector<int4> top_items, sc_items;
    std::vector<int2> pair_items, host_items;
    std::vector<int> pair_win, frame_win, rs_point, pt_nres, pt_res, pt_host;
    std::vector<uint8_t> rs_tgt, rs_flags;
    std::vector<int8_t> rs_state;
    std::vector<float> rs_energy, pt_data, precalc, frame_th;
    std::vector<double> adH, adT;
    long long sc_slab_total = 0, g_total = 0, sc_rec_total = 0, top_rec_total = 0, sys_total = 0;
    int frame_base = 0, pair_base = 0, point_base = 0, res_base = 0;
    size_t smem_max = 0;

    for (int w = 0; w < n_windows; w++) {
        const ldso_ba_window &in = ws[w];
        WinHost &H = c->wh[w];
        WinDev &D = c->wd[w];
        const int N = in.n_frames;
        H.N = N;
        H.P_all = in.n_points;
        H.R_all = in.n_residuals;
        H.add_priors = (shard_rank == 0);
        H.c_prior.assign(in.c_prior, in.c_prior + 4);
        H.c_delta.assign(in.c_delta, in.c_delta + 4);
        H.frame_prior.assign(in.frame_prior, in.frame_prior + 8 * N);
        H.frame_delta_prior.assign(in.frame_delta_prior, in.frame_delta_prior + 8 * N);
        H.adHF.resize((size_t)N * N * 64);
        H.adTF.resize((size_t)N * N * 64);
        for (size_t k = 0; k < H.adHF.size(); k++) {
            H.adHF[k] = (float)in.ad_host[k];
            H.adTF[k] = (float)in.ad_target[k];
        }
        // points: stable order by host frame, then round-robin shard
        std::vector<int> order;
        order.reserve(in.n_points);
        for (int f = 0; f < N; f++)
            for (int p = 0; p < in.n_points; p++)
                if (in.point_host[p] == f) order.push_back(p);
        for (size_t q = 0; q < order.size(); q++)
            if ((int)(q % shard_count) == shard_rank) H.pt_orig.push_back(order[q]);
        const int P = (int)H.pt_orig.size();
        H.P = P;
        // residual bucket sort by pair index h + N t (stable in point order)
        std::vector<int> bucket_cnt(N * N, 0);
        int R = 0;
        for (int q = 0; q < P; q++) {
            const int p = H.pt_orig[q], h = in.point_host[p];
            for (int k = in.point_res_begin[p]; k < in.point_res_begin[p + 1]; k++) {
                bucket_cnt[h + N * in.res_target[k]]++;
                R++;
            }
        }
        H.R = R;
        std::vector<int> bucket_start(N * N + 1, 0);
        for (int b = 0; b < N * N; b++) bucket_start[b + 1] = bucket_start[b] + bucket_cnt[b];
        std::vector<int> fill(bucket_start.begin(), bucket_start.end() - 1);
        H.rs_orig.assign(R, -1);
        std::vector<int> res_pos_of(in.n_residuals, -1);
        for (int q = 0; q < P; q++) {
            const int p = H.pt_orig[q], h = in.point_host[p];
            for (int k = in.point_res_begin[p]; k < in.point_res_begin[p + 1]; k++) {
                const int pos = fill[h + N * in.res_target[k]]++;
                H.rs_orig[pos] = k;
                res_pos_of[k] = pos;
            }
        }
        // per-residual arrays (global, sorted)
        for (int pos = 0; pos < R; pos++) {
            const int k = H.rs_orig[pos];
            rs_tgt.push_back((uint8_t)in.res_target[k]);
            rs_flags.push_back(in.res_flags[k]);
            rs_state.push_back(in.res_state[k]);
            rs_energy.push_back(in.res_energy[k]);
            rs_point.push_back(0);
        }
        // per-point arrays
        H.pt_host.resize(P);
        for (int q = 0; q < P; q++) {
            const int p = H.pt_orig[q];
            H.pt_host[q] = in.point_host[p];
            pt_host.push_back(in.point_host[p]);
            pt_data.insert(pt_data.end(), in.point_data + (size_t)p * LDSO_BA_POINT_STRIDE,
                           in.point_data + (size_t)(p + 1) * LDSO_BA_POINT_STRIDE);
            const int b = in.point_res_begin[p], e = in.point_res_begin[p + 1];
            pt_nres.push_back(e - b);
            for (int k = 0; k < kMaxRes; k++) {
                const int pos = k < e - b ? res_pos_of[b + k] : 0;
                pt_res.push_back(k < e - b ? res_base + pos : 0);
                if (k < e - b) rs_point[res_base + pos] = point_base + q;
            }
        }
        // descriptors
        D.N = N;
        D.P = P;
        D.R = R;
        D.D = 8 * N + 4;
        D.frame_base = frame_base;
        D.pair_base = pair_base;
        D.point_base = point_base;
        D.res_base = res_base;
        D.width = in.width;
        D.height = in.height;
        D.wM3 = (float)(in.width - 3);
        D.hM3 = (float)(in.height - 3);
        for (int i = 0; i < 4; i++) D.calib[i] = in.calib[i];
        D.K = 8 * (N - 1) + 5;
        D.KP = (D.K + 3) / 4 * 4;
        const int nt = D.KP / 4;
        D.ntiles = nt * (nt + 1) / 2;
        smem_max = std::max(smem_max, sc_smem_bytes(D.KP));
        // top items: chunks of 64 residuals of one bucket
        D.top_item_base = (int)top_items.size();
        for (int b = 0; b < N * N; b++) {
            const int first = (int)top_items.size();
            for (int s = bucket_start[b]; s < bucket_start[b + 1]; s += kWave)
                top_items.push_back(make_int4(res_base + s, std::min(kWave, bucket_start[b + 1] - s), pair_base + b, w));
            pair_items.push_back(make_int2(first, (int)top_items.size() - first));
            pair_win.push_back(w);
        }
        D.n_top_items = (int)top_items.size() - D.top_item_base;
        // sc items: chunks of 64 points of one host
        D.sc_item_base = (int)sc_items.size();
        {
            int q = 0;
            for (int f = 0; f < N; f++) {
                const int first = (int)sc_items.size();
                int q0 = q;
                while (q < P && H.pt_host[q] == f) q++;
                for (int s = q0; s < q; s += kWave)
                    sc_items.push_back(make_int4(point_base + s, std::min(kWave, q - s), f, w));
                host_items.push_back(make_int2(first, (int)sc_items.size() - first));
                frame_win.push_back(w);
            }
        }
        D.n_sc_items = (int)sc_items.size() - D.sc_item_base;
        D.sc_slab_base = sc_slab_total;
        sc_slab_total += (long long)D.n_sc_items * D.ntiles * 16;
        D.g_base = g_total;
        g_total += (long long)N * D.KP * D.KP;
        D.sc_rec_base = sc_rec_total;
        sc_rec_total += (long long)N * N * sc_rec_len(N);
        D.top_rec_base = top_rec_total;
        top_rec_total += (long long)N * N * kTopRecLen;
        D.sys_base = sys_total;
        sys_total += sys_len(D.D);
        D.newest_begin = res_base + bucket_start[N * (N - 1)];
        D.newest_end = res_base + bucket_start[N * N];
        // frame-level inputs
        precalc.insert(precalc.end(), in.precalc, in.precalc + (size_t)N * N * LDSO_BA_PRECALC_STRIDE);
        adH.insert(adH.end(), in.ad_host, in.ad_host + (size_t)N * N * 64);
        adT.insert(adT.end(), in.ad_target, in.ad_target + (size_t)N * N * 64);
        frame_th.insert(frame_th.end(), in.frame_energy_th, in.frame_energy_th + N);
        frame_base += N;
        pair_base += N * N;
        point_base += P;
        res_base += R;
    }
    c->n_top_items = (int)top_items.size();
    c->n_sc_items = (int)sc_items.size();
    c->n_pairs = pair_base;
    c->n_frames = frame_base;
    c->P_tot = point_base;
    c->R_tot = res_base;
    c->sc_smem_max = smem_max;

    int rc = 0;
#define ALLOC(buf, n)                   \
    do {                                \
        rc = (buf).alloc(n);            \
        if (rc) return rc;              \
    } while (0)
    ALLOC(c->d_wins, n_windows);
    ALLOC(c->d_img, (size_t)c->n_frames * c->npix);
    ALLOC(c->d_precalc, precalc.size());
    ALLOC(c->d_frame_th, frame_th.size());
    ALLOC(c->d_pt_data, std::max<size_t>(1, pt_data.size()));
    ALLOC(c->d_pt_out, std::max<size_t>(1, (size_t)c->P_tot * 12));
    ALLOC(c->d_pt_step, std::max<size_t>(1, (size_t)c->P_tot));
    ALLOC(c->d_pt_host, std::max<size_t>(1, pt_host.size()));
    ALLOC(c->d_adH, adH.size());
    ALLOC(c->d_adT, adT.size());
    ALLOC(c->d_rs_point, std::max<size_t>(1, rs_point.size()));
    ALLOC(c->d_pt_nres, std::max<size_t>(1, pt_nres.size()));
    ALLOC(c->d_pt_res, std::max<size_t>(1, pt_res.size()));
    ALLOC(c->d_pair_win, pair_win.size());
    ALLOC(c->d_frame_win, frame_win.size());
    ALLOC(c->d_rs_tgt, std::max<size_t>(1, rs_tgt.size()));
    ALLOC(c->d_rs_flags, std::max<size_t>(1, rs_flags.size()));
    ALLOC(c->d_rs_state, std::max<size_t>(1, rs_state.size()));
    ALLOC(c->d_rs_newstate, std::max<size_t>(1, rs_state.size()));
    ALLOC(c->d_rs_energy, std::max<size_t>(1, rs_energy.size()));
    ALLOC(c->d_rs_newenergy, std::max<size_t>(1, rs_energy.size()));
    ALLOC(c->d_rs_energy_wo, std::max<size_t>(1, rs_energy.size()));
    ALLOC(c->d_rs_center, std::max<size_t>(1, rs_energy.size()));
    ALLOC(c->d_rs_rec, std::max<size_t>(1, rs_energy.size() * 4));
    ALLOC(c->d_top_items, std::max<size_t>(1, top_items.size()));
    ALLOC(c->d_sc_items, std::max<size_t>(1, sc_items.size()));
    ALLOC(c->d_pair_items, pair_items.size());
    ALLOC(c->d_host_items, host_items.size());
    ALLOC(c->d_top_slab, std::max<size_t>(1, top_items.size() * kTopVals));
    ALLOC(c->d_sc_slab, std::max<size_t>(1, (size_t)sc_slab_total));
    ALLOC(c->d_item_energy, std::max<size_t>(1, top_items.size() * 2));
    ALLOC(c->d_top_rec, (size_t)top_rec_total);
    ALLOC(c->d_sc_rec, (size_t)sc_rec_total);
    ALLOC(c->d_G, (size_t)g_total);
    ALLOC(c->d_sys, (size_t)sys_total);
    ALLOC(c->d_win_energy, (size_t)n_windows * 2);
    ALLOC(c->d_xad, (size_t)LDSO_BA_MAX_FRAMES * LDSO_BA_MAX_FRAMES * 8 + 4);
#undef ALLOC
    auto up = [&](void *dst, const void *src, size_t bytes) -> int {
        if (bytes == 0) return 0;
        HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
        return 0;
    };
#define UP(buf, vec)                                                   \
    do {                                                               \
        rc = up((buf).p, (vec).data(), (vec).size() * sizeof((vec)[0])); \
        if (rc) return rc;                                             \
    } while (0)
    UP(c->d_wins, c->wd);
    UP(c->d_precalc, precalc);
    UP(c->d_frame_th, frame_th);
    UP(c->d_pt_data, pt_data);
    UP(c->d_pt_host, pt_host);
    UP(c->d_adH, adH);
    UP(c->d_adT, adT);
    UP(c->d_rs_point, rs_point);
    UP(c->d_pt_nres, pt_nres);
    UP(c->d_pt_res, pt_res);
    UP(c->d_pair_win, pair_win);
    UP(c->d_frame_win, frame_win);
    UP(c->d_rs_tgt, rs_tgt);
    UP(c->d_rs_flags, rs_flags);
    UP(c->d_rs_state, rs_state);
    UP(c->d_rs_energy, rs_energy);
    UP(c->d_rs_newenergy, rs_energy);
    UP(c->d_top_items, top_items);
    UP(c->d_sc_items, sc_items);
    UP(c->d_pair_items, pair_items);
    UP(c->d_host_items, host_items);
#undef UP
    HIP_TRY(hipMemsetAsync(c->d_rs_center.p, 0, c->d_rs_center.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_rs_rec.p, 0, c->d_rs_rec.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_pt_out.p, 0, c->d_pt_out.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_pt_step.p, 0, c->d_pt_step.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_sys.p, 0, c->d_sys.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_G.p, 0, c->d_G.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_rs_newstate.p, LDSO_BA_RES_OUTLIER, c->d_rs_newstate.bytes(), c->stream));
    {
        std::vector<float> neg(rs_energy.size(), -1.0f);
        rc = up(c->d_rs_energy_wo.p, neg.data(), neg.size() * sizeof(float));
        if (rc) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    // images: per frame through a float3 staging buffer, repacked to float4 on the device
    {
        float *stage = nullptr;
        HIP_TRY(hipMalloc(&stage, (size_t)c->npix * 3 * sizeof(float)));
        int fb = 0;
        for (int w = 0; w < n_windows; w++)
            for (int f = 0; f < ws[w].n_frames; f++, fb++) {
                hipError_t e = hipMemcpyAsync(stage, ws[w].dI + (size_t)f * c->npix * 3, (size_t)c->npix * 3 * sizeof(float),
                                              hipMemcpyHostToDevice, c->stream);
                if (e != hipSuccess) {
                    (void)hipFree(stage);
                    return fail(-2, std::string("image upload: ") + hipGetErrorString(e));
                }
                k_repack<<<(c->npix + 255) / 256, 256, 0, c->stream>>>(stage, c->d_img.p + (size_t)fb * c->npix, c->npix);
            }
        hipError_t e = hipStreamSynchronize(c->stream);
        (void)hipFree(stage);
        if (e != hipSuccess) return fail(-2, std::string("image repack: ") + hipGetErrorString(e));
    }
    if (c->sc_smem_max > 64 * 1024) {
        HIP_TRY(hipFuncSetAttribute((const void *)k_point_sc, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)c->sc_smem_max));
    }
    return 0;
}

int ldso_ba_update(ldso_ba_ctx *c, int32_t win, const ldso_ba_window *w) {
    if (!c || !w || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    WinHost &H = c->wh[win];
    WinDev &D = c->wd[win];
    if (w->n_frames != H.N || w->n_points != H.P_all || w->n_residuals != H.R_all)
        return fail(-1, "update() cannot change the window structure; call ldso_ba_load");
    const int N = H.N;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int i = 0; i < 4; i++) D.calib[i] = w->calib[i];
    H.c_prior.assign(w->c_prior, w->c_prior + 4);
    H.c_delta.assign(w->c_delta, w->c_delta + 4);
    H.frame_prior.assign(w->frame_prior, w->frame_prior + 8 * N);
    H.frame_delta_prior.assign(w->frame_delta_prior, w->frame_delta_prior + 8 * N);
    for (size_t k = 0; k < H.adHF.size(); k++) {
        H.adHF[k] = (float)w->ad_host[k];
        H.adTF[k] = (float)w->ad_target[k];
    }
    std::vector<float> pd((size_t)H.P * LDSO_BA_POINT_STRIDE);
    for (int q = 0; q < H.P; q++)
        std::memcpy(&pd[(size_t)q * LDSO_BA_POINT_STRIDE], w->point_data + (size_t)H.pt_orig[q] * LDSO_BA_POINT_STRIDE,
                    LDSO_BA_POINT_STRIDE * sizeof(float));
    HIP_TRY(hipMemcpyAsync(c->d_wins.p + win, &D, sizeof(WinDev), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_precalc.p + (size_t)D.pair_base * LDSO_BA_PRECALC_STRIDE, w->precalc,
                           (size_t)N * N * LDSO_BA_PRECALC_STRIDE * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_adH.p + (size_t)D.pair_base * 64, w->ad_host, (size_t)N * N * 64 * sizeof(double),
                           hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_adT.p + (size_t)D.pair_base * 64, w->ad_target, (size_t)N * N * 64 * sizeof(double),
                           hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_frame_th.p + D.frame_base, w->frame_energy_th, N * sizeof(float),
                           hipMemcpyHostToDevice, c->stream));
    if (H.P)
        HIP_TRY(hipMemcpyAsync(c->d_pt_data.p + (size_t)D.point_base * LDSO_BA_POINT_STRIDE, pd.data(),
                               pd.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->sys_host_valid = false;
    return 0;
}

int ldso_ba_reset_oob(ldso_ba_ctx *c, int32_t win) {
    if (!c || win >= c->n_win) return fail(-1, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const int w0 = win < 0 ? 0 : win, w1 = win < 0 ? c->n_win : win + 1;
    for (int w = w0; w < w1; w++) {
        const WinDev &D = c->wd[w];
        if (!D.R) continue;
        // resetOOB(): state_NewEnergy = state_energy = 0; state_NewState = OUTLIER; state_state = IN
        HIP_TRY(hipMemsetAsync(c->d_rs_state.p + D.res_base, LDSO_BA_RES_IN, D.R, c->stream));
        HIP_TRY(hipMemsetAsync(c->d_rs_newstate.p + D.res_base, LDSO_BA_RES_OUTLIER, D.R, c->stream));
        HIP_TRY(hipMemsetAsync(c->d_rs_energy.p + D.res_base, 0, (size_t)D.R * sizeof(float), c->stream));
        HIP_TRY(hipMemsetAsync(c->d_rs_newenergy.p + D.res_base, 0, (size_t)D.R * sizeof(float), c->stream));
    }
    return 0;
}

int ldso_ba_linearize(ldso_ba_ctx *c, int32_t fix, int32_t accumulate) {
    if (!c || c->n_win == 0) return fail(-1, "no windows loaded");
    HIP_TRY(hipSetDevice(c->device));
    c->sys_host_valid = false;
    c->energy_valid = false;
    int rc;
    if (c->n_top_items > 0) {
        LinParams L;
        L.items = c->d_top_items.p;
        L.wins = c->d_wins.p;
        L.img = c->d_img.p;
        L.precalc = c->d_precalc.p;
        L.frame_th = c->d_frame_th.p;
        L.rs_point = c->d_rs_point.p;
        L.pt_data = c->d_pt_data.p;
        L.rs_state = c->d_rs_state.p;
        L.rs_newstate = c->d_rs_newstate.p;
        L.rs_flags = c->d_rs_flags.p;
        L.rs_energy = c->d_rs_energy.p;
        L.rs_newenergy = c->d_rs_newenergy.p;
        L.rs_energy_wo = c->d_rs_energy_wo.p;
        L.rs_center = c->d_rs_center.p;
        L.rs_rec = c->d_rs_rec.p;
        L.top_slab = c->d_top_slab.p;
        L.item_energy = c->d_item_energy.p;
        L.n_items = c->n_top_items;
        L.npix = c->npix;
        L.fix = fix;
        L.accumulate = accumulate;
        rc = timed_launch(c, 0, [&] { k_linearize<<<(c->n_top_items + 3) / 4, 256, 0, c->stream>>>(L); });
        if (rc) return rc;
    }
    rc = timed_launch(c, 1, [&] {
        k_frame_th<<<c->n_win, 256, 0, c->stream>>>(c->d_wins.p, c->d_rs_energy_wo.p, c->d_frame_th.p);
    });
    if (rc) return rc;
    if (accumulate) {
        if (c->n_sc_items > 0) {
            PointParams Pp;
            Pp.items = c->d_sc_items.p;
            Pp.wins = c->d_wins.p;
            Pp.pt_data = c->d_pt_data.p;
            Pp.pt_nres = c->d_pt_nres.p;
            Pp.pt_res = c->d_pt_res.p;
            Pp.rs_tgt = c->d_rs_tgt.p;
            Pp.rs_flags = c->d_rs_flags.p;
            Pp.rs_rec = c->d_rs_rec.p;
            Pp.pt_out = c->d_pt_out.p;
            Pp.sc_slab = c->d_sc_slab.p;
            Pp.n_items = c->n_sc_items;
            rc = timed_launch(c, 2, [&] { k_point_sc<<<c->n_sc_items, 256, c->sc_smem_max, c->stream>>>(Pp); });
            if (rc) return rc;
        }
        TopStitchParams T{c->d_wins.p, c->d_pair_win.p, c->d_pair_items.p, c->d_top_slab.p, c->d_adH.p, c->d_adT.p,
                          c->d_top_rec.p};
        rc = timed_launch(c, 3, [&] { k_stitch_top<<<c->n_pairs, 64, 0, c->stream>>>(T); });
        if (rc) return rc;
        ScReduceParams Sr{c->d_wins.p, c->d_frame_win.p, c->d_host_items.p, c->d_sc_slab.p, c->d_G.p};
        rc = timed_launch(c, 4, [&] { k_sc_reduce<<<c->n_frames, 256, 0, c->stream>>>(Sr); });
        if (rc) return rc;
        ScStitchParams Ss{c->d_wins.p, c->d_pair_win.p, c->d_G.p, c->d_adH.p, c->d_adT.p, c->d_sc_rec.p};
        rc = timed_launch(c, 5, [&] { k_stitch_sc<<<c->n_pairs, 64, 0, c->stream>>>(Ss); });
        if (rc) return rc;
    }
    FinalParams F{c->d_wins.p, c->d_top_rec.p, c->d_sc_rec.p, c->d_G.p, c->d_item_energy.p, c->d_sys.p,
                  c->d_win_energy.p, accumulate};
    rc = timed_launch(c, 6, [&] { k_final<<<c->n_win, 256, 0, c->stream>>>(F); });
    return rc;
}

int ldso_ba_sync(ldso_ba_ctx *c) {
    if (!c) return fail(-1, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    drain_events(c);
    return 0;
}

int ldso_ba_get_energy(ldso_ba_ctx *c, int32_t win, double *out) {
    if (!c || !out || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    int rc = ldso_ba_sync(c);
    if (rc) return rc;
    double e[2];
    HIP_TRY(hipMemcpy(e, c->d_win_energy.p + 2 * win, sizeof(e), hipMemcpyDeviceToHost));
    out[0] = e[0];
    out[1] = 0;
    out[2] = e[1];
    return 0;
}

static int fetch_sys(ldso_ba_ctx *c) {
    if (c->sys_host_valid) return 0;
    int rc = ldso_ba_sync(c);
    if (rc) return rc;
    c->sys_host.resize(c->d_sys.n);
    HIP_TRY(hipMemcpy(c->sys_host.data(), c->d_sys.p, c->d_sys.bytes(), hipMemcpyDeviceToHost));
    c->sys_host_valid = true;
    return 0;
}

static void expand(const double *packed, int D, double *full) {
    long long q = 0;
    for (int r = 0; r < D; r++)
        for (int col = r; col < D; col++, q++) full[(size_t)r * D + col] = full[(size_t)col * D + r] = packed[q];
}

int ldso_ba_get_system(ldso_ba_ctx *c, int32_t win, double *HA, double *bA, double *HL, double *bL, double *Hsc,
                       double *bsc) {
    if (!c || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    int rc = fetch_sys(c);
    if (rc) return rc;
    const WinDev &D = c->wd[win];
    const WinHost &H = c->wh[win];
    const int n = D.D;
    const long long pl = packed_len(n);
    const double *s = c->sys_host.data() + D.sys_base;
    if (HA) expand(s, n, HA);
    if (bA) std::memcpy(bA, s + pl, n * sizeof(double));
    if (Hsc) expand(s + pl + n, n, Hsc);
    if (bsc) std::memcpy(bsc, s + 2 * pl + n, n * sizeof(double));
    // HL / bL: accumulateLF_MT in the hot path has no linearized residuals, so it is exactly the
    // priors of stitchDoubleInternal(usePrior=true) (AccumulatedTopHessian.cc:241-250).
    if (HL) {
        std::memset(HL, 0, sizeof(double) * n * n);
        if (H.add_priors) {
            for (int i = 0; i < 4; i++) HL[(size_t)i * n + i] = H.c_prior[i];
            for (int f = 0; f < H.N; f++)
                for (int i = 0; i < 8; i++) {
                    const int q = 4 + 8 * f + i;
                    HL[(size_t)q * n + q] = H.frame_prior[8 * f + i];
                }
        }
    }
    if (bL) {
        std::memset(bL, 0, sizeof(double) * n);
        if (H.add_priors) {
            for (int i = 0; i < 4; i++) bL[i] = H.c_prior[i] * (double)H.c_delta[i];
            for (int f = 0; f < H.N; f++)
                for (int i = 0; i < 8; i++) bL[4 + 8 * f + i] = H.frame_prior[8 * f + i] * H.frame_delta_prior[8 * f + i];
        }
    }
    return 0;
}

int ldso_ba_solve(ldso_ba_ctx *c, int32_t win, int32_t iteration, double lambda, const double *ns, int32_t n_null,
                  double *x_out) {
    if (!c || !x_out || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    const int n = c->wd[win].D;
    std::vector<double> HA((size_t)n * n), bA(n), HL((size_t)n * n), bL(n), Hsc((size_t)n * n), bsc(n);
    int rc = ldso_ba_get_system(c, win, HA.data(), bA.data(), HL.data(), bL.data(), Hsc.data(), bsc.data());
    if (rc) return rc;
    return solve_system(c->wh[win].N, iteration, lambda, HA.data(), bA.data(), HL.data(), bL.data(), nullptr, nullptr,
                        Hsc.data(), bsc.data(), ns, n_null, x_out);
}

int ldso_ba_get_residuals(ldso_ba_ctx *c, int32_t win, int8_t *new_state, int8_t *state, float *state_energy,
                          float *new_energy_wo, float *center, uint8_t *flags, float *jpjdf, float *rel_bs) {
    if (!c || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    int rc = ldso_ba_sync(c);
    if (rc) return rc;
    const WinDev &D = c->wd[win];
    const WinHost &H = c->wh[win];
    const int R = D.R;
    if (R == 0) return 0;
    std::vector<int8_t> ns(R), st(R);
    std::vector<uint8_t> fl(R);
    std::vector<float> se(R), ew(R);
    std::vector<float4> ce(R), rec((size_t)R * 4);
    HIP_TRY(hipMemcpy(ns.data(), c->d_rs_newstate.p + D.res_base, R, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(st.data(), c->d_rs_state.p + D.res_base, R, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(fl.data(), c->d_rs_flags.p + D.res_base, R, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(se.data(), c->d_rs_energy.p + D.res_base, R * sizeof(float), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(ew.data(), c->d_rs_energy_wo.p + D.res_base, R * sizeof(float), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(ce.data(), c->d_rs_center.p + D.res_base, R * sizeof(float4), hipMemcpyDeviceToHost));
    if (jpjdf)
        HIP_TRY(hipMemcpy(rec.data(), c->d_rs_rec.p + (size_t)D.res_base * 4, (size_t)R * 4 * sizeof(float4),
                          hipMemcpyDeviceToHost));
    for (int pos = 0; pos < R; pos++) {
        const int k = H.rs_orig[pos];
        if (new_state) new_state[k] = ns[pos];
        if (state) state[k] = st[pos];
        if (state_energy) state_energy[k] = se[pos];
        if (new_energy_wo) new_energy_wo[k] = ew[pos];
        if (center) {
            center[3 * k] = ce[pos].x;
            center[3 * k + 1] = ce[pos].y;
            center[3 * k + 2] = ce[pos].z;
        }
        if (flags) flags[k] = fl[pos];
        if (rel_bs) rel_bs[k] = ce[pos].w;
        if (jpjdf) {
            const float4 a = rec[(size_t)pos * 4], b = rec[(size_t)pos * 4 + 1];
            const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            std::memcpy(jpjdf + 8 * (size_t)k, v, sizeof(v));
        }
    }
    return 0;
}

int ldso_ba_get_points(ldso_ba_ctx *c, int32_t win, float *HdiF, float *bdSumF, float *ih, float *Hdd, float *bd,
                       float *Hcd) {
    if (!c || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    int rc = ldso_ba_sync(c);
    if (rc) return rc;
    const WinDev &D = c->wd[win];
    const WinHost &H = c->wh[win];
    if (D.P == 0) return 0;
    std::vector<float> o((size_t)D.P * 12);
    HIP_TRY(hipMemcpy(o.data(), c->d_pt_out.p + (size_t)D.point_base * 12, o.size() * sizeof(float), hipMemcpyDeviceToHost));
    for (int q = 0; q < D.P; q++) {
        const int p = H.pt_orig[q];
        const float *v = &o[(size_t)q * 12];
        if (HdiF) HdiF[p] = v[0];
        if (bdSumF) bdSumF[p] = v[1];
        if (ih) ih[p] = v[2];
        if (Hdd) Hdd[p] = v[3];
        if (bd) bd[p] = v[4];
        if (Hcd)
            for (int i = 0; i < 4; i++) Hcd[4 * (size_t)p + i] = v[5 + i];
    }
    return 0;
}

int ldso_ba_get_frame_energy_th(ldso_ba_ctx *c, int32_t win, float *th) {
    if (!c || !th || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    int rc = ldso_ba_sync(c);
    if (rc) return rc;
    HIP_TRY(hipMemcpy(th, c->d_frame_th.p + c->wd[win].frame_base, c->wd[win].N * sizeof(float), hipMemcpyDeviceToHost));
    return 0;
}

int ldso_ba_resubstitute(ldso_ba_ctx *c, int32_t win, const double *x, double lambda, float *point_step_out) {
    if (!c || !x || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const WinDev &D = c->wd[win];
    const WinHost &H = c->wh[win];
    const int N = H.N;
    // xAd[N*h + t] = x_h^T adHostF[h + N t] + x_t^T adTargetF[h + N t] (EnergyFunctional.cc:624-632)
    std::vector<float> xF(D.D), host((size_t)N * N * 8 + 4);
    for (int i = 0; i < D.D; i++) xF[i] = (float)x[i];
    for (int h = 0; h < N; h++)
        for (int t = 0; t < N; t++) {
            const float *AH = &H.adHF[(size_t)(h + N * t) * 64], *AT = &H.adTF[(size_t)(h + N * t) * 64];
            for (int cc = 0; cc < 8; cc++) {
                float s1 = 0, s2 = 0;
                for (int k = 0; k < 8; k++) s1 += xF[4 + 8 * h + k] * AH[k * 8 + cc];
                for (int k = 0; k < 8; k++) s2 += xF[4 + 8 * t + k] * AT[k * 8 + cc];
                host[(size_t)(N * h + t) * 8 + cc] = s1 + s2;
            }
        }
    for (int i = 0; i < 4; i++) host[(size_t)N * N * 8 + i] = xF[i];
    HIP_TRY(hipMemcpyAsync(c->d_xad.p, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if (D.P > 0) {
        ResubParams R;
        R.xad = c->d_xad.p;
        R.xc = c->d_xad.p + (size_t)N * N * 8;
        R.pt_nres = c->d_pt_nres.p;
        R.pt_res = c->d_pt_res.p;
        R.rs_tgt = c->d_rs_tgt.p;
        R.rs_flags = c->d_rs_flags.p;
        R.rs_rec = c->d_rs_rec.p;
        R.pt_out = c->d_pt_out.p;
        R.pt_host = c->d_pt_host.p;
        R.pt_step = c->d_pt_step.p;
        R.begin = D.point_base;
        R.count = D.P;
        R.N = N;
        R.lambda = (float)lambda;
        int rc = timed_launch(c, 7, [&] { k_resubstitute<<<(D.P + 255) / 256, 256, 0, c->stream>>>(R); });
        if (rc) return rc;
    }
    if (point_step_out) {
        int rc = ldso_ba_sync(c);
        if (rc) return rc;
        std::vector<float> st(D.P);
        if (D.P)
            HIP_TRY(hipMemcpy(st.data(), c->d_pt_step.p + D.point_base, D.P * sizeof(float), hipMemcpyDeviceToHost));
        for (int q = 0; q < D.P; q++) point_step_out[H.pt_orig[q]] = st[q];
    }
    return 0;
}

int ldso_ba_packed_system(ldso_ba_ctx *c, void **dev_ptr, int64_t *n_doubles, int64_t *stride) {
    if (!c || !dev_ptr) return fail(-1, "bad arguments");
    *dev_ptr = c->d_sys.p;
    if (n_doubles) *n_doubles = (int64_t)c->d_sys.n;
    if (stride) *stride = c->n_win ? (int64_t)sys_len(c->wd[0].D) : 0;
    return 0;
}

int ldso_ba_unpack_system(ldso_ba_ctx *c) {
    if (!c) return fail(-1, "null ctx");
    c->sys_host_valid = false;  // get_system re-reads the (externally reduced) device buffer
    return 0;
}

int ldso_ba_set_kernel_timing(ldso_ba_ctx *c, int32_t enable) {
    if (!c) return fail(-1, "null ctx");
    int rc = ldso_ba_sync(c);
    if (rc) return rc;
    c->timing = enable != 0;
    for (int i = 0; i < kNumKernels; i++) {
        c->kms[i] = 0;
        c->kcount[i] = 0;
    }
    return 0;
}

int ldso_ba_get_kernel_times(ldso_ba_ctx *c, double *ms, int64_t *counts, int32_t n) {
    if (!c) return fail(-1, "null ctx");
    int rc = ldso_ba_sync(c);
    if (rc) return rc;
    for (int i = 0; i < n && i < kNumKernels; i++) {
        if (ms) ms[i] = c->kms[i];
        if (counts) counts[i] = c->kcount[i];
    }
    return 0;
}

const char *ldso_ba_kernel_name(int32_t i) { return (i >= 0 && i < kNumKernels) ? kKernelNames[i] : ""; }
int32_t ldso_ba_num_kernels(void) { return kNumKernels; }

int ldso_ba_stats(ldso_ba_ctx *c, int64_t *device_bytes, int64_t *n_points, int64_t *n_residuals) {
    if (!c) return fail(-1, "null ctx");
    if (device_bytes)
        *device_bytes = (int64_t)(c->d_img.bytes() + c->d_precalc.bytes() + c->d_pt_data.bytes() + c->d_rs_rec.bytes() +
                                  c->d_top_slab.bytes() + c->d_sc_slab.bytes() + c->d_G.bytes() + c->d_sys.bytes() +
                                  c->d_top_rec.bytes() + c->d_sc_rec.bytes() + c->d_pt_res.bytes());
    if (n_points) *n_points = c->P_tot;
    if (n_residuals) *n_residuals = c->R_tot;
    return 0;
}

}  // extern "C"
