// ldso_ct.hip -- MI355X (gfx950) kernels and C ABI of LDSO's coarse tracker (include/ldso_ct.h).
//
// Per new frame (FrameHessian::makeImages, FrameHessian.cc:59-115), two launches:
//   k_ct_pyr_down   block per T x T level-0 tile (T = 2^(levels-1)): the tile's intensities go to
//                   LDS once and every coarser level of that tile is averaged there
//                   (0.25f * (((a + b) + c) + d), the reference's order), so one pass over the
//                   level-0 image builds the whole intensity pyramid.
//   k_ct_pyr_grad   thread per pixel of every level: central differences on the flattened index
//                   (rows 0 and h-1 zero, x = 0 / w-1 read across the row boundary exactly as the
//                   reference's idx +- 1 does), NaN / |d| > 255 -> 0, absSquaredGrad with the optional
//                   response-gradient weight; written as one float4 texel [I, dx, dy, |g|^2].
// Per calcRes / calcGSSSE call (CoarseTracker.cc:540-741), one launch each:
//   k_ct_calc_res   thread per reference point, grid.y = pose hypothesis: warp, bounds, bilinear
//                   [I, dx, dy] of the new frame, Huber energy, saturation; per point a state byte
//                   and the two float4 of the warped record (the reference's buf_warped_* before
//                   compaction); per block the {E, nE, nSat, shiftT, shiftRT, shiftNum, nWarped}
//                   partials, summed on the host in block order.
//   k_ct_calc_gs    thread per point with state "warped": the 8 Jacobian entries + residual of
//                   calcGSSSE and the 45 weighted outer-product terms of Accumulator9, reduced over
//                   the wavefront and the block into 45 partials per block.
// Immature points (ImmaturePoint.cc:14-39, 47-317; FullSystem::traceNewCoarse):
//   k_ct_make_immature  thread per new point: 8 bilinear pattern samples of the new frame.
//   k_ct_trace          wavefront per immature point: the scalar preamble (epipolar segment,
//                       bounds, error bound) runs uniformly on all lanes; lane i evaluates
//                       discrete search step i (and i + 64), its position reproduced by the
//                       reference's sequential ptx += dx; argmin (first index of the minimum)
//                       and the second best outside +-2 steps are wave reductions; each GN
//                       iteration samples the 8 pattern taps on lanes 0-7 and every lane sums
//                       them in pattern order.  Statuses and intervals are bit-identical to the
//                       CPU restatement.
//   k_ct_ip_count       one block: the traceNewCoarse status counters.
// The per-point arithmetic is compiled with contraction off in the reference's statement order
// (states, warped records bit-identical to the CPU restatement); E and the H/b sums are
// reassociated (the reference sums them sequentially in float) and tolerance-checked.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ldso_ba.h"
#include "../../include/ldso_ct.h"
#include "ldso_ba_internal.h"

#pragma clang fp contract(off)

using ldso_ba::set_error;

namespace {

constexpr int kWave = 64;
constexpr int kCtThreads = 256;
constexpr int kResParts = 8;   // E, nE, nSat, shiftT, shiftRT, shiftNum, nWarped, pad
constexpr int kGsParts = 45;   // upper 9x9 of Accumulator9
constexpr int kMaxHyp = 256;
constexpr int kNumCtKernels = 7;
const char *kCtKernelNames[kNumCtKernels] = {"k_ct_pyr_down",      "k_ct_pyr_grad", "k_ct_calc_res", "k_ct_calc_gs",
                                             "k_ct_make_immature", "k_ct_trace",    "k_ct_ip_count"};
constexpr float kHuberTH = ldso_ba::kHuberTH;  // setting_huberTH, Setting.cc:76
constexpr float kScaleXiRot = 1.0f, kScaleXiTrans = 0.5f, kScaleA = 10.0f, kScaleB = 1000.0f;  // Settings.h:29-35

#define CT_TRY(expr)                                                                                    \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) return set_error(-2, std::string(#expr) + ": " + hipGetErrorString(e_));  \
    } while (0)

struct PyrParams {
    int w, h, levels, tile;                  // tile = 2^(levels-1) level-0 pixels
    int wl[LDSO_CT_MAX_LEVELS], hl[LDSO_CT_MAX_LEVELS];
    int off[LDSO_CT_MAX_LEVELS + 1];         // pixel offset of each level in the flat buffers
};

// ---------------------------------------------------------------------------------------------
// k_ct_pyr_down: levels 0..L-1 intensities of one T x T level-0 tile (FrameHessian.cc:73-92)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kCtThreads) void k_ct_pyr_down(const float *__restrict__ color, float *__restrict__ inten,
                                                            PyrParams P) {
    extern __shared__ float tile_lds[];  // [T*T] + [(T/2)*(T/2)]
    const int T = P.tile, tx0 = blockIdx.x * T, ty0 = blockIdx.y * T;
    float *A = tile_lds, *B = tile_lds + T * T;
    for (int i = threadIdx.x; i < T * T; i += kCtThreads) {
        const int x = tx0 + (i % T), y = ty0 + (i / T);
        const float v = color[(size_t)y * P.w + x];
        A[i] = v;
        inten[(size_t)y * P.w + x] = v;
    }
    __syncthreads();
    float *src = A, *dst = B;
    for (int l = 1; l < P.levels; l++) {
        const int Ts = T >> (l - 1), Td = T >> l;  // source / destination tile sides
        for (int i = threadIdx.x; i < Td * Td; i += kCtThreads) {
            const int x = i % Td, y = i / Td;
            const float *s = src + 2 * y * Ts + 2 * x;
            const float v = 0.25f * (s[0] + s[1] + s[Ts] + s[Ts + 1]);
            dst[i] = v;
            inten[P.off[l] + (size_t)(blockIdx.y * Td + y) * P.wl[l] + blockIdx.x * Td + x] = v;
        }
        __syncthreads();
        float *t = src;
        src = dst;
        dst = t;
    }
}

// ---------------------------------------------------------------------------------------------
// k_ct_pyr_grad: gradients and absSquaredGrad of every level (FrameHessian.cc:94-114)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kCtThreads) void k_ct_pyr_grad(const float *__restrict__ inten, float4 *__restrict__ dIp,
                                                            const float *__restrict__ Bresp, PyrParams P) {
    const int g = blockIdx.x * kCtThreads + threadIdx.x;
    if (g >= P.off[P.levels]) return;
    int l = 0;
    while (g >= P.off[l + 1]) l++;
    const int wl = P.wl[l], hl = P.hl[l], idx = g - P.off[l];
    const float *I = inten + P.off[l];
    const float c = I[idx];
    float dx = 0, dy = 0, a = 0;
    if (idx >= wl && idx < wl * (hl - 1)) {
        dx = 0.5f * (I[idx + 1] - I[idx - 1]);
        dy = 0.5f * (I[idx + wl] - I[idx - wl]);
        if (isnan(dx) || fabsf(dx) > 255.0f) dx = 0;
        if (isnan(dy) || fabsf(dy) > 255.0f) dy = 0;
        a = dx * dx + dy * dy;
        if (Bresp) {  // CalibHessian::getBGradOnly (CalibHessian.h:102-111)
            int ci = c + 0.5f;
            if (ci < 5) ci = 5;
            if (ci > 250) ci = 250;
            const float gw = Bresp[ci + 1] - Bresp[ci];
            a *= gw * gw;
        }
    }
    dIp[g] = make_float4(c, dx, dy, a);
}

// ---------------------------------------------------------------------------------------------
// k_ct_calc_res
// ---------------------------------------------------------------------------------------------
struct CtPose {  // per hypothesis, computed on the host in the reference's float arithmetic
    float RKi[9], t[3], aLL, bLL, pad[2];
};
struct CtResParams {
    const float4 *__restrict__ pc;    // (u, v, idepth, color) of this level's points
    const float4 *__restrict__ img;   // this level of the new frame
    const CtPose *__restrict__ poses;
    uint8_t *state;                   // 0 skipped, 1 saturated, 2 warped (write_warp only)
    float4 *warp;                     // [n][2]: {idepth, u, v, dx}, {dy, residual, weight, refColor}
    double *parts;                    // [hyp][blocks][kResParts]
    int n, wl, hl, lvl, write_warp, n_blocks;
    float fxl, fyl, cxl, cyl, cutoffTH, maxEnergy;
    float Ki[9];
    // k_ct_calc_res<true> (ldso_ct_calc_res_gs): one pose passed by value, and calcGSSSE's 45
    // Accumulator9 terms of every warped point summed in the same pass
    CtPose pose0;
    float gs_a, gs_b0;
    double *gs_parts;  // [blocks][kGsParts]
};

template <int K>
__device__ __forceinline__ void block_sum_write(double (&v)[K], double *dst) {
    __shared__ double red[kCtThreads / kWave][K];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
#pragma unroll
    for (int k = 0; k < K; k++) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v[k] += __shfl_xor(v[k], m, kWave);
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; k++) red[wv][k] = v[k];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < K; k += kCtThreads) dst[k] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
}

// calcGSSSE's Jacobian row of one warped point (CoarseTracker.cc:696-722) from the values the
// warped buffers hold: id, u, v, dx = dI.y fxl, dy = dI.z fyl, refColor, residual
__device__ __forceinline__ void ct_gs_terms(float id, float u, float v, float dx, float dy, float a, float b0,
                                            float refColor, float residual, float w, double *acc) {
    float J[9];
    J[0] = id * dx;
    J[1] = id * dy;
    J[2] = 0 - id * (u * dx + v * dy);
    J[3] = 0 - ((u * v) * dx + dy * (1 + v * v));
    J[4] = (u * v) * dy + dx * (1 + u * u);
    J[5] = u * dy - v * dx;
    J[6] = a * (b0 - refColor);
    J[7] = -1;
    J[8] = residual;
    int k = 0;
#pragma unroll
    for (int r = 0; r < 9; r++) {
        const float Jw = J[r] * w;
#pragma unroll
        for (int c = r; c < 9; c++) acc[k++] = (double)(Jw * J[c]);
    }
}

template <bool kGS>
__global__ __launch_bounds__(kCtThreads) void k_ct_calc_res(CtResParams P) {
    const CtPose &T = kGS ? P.pose0 : P.poses[blockIdx.y];
    double gs[kGS ? kGsParts : 1];
#pragma unroll
    for (int k = 0; k < (kGS ? kGsParts : 1); k++) gs[k] = 0;
    const int i = blockIdx.x * kCtThreads + threadIdx.x;
    double acc[kResParts] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (i < P.n) {
        const float4 q = P.pc[i];
        const float x = q.x, y = q.y, id = q.z;
        const float *RKi = T.RKi, *t = T.t;
        float pt[3];
#pragma unroll
        for (int k = 0; k < 3; k++) pt[k] = (RKi[3 * k] * x + RKi[3 * k + 1] * y + RKi[3 * k + 2] * 1) + t[k] * id;
        const float u = pt[0] / pt[2], v = pt[1] / pt[2];
        const float Ku = P.fxl * u + P.cxl, Kv = P.fyl * v + P.cyl;
        const float new_idepth = id / pt[2];
        if (P.lvl == 0 && i % 32 == 0) {  // CoarseTracker.cc:583-619
            float ptT[3], ptT2[3], pt3[3];
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const float kx = P.Ki[3 * k] * x + P.Ki[3 * k + 1] * y + P.Ki[3 * k + 2] * 1;
                ptT[k] = kx + t[k] * id;
                ptT2[k] = kx - t[k] * id;
                pt3[k] = (RKi[3 * k] * x + RKi[3 * k + 1] * y + RKi[3 * k + 2] * 1) - t[k] * id;
            }
            const float uT = ptT[0] / ptT[2], vT = ptT[1] / ptT[2];
            const float KuT = P.fxl * uT + P.cxl, KvT = P.fyl * vT + P.cyl;
            const float uT2 = ptT2[0] / ptT2[2], vT2 = ptT2[1] / ptT2[2];
            const float KuT2 = P.fxl * uT2 + P.cxl, KvT2 = P.fyl * vT2 + P.cyl;
            const float u3 = pt3[0] / pt3[2], v3 = pt3[1] / pt3[2];
            const float Ku3 = P.fxl * u3 + P.cxl, Kv3 = P.fyl * v3 + P.cyl;
            float sT = (KuT - x) * (KuT - x) + (KvT - y) * (KvT - y);
            const float sT2 = (KuT2 - x) * (KuT2 - x) + (KvT2 - y) * (KvT2 - y);
            float sRT = (Ku - x) * (Ku - x) + (Kv - y) * (Kv - y);
            const float sRT2 = (Ku3 - x) * (Ku3 - x) + (Kv3 - y) * (Kv3 - y);
            acc[3] = (double)sT + (double)sT2;
            acc[4] = (double)sRT + (double)sRT2;
            acc[5] = 2;
        }
        uint8_t st = 0;
        if (Ku > 2 && Kv > 2 && Ku < P.wl - 3 && Kv < P.hl - 3 && new_idepth > 0) {
            const float refColor = q.w;
            // getInterpolatedElement33 (GlobalFuncs.h:89-103)
            const int ix = (int)Ku, iy = (int)Kv;
            const float dx = Ku - ix, dy = Kv - iy, dxdy = dx * dy;
            const float4 *bp = P.img + ix + (size_t)iy * P.wl;
            const float4 t11 = bp[1 + P.wl], t01 = bp[P.wl], t10 = bp[1], t00 = bp[0];
            const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
            const float h0 = w11 * t11.x + w01 * t01.x + w10 * t10.x + w00 * t00.x;
            const float h1 = w11 * t11.y + w01 * t01.y + w10 * t10.y + w00 * t00.y;
            const float h2 = w11 * t11.z + w01 * t01.z + w10 * t10.z + w00 * t00.z;
            if (isfinite(h0)) {
                const float residual = h0 - (float)(T.aLL * refColor + T.bLL);
                const float hw = fabsf(residual) < kHuberTH ? 1 : kHuberTH / fabsf(residual);
                acc[1] = 1;
                if (fabsf(residual) > P.cutoffTH) {
                    acc[0] = P.maxEnergy;
                    acc[2] = 1;
                    st = 1;
                } else {
                    acc[0] = hw * residual * residual * (2 - hw);
                    acc[6] = 1;
                    st = 2;
                    if (P.write_warp) {
                        P.warp[2 * (size_t)i] = make_float4(new_idepth, u, v, h1);
                        P.warp[2 * (size_t)i + 1] = make_float4(h2, residual, hw, refColor);
                    }
                    if constexpr (kGS)
                        ct_gs_terms(new_idepth, u, v, h1 * P.fxl, h2 * P.fyl, P.gs_a, P.gs_b0, refColor, residual, hw, gs);
                }
            }
        }
        if (P.write_warp) P.state[i] = st;
    }
    block_sum_write<kResParts>(acc, P.parts + ((size_t)blockIdx.y * P.n_blocks + blockIdx.x) * kResParts);
    if constexpr (kGS) {
        __syncthreads();  // block_sum_write's LDS is reused
        block_sum_write<kGsParts>(gs, P.gs_parts + (size_t)blockIdx.x * kGsParts);
    }
}

// ---------------------------------------------------------------------------------------------
// k_ct_calc_gs: calcGSSSE's Jacobian (CoarseTracker.cc:696-722) and Accumulator9's weighted
// outer products (MatrixAccumulators.h:1250-1368), upper 9x9 = 45 terms
// ---------------------------------------------------------------------------------------------
struct CtGsParams {
    const uint8_t *__restrict__ state;
    const float4 *__restrict__ warp;
    double *parts;  // [blocks][kGsParts]
    int n;
    float fxl, fyl, a, b0;
};

__global__ __launch_bounds__(kCtThreads) void k_ct_calc_gs(CtGsParams P) {
    const int i = blockIdx.x * kCtThreads + threadIdx.x;
    double acc[kGsParts];
#pragma unroll
    for (int k = 0; k < kGsParts; k++) acc[k] = 0;
    if (i < P.n && P.state[i] == 2) {
        const float4 q0 = P.warp[2 * (size_t)i], q1 = P.warp[2 * (size_t)i + 1];
        ct_gs_terms(q0.x, q0.y, q0.z, q0.w * P.fxl, q1.x * P.fyl, P.a, P.b0, q1.w, q1.y, q1.z, acc);
    }
    block_sum_write<kGsParts>(acc, P.parts + (size_t)blockIdx.x * kGsParts);
}

// ---------------------------------------------------------------------------------------------
// immature points: ImmaturePoint::ImmaturePoint and ::traceOn (ImmaturePoint.cc:14-39, 47-317)
// ---------------------------------------------------------------------------------------------
constexpr int kPatX[8] = {0, -1, 1, -2, 0, 2, -1, 0}, kPatY[8] = {-2, -1, -1, 0, 0, 0, 1, 2};  // Setting.cc:275
constexpr float kOutlierTHSumComponent = ldso_ba::kOutlierTHSumComponent;  // Setting.cc:41
constexpr float kOutlierTH = 12 * 12;                    // Setting.cc:39
constexpr float kOverallEnergyTHWeight = ldso_ba::kOverallEnergyTHWeight;
constexpr float kMaxPixSearch = 0.027f;                  // Setting.cc:28
constexpr int kMinTraceTestRadius = 2;                   // Setting.cc:52
constexpr float kTraceStepsize = 1.0f;                   // Setting.cc:89
constexpr int kTraceGNIterations = 3;                    // Setting.cc:90
constexpr float kTraceGNThreshold = 0.1f;                // Setting.cc:91
constexpr float kTraceExtraSlackOnTH = 1.2f;             // Setting.cc:92
constexpr float kTraceSlackInterval = 1.5f;              // Setting.cc:93
constexpr float kTraceMinImprovementFactor = 2;          // Setting.cc:94
constexpr int kHostStride = 16;                          // KRKi[9], Kt[3], aff[2], pad[2]

// top-left texel of a bilinear tap, clamped into [0, w-2] x [0, h-2] (the reference would read
// past the image there; the oracle clamps the same way)
__device__ __forceinline__ int ip_base(float x, float y, int w, int h, float &fx, float &fy) {
    const int ix = (int)x, iy = (int)y;
    fx = x - ix;
    fy = y - iy;
    return min(max(ix, 0), w - 2) + min(max(iy, 0), h - 2) * w;
}

struct IpRec {  // ldso_ct_immature viewed as 32 words
    float u, v, idepth_min, idepth_max, quality, energy_th, color[8], weights[8], grad_h[4];
    int host, last_status;
    float last_uv[2], last_interval, type;
};
static_assert(sizeof(IpRec) == sizeof(ldso_ct_immature), "record layout");

// new ImmaturePoint(newFrame, feat, type, HCalib): getInterpolatedElement33BiLin (GlobalFuncs.h:186-207)
__global__ __launch_bounds__(kCtThreads) void k_ct_make_immature(const float4 *__restrict__ dI, int w, int h, int n,
                                                                 const float2 *__restrict__ uv, float type, int host,
                                                                 IpRec *__restrict__ out) {
    const int k = blockIdx.x * kCtThreads + threadIdx.x;
    if (k >= n) return;
    IpRec p;
    p.u = uv[k].x;
    p.v = uv[k].y;
    p.idepth_min = 0;
    p.idepth_max = __builtin_nanf("");
    p.quality = 10000;
    p.type = type;
    p.host = host;
    p.last_status = LDSO_CT_IPS_UNINITIALIZED;
    p.last_uv[0] = p.last_uv[1] = 0;
    p.last_interval = 0;
    float G0 = 0, G1 = 0, G2 = 0, G3 = 0;
    bool ok = true;
#pragma unroll
    for (int idx = 0; idx < 8; idx++) p.color[idx] = p.weights[idx] = 0;
#pragma unroll
    for (int idx = 0; idx < 8; idx++) {
        if (!ok) break;
        float dx, dy;
        const int b = ip_base(p.u + kPatX[idx], p.v + kPatY[idx], w, h, dx, dy);
        const float tl = dI[b].x, tr = dI[b + 1].x, bl = dI[b + w].x, br = dI[b + w + 1].x;
        const float topInt = dx * tr + (1 - dx) * tl;
        const float botInt = dx * br + (1 - dx) * bl;
        const float leftInt = dy * bl + (1 - dy) * tl;
        const float rightInt = dy * br + (1 - dy) * tr;
        const float c0 = dx * rightInt + (1 - dx) * leftInt, g0 = rightInt - leftInt, g1 = botInt - topInt;
        p.color[idx] = c0;
        if (!isfinite(c0)) {
            ok = false;
            break;
        }
        G0 += g0 * g0;
        G1 += g0 * g1;
        G2 += g1 * g0;
        G3 += g1 * g1;
        p.weights[idx] = sqrtf(kOutlierTHSumComponent / (kOutlierTHSumComponent + (g0 * g0 + g1 * g1)));
    }
    p.grad_h[0] = G0;
    p.grad_h[1] = G1;
    p.grad_h[2] = G2;
    p.grad_h[3] = G3;
    float e = 8 * kOutlierTH;
    e *= kOverallEnergyTHWeight * kOverallEnergyTHWeight;
    p.energy_th = ok ? e : __builtin_nanf("");
    out[k] = p;
}

struct TraceParams {
    const float4 *__restrict__ dI;  // level 0 [I, dx, dy, |g|^2] (GN taps)
    const float *__restrict__ inten;  // level 0 intensities, = dI[].x (discrete-search taps: 4 B, not 16)
    const float *__restrict__ hosts;  // [n_hosts][kHostStride]
    IpRec *pts;
    int n, w, h;
};

__device__ __forceinline__ void ip_finish(IpRec *q, int status, float u, float v, float interval) {
    if (threadIdx.x % kWave == 0) {
        q->last_status = status;
        q->last_uv[0] = u;
        q->last_uv[1] = v;
        q->last_interval = interval;
    }
}

// getInterpolatedElement31 (GlobalFuncs.h:146-159)
__device__ __forceinline__ float interp31(const float *__restrict__ I, float x, float y, int w, int h) {
    float dx, dy;
    const int b = ip_base(x, y, w, h, dx, dy);
    const float dxdy = dx * dy;
    return dxdy * I[b + 1 + w] + (dy - dxdy) * I[b + w] + (dx - dxdy) * I[b + 1] + (1 - dx - dy + dxdy) * I[b];
}

// one wavefront per immature point; every branch before the search is wave-uniform
__global__ __launch_bounds__(kCtThreads) void k_ct_trace(TraceParams P) {
    const int lane = threadIdx.x % kWave;
    const int k = __builtin_amdgcn_readfirstlane(blockIdx.x * (kCtThreads / kWave) + threadIdx.x / kWave);
    if (k >= P.n) return;
    IpRec *q = P.pts + k;
    const int last = q->last_status;
    if (last == LDSO_CT_IPS_OOB) return;
    const int w = P.w, h = P.h;
    const float *H = P.hosts + (size_t)q->host * kHostStride;
    const float KR[9] = {H[0], H[1], H[2], H[3], H[4], H[5], H[6], H[7], H[8]};
    const float Kt[3] = {H[9], H[10], H[11]}, aff0 = H[12], aff1 = H[13];
    const float u = q->u, v = q->v, idepth_min = q->idepth_min, idepth_max = q->idepth_max;
    const float maxPixSearch = (w + h) * kMaxPixSearch;
    float pr[3], ptpMin[3];
#pragma unroll
    for (int i = 0; i < 3; i++) pr[i] = KR[3 * i] * u + KR[3 * i + 1] * v + KR[3 * i + 2] * 1.0f;
#pragma unroll
    for (int i = 0; i < 3; i++) ptpMin[i] = pr[i] + Kt[i] * idepth_min;
    const float uMin = ptpMin[0] / ptpMin[2], vMin = ptpMin[1] / ptpMin[2];
    if (!(uMin > 4 && vMin > 4 && uMin < w - 5 && vMin < h - 5)) return ip_finish(q, LDSO_CT_IPS_OOB, -1, -1, 0);
    const bool finite_max = isfinite(idepth_max);
    float dist, uMax, vMax;
    if (finite_max) {
        float ptpMax[3];
#pragma unroll
        for (int i = 0; i < 3; i++) ptpMax[i] = pr[i] + Kt[i] * idepth_max;
        uMax = ptpMax[0] / ptpMax[2];
        vMax = ptpMax[1] / ptpMax[2];
        if (!(uMax > 4 && vMax > 4 && uMax < w - 5 && vMax < h - 5)) return ip_finish(q, LDSO_CT_IPS_OOB, -1, -1, 0);
        dist = (uMin - uMax) * (uMin - uMax) + (vMin - vMax) * (vMin - vMax);
        dist = sqrtf(dist);
        if (dist < kTraceSlackInterval)
            return ip_finish(q, LDSO_CT_IPS_SKIPPED, (uMax + uMin) * 0.5f, (vMax + vMin) * 0.5f, dist);
    } else {
        dist = maxPixSearch;
        float ptpMax[3];
#pragma unroll
        for (int i = 0; i < 3; i++) ptpMax[i] = pr[i] + Kt[i] * 0.01f;
        uMax = ptpMax[0] / ptpMax[2];
        vMax = ptpMax[1] / ptpMax[2];
        const float dx = uMax - uMin, dy = vMax - vMin;
        const float d = 1.0f / sqrtf(dx * dx + dy * dy);
        uMax = uMin + dist * dx * d;
        vMax = vMin + dist * dy * d;
        if (!(uMax > 4 && vMax > 4 && uMax < w - 5 && vMax < h - 5)) return ip_finish(q, LDSO_CT_IPS_OOB, -1, -1, 0);
    }
    if (!(idepth_min < 0 || (ptpMin[2] > 0.75f && ptpMin[2] < 1.5f))) return ip_finish(q, LDSO_CT_IPS_OOB, -1, -1, 0);

    float dx = kTraceStepsize * (uMax - uMin);
    float dy = kTraceStepsize * (vMax - vMin);
    const float G0 = q->grad_h[0], G1 = q->grad_h[1], G2 = q->grad_h[2], G3 = q->grad_h[3];
    const float a = (dx * G0 + dy * G2) * dx + (dx * G1 + dy * G3) * dy;
    const float b = (dy * G0 + -dx * G2) * dy + (dy * G1 + -dx * G3) * -dx;
    float errorInPixel = 0.2f + 0.2f * (a + b) / a;
    if (errorInPixel * kTraceMinImprovementFactor > dist && finite_max)
        return ip_finish(q, LDSO_CT_IPS_BADCONDITION, (uMax + uMin) * 0.5f, (vMax + vMin) * 0.5f, dist);
    if (errorInPixel > 10) errorInPixel = 10;
    dx /= dist;
    dy /= dist;
    if (dist > maxPixSearch) dist = maxPixSearch;  // (uMax, vMax are not used past this point)
    int numSteps = 1.9999f + dist / kTraceStepsize;
    const float randShift = uMin * 1000 - floorf(uMin * 1000);
    const float ptx0 = uMin - randShift * dx, pty0 = vMin - randShift * dy;
    float rpx[8], rpy[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        rpx[i] = KR[0] * (float)kPatX[i] + KR[1] * (float)kPatY[i];
        rpy[i] = KR[3] * (float)kPatX[i] + KR[4] * (float)kPatY[i];
    }
    if (!isfinite(dx) || !isfinite(dy)) return ip_finish(q, LDSO_CT_IPS_OOB, -1, -1, 0);
    if (numSteps >= 100) numSteps = 99;
    float col[8], wts[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        col[i] = q->color[i];
        wts[i] = q->weights[i];
    }

    // ---- discrete search: lane i takes step i and step i + 64 ----
    float x0 = 0, y0 = 0, x1 = 0, y1 = 0;  // ptx, pty of the lane's steps (sequential sums)
    {
        float px = ptx0, py = pty0;
        for (int i = 0; i < numSteps; i++) {
            if (i == lane) {
                x0 = px;
                y0 = py;
            }
            if (i == lane + kWave) {
                x1 = px;
                y1 = py;
            }
            px += dx;
            py += dy;
        }
    }
    auto step_energy = [&](float ptx, float pty) {
        float energy = 0;
#pragma unroll
        for (int idx = 0; idx < 8; idx++) {
            const float hitColor = interp31(P.inten, (float)(ptx + rpx[idx]), (float)(pty + rpy[idx]), w, h);
            if (!isfinite(hitColor)) {
                energy += 1e5f;
                continue;
            }
            const float residual = hitColor - (float)(aff0 * col[idx] + aff1);
            const float hw = fabsf(residual) < kHuberTH ? 1 : kHuberTH / fabsf(residual);
            energy += hw * residual * residual * (2 - hw);
        }
        return energy;
    };
    const bool has0 = lane < numSteps, has1 = lane + kWave < numSteps;
    const float e0 = has0 ? step_energy(x0, y0) : 0.f;
    const float e1 = has1 ? step_energy(x1, y1) : 0.f;
    // first index of the minimum among energies < 1e10 (energies are >= 0 or NaN)
    auto key = [](bool has, float e, int i) -> unsigned long long {
        return (has && e < 1e10f) ? ((unsigned long long)__float_as_uint(e) << 32) | (unsigned)i : ~0ull;
    };
    unsigned long long kmin = min(key(has0, e0, lane), key(has1, e1, lane + kWave));
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) kmin = min(kmin, (unsigned long long)__shfl_xor(kmin, m, kWave));
    int bestIdx = -1;
    float bestEnergy = 1e10f, bestU = 0, bestV = 0;
    if (kmin != ~0ull) {
        bestIdx = (int)(unsigned)kmin;
        bestEnergy = __uint_as_float((unsigned)(kmin >> 32));
        const int src = bestIdx & (kWave - 1);
        const float bx0 = __shfl(x0, src, kWave), by0 = __shfl(y0, src, kWave);
        const float bx1 = __shfl(x1, src, kWave), by1 = __shfl(y1, src, kWave);
        bestU = bestIdx < kWave ? bx0 : bx1;
        bestV = bestIdx < kWave ? by0 : by1;
    }
    auto outside = [&](int i) { return i < bestIdx - kMinTraceTestRadius || i > bestIdx + kMinTraceTestRadius; };
    float sb = 1e10f;
    if (has0 && outside(lane) && e0 < sb) sb = e0;
    if (has1 && outside(lane + kWave) && e1 < sb) sb = e1;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) sb = fminf(sb, __shfl_xor(sb, m, kWave));
    const float newQuality = sb / bestEnergy;
    float quality = q->quality;
    if (newQuality < quality || numSteps > 10) quality = newQuality;

    // ---- GN refinement: taps on lanes 0-7, sums in pattern order on every lane ----
    float uBak = bestU, vBak = bestV, gnstepsize = 1, stepBack = 0;
    if (kTraceGNIterations > 0) bestEnergy = 1e5f;
    for (int it = 0; it < kTraceGNIterations; it++) {
        const int idx = lane & 7;
        float rpxi = rpx[0], rpyi = rpy[0], ci = col[0], wi = wts[0];
#pragma unroll
        for (int i = 1; i < 8; i++)
            if (idx == i) {
                rpxi = rpx[i];
                rpyi = rpy[i];
                ci = col[i];
                wi = wts[i];
            }
        float fx, fy;
        const int bb = ip_base((float)(bestU + rpxi), (float)(bestV + rpyi), w, h, fx, fy);
        const float4 t00 = P.dI[bb], t10 = P.dI[bb + 1], t01 = P.dI[bb + w], t11 = P.dI[bb + w + 1];
        const float dxdy = fx * fy;
        const float w11 = dxdy, w01 = fy - dxdy, w10 = fx - dxdy, w00 = 1 - fx - fy + dxdy;
        const float hc0 = w11 * t11.x + w01 * t01.x + w10 * t10.x + w00 * t00.x;
        const float hc1 = w11 * t11.y + w01 * t01.y + w10 * t10.y + w00 * t00.y;
        const float hc2 = w11 * t11.z + w01 * t01.z + w10 * t10.z + w00 * t00.z;
        const bool fin = isfinite(hc0);
        const float residual = hc0 - (aff0 * ci + aff1);
        const float dResdDist = dx * hc1 + dy * hc2;
        const float hw = fabsf(residual) < kHuberTH ? 1 : kHuberTH / fabsf(residual);
        const float tH = hw * dResdDist * dResdDist;
        const float tb = hw * residual * dResdDist;
        const float tE = wi * wi * hw * residual * residual * (2 - hw);
        float Hs = 1, bs = 0, energy = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const bool f = __shfl(fin ? 1 : 0, i, kWave) != 0;
            const float h_ = __shfl(tH, i, kWave), b_ = __shfl(tb, i, kWave), e_ = __shfl(tE, i, kWave);
            if (!f) {
                energy += 1e5f;
                continue;
            }
            Hs += h_;
            bs += b_;
            energy += e_;
        }
        if (energy > bestEnergy) {
            stepBack *= 0.5f;
            bestU = uBak + stepBack * dx;
            bestV = vBak + stepBack * dy;
        } else {
            float step = -gnstepsize * bs / Hs;
            if (step < -0.5f) step = -0.5f;
            else if (step > 0.5f) step = 0.5f;
            if (!isfinite(step)) step = 0;
            uBak = bestU;
            vBak = bestV;
            stepBack = step;
            bestU += step * dx;
            bestV += step * dy;
            bestEnergy = energy;
        }
        if (fabsf(stepBack) < kTraceGNThreshold) break;
    }
    if (lane == 0) q->quality = quality;

    if (!(bestEnergy < q->energy_th * kTraceExtraSlackOnTH))
        return ip_finish(q, last == LDSO_CT_IPS_OUTLIER ? LDSO_CT_IPS_OOB : LDSO_CT_IPS_OUTLIER, -1, -1, 0);
    float imin, imax;
    if (dx * dx > dy * dy) {
        imin = (pr[2] * (bestU - errorInPixel * dx) - pr[0]) / (Kt[0] - Kt[2] * (bestU - errorInPixel * dx));
        imax = (pr[2] * (bestU + errorInPixel * dx) - pr[0]) / (Kt[0] - Kt[2] * (bestU + errorInPixel * dx));
    } else {
        imin = (pr[2] * (bestV - errorInPixel * dy) - pr[1]) / (Kt[1] - Kt[2] * (bestV - errorInPixel * dy));
        imax = (pr[2] * (bestV + errorInPixel * dy) - pr[1]) / (Kt[1] - Kt[2] * (bestV + errorInPixel * dy));
    }
    if (imin > imax) {
        const float t = imin;
        imin = imax;
        imax = t;
    }
    if (lane == 0) {
        q->idepth_min = imin;
        q->idepth_max = imax;
    }
    if (!isfinite(imin) || !isfinite(imax) || (imax < 0)) return ip_finish(q, LDSO_CT_IPS_OUTLIER, -1, -1, 0);
    ip_finish(q, LDSO_CT_IPS_GOOD, bestU, bestV, 2 * errorInPixel);
}

// traceNewCoarse's counters (FullSystem.cc:1184-1190): one block
__global__ __launch_bounds__(1024) void k_ct_ip_count(const IpRec *__restrict__ pts, int n, int *__restrict__ counts) {
    __shared__ int c[8];
    if (threadIdx.x < 8) c[threadIdx.x] = 0;
    __syncthreads();
    int loc[6] = {0, 0, 0, 0, 0, 0};
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const int s = pts[k].last_status;
#pragma unroll
        for (int j = 0; j < 6; j++) loc[j] += s == j;
    }
#pragma unroll
    for (int j = 0; j < 6; j++) {
        int x = loc[j];
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, kWave);
        if (threadIdx.x % kWave == 0 && x) atomicAdd(&c[j], x);
    }
    __syncthreads();
    if (threadIdx.x < 6) counts[threadIdx.x] = c[threadIdx.x];
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
void affine_from_to(float expF, float expT, float aF, float bF, float aT, float bT, float &a, float &b) {
    if (expF == 0 || expT == 0) expT = expF = 1;  // AffLight::fromToVecExposure (AffLight.h:27-35)
    a = std::exp(aT - aF) * expT / expF;
    b = bT - a * bF;
}

}  // namespace

struct ldso_ct_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    PyrParams pyr{};
    int levels = 1;
    float fx[LDSO_CT_MAX_LEVELS], fy[LDSO_CT_MAX_LEVELS], cx[LDSO_CT_MAX_LEVELS], cy[LDSO_CT_MAX_LEVELS];
    float Ki[LDSO_CT_MAX_LEVELS][9];
    bool have_k = false, have_frame = false, have_ref = false;
    float *d_color = nullptr, *d_inten = nullptr, *d_B = nullptr;
    float4 *d_dIp = nullptr;
    float new_exposure = 0, ref_exposure = 0, ref_a = 0, ref_b = 0;
    // reference point clouds, all levels back to back
    float4 *d_pc = nullptr;
    int pc_off[LDSO_CT_MAX_LEVELS + 1] = {0};
    int pc_cap = 0;
    // warped buffers of the last single-pose calcRes
    uint8_t *d_state = nullptr;
    float4 *d_warp = nullptr;
    int warp_cap = 0, last_lvl = -1, last_warped = 0;
    // per-call staging
    CtPose *h_poses = nullptr, *d_poses = nullptr;
    double *h_parts = nullptr, *d_parts = nullptr;
    size_t parts_cap = 0;
    // immature points (resident records, per-host tables, make staging, counters)
    IpRec *d_ip = nullptr;
    int ip_n = 0, ip_cap = 0, ip_max_host = -1;
    float *d_hosts = nullptr, *h_hosts = nullptr;
    int hosts_cap = 0;
    float2 *d_uv = nullptr;
    IpRec *d_mk = nullptr;
    int mk_cap = 0;
    int *d_counts = nullptr, *h_counts = nullptr;
    // kernel timing
    bool timing = false;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
    double ms[kNumCtKernels] = {0};
    long long cnt[kNumCtKernels] = {0};
};

namespace {

template <typename F>
int ct_launch(ldso_ct_ctx *c, int slot, F &&launch) {
    hipEvent_t a = nullptr, b = nullptr;
    if (c->timing) {
        CT_TRY(hipEventCreate(&a));
        CT_TRY(hipEventCreate(&b));
        CT_TRY(hipEventRecord(a, c->stream));
    }
    launch();
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(-2, std::string("launch ") + kCtKernelNames[slot] + ": " + hipGetErrorString(e));
    if (c->timing) {
        CT_TRY(hipEventRecord(b, c->stream));
        c->pending.push_back({slot, {a, b}});
    }
    return 0;
}

// The block partials live in coherent mapped host memory: the kernels write them straight to the
// host (a few KB), so a call needs no copy launch, only the synchronisation (d_parts is the
// device address of h_parts)
int ensure_parts(ldso_ct_ctx *c, size_t n) {
    if (n <= c->parts_cap) return 0;
    if (c->h_parts) {
        CT_TRY(hipStreamSynchronize(c->stream));
        (void)hipHostFree(c->h_parts);
    }
    c->d_parts = nullptr;
    c->h_parts = nullptr;
    c->parts_cap = 0;
    CT_TRY(hipHostMalloc(&c->h_parts, n * sizeof(double), hipHostMallocCoherent | hipHostMallocMapped));
    void *d = nullptr;
    CT_TRY(hipHostGetDevicePointer(&d, c->h_parts, 0));
    c->d_parts = static_cast<double *>(d);
    c->parts_cap = n;
    return 0;
}

// the per-hypothesis constants of calcRes (CoarseTracker.cc:555-558), float as the reference
void make_pose(const ldso_ct_ctx *c, int lvl, const double *T, float aff_a, float aff_b, CtPose &p) {
    float R[9], t[3];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) R[3 * i + j] = (float)T[4 * i + j];
        t[i] = (float)T[4 * i + 3];
    }
    const float *Ki = c->Ki[lvl];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            p.RKi[3 * i + j] = R[3 * i] * Ki[j] + R[3 * i + 1] * Ki[3 + j] + R[3 * i + 2] * Ki[6 + j];
    for (int i = 0; i < 3; i++) p.t[i] = t[i];
    affine_from_to(c->ref_exposure, c->new_exposure, c->ref_a, c->ref_b, aff_a, aff_b, p.aLL, p.bLL);
    p.pad[0] = p.pad[1] = 0;
}

int check_level(const ldso_ct_ctx *c, int lvl) {
    if (!c) return set_error(-1, "null context");
    if (lvl < 0 || lvl >= c->levels) return set_error(-1, "pyramid level out of range");
    if (!c->have_k) return set_error(-1, "ldso_ct_make_k not called");
    if (!c->have_frame) return set_error(-1, "ldso_ct_set_new_frame not called");
    if (!c->have_ref) return set_error(-1, "ldso_ct_set_reference not called");
    return 0;
}

// launch calcRes for n_hyp poses already staged in h_poses (partials to d_parts[0, n_hyp*nb*8))
// gs (n_hyp == 1): the pose by value and calcGSSSE in the same kernel (k_ct_calc_res<true>), its
// partials at d_parts + n_hyp * nb * kResParts
int launch_calc_res(ldso_ct_ctx *c, int lvl, int n_hyp, float cutoffTH, bool write_warp, size_t extra_parts,
                    bool gs = false, double aff_a = 0, double aff_b = 0) {
    const int n = c->pc_off[lvl + 1] - c->pc_off[lvl];
    const int nb = std::max(1, (n + kCtThreads - 1) / kCtThreads);
    int rc = ensure_parts(c, (size_t)n_hyp * nb * kResParts + extra_parts);
    if (rc) return rc;
    if (!gs)
        CT_TRY(hipMemcpyAsync(c->d_poses, c->h_poses, (size_t)n_hyp * sizeof(CtPose), hipMemcpyHostToDevice,
                              c->stream));
    CtResParams P;
    P.pc = c->d_pc + c->pc_off[lvl];
    P.img = c->d_dIp + c->pyr.off[lvl];
    P.poses = c->d_poses;
    P.state = c->d_state;
    P.warp = c->d_warp;
    P.parts = c->d_parts;
    P.n = n;
    P.wl = c->pyr.wl[lvl];
    P.hl = c->pyr.hl[lvl];
    P.lvl = lvl;
    P.write_warp = write_warp ? 1 : 0;
    P.n_blocks = nb;
    P.fxl = c->fx[lvl];
    P.fyl = c->fy[lvl];
    P.cxl = c->cx[lvl];
    P.cyl = c->cy[lvl];
    P.cutoffTH = cutoffTH;
    P.maxEnergy = 2 * kHuberTH * cutoffTH - kHuberTH * kHuberTH;  // CoarseTracker.cc:565-566
    for (int k = 0; k < 9; k++) P.Ki[k] = c->Ki[lvl][k];
    P.pose0 = c->h_poses[0];
    P.gs_parts = c->d_parts + (size_t)n_hyp * nb * kResParts;
    P.gs_a = 0;
    P.gs_b0 = 0;
    if (gs) {
        float aLL, bLL;
        affine_from_to(c->ref_exposure, c->new_exposure, c->ref_a, c->ref_b, (float)aff_a, (float)aff_b, aLL, bLL);
        P.gs_a = (float)(double)aLL;
        P.gs_b0 = c->ref_b;
        return ct_launch(c, 2, [&] { k_ct_calc_res<true><<<dim3(nb, 1), kCtThreads, 0, c->stream>>>(P); });
    }
    return ct_launch(c, 2, [&] { k_ct_calc_res<false><<<dim3(nb, n_hyp), kCtThreads, 0, c->stream>>>(P); });
}

// the Vec6 of every hypothesis from the block partials already on the host
void finish_calc_res(ldso_ct_ctx *c, int lvl, int n_hyp, bool write_warp, double *rs_out) {
    const int n = c->pc_off[lvl + 1] - c->pc_off[lvl];
    const int nb = std::max(1, (n + kCtThreads - 1) / kCtThreads);
    for (int hI = 0; hI < n_hyp; hI++) {
        double s[kResParts] = {0};
        const double *p = c->h_parts + (size_t)hI * nb * kResParts;
        for (int b = 0; b < nb; b++)
            for (int k = 0; k < kResParts; k++) s[k] += p[(size_t)b * kResParts + k];
        // Vec6 of CoarseTracker.cc:662-670; E and the shift sums are floats in the reference
        const float E = (float)s[0], sT = (float)s[3], sRT = (float)s[4], sNum = (float)s[5];
        const int nE = (int)s[1], nSat = (int)s[2];
        double *rs = rs_out + 6 * (size_t)hI;
        rs[0] = E;
        rs[1] = nE;
        rs[2] = sT / (sNum + 0.1);
        rs[3] = 0;
        rs[4] = sRT / (sNum + 0.1);
        rs[5] = nSat / (float)nE;
        if (write_warp && hI == 0) c->last_warped = (int)s[6];
    }
}

int run_calc_res(ldso_ct_ctx *c, int lvl, int n_hyp, float cutoffTH, bool write_warp, double *rs_out) {
    int rc = launch_calc_res(c, lvl, n_hyp, cutoffTH, write_warp, 0);
    if (rc) return rc;
    const int n = c->pc_off[lvl + 1] - c->pc_off[lvl];
    const int nb = std::max(1, (n + kCtThreads - 1) / kCtThreads);
    (void)nb;
    CT_TRY(hipStreamSynchronize(c->stream));  // the partials are in h_parts already
    finish_calc_res(c, lvl, n_hyp, write_warp, rs_out);
    return 0;
}

// calcGSSSE launch over the warped buffers, partials at d_parts + off
int launch_calc_gs(ldso_ct_ctx *c, int lvl, double aff_a, double aff_b, size_t off) {
    const int n = c->pc_off[lvl + 1] - c->pc_off[lvl];
    const int nb = std::max(1, (n + kCtThreads - 1) / kCtThreads);
    float aLL, bLL;
    affine_from_to(c->ref_exposure, c->new_exposure, c->ref_a, c->ref_b, (float)aff_a, (float)aff_b, aLL, bLL);
    CtGsParams P;
    P.state = c->d_state;
    P.warp = c->d_warp;
    P.parts = c->d_parts + off;
    P.n = n;
    P.fxl = c->fx[lvl];
    P.fyl = c->fy[lvl];
    P.a = (float)(double)aLL;
    P.b0 = c->ref_b;
    return ct_launch(c, 3, [&] { k_ct_calc_gs<<<nb, kCtThreads, 0, c->stream>>>(P); });
}

// Accumulator9::finish + CoarseTracker.cc:725-740 from the GS block partials on the host
void finish_calc_gs(ldso_ct_ctx *c, int lvl, const double *parts, double *H_out, double *b_out) {
    const int n = c->pc_off[lvl + 1] - c->pc_off[lvl];
    const int nb = std::max(1, (n + kCtThreads - 1) / kCtThreads);
    double s[kGsParts] = {0};
    for (int b = 0; b < nb; b++)
        for (int k = 0; k < kGsParts; k++) s[k] += parts[(size_t)b * kGsParts + k];
    float H[9][9];
    int k = 0;
    for (int r = 0; r < 9; r++)
        for (int cc = r; cc < 9; cc++, k++) H[r][cc] = H[cc][r] = (float)s[k];
    const int nw = (c->last_warped + 3) / 4 * 4;  // buf_warped_n (padded to a multiple of 4)
    const double inv_n = (double)(1.0f / nw);
    const float scale[8] = {kScaleXiTrans, kScaleXiTrans, kScaleXiTrans, kScaleXiRot,
                            kScaleXiRot,   kScaleXiRot,   kScaleA,       kScaleB};
    for (int r = 0; r < 8; r++) {
        for (int cc = 0; cc < 8; cc++) H_out[8 * r + cc] = (double)H[r][cc] * inv_n * scale[cc] * scale[r];
        b_out[r] = (double)H[r][8] * inv_n * scale[r];
    }
}

}  // namespace

extern "C" {

int ldso_ct_create(int32_t device, int32_t width, int32_t height, ldso_ct_ctx **out, int32_t *n_levels_out) {
    if (!out) return set_error(-1, "null output pointer");
    *out = nullptr;
    if (width < 8 || height < 8) return set_error(-1, "image too small");
    ldso_ct_ctx *c = new ldso_ct_ctx();
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return set_error(-2, std::string("hip init: ") + hipGetErrorString(e));
    }
    // setGlobalCalib's level rule (GlobalCalib.cc:20-30)
    int wl = width, hl = height, L = 1;
    while (wl % 2 == 0 && hl % 2 == 0 && wl * hl > 5000 && L < LDSO_CT_MAX_LEVELS) {
        wl /= 2;
        hl /= 2;
        L++;
    }
    c->levels = L;
    PyrParams &P = c->pyr;
    P.w = width;
    P.h = height;
    P.levels = L;
    P.tile = 1 << (L - 1);
    int off = 0;
    for (int l = 0; l < L; l++) {
        P.wl[l] = width >> l;
        P.hl[l] = height >> l;
        P.off[l] = off;
        off += P.wl[l] * P.hl[l];
    }
    P.off[L] = off;
    e = hipMalloc(&c->d_color, (size_t)width * height * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&c->d_inten, (size_t)off * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&c->d_dIp, (size_t)off * sizeof(float4));
    if (e == hipSuccess) e = hipMalloc(&c->d_B, 256 * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&c->d_poses, kMaxHyp * sizeof(CtPose));
    if (e == hipSuccess) e = hipHostMalloc(&c->h_poses, kMaxHyp * sizeof(CtPose), hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(&c->d_counts, 8 * sizeof(int));
    if (e == hipSuccess) e = hipHostMalloc(&c->h_counts, 8 * sizeof(int), hipHostMallocDefault);
    if (e != hipSuccess) {
        ldso_ct_destroy(c);
        return set_error(-3, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    if (n_levels_out) *n_levels_out = L;
    *out = c;
    return 0;
}

void ldso_ct_destroy(ldso_ct_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto &p : c->pending) {
        (void)hipEventDestroy(p.second.first);
        (void)hipEventDestroy(p.second.second);
    }
    void *dev[] = {c->d_color, c->d_inten, c->d_B,  c->d_dIp, c->d_pc,  c->d_state,  c->d_warp,
                   c->d_poses, c->d_ip, c->d_hosts, c->d_uv, c->d_mk, c->d_counts};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    if (c->h_poses) (void)hipHostFree(c->h_poses);
    if (c->h_hosts) (void)hipHostFree(c->h_hosts);
    if (c->h_counts) (void)hipHostFree(c->h_counts);
    if (c->h_parts) (void)hipHostFree(c->h_parts);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int ldso_ct_make_k(ldso_ct_ctx *c, const float calib[4], float *k_out) {
    if (!c || !calib) return set_error(-1, "null argument");
    // CoarseTracker::makeK (CoarseTracker.cc:312-339): fx/cx of level l from level 0 in double
    c->fx[0] = calib[0];
    c->fy[0] = calib[1];
    c->cx[0] = calib[2];
    c->cy[0] = calib[3];
    for (int l = 1; l < c->levels; l++) {
        c->fx[l] = c->fx[l - 1] * 0.5;
        c->fy[l] = c->fy[l - 1] * 0.5;
        c->cx[l] = (c->cx[0] + 0.5) / ((int)1 << l) - 0.5;
        c->cy[l] = (c->cy[0] + 0.5) / ((int)1 << l) - 0.5;
    }
    for (int l = 0; l < c->levels; l++) {
        // Eigen's cofactor inverse of K (Eigen/src/LU/InverseImpl.h), as FrameFramePrecalc's
        const float fx = c->fx[l], fy = c->fy[l], cx = c->cx[l], cy = c->cy[l];
        const float invdet = 1.0f / (fy * fx);
        float *Ki = c->Ki[l];
        Ki[0] = fy * invdet;
        Ki[1] = 0 * invdet;
        Ki[2] = (0 * cy - cx * fy) * invdet;
        Ki[3] = 0 * invdet;
        Ki[4] = fx * invdet;
        Ki[5] = (cx * 0 - fx * cy) * invdet;
        Ki[6] = 0 * invdet;
        Ki[7] = 0 * invdet;
        Ki[8] = (fx * fy - 0 * 0) * invdet;
        if (k_out) {
            float *o = k_out + 13 * l;
            o[0] = fx;
            o[1] = fy;
            o[2] = cx;
            o[3] = cy;
            std::memcpy(o + 4, Ki, 9 * sizeof(float));
        }
    }
    c->have_k = true;
    return 0;
}

int ldso_ct_set_new_frame(ldso_ct_ctx *c, const float *color, double ab_exposure, const float *b_response) {
    if (!c || !color) return set_error(-1, "null argument");
    CT_TRY(hipSetDevice(c->device));
    const PyrParams &P = c->pyr;
    CT_TRY(hipMemcpyAsync(c->d_color, color, (size_t)P.w * P.h * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if (b_response)
        CT_TRY(hipMemcpyAsync(c->d_B, b_response, 256 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    const float *B = b_response ? c->d_B : nullptr;
    const dim3 grid(P.w / P.tile, P.h / P.tile);
    const size_t lds = ((size_t)P.tile * P.tile + (size_t)(P.tile / 2) * (P.tile / 2) + 1) * sizeof(float);
    int rc = ct_launch(c, 0, [&] { k_ct_pyr_down<<<grid, kCtThreads, lds, c->stream>>>(c->d_color, c->d_inten, P); });
    if (rc) return rc;
    const int npx = P.off[P.levels];
    rc = ct_launch(c, 1, [&] {
        k_ct_pyr_grad<<<(npx + kCtThreads - 1) / kCtThreads, kCtThreads, 0, c->stream>>>(c->d_inten, c->d_dIp, B, P);
    });
    if (rc) return rc;
    CT_TRY(hipStreamSynchronize(c->stream));  // the caller's buffers may be reused on return
    c->new_exposure = (float)ab_exposure;
    c->have_frame = true;
    return 0;
}

int ldso_ct_get_frame_level(ldso_ct_ctx *c, int32_t lvl, float *dI, float *abs_sq_grad) {
    if (!c) return set_error(-1, "null context");
    if (lvl < 0 || lvl >= c->levels) return set_error(-1, "pyramid level out of range");
    if (!c->have_frame) return set_error(-1, "ldso_ct_set_new_frame not called");
    const int n = c->pyr.wl[lvl] * c->pyr.hl[lvl];
    std::vector<float4> tmp(n);
    CT_TRY(hipMemcpyAsync(tmp.data(), c->d_dIp + c->pyr.off[lvl], (size_t)n * sizeof(float4), hipMemcpyDeviceToHost,
                          c->stream));
    CT_TRY(hipStreamSynchronize(c->stream));
    for (int i = 0; i < n; i++) {
        if (dI) {
            dI[3 * i] = tmp[i].x;
            dI[3 * i + 1] = tmp[i].y;
            dI[3 * i + 2] = tmp[i].z;
        }
        if (abs_sq_grad) abs_sq_grad[i] = tmp[i].w;
    }
    return 0;
}

int ldso_ct_set_reference(ldso_ct_ctx *c, const int32_t *pc_n, const float *const *pc_u, const float *const *pc_v,
                          const float *const *pc_idepth, const float *const *pc_color, double ref_ab_exposure,
                          double ref_aff_a, double ref_aff_b) {
    if (!c || !pc_n || !pc_u || !pc_v || !pc_idepth || !pc_color) return set_error(-1, "null argument");
    CT_TRY(hipSetDevice(c->device));
    int off = 0, nmax = 0;
    for (int l = 0; l < c->levels; l++) {
        if (pc_n[l] < 0) return set_error(-1, "negative point count");
        if (pc_n[l] > 0 && (!pc_u[l] || !pc_v[l] || !pc_idepth[l] || !pc_color[l]))
            return set_error(-1, "null point-cloud level");
        c->pc_off[l] = off;
        off += pc_n[l];
        nmax = std::max(nmax, pc_n[l]);
    }
    c->pc_off[c->levels] = off;
    std::vector<float4> h(std::max(1, off));
    for (int l = 0; l < c->levels; l++)
        for (int i = 0; i < pc_n[l]; i++)
            h[c->pc_off[l] + i] = make_float4(pc_u[l][i], pc_v[l][i], pc_idepth[l][i], pc_color[l][i]);
    CT_TRY(hipStreamSynchronize(c->stream));
    if (off > c->pc_cap) {
        if (c->d_pc) (void)hipFree(c->d_pc);
        c->d_pc = nullptr;
        CT_TRY(hipMalloc(&c->d_pc, (size_t)off * sizeof(float4)));
        c->pc_cap = off;
    }
    if (nmax > c->warp_cap) {
        if (c->d_state) (void)hipFree(c->d_state);
        if (c->d_warp) (void)hipFree(c->d_warp);
        c->d_state = nullptr;
        c->d_warp = nullptr;
        CT_TRY(hipMalloc(&c->d_state, (size_t)nmax));
        CT_TRY(hipMalloc(&c->d_warp, (size_t)nmax * 2 * sizeof(float4)));
        c->warp_cap = nmax;
    }
    if (off)
        CT_TRY(hipMemcpyAsync(c->d_pc, h.data(), (size_t)off * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    CT_TRY(hipStreamSynchronize(c->stream));
    c->ref_exposure = (float)ref_ab_exposure;
    c->ref_a = (float)ref_aff_a;
    c->ref_b = (float)ref_aff_b;
    c->have_ref = true;
    c->last_lvl = -1;
    return 0;
}

int ldso_ct_calc_res(ldso_ct_ctx *c, int32_t lvl, const double ref_to_new[12], double aff_a, double aff_b,
                     float cutoff_th, double rs_out[6]) {
    int rc = check_level(c, lvl);
    if (rc) return rc;
    if (!ref_to_new || !rs_out) return set_error(-1, "null argument");
    CT_TRY(hipSetDevice(c->device));
    make_pose(c, lvl, ref_to_new, (float)aff_a, (float)aff_b, c->h_poses[0]);
    rc = run_calc_res(c, lvl, 1, cutoff_th, true, rs_out);
    if (rc) return rc;
    c->last_lvl = lvl;
    return 0;
}

int ldso_ct_calc_res_batch(ldso_ct_ctx *c, int32_t lvl, int32_t n_hyp, const double *ref_to_new, const double *aff_ab,
                           float cutoff_th, double *rs_out) {
    int rc = check_level(c, lvl);
    if (rc) return rc;
    if (!ref_to_new || !aff_ab || !rs_out) return set_error(-1, "null argument");
    if (n_hyp < 1 || n_hyp > kMaxHyp) return set_error(-1, "n_hyp out of range [1, 256]");
    CT_TRY(hipSetDevice(c->device));
    for (int k = 0; k < n_hyp; k++)
        make_pose(c, lvl, ref_to_new + 12 * k, (float)aff_ab[2 * k], (float)aff_ab[2 * k + 1], c->h_poses[k]);
    return run_calc_res(c, lvl, n_hyp, cutoff_th, false, rs_out);
}

int ldso_ct_calc_gs(ldso_ct_ctx *c, int32_t lvl, const double ref_to_new[12], double aff_a, double aff_b,
                    double *H_out, double *b_out) {
    int rc = check_level(c, lvl);
    if (rc) return rc;
    if (!H_out || !b_out) return set_error(-1, "null argument");
    if (c->last_lvl != lvl) return set_error(-1, "calcGSSSE needs a calcRes at this level first");
    (void)ref_to_new;  // calcGSSSE reads only the warped buffers and the affine parameters
    CT_TRY(hipSetDevice(c->device));
    const int n = c->pc_off[lvl + 1] - c->pc_off[lvl];
    const int nb = std::max(1, (n + kCtThreads - 1) / kCtThreads);
    rc = ensure_parts(c, (size_t)nb * kGsParts);
    if (rc) return rc;
    rc = launch_calc_gs(c, lvl, aff_a, aff_b, 0);
    if (rc) return rc;
    CT_TRY(hipStreamSynchronize(c->stream));  // the partials are in h_parts already
    finish_calc_gs(c, lvl, c->h_parts, H_out, b_out);
    return 0;
}

int ldso_ct_calc_res_gs(ldso_ct_ctx *c, int32_t lvl, const double ref_to_new[12], double aff_a, double aff_b,
                        float cutoff_th, double rs_out[6], double *H_out, double *b_out) {
    int rc = check_level(c, lvl);
    if (rc) return rc;
    if (!ref_to_new || !rs_out || !H_out || !b_out) return set_error(-1, "null argument");
    CT_TRY(hipSetDevice(c->device));
    const int n = c->pc_off[lvl + 1] - c->pc_off[lvl];
    const int nb = std::max(1, (n + kCtThreads - 1) / kCtThreads);
    const size_t res_parts = (size_t)nb * kResParts;
    make_pose(c, lvl, ref_to_new, (float)aff_a, (float)aff_b, c->h_poses[0]);
    // calcRes and calcGSSSE in one launch (the GS terms of each warped point from the same values
    // the warped buffers receive; the block partials are those of k_ct_calc_gs)
    rc = launch_calc_res(c, lvl, 1, cutoff_th, true, (size_t)nb * kGsParts, true, aff_a, aff_b);
    if (rc) return rc;
    CT_TRY(hipStreamSynchronize(c->stream));  // the partials are in h_parts already
    finish_calc_res(c, lvl, 1, true, rs_out);
    c->last_lvl = lvl;
    finish_calc_gs(c, lvl, c->h_parts + res_parts, H_out, b_out);
    return 0;
}

int ldso_ct_get_warped(ldso_ct_ctx *c, int32_t *n_out, float *out, int32_t capacity) {
    if (!c || !n_out) return set_error(-1, "null argument");
    if (c->last_lvl < 0) return set_error(-1, "no calcRes yet");
    const int nw = (c->last_warped + 3) / 4 * 4;
    *n_out = nw;
    if (!out) return 0;
    if (capacity < nw) return set_error(-1, "capacity below buf_warped_n");
    const int n = c->pc_off[c->last_lvl + 1] - c->pc_off[c->last_lvl];
    std::vector<uint8_t> st(std::max(1, n));
    std::vector<float4> wp(2 * (size_t)std::max(1, n));
    CT_TRY(hipSetDevice(c->device));
    if (n) {
        CT_TRY(hipMemcpyAsync(st.data(), c->d_state, (size_t)n, hipMemcpyDeviceToHost, c->stream));
        CT_TRY(hipMemcpyAsync(wp.data(), c->d_warp, (size_t)n * 2 * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    }
    CT_TRY(hipStreamSynchronize(c->stream));
    int k = 0;
    for (int i = 0; i < n; i++) {
        if (st[i] != 2) continue;
        const float4 a = wp[2 * (size_t)i], b = wp[2 * (size_t)i + 1];
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        std::memcpy(out + 8 * (size_t)k, v, sizeof v);
        k++;
    }
    for (; k < nw; k++) std::memset(out + 8 * (size_t)k, 0, 8 * sizeof(float));
    return 0;
}

int ldso_ct_make_immature(ldso_ct_ctx *c, int32_t n, const float *uv, float type, int32_t host,
                          ldso_ct_immature *out) {
    if (!c) return set_error(-1, "null context");
    if (n < 0 || (n > 0 && (!uv || !out))) return set_error(-1, "bad point arguments");
    if (!c->have_frame) return set_error(-1, "ldso_ct_set_new_frame has not been called");
    if (n == 0) return 0;
    CT_TRY(hipSetDevice(c->device));
    if (n > c->mk_cap) {
        if (c->d_uv) CT_TRY(hipFree(c->d_uv));
        if (c->d_mk) CT_TRY(hipFree(c->d_mk));
        c->d_uv = nullptr;
        c->d_mk = nullptr;
        c->mk_cap = 0;
        CT_TRY(hipMalloc(&c->d_uv, (size_t)n * sizeof(float2)));
        CT_TRY(hipMalloc(&c->d_mk, (size_t)n * sizeof(IpRec)));
        c->mk_cap = n;
    }
    CT_TRY(hipMemcpyAsync(c->d_uv, uv, (size_t)n * sizeof(float2), hipMemcpyHostToDevice, c->stream));
    const int w = c->pyr.w, h = c->pyr.h;
    int rc = ct_launch(c, 4, [&] {
        k_ct_make_immature<<<(n + kCtThreads - 1) / kCtThreads, kCtThreads, 0, c->stream>>>(
            c->d_dIp, w, h, n, c->d_uv, type, host, c->d_mk);
    });
    if (rc) return rc;
    CT_TRY(hipMemcpyAsync(out, c->d_mk, (size_t)n * sizeof(IpRec), hipMemcpyDeviceToHost, c->stream));
    CT_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int ldso_ct_immature_upload(ldso_ct_ctx *c, int32_t n, const ldso_ct_immature *pts) {
    if (!c) return set_error(-1, "null context");
    if (n < 0 || (n > 0 && !pts)) return set_error(-1, "bad point arguments");
    int max_host = -1;
    for (int k = 0; k < n; k++) {
        if (pts[k].host < 0) return set_error(-1, "immature point with a negative host index");
        if (pts[k].last_status < 0 || pts[k].last_status > LDSO_CT_IPS_UNINITIALIZED)
            return set_error(-1, "immature point with an invalid status");
        max_host = std::max(max_host, (int)pts[k].host);
    }
    CT_TRY(hipSetDevice(c->device));
    if (n > c->ip_cap) {
        if (c->d_ip) CT_TRY(hipFree(c->d_ip));
        c->d_ip = nullptr;
        c->ip_cap = 0;
        CT_TRY(hipMalloc(&c->d_ip, (size_t)n * sizeof(IpRec)));
        c->ip_cap = n;
    }
    if (n) CT_TRY(hipMemcpyAsync(c->d_ip, pts, (size_t)n * sizeof(IpRec), hipMemcpyHostToDevice, c->stream));
    CT_TRY(hipStreamSynchronize(c->stream));
    c->ip_n = n;
    c->ip_max_host = max_host;
    return 0;
}

int ldso_ct_immature_download(ldso_ct_ctx *c, int32_t n, ldso_ct_immature *pts) {
    if (!c) return set_error(-1, "null context");
    if (n != c->ip_n) return set_error(-1, "count differs from the resident immature points");
    if (n == 0) return 0;
    if (!pts) return set_error(-1, "null output");
    CT_TRY(hipSetDevice(c->device));
    CT_TRY(hipMemcpyAsync(pts, c->d_ip, (size_t)n * sizeof(IpRec), hipMemcpyDeviceToHost, c->stream));
    CT_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int ldso_ct_trace(ldso_ct_ctx *c, int32_t n_hosts, const float *krki, const float *kt, const float *aff,
                  int32_t *counts_out) {
    if (!c) return set_error(-1, "null context");
    if (!c->have_frame) return set_error(-1, "ldso_ct_set_new_frame has not been called");
    if (n_hosts <= c->ip_max_host) return set_error(-1, "an immature point's host index is >= n_hosts");
    if (n_hosts > 0 && (!krki || !kt || !aff)) return set_error(-1, "null host tables");
    CT_TRY(hipSetDevice(c->device));
    if (n_hosts > c->hosts_cap) {
        if (c->d_hosts) CT_TRY(hipFree(c->d_hosts));
        if (c->h_hosts) CT_TRY(hipHostFree(c->h_hosts));
        c->d_hosts = c->h_hosts = nullptr;
        c->hosts_cap = 0;
        CT_TRY(hipMalloc(&c->d_hosts, (size_t)n_hosts * kHostStride * sizeof(float)));
        CT_TRY(hipHostMalloc(&c->h_hosts, (size_t)n_hosts * kHostStride * sizeof(float), hipHostMallocDefault));
        c->hosts_cap = n_hosts;
    }
    CT_TRY(hipStreamSynchronize(c->stream));  // the staging buffer may still feed a previous copy
    for (int i = 0; i < n_hosts; i++) {
        float *o = c->h_hosts + (size_t)i * kHostStride;
        std::memcpy(o, krki + 9 * (size_t)i, 9 * sizeof(float));
        std::memcpy(o + 9, kt + 3 * (size_t)i, 3 * sizeof(float));
        o[12] = aff[2 * (size_t)i];
        o[13] = aff[2 * (size_t)i + 1];
        o[14] = o[15] = 0;
    }
    if (n_hosts)
        CT_TRY(hipMemcpyAsync(c->d_hosts, c->h_hosts, (size_t)n_hosts * kHostStride * sizeof(float),
                              hipMemcpyHostToDevice, c->stream));
    const int n = c->ip_n;
    if (n > 0) {
        TraceParams P{c->d_dIp, c->d_inten, c->d_hosts, c->d_ip, n, c->pyr.w, c->pyr.h};
        const int per = kCtThreads / kWave;
        int rc = ct_launch(c, 5, [&] { k_ct_trace<<<(n + per - 1) / per, kCtThreads, 0, c->stream>>>(P); });
        if (rc) return rc;
    }
    if (counts_out) {
        int rc = ct_launch(c, 6, [&] { k_ct_ip_count<<<1, 1024, 0, c->stream>>>(c->d_ip, n, c->d_counts); });
        if (rc) return rc;
        CT_TRY(hipMemcpyAsync(c->h_counts, c->d_counts, 6 * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    }
    CT_TRY(hipStreamSynchronize(c->stream));
    if (counts_out) std::memcpy(counts_out, c->h_counts, 6 * sizeof(int));
    return 0;
}

int ldso_ct_set_kernel_timing(ldso_ct_ctx *c, int32_t enable) {
    if (!c) return set_error(-1, "null context");
    c->timing = enable != 0;
    if (c->timing)
        for (int i = 0; i < kNumCtKernels; i++) {
            c->ms[i] = 0;
            c->cnt[i] = 0;
        }
    return 0;
}

int ldso_ct_get_kernel_times(ldso_ct_ctx *c, double *ms, int64_t *counts, int32_t n) {
    if (!c) return set_error(-1, "null context");
    CT_TRY(hipStreamSynchronize(c->stream));
    for (auto &p : c->pending) {
        float t = 0;
        CT_TRY(hipEventElapsedTime(&t, p.second.first, p.second.second));
        c->ms[p.first] += t;
        c->cnt[p.first]++;
        (void)hipEventDestroy(p.second.first);
        (void)hipEventDestroy(p.second.second);
    }
    c->pending.clear();
    for (int i = 0; i < std::min<int>(n, kNumCtKernels); i++) {
        if (ms) ms[i] = c->ms[i];
        if (counts) counts[i] = c->cnt[i];
    }
    return 0;
}

const char *ldso_ct_kernel_name(int32_t i) { return (i >= 0 && i < kNumCtKernels) ? kCtKernelNames[i] : nullptr; }
int32_t ldso_ct_num_kernels(void) { return kNumCtKernels; }

}  // extern "C"
