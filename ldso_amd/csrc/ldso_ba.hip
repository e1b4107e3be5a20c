// ldso_ba.hip -- MI355X (gfx950) kernels and C ABI of LDSO's photometric-BA hot path.
//
// One Gauss-Newton pass over every loaded window (ldso_ba_linearize) is four stream-ordered
// launches:
//
//   k_linearize        one wavefront per <= 64-residual chunk of one (host,target) bucket:
//                      linearize (Residuals.cc:15-217) with 8 lanes per residual (one per pattern
//                      pixel; the residual's tap footprint loaded as 16-B band columns into an LDS
//                      box, phase_a_pieces), applyRes (Residuals.h:70-88) with a lane per residual,
//                      and the chunk's AccumulatorApprox block (AccumulatedTopHessian.cc:66-99,
//                      MatrixAccumulators.h:893-1045) as 32 fp32 MFMAs into a 96-float partial.
//                      The pair precalc, frame thresholds and image base are wave-uniform.
//   k_point_sc         per point: Hdd/bd/Hcd sums (AccumulatedTopHessian.cc:94-116), HdiF
//                      (AccumulatedSCHessian.cc:24-33); then the Schur terms of a 64-point chunk of
//                      one host as one symmetric rank-64 update G += U^T diag(HdiF) U staged in LDS
//                      (the accD/accE/accEB/accHcc/accbc sums of AccumulatedSCHessian.cc:35-50).
//                      Inside ldso_ba_optimize its leading blocks also sum doStepFromBackup's sumNID.
//   k_stitch_host      block per host frame (windows of up to 12 keyframes): the host's dense
//                      partial {HA, bA, Hsc, bsc} from its Top blocks and chunk SYRK partials
//                      (AccumulatedTopHessian.cc:213-239, AccumulatedSCHessian.cc:80-114) in double;
//                      one block per window runs setNewFrameEnergyTH (FullSystem.cc:2078-2109) as a
//                      radix select and sums the linearizeAll energy.
//   k_stitch_host_sum  thread per packed output element: the window's host partials summed in host
//                      order (no atomics: the stitched system is bitwise repeatable).
// Windows of 13-16 keyframes use k_stitch + k_stitch_sum instead (one contribution record per
// (pair, block), summed in a fixed pair order).
//
// Outside the pass: the device solve (k_solve_fast; exact mode k_solve_reg / k_solve), k_step_resub
// (doStepFromBackup + setPrecalcValues + resubstituteFPt inside ldso_ba_optimize), k_resubstitute,
// k_activate (optimizeImmaturePoint), k_tile_image / k_intensity_image (image staging at load),
// k_export_newest + k_frame_th (sharded threshold exchange), k_pack_out (results to mapped memory).
//
// The per-residual arithmetic of k_linearize is compiled with contraction off and follows the
// reference's statement order, so states, energies, JpJdF and the per-point sums are
// bit-identical to the CPU restatement; the H/b sums are reassociated (tolerance-checked).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ldso_ba.h"
#include "../../include/ldso_ct.h"
#include "ldso_ba_internal.h"
#include "se3.h"

using namespace ldso_ba;

namespace {

constexpr int kWave = 64;
constexpr int kTopVals = 96;    // 55 + 30 + 6 AccumulatorApprox entries, padded to 96
constexpr int kMaxRes = LDSO_BA_MAX_FRAMES - 1;
constexpr int kNumKernels = 8;
const char *kKernelNames[kNumKernels] = {"k_linearize", "k_point_sc", "k_stitch",   "k_resubstitute",
                                         "k_frame_th",  "k_solve",    "k_activate", "k_stitch_sum"};

thread_local std::string g_err;
int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

}  // namespace

namespace ldso_ba {
int set_error(int code, const std::string &msg) { return fail(code, msg); }
}  // namespace ldso_ba

namespace {
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
    int K, KP, ntiles, p_all;  // p_all: the window's points over every shard (numID)
    long long sc_slab_base;  // floats
    long long sys_base;      // doubles: packed system
    long long stage_base;    // doubles: k_stitch contribution records, N^2 pairs x stage_rec(N)
    int newest_begin, newest_end;
    int rec_base;            // record slots: rec_base + s * P + q (s = target slot of host's point q)
    int vec_base;            // per-window (8N+4)-vectors (priors, x): vec_base + i
    int width, height;
    float wM3, hM3;
    float calib[4];
    float cdelta[4];         // EnergyFunctional::cDeltaF (marginalisation pass only)
};

// a debugging / A-B switch from the environment: set and not "0"
inline bool getenv_flag(const char *name) {
    const char *v = std::getenv(name);
    return v && *v && !(v[0] == '0' && v[1] == 0);
}
__host__ __device__ inline long long packed_len(int D) { return (long long)D * (D + 1) / 2; }
__host__ __device__ inline long long sys_len(int D) { return 2 * (packed_len(D) + D); }

// k_stitch's contribution record of one (h, t) pair (doubles): every term the reference's
// stitchDouble adds for this pair, stored instead of accumulated, so that k_stitch_sum can add
// each output element's terms in one fixed order (bitwise repeatable, no atomics).
//   Top  (AccumulatedTopHessian.cc:213-239): T1 (h,h) 8x8, T2 (t,t) 8x8, T3 AH A AT^T 8x8,
//        T4a/T4b the (calib, h) / (calib, t) 8x4 column blocks [rr * 4 + cc], T5 the 4x4
//        calibration block, T6a/T6b b(h) / b(t), T7 b(calib)
//   SC   (AccumulatedSCHessian.cc:80-114, i = h, j = t): S1 the (j, k) blocks for the N-1 k != i,
//        S2 H(j, i), S3 H(i, i), S4a/S4b (calib, i) / (calib, j) [rr * 4 + cc], S5a/S5b b(i) / b(j),
//        S6 accHcc / accbc [r * 5 + c] (only in the record of host i's first target)
enum : int { kT1 = 0, kT2 = 64, kT3 = 128, kT4a = 192, kT4b = 224, kT5 = 256, kT6a = 272, kT6b = 280, kT7 = 288,
             kS1 = 292 };
__host__ __device__ inline int stage_rec(int N) { return 520 + 64 * (N - 1); }
__host__ __device__ inline int st_S2(int N) { return kS1 + 64 * (N - 1); }

// ============================================================================================
// k_linearize
// ============================================================================================
struct LinParams {
    const int4 *__restrict__ items;  // {res_begin, count, pair_global, win}
    const WinDev *__restrict__ wins;
    const float4 *__restrict__ img;  // frames: layout 3 (band_offset) or layout 1 (tex())
    const float *__restrict__ precalc;
    const float *__restrict__ frame_th;
    const int *__restrict__ rs_slot;   // record slot (WinDev::rec_base layout)
    const float *__restrict__ pt_data;
    int8_t *rs_state;
    int8_t *rs_newstate;
    uint8_t *rs_flags;
    float *rs_energy;      // state_energy
    float *rs_newenergy;   // state_NewEnergy (persists: applyRes copies it on a later OOB)
    float *rs_energy_wo;   // state_NewEnergyWithOutlier
    float *rs_center;      // four planes of center_stride floats: centerProjectedTo x, y, z and relBS
    long long center_stride;
    float4 *rec_a;         // [slots]: (j0, j1, JpJdF[6], JpJdF[7]) -- see write_record
    float2 *rec_b;         // [slots]: (bd_r, idepth linearised at; NaN: not active)
    float *geo_snap;       // [pairs][kGeoSnap]: the pass's R0, t0 and calibration (the first chunk of a pair)
    float *top_slab;       // [items][96]
    double *item_energy;   // [items][2]
    int n_items;             // chunks of this launch: [item_base, item_base + n_items)
    int item_base;
    int n_blocks;
    long long frame_stride;  // float4 units per frame
    int tiles_per_row;       // layout 3: 8-pixel tiles per row; layout 1: 2-texel tiles per row
    int fix;
    int accumulate;
    const float *ad_ht_delta;  // [pair_global][8] EnergyFunctional::adHTdeltaF (marginalisation pass)
    const int *stop;           // ldso_ba_optimize: [win] first pass index a window skips - 1 (see opt_pass)
    int pass;                  // ldso_ba_optimize: this pass's index (0 = the initial linearizeAll)
    int aff_fix;               // bit 0: setting_affineOptModeA < 0, bit 1: ...B < 0 (JabF zeroed, Residuals.cc:186-187)
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

// Image layout 1 texel fetch: FrameHessian::dI texels [I, dx, dy, 0] (16 B) tiled 2 (x) by 4 (y)
// per 128-byte line.  Used when the caller's gradients are not makeImages' (layout 3 would then
// not reproduce them) and by k_activate on such frames.
__device__ inline float3 tex(const float4 *__restrict__ img, int tpr2, int x, int y) {
    const float4 v = img[(((y >> 2) * tpr2 + (x >> 1)) << 3) + ((y & 3) << 1) + (x & 1)];
    return make_float3(v.x, v.y, v.z);
}

// Image layout 3 (default): the intensity channel only, in bands of 4 rows stored column by
// column, i.e. byte offset (y >> 2) * band + 16 x + 4 (y & 3) with band = 16 * padded width.
// A 128-byte line is an 8 x 4 pixel tile, and the four taps of one row of a pixel's
// neighbourhood are 16 B apart, so one row offset serves all of them (immediate offsets).
__device__ __forceinline__ unsigned band_offset(int x, int y, unsigned band) {
    return ((unsigned)y >> 2) * band + ((unsigned)x << 4) + (((unsigned)y & 3u) << 2);
}
__device__ __forceinline__ float ldb(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const float *base, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), (short)0, (int)bytes, 0x00020000);
}

// makeImages' gradient rule (FrameHessian.cc:96-101): 0.5 (a - b), zeroed when NaN or |d| > 255
// (one compare: NaN fails it too)
__device__ __forceinline__ float make_grad(float a, float b) {
#pragma clang fp contract(off)
    const float d = 0.5f * (a - b);
    return fabsf(d) <= 255.0f ? d : 0.0f;
}

// The 12 intensities a bilinear [I, dx, dy] sample at (ix + dx, iy + dy) needs, layout 3:
// rows iy-1 (ix, ix+1), iy and iy+1 (ix-1 .. ix+2), iy+2 (ix, ix+1).
__device__ __forceinline__ void load12(__amdgpu_buffer_rsrc_t r, unsigned band, int ix, int iy, float *iv) {
    const unsigned o0 = band_offset(ix - 1, iy - 1, band), o1 = band_offset(ix - 1, iy, band),
                   o2 = band_offset(ix - 1, iy + 1, band), o3 = band_offset(ix - 1, iy + 2, band);
    iv[0] = ldb(r, o0 + 16);
    iv[1] = ldb(r, o0 + 32);
    iv[2] = ldb(r, o1);
    iv[3] = ldb(r, o1 + 16);
    iv[4] = ldb(r, o1 + 32);
    iv[5] = ldb(r, o1 + 48);
    iv[6] = ldb(r, o2);
    iv[7] = ldb(r, o2 + 16);
    iv[8] = ldb(r, o2 + 32);
    iv[9] = ldb(r, o2 + 48);
    iv[10] = ldb(r, o3 + 16);
    iv[11] = ldb(r, o3 + 32);
}
// getInterpolatedElement33 (GlobalFuncs.h:89-103) from those 12 values with the gradients
// recomputed; bit-identical to sampling the caller's dI when dI's gradients are makeImages'.
__device__ __forceinline__ float3 bilin12(const float *v, float dx, float dy) {
#pragma clang fp contract(off)
    const float dxdy = dx * dy;
    const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
    const float3 t00 = make_float3(v[3], make_grad(v[4], v[2]), make_grad(v[7], v[0]));
    const float3 t10 = make_float3(v[4], make_grad(v[5], v[3]), make_grad(v[8], v[1]));
    const float3 t01 = make_float3(v[7], make_grad(v[8], v[6]), make_grad(v[10], v[3]));
    const float3 t11 = make_float3(v[8], make_grad(v[9], v[7]), make_grad(v[11], v[4]));
    return make_float3(w11 * t11.x + w01 * t01.x + w10 * t10.x + w00 * t00.x,
                       w11 * t11.y + w01 * t01.y + w10 * t10.y + w00 * t00.y,
                       w11 * t11.z + w01 * t01.z + w10 * t10.z + w00 * t00.z);
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

// applyRes(true) + takeData record of one residual (Residuals.h:70-88, 120-129) at its slot
// (target-slot major, point minor: a bucket chunk writes consecutive records and a block of
// k_point_sc reads them back coalesced), 24 B in two arrays: A = (j0, j1, JpJdF[6], JpJdF[7]) with
// (j0, j1) = JIdx2 Jpdd, B = (bd_r, idepth) if active; only B = (0, NaN) otherwise (an active
// residual's idepth is never NaN: its centre projection would have failed).  Everything else of
// the residual's takeData is a function of (j0, j1) and its centre geometry -- JpJdF[0..5] =
// Jpdxi^T (j0, j1), Hdd_r = Jpdd^T (j0, j1), Hcd_r = Jpdc^T (j0, j1) (AccumulatedTopHessian.cc:
// 94-97) -- and the geometry is recomputed from the point, the pair precalc and the calibration of
// the pass (centre_projection: the same statements, so the same bits as if they had been stored):
// k_point_sc from the live precalc of the pass, the resubstitution and the JpJdF read-back from the
// geometry snapshot the pass's first chunk of each pair writes (the frame step rewrites the live
// precalc in the same launch as the resubstitution).  64 -> 48 -> 24 B written and read back.
// non-temporal stores for k_linearize's per-residual outputs: nothing reads them again while the
// pass's image lines want the L2 (the next pass, or k_point_sc after the XCD's L2 has turned over
// many times); k_linearize 93.6 -> 91.2 us, FETCH -1.7 MB (r5, profiles/r5/af)
typedef float ntf4 __attribute__((ext_vector_type(4)));
typedef float ntf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_nt(float4 *p, float4 v) { __builtin_nontemporal_store(ntf4{v.x, v.y, v.z, v.w}, reinterpret_cast<ntf4 *>(p)); }
__device__ __forceinline__ void st_nt(float2 *p, float2 v) { __builtin_nontemporal_store(ntf2{v.x, v.y}, reinterpret_cast<ntf2 *>(p)); }
template <typename T>
__device__ __forceinline__ void st_nt(T *p, T v) { __builtin_nontemporal_store(v, p); }
constexpr int kGeoSnap = 16;  // floats per pair: R0 [0..8], t0 [9..11], calib fxl, fyl, cxl, cyl [12..15]
__device__ __forceinline__ void write_record(float4 *rec_a, float2 *rec_b, bool active, float idz, const Geo &g,
                                             const PhotoSums &s) {
    if (active) {
        float jp[8], hc[4], hdd, bd;
        point_terms(g, s, jp, hc, hdd, bd);  // jp[0..5], hc, hdd: dead here (recomputed from the geometry)
        const float j0 = s.JIdx2_00 * g.d_d_x + s.JIdx2_10 * g.d_d_y;  // point_terms' statements
        const float j1 = s.JIdx2_10 * g.d_d_x + s.JIdx2_11 * g.d_d_y;
        st_nt(rec_a, make_float4(j0, j1, jp[6], jp[7]));
        st_nt(rec_b, make_float2(bd, idz));
    } else {
        st_nt(rec_b, make_float2(0.f, __builtin_nanf("")));
    }
}
// JpJdF[0..5] of a record from its centre geometry: point_terms' statements
__device__ __forceinline__ void record_jp6(const Geo &g, float j0, float j1, float jp[6]) {
#pragma clang fp contract(off)
#pragma unroll
    for (int i = 0; i < 6; i++) jp[i] = g.d_xi_x[i] * j0 + g.d_xi_y[i] * j1;
}
constexpr int kSums = 17;      // energy, wJI2, JIdx2 (3), JabJIdx (4), Jab2 (3), JI_r (2), Jab_r (2), rr
constexpr int kSumStride = kSums;  // floats per residual in the sums buffer (energy < 0: pattern not ok)

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a / b rounded to nearest, without v_div_scale / v_div_fmas / v_div_fixup: the compiler's IEEE
// sequence's rcp, Newton step and two fma corrections, so the same bits as a / b (8 instead of 11
// VALU) PROVIDED a and b are finite, |b| is normal and below 2^126 (so rcp(b) is normal) and the
// quotient and the intermediate products stay in the normal range.  Outside that precondition the
// result may differ from IEEE division (e.g. a denormal b makes rcp overflow to inf and the result
// NaN).  Used for the pattern-pixel projections, where a pixel is kept only when 1.1 < Ku < w - 3:
// a non-finite or out-of-range quotient fails that test whichever way it was rounded, so the one
// input that can decide differently is a subnormal (or > 2^126) homogeneous depth ptp[2] with a
// comparably tiny ptp[0] / ptp[1] -- a point on the target camera's plane at infinity, which LDSO's
// windows do not produce -- that IEEE division would place inside the image and this sequence
// marks OOB.  pixel_terms uses it only on image layout 3 (see there).
__device__ __forceinline__ float div_rn_normal(float a, float b) {
#pragma clang fp contract(off)
    float r = __builtin_amdgcn_rcpf(b);
    const float e = fmaf(-b, r, 1.0f);
    r = fmaf(e, r, r);
    float q = a * r;
    float rem = fmaf(-b, q, a);
    q = fmaf(rem, r, q);
    rem = fmaf(-b, q, a);
    return fmaf(rem, r, q);
}

// sqrt rounded to nearest for a normal, finite a >= 2^-96: the compiler's correctly rounded
// sequence (v_sqrt_f32, then the neighbours one ulp down / up tested by an fma residual) without its
// denormal scaling and its 0 / inf class fixup, which only act outside that range (outside it the
// result may differ from sqrtf; pixel_terms only takes roots of quotients in (1e-5, 1]).
__device__ __forceinline__ float sqrt_rn_normal(float a) {
    const float s = __builtin_amdgcn_sqrtf(a);
    const float sd = __int_as_float(__float_as_int(s) - 1), su = __int_as_float(__float_as_int(s) + 1);
    float r = fmaf(-sd, s, a) <= 0.0f ? sd : s;
    return fmaf(-su, s, a) > 0.0f ? su : r;
}

// one pattern pixel of Residuals.cc:128-190: the 17 addends, in the reference's expression order.
// kMarg: the JI_r / Jab_r / rr addends use res_toZeroF of fixLinearizationF (Residuals.cc:219-245,
// resF - JIdx Jp_delta - JabF delta_ab) as AccumulatedTopHessianSSE::addPoint<2> does
// (AccumulatedTopHessian.cc:44-45, 66-76); jx, jy = Jp_delta_x/y, da, db = adHTdeltaF[6], [7].
// fixA / fixB (setting_affineOptModeA / B < 0, wave-uniform): JabF[0] / JabF[1] are zeroed after the
// pattern sums (Residuals.cc:186-187), i.e. they leave JabJIdx and Jab2 alone and remove the affine
// parameter from Jab_r (AccumulatedTopHessian.cc:71-72) and from res_toZeroF (Residuals.cc:239-240).
// kIeee: plain IEEE division and sqrtf (image layout 1, whose gradients are the caller's and may be
// anything, e.g. inf, where 2500 / (2500 + inf) must give 0).  Otherwise (layout 3: the gradients are
// recomputed with makeImages' clamp, |g| <= 255, and the sample is finite wherever the sums are
// kept) the quotients lie in (0.01, 1], the square roots' arguments in (1e-5, 1] and the Huber
// quotient's |residual| below 2^126, i.e. inside div_rn_normal / sqrt_rn_normal's precondition: same bits.
template <bool kMarg, bool kIeee = false>
__device__ __forceinline__ void pixel_terms(float I, float gx, float gy, float color, float weight, float aff0,
                                            float aff1, float b0, float t[kSums], float jx, float jy, float da,
                                            float db, bool fixA, bool fixB) {
#pragma clang fp contract(off)
    const float residual = I - (float)(aff0 * color + aff1);
    const float drdA = (color - b0);
    auto div = [](float a, float b) { return kIeee ? a / b : div_rn_normal(a, b); };
    auto sqrt_ = [](float a) { return kIeee ? sqrtf(a) : sqrt_rn_normal(a); };
    float wg = sqrt_(div(kOutlierTHSumComponent, kOutlierTHSumComponent + (gx * gx + gy * gy)));
    wg = 0.5f * (wg + weight);
    float hw = fabsf(residual) < kHuberTH ? 1 : div(kHuberTH, fabsf(residual));
    t[0] = wg * wg * hw * residual * residual * (2 - hw);
    if (hw < 1) hw = sqrt_(hw);
    hw = hw * wg;
    gx *= hw;
    gy *= hw;
    const float resF = residual * hw;
    const float jab0 = fixA ? 0.0f : drdA * hw;  // JabF[0], JabF[1] as Jab_r and res_toZeroF see them
    const float jab1 = fixB ? 0.0f : hw;
    t[2] = gx * gx;
    t[4] = gy * gy;
    t[3] = gx * gy;
    t[5] = drdA * hw * gx;
    t[6] = drdA * hw * gy;
    t[7] = hw * gx;
    t[8] = hw * gy;
    t[9] = drdA * drdA * hw * hw;
    t[10] = drdA * hw * hw;
    t[11] = hw * hw;
    t[1] = hw * hw * (gx * gx + gy * gy);
    float ra = resF;
    if constexpr (kMarg) {
        ra = ra - gx * jx;
        ra = ra - gy * jy;
        ra = ra - jab0 * da;
        ra = ra - jab1 * db;
    }
    t[12] = ra * gx;
    t[13] = ra * gy;
    t[14] = ra * jab0;
    t[15] = ra * jab1;
    t[16] = ra * ra;
}

// G += U'^T U' over the upper 4x4 tiles of the (KP x KP) block of one point chunk, whose rows U' carry
// sqrt(HdiF) (k_point_sc): U'^T U' = U^T diag(HdiF) U
// (AccumulatedSCHessianSSE::addPoint's accD/accE/accEB/accHcc/accbc updates, summed by point):
// 16 products per point as 8 packed FMAs on diagonal pairs (after 2 packed weight multiplies),
// e.g. {acc00, acc11} += {ua.x, ua.y} * {ub.x, ub.y} and {acc01, acc10} += {ua.x, ua.y} *
// {ub.y, ub.x}: both operands are natural register pairs (or a swapped one), no broadcast moves.
__device__ __forceinline__ void syrk_tiles(const float *U, int pitch, int nt, int ntiles, int cnt,
                                           float *slab, int tid, int nthreads) {
    for (int tile = tid; tile < ntiles; tile += nthreads) {
        int a = 0, rem = tile;
        while (rem >= nt - a) {
            rem -= nt - a;
            a++;
        }
        const int bb = a + rem;
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 c[8];
#pragma unroll
        for (int i = 0; i < 8; i++) c[i] = f2{0.f, 0.f};
        const float *pa = U + 4 * a, *pb = U + 4 * bb;
#pragma unroll 4
        for (int p = 0; p < cnt; p++, pa += pitch, pb += pitch) {
            const float4 ua = *(const float4 *)pa;
            const float4 ub = *(const float4 *)pb;
            const f2 a01 = f2{ua.x, ua.y}, a23 = f2{ua.z, ua.w};
            const f2 b01 = {ub.x, ub.y}, b10 = {ub.y, ub.x}, b23 = {ub.z, ub.w}, b32 = {ub.w, ub.z};
            c[0] += a01 * b01;  // (0,0) (1,1)
            c[1] += a01 * b10;  // (0,1) (1,0)
            c[2] += a01 * b23;  // (0,2) (1,3)
            c[3] += a01 * b32;  // (0,3) (1,2)
            c[4] += a23 * b01;  // (2,0) (3,1)
            c[5] += a23 * b10;  // (2,1) (3,0)
            c[6] += a23 * b23;  // (2,2) (3,3)
            c[7] += a23 * b32;  // (2,3) (3,2)
        }
        float acc[16];
        acc[0] = c[0].x, acc[5] = c[0].y, acc[1] = c[1].x, acc[4] = c[1].y;
        acc[2] = c[2].x, acc[7] = c[2].y, acc[3] = c[3].x, acc[6] = c[3].y;
        acc[8] = c[4].x, acc[13] = c[4].y, acc[9] = c[5].x, acc[12] = c[5].y;
        acc[10] = c[6].x, acc[15] = c[6].y, acc[11] = c[7].x, acc[14] = c[7].y;
        float4 *o = (float4 *)(slab + (size_t)tile * 16);
        o[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        o[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
        o[2] = make_float4(acc[8], acc[9], acc[10], acc[11]);
        o[3] = make_float4(acc[12], acc[13], acc[14], acc[15]);
    }
}

// ---------------------------------------------------------------------------------------------
// AccumulatorApprox of one chunk on the matrix cores.  The chunk's Top block (13x13, index layout
// [0:4 intrinsics, 4:10 xi, 10 a, 11 b, 12 r]) is
//   [0:10, 0:10]  sum_r Jp^T JIdx2 Jp                 (update, MatrixAccumulators.h:893-979)
//   [0:10, 10:13] sum_r Jp^T [JabJIdx | JI_r]          (updateTopRight, :982-1030)
//   [10:13,10:13] sum_r [Jab2, Jab_r; ., rr]           (updateBotRight, :1032-1045)
// with Jp = [x; y] = [Jpdc | Jpdxi] (2x10).  As one GEMM over K = 2 x 64 (residual, row of Jp):
//   D = A B,  A[i][(r,c)] = Jp_r[c][i],  B[(r,0)][j] = (a x + b y)_j,  B[(r,1)][j] = (b x + c y)_j
//   for j < 10, and B[(r,c)][10 + m] = column m of [JabJIdx | JI_r] row c.
// Rows 13 / 14 of A are the indicators of c = 0 / c = 1 and columns 13..15 of B carry the six
// BotRight terms, so D[13][13..15] and D[14][13..15] are their sums.  32 v_mfma_f32_16x16x4f32
// per wavefront, operands staged through the wave's LDS (36 floats per residual, all 64 rows at
// once).  fp32 products accumulated in fp32 like the blocked AccumulatorApprox sums
// (tolerance-checked).
// ---------------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kTopRow = 36;
constexpr int kTermQ = 9;                      // quantities per transposition round (17 = 9 + 8)
// k_linearize footprint box of one residual (layout 3): 3 bands x 9 columns of
// 16-B band-column pieces (4 rows each) + one dummy slot, in floats
constexpr int kBoxCols = 9, kBoxBands = 3, kBoxFloats = 112;
static_assert(kBoxFloats >= (kBoxCols * kBoxBands + 1) * 4, "box");
// floats between the 8 residuals' term tables of a step (dense).  Bank-swizzled bases that make the
// pattern-order sums' 16-B reads conflict-free turn the terms' paired 4-B stores into 2-way
// conflicts instead (r4, PMC ablations: 8.66 vs 8.36 M conflict cycles per launch, time unchanged)
constexpr int kTermStride = 72;
constexpr int kRoundQ = kTermQ;
static_assert(kTermStride >= kRoundQ * 8, "term tables");
constexpr int kTermsOnly = 8 * kTermStride;      // per-pixel addends of one round [8 residuals][kRoundQ][8]
// the terms region also holds the 8 residuals' footprint boxes of a step (used before the terms)
constexpr int kTermsPerWave = 8 * kBoxFloats > kTermsOnly ? 8 * kBoxFloats : kTermsOnly;
constexpr int kSumsPerWave = 64 * kSumStride;   // per-residual sums [64][17]

__device__ __forceinline__ void top_mfma(float *tab, int lane, bool active, const Geo &g, const PhotoSums &s,
                                         float *slab_item) {
    // the residual's operand row; an inactive residual's row is zero (written by a separate
    // exec-masked path, so the active values need no zero-select merge in registers)
    auto stage = [&](float4 *row) {
        if (active) {
            row[0] = make_float4(g.d_C_x[0], g.d_C_y[0], g.d_C_x[1], g.d_C_y[1]);
            row[1] = make_float4(g.d_C_x[2], g.d_C_y[2], g.d_C_x[3], g.d_C_y[3]);
            row[2] = make_float4(g.d_xi_x[0], g.d_xi_y[0], g.d_xi_x[1], g.d_xi_y[1]);
            row[3] = make_float4(g.d_xi_x[2], g.d_xi_y[2], g.d_xi_x[3], g.d_xi_y[3]);
            row[4] = make_float4(g.d_xi_x[4], g.d_xi_y[4], g.d_xi_x[5], g.d_xi_y[5]);
            row[5] = make_float4(s.JabJIdx_00, s.JabJIdx_01, s.JabJIdx_10, s.JabJIdx_11);
            row[6] = make_float4(s.JI_r0, s.JI_r1, s.Jab2_00, s.Jab2_11);
            row[7] = make_float4(s.Jab2_01, s.Jab_r1, s.Jab_r0, s.rr);
            row[8] = make_float4(s.JIdx2_00, s.JIdx2_10, s.JIdx2_11, 0.f);
        } else {
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int k = 0; k < 9; k++) row[k] = z;
        }
    };
    const int i = lane & 15, kk = lane >> 4;
    const bool geo = i < 10, ind = i >= 13;
    const float a0c = i == 13 ? 1.f : 0.f, a1c = i == 14 ? 1.f : 0.f;
    // all 64 rows staged at once (one table, one barrier), two independent accumulator chains
    stage(reinterpret_cast<float4 *>(tab + lane * kTopRow));
    wave_lds_sync();
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    {
        // K rows (residual 4 (m + u) + kk, c): the four lane groups read consecutive rows, 36 floats
        // apart, not rows 16 x 36 = 0 mod 64 banks apart (LDS bank conflicts 8.78 -> 7.51 M cycles)
        const float *base = tab + kk * kTopRow;
#pragma unroll 4
        for (int m = 0; m < 16; m += 2) {
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const float *rr = base + 4 * (m + u) * kTopRow;
                const float2 p = *reinterpret_cast<const float2 *>(rr + 2 * i);
                const float4 q = *reinterpret_cast<const float4 *>(rr + 32);
                const float A0 = ind ? a0c : p.x, A1 = ind ? a1c : p.y;
                const float B0 = geo ? q.x * p.x + q.y * p.y : p.x;
                const float B1 = geo ? q.y * p.x + q.z * p.y : p.y;
                f32x4 &acc = u ? acc1 : acc0;
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A0, B0, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A1, B1, acc, 0, 0, 0);
            }
        }
    }
    wave_lds_sync();
    const f32x4 acc = acc0 + acc1;
    // lane holds D[4 kk + v][i]; scatter into the 96-slot partial layout read by k_stitch
#pragma unroll
    for (int v = 0; v < 4; v++) {
        const int r = 4 * kk + v, c = i;
        int slot = -1;
        if (r < 10 && c < 10 && c >= r) slot = r * 10 - r * (r - 1) / 2 + (c - r);
        else if (r < 10 && c >= 10 && c < 13) slot = 55 + 3 * r + (c - 10);
        else if (r == 13 && c >= 13) slot = 85 + (c - 13);
        else if (r == 14 && c >= 13) slot = 88 + (c - 13);
        if (slot >= 0) slab_item[slot] = acc[v];
        else if (r == 15 && c < 5) slab_item[91 + c] = 0.f;
    }
}

// ============================================================================================
// k_linearize: one wavefront per chunk of <= 64 residuals of one (host, target) bucket, 4 per
// workgroup, XCD-contiguous chunk ranges.
//   phase A  8 lanes per residual (lane = pattern pixel), 8 residuals per step, a one-step
//            software pipeline: the projection and the 12 intensity taps (layout 3) or 4 texels
//            (layout 1) of step k+1 are issued before step k's arithmetic.  The 17 per-pixel
//            addends of Residuals.cc:128-190 go through LDS and are summed in pattern order.
//   phase B  lane per residual: centre projection (FEJ Jacobians), state / energy
//            (Residuals.cc:192-217), applyRes + the takeData record, relBS on the fix pass.
//   Top      the chunk's AccumulatorApprox block on the matrix cores (top_mfma).
// kMarg: the marginalisation pass (addPoint<2> sums with fixLinearizationF's res_toZeroF).
// ============================================================================================
constexpr int kPtTable = 64 * 4;  // floats: [64 residuals][u, v, idepth, state]
// the Top operand table holds all 64 rows: one stage, one barrier, two independent MFMA chains
// (r5: 94.6 vs 96.5 us against two 32-row halves in one chain; fits the wave's 10 KB of LDS)
constexpr int kTopRows = 64;
constexpr int kTopTab = kTopRows * kTopRow;
constexpr int kWaveLdsA = kTermsPerWave + kSumsPerWave + kPtTable;
// floats of LDS per wavefront (the Top operand table reuses the wave's region after phase B)
constexpr int kWaveLds = kWaveLdsA > kTopTab ? kWaveLdsA : kTopTab;
// LDS requested per 4-wave workgroup: sets the resident workgroups per CU (= waves per SIMD).
// 160 KB / 32 KB = 5: measured fastest (64 x S7: 121.6 us; 4 blocks 125.7, 3 blocks 143.5; 6
// waves/SIMD need <= 80 VGPRs and spill, 145 us).
// 4 workgroups (16 waves) per CU: LDS (kLinLdsBytes) and the register budget of __launch_bounds__
// (<= 128 VGPRs; 101 used).  5 per CU measured slower (r3: 127.5 vs 117.4 us with 44 B spilled; r4:
// 123.7 vs 106.1 us, 32 B spilled, the pt table dropped for LDS)
constexpr int kLinBlocksPerCu = 4;
constexpr size_t kLinLdsBytes = (160 * 1024 / kLinBlocksPerCu) & ~(size_t)511;
static_assert(kLinLdsBytes >= 4 * kWaveLds * sizeof(float), "k_linearize LDS");

// 8-lane group reductions (lanes 8g .. 8g+7) on DPP: quad swaps, then the half-row mirror
// (lane i <-> 7 - i) joins the two quads.
// every lane active, full row / bank masks: no "old" value, so the DPP move can fold into the
// min / or (one DPP-modified VALU op per stage instead of a copy, a DPP move and the op)
#define LDSO_DPP(v, ctrl) __builtin_amdgcn_mov_dpp(v, ctrl, 0xF, 0xF, true)
__device__ __forceinline__ int grp8_min(int v) {
    v = min(v, LDSO_DPP(v, 0xB1));    // quad_perm [1,0,3,2]
    v = min(v, LDSO_DPP(v, 0x4E));    // quad_perm [2,3,0,1]
    return min(v, LDSO_DPP(v, 0x141));  // row_half_mirror
}
__device__ __forceinline__ int grp8_or(int v) {
    v |= LDSO_DPP(v, 0xB1);
    v |= LDSO_DPP(v, 0x4E);
    return v | LDSO_DPP(v, 0x141);
}
__device__ __forceinline__ float4 ldb4(__amdgpu_buffer_rsrc_t r, unsigned off) {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const i32x4 v = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
    return make_float4(__int_as_float(v.x), __int_as_float(v.y), __int_as_float(v.z), __int_as_float(v.w));
}

// Phase A of k_linearize on image layout 3 with footprint pieces.  The 8 pattern
// pixels of a residual read their 96 taps (12 each, load12's stencil) from the residual's tap
// footprint: the 16-B band columns (4 rows of one column) that hold at least one of the taps,
// i.e. exactly the 128-B lines the per-lane gathers touch.  The residual's 8 lanes load them with
// one buffer_load_dwordx4 per box band (lane = column) plus one for a 9th column, into a box of
// 3 bands x 9 columns in the wave's LDS (aliasing the terms table of the same step), and the
// pattern lanes read their taps from there: 4 wide loads per lane instead of 12 scalar ones
// (TCP accesses per launch 64.9 M -> 12.4 M on 64 x S7).  The pieces of step k+1 are in flight
// while step k reads its box and sums its terms.  A residual whose footprint does not fit the box
// (pattern spread > 5 pixels) is left out of the pipelined loop and gathered per lane in a second
// loop over the steps that hold one (a gather inside the pipelined loop would make the compiler
// wait for every load in flight, the next step's pieces included).  Taps bit-identical to load12's.
template <bool kMarg>
__device__ __forceinline__ void phase_a_pieces(int lane, float *lds_terms_w, float *S, const float *pre, int jlimit,
                                               int my_state, float4 my_pd0, float jp_dx, float jp_dy, float da,
                                               float db, __amdgpu_buffer_rsrc_t rsrc, unsigned band, float wM3,
                                               float hM3, int aff_fix) {
#pragma clang fp contract(off)
    const int g = lane >> 3, sl = lane & 7;
    const bool fixA = (aff_fix & 1) != 0, fixB = (aff_fix & 2) != 0;
    // staticPattern[8] (Setting.cc:275) offset of this lane's pixel
    const int px = sl == 1 || sl == 6 ? -1 : sl == 2 ? 1 : sl == 3 ? -2 : sl == 5 ? 2 : 0;
    const int py = sl == 0 ? -2 : sl <= 2 ? -1 : sl <= 5 ? 0 : sl == 6 ? 1 : 2;
    const float aff0 = pre[24], aff1 = pre[25], b0a = pre[26];
    float *T = lds_terms_w + g * kTermStride;
    float *box = lds_terms_w + g * kBoxFloats;
    const int nsteps = (jlimit + 7) >> 3;
    constexpr unsigned kOOB = 0x7FFFFFF0u;  // beyond the frame's buffer range: the load returns 0, no access

    struct Geo8 {
        float Ku, Kv, jx, jy;
        int cx0, b0, m;  // box origin (column, band); needed pieces, bit 9 band + column
        bool gok, wide;
    };
    // projection of the lane's pattern pixel of residual 8k + g (Residuals.cc:128-135) and the box
    auto geo = [&](int k, Geo8 &q) {
        const int j = 8 * k + g;
        const float4 pt = *reinterpret_cast<const float4 *>(S + kSumsPerWave + 4 * (j & 63));
        const float pu = pt.x, pv = pt.y, pz = pt.z;
        const int st = __float_as_int(pt.w);
        const bool go = j < jlimit && st != LDSO_BA_RES_OOB;
        if constexpr (kMarg) {
            q.jx = __shfl(jp_dx, j, kWave);
            q.jy = __shfl(jp_dy, j, kWave);
        }
        const float up = pu + px, vp = pv + py;
        float ptp[3];
#pragma unroll
        for (int i = 0; i < 3; i++) ptp[i] = (pre[3 * i] * up + pre[3 * i + 1] * vp + pre[3 * i + 2] * 1.0f) + pre[9 + i] * pz;
        q.Ku = div_rn_normal(ptp[0], ptp[2]);
        q.Kv = div_rn_normal(ptp[1], ptp[2]);
        const bool pok = go && q.Ku > 1.1f && q.Kv > 1.1f && q.Ku < wM3 && q.Kv < hM3;
        const unsigned long long m1 = __ballot(pok);
        q.gok = ((m1 >> (8 * g)) & 0xFFull) == 0xFFull;
        const int ix = pok ? (int)q.Ku : 1, iy = pok ? (int)q.Kv : 1;
        // the box: columns from min(ix) - 1, bands from that of min(iy) - 1
        const int cx0 = grp8_min(ix) - 1, b0 = (grp8_min(iy) - 1) >> 2;
        const int rx = ix - cx0;  // >= 1
        // rows iy-1 / iy+2 use columns ix, ix+1 (pattern 0110 from column ix-1), rows iy, iy+1
        // columns ix-1 .. ix+2 (1111).  The four rows lie in band bA = band(iy-1) and, from row
        // 4 - ph on (ph = (iy-1) & 3), in band bA + 1: the columns needed in band bA are 1111 unless
        // only row iy-1 is there (ph 3: 0110); in band bA + 1 none (ph 0), row iy+2 only (ph 1:
        // 0110) or 1111 (ph 2, 3)
        const int ph = (iy - 1) & 3, bA = ((iy - 1) >> 2) - b0, bD = bA + (ph != 0 ? 1 : 0);
        const int colA = ph == 3 ? 6 : 15, colB = ph == 0 ? 0 : ph == 1 ? 6 : 15;
        const bool wide_l = rx + 2 >= kBoxCols || bD >= kBoxBands;
        int m = wide_l ? 0 : (colA | (colB << kBoxCols)) << (bA * kBoxCols + rx - 1);
        m = grp8_or(m);
        const unsigned long long mw = __ballot(wide_l);
        q.wide = ((mw >> (8 * g)) & 0xFFull) != 0;
        q.m = (q.gok && !q.wide) ? m : 0;
        q.cx0 = cx0;
        q.b0 = b0;
    };
    float4 pc[4];
    bool any8 = true;  // some residual of the step in flight needs the 9th column
    auto issue = [&](int k, Geo8 &q) {
        geo(k, q);
        const int m = q.m;
        const unsigned col = (unsigned)(q.cx0 + sl) << 4, base = (unsigned)q.b0 * band;
#pragma unroll
        for (int b = 0; b < kBoxBands; b++)
            pc[b] = ldb4(rsrc, (m >> (b * kBoxCols + sl)) & 1 ? base + b * band + col : kOOB);
        const bool n8 = sl < kBoxBands && ((m >> (sl * kBoxCols + 8)) & 1);
        any8 = __ballot(n8) != 0;
        if (any8)
            pc[3] = ldb4(rsrc, n8 ? base + sl * band + ((unsigned)(q.cx0 + 8) << 4) : kOOB);
    };
    auto store = [&]() {
        float4 *bx = reinterpret_cast<float4 *>(box);
#pragma unroll
        for (int b = 0; b < kBoxBands; b++) bx[b * kBoxCols + sl] = pc[b];
        if (any8)
            bx[sl < kBoxBands ? sl * kBoxCols + 8 : kBoxBands * kBoxCols] = pc[3];
    };
    // the 12 taps of the lane's pixel from the residual's box
    auto box_taps = [&](const Geo8 &q, float *iv) {
        const int ix = (int)q.Ku, iy = (int)q.Kv;
        // row y of column ix - 1: box float (((y >> 2) - b0) * 9 + ix - 1 - cx0) * 4 + (y & 3)
        // = y + 32 (y >> 2) + 4 (ix - 1 - cx0) - 36 b0; the next columns are 4 floats apart
        static_assert(kBoxCols == 9, "row offsets below assume 9 columns of 4 floats per band");
        const int base = 4 * (ix - 1 - q.cx0) - 36 * q.b0;
        auto row = [&](int y) { return box + (y + ((y >> 2) << 5) + base); };
        const float *r0 = row(iy - 1), *r1 = row(iy), *r2 = row(iy + 1), *r3 = row(iy + 2);
        iv[0] = r0[4];
        iv[1] = r0[8];
        iv[2] = r1[0];
        iv[3] = r1[4];
        iv[4] = r1[8];
        iv[5] = r1[12];
        iv[6] = r2[0];
        iv[7] = r2[4];
        iv[8] = r2[8];
        iv[9] = r2[12];
        iv[10] = r3[4];
        iv[11] = r3[8];
    };
    // the 17 addends of the residuals this pass owns (kWide: the wide ones), summed in pattern order
    // into their sums rows; an owned residual with a pixel out of bounds or not finite gets the
    // "pattern not ok" mark.  Residuals the pass does not own are left untouched.
    auto terms = [&](int k, const Geo8 &q, bool owner, const float *iv) {
        const int j = 8 * k + g;
        const bool part = owner && q.gok;
        bool fin = false;
        float tt[kSums];
        if (part) {
            const float color = S[j * kSumStride + sl], weight = S[j * kSumStride + 8 + sl];
            const int ix = (int)q.Ku, iy = (int)q.Kv;
            const float3 s3 = bilin12(iv, q.Ku - ix, q.Kv - iy);
            fin = isfinite(s3.x);
            pixel_terms<kMarg>(s3.x, s3.y, s3.z, color, weight, aff0, aff1, b0a, tt, kMarg ? q.jx : 0.f,
                               kMarg ? q.jy : 0.f, da, db, fixA, fixB);
        }
        const unsigned long long m2 = __ballot(fin);
        const bool rok = part && ((m2 >> (8 * g)) & 0xFFull) == 0xFFull;
        auto sum8 = [&](int qq, int e) {
            const float4 a = *(const float4 *)&T[e * 8], b = *(const float4 *)&T[e * 8 + 4];
            float sum = 0.0f;
            sum += a.x;
            sum += a.y;
            sum += a.z;
            sum += a.w;
            sum += b.x;
            sum += b.y;
            sum += b.z;
            sum += b.w;
            S[j * kSumStride + qq] = sum;
        };
        wave_lds_sync();  // every box read is done before the terms overwrite the boxes
        if (part) {
#pragma unroll
            for (int e = 0; e < kTermQ; e++) T[e * 8 + sl] = tt[e];
        }
        wave_lds_sync();
        if (rok) {
            sum8(sl, sl);
            if (sl == 0) sum8(8, 8);
        } else if (owner && sl == 0 && j < jlimit) {
            S[j * kSumStride] = -1.0f;  // energy slot: pattern not ok
        }
        wave_lds_sync();
        if (part) {
#pragma unroll
            for (int e = 0; e < kSums - kTermQ; e++) T[e * 8 + sl] = tt[kTermQ + e];
        }
        wave_lds_sync();
        if (rok) sum8(kTermQ + sl, sl);
        wave_lds_sync();
    };
    Geo8 cur, nxt;
    pc[3] = make_float4(0.f, 0.f, 0.f, 0.f);
    unsigned wide_steps = 0;
    auto step = [&](int k, Geo8 &now, Geo8 &next) {
        store();             // waits for step k's pieces
        issue(k + 1, next);  // step k+1's pieces in flight during step k's arithmetic
        wave_lds_sync();
        const bool wide = now.gok && now.wide;
        if (__ballot(wide)) wide_steps |= 1u << k;
        float iv[12];
        if (now.gok && !wide) box_taps(now, iv);
        terms(k, now, !wide, iv);
    };
    issue(0, cur);
    for (int k = 0; k < nsteps; k += 2) {  // ping-pong: no copies of the in-flight step's geometry
        step(k, cur, nxt);
        if (k + 1 >= nsteps) break;
        step(k + 1, nxt, cur);
    }
    // residuals whose footprint exceeds the box: per-lane gathers, step by step
    while (wide_steps) {
        const int k = __builtin_ctz(wide_steps);
        wide_steps &= wide_steps - 1;
        geo(k, cur);
        const bool wide = cur.gok && cur.wide;
        float iv[12];
        if (wide) load12(rsrc, band, (int)cur.Ku, (int)cur.Kv, iv);
        terms(k, cur, wide, iv);
    }
}

template <int kImg, bool kMarg>
__global__ __launch_bounds__(256, kLinBlocksPerCu) void k_linearize(LinParams P) {
    static_assert(kImg == 1 || kImg == 3, "image layouts 1 and 3");
    extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float *lds_terms_w = lds_dyn + wave * kWaveLds;
    float *lds_sums_w = lds_terms_w + kTermsPerWave;
    // XCD-aware mapping: blocks b, b+8, b+16, ... share an XCD (round-robin dispatch), so each XCD
    // gets one contiguous range of chunks; chunks are ordered (window, target, host), so the
    // chunks reading one target frame run on one XCD and share its L2.
    const int nb = P.n_blocks, xcd = blockIdx.x & 7, q8 = nb >> 3, r8 = nb & 7;
    const int lblock = xcd * q8 + min(xcd, r8) + (blockIdx.x >> 3);
    if (lblock * 4 + wave >= P.n_items) return;
    const int itemL = P.item_base + lblock * 4 + wave;  // global chunk index
    const int4 it = P.items[itemL];                     // {res_begin, count, pair_global, win}
    if (P.stop && P.pass > P.stop[__builtin_amdgcn_readfirstlane(it.w)]) return;  // window left the GN loop
    const int cnt = it.y & 0xFFFF;  // bit 16: the pair's first chunk (writes the geometry snapshot)
    const bool valid = lane < cnt;
    const int pair = __builtin_amdgcn_readfirstlane(it.z), jlimit = __builtin_amdgcn_readfirstlane(cnt);
    const WinDev &W = P.wins[__builtin_amdgcn_readfirstlane(it.w)];
    const int N = W.N;
    const int h = (pair - W.pair_base) % N, t = (pair - W.pair_base) / N;
    const float *pre = P.precalc + (size_t)pair * LDSO_BA_PRECALC_STRIDE;
    const float th = fmaxf(P.frame_th[W.frame_base + h], P.frame_th[W.frame_base + t]);
    const float wM3 = W.wM3, hM3 = W.hM3;
    const float4 *img = P.img + (size_t)(W.frame_base + t) * P.frame_stride;
    const __amdgpu_buffer_rsrc_t rsrc = frame_rsrc(reinterpret_cast<const float *>(img), P.frame_stride * 16);
    const unsigned band = (unsigned)P.tiles_per_row * 8u * 16u;

    const int r = it.x + lane;
    // Everything phase B needs is loaded up front (unconditionally, from a clamped index: a load
    // inside a divergent branch is waited for at the branch's end) so it lands during phase A.
    const int rq = valid ? r : 0;
    int my_state = P.rs_state[rq];
    const int my_slot = P.rs_slot[rq];
    // the point from the record slot (rec_base + s P + q, s = the target's slot of host h): no
    // per-residual point index is read
    const int my_point = valid ? W.point_base + (my_slot - W.rec_base - (t < h ? t : t - 1) * W.P) : W.point_base;
    uint8_t flags = P.rs_flags[rq];
    float state_energy = P.rs_energy[rq];
    float new_energy = P.rs_newenergy[rq];
    const float4 my_pd0 = *(const float4 *)(P.pt_data + (size_t)my_point * LDSO_BA_POINT_STRIDE);
    // the point's color[8] and weights[8] (record floats 8..23: one 64-B piece per residual)
    // into this residual's row of the sums table: phase A's pattern lanes read them from LDS at
    // the step that later overwrites the row with the residual's sums (no per-step gathers)
    {
        const float4 *cw = reinterpret_cast<const float4 *>(P.pt_data + (size_t)my_point * LDSO_BA_POINT_STRIDE + 8);
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = cw[u];
        float *row = lds_sums_w + lane * kSumStride;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            row[4 * u] = v[u].x;
            row[4 * u + 1] = v[u].y;
            row[4 * u + 2] = v[u].z;
            row[4 * u + 3] = v[u].w;
        }
    }
    if (!valid) my_state = LDSO_BA_RES_OOB;
    // marginalisation pass: Jp * delta of fixLinearizationF (Residuals.cc:221-232) from the centre
    // geometry, per residual, before the pattern pixels need it (dot products left to right)
    float jp_dx = 0.f, jp_dy = 0.f, da = 0.f, db = 0.f;
    if constexpr (kMarg) {
#pragma clang fp contract(off)
        const float *dp = P.ad_ht_delta + (size_t)pair * 8;
        da = dp[6];  // delta_a, delta_b of the pair (adHTdeltaF[6], [7])
        db = dp[7];
        Geo gm;
        if (centre_projection(pre, my_pd0.x, my_pd0.y, my_pd0.w, W.calib[0], W.calib[1], W.calib[2], W.calib[3],
                              wM3, hM3, gm)) {
            const float dd = P.pt_data[(size_t)my_point * LDSO_BA_POINT_STRIDE + 5];
            float x6 = 0.f, y6 = 0.f, x4 = 0.f, y4 = 0.f;
#pragma unroll
            for (int i = 0; i < 6; i++) {
                x6 += gm.d_xi_x[i] * dp[i];
                y6 += gm.d_xi_y[i] * dp[i];
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                x4 += gm.d_C_x[i] * W.cdelta[i];
                y4 += gm.d_C_y[i] * W.cdelta[i];
            }
            jp_dx = x6 + x4 + gm.d_d_x * dd;
            jp_dy = y6 + y4 + gm.d_d_y * dd;
        }
    }

    // ---------------- phase A: pattern pixels, 8 residuals per step -------------------------
    wave_lds_sync();  // every row's color / weights are in before any lane reads another's
    if constexpr (kImg == 3) {
        *reinterpret_cast<float4 *>(lds_sums_w + kSumsPerWave + 4 * lane) =
            make_float4(my_pd0.x, my_pd0.y, my_pd0.z, __int_as_float(my_state));
        wave_lds_sync();
        phase_a_pieces<kMarg>(lane, lds_terms_w, lds_sums_w, pre, jlimit, my_state, my_pd0, jp_dx, jp_dy, da, db,
                              rsrc, band, wM3, hM3, __builtin_amdgcn_readfirstlane(P.aff_fix));
    } else {
#pragma clang fp contract(off)
        const int g = lane >> 3, sl = lane & 7;
        // staticPattern[8] (Setting.cc:275) offset of this lane's pixel
        const int px = sl == 1 || sl == 6 ? -1 : sl == 2 ? 1 : sl == 3 ? -2 : sl == 5 ? 2 : 0;
        const int py = sl == 0 ? -2 : sl <= 2 ? -1 : sl <= 5 ? 0 : sl == 6 ? 1 : 2;
        const float aff0 = pre[24], aff1 = pre[25], b0 = pre[26];
        float *T = lds_terms_w + g * (kTermQ * 8);
        float *S = lds_sums_w;
        const int nsteps = (jlimit + 7) >> 3;
        const int tpr2 = P.tiles_per_row;

        struct Stage {
            float Ku, Kv, color, weight;
            float iv[12];               // layout 3: the 12 intensities (load12)
            float3 t00, t10, t01, t11;  // layout 1: the four texels
            float jx, jy;               // kMarg: Jp_delta of the residual
            bool gok;
        };
        auto issue = [&](int k, Stage &q) {
            const int j = 8 * k + g;
            const int st = __shfl(my_state, j, kWave);
            const int p = __shfl(my_point, j, kWave);
            const float pu = __shfl(my_pd0.x, j, kWave), pv = __shfl(my_pd0.y, j, kWave),
                        pz = __shfl(my_pd0.z, j, kWave);
            const bool go = j < jlimit && st != LDSO_BA_RES_OOB;
            if constexpr (kMarg) {
                q.jx = __shfl(jp_dx, j, kWave);
                q.jy = __shfl(jp_dy, j, kWave);
            }
            (void)p;
            q.color = S[j * kSumStride + sl];
            q.weight = S[j * kSumStride + 8 + sl];
            const float up = pu + px, vp = pv + py;
            float ptp[3];
#pragma unroll
            for (int i = 0; i < 3; i++)
                ptp[i] = (pre[3 * i] * up + pre[3 * i + 1] * vp + pre[3 * i + 2] * 1.0f) + pre[9 + i] * pz;
            q.Ku = ptp[0] / ptp[2];
            q.Kv = ptp[1] / ptp[2];
            const bool pok = go && q.Ku > 1.1f && q.Kv > 1.1f && q.Ku < wM3 && q.Kv < hM3;
            const unsigned long long m1 = __ballot(pok);
            q.gok = ((m1 >> (8 * g)) & 0xFFull) == 0xFFull;
            // taps of an in-bounds pixel are always addressable; others read around texel (1, 1)
            const int ix = pok ? (int)q.Ku : 1, iy = pok ? (int)q.Kv : 1;
            if constexpr (kImg == 3) {
                load12(rsrc, band, ix, iy, q.iv);
            } else {
                q.t00 = tex(img, tpr2, ix, iy);
                q.t10 = tex(img, tpr2, ix + 1, iy);
                q.t01 = tex(img, tpr2, ix, iy + 1);
                q.t11 = tex(img, tpr2, ix + 1, iy + 1);
            }
        };
        auto consume = [&](int k, const Stage &q) {
            const int j = 8 * k + g;
            bool fin = false;
            float tt[kSums];
            if (q.gok) {
                const int ix = (int)q.Ku, iy = (int)q.Kv;
                const float dx = q.Ku - ix, dy = q.Kv - iy;
                float I, gx, gy;
                if constexpr (kImg == 3) {
                    const float3 s3 = bilin12(q.iv, dx, dy);
                    I = s3.x;
                    gx = s3.y;
                    gy = s3.z;
                } else {
                    const float dxdy = dx * dy;
                    const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
                    I = w11 * q.t11.x + w01 * q.t01.x + w10 * q.t10.x + w00 * q.t00.x;
                    gx = w11 * q.t11.y + w01 * q.t01.y + w10 * q.t10.y + w00 * q.t00.y;
                    gy = w11 * q.t11.z + w01 * q.t01.z + w10 * q.t10.z + w00 * q.t00.z;
                }
                fin = isfinite(I);
                pixel_terms<kMarg, kImg == 1>(I, gx, gy, q.color, q.weight, aff0, aff1, b0, tt, kMarg ? q.jx : 0.f,
                                   kMarg ? q.jy : 0.f, da, db, (P.aff_fix & 1) != 0, (P.aff_fix & 2) != 0);
            }
            const unsigned long long m2 = __ballot(fin);
            const bool rok = q.gok && ((m2 >> (8 * g)) & 0xFFull) == 0xFFull;
            // two transposition rounds (quantities 0-8, then 9-16): lane sl adds quantity q0 + sl
            // (lane 0 also quantity 8) over the 8 pixels in pattern order
            auto sum8 = [&](int qq, int e) {
                const float4 a = *(const float4 *)&T[e * 8], b = *(const float4 *)&T[e * 8 + 4];
                float sum = 0.0f;
                sum += a.x;
                sum += a.y;
                sum += a.z;
                sum += a.w;
                sum += b.x;
                sum += b.y;
                sum += b.z;
                sum += b.w;
                S[j * kSumStride + qq] = sum;
            };
            if (q.gok) {
#pragma unroll
                for (int e = 0; e < kTermQ; e++) T[e * 8 + sl] = tt[e];
            }
            wave_lds_sync();
            if (rok) {
                sum8(sl, sl);
                if (sl == 0) sum8(8, 8);
            } else if (sl == 0 && j < jlimit) {
                S[j * kSumStride] = -1.0f;  // energy slot: pattern not ok
            }
            wave_lds_sync();
            if (q.gok) {
#pragma unroll
                for (int e = 0; e < kSums - kTermQ; e++) T[e * 8 + sl] = tt[kTermQ + e];
            }
            wave_lds_sync();
            if (rok) sum8(kTermQ + sl, sl);
            wave_lds_sync();
        };
        // ping-pong stages, loads issued unconditionally (a step past the chunk's end has no valid
        // group and reads around texel (1, 1)), so no load result crosses a branch join
        Stage A, B;
        issue(0, A);
        for (int k = 0; k < nsteps; k += 2) {
            issue(k + 1, B);
            consume(k, A);
            issue(k + 2, A);
            consume(k + 1, B);
        }
    }

    // ---------------- phase B: lane per residual ---------------------------------------------
    double energy = 0;
    bool isIN = false, active = false;
    Geo g;
    PhotoSums s;
    if (valid) {
        const int8_t old_state = (int8_t)my_state;
        int8_t new_state = LDSO_BA_RES_OOB;
        float e_wo = -1;
        if (old_state == LDSO_BA_RES_OOB) {
            energy = state_energy;  // linearize returns state_energy; applyRes returns early
            st_nt(P.rec_b + my_slot, make_float2(0.f, __builtin_nanf("")));  // not active
        } else {
            const float4 pd0 = my_pd0;
            const float *Sr = lds_sums_w + lane * kSumStride;
            s.energy = Sr[0];
            s.wJI2 = Sr[1];
            s.JIdx2_00 = Sr[2];
            s.JIdx2_10 = Sr[3];
            s.JIdx2_11 = Sr[4];
            s.JabJIdx_00 = Sr[5];
            s.JabJIdx_01 = Sr[6];
            s.JabJIdx_10 = Sr[7];
            s.JabJIdx_11 = Sr[8];
            s.Jab2_00 = Sr[9];
            s.Jab2_01 = Sr[10];
            s.Jab2_11 = Sr[11];
            s.JI_r0 = Sr[12];
            s.JI_r1 = Sr[13];
            s.Jab_r0 = Sr[14];
            s.Jab_r1 = Sr[15];
            s.rr = Sr[16];
            const bool pat_ok = !(s.energy < 0.0f);
            bool ok = centre_projection(pre, pd0.x, pd0.y, pd0.w, W.calib[0], W.calib[1], W.calib[2], W.calib[3],
                                        wM3, hM3, g);
            // centerProjectedTo: written where projected, kept (not re-read) where not
            float *centre = P.rs_center + r;  // planes: coalesced 4-B stores, whole lines
            const long long cs = P.center_stride;
            if (ok) {
                st_nt(centre, g.Ku);
                st_nt(centre + cs, g.Kv);
                st_nt(centre + 2 * cs, g.new_idepth);
            }
            ok = ok && pat_ok;
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
            write_record(P.rec_a + my_slot, P.rec_b + my_slot, active, pd0.w, g, s);
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
                centre[3 * cs] = 0.01f * sqrtf(dx * dx + dy * dy);
            }
            st_nt(P.rs_state + r, new_state);
            st_nt(P.rs_flags + r, flags);
            st_nt(P.rs_energy + r, state_energy);
            st_nt(P.rs_newenergy + r, new_energy);
        }
        isIN = (new_state == LDSO_BA_RES_IN);
        st_nt(P.rs_newstate + r, new_state);
        st_nt(P.rs_energy_wo + r, e_wo);
    }

    // linearizeAll stats: sum of returned energies (double) and #IN, per chunk
    double esum = energy;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) esum += __shfl_xor(esum, m, kWave);
    const unsigned long long inmask = __ballot(isIN);
    if (lane == 0) {
        P.item_energy[2 * itemL] = esum;
        P.item_energy[2 * itemL + 1] = (double)__popcll(inmask);
    }
    // the pass's centre geometry inputs of this pair, for the readers of the records after the
    // live precalc has moved on (write_record); by the pair's first chunk, after its real work
    if ((it.y >> 16) && P.geo_snap && lane < kGeoSnap)
        P.geo_snap[(size_t)pair * kGeoSnap + lane] = lane < 12 ? pre[12 + lane] : W.calib[lane - 12];
    if (!P.accumulate) return;
    wave_lds_sync();  // every lane has read its sums: the wave's LDS becomes the operand table
    top_mfma(lds_terms_w, lane, active, g, s, P.top_slab + (size_t)itemL * kTopVals);
}

// ============================================================================================
// k_point_sc
// ============================================================================================
struct PointParams {
    const int4 *__restrict__ items;  // {pt_begin, count, host, win}
    const WinDev *__restrict__ wins;
    const float *__restrict__ pt_data;
    const int *__restrict__ pt_nres;
    const unsigned long long *__restrict__ pt_tgt;  // [P]: residual targets, 4 bits each, caller order
    const float4 *__restrict__ rec_a;                // [slots] (WinDev::rec_base layout, write_record)
    const float2 *__restrict__ rec_b;
    const float *__restrict__ precalc;               // the pass's pair precalc (centre geometry)
    float *pt_out;                     // [P][12]
    float *sc_slab;
    int n_items;
    int item_base;
    int shift_prior;  // AccumulatedSCHessianSSE::addPoint's shiftPriorToZero (false when marginalising)
    const int *stop;  // ldso_ba_optimize (LinParams::stop)
    int pass;
    // ldso_ba_optimize: blocks [0, n_nid) compute doStepFromBackup's sumNID / numID of window
    // blockIdx.x (point_nid); the point-chunk blocks follow
    double *win_nid;  // [win][2] (ldso_ba_ctx::win_nid)
    int n_nid, nid_chunk;
};

// doStepFromBackup's sumNID and numID (FullSystem.cc:1899-1909) for the step that follows this
// pass: the float sum of fabsf(idepth_backup) over the window's points in frames -> features order
// (host frames in window order, each host's points in the caller's order: the device point order),
// i.e. over the idepths this pass linearised at.  The chain of float adds is sequential by
// definition, so one lane walks it from LDS (the block stages chunks of the idepths), in a block of
// its own beside other work: extra blocks of k_solve_fast (the default), of k_point_sc (exact solve
// modes), or, with points sharded over ranks, over the exchange's gathered runs (NidSrc).
// The idepths of one window's chain: its own points (pt_data), or, with points sharded over ranks,
// every rank's run of |idepth| from the exchange's all-gather, concatenated in rank order -- the
// runs are contiguous pieces of the host-frame order, so the concatenation is the unsharded order
// and the chain is bit for bit the single-GPU one (runs zero-padded to prun: + 0 leaves s as is).
struct NidSrc {
    const float *pt_data;   // [points][LDSO_BA_POINT_STRIDE], idepth at + 2
    const float *gathered;  // non-null: [rank][window][slot] exchange slots, the run at + off
    long long slot, off;
    int n_ranks, n_win, prun;
};
__device__ void nid_chain(const WinDev &W, const NidSrc &src, double *win_nid, int w, float *lds, int chunk) {
    const int n = src.gathered ? src.n_ranks * src.prun : W.P, tid = threadIdx.x;
    const float *pd = src.pt_data + (size_t)W.point_base * LDSO_BA_POINT_STRIDE + 2;
    auto value = [&](int i) {
        if (!src.gathered) return fabsf(pd[(size_t)i * LDSO_BA_POINT_STRIDE]);
        const int r = i / src.prun, q = i - r * src.prun;
        return src.gathered[((size_t)r * src.n_win + w) * src.slot + src.off + q];
    };
    float s = 0.0f;
    for (int q0 = 0; q0 < n; q0 += chunk) {
        const int m = min(chunk, n - q0);
        for (int i = tid; i < m; i += blockDim.x) lds[i] = value(q0 + i);
        for (int i = m + tid; i < ((m + 3) & ~3); i += blockDim.x) lds[i] = 0.0f;  // +0 leaves s unchanged
        __syncthreads();
        if (tid == 0) {
            const float4 *l4 = reinterpret_cast<const float4 *>(lds);
#pragma unroll 8
            for (int i = 0; i < (m + 3) / 4; i++) {
                const float4 v = l4[i];
                s += v.x;
                s += v.y;
                s += v.z;
                s += v.w;
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        win_nid[2 * w] = (double)s;  // exact; read back as float
        win_nid[2 * w + 1] = (double)(float)W.p_all;  // numID++ per point (float): exact below 2^24
    }
}
__device__ void point_nid(const PointParams &P, int w, float *lds) {
    if (P.stop && P.pass > P.stop[w]) return;
    NidSrc src{};
    src.pt_data = P.pt_data;
    nid_chain(P.wins[w], src, P.win_nid, w, lds, P.nid_chunk);
}

// points per k_point_sc block (one SYRK chunk partial).  128 (both waves gather, half the slab
// partials) measured 28.5 vs 26.5 us with the stitch 0.8 us faster: the SYRK chains double (r4)
constexpr int kScPoints = 64;
constexpr int kPrePitch = 12;  // floats of staged precalc (R0, t0) per target in k_point_sc's LDS
constexpr int kScThreads = 128;  // 2 waves: a lane per point gathers, both run the SYRK tiles
static_assert(kScPoints <= kScThreads, "one gathering lane per point");
// residual records per round trip (r4: 3 -> two round trips at N = 7, 27.6 vs 28.3 us; r5: 6 -> one round
// trip, 30.0 vs 27.6 us with 48-B records, 30.6 vs 25.9 us with 24-B records)
constexpr int kScBatch = 3;
__global__ __launch_bounds__(kScThreads) void k_point_sc(PointParams P) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    if ((int)blockIdx.x < P.n_nid) {
        point_nid(P, blockIdx.x, smem);
        return;
    }
    const int item = P.item_base + blockIdx.x - P.n_nid;
    const int4 it = P.items[item];
    if (P.stop && P.pass > P.stop[it.w]) return;  // window left the GN loop
    const WinDev &W = P.wins[it.w];
    const int host = it.z, KP = W.KP, nt = KP / 4, ntiles = W.ntiles;
    const int Kj = 8 * (W.N - 1);
    // rows of KP + 4 floats: KP is a multiple of 8, so a pitch of 4 mod 8 dwords spreads the lanes'
    // 16-B row accesses (a lane per point) over distinct bank slots (ds_write_b128: 8-lane groups,
    // banks mod 32; ds_read_b128: 16-lane groups, banks mod 64); a pitch of KP put lanes q and q + 4
    // (writes) or q and q + 24 (reads) on the same banks
    const int KPP = KP + 4;
    float *U = smem;               // [kScPoints][KPP]
    const int tid = threadIdx.x;
    // this lane's point and its first records are requested before the block waits for the
    // precalc staging below, so those round trips overlap (unconditional loads from a clamped index)
    const bool mine = tid < it.y;
    const int p = it.x + (mine ? tid : 0);
    const int nres = P.pt_nres[p];
    const unsigned long long tgs = P.pt_tgt[p];
    const float4 pd0 = *reinterpret_cast<const float4 *>(P.pt_data + (size_t)p * LDSO_BA_POINT_STRIDE);
    const float2 pd1 = *reinterpret_cast<const float2 *>(P.pt_data + (size_t)p * LDSO_BA_POINT_STRIDE + 4);
    const size_t rp = (size_t)W.rec_base + (p - W.point_base), sstride = (size_t)W.P;
    float4 ra[kScBatch];
    float2 rb[kScBatch];
    auto load_batch = [&](int k0) {  // records k0 .. k0 + kScBatch - 1 (clamped to the point's last)
#pragma unroll
        for (int u = 0; u < kScBatch; u++) {
            const int k = max(0, min(k0 + u, nres - 1));
            const int tg = (int)((tgs >> (4 * k)) & 15ull);
            const size_t q = rp + (nres > 0 ? (tg < host ? tg : tg - 1) : 0) * sstride;
            ra[u] = P.rec_a[q];
            rb[u] = P.rec_b[q];
        }
    };
    load_batch(0);
    // the host's pair precalc R0 / t0 (record floats 12..23) for every target, staged once per block:
    // every residual's centre geometry reads them from LDS (kPrePitch floats per target)
    float *pre_lds = smem + kScPoints * KPP;
    for (int e = tid; e < W.N * 12; e += blockDim.x) {
        const int t = e / 12, k = e - 12 * t;
        pre_lds[t * kPrePitch + k] = P.precalc[(size_t)(W.pair_base + host + W.N * t) * LDSO_BA_PRECALC_STRIDE + 12 + k];
    }
    __syncthreads();
    if (mine) {
#pragma clang fp contract(off)
        // the sums in residual order exactly as AccumulatedTopHessian.cc:94-116 adds them
        float hdd = 0, bd = 0, hcd[4] = {0, 0, 0, 0};
        int ngood = 0;
        float *row = U + tid * KPP;
        unsigned filled = 0;  // target slots whose JpJdF is in the row
        for (int k0 = 0; k0 < nres; k0 += kScBatch) {
            if (k0) load_batch(k0);
#pragma unroll
            for (int u = 0; u < kScBatch; u++) {
                const int k = k0 + u;
                if (k >= nres || rb[u].y != rb[u].y) continue;  // NaN idepth: not active
                ngood++;
                const int tg = (int)((tgs >> (4 * k)) & 15ull);
                // the residual's centre geometry, as k_linearize's phase B formed it (same inputs,
                // same statements), then point_terms' Hdd_r / Hcd_r from its (j0, j1)
                Geo g;
                (void)centre_projection(pre_lds + tg * kPrePitch - 12,  // R0 = [12..20], t0 = [21..23]
                                        pd0.x, pd0.y, pd0.w, W.calib[0], W.calib[1], W.calib[2], W.calib[3], W.wM3,
                                        W.hM3, g);
                const float4 ja = ra[u];
                float jp[6];
                record_jp6(g, ja.x, ja.y, jp);
                bd += rb[u].x;
                hdd += ja.x * g.d_d_x + ja.y * g.d_d_y;
#pragma unroll
                for (int i = 0; i < 4; i++) hcd[i] += g.d_C_x[i] * ja.x + g.d_C_y[i] * ja.y;
                const int slot = tg < host ? tg : tg - 1;
                *(float4 *)(row + 8 * slot) = make_float4(jp[0], jp[1], jp[2], jp[3]);
                *(float4 *)(row + 8 * slot + 4) = make_float4(jp[4], jp[5], ja.z, ja.w);
                filled |= 1u << slot;
            }
        }
        {  // the rest of the row: zeros (the SYRK reads every column of the point's row)
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int sl = 0; sl < W.N - 1; sl++)
                if (!((filled >> sl) & 1u)) {
                    *(float4 *)(row + 8 * sl) = z;
                    *(float4 *)(row + 8 * sl + 4) = z;
                }
            for (int c = Kj; c < KP; c++) row[c] = 0.f;
        }
        const float priorF = pd1.x, deltaF = pd1.y;
        float HdiF = 0, bdSum = 0, ih = 0;
        if (ngood > 0) {
            // AccumulatedSCHessian.cc:24-33 (Hdd_accLF = bd_accLF = Hcd_accLF = 0 in the hot path)
            float H = hdd + 0.0f + priorF;
            if (H < 1e-10f) H = 1e-10f;
            ih = H;
            HdiF = (float)(1.0 / (double)H);
            bdSum = bd + 0.0f;
            if (P.shift_prior) bdSum += priorF * deltaF;
            row[Kj + 0] = hcd[0] + 0.0f;
            row[Kj + 1] = hcd[1] + 0.0f;
            row[Kj + 2] = hcd[2] + 0.0f;
            row[Kj + 3] = hcd[3] + 0.0f;
            row[Kj + 4] = bdSum;
        }
        {
            const float sw = sqrtf(HdiF);
            float4 *r4 = reinterpret_cast<float4 *>(row);
            for (int q = 0; q < (Kj + 5 + 3) / 4; q++) {
                float4 v = r4[q];
                v.x *= sw;
                v.y *= sw;
                v.z *= sw;
                v.w *= sw;
                r4[q] = v;
            }
        }
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
    float *slab = P.sc_slab + W.sc_slab_base + (size_t)(item - W.sc_item_base) * ntiles * 16;
    syrk_tiles(U, KPP, nt, ntiles, it.y, slab, tid, blockDim.x);
}

// ============================================================================================
// k_stitch: one 256-thread block per frame pair (h,t) of every window, straight from the
// partial slabs of k_linearize / k_point_sc, writing the pair's contributions to the packed
// upper triangles of {HA, bA, Hsc, bsc} as one record per (pair, block) that k_stitch_sum adds
// in a fixed pair order (no atomics: the system is bitwise repeatable):
//   Top  bucket (h,t): sum the chunk partials, AccumulatorApprox::finish layout, adjoint
//        sandwiches (AccumulatedTopHessian.cc:213-239), symmetrised as stitchDoubleMT does
//        (H(a,b) = H(a,b) + H(b,a)^T, H(c,h) = H(h,c)^T; AccumulatedTopHessian.h:91-104)
//   SC   host i = h, target j = t: rows of G_i for slot j (accD/accE/accEB of
//        AccumulatedSCHessian.cc:35-50) summed from the SYRK chunk partials, then
//        AccumulatedSCHessian.cc:80-114; only the upper triangle is produced (the solve reads
//        only it, EnergyFunctional.cc:378) using D_kj = D_jk^T.
// The diagonal (h == t) blocks have no residuals; block (0,0) of each window instead runs
// setNewFrameEnergyTH (FullSystem.cc:2078-2109) and the linearizeAll energy sum.
// ============================================================================================
constexpr int kStThreads = 256;
constexpr int kStTopLds = 528;  // doubles of k_stitch LDS used by the Top half (521, padded)
constexpr int kThMaxLds = 8192;  // k_frame_th: candidate energies staged in LDS; larger sets re-read HBM

struct StitchParams {
    const WinDev *__restrict__ wins;
    const int *__restrict__ pair_win;
    const float *__restrict__ e_wo;
    float *frame_th;
    const int2 *__restrict__ pair_items;  // per global pair: {first top item, n items}
    const float *__restrict__ top_slab;
    const double *__restrict__ item_energy;
    const int2 *__restrict__ host_items;  // per global frame: {first sc item, n items}
    const float *__restrict__ sc_slab;
    const double *__restrict__ adH;
    const double *__restrict__ adT;
    double *sys;
    double *stage;  // k_stitch -> k_stitch_sum contribution records (WinDev::stage_base)
    double *win_energy;
    double *ehist;         // non-null (ldso_ba_optimize): also win_energy into row `pass` of the history
    const int *stop;       // ldso_ba_optimize (LinParams::stop): host / pair blocks of stopped windows skip
    int pass;
    int accumulate;
    int th_cap;  // newest-frame energies staged in LDS by setNewFrameEnergyTH
    int pair_base;  // first global pair of this launch
    int hs_split;   // k_stitch_host: two blocks per host (Top / SC halves)
    const int *__restrict__ frame_win;  // k_stitch_host: window of each global frame
    int frame_base;                     // k_stitch_host: first global host frame of this launch
    int win_base;   // first window of this launch
    int n_win;      // windows of this launch: blocks [0, n_win) run their setNewFrameEnergyTH
};

__device__ __forceinline__ long long pk_index(int row, int col, int D) {  // row <= col
    return (long long)row * D - (long long)row * (row - 1) / 2 + (col - row);
}

// setNewFrameEnergyTH (FullSystem.cc:2078-2109) as an exact 4-pass radix select with
// nth_element semantics over the candidates get(i), i in [0, n_cand), that are >= 0.
// Candidates are staged in LDS when they fit; larger sets are re-read from global memory.
// Every thread of the block must call it; thread 0 writes *th_out.
// LDS behind the candidate keys: a 256-bin histogram per wave, 16 words of shared scalars, and
// two doubles per wave for the energy sum
__host__ __device__ constexpr size_t th_fixed_bytes(int threads) {
    return ((size_t)(threads / 64) * 256 + 16) * sizeof(unsigned) + (size_t)(threads / 64) * 2 * sizeof(double);
}
template <int kT, class Get>
__device__ void select_frame_th(Get get, int n_cand, unsigned *keys, int cap, float *th_out) {
    // LDS: keys[cap] | hist[kW waves][256] | sh[16]
    constexpr int kW = kT / 64;
    unsigned *hist = keys + cap;
    unsigned *sh = hist + kW * 256;  // [0..kW) per-wave valid counts, [kW] prefix, [kW+1] rank
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool in_lds = n_cand <= cap;
    // stage every candidate at its own index (no compaction, so no dependent slot atomics):
    // an invalid one (NewEnergyWithOutlier < 0) becomes 0xFFFFFFFF, above every valid key, and
    // is never selected because the rank is taken among the valid ones only
    constexpr int kU = 8;
    unsigned cnt = 0;
    for (int i0 = 0; i0 < n_cand; i0 += kT * kU) {
        float x[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) x[u] = get(min(i0 + u * kT + tid, n_cand - 1));  // loads in flight
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int idx = i0 + u * kT + tid;
            const bool ok = idx < n_cand && x[u] >= 0;
            cnt += ok ? 1u : 0u;
            if (in_lds && idx < n_cand) keys[idx] = ok ? (__float_as_uint(x[u]) & 0x7FFFFFFFu) : 0xFFFFFFFFu;
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) cnt += __shfl_xor(cnt, m, kWave);
    if (lane == 0) sh[wid] = cnt;
    __syncthreads();
    unsigned n = 0;
#pragma unroll
    for (int q = 0; q < kW; q++) n += sh[q];
    if (n == 0) {
        if (tid == 0) *th_out = 12 * 12 * LDSO_BA_PATTERN_NUM;
        __syncthreads();
        return;
    }
    unsigned prefix = 0, rank = (unsigned)(int)(kFrameEnergyTHN * (float)n);  // int nthIdx = 0.7f * size()
    unsigned *wh = hist + 256 * wid;  // per-wave sub-histogram: 4x less same-address contention
    for (int pass = 0; pass < 4; pass++) {
        const int shift = 24 - 8 * pass;
        const unsigned pmask = pass == 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * pass));
        for (int b = lane; b < 256; b += 64) wh[b] = 0;
        __syncthreads();
        if (in_lds) {
            for (int i = tid; i < n_cand; i += kT) {
                const unsigned key = keys[i];
                if ((key & pmask) == (prefix & pmask)) atomicAdd(&wh[(key >> shift) & 255u], 1u);
            }
        } else {
            for (int i = tid; i < n_cand; i += kT) {
                const float x = get(i);
                const unsigned key = x >= 0 ? (__float_as_uint(x) & 0x7FFFFFFFu) : 0xFFFFFFFFu;
                if ((key & pmask) == (prefix & pmask)) atomicAdd(&wh[(key >> shift) & 255u], 1u);
            }
        }
        __syncthreads();
        if (tid < 64) {  // one wave: lane l owns bins 4l..4l+3
            unsigned hb[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                hb[q] = 0;
#pragma unroll
                for (int v = 0; v < kW; v++) hb[q] += hist[256 * v + 4 * tid + q];
            }
            unsigned incl = hb[0] + hb[1] + hb[2] + hb[3];
#pragma unroll
            for (int m = 1; m < 64; m <<= 1) {
                const unsigned y = __shfl_up(incl, m, kWave);
                if (tid >= m) incl += y;
            }
            const unsigned long long hit = __ballot(incl > rank);
            const int first = __ffsll((long long)hit) - 1;
            if (tid == first) {
                unsigned acc = incl - (hb[0] + hb[1] + hb[2] + hb[3]);
                int d = 4 * tid;
                for (int q = 0; q < 4; q++, d++) {
                    if (acc + hb[q] > rank) break;
                    acc += hb[q];
                }
                sh[kW + 1] = rank - acc;
                sh[kW] = prefix | ((unsigned)d << shift);
            }
        }
        __syncthreads();
        prefix = sh[kW];
        rank = sh[kW + 1];
    }
    if (tid == 0) {
#pragma clang fp contract(off)
        const float nth = sqrtf(__uint_as_float(prefix));
        float v = nth * kFrameEnergyTHFacMedian;
        v = 26.0f * kFrameEnergyTHConstWeight + v * (1 - kFrameEnergyTHConstWeight);
        v = v * v;
        v *= kOverallEnergyTHWeight * kOverallEnergyTHWeight;
        *th_out = v;
    }
    __syncthreads();
}

template <int kT>
__device__ void frame_threshold_and_energy(const StitchParams &P, const WinDev &W, int w, unsigned *keys) {
    constexpr int kW = kT / 64;
    const int tid = threadIdx.x, N = W.N;
    const float *e_wo = P.e_wo + W.newest_begin;
    select_frame_th<kT>([&](int i) { return e_wo[i]; }, W.newest_end - W.newest_begin, keys, P.th_cap,
                        P.frame_th + W.frame_base + N - 1);
    double *red = reinterpret_cast<double *>(keys + P.th_cap + kW * 256 + 16);
    // linearizeAll: sum of returned energies and #IN in a fixed order (strided per thread, then
    // a fixed tree), so repeated passes give identical sums
    double se = 0, sn = 0;
    for (int k = tid; k < W.n_top_items; k += kT) {
        se += P.item_energy[2 * (W.top_item_base + k)];
        sn += P.item_energy[2 * (W.top_item_base + k) + 1];
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        se += __shfl_xor(se, m, kWave);
        sn += __shfl_xor(sn, m, kWave);
    }
    if ((tid & 63) == 0) {
        red[2 * (tid >> 6)] = se;
        red[2 * (tid >> 6) + 1] = sn;
    }
    __syncthreads();
    if (tid == 0) {
        double e = 0, nin = 0;  // the waves in a fixed tree: pairs, then pairs of pairs
        if constexpr (kW == 4) {
            e = (red[0] + red[2]) + (red[4] + red[6]);
            nin = (red[1] + red[3]) + (red[5] + red[7]);
        } else {
            static_assert(kW == 8, "4 or 8 waves");
            e = ((red[0] + red[2]) + (red[4] + red[6])) + ((red[8] + red[10]) + (red[12] + red[14]));
            nin = ((red[1] + red[3]) + (red[5] + red[7])) + ((red[9] + red[11]) + (red[13] + red[15]));
        }
        P.win_energy[2 * w] = e;
        P.win_energy[2 * w + 1] = nin;
        if (P.ehist) {  // the optimize() energy history, without a launch of its own
            double *hs = P.ehist + (size_t)P.pass * 2 * P.n_win;
            hs[2 * w] = e;
            hs[2 * w + 1] = nin;
        }
    }
}

// slot (r, c) of the 13x13 finish() matrix -> index into the 96-slot partial layout
__device__ __forceinline__ int top_slot(int r, int c) {
    if (r > c) {
        const int t = r;
        r = c;
        c = t;
    }
    if (c < 10) return r * 10 - r * (r - 1) / 2 + (c - r);  // Data[] (upper row-major)
    if (r < 10) return 55 + 3 * r + (c - 10);                // TopRight
    const int a = r - 10, b = c - 10;                        // BotRight
    return 85 + (a == 0 ? b : a == 1 ? 2 + b : 5);
}

// element (row, col) of G_h summed over the host's SYRK chunk partials (upper tiles only)
__device__ __forceinline__ double g_elem(const float *__restrict__ slab, int n_items, int per, int nt, int row,
                                         int col) {
    if (row > col) {
        const int t = row;
        row = col;
        col = t;
    }
    const int a = row >> 2, b = col >> 2;
    const int tile = a * nt - a * (a - 1) / 2 + (b - a);
    const float *src = slab + (size_t)tile * 16 + ((row & 3) << 2) + (col & 3);
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0;  // 4 independent loads in flight
    int k = 0;
    for (; k + 4 <= n_items; k += 4) {
        s0 += (double)src[(size_t)k * per];
        s1 += (double)src[(size_t)(k + 1) * per];
        s2 += (double)src[(size_t)(k + 2) * per];
        s3 += (double)src[(size_t)(k + 3) * per];
    }
    for (; k < n_items; k++) s0 += (double)src[(size_t)k * per];
    return (s0 + s1) + (s2 + s3);
}

__global__ __launch_bounds__(kStThreads) void k_stitch(StitchParams P) {
    extern __shared__ double sm[];  // sized on the host for the largest window (stitch_smem_bytes)
    if ((int)blockIdx.x < P.n_win) {  // the longest single-block chain goes first in the grid
        const int w = P.win_base + blockIdx.x;
        frame_threshold_and_energy<kStThreads>(P, P.wins[w], w, reinterpret_cast<unsigned *>(sm));
        return;
    }
    const int pair = P.pair_base + blockIdx.x - P.n_win;
    const int w = P.pair_win[pair];
    if (P.stop && P.pass > P.stop[w]) return;  // window left the GN loop: its records stay as they are
    const WinDev &W = P.wins[w];
    const int N = W.N, D = W.D, aidx = pair - W.pair_base, h = aidx % N, t = aidx / N;
    const int tid = threadIdx.x;
    if (h == t) return;
    if (!P.accumulate) return;
    (void)D;
    double *rec = P.stage + W.stage_base + (size_t)aidx * stage_rec(N);

    // All global loads of both halves are issued first (one round trip for the block): the
    // Top bucket partial sums and pair adjoints, and the SC rows of G_i with the host's adjoints.
    const bool do_top = true, do_sc = true;
    double *acc = sm, *A = acc + 96, *AH = A + 169, *AT = AH + 64, *TH = AT + 64, *TT = TH + 64;  // 521
    const int i = h, j = t, KP = W.KP, nt = KP / 4, per = W.ntiles * 16, Kc = 8 * (N - 1);
    const int sj = j < i ? j : j - 1;
    double *Gj = sm + kStTopLds;           // [8][KP]: rows 8 sj.. of G_i
    double *AHk = Gj + 8 * KP;             // [N-1][64] AH_ik
    double *ATk = AHk + (N - 1) * 64;      // [N-1][64] AT_ik
    double *X = ATk + (N - 1) * 64;        // [N-1][64]
    double *Sk = X + (N - 1) * 64;         // [N-1][64]
    double *Cc = Sk + (N - 1) * 64;        // [4][5]: G_i[Kc+r][Kc+c], bc
    const double *Ah = AH, *At = AT;       // AH_ij, AT_ij are the Top pair's adjoints
    {
        const int2 pi = P.pair_items[pair];
        if (tid < kTopVals) {
            if (do_top) {
            const float *src = P.top_slab + (size_t)pi.x * kTopVals + tid;
            double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
            int k = 0;
            for (; k + 4 <= pi.y; k += 4) {  // 4 independent loads in flight
                s0 += (double)src[(size_t)k * kTopVals];
                s1 += (double)src[(size_t)(k + 1) * kTopVals];
                s2 += (double)src[(size_t)(k + 2) * kTopVals];
                s3 += (double)src[(size_t)(k + 3) * kTopVals];
            }
            for (; k < pi.y; k++) s0 += (double)src[(size_t)k * kTopVals];
            acc[tid] = (s0 + s1) + (s2 + s3);
            }
        } else if (tid < kTopVals + 64) {
            AH[tid - kTopVals] = P.adH[(size_t)pair * 64 + tid - kTopVals];
        } else if (tid < kTopVals + 128) {
            AT[tid - kTopVals - 64] = P.adT[(size_t)pair * 64 + tid - kTopVals - 64];
        }
        const int2 hi = P.host_items[W.frame_base + i];
        const float *slab = P.sc_slab + W.sc_slab_base + (size_t)(hi.x - W.sc_item_base) * per;
        for (int e = do_sc ? tid : 8 * KP; e < 8 * KP; e += kStThreads) {
            const int r = e / KP, col = e % KP;
            Gj[e] = col < Kc + 5 ? g_elem(slab, hi.y, per, nt, 8 * sj + r, col) : 0.0;
        }
        if (do_sc && sj == 0 && tid < 20) {  // accHcc / accbc once per host (AccumulatedSCHessian.cc:105-113)
            const int r = tid / 5, c = tid % 5;
            Cc[tid] = g_elem(slab, hi.y, per, nt, Kc + r, Kc + c);
        }
        for (int e = do_sc ? tid : (N - 1) * 64; e < (N - 1) * 64; e += kStThreads) {
            const int s = e >> 6, k = s + (s >= i), pik = W.pair_base + i + N * k;
            AHk[e] = P.adH[(size_t)pik * 64 + (e & 63)];
            ATk[e] = P.adT[(size_t)pik * 64 + (e & 63)];
        }
    }
    __syncthreads();

    // ---------------- Top: bucket (h, t) ------------------------------------------------
    if (tid < 169) A[tid] = acc[top_slot(tid / 13, tid % 13)];
    __syncthreads();
    if (tid < 128) {
        const int l = tid & 63, r = l >> 3, c = l & 7;
        const double *Ad = tid < 64 ? AH : AT;
        double sacc = 0;
        for (int k = 0; k < 8; k++) sacc += Ad[r * 8 + k] * A[(4 + k) * 13 + 4 + c];
        (tid < 64 ? TH : TT)[l] = sacc;
    }
    __syncthreads();
    if (tid < 192) {
        const int which = tid >> 6, l = tid & 63, r = l >> 3, c = l & 7;
        double v = 0;
        if (which == 0) {  // H(h,h) += AH A AH^T
            for (int k = 0; k < 8; k++) v += TH[r * 8 + k] * AH[c * 8 + k];
            rec[kT1 + l] = v;
        } else if (which == 1) {  // H(t,t) += AT A AT^T
            for (int k = 0; k < 8; k++) v += TT[r * 8 + k] * AT[c * 8 + k];
            rec[kT2 + l] = v;
        } else {  // H(h,t) += AH A AT^T; the (t,h) term is its transpose (symmetrisation)
            for (int k = 0; k < 8; k++) v += TH[r * 8 + k] * AT[c * 8 + k];
            rec[kT3 + l] = v;
        }
    } else {  // 64 threads: H(h,c) = AH A_8C and H(t,c) = AT A_8C
        const int l = tid - 192, which = l >> 5, rr = (l & 31) >> 2, cc = l & 3;
        const double *Ad = which == 0 ? AH : AT;
        double v = 0;
        for (int k = 0; k < 8; k++) v += Ad[rr * 8 + k] * A[(4 + k) * 13 + cc];
        rec[(which == 0 ? kT4a : kT4b) + rr * 4 + cc] = v;
    }
    if (tid < 16) {
        rec[kT5 + tid] = A[(tid >> 2) * 13 + (tid & 3)];
    } else if (tid < 32) {
        const int l = tid - 16, which = l >> 3, r = l & 7;
        const double *Ad = which == 0 ? AH : AT;
        double v = 0;
        for (int k = 0; k < 8; k++) v += Ad[r * 8 + k] * A[(4 + k) * 13 + 12];
        rec[(which == 0 ? kT6a : kT6b) + r] = v;
    } else if (tid < 36) {
        rec[kT7 + tid - 32] = A[(tid - 32) * 13 + 12];
    }

    // ---------------- SC: host i = h, target j = t ---------------------------------------
    // per k != i: X_k = AT_ij D_jk, S_k = D_jk AH_ik^T
    for (int e = tid; e < (N - 1) * 64; e += kStThreads) {
        const int s = e >> 6, r = (e >> 3) & 7, c = e & 7;
        const double *Dm = Gj + 8 * s;  // D_jk[r][c] = Gj[r * KP + 8 s + c]
        double x = 0, sv = 0;
        for (int q = 0; q < 8; q++) {
            x += At[r * 8 + q] * Dm[q * KP + c];
            sv += Dm[r * KP + q] * AHk[s * 64 + c * 8 + q];
        }
        X[e] = x;
        Sk[e] = sv;
    }
    __syncthreads();
    // H(j,k) += AT_ij D_jk AT_ik^T (k_stitch_sum keeps the upper-triangle ones)
    for (int e = tid; e < (N - 1) * 64; e += kStThreads) {
        const int s = e >> 6, r = (e >> 3) & 7, c = e & 7;
        double v = 0;
        for (int q = 0; q < 8; q++) v += X[s * 64 + r * 8 + q] * ATk[s * 64 + c * 8 + q];
        rec[kS1 + e] = v;
    }
    const int s2 = st_S2(N);
    if (tid < 64) {
        const int r = tid >> 3, c = tid & 7;
        double hji = 0, hii = 0;
        for (int q = 0; q < 8; q++) {
            double sq = 0;  // S = sum_k S_k, fixed order
            for (int s = 0; s < N - 1; s++) sq += Sk[s * 64 + q * 8 + c];
            hji += At[r * 8 + q] * sq;
            hii += Ah[r * 8 + q] * sq;
        }
        rec[s2 + tid] = hji;       // H(j,i) += sum_k AT_ij D AH_ik^T
        rec[s2 + 64 + tid] = hii;  // H(i,i)
    } else if (tid < 128) {  // H(i,c) += AH_ij E, H(j,c) += AT_ij E
        const int l = tid - 64, which = l >> 5, rr = (l & 31) >> 2, cc = l & 3;
        const double *Ad = which == 0 ? Ah : At;
        double v = 0;
        for (int q = 0; q < 8; q++) v += Ad[rr * 8 + q] * Gj[q * KP + Kc + cc];
        rec[s2 + 128 + which * 32 + rr * 4 + cc] = v;
    } else if (tid < 144) {  // b(i) += AH_ij EB, b(j) += AT_ij EB
        const int l = tid - 128, which = l >> 3, rr = l & 7;
        const double *Ad = which == 0 ? Ah : At;
        double v = 0;
        for (int q = 0; q < 8; q++) v += Ad[rr * 8 + q] * Gj[q * KP + Kc + 4];
        rec[s2 + 192 + which * 8 + rr] = v;
    } else if (sj == 0 && tid < 164) {  // H_cc += accHcc, b_c += accbc (once per host)
        rec[s2 + 208 + tid - 144] = Cc[tid - 144];
    }
}

// Sum of every stitch term of one packed output element, in one fixed order over the window's
// pairs (t major, h minor): HA / bA from the Top records, Hsc / bsc from the SC records.  One
// thread per element of {HA upper, bA, Hsc upper, bsc} of every window; writes every element
// (no memset, no atomics: the stitched system is bitwise repeatable).  Each element's terms
// form one of five closed-form sequences (below), so the k-th term's record offset is a formula
// and the loads go out eight at a time instead of one per visited pair.
enum StitchSeq : int {
    kSeqAll = 0,    // every pair (h, t), h != t, one record index
    kSeqScCal = 1,  // the pairs (h, first target of h): (1..N-1, 0), then (0, 1)
    kSeqAB = 2,     // (f, t) for t < f [A], (h, f) for h != f [B], (f, t) for t > f [A]
    kSeqHaOff = 3,  // (f2, f1) then (f1, f2): H(h,t) of the two orientations
    kSeqScOff = 4   // (h, f1) for h != f1 (S2 term at h = f2, S1 otherwise), then (f1, f2)
};
struct StitchTerms {
    int seq, N, f, f2, idxA, idxB, s1rc, s2;  // s1rc >= 0: B index = kS1 + (F - (F > h)) * 64 + s1rc
    int r, c;
    __device__ int count() const {
        switch (seq) {
        case kSeqAll: return N * (N - 1);
        case kSeqScCal: return N;
        case kSeqAB: return 2 * (N - 1);
        case kSeqHaOff: return 2;
        default: return N;
        }
    }
    __device__ long long offset(int k, int R) const {
        int h, t, idx;
        switch (seq) {
        case kSeqAll: {
            t = k / (N - 1);
            const int hh = k - t * (N - 1);
            h = hh < t ? hh : hh + 1;
            idx = idxA;
            break;
        }
        case kSeqScCal:
            h = k < N - 1 ? k + 1 : 0;
            t = k < N - 1 ? 0 : 1;
            idx = idxA;
            break;
        case kSeqAB:
            if (k < f) {
                h = f;
                t = k;
                idx = idxA;
            } else if (k - f < N - 1) {
                const int kk = k - f;
                h = kk < f ? kk : kk + 1;
                t = f;
                idx = s1rc >= 0 ? kS1 + (f - (f > h ? 1 : 0)) * 64 + s1rc : idxB;
            } else {
                h = f;
                t = f + 1 + (k - f - (N - 1));
                idx = idxA;
            }
            break;
        case kSeqHaOff:
            h = k == 0 ? f2 : f;
            t = k == 0 ? f : f2;
            idx = k == 0 ? kT3 + c * 8 + r : kT3 + r * 8 + c;
            break;
        default:  // kSeqScOff, f = f1
            if (k < N - 1) {
                h = k < f ? k : k + 1;
                t = f;
                idx = h == f2 ? s2 + r * 8 + c : kS1 + (f2 - (f2 > h ? 1 : 0)) * 64 + r * 8 + c;
            } else {
                h = f;
                t = f2;
                idx = s2 + c * 8 + r;
            }
            break;
        }
        return (long long)(h + N * t) * R + idx;
    }
};
__global__ __launch_bounds__(256) void k_stitch_sum(const WinDev *__restrict__ wins, const int2 *__restrict__ blocks,
                                                     const double *__restrict__ stage, double *sys) {
    const int2 bw = blocks[blockIdx.x];  // {window, first element of this block}
    const WinDev &W = wins[bw.x];
    const int N = W.N, D = W.D;
    const long long pl = packed_len(D), n_el = 2 * (pl + D);
    const long long e = (long long)bw.y + threadIdx.x;
    if (e >= n_el) return;
    const int R = stage_rec(N), s2 = st_S2(N);
    const double *st = stage + W.stage_base;
    const bool sc = e >= pl + D;
    const long long q = sc ? e - (pl + D) : e;
    StitchTerms T;
    T.N = N;
    T.s2 = s2;
    T.s1rc = -1;
    T.f = T.f2 = T.r = T.c = 0;
    T.idxA = T.idxB = 0;
    if (q >= pl) {  // b element
        const int r = (int)(q - pl);
        if (r < 4) {
            T.seq = sc ? kSeqScCal : kSeqAll;
            T.idxA = sc ? s2 + 208 + r * 5 + 4 : kT7 + r;
        } else {
            const int rr = (r - 4) & 7;
            T.seq = kSeqAB;
            T.f = (r - 4) >> 3;
            T.idxA = (sc ? s2 + 192 : kT6a) + rr;
            T.idxB = (sc ? s2 + 200 : kT6b) + rr;
        }
    } else {  // upper element (row, col) of the packed triangle
        int row = (int)((2 * D + 1 - sqrt((double)(2 * D + 1) * (2 * D + 1) - 8.0 * (double)q)) * 0.5);
        row = row < 0 ? 0 : (row > D - 1 ? D - 1 : row);
        while (row < D - 1 && pk_index(row + 1, row + 1, D) <= q) row++;
        while (row > 0 && pk_index(row, row, D) > q) row--;
        const int col = row + (int)(q - pk_index(row, row, D));
        if (col < 4) {  // calibration block (row <= col < 4)
            T.seq = sc ? kSeqScCal : kSeqAll;
            T.idxA = sc ? s2 + 208 + row * 5 + col : kT5 + row * 4 + col;
        } else if (row < 4) {  // (calib cc = row, frame f, rr)
            const int rr = (col - 4) & 7, cc = row;
            T.seq = kSeqAB;
            T.f = (col - 4) >> 3;
            T.idxA = (sc ? s2 + 128 : kT4a) + rr * 4 + cc;
            T.idxB = (sc ? s2 + 160 : kT4b) + rr * 4 + cc;
        } else {
            const int f1 = (row - 4) >> 3, r = (row - 4) & 7, f2 = (col - 4) >> 3, c = (col - 4) & 7;
            T.r = r;
            T.c = c;
            if (f1 == f2) {
                T.seq = kSeqAB;
                T.f = f1;
                if (!sc) {
                    T.idxA = kT1 + r * 8 + c;  // h == f1
                    T.idxB = kT2 + r * 8 + c;  // t == f1
                } else {
                    T.idxA = s2 + 64 + r * 8 + c;  // i == f1: H(i,i)
                    T.s1rc = r * 8 + c;             // j == f1: H(j,j) from S1
                }
            } else {
                T.seq = sc ? kSeqScOff : kSeqHaOff;
                T.f = f1;
                T.f2 = f2;
            }
        }
    }
    const int cnt = T.count();
    double v = 0;
    constexpr int kBatch = 24;  // the 42-term calibration sums in two round trips
    for (int k0 = 0; k0 < cnt; k0 += kBatch) {
        double x[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; u++) x[u] = st[k0 + u < cnt ? T.offset(k0 + u, R) : 0];
#pragma unroll
        for (int u = 0; u < kBatch; u++)
            if (k0 + u < cnt) v += x[u];
    }
    sys[W.sys_base + e] = v;
}

// ============================================================================================
// k_stitch_host + k_stitch_host_sum (the default for windows of up to kHostStitchMaxN keyframes):
// one 256-thread block per host frame i of every window stitches everything host i owns --
// the Top pairs (i, t) (AccumulatedTopHessian.cc:213-239) and host i's Schur complement
// (AccumulatedSCHessian.cc:80-114, its targets j, k) -- into a dense packed partial system
// {HA, bA, Hsc, bsc} of the window, and k_stitch_host_sum adds the N partials of every element in
// host order (no atomics: the system is bitwise repeatable).  The terms are k_stitch's, grouped
// by host instead of by pair:
//   HA  (f,f): f == i: sum_t AH_it A_t AH_it^T; else AT_if A_f AT_if^T
//       (f1<f2): f1 == i: AH_i,f2 A AT_i,f2^T; f2 == i: (AH_i,f1 A AT_i,f1^T)^T; else 0
//       (c,f): f == i: sum_t AH_it A_t[8C]; else AT_if A_f[8C]    b(f) likewise, (c,c) / b(c): sum_t
//   Hsc (f,f): f == i: sum_j AH_ij S_j; else AT_if D_ff AT_if^T   with S_j = sum_k D_jk AH_ik^T
//       (f1<f2): i not in {f1,f2}: AT_i,f1 D_f1f2 AT_i,f2^T; f2 == i: AT_i,f1 S_f1; f1 == i: (AT_i,f2 S_f2)^T
//       (c,f) / b(f): f == i: sum_j AH_ij E_j / EB_j; else AT_if E_f / EB_f;  (c,c) / b(c): accHcc / accbc
// where A_t is pair (i,t)'s 13x13 AccumulatorApprox block and D, E, EB, accHcc, accbc the blocks of
// G_i = U^T diag(HdiF) U (k_point_sc's chunk partials summed in double).  Everything host i
// reads is staged in LDS once: G_i (both triangles), the adjoints of the N pairs (i, k), the
// N-1 Top accumulators; then X_jk = AT_ij D_jk (j <= k), S_j, TH_t = AH_it A_t, TT_t = AT_it A_t;
// then every element of the partial.  Windows with more keyframes use k_stitch's records.
// ============================================================================================
constexpr int kHostStitchMaxN = 11;
constexpr int kHsThreads = 512;
// the 8x8 blocks in LDS: row r at hs_row(r) (rows 4..7 shifted by two doubles), blocks kHsB = 72
// doubles apart, so the rows {0, 2, 4, 6} a 2x2 task group reads, in a block and in its
// neighbour, fall on distinct bank quads of ds_read_b128's 16-lane groups (dense 8x8 blocks put
// rows r and r + 4, and neighbouring blocks, on the same banks).  Rows r0, r0 + 1 (r0 even) stay
// 8 doubles apart.
constexpr int kHsB = 72;
__device__ __forceinline__ int hs_row(int r) { return 8 * r + ((r & 4) >> 1); }
__host__ __device__ inline int hs_k5(int N) { return 8 * (N - 1) + 5; }
__host__ __device__ inline int hs_ldg(int N) { return (hs_k5(N) + 1) & ~1; }  // even: 16-byte aligned rows
__host__ __device__ inline int hs_npair(int N) { return (N - 1) * N / 2; }
__host__ __device__ inline size_t hs_lds_doubles(int N) {
    return (size_t)hs_k5(N) * hs_ldg(N) + 2 * kHsB * (size_t)N + 182 * (size_t)N + kHsB * (size_t)hs_npair(N) +
           3 * kHsB * (size_t)N + 208 * (size_t)(N - 1);
}
// tile index t of the upper-tile order (a <= b) over nt tile rows -> (a, b)
__device__ __forceinline__ void tile_ab(int t, int nt, int &a, int &b) {
    int r = 0;
    while (t >= nt - r) {
        t -= nt - r;
        r++;
    }
    a = r;
    b = r + t;
}
// the (r, c) of top-partial slot s (the inverse of top_slot, r <= c)
__device__ __forceinline__ void top_slot_rc(int s, int &r, int &c) {
    if (s < 55) {  // Data[]: upper row-major 10x10
        int a = 0;
        while (s >= 10 - a) {
            s -= 10 - a;
            a++;
        }
        r = a;
        c = a + s;
    } else if (s < 85) {  // TopRight 10x3
        r = (s - 55) / 3;
        c = 10 + (s - 55) % 3;
    } else {  // BotRight: (0,0) (0,1) (0,2) (1,1) (1,2) (2,2)
        const int b = s - 85;
        r = 10 + (b < 3 ? 0 : b < 5 ? 1 : 2);
        c = 10 + (b < 3 ? b : b < 5 ? b - 2 : 2);
    }
}
// v[a][b] += sum_q L_a[q] R_b[q] (a, b in {0, 1}): two q-contiguous, 16-byte aligned 8-double
// rows of each operand; each element's 8 products summed in q order, then added to v
__device__ __forceinline__ void mm22(const double *L0, const double *L1, const double *R0, const double *R1,
                                     double (&v)[2][2]) {
    double l[2][8], r[2][8];
#pragma unroll
    for (int q = 0; q < 8; q += 2) {
        const double2 a0 = *reinterpret_cast<const double2 *>(L0 + q), a1 = *reinterpret_cast<const double2 *>(L1 + q);
        const double2 b0 = *reinterpret_cast<const double2 *>(R0 + q), b1 = *reinterpret_cast<const double2 *>(R1 + q);
        l[0][q] = a0.x;
        l[0][q + 1] = a0.y;
        l[1][q] = a1.x;
        l[1][q + 1] = a1.y;
        r[0][q] = b0.x;
        r[0][q + 1] = b0.y;
        r[1][q] = b1.x;
        r[1][q + 1] = b1.y;
    }
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) {
            double t = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) t += l[a][q] * r[b][q];
            v[a][b] += t;
        }
}
__global__ __launch_bounds__(kHsThreads) void k_stitch_host(StitchParams P) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    if ((int)blockIdx.x < P.n_win) {  // setNewFrameEnergyTH + the energy sum, as k_stitch
        const int w = P.win_base + blockIdx.x;
        frame_threshold_and_energy<kHsThreads>(P, P.wins[w], w, reinterpret_cast<unsigned *>(sm));
        return;
    }
    if (!P.accumulate) return;
    // one block per host, or (hs_split: grids that fit the GPU at once, e.g. one window) two: the
    // Top half (HA, bA) and the Schur complement (Hsc, bsc) of the host's partial
    const int hb = blockIdx.x - P.n_win;
    const int fr = P.frame_base + (P.hs_split ? hb >> 1 : hb);
    const bool do_top = !P.hs_split || (hb & 1) == 0, do_sc = !P.hs_split || (hb & 1) == 1;
    const int w = P.frame_win[fr];
    if (P.stop && P.pass > P.stop[w]) return;  // window left the GN loop: its partials stay as they are
    const WinDev &W = P.wins[w];
    const int N = W.N, D = W.D, i = fr - W.frame_base, tid = threadIdx.x;
    const int Kc = 8 * (N - 1), K5 = Kc + 5, ldg = hs_ldg(N), nt = W.KP / 4, per = W.ntiles * 16;
    const int Nm1 = N - 1, npair = hs_npair(N);
    // LDS (every region an even number of doubles: 16-byte aligned rows for the b128 reads)
    double *Gd = sm;                     // [K5][ldg] G_i, both triangles
    double *AH = Gd + (size_t)K5 * ldg;  // [N][8][8] adH of pair (i, k)
    double *AT = AH + kHsB * N;          // [N][8][8] adT of pair (i, k)
    double *A14 = AT + kHsB * N;         // [N][13][14] pair (i, t)'s 13x13 Top block (t == i unused)
    double *X = A14 + 182 * N;           // [npair][8][8] X_jk = AT_ij D_jk, target slots sj <= sk
    double *SSt = X + kHsB * npair;      // [N][8][8] S_j^T, S_j = sum_k D_jk AH_ik^T
    double *TH = SSt + kHsB * N;         // [N][8][8] AH_it A_t(88)
    double *TT = TH + kHsB * N;          // [N][8][8] AT_it A_t(88)
    double *HP = TT + kHsB * N;          // [2 parts][16 2x2s][N-1][4] the (i,i) block's per-term 2x2s
    double *CP = HP + 128 * (N - 1);     // [2 parts][40 items][N-1] the (calib, i) / b(i) per-term dots
    auto frame_of = [&](int slot) { return slot < i ? slot : slot + 1; };
    auto A_t = [&](int t, int r, int c) { return A14[182 * t + 14 * r + c]; };
    // ---- every load of the block in one round trip -------------------------------------
    {
        // G_i: each float4 of the host's chunk partials is one row of a 4x4 tile; summed over the
        // chunks in order (four in flight), then written to both triangles
        const int2 hi = P.host_items[W.frame_base + i];
        const float4 *slab = reinterpret_cast<const float4 *>(P.sc_slab + W.sc_slab_base +
                                                              (size_t)(hi.x - W.sc_item_base) * per);
        const int per4 = per / 4;
        for (int q = tid; q < (do_sc ? per4 : 0); q += kHsThreads) {
            double s[4] = {0, 0, 0, 0};
            int k = 0;
            for (; k + 4 <= hi.y; k += 4) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) v[u] = slab[(size_t)(k + u) * per4 + q];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    s[0] += (double)v[u].x;
                    s[1] += (double)v[u].y;
                    s[2] += (double)v[u].z;
                    s[3] += (double)v[u].w;
                }
            }
            for (; k < hi.y; k++) {
                const float4 v = slab[(size_t)k * per4 + q];
                s[0] += (double)v.x;
                s[1] += (double)v.y;
                s[2] += (double)v.z;
                s[3] += (double)v.w;
            }
            int a, b;
            tile_ab(q >> 2, nt, a, b);
            const int row = 4 * a + (q & 3);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int col = 4 * b + u;
                if (row < K5 && col < K5 && row <= col) {
                    Gd[row * ldg + col] = s[u];
                    Gd[col * ldg + row] = s[u];
                }
            }
        }
        // the adjoints of the pairs (i, k), k = 0..N-1
        for (int e = tid; e < 64 * N; e += kHsThreads) {
            const size_t pk = (size_t)(W.pair_base + i + N * (e >> 6)) * 64 + (e & 63);
            const int eb = kHsB * (e >> 6) + hs_row((e >> 3) & 7) + (e & 7);
            AH[eb] = P.adH[pk];
            AT[eb] = P.adT[pk];
        }
        // Top accumulators of the pairs (i, t): 24 float4 per item, summed over the pair's items
        for (int e = tid; e < (do_top ? 24 * Nm1 : 0); e += kHsThreads) {
            const int t = frame_of(e / 24), q = e % 24;
            const int2 pi = P.pair_items[W.pair_base + i + N * t];
            const float4 *src = reinterpret_cast<const float4 *>(P.top_slab + (size_t)pi.x * kTopVals) + q;
            double s[4] = {0, 0, 0, 0};
            int k = 0;
            for (; k + 4 <= pi.y; k += 4) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) v[u] = src[(size_t)(k + u) * (kTopVals / 4)];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    s[0] += (double)v[u].x;
                    s[1] += (double)v[u].y;
                    s[2] += (double)v[u].z;
                    s[3] += (double)v[u].w;
                }
            }
            for (; k < pi.y; k++) {
                const float4 v = src[(size_t)k * (kTopVals / 4)];
                s[0] += (double)v.x;
                s[1] += (double)v.y;
                s[2] += (double)v.z;
                s[3] += (double)v.w;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {  // both triangles of the 13x13 block (slots 91..95: padding)
                if (4 * q + u >= 91) continue;
                int r, c;
                top_slot_rc(4 * q + u, r, c);
                A14[182 * t + 14 * r + c] = s[u];
                A14[182 * t + 14 * c + r] = s[u];
            }
        }
    }
    __syncthreads();
    // ---- intermediates, 2x2 per thread, 16 threads per 8x8 block: S_j^T (N-1 blocks of N-1
    // terms each, first), X_jk (sj <= sk), TH_t, TT_t ---------------------------------------
    {
        const int n_ss = do_sc ? Nm1 : 0, n_x = do_sc ? npair : 0, n_th = do_top ? Nm1 : 0;
        const int total = 16 * (n_ss + n_x + 2 * n_th);
        for (int u = tid; u < total; u += kHsThreads) {
            int blk = u >> 4;
            const int r0 = 2 * ((u & 15) >> 2), c0 = 2 * (u & 3);
            double v[2][2] = {{0, 0}, {0, 0}};
            if (blk < n_ss) {  // S_j[r][c] = sum_k sum_q D_jk[r][q] AH_ik[c][q], k in slot order
                const int sj = blk, j = frame_of(sj);
                for (int sk = 0; sk < Nm1; sk++) {
                    const double *d = Gd + (size_t)(8 * sj + r0) * ldg + 8 * sk, *ah = AH + kHsB * frame_of(sk) + hs_row(c0);
                    mm22(d, d + ldg, ah, ah + 8, v);
                }
#pragma unroll
                for (int a = 0; a < 2; a++)
#pragma unroll
                    for (int b = 0; b < 2; b++) SSt[kHsB * j + hs_row(c0 + b) + r0 + a] = v[a][b];
                continue;
            }
            blk -= n_ss;
            if (blk < n_x) {  // X_jk[r][c] = sum_q AT_ij[r][q] D_jk[q][c], D_jk[q][c] = G[8sk+c][8sj+q]
                int sj = 0, rem = blk;
                while (rem >= Nm1 - sj) {
                    rem -= Nm1 - sj;
                    sj++;
                }
                const int sk = sj + rem;
                const double *at = AT + kHsB * frame_of(sj) + hs_row(r0), *d = Gd + (size_t)(8 * sk + c0) * ldg + 8 * sj;
                mm22(at, at + 8, d, d + ldg, v);
                double *o = X + kHsB * blk;
#pragma unroll
                for (int a = 0; a < 2; a++)
#pragma unroll
                    for (int b = 0; b < 2; b++) o[hs_row(r0 + a) + c0 + b] = v[a][b];
                continue;
            }
            blk -= n_x;  // TH_t / TT_t [r][c] = sum_k AH_it / AT_it [r][k] A_t(4+c, 4+k)
            const bool th = blk < n_th;
            const int t = frame_of(th ? blk : blk - n_th);
            const double *ad = (th ? AH : AT) + kHsB * t + hs_row(r0), *at = A14 + 182 * t + 14 * (4 + c0) + 4;
            mm22(ad, ad + 8, at, at + 14, v);
            double *o = (th ? TH : TT) + kHsB * t;
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int b = 0; b < 2; b++) o[hs_row(r0 + a) + c0 + b] = v[a][b];
        }
    }
    __syncthreads();
    // ---- host i's partial system: every packed element written (zeros included) ------------
    const long long pl = packed_len(D);
    double *HAp = P.stage + W.stage_base + (size_t)i * sys_len(D), *bAp = HAp + pl, *Hsp = bAp + D, *bsp = Hsp + pl;
    auto xblk = [&](int sj, int sk) { return X + kHsB * (sj * Nm1 - sj * (sj - 1) / 2 + (sk - sj)); };
    const int n_fb = 16 * (N * (N + 1) / 2), n_rest = 32 * N + 8 * N + 20, per_part = n_fb + n_rest;
    // The sums over t / j of the (i, i) block and of the (calib, i) / b(i) items are split into
    // one task per term (partials to HP / CP, summed after a barrier in the same order as one
    // task would: (0 + t_0) + t_1 + ...), so no thread carries N-1 terms of them alone.
    const int nH = 56 * Nm1, nparts = do_top + do_sc, pbase = do_top ? 0 : 1;
    for (int uh = tid; uh < nparts * nH; uh += kHsThreads) {
        const int part = pbase + uh / nH, hu = uh % nH;
        const bool top = part == 0;
        if (hu < 16 * Nm1) {  // (i, i) 2x2 sub-block `sub`, term st
            const int sub = hu / Nm1, st = hu % Nm1, r0 = 2 * (sub >> 2), c0 = 2 * (sub & 3);
            if (r0 > c0) continue;
            const int t = frame_of(st);
            const double *th = TH + kHsB * t + hs_row(r0), *ah = AH + kHsB * t, *ss = SSt + kHsB * t + hs_row(c0);
            double v[2][2] = {{0, 0}, {0, 0}};
            if (top)
                mm22(th, th + 8, ah + hs_row(c0), ah + hs_row(c0) + 8, v);
            else
                mm22(ah + hs_row(r0), ah + hs_row(r0) + 8, ss, ss + 8, v);
            double *o = HP + ((part * 16 + sub) * Nm1 + st) * 4;
            o[0] = v[0][0];
            o[1] = v[0][1];
            o[2] = v[1][0];
            o[3] = v[1][1];
        } else {  // (calib cc, frame i, rr) item < 32 / b(i)[rr] item >= 32, term st
            const int item = (hu - 16 * Nm1) / Nm1, st = (hu - 16 * Nm1) % Nm1;
            const int rr = item < 32 ? item >> 2 : item - 32, cI = item < 32 ? (item & 3) : 12, cS = item < 32 ? (item & 3) : 4;
            const int t = frame_of(st);
            double a = 0;
#pragma unroll
            for (int k = 0; k < 8; k++)
                a += AH[kHsB * t + hs_row(rr) + k] * (top ? A_t(t, 4 + k, cI) : Gd[(8 * st + k) * ldg + Kc + cS]);
            CP[(part * 40 + item) * Nm1 + st] = a;
        }
    }
    for (int uo = tid; uo < nparts * per_part; uo += kHsThreads) {
        const bool top = do_top && uo < per_part;  // the Top items first, then the SC ones
        const int u = uo - (do_top && !top ? per_part : 0);
        if (u < n_fb) {  // a 2x2 of frame block (f1 <= f2), upper-block order
            const int r0 = 2 * ((u & 15) >> 2), c0 = 2 * (u & 3);
            int f1 = 0, rem = u >> 4;
            while (rem >= N - f1) {
                rem -= N - f1;
                f1++;
            }
            const int f2 = f1 + rem;
            if (f1 == f2 && r0 > c0) continue;  // below the diagonal
            if (f1 == f2 && f1 == i) continue;  // the (i, i) block: per-term tasks above
            double v[2][2] = {{0, 0}, {0, 0}};
            if (f1 == f2) {
                const int f = f1, sf = f < i ? f : f - 1;
                const double *tt = TT + kHsB * f + hs_row(r0), *at = AT + kHsB * f + hs_row(c0);
                const double *x = top ? tt : xblk(sf, sf) + hs_row(r0);
                mm22(top ? tt : x, (top ? tt : x) + 8, at, at + 8, v);
            } else if (f1 == i) {
                const double *th = TH + kHsB * f2 + hs_row(r0), *at = AT + kHsB * f2 + hs_row(c0), *ss = SSt + kHsB * f2 + hs_row(r0);
                const double *l = top ? th : ss;  // (AT_i,f2 S_f2)^T on the SC side
                mm22(l, l + 8, at, at + 8, v);
            } else if (f2 == i) {
                const double *at = AT + kHsB * f1 + hs_row(r0), *th = TH + kHsB * f1 + hs_row(c0), *ss = SSt + kHsB * f1 + hs_row(c0);
                const double *rr = top ? th : ss;  // (AH A AT^T)^T of pair (i, f1) / AT_i,f1 S_f1
                mm22(at, at + 8, rr, rr + 8, v);
            } else if (!top) {
                const int s1 = f1 < i ? f1 : f1 - 1, s2 = f2 < i ? f2 : f2 - 1;
                const double *x = xblk(s1, s2) + hs_row(r0), *at = AT + kHsB * f2 + hs_row(c0);
                mm22(x, x + 8, at, at + 8, v);
            }
            double *o = top ? HAp : Hsp;
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int b = 0; b < 2; b++) {
                    if (f1 == f2 && r0 + a > c0 + b) continue;
                    o[pk_index(4 + 8 * f1 + r0 + a, 4 + 8 * f2 + c0 + b, D)] = v[a][b];
                }
            continue;
        }
        const int l0 = u - n_fb;
        double ha = 0;  // this part's value: HA / bA (top) or Hsc / bsc
        long long q;
        bool bvec = false;
        if (l0 < 32 * N) {  // (calib cc, frame f, rr)
            const int f = l0 >> 5, rr = (l0 >> 2) & 7, cc = l0 & 3;
            if (f == i) continue;  // per-term tasks above
            {
                const int sf = f < i ? f : f - 1;
#pragma unroll
                for (int k = 0; k < 8; k++)
                    ha += AT[kHsB * f + hs_row(rr) + k] * (top ? A_t(f, 4 + k, cc) : Gd[(8 * sf + k) * ldg + Kc + cc]);
            }
            q = pk_index(cc, 4 + 8 * f + rr, D);
        } else if (l0 < 40 * N) {  // b(f)[rr]
            const int f = (l0 - 32 * N) >> 3, rr = l0 & 7;
            if (f == i) continue;  // per-term tasks above
            {
                const int sf = f < i ? f : f - 1;
#pragma unroll
                for (int k = 0; k < 8; k++)
                    ha += AT[kHsB * f + hs_row(rr) + k] * (top ? A_t(f, 4 + k, 12) : Gd[(8 * sf + k) * ldg + Kc + 4]);
            }
            q = 4 + 8 * f + rr;
            bvec = true;
        } else {  // the calibration block (16, upper used) and b(calib) (4)
            const int l = l0 - 40 * N;
            const int r = l < 16 ? l >> 2 : l - 16, cI = l < 16 ? (l & 3) : 12, cS = l < 16 ? (l & 3) : 4;
            if (l < 16 && r > cI) continue;
            if (top)
                for (int st = 0; st < Nm1; st++) ha += A_t(frame_of(st), r, cI);
            else
                ha = Gd[(Kc + r) * ldg + Kc + cS];
            bvec = l >= 16;
            q = bvec ? r : pk_index(r, cI, D);
        }
        (bvec ? (top ? bAp : bsp) : (top ? HAp : Hsp))[q] = ha;
    }
    __syncthreads();
    for (int uf = tid; uf < nparts * 56; uf += kHsThreads) {  // the split sums, terms in order
        const int part = pbase + uf / 56, fu = uf % 56;
        const bool top = part == 0;
        if (fu < 16) {
            const int r0 = 2 * (fu >> 2), c0 = 2 * (fu & 3);
            if (r0 > c0) continue;
            double v[4] = {0, 0, 0, 0};
            for (int st = 0; st < Nm1; st++) {
                const double *hp = HP + ((part * 16 + fu) * Nm1 + st) * 4;
#pragma unroll
                for (int e = 0; e < 4; e++) v[e] += hp[e];
            }
            double *o = top ? HAp : Hsp;
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int b = 0; b < 2; b++) {
                    if (r0 + a > c0 + b) continue;
                    o[pk_index(4 + 8 * i + r0 + a, 4 + 8 * i + c0 + b, D)] = v[2 * a + b];
                }
        } else {
            const int item = fu - 16, rr = item < 32 ? item >> 2 : item - 32, cc = item & 3;
            double ha = 0;
            for (int st = 0; st < Nm1; st++) ha += CP[(part * 40 + item) * Nm1 + st];
            if (item < 32)
                (top ? HAp : Hsp)[pk_index(cc, 4 + 8 * i + rr, D)] = ha;
            else
                (top ? bAp : bsp)[4 + 8 * i + rr] = ha;
        }
    }
}
// sys = sum over the window's hosts of their partials, in host order, one thread per element
__global__ __launch_bounds__(256) void k_stitch_host_sum(const WinDev *__restrict__ wins,
                                                          const int2 *__restrict__ blocks,
                                                          const double *__restrict__ stage, double *sys) {
    const int2 bw = blocks[blockIdx.x];  // {window, first element of this block}
    const WinDev &W = wins[bw.x];
    const long long n_el = sys_len(W.D), e = (long long)bw.y + threadIdx.x;
    if (e >= n_el) return;
    const double *p = stage + W.stage_base + e;
    double x[kHostStitchMaxN];
#pragma unroll
    for (int h = 0; h < kHostStitchMaxN; h++) x[h] = p[(size_t)min(h, W.N - 1) * n_el];
    double v = 0;
#pragma unroll
    for (int h = 0; h < kHostStitchMaxN; h++)
        if (h < W.N) v += x[h];
    sys[W.sys_base + e] = v;
}

// ============================================================================================
// k_solve: EnergyFunctional::solveSystemF on the GPU, one workgroup of 4 wavefronts per window
// (SURVEY §8f row 1).  Statement for statement the host solver (host_math.cpp solve_system:
// assembly with the FIX_LAMBDA damping, Jacobi scaling, lower-triangle LDL^T with diagonal
// pivoting, column substitutions, orthogonalize); every element sees the host's operations in
// the host's order, so x is bit-identical to ldso_ba_solve's.  H lives in LDS (n <= kSolveMaxDim).
// ============================================================================================
constexpr int kSolveMaxDim = 8 * 11 + 4;  // windows up to 11 keyframes (68 KB of LDS for H)
#ifndef LDSO_SOLVE_THREADS
#define LDSO_SOLVE_THREADS 256
#endif
constexpr int kSolveThreads = LDSO_SOLVE_THREADS;  // wavefronts share the assembly and the LDL^T updates
// Round-robin (circle method) schedule of the 7 x 7 Jacobi sweep: 7 rounds of 3 disjoint pairs
// (p < q); player r sits out round r.  Shared with host_math.cpp's project_out.
__device__ constexpr int kJacobiRounds[7][3][2] = {
    {{1, 6}, {2, 5}, {3, 4}}, {{0, 2}, {3, 6}, {4, 5}}, {{1, 3}, {0, 4}, {5, 6}}, {{2, 4}, {1, 5}, {0, 6}},
    {{3, 5}, {2, 6}, {0, 1}}, {{4, 6}, {0, 3}, {1, 2}}, {{0, 5}, {1, 4}, {2, 3}}};
constexpr int kXadStride = LDSO_BA_MAX_FRAMES * LDSO_BA_MAX_FRAMES * 8 + 4;  // floats per window
// xAd[N*h + t] = x_h^T adHostF[h + N t] + x_t^T adTargetF[h + N t] in float (EnergyFunctional.cc:
// 624-632), then x_c: the statements of the host path of ldso_ba_resubstitute, over threads
// tid, tid + nthreads, ... of one window
__device__ __forceinline__ void xad_fill(const WinDev &W, const double *xw, const double *__restrict__ adH,
                                         const double *__restrict__ adT, float *o, int tid, int nthreads) {
#pragma clang fp contract(off)
    const int N = W.N;
    for (int e = tid; e < N * N * 8; e += nthreads) {
        const int cc = e & 7, ht = e >> 3, h = ht / N, t = ht % N;
        const double *AH = adH + (size_t)(W.pair_base + h + N * t) * 64, *AT = adT + (size_t)(W.pair_base + h + N * t) * 64;
        float s1 = 0, s2 = 0;
        for (int k = 0; k < 8; k++) s1 += (float)xw[4 + 8 * h + k] * (float)AH[k * 8 + cc];
        for (int k = 0; k < 8; k++) s2 += (float)xw[4 + 8 * t + k] * (float)AT[k * 8 + cc];
        o[(size_t)(N * h + t) * 8 + cc] = s1 + s2;
    }
    if (tid < 4) o[(size_t)N * N * 8 + tid] = (float)xw[tid];
}
// xad_fill with the adjoint columns of item tid loaded at kernel start (their load latency hides
// behind the factorisation); items tid + nthreads, ... as xad_fill
struct XadPre {
    float ah[8], at[8];
    __device__ void load(const WinDev &W, const double *__restrict__ adH, const double *__restrict__ adT, int tid) {
        const int N = W.N, e = min(tid, N * N * 8 - 1), cc = e & 7, ht = e >> 3, h = ht / N, t = ht % N;
        const double *AH = adH + (size_t)(W.pair_base + h + N * t) * 64, *AT = adT + (size_t)(W.pair_base + h + N * t) * 64;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            ah[k] = (float)AH[k * 8 + cc];
            at[k] = (float)AT[k * 8 + cc];
        }
    }
    __device__ void fill(const WinDev &W, const double *xw, const double *__restrict__ adH,
                         const double *__restrict__ adT, float *o, int tid, int nthreads) const {
#pragma clang fp contract(off)
        const int N = W.N;
        if (tid < N * N * 8) {
            const int cc = tid & 7, ht = tid >> 3, h = ht / N, t = ht % N;
            float s1 = 0, s2 = 0;
            for (int k = 0; k < 8; k++) s1 += (float)xw[4 + 8 * h + k] * ah[k];
            for (int k = 0; k < 8; k++) s2 += (float)xw[4 + 8 * t + k] * at[k];
            o[(size_t)(N * h + t) * 8 + cc] = s1 + s2;
        }
        for (int e = tid + nthreads; e < N * N * 8; e += nthreads) {
            const int cc = e & 7, ht = e >> 3, h = ht / N, t = ht % N;
            const double *AH = adH + (size_t)(W.pair_base + h + N * t) * 64, *AT = adT + (size_t)(W.pair_base + h + N * t) * 64;
            float s1 = 0, s2 = 0;
            for (int k = 0; k < 8; k++) s1 += (float)xw[4 + 8 * h + k] * (float)AH[k * 8 + cc];
            for (int k = 0; k < 8; k++) s2 += (float)xw[4 + 8 * t + k] * (float)AT[k * 8 + cc];
            o[(size_t)(N * h + t) * 8 + cc] = s1 + s2;
        }
        if (tid < 4) o[(size_t)N * N * 8 + tid] = (float)xw[tid];
    }
};

struct SolveParams {
    const WinDev *__restrict__ wins;
    const double *__restrict__ sys;
    const double *__restrict__ prior;  // [vec][2]: HL diagonal, bL
    const double *__restrict__ ns;     // [win][7][n] nullspaces (iteration >= 2)
    double *x;                         // [vec]
    const double *adH, *adT;           // k_solve_reg with xad non-null: also the resubstitution's
    float *xad;                        // xAd from the solution (k_xad fused)
    const double *prep_nm, *prep_g;    // k_ortho_prep's results: Nm [vec][n_null], per window G | G^-1 | fast
    int iteration, n_null;
    int *stop, *status;  // ldso_ba_optimize: windows with iteration >= stop skip; a NaN x marks the window lost
    // ldso_ba_optimize without a communicator (k_solve_fast): blocks [n_win, 2 n_win) compute the
    // sumNID / numID of the step that follows (nid_chain) over the idepths this solve's system was
    // linearised at -- a chain of ~P dependent float adds that fits inside the solve's own time
    double *win_nid;
    NidSrc nid_src;
    int n_win, nid_chunk;
};
constexpr int kPrepGStride = 192;  // doubles per window in prep_g: G [49], G^-1 [49], fast flag, V [49], ev [7], keep [7]
// H's row stride in LDS: odd (in doubles), so a column walk touches 32 distinct bank pairs
__host__ __device__ inline int solve_ld(int n) { return n | 1; }
__host__ __device__ inline size_t solve_smem_bytes(int n) {
    return ((size_t)n * solve_ld(n) + 7 * (size_t)n + 9 * (size_t)n + 7 * 7 * 3 + 64) * sizeof(double) +
           ((size_t)n + 1) * sizeof(int) + kSolveThreads * sizeof(double);
}

// wave-wide maximum of a 64-bit key, broadcast to every lane: inclusive max-scan within each
// row of 16 (row_shr 1/2/4/8), then row_bcast15 / row_bcast31 carry rows 0-2 into lane 63.
// Keys >= 0 with 0 as identity; every lane of the wave must be active.
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long x) {
#define LDSO_DPP_MAX(CTRL, ROWS)                                                                  \
    {                                                                                             \
        const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)x, CTRL, ROWS, 0xF, true); \
        const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(x >> 32), CTRL, ROWS, 0xF, true); \
        const unsigned long long o = ((unsigned long long)hi << 32) | lo;                         \
        x = o > x ? o : x;                                                                        \
    }
    LDSO_DPP_MAX(0x111, 0xF)
    LDSO_DPP_MAX(0x112, 0xF)
    LDSO_DPP_MAX(0x114, 0xF)
    LDSO_DPP_MAX(0x118, 0xF)
    LDSO_DPP_MAX(0x142, 0xA)
    LDSO_DPP_MAX(0x143, 0xC)
#undef LDSO_DPP_MAX
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)x, 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(x >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// |v| as an order-preserving key; NaN never wins (the host's '>' never selects one)
__device__ __forceinline__ unsigned long long abs_key(double v) {
    const double a = fabs(v);
    return a == a ? (unsigned long long)__double_as_longlong(a) : 0ull;
}

// LDS layout shared by both solve kernels (doubles unless noted)
struct SolveLds {
    double *H, *b, *sc, *y, *col, *Nm, *lr, *G, *V, *Gi, *misc;
    int *perm;
    __device__ SolveLds(double *lds, int n) {
        H = lds;                  // [n][ld] row-major (the host's [n][n]); lower triangle used
        b = H + (size_t)n * solve_ld(n);
        sc = b + n;
        y = sc + n;
        col = y + n;
        Nm = col + n;             // [n][7]
        lr = Nm + 7 * (size_t)n;  // [n]
        G = lr + n;
        V = G + 49;
        Gi = V + 49;              // (N^T N)^-1 of the fast projection path
        misc = Gi + 49;           // ntx[7], fast flag, coef[7], rd
        perm = reinterpret_cast<int *>(misc + 16);
    }
};

// ---- assembly (EnergyFunctional.cc:342-378), every thread of the block, each element in the
// host's order of operations: H = (HL + 0) + HA, diagonal *= (1 + lambda), H -= Hsc * scl,
// mirror, H(i,j) *= s_i s_j.  Every global load is issued up front (one memory round trip):
// the packed upper elements f = tid + kThreads u, and for row tid < n its diagonal, prior and
// b terms; the Jacobi scale of row tid from its diagonal, a barrier, then every element
// straight into its scaled lower position (c, r) (products of two scales commute exactly).
// Ends with a block barrier.
template <int kThreads>
__device__ __forceinline__ void solve_assemble(const SolveParams &P, const WinDev &W, const SolveLds &S, int tid) {
#pragma clang fp contract(off)
    const int n = W.D, ld = solve_ld(n);
    const long long pl = packed_len(n);
    const double *HA = P.sys + W.sys_base, *bA = HA + pl, *Hs = HA + pl + n, *bs = HA + 2 * pl + n;
    const double lambda = 1e-5;  // SOLVER_FIX_LAMBDA
    const double scl = 1.0f / (1 + lambda);
    auto element = [&](bool diag, double prior, double ha, double hs) {
        double h = ((diag ? prior : 0.0) + 0.0) + ha;
        if (diag) h *= (1 + lambda);
        return h - hs * scl;
    };
    constexpr int kPer = (int)((kSolveMaxDim * (kSolveMaxDim + 1) / 2 + kThreads - 1) / kThreads);
    static_assert(kSolveMaxDim <= kThreads, "one row per thread for the diagonal terms");
    // element u of this thread: f = tid + kThreads u in the "folded" order of the packed upper
    // triangle (row p paired with row n-1-p: n/2 rows of n+1 elements, n = 8N+4 is even), decoded
    // without loops; then unconditional loads at clamped positions (a guarded load becomes a
    // branch with its own wait)
    const int np1 = n + 1;
    const float inv = 1.0f / (float)np1;
    int rr[kPer], cc[kPer];
    double ha[kPer], hs[kPer];
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const int f = min(tid + kThreads * u, (int)pl - 1);
        int p = (int)((float)f * inv);
        p = p * np1 > f ? p - 1 : ((p + 1) * np1 <= f ? p + 1 : p);
        const int o = f - p * np1;
        const bool first = o < n - p;
        const int r = first ? p : n - 1 - p;
        rr[u] = r;
        cc[u] = first ? p + o : r + (o - (n - p));
        const int q = r * (2 * n - r + 1) / 2 + (cc[u] - r);  // pk_index(r, c, n)
        ha[u] = HA[q];
        hs[u] = Hs[q];
    }
    const int tr = min(tid, n - 1);
    const long long qd = pk_index(tr, tr, n);
    const double dha = HA[qd], dhs = Hs[qd], dpr = P.prior[2 * (W.vec_base + tr)],
                 bpr = P.prior[2 * (W.vec_base + tr) + 1], ba = bA[tr], bsv = bs[tr];
    double sci = 0, hdiag = 0;
    if (tid < n) {
        hdiag = element(true, dpr, dha, dhs);
        sci = 1.0 / sqrt(hdiag + 10);
        S.sc[tid] = sci;
        S.perm[tid] = tid;
    }
    __syncthreads();
    if (tid < n) {
        S.b[tid] = (((bpr + 0.0) + ba) - bsv / (1 + lambda)) * sci;
        S.H[tid * ld + tid] = hdiag * (sci * sci);
    }
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const int f = tid + kThreads * u, r = rr[u], c = cc[u];
        if (f < pl && r != c) S.H[c * ld + r] = element(false, 0.0, ha[u], hs[u]) * (S.sc[c] * S.sc[r]);
    }
    __syncthreads();
}

// ---- orthogonalize (EnergyFunctional.cc:809-841), iteration >= 2: x -= N (N^T N)^+ N^T x.
// solve_ortho_prepare (one wavefront) does the x-independent half -- normalised nullspaces Nm,
// G = Nm^T Nm and, for 7 nullspaces, the fast path's G^-1 (gram_pinv7; misc[7] = 1 when it
// applies) -- so it can run beside the factorisation; raw: >= 7 n doubles of free LDS.
__device__ __forceinline__ void solve_ortho_prepare(const SolveParams &P, const WinDev &W, const SolveLds &S,
                                                    double *raw, int lane) {
#pragma clang fp contract(off)
    const int n = W.D, kk = P.n_null;
    double *Nm = S.Nm, *lr = S.lr, *G = S.G, *V = S.V;
    const double *ns = P.ns + (size_t)7 * W.vec_base;
    for (int e = lane; e < kk * n; e += 64) raw[e] = ns[e];  // raw nullspaces [kk][n], coalesced
    wave_lds_sync();
    if (lane < kk) {
        double s2 = 0;
#pragma unroll 1
        for (int i0 = 0; i0 < n; i0 += 4) {
            double p[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const double v = raw[lane * n + min(i0 + u, n - 1)];
                p[u] = v * v;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) s2 = i0 + u < n ? s2 + p[u] : s2;
        }
        lr[lane] = sqrt(s2);
    }
    wave_lds_sync();
    for (int e = lane; e < kk * n; e += 64) {
        const int i = e / kk, a = e - i * kk;
        Nm[e] = raw[a * n + i] / lr[a];
    }
    wave_lds_sync();
    if (lane < kk * kk) {
        const int a = lane / kk, c = lane % kk;
        double g = 0.0;
#pragma unroll 1
        for (int i0 = 0; i0 < n; i0 += 4) {
            double p[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int ic = min(i0 + u, n - 1);
                p[u] = Nm[(size_t)ic * kk + a] * Nm[(size_t)ic * kk + c];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) g = i0 + u < n ? g + p[u] : g;
        }
        G[lane] = g;
        V[lane] = a == c ? 1.0 : 0.0;
    }
    wave_lds_sync();
    bool fast = false;
    if (kk == 7) {  // every lane redundantly; lane 0 stores
        double g[7][7], gi[7][7];
#pragma unroll
        for (int r = 0; r < 7; r++)
#pragma unroll
            for (int q = 0; q < 7; q++) g[r][q] = G[r * 7 + q];
        fast = gram_pinv7(g, gi);
        if (lane == 0 && fast)
#pragma unroll
            for (int r = 0; r < 7; r++)
#pragma unroll
                for (int q = 0; q < 7; q++) S.Gi[r * 7 + q] = gi[r][q];
    }
    if (lane == 0) S.misc[7] = fast ? 1.0 : 0.0;
    if (!fast) {  // the round-robin Jacobi eigen-decomposition of host_math.cpp project_out (lane 0)
        if (lane == 0) {
            double g[7][7], v[7][7];
#pragma unroll
            for (int r = 0; r < 7; r++)
#pragma unroll
                for (int q = 0; q < 7; q++) {
                    g[r][q] = r < kk && q < kk ? G[r * kk + q] : 0.0;
                    v[r][q] = r == q ? 1.0 : 0.0;
                }
            for (int sweep = 0; sweep < 64; sweep++) {
                double off = 0;
                for (int p = 0; p < 7; p++)
                    for (int q = p + 1; q < 7; q++)
                        if (q < kk) off += g[p][q] * g[p][q];
                if (off < 1e-30) break;
                for (int rd = 0; rd < 7; rd++) {
                    double c[3], sn[3];
                    bool on[3];
                    for (int e = 0; e < 3; e++) {
                        const int p = kJacobiRounds[rd][e][0], q = kJacobiRounds[rd][e][1];
                        const double apq = g[p][q];
                        on[e] = q < kk && apq != 0;
                        const double th = (g[q][q] - g[p][p]) / (2 * apq);
                        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1));
                        c[e] = 1 / sqrt(t * t + 1);
                        sn[e] = t * c[e];
                    }
                    for (int e = 0; e < 3; e++) {  // column phase
                        const int p = kJacobiRounds[rd][e][0], q = kJacobiRounds[rd][e][1];
                        if (!on[e]) continue;
                        for (int r = 0; r < 7; r++) {
                            const double gp = g[r][p], gq = g[r][q];
                            g[r][p] = c[e] * gp - sn[e] * gq;
                            g[r][q] = sn[e] * gp + c[e] * gq;
                        }
                    }
                    for (int e = 0; e < 3; e++) {  // row phase, then V
                        const int p = kJacobiRounds[rd][e][0], q = kJacobiRounds[rd][e][1];
                        if (!on[e]) continue;
                        for (int r = 0; r < 7; r++) {
                            const double gp = g[p][r], gq = g[q][r];
                            g[p][r] = c[e] * gp - sn[e] * gq;
                            g[q][r] = sn[e] * gp + c[e] * gq;
                            const double vp = v[r][p], vq = v[r][q];
                            v[r][p] = c[e] * vp - sn[e] * vq;
                            v[r][q] = sn[e] * vp + c[e] * vq;
                        }
                    }
                }
            }
            double smax = 0;
            for (int e = 0; e < 7; e++)
                if (e < kk) smax = fmax(smax, sqrt(fmax(0.0, g[e][e])));
            for (int e = 0; e < 7; e++) {
                S.lr[e] = g[e][e];  // eigenvalue
                S.lr[7 + e] = e < kk && sqrt(fmax(0.0, g[e][e])) > kSolverModeDelta * smax ? 1.0 : 0.0;
                for (int a = 0; a < 7; a++) V[a * 7 + e] = v[a][e];
            }
        }
    }
    wave_lds_sync();
}

// k_ortho_prep runs solve_ortho_prepare once per nullspace upload (the nullspaces, hence Nm, G
// and G^-1, stay fixed over an optimize() call and usually over consecutive iterate calls); the
// solve kernels load the results with their assembly loads, every thread, before the assembly's
// barriers.
__device__ __forceinline__ void solve_ortho_load(const SolveParams &P, const WinDev &W, const SolveLds &S, int tid,
                                                 int nthreads) {
    if (P.iteration < 2 || P.n_null <= 0) return;
    const int n = W.D, kk = P.n_null;
    const double *nm = P.prep_nm + (size_t)7 * W.vec_base, *g = P.prep_g + (size_t)kPrepGStride * blockIdx.x;
    for (int e = tid; e < kk * n; e += nthreads) S.Nm[e] = nm[e];
    if (tid < 49) {
        S.G[tid] = g[tid];
        S.Gi[tid] = g[49 + tid];
        S.V[tid] = g[99 + tid];
    }
    if (tid < 14) S.lr[tid] = g[148 + tid];  // eigenvalues, kept modes (the Jacobi fallback)
    if (tid == 0) S.misc[7] = g[98];
}

// solve_ortho_load split in two for k_solve_fast: the loads into registers at kernel start (their
// round trip overlaps the assembly's), the LDS stores after the assembly (read only after the
// factorisation's barriers).  Thread tid holds Nm elements tid + k nthreads (k < 2: n <= 92, 7 n <=
// 2 x 512) and, below 49 / 14 / 1, its G / G^-1 / V, lr and fast-flag entries.
struct OrthoPre {
    double nm[2], g, gi, v, lr, fast;
    bool on;
    __device__ void load(const SolveParams &P, const WinDev &W, int tid, int nthreads) {
        on = P.iteration >= 2 && P.n_null > 0;
        if (!on) return;
        const int n = W.D, kk = P.n_null;
        const double *pnm = P.prep_nm + (size_t)7 * W.vec_base, *pg = P.prep_g + (size_t)kPrepGStride * blockIdx.x;
#pragma unroll
        for (int k = 0; k < 2; k++) nm[k] = pnm[min(tid + k * nthreads, kk * n - 1)];
        const int t49 = min(tid, 48), t14 = min(tid, 13);
        g = pg[t49];
        gi = pg[49 + t49];
        v = pg[99 + t49];
        lr = pg[148 + t14];
        fast = pg[98];
    }
    __device__ void store(const SolveParams &P, const WinDev &W, const SolveLds &S, int tid, int nthreads) const {
        if (!on) return;
        const int n = W.D, kk = P.n_null;
#pragma unroll
        for (int k = 0; k < 2; k++)
            if (tid + k * nthreads < kk * n) S.Nm[tid + k * nthreads] = nm[k];
        if (tid < 49) {
            S.G[tid] = g;
            S.Gi[tid] = gi;
            S.V[tid] = v;
        }
        if (tid < 14) S.lr[tid] = lr;
        if (tid == 0) S.misc[7] = fast;
    }
};

__global__ __launch_bounds__(64) void k_ortho_prep(SolveParams P, double *prep_nm, double *prep_g) {
    extern __shared__ double lds[];
    const WinDev W = P.wins[blockIdx.x];
    const int n = W.D, kk = P.n_null, lane = threadIdx.x;
    const SolveLds S(lds, n);
    double *raw = lds + (solve_smem_bytes(n) + 15) / 16 * 2;
    solve_ortho_prepare(P, W, S, raw, lane);  // ends with its results visible to the wave
    double *nm = prep_nm + (size_t)7 * W.vec_base, *g = prep_g + (size_t)kPrepGStride * blockIdx.x;
    for (int e = lane; e < kk * n; e += 64) nm[e] = S.Nm[e];
    if (lane < 49) {
        g[lane] = S.G[lane];
        g[49 + lane] = S.Gi[lane];
        g[99 + lane] = S.V[lane];
    }
    if (lane < 14) g[148 + lane] = S.lr[lane];
    if (lane == 0) g[98] = S.misc[7];
}

// the x-dependent half (one wavefront, after solve_ortho_load's results are visible): N^T y,
// coef = G^-1 N^T y (fast path) or the round-robin Jacobi pseudo-inverse of host_math.cpp
// project_out, y -= Nm coef; then x (= y) to global memory.
__device__ __forceinline__ void solve_ortho_apply_store(const SolveParams &P, const WinDev &W, const SolveLds &S,
                                                        int lane) {
#pragma clang fp contract(off)
    const int n = W.D;
    double *y = S.y, *Nm = S.Nm;
    const int kk = P.n_null;
    if (P.iteration >= 2 && kk > 0) {
        double *ntx = S.misc, *coef = S.misc + 8;
        if (lane < kk) {  // t += Nm(i, a) y(i) in row order; only the adds chain (no selects on it):
                          // blocks of 4 rows whose operands are loaded one block ahead, then the tail
            double t = 0.0;
            const int a = lane, nb = n >> 2;
            double cn[4], cy[4], nn[4], ny[4];
            auto ld4 = [&](int blk, double (&m)[4], double (&v)[4]) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    m[u] = Nm[(size_t)(4 * blk + u) * kk + a];
                    v[u] = y[4 * blk + u];
                }
            };
            if (nb > 0) ld4(0, cn, cy);
#pragma unroll 1
            for (int bk = 0; bk < nb; bk++) {
                ld4(min(bk + 1, nb - 1), nn, ny);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const double p = cn[u] * cy[u];
                    t += p;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    cn[u] = nn[u];
                    cy[u] = ny[u];
                }
            }
            for (int i = 4 * nb; i < n; i++) {
                const double p = Nm[(size_t)i * kk + a] * y[i];
                t += p;
            }
            ntx[lane] = t;
            coef[lane] = 0.0;
        }
        wave_lds_sync();
        if (kk == 7 && S.misc[7] != 0.0) {  // fast path: coef = G^-1 N^T y, one row per lane
            if (lane < 7) {
                double gr[7], nt[7];
#pragma unroll
                for (int b = 0; b < 7; b++) {
                    gr[b] = S.Gi[7 * lane + b];
                    nt[b] = ntx[b];
                }
                coef[lane] = gram_apply7_row(gr, nt);
            }
        } else {  // (NtN)^+ NtX from k_ortho_prep's eigen-decomposition (V, eigenvalues, kept modes)
            if (lane < kk) {
                const double *V = S.V, *ev = S.lr, *keep = S.lr + 7;
                double cf = 0, nt[7];
#pragma unroll
                for (int a = 0; a < 7; a++) nt[a] = a < kk ? ntx[a] : 0.0;
#pragma unroll
                for (int e = 0; e < 7; e++) {  // host_math.cpp project_out's accumulation, row `lane`
                    if (e >= kk || keep[e] == 0.0) continue;
                    double proj = 0;
#pragma unroll
                    for (int a = 0; a < 7; a++)
                        if (a < kk) proj += V[a * 7 + e] * nt[a];
                    cf += V[lane * 7 + e] * proj / ev[e];
                }
                coef[lane] = cf;
            }
        }
        wave_lds_sync();
        for (int i = lane; i < n; i += 64) {
            double t = 0;
#pragma unroll
            for (int a = 0; a < 7; a++) {
                const int ac = min(a, kk - 1);
                const double p = Nm[(size_t)i * kk + ac] * coef[ac];
                t = a < kk ? t + p : t;
            }
            y[i] -= t;
        }
        wave_lds_sync();
    }
    bool nan = false;
    for (int i = lane; i < n; i += 64) {
        P.x[W.vec_base + i] = y[i];
        nan |= isnan(y[i]);
    }
    // FullSystem::optimize (FullSystem.cc:907-911): isnan(lastX.norm()) -- a NaN element (inf
    // elements give an inf norm, not NaN) -- is isLost: no step in this iteration, the loop ends
    if (P.stop && __any(nan) && lane == 0) {
        P.stop[blockIdx.x] = P.iteration;
        P.status[blockIdx.x] = LDSO_BA_OPT_LOST;
    }
}

// The trailing update of step k is A(i,j) = fma(-(c_i c_j), 1/d, A(i,j)) with c = column k and
// d the pivot (host_math.cpp ldlt_solve states the same): symmetric in i and j, so a kernel may
// hold both triangles and update either copy; L(i,k) = c_i / d is the exact quotient.
__global__ __launch_bounds__(kSolveThreads) void k_solve(SolveParams P) {
#pragma clang fp contract(off)
    extern __shared__ double lds[];
    if (P.stop && P.iteration >= P.stop[blockIdx.x]) return;  // the window left the GN loop
    const WinDev W = P.wins[blockIdx.x];  // a register copy: the helpers would re-read global memory after every LDS store
    const int n = W.D, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ld = solve_ld(n);
    const SolveLds S(lds, n);
    double *H = S.H, *b = S.b, *sc = S.sc, *y = S.y, *col = S.col, *misc = S.misc;
    int *perm = S.perm;
    // one private dummy slot per thread: masked-off update elements land there (no branches)
    double *dummy = reinterpret_cast<double *>(perm + (n + 1) / 2 * 2) + tid;
    // Strictly-lower elements (i, j), j < i, ordered by column j descending: the elements LDL^T
    // step k updates (k < j < i) are exactly a prefix, so every step is element-parallel.  Wave w
    // lane l always owns the elements e = l + 64 (w + 4 t).  Column n-2-mm holds mm+1 elements
    // and starts at e = mm (mm + 1) / 2.  Entry: offset of (i, j) in H (16 bits) | i << 16 | j << 23.
    constexpr int kWaves = kSolveThreads / 64;
    constexpr int kOffRegs = ((kSolveMaxDim - 1) * kSolveMaxDim / 2 + 64 * kWaves - 1) / (64 * kWaves);
    int tri[kOffRegs];
    const int noff = n * (n - 1) / 2;
#pragma unroll
    for (int t = 0; t < kOffRegs; t++) {
        const int e = lane + 64 * (wave + kWaves * t);
        int mm = (int)((sqrtf(8.0f * e + 1.0f) - 1.0f) * 0.5f);
        if (mm * (mm + 1) / 2 > e) mm--;
        if ((mm + 1) * (mm + 2) / 2 <= e) mm++;
        const int j = n - 2 - mm, i = j + 1 + (e - mm * (mm + 1) / 2);
        tri[t] = e < noff ? ((i * ld + j) | (i << 16) | (j << 23)) : 0;  // padding: (0, 0), never stored
    }
    auto at = [&](int r, int c) -> double & { return H[r * ld + c]; };
    solve_ortho_load(P, W, S, tid, kSolveThreads);
    solve_assemble<kSolveThreads>(P, W, S, tid);
    // ---- LDL^T with symmetric diagonal pivoting (lower triangle).  Wave 0 runs the serial part
    // of each step (pivot, swap, column k) with the diagonal in its registers (lane i mod 64); all
    // waves then share the trailing update.
    double dg0 = lane < n ? at(lane, lane) : 0.0, dg1 = lane + 64 < n ? at(lane + 64, lane + 64) : 0.0;
    for (int k = 0; k < n; k++) {
        if (wave == 0) {
            // pivot = first index of the largest |diag| (the host's strict '>' scan from k: a NaN
            // never wins, except that a NaN at k itself keeps k)
            int piv;
            {
                const int i0 = lane, i1 = lane + 64;
                const bool c0 = i0 >= k && i0 < n, c1 = i1 >= k && i1 < n;
                const unsigned long long k0 = !c0 ? 0ull : (dg0 != dg0 && i0 == k) ? ~0ull : abs_key(dg0);
                const unsigned long long k1 = !c1 ? 0ull : (dg1 != dg1 && i1 == k) ? ~0ull : abs_key(dg1);
                const unsigned long long mx = wave_max_u64(k0 > k1 ? k0 : k1);
                const unsigned long long b0 = __ballot(c0 && k0 == mx);
                piv = b0 ? __builtin_ctzll(b0) : 64 + __builtin_ctzll(__ballot(c1 && k1 == mx));
            }
            // symmetric swap k <-> piv (lower triangle: (k,j)<->(piv,j) for j < k, (i,k)<->(piv,i)
            // for k < i < piv, (i,k)<->(i,piv) for i > piv, the two diagonals), fused with taking
            // column k: col = the new A(i,k), L(i,k) = col / d written back; the diagonal's share
            // of the trailing update happens here
            const double dk = readlane_f64(k < 64 ? dg0 : dg1, k & 63);
            const double d = readlane_f64(piv < 64 ? dg0 : dg1, piv & 63);
            const double rd = d != 0 ? 1.0 / d : 0.0;
            if (piv != k) {
                if (lane == (k & 63)) (k < 64 ? dg0 : dg1) = d;
                if (lane == (piv & 63)) (piv < 64 ? dg0 : dg1) = dk;
                for (int j = lane; j < k; j += 64) {
                    const double t = at(k, j), u = at(piv, j);
                    at(k, j) = u;
                    at(piv, j) = t;
                }
            }
#pragma unroll
            for (int sgm = 0; sgm < 2; sgm++) {
                const int i = lane + 64 * sgm;
                if (i <= k || i >= n) continue;
                double *own = &at(i, k);
                double *src = piv == k || i == piv ? own : (i < piv ? &at(piv, i) : &at(i, piv));
                const double old = *own, v = *src;
                *(src != own ? src : dummy) = old;
                col[i] = v;
                *own = d != 0 ? v / d : 0.0;
                double &dgi = sgm == 0 ? dg0 : dg1;
                dgi = fma(-(v * v), rd, dgi);
            }
            if (lane == 0) {
                misc[15] = rd;
                if (piv != k) {
                    const int pt = perm[k];
                    perm[k] = perm[piv];
                    perm[piv] = pt;
                }
            }
        }
        __syncthreads();
        const int m = (n - k - 2) * (n - k - 1) / 2;  // off-diagonal elements with k < j < i
        const double rd = misc[15];
        constexpr int kUpdBatch = 6;
#pragma unroll
        for (int t0 = 0; t0 < kOffRegs; t0 += kUpdBatch) {
            if (64 * (wave + kWaves * t0) >= m) continue;  // uniform per wave: chunks past the prefix
            double a[kUpdBatch], ci[kUpdBatch], cj[kUpdBatch], *dst[kUpdBatch];
#pragma unroll
            for (int u = 0; u < kUpdBatch; u++) {
                if (t0 + u >= kOffRegs) continue;
                const int x = tri[t0 + u], off = x & 0xFFFF, i = (x >> 16) & 0x7F, j = x >> 23;
                ci[u] = col[i];
                cj[u] = col[j];
                a[u] = H[off];
                dst[u] = lane + 64 * (wave + kWaves * (t0 + u)) < m ? H + off : dummy;
            }
#pragma unroll
            for (int u = 0; u < kUpdBatch; u++) {
                if (t0 + u >= kOffRegs) continue;
                *dst[u] = fma(-(ci[u] * cj[u]), rd, a[u]);
            }
        }
        __syncthreads();
    }
    if (wave != 0) return;  // the rest is one wavefront's work (wave-level synchronisation only)
    if (lane < n) at(lane, lane) = dg0;
    if (lane + 64 < n) at(lane + 64, lane + 64) = dg1;
    wave_lds_sync();
    // ---- substitutions (column by column, as the host); y[i] lives in lane i (mod 64); the
    // matrix entries of the next 4 columns are loaded ahead of the dependent chain
    const int ia = lane, ib = lane + 64, ra = min(ia, n - 1), rb = min(ib, n - 1);
    double ya = ia < n ? b[perm[ia]] : 0.0, yb = ib < n ? b[perm[ib]] : 0.0;
    constexpr int kSubAhead = 4;
    for (int j0 = 0; j0 < n; j0 += kSubAhead) {
        double fa[kSubAhead], fb[kSubAhead];
#pragma unroll
        for (int u = 0; u < kSubAhead; u++) {
            const int j = min(j0 + u, n - 1);
            fa[u] = at(ra, j);
            fb[u] = at(rb, j);
        }
#pragma unroll
        for (int u = 0; u < kSubAhead; u++) {
            const int j = j0 + u;
            if (j >= n) break;
            const double yj = j < 64 ? readlane_f64(ya, j) : readlane_f64(yb, j - 64);
            if (ia > j && ia < n) ya = fma(-fa[u], yj, ya);
            if (ib > j && ib < n) yb = fma(-fb[u], yj, yb);
        }
    }
    if (ia < n) ya = at(ia, ia) != 0 ? ya / at(ia, ia) : 0.0;
    if (ib < n) yb = at(ib, ib) != 0 ? yb / at(ib, ib) : 0.0;
    for (int j0 = n - 1; j0 >= 0; j0 -= kSubAhead) {
        double fa[kSubAhead], fb[kSubAhead];
#pragma unroll
        for (int u = 0; u < kSubAhead; u++) {
            const int j = max(j0 - u, 0);
            fa[u] = at(j, ra);
            fb[u] = at(j, rb);
        }
#pragma unroll
        for (int u = 0; u < kSubAhead; u++) {
            const int j = j0 - u;
            if (j < 0) break;
            const double yj = j < 64 ? readlane_f64(ya, j) : readlane_f64(yb, j - 64);
            if (ia < j) ya = fma(-fa[u], yj, ya);
            if (ib < j) yb = fma(-fb[u], yj, yb);
        }
    }
    if (ia < n) b[perm[ia]] = ya;
    if (ib < n) b[perm[ib]] = yb;
    wave_lds_sync();
    for (int i = lane; i < n; i += 64) y[i] = sc[i] * b[i];  // x
    wave_lds_sync();
    solve_ortho_apply_store(P, W, S, lane);
}

// ============================================================================================
// k_solve_reg: the same solve for windows of up to 7 keyframes (n <= 64), factorised out of
// registers by four wavefronts without block barriers.  Lane p of wave w holds H(p, q) for the
// 16 columns q = 16w .. 16w+15 of the scaled symmetric H (both triangles) and, in every wave,
// the diagonal of row p.  Pivoting is logical: rows never move, pos tracks the host's index of
// each physical row (the swap k <-> piv is bookkeeping), and every wave selects the pivot
// itself from its copy of the diagonal (the copies are bitwise equal).  The wave owning the
// pivot's column publishes it in LDS (one slot per step, then a ready flag; LDS requests of a
// wave are served in order, so a flag seen set means the column is there).  Look-ahead: right
// after a step's column arrives each wave updates the diagonal and picks the next pivot, and
// its owner updates and publishes that one column before its own trailing update, so the
// serial chain per step is read column -> diagonal -> pivot -> one fma -> publish; 1/d is
// computed off that chain.  Every element sees the host's operations in the host's order (the
// update is symmetric in i, j), so x stays bit-identical to ldso_ba_solve.
// A fifth wave prepares the nullspace projection, then follows the published columns: L(i,k)
// = c_i / d into Ls and the forward substitution step by step (the host's per-element order),
// then the diagonal, the backward substitution and the projection -- all in physical row order
// (b[perm[i]] = y_i makes the host's permutation disappear).
// ============================================================================================
constexpr int kSolveRegDim = 64;
constexpr int kSolveLsLd = 65;            // odd: a column walk of Ls is bank-conflict free
constexpr int kSolveRegThreads = 5 * 64;  // 4 factorisation waves + the substitution wave
__host__ __device__ inline size_t solve_reg_base(int n) { return (solve_smem_bytes(n) + 15) / 16 * 2; }  // doubles
__host__ __device__ inline size_t solve_reg_smem_bytes(int n) {
    return solve_reg_base(n) * sizeof(double) +
           ((size_t)kSolveRegDim * kSolveLsLd + kSolveRegDim * kSolveRegDim + kSolveRegDim + 7 * kSolveRegDim + 1) *
               sizeof(double) +
           2 * kSolveRegDim * sizeof(int);
}
struct RegLds {
    double *cb, *Ls, *Dv, *raw;  // cb: [step][64] published columns (16-byte aligned); Dv: d of step
    int *pv, *flag;              // pivot row and ready flag of each step
    __device__ RegLds(double *lds, int n) {
        cb = lds + solve_reg_base(n);
        Ls = cb + kSolveRegDim * kSolveRegDim;
        Dv = Ls + kSolveRegDim * kSolveLsLd;
        raw = Dv + kSolveRegDim;
        pv = reinterpret_cast<int *>(raw + 7 * kSolveRegDim + 1);
        flag = pv + kSolveRegDim;
    }
};
#define LDSO_COMPILER_FENCE() asm volatile("" ::: "memory")
// wave-wide maximum of a 32-bit key (0 = identity), broadcast: row_shr 1/2/4/8 within each row
// of 16, then row_bcast15 / row_bcast31 carry rows 0-2 into lane 63
__device__ __forceinline__ unsigned wave_max_u32(unsigned x) {
#define LDSO_DPP_MAX32(CTRL, ROWS)                                                                          \
    {                                                                                                       \
        const unsigned o = (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, true);         \
        x = o > x ? o : x;                                                                                  \
    }
    LDSO_DPP_MAX32(0x111, 0xF)
    LDSO_DPP_MAX32(0x112, 0xF)
    LDSO_DPP_MAX32(0x114, 0xF)
    LDSO_DPP_MAX32(0x118, 0xF)
    LDSO_DPP_MAX32(0x142, 0xA)
    LDSO_DPP_MAX32(0x143, 0xC)
#undef LDSO_DPP_MAX32
    return (unsigned)__builtin_amdgcn_readlane((int)x, 63);
}
// pivot of step k: the largest |diag| among the live rows, ties to the smallest host index; a
// NaN never wins, except at the host's row k itself, which then keeps k (the host's strict '>'
// scan from k).  The maximum of the order-preserving 64-bit keys: the high words by DPP first,
// the low words among high-word ties (an LDS atomic-max variant measured slower).
__device__ __forceinline__ int reg_pivot(double dg, unsigned long long act, int pos, int k, int lane) {
    const bool live = (act >> lane) & 1;
    const unsigned long long key = !live ? 0ull : (dg != dg && pos == k) ? ~0ull : abs_key(dg);
    const unsigned hi = (unsigned)(key >> 32), lo = (unsigned)key;
    const unsigned mh = wave_max_u32(hi);
    unsigned long long cand = __ballot(live && hi == mh);
    if (cand & (cand - 1)) {
        const bool c = (cand >> lane) & 1;
        const unsigned ml = wave_max_u32(c ? lo : 0u);
        cand = __ballot(c && lo == ml);
    }
    int piv = __builtin_ctzll(cand);
    if (cand & (cand - 1)) {  // exact tie: the smallest host index
        int best = __builtin_amdgcn_readlane(pos, piv);
        for (unsigned long long m = cand & (cand - 1); m; m &= m - 1) {
            const int l = __builtin_ctzll(m), pl = __builtin_amdgcn_readlane(pos, l);
            if (pl < best) {
                best = pl;
                piv = l;
            }
        }
    }
    return __builtin_amdgcn_readfirstlane(piv);
}
// column of step k, then its ready flag = pivot row + 1 (no wait: the LDS serves a wave's
// requests in order).  The pivot row's own entry of the column is d.
__device__ __forceinline__ void reg_publish(const RegLds &R, int k, int lane, double c, int piv) {
    R.cb[k * kSolveRegDim + lane] = c;
    LDSO_COMPILER_FENCE();
    if (lane == 0) __hip_atomic_store(R.flag + k, piv + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    LDSO_COMPILER_FENCE();
}
// poll the flag and the column together: a set flag read before the column read means the
// column read returns the published value; returns the pivot row
// A bounded wait: after ~2^22 polls (well over 100 ms) it gives up with a NaN column and row 0,
// so the kernel always drains even if a publication were ever missing (x then reads NaN).
template <bool kSleep = false>
__device__ __forceinline__ int reg_wait(const RegLds &R, int k, int lane, double &v) {
    int f;
    unsigned polls = 0;
    do {
        f = __hip_atomic_load(R.flag + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        LDSO_COMPILER_FENCE();
        v = R.cb[k * kSolveRegDim + lane];
        LDSO_COMPILER_FENCE();
        f = __builtin_amdgcn_readfirstlane(f);
        if (kSleep && f == 0) __builtin_amdgcn_s_sleep(2);
        if (f == 0 && ++polls > (1u << 22)) {
            v = __longlong_as_double(0x7ff8000000000000ll);
            return 0;
        }
    } while (f == 0);
    return f - 1;
}
// the factorisation waves of k_solve_reg: 16 columns of H in registers per wave
__device__ __forceinline__ void solve_reg_factor(const RegLds &R, const SolveLds &S, int n, int ld, int wave,
                                                 int lane) {
#pragma clang fp contract(off)
    typedef double d16 __attribute__((ext_vector_type(16)));
    d16 rv;
    const int q0 = 16 * wave;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int q = q0 + j, r = lane > q ? lane : q, c = lane > q ? q : lane;
        rv[j] = q < n && lane < n ? S.H[r * ld + c] : 0.0;
    }
    double dg = lane < n ? S.H[lane * ld + lane] : 0.0;
    int pos = lane;
    unsigned long long act = n >= 64 ? ~0ull : ((1ull << n) - 1);  // rows not yet pivoted
    int piv = reg_pivot(dg, act, pos, 0, lane);
    double d = readlane_f64(dg, piv);
    double cl = 0.0;
    if ((piv >> 4) == wave) {
        cl = rv[piv & 15];
        reg_publish(R, 0, lane, cl, piv);
    }
    double rd = d != 0 ? 1.0 / d : 0.0;
    for (int k = 0; k < n; k++) {
        if ((piv >> 4) != wave) (void)reg_wait(R, k, lane, cl);  // column k of the host: A(i, k) after the swap
        const int kphys = __builtin_ctzll(__ballot(((act >> lane) & 1) && pos == k));
        const int ppos = __builtin_amdgcn_readlane(pos, piv);
        pos = lane == piv ? k : (lane == kphys ? ppos : pos);
        act &= ~(1ull << piv);
        dg = fma(-(cl * cl), rd, dg);
        int nxt = 0;
        double cn = 0.0, rdn = 0.0;
        if (k + 1 < n) {
            nxt = reg_pivot(dg, act, pos, k + 1, lane);
            const double dn = readlane_f64(dg, nxt);
            if ((nxt >> 4) == wave) {  // look-ahead: the next pivot's column first
                cn = fma(-(cl * readlane_f64(cl, nxt)), rd, rv[nxt & 15]);
                reg_publish(R, k + 1, lane, cn, nxt);
            }
            rdn = dn != 0 ? 1.0 / dn : 0.0;
        }
        // trailing update of this wave's 16 columns, c_q broadcast from the published column
        // (dead columns too: never read again; the look-ahead column gets the same bits again)
        const double2 *cq2 = reinterpret_cast<const double2 *>(R.cb + k * kSolveRegDim + q0);
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const double2 cq = cq2[u];
            rv[2 * u] = fma(-(cl * cq.x), rd, rv[2 * u]);
            rv[2 * u + 1] = fma(-(cl * cq.y), rd, rv[2 * u + 1]);
        }
        piv = nxt;
        cl = cn;
        rd = rdn;
    }
}
__global__ __launch_bounds__(kSolveRegThreads) void k_solve_reg(SolveParams P) {
#pragma clang fp contract(off)
    extern __shared__ double lds[];
    if (P.stop && P.iteration >= P.stop[blockIdx.x]) return;  // the window left the GN loop
    const WinDev W = P.wins[blockIdx.x];  // a register copy (see k_solve)
    const int n = W.D, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ld = solve_ld(n);
    const SolveLds S(lds, n);
    const RegLds R(lds, n);
    for (int i = tid; i < kSolveRegDim; i += kSolveRegThreads) R.flag[i] = 0;
    solve_ortho_load(P, W, S, tid, kSolveRegThreads);
    solve_assemble<kSolveRegThreads>(P, W, S, tid);  // its barriers also publish the flags
    if (wave == 4) __builtin_amdgcn_s_setprio(0);  // the factorisation's chain first
    else __builtin_amdgcn_s_setprio(2);
    if (wave == 4) {
        // ---- the projection's x-independent half, then the substitutions (physical rows)
        double y = lane < n ? S.b[lane] : 0.0;
        unsigned long long act = n >= 64 ? ~0ull : ((1ull << n) - 1);
        for (int k = 0; k < n; k++) {  // forward: y_i = fma(-L(i,k), y_k, y_i), k ascending
            double cl;
            const int piv = reg_wait<true>(R, k, lane, cl);  // off the critical chain: poll gently
            const double d = readlane_f64(cl, piv);
            if (lane == 0) {
                R.Dv[k] = d;
                R.pv[k] = piv;
            }
            act &= ~(1ull << piv);
            const double yk = readlane_f64(y, piv);
            if ((act >> lane) & 1) {
                const double l = d != 0 ? cl / d : 0.0;
                R.Ls[k * kSolveLsLd + lane] = l;
                y = fma(-l, yk, y);
            }
        }
        // to the host's order: lane i takes y_i = y of physical row pv[i]; then the diagonal
        if (lane < n) S.col[lane] = y;
        wave_lds_sync();
        const int pvl = lane < n ? R.pv[lane] : 0;
        double yl = lane < n ? S.col[pvl] : 0.0;
        if (lane < n) {
            const double dd = R.Dv[lane];
            yl = dd != 0 ? yl / dd : 0.0;
        }
        // backward: y_i = fma(-L(j,i), y_j, y_i) for j descending, L(j,i) = Ls[i][pv[j]] (a
        // rolled loop: this code runs once, so its size is instruction fetches)
        const int me = min(lane, n - 1);
        constexpr int kSubAhead = 4;
#pragma unroll 1
        for (int j0 = n - 1; j0 >= 0; j0 -= kSubAhead) {
            double fa[kSubAhead];
#pragma unroll
            for (int u = 0; u < kSubAhead; u++)
                fa[u] = R.Ls[me * kSolveLsLd + __builtin_amdgcn_readlane(pvl, max(j0 - u, 0))];
#pragma unroll
            for (int u = 0; u < kSubAhead; u++) {
                const int j = j0 - u;
                if (j < 0) break;
                const double t = fma(-fa[u], readlane_f64(yl, j), yl);
                yl = lane < j ? t : yl;
            }
        }
        if (lane < n) S.b[pvl] = yl;  // b[perm[i]] = y_i
        wave_lds_sync();
        y = lane < n ? S.b[lane] : 0.0;
        if (lane < n) S.y[lane] = S.sc[lane] * y;  // x = s b, b[perm[i]] = y_i
        wave_lds_sync();
        solve_ortho_apply_store(P, W, S, lane);
    } else {
        solve_reg_factor(R, S, n, ld, wave, lane);
    }
    if (P.xad) {  // x is in S.y: the resubstitution's xAd by all five waves
        __syncthreads();
        xad_fill(W, S.y, P.adH, P.adT, P.xad + (size_t)blockIdx.x * kXadStride, tid, kSolveRegThreads);
    }
}

// ============================================================================================
// k_solve_fast: the same solveSystemF without pivoting (LDSO_BA_SOLVE_FAST, the default; windows
// up to 11 keyframes).  After solve_assemble the scaled matrix is symmetric positive definite
// (Jacobi-scaled HA + priors + lambda damping - Hsc / (1 + lambda)), so an unpivoted LDL^T is
// stable; dropping the pivot search removes the serial pivot reduction and the cross-wave
// hand-off of every step.  Blocked right-looking LDL^T in LDS: wave 0 factorises an 8-column
// panel out of registers (lane = row, the in-panel columns broadcast with readlane) together with
// the forward substitution, while the other waves apply the previous panel's rank-8 update to
// the trailing matrix (look-ahead, two barriers per panel).  Trailing elements see
// fma(-(c_i c_j), 1/d, A(i,j)) for the steps in ascending order, as the host solver, just without
// the row exchanges; in-panel ones fma(-c_i, c_j / d, A(i,j)); L(i,k) = c_i * (1/d).  Wave 0
// then runs the backward substitution and the projection (prepared by k_ortho_prep).  x differs from the pivoted
// solve (k_solve_reg / k_solve / ldso_ba_solve) only by rounding (tests: within the system's
// float sensitivity envelope; optimize energies within 1e-4).
// ============================================================================================
#ifndef LDSO_SOLVE_FAST_THREADS
#define LDSO_SOLVE_FAST_THREADS 512
#endif
constexpr int kSolveFastThreads = LDSO_SOLVE_FAST_THREADS;  // 8 waves: the trailing updates hide LDS latency
constexpr int kSolveFastPanel = 8;
__host__ __device__ inline size_t solve_fast_smem_bytes(int n) {
    // SolveLds | W [2][8][128] panel columns (double-buffered) | rd [2][8]
    return solve_smem_bytes(n) + 16 + 2 * ((size_t)kSolveFastPanel * 128 + kSolveFastPanel) * sizeof(double);
}
// row k's value of a lane-per-row register pair (rows lane, lane + 64)
template <int kH>
__device__ __forceinline__ double fast_row(const double *v, int k) {
    if constexpr (kH == 1)
        return readlane_f64(v[0], k);
    else
        return k < 64 ? readlane_f64(v[0], k) : readlane_f64(v[1], k - 64);
}
// Wave 0: LDL^T of panel columns p .. p+w-1 (rows lane + 64 h).  Lane i updates its rows' panel
// entries unconditionally -- entries above the diagonal and rows past n turn into finite junk that
// is never stored nor read -- so a step is one readlane pair, one product cj / d and one fma per
// later column and row half, with the h = 1 half compiled out for n <= 64.  Only what the pivot
// chain needs runs here: the step's column c and 1/d go to LDS (Wc, rdv), and the other waves
// write L(i, k) = c_i / d and d into H (fast_store_l) and run the forward substitution
// (fast_forward) from them while this wave factorises the next panel: the same statements, so the
// same bits as when this wave did both (round 6: 40 -> 25 instructions per pivot on the chain).
template <int kH>
__device__ __forceinline__ void fast_panel(double *H, double *Wc, double *rdv, int n, int ld, int p, int w, int lane) {
#pragma clang fp contract(off)
    double r[kSolveFastPanel][kH];
#pragma unroll
    for (int h = 0; h < kH; h++)
#pragma unroll
        for (int jj = 0; jj < kSolveFastPanel; jj++) {
            const int i = lane + 64 * h;
            r[jj][h] = i < n && jj < w && i >= p + jj ? H[i * ld + p + jj] : 0.0;
        }
#pragma unroll
    for (int kk = 0; kk < kSolveFastPanel; kk++) {
        if (kk >= w) break;
        const int k = p + kk;
        const double d = fast_row<kH>(r[kk], k);
        // 1/d: v_rcp_f64 and two Newton steps (the IEEE divide's 10-deep chain sits on every step)
        double rd = __builtin_amdgcn_rcp(d);
        rd = fma(rd, fma(-d, rd, 1.0), rd);
        rd = fma(rd, fma(-d, rd, 1.0), rd);
        rd = d != 0 ? rd : 0.0;
#pragma unroll
        for (int jj = kk + 1; jj < kSolveFastPanel; jj++) {
            const double wj = fast_row<kH>(r[kk], p + jj) * rd;  // A(j, k) / d; columns past n are junk
#pragma unroll
            for (int h = 0; h < kH; h++) r[jj][h] = fma(-r[kk][h], wj, r[jj][h]);
        }
#pragma unroll
        for (int h = 0; h < kH; h++) Wc[kk * 128 + lane + 64 * h] = r[kk][h];  // 128 rows a column
        rdv[kk] = rd;  // every lane the same value: no exec-mask branch
    }
}
// L(i, k) = c_i * (1/d) below the diagonal and d on it, for the w columns of panel p (columns c and
// 1/d from Wc / rdv), threads t, t + nth, ...; rows above the diagonal are never read
__device__ __forceinline__ void fast_store_l(double *H, const double *Wp, const double *rp, int n, int ld, int p,
                                             int w, int t, int nth) {
#pragma clang fp contract(off)
    for (int e = t; e < (n - p) * w; e += nth) {
        const int i = p + e / w, kk = e % w, k = p + kk;
        if (i >= k) H[i * ld + k] = i > k ? Wp[kk * 128 + i] * rp[kk] : Wp[kk * 128 + i];
    }
}
// the forward substitution L y = b over panel p's w columns (y in the calling wave's registers,
// rows lane, lane + 64): y_i = fma(-L(i, k), y_k, y_i) for k in order
template <int kH>
__device__ __forceinline__ void fast_forward(const double *Wp, const double *rp, double *y, int p, int w, int lane) {
#pragma clang fp contract(off)
    for (int kk = 0; kk < w; kk++) {
        const int k = p + kk;
        const double yk = fast_row<kH>(y, k), rd = rp[kk];
#pragma unroll
        for (int h = 0; h < kH; h++) {
            const int i = lane + 64 * h;
            const double l = i > k ? Wp[kk * 128 + i] * rd : 0.0;  // L(i,k) (rd = 0 for d = 0)
            y[h] = fma(-l, yk, y[h]);
        }
    }
}
// After the last panel (the wave holding y): D, L^T x = y (y in lanes i, i + 64), x = s y into S.y
template <int kH>
__device__ __forceinline__ void fast_back_subst(const double *H, const SolveLds &S, double *y, int n, int ld,
                                                int lane) {
#pragma clang fp contract(off)
    int ri[kH];
#pragma unroll
    for (int h = 0; h < kH; h++) {
        const int i = lane + 64 * h;
        ri[h] = min(i, n - 1);
        if (i < n) y[h] = H[i * ld + i] != 0 ? y[h] / H[i * ld + i] : 0.0;
    }
    constexpr int kSubAhead = 4;
    // the L columns of a block of kSubAhead steps, loaded one block ahead (H is read-only here)
    double f[kSubAhead][kH], fn[kSubAhead][kH];
    auto ldf = [&](int j0, double (&F)[kSubAhead][kH]) {
#pragma unroll
        for (int u = 0; u < kSubAhead; u++)
#pragma unroll
            for (int h = 0; h < kH; h++) F[u][h] = H[max(j0 - u, 0) * ld + ri[h]];
    };
    ldf(n - 1, f);
    for (int j0 = n - 1; j0 >= 0; j0 -= kSubAhead) {
        ldf(max(j0 - kSubAhead, 0), fn);
#pragma unroll
        for (int u = 0; u < kSubAhead; u++) {
            const int j = j0 - u;
            if (j < 0) break;
            const double yj = fast_row<kH>(y, j);
#pragma unroll
            for (int h = 0; h < kH; h++) {
                const int i = lane + 64 * h;
                if (i < j) y[h] = fma(-f[u][h], yj, y[h]);
            }
        }
#pragma unroll
        for (int u = 0; u < kSubAhead; u++)
#pragma unroll
            for (int h = 0; h < kH; h++) f[u][h] = fn[u][h];
    }
#pragma unroll
    for (int h = 0; h < kH; h++) {
        const int i = lane + 64 * h;
        if (i < n) S.y[i] = S.sc[i] * y[h];  // x = s y
    }
}
// panel (Wp, rp: its c columns and 1/d, w steps) applied to A(i, j), steps in order
__device__ __forceinline__ double fast_update(const double *Wp, const double *rp, int w, int i, int j, double a) {
#pragma clang fp contract(off)
    double wi[kSolveFastPanel], wj[kSolveFastPanel], rk[kSolveFastPanel];
#pragma unroll
    for (int kk = 0; kk < kSolveFastPanel; kk++) {  // every operand in flight before the chain
        wi[kk] = Wp[kk * 128 + i];
        wj[kk] = Wp[kk * 128 + j];
        rk[kk] = rp[kk];
    }
#pragma unroll
    for (int kk = 0; kk < kSolveFastPanel; kk++)
        if (kk < w) a = fma(-(wi[kk] * wj[kk]), rk[kk], a);
    return a;
}
__global__ __launch_bounds__(kSolveFastThreads) void k_solve_fast(SolveParams P) {
#pragma clang fp contract(off)
    extern __shared__ double lds[];
    if (P.win_nid && (int)blockIdx.x >= P.n_win) {  // doStepFromBackup's sumNID (FullSystem.cc:1899-1909)
        const int w = blockIdx.x - P.n_win;
        if (P.stop && P.iteration >= P.stop[w]) return;
        nid_chain(P.wins[w], P.nid_src, P.win_nid, w, reinterpret_cast<float *>(lds), P.nid_chunk);
        return;
    }
    static_assert(7 * kSolveMaxDim <= 2 * kSolveFastThreads, "OrthoPre: two Nm elements per thread");
    // the stop flag and the window's descriptor in one round trip, then the exit
    const int stop_it = P.stop ? P.stop[blockIdx.x] : INT_MAX;
    const WinDev W = P.wins[blockIdx.x];  // a register copy (see k_solve)
    if (P.iteration >= stop_it) return;  // the window left the GN loop
    const int n = W.D, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ld = solve_ld(n);
    const SolveLds S(lds, n);
    double *H = S.H;
    double *Wc = lds + (solve_smem_bytes(n) + 16) / sizeof(double);  // [2][8][128]: c of each panel step
    double *rdv = Wc + 2 * kSolveFastPanel * 128;                     // [2][8]: 1/d of each panel step
    XadPre xp;
    if (P.xad) xp.load(W, P.adH, P.adT, tid);
    OrthoPre op;
    op.load(P, W, tid, kSolveFastThreads);
    solve_assemble<kSolveFastThreads>(P, W, S, tid);
    op.store(P, W, S, tid, kSolveFastThreads);  // published by the factorisation's barriers
    double y[2] = {0.0, 0.0};  // wave 1: the forward substitution's y (rows lane, lane + 64)
    if (wave == 1) {
        y[0] = lane < n ? S.b[lane] : 0.0;
        y[1] = lane + 64 < n ? S.b[lane + 64] : 0.0;
    }
    auto panel = [&](int p, int w, int buf) {
        double *Wb = Wc + buf * kSolveFastPanel * 128, *rb = rdv + buf * kSolveFastPanel;
        if (n > 64)
            fast_panel<2>(H, Wb, rb, n, ld, p, w, lane);
        else
            fast_panel<1>(H, Wb, rb, n, ld, p, w, lane);
    };
    auto forward = [&](const double *Wp, const double *rp, int p, int w) {
        if (n > 64)
            fast_forward<2>(Wp, rp, y, p, w, lane);
        else
            fast_forward<1>(Wp, rp, y, p, w, lane);
    };
    // Blocked right-looking LDL^T with look-ahead: after panel p is factorised, all waves apply
    // it to the next panel's columns; then wave 0 factorises the next panel while the other
    // waves apply panel p to the rest of the trailing triangle (double-buffered panel columns).
    if (wave == 0) panel(0, min(kSolveFastPanel, n), 0);
    __syncthreads();
    int p = 0, buf = 0;
    for (; p + kSolveFastPanel < n; p += kSolveFastPanel, buf ^= 1) {
        const int w = kSolveFastPanel, m0 = p + w, w1 = min(kSolveFastPanel, n - m0), m1 = m0 + w1;
        const double *Wp = Wc + buf * kSolveFastPanel * 128, *rp = rdv + buf * kSolveFastPanel;
        for (int e = tid; e < (n - m0) * w1; e += kSolveFastThreads) {  // the next panel's columns
            const int i = m0 + e / w1, j = m0 + e % w1;
            if (i >= j) H[i * ld + j] = fast_update(Wp, rp, w, i, j, H[i * ld + j]);
        }
        __syncthreads();
        if (wave == 0) {
            panel(m0, w1, buf ^ 1);
        } else {  // panel p's forward substitution, the rest of the trailing triangle (m1 <= j <= i < n), L and d of panel p
            if (wave == 1) forward(Wp, rp, p, w);
            const int nt = n - m1, ne = nt * (nt + 1) / 2;
            for (int e = tid - 64; e < ne; e += kSolveFastThreads - 64) {
                int ii = (int)((sqrtf(8.0f * e + 1.0f) - 1.0f) * 0.5f);  // row ii of the nt x nt triangle
                if (ii * (ii + 1) / 2 > e) ii--;
                if ((ii + 1) * (ii + 2) / 2 <= e) ii++;
                const int i = m1 + ii, j = m1 + (e - ii * (ii + 1) / 2);
                H[i * ld + j] = fast_update(Wp, rp, w, i, j, H[i * ld + j]);
            }
            fast_store_l(H, Wp, rp, n, ld, p, w, tid - 64, kSolveFastThreads - 64);
        }
        __syncthreads();
    }
    {  // the last panel (p, buffer buf): its forward substitution and L, then the backward one
        const double *Wl = Wc + buf * kSolveFastPanel * 128, *rl = rdv + buf * kSolveFastPanel;
        const int wl = n - p;
        if (wave == 1) forward(Wl, rl, p, wl);
        fast_store_l(H, Wl, rl, n, ld, p, wl, tid, kSolveFastThreads);
    }
    __syncthreads();
    if (wave == 1) {
        if (n > 64)
            fast_back_subst<2>(H, S, y, n, ld, lane);
        else
            fast_back_subst<1>(H, S, y, n, ld, lane);
    }
    __syncthreads();
    if (wave == 0) solve_ortho_apply_store(P, W, S, lane);
    if (P.xad) {  // x is in S.y: the resubstitution's xAd by all waves
        __syncthreads();
        xp.fill(W, S.y, P.adH, P.adT, P.xad + (size_t)blockIdx.x * kXadStride, tid, kSolveFastThreads);
    }
}

// ============================================================================================
// k_resubstitute: EnergyFunctional::resubstituteFPt (EnergyFunctional.cc:638-667)
// ============================================================================================
// ---- sharded setNewFrameEnergyTH ---------------------------------------
// With points sharded over ranks, the newest frame's NewEnergyWithOutlier values are spread
// over the ranks; nth_element needs all of them.  Each rank exports its newest-frame segment
// of every window into a fixed-stride slot (padding -1, which the selection skips), the host
// all-gathers the slots, and k_frame_th reruns the exact selection over all ranks' values.
// slot of window w (pitch `slot` floats): the newest-frame energies [0, stride) (padding -1), then,
// with prun > 0, the rank's |idepth| run of the window in device point order [stride, stride +
// prun) (padding 0) -- the sharded sumNID chain's input (NidSrc)
__global__ __launch_bounds__(256) void k_export_newest(const WinDev *__restrict__ wins, const float *__restrict__ e_wo,
                                                       float *out, long long stride, long long slot,
                                                       const float *__restrict__ pt_data, int prun) {
    const WinDev &W = wins[blockIdx.y];
    const int n = W.newest_end - W.newest_begin;
    float *dst = out + (size_t)blockIdx.y * slot;
    for (long long i = blockIdx.x * 256 + threadIdx.x; i < stride; i += (long long)gridDim.x * 256)
        dst[i] = i < n ? e_wo[W.newest_begin + i] : -1.0f;
    for (long long i = blockIdx.x * 256 + threadIdx.x; i < prun; i += (long long)gridDim.x * 256)
        dst[stride + i] = i < W.P ? fabsf(pt_data[(size_t)(W.point_base + i) * LDSO_BA_POINT_STRIDE + 2]) : 0.0f;
}

// blocks [0, n_win): the exact setNewFrameEnergyTH over every rank's slot; with nid.gathered, blocks
// [n_win, 2 n_win) the windows' sumNID chains over the gathered runs (ldso_ba_optimize, exact solve modes)
__global__ __launch_bounds__(kStThreads) void k_frame_th(const WinDev *__restrict__ wins, const float *__restrict__ buf,
                                                         int n_ranks, int n_win, long long stride, long long slot,
                                                         float *frame_th, NidSrc nid, double *win_nid,
                                                         const int *stop, int pass) {
    __shared__ unsigned keys[kThMaxLds + th_fixed_bytes(kStThreads) / sizeof(unsigned)];
    if ((int)blockIdx.x >= n_win) {
        const int w = blockIdx.x - n_win;
        if (stop && pass > stop[w]) return;
        nid_chain(wins[w], nid, win_nid, w, reinterpret_cast<float *>(keys), kThMaxLds);
        return;
    }
    const int w = blockIdx.x;
    const WinDev &W = wins[w];
    const long long n_cand = (long long)n_ranks * stride;
    select_frame_th<kStThreads>(
        [&](int i) {
            const int r = (int)(i / stride);
            return buf[((size_t)r * n_win + w) * slot + (i - (long long)r * stride)];
        },
        (int)n_cand, keys, kThMaxLds, frame_th + W.frame_base + W.N - 1);
}

struct ResubParams {
    const float *__restrict__ xad;   // [win][kXadStride]: xAd[h*N + t][8], then x_c[4]
    const WinDev *__restrict__ wins;
    const int *__restrict__ pt_win;
    const int *__restrict__ pt_nres;
    const unsigned long long *__restrict__ pt_tgt;
    const float4 *__restrict__ rec_a;     // the pass's records (write_record)
    const float2 *__restrict__ rec_b;
    const float *__restrict__ geo_snap;   // [pairs][kGeoSnap]: the pass's centre geometry inputs
    const float *__restrict__ pt_geo;     // the point records (u, v)
    const float *__restrict__ pt_out;
    const int *__restrict__ pt_host;
    float *pt_step;
    float *pt_data;  // non-null: apply doStepFromBackup's point step in place (ldso_ba_optimize)
    int begin, count;
    float lambda;
    const int *stop;  // ldso_ba_optimize: points of windows with it >= stop[w] skip
    int it;
};

// xAd from the device solution (windows solved by k_solve, or x set otherwise)
__global__ __launch_bounds__(256) void k_xad(const WinDev *__restrict__ wins, const double *__restrict__ x,
                                             const double *__restrict__ adH, const double *__restrict__ adT,
                                             float *xad) {
    const WinDev &W = wins[blockIdx.x];
    xad_fill(W, x + W.vec_base, adH, adT, xad + (size_t)blockIdx.x * kXadStride, threadIdx.x, blockDim.x);
}

// ============================================================================================
// k_activate: FullSystem::optimizeImmaturePoint (FullSystem.cc:1035-1156) with
// ImmaturePoint::linearizeResidual (ImmaturePoint.cc:319-389), SURVEY §8f row 4.
// One wavefront per immature point; the temporary residual to the r-th other frame (window order)
// is evaluated by eight lanes, one per pattern pixel (see k_activate); the point's Hdd, bd and
// energy are summed on every lane in the reference's order (residual by residual, pixel by pixel,
// with the pixels before an OOB pixel still counted), so the LM steps are wave-uniform and
// bit-identical to the CPU restatement.
// ============================================================================================
struct ActParams {
    const WinDev *__restrict__ wins;
    const float4 *__restrict__ img;
    const float *__restrict__ precalc;
    const ldso_ct_immature *__restrict__ pts;
    ldso_ba_activation *out;
    long long frame_stride;
    int tpr, img_mode, win, n, min_obs;
};

// getInterpolatedElement33 (GlobalFuncs.h:89-103) of a resident frame (layout 3 or 1)
__device__ inline float3 sample33(const float4 *__restrict__ img, int mode, int tpr, long long frame_stride, float x,
                                  float y) {
#pragma clang fp contract(off)
    const int ix = (int)x, iy = (int)y;
    const float dx = x - ix, dy = y - iy;
    if (mode == 3) {
        float v[12];
        load12(frame_rsrc(reinterpret_cast<const float *>(img), frame_stride * 16), (unsigned)tpr * 128u, ix, iy, v);
        return bilin12(v, dx, dy);
    }
    const float dxdy = dx * dy;
    const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
    const float3 t00 = tex(img, tpr, ix, iy), t10 = tex(img, tpr, ix + 1, iy), t01 = tex(img, tpr, ix, iy + 1),
                 t11 = tex(img, tpr, ix + 1, iy + 1);
    return make_float3(w11 * t11.x + w01 * t01.x + w10 * t10.x + w00 * t00.x,
                       w11 * t11.y + w01 * t01.y + w10 * t10.y + w00 * t00.y,
                       w11 * t11.z + w01 * t01.z + w10 * t10.z + w00 * t00.z);
}

// Lanes per (residual, pattern pixel): lane 8 r' + idx evaluates pattern pixel idx of the
// temporary residual r = 8 round + r' (up to 8 residuals per round, two rounds for windows above
// 9 keyframes), so a residual's eight taps are sampled in parallel instead of one after another.
// The per-pixel terms go through the wave's LDS slot and every lane then folds them in the
// reference's order -- per residual the pixels up to its first OOB pixel, the residuals in window
// order -- so the point's energy, Hdd and bd, and every residual state, are wave-uniform and
// bit-identical to the CPU restatement.
constexpr int kActRes = 16;  // residual slots per point (N <= 16 -> at most 15)
struct ActLds {              // one wavefront's slot
    float e[kActRes][8], h[kActRes][8], b[kActRes][8];
    int first_oob[kActRes];  // pattern index of the first OOB pixel (8: none)
    float st_energy[kActRes], st_newenergy[kActRes];
    int st_state[kActRes], st_new[kActRes];
};
__global__ __launch_bounds__(256) void k_activate(ActParams P) {
#pragma clang fp contract(off)
    constexpr int pat[8][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0}, {0, 0}, {2, 0}, {-1, 1}, {0, 2}};
    constexpr float kMinIdepthHAct = 100;  // setting_minIdepthH_act, Setting.cc:25
    constexpr int kGNItsOnPointActivation = 3;  // Setting.cc:47
    __shared__ ActLds lds_act[4];
    const int lane = threadIdx.x & 63;
    const int k = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (k >= P.n) return;
    ActLds &A = lds_act[threadIdx.x >> 6];
    const WinDev &W = P.wins[P.win];
    const ldso_ct_immature &ip = P.pts[k];
    const int N = W.N, host = ip.host, nres = N - 1, rounds = (nres + 7) >> 3;
    const float fxl = W.calib[0], fyl = W.calib[1], cxl = W.calib[2], cyl = W.calib[3];
    const float fxli = 1.0f / fxl, fyli = 1.0f / fyl;
    const float eth = ip.energy_th;
    const int idx = lane & 7;
    // this lane's pattern pixel in the host frame (ImmaturePoint.cc:336-343)
    const float K0 = (ip.u + pat[idx][0] - cxl) * fxli, K1 = (ip.v + pat[idx][1] - cyl) * fyli;
    const float col = ip.color[idx], wsq = ip.weights[idx] * ip.weights[idx];
    if (lane < kActRes) {  // ImmaturePointTemporaryResidual (ImmaturePoint.h:18-26) of slot lane
        A.st_state[lane] = LDSO_BA_RES_IN;
        A.st_new[lane] = LDSO_BA_RES_OUTLIER;
        A.st_energy[lane] = 0;
        A.st_newenergy[lane] = 0;
    }
    wave_lds_sync();

    // linearizeResidual(HCalib, slack, tmpRes, Hdd, bd, idepth) of every residual, then the
    // point's sums in the reference's order -> (energy, Hdd, bd), identical on every lane
    auto evaluate = [&](float slack, float idepth, float &E, float &Hdd, float &bd) {
        for (int rd = 0; rd < rounds; rd++) {
            const int r = 8 * rd + (lane >> 3);
            if (r < nres && A.st_state[r] != LDSO_BA_RES_OOB) {
                const int tgt = r + (r >= host);
                const float *pre = P.precalc + (size_t)(W.pair_base + host + N * tgt) * LDSO_BA_PRECALC_STRIDE;
                const float *R = pre + 27, *t = pre + 36;  // PRE_RTll, PRE_tTll (current poses)
                bool oob = false;
                float e = 0, h = 0, b = 0;
                float ptp[3];
#pragma unroll
                for (int i = 0; i < 3; i++) ptp[i] = (R[3 * i] * K0 + R[3 * i + 1] * K1 + R[3 * i + 2] * 1.0f) + t[i] * idepth;
                const float drescale = 1.0f / ptp[2];
                const float uu = ptp[0] * drescale, vv = ptp[1] * drescale;
                const float Ku = uu * fxl + cxl, Kv = vv * fyl + cyl;
                if (!(drescale > 0) || !(Ku > 1.1f && Kv > 1.1f && Ku < W.wM3 && Kv < W.hM3)) {
                    oob = true;
                } else {
                    const float4 *img = P.img + (size_t)(W.frame_base + tgt) * P.frame_stride;
                    const float3 hc = sample33(img, P.img_mode, P.tpr, P.frame_stride, Ku, Kv);
                    if (!isfinite(hc.x)) {
                        oob = true;
                    } else {
                        const float residual = hc.x - (pre[24] * col + pre[25]);
                        float hw = fabsf(residual) < kHuberTH ? 1 : kHuberTH / fabsf(residual);
                        e = wsq * hw * residual * residual * (2 - hw);
                        const float dxInterp = hc.y * fxl, dyInterp = hc.z * fyl;
                        const float d_idepth =
                            (dxInterp * drescale * (t[0] - t[2] * uu) + dyInterp * drescale * (t[1] - t[2] * vv)) *
                            kScaleIdepth;
                        hw *= wsq;
                        h = (hw * d_idepth) * d_idepth;
                        b = (hw * residual) * d_idepth;
                    }
                }
                A.e[r][idx] = e;
                A.h[r][idx] = h;
                A.b[r][idx] = b;
                const unsigned long long m = __ballot(oob);  // this round's OOB pixels
                if (idx == 0) {
                    const unsigned g = (unsigned)(m >> (8 * (lane >> 3))) & 0xFFu;
                    A.first_oob[r] = g ? __builtin_ctz(g) : 8;
                }
            } else {
                (void)__ballot(false);  // every lane takes part in the ballot
            }
        }
        wave_lds_sync();
        // the reference's order on every lane: residual by residual, pixel by pixel
        for (int r = 0; r < nres; r++) {
            float ret = A.st_energy[r];
            if (A.st_state[r] == LDSO_BA_RES_OOB) {
                if (lane == 0) A.st_new[r] = LDSO_BA_RES_OOB;
            } else {
                const int fo = A.first_oob[r];
                float energyLeft = 0;
                for (int i = 0; i < fo; i++) {
                    energyLeft += A.e[r][i];
                    Hdd += A.h[r][i];
                    bd += A.b[r][i];
                }
                int ns;
                if (fo < 8) {
                    ns = LDSO_BA_RES_OOB;
                } else {
                    if (energyLeft > eth * slack) {
                        energyLeft = eth * slack;
                        ns = LDSO_BA_RES_OUTLIER;
                    } else {
                        ns = LDSO_BA_RES_IN;
                    }
                    ret = energyLeft;
                    if (lane == 0) A.st_newenergy[r] = energyLeft;
                }
                if (lane == 0) A.st_new[r] = ns;
            }
            E = (float)((double)E + (double)ret);
        }
        wave_lds_sync();
    };
    auto commit = [&]() {
        if (lane < nres) {
            A.st_state[lane] = A.st_new[lane];
            A.st_energy[lane] = A.st_newenergy[lane];
        }
        wave_lds_sync();
    };

    float lastEnergy = 0, lastHdd = 0, lastbd = 0;
    float currentIdepth = (ip.idepth_max + ip.idepth_min) * 0.5f;
    evaluate(1000.f, currentIdepth, lastEnergy, lastHdd, lastbd);
    commit();
    int status = 0;
    if (!isfinite(lastEnergy) || lastHdd < kMinIdepthHAct) {
        status = 2;
    } else {
        float lambda = 0.1f;
        for (int iteration = 0; iteration < kGNItsOnPointActivation; iteration++) {
            float H = lastHdd;
            H *= 1 + lambda;
            const float step = (float)((1.0 / (double)H) * (double)lastbd);
            const float newIdepth = currentIdepth - step;
            float newHdd = 0, newbd = 0, newEnergy = 0;
            evaluate(1.f, newIdepth, newEnergy, newHdd, newbd);
            if (!isfinite(lastEnergy) || newHdd < kMinIdepthHAct) {
                status = 2;
                break;
            }
            if (newEnergy < lastEnergy) {
                currentIdepth = newIdepth;
                lastHdd = newHdd;
                lastbd = newbd;
                lastEnergy = newEnergy;
                commit();
                lambda *= 0.5f;
            } else {
                lambda = (float)((double)lambda * 5.0);
            }
            if ((double)fabsf(step) < 0.0001 * (double)currentIdepth) break;
        }
        if (status == 0 && !isfinite(currentIdepth)) status = 1;
    }
    unsigned mask = 0;
    if (status == 0) {
        const unsigned long long in = __ballot(lane < nres && A.st_state[lane] == LDSO_BA_RES_IN);
        if (__popcll(in) < P.min_obs) {
            status = 1;
        } else {
            for (int r = 0; r < nres; r++)
                if ((in >> r) & 1ull) mask |= 1u << (r + (r >= host));
        }
    }
    if (lane == 0) {
        ldso_ba_activation o;
        o.idepth = currentIdepth;
        o.status = status;
        o.in_mask = mask;
        o.energy = lastEnergy;
        P.out[k] = o;
    }
}

__device__ __forceinline__ void resubstitute_one(const ResubParams &P, int k) {
#pragma clang fp contract(off)
    if (k >= P.count) return;
    const int p = P.begin + k;
    // every per-point load first (one round trip), then the exits
    const int w = P.pt_win[p], h = P.pt_host[p], nres = P.pt_nres[p];
    const unsigned long long tgs = P.pt_tgt[p];
    const float *po = P.pt_out + (size_t)p * 12;
    const float po0 = po[0], po1 = po[1], po5 = po[5], po6 = po[6], po7 = po[7], po8 = po[8], po9 = po[9];
    const float2 uv = *reinterpret_cast<const float2 *>(P.pt_geo + (size_t)p * LDSO_BA_POINT_STRIDE);
    if (P.stop && P.it >= P.stop[w]) return;
    // doStepFromBackup's point step (setIdepth / setIdepthZero / setDeltaF)
    auto apply = [&](float step) {
        if (!P.pt_data) return;
        float *d = P.pt_data + (size_t)p * LDSO_BA_POINT_STRIDE;
        const float idepth = d[2] + 1.0f * step;
        d[2] = kScaleIdepth * idepth;  // setIdepth
        d[3] = kScaleIdepth * idepth;  // setIdepthZero (LDSO's doStepFromBackup)
        d[5] = idepth - idepth;        // setDeltaF: idepth - idepth_zero
    };
    if (po9 == 0) {
        P.pt_step[p] = 0;
        apply(0.0f);
        return;
    }
    const WinDev &W = P.wins[w];
    const int N = W.N;
    const float *xad = P.xad + (size_t)w * kXadStride, *xc = xad + (size_t)N * N * 8;
    const size_t rp = (size_t)W.rec_base + (p - W.point_base);
    // residual q's operands -- its record, the pass's geometry of its pair, its xAd row -- loaded
    // unconditionally (the record's activity is tested after they land) and one residual ahead,
    // so the chain is one round trip per point instead of two per residual
    struct Ops {
        float2 rb;
        float4 ja;
        float4 g[4];  // geometry snapshot: R0 (9), t0 (3), calib (4)
        float4 xa[2];
    };
    auto load = [&](int q, Ops &o) {
        const int tg = (int)((tgs >> (4 * q)) & 15ull);
        const size_t rq = rp + (size_t)(tg < h ? tg : tg - 1) * W.P;
        o.rb = P.rec_b[rq];
        o.ja = P.rec_a[rq];
        const float4 *gs = reinterpret_cast<const float4 *>(P.geo_snap + (size_t)(W.pair_base + h + N * tg) * kGeoSnap);
#pragma unroll
        for (int e = 0; e < 4; e++) o.g[e] = gs[e];
        const float4 *xa = reinterpret_cast<const float4 *>(xad + (size_t)(h * N + tg) * 8);
        o.xa[0] = xa[0];
        o.xa[1] = xa[1];
    };
    Ops cur, nxt;
    if (nres > 0) load(0, cur);
    float b = po1;
    const float d = xc[0] * po5 + xc[1] * po6 + xc[2] * po7 + xc[3] * po8;
    b -= d;
    for (int q = 0; q < nres; q++) {
        load(min(q + 1, nres - 1), nxt);  // unconditional (a guarded load would be waited for at once)
        if (cur.rb.y == cur.rb.y) {       // active
            // the residual's JpJdF: (j0, j1) through the centre geometry of the pass (write_record)
            float pre[24];
#pragma unroll
            for (int e = 0; e < 3; e++) {
                pre[12 + 4 * e] = cur.g[e].x;
                pre[13 + 4 * e] = cur.g[e].y;
                pre[14 + 4 * e] = cur.g[e].z;
                pre[15 + 4 * e] = cur.g[e].w;
            }
            Geo g;
            (void)centre_projection(pre, uv.x, uv.y, cur.rb.y, cur.g[3].x, cur.g[3].y, cur.g[3].z, cur.g[3].w, W.wM3,
                                    W.hM3, g);
            float jp[6];
            record_jp6(g, cur.ja.x, cur.ja.y, jp);
            const float4 xa0 = cur.xa[0], xa1 = cur.xa[1];
            const float dd = xa0.x * jp[0] + xa0.y * jp[1] + xa0.z * jp[2] + xa0.w * jp[3] + xa1.x * jp[4] +
                             xa1.y * jp[5] + xa1.z * cur.ja.z + xa1.w * cur.ja.w;
            b -= dd;
        }
        cur = nxt;
    }
    if (!isfinite(b)) {  // reference returns from the chunk; the step is left unchanged
        apply(P.pt_step[p]);
        return;
    }
    const float step = -b * po0 / (1 + P.lambda);
    P.pt_step[p] = step;
    apply(step);
}
__global__ __launch_bounds__(256) void k_resubstitute(ResubParams P) {
    resubstitute_one(P, blockIdx.x * blockDim.x + threadIdx.x);
}
// JpJdF[8] of window w's residuals (device order) from their records and the geometry snapshot of
// the pass that wrote them (ldso_ba_get_residuals / _linearize_residuals); 0 where not active
__global__ __launch_bounds__(256) void k_record_jpjdf(const WinDev *__restrict__ wins, int w, const int *__restrict__ rs_slot,
                                                      const int *__restrict__ pt_host, const float *__restrict__ pt_geo,
                                                      const float4 *__restrict__ rec_a, const float2 *__restrict__ rec_b,
                                                      const float *__restrict__ geo_snap, float *out) {
    const WinDev &W = wins[w];
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= W.R) return;
    const int slot = rs_slot[W.res_base + k], sl = (slot - W.rec_base) / W.P, q = (slot - W.rec_base) - sl * W.P;
    const int p = W.point_base + q, h = pt_host[p], tg = sl < h ? sl : sl + 1;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const float2 rb = rec_b[slot];
    if (rb.y == rb.y) {
        const float4 ja = rec_a[slot];
        const float *gs = geo_snap + (size_t)(W.pair_base + h + W.N * tg) * kGeoSnap;
        const float2 uv = *reinterpret_cast<const float2 *>(pt_geo + (size_t)p * LDSO_BA_POINT_STRIDE);
        Geo g;
        (void)centre_projection(gs - 12, uv.x, uv.y, rb.y, gs[12], gs[13], gs[14], gs[15], W.wM3, W.hM3, g);
        record_jp6(g, ja.x, ja.y, v);
        v[6] = ja.z;
        v[7] = ja.w;
    }
    float4 *o = reinterpret_cast<float4 *>(out + (size_t)k * 8);
    o[0] = make_float4(v[0], v[1], v[2], v[3]);
    o[1] = make_float4(v[4], v[5], v[6], v[7]);
}

// image layout 3 (default): the intensity channel only, band-interleaved (band_offset: an 8x4
// pixel tile per 128-byte line, 1/4 of the float4 texel bytes); k_linearize recomputes the
// gradients with makeImages' rule.  That is exact only if the caller's gradients ARE makeImages'
// (FrameHessian.cc:96-101): every pixel the taps can reach (x in [1, w-2], y in [1, h-2]) is
// checked and *mismatch is set if not (the context then falls back to layout 1).
// ============================================================================================
// Device GN loop (ldso_ba_optimize): FullSystem::doStepFromBackup +
// setPrecalcValues without a host round trip.  k_frame_step: one block per window, se3.h's
// statements (the host helpers' own code): calibration and frame steps from x, then
// FrameFramePrecalc::Set for every pair and the solver's prior vector (takeData's prior /
// delta_prior, cPrior * cDeltaF), with k_xad's xAd for the resubstitution computed in the same
// launch.  The point step -- setIdepth / setIdepthZero(idepth_backup + step), deltaF = 0
// (setDeltaF) -- is applied by k_resubstitute as it computes the step.
// ============================================================================================
struct FrameStepParams {
    WinDev *wins;
    ldso_ba_frame_state *fstate;  // [frames]
    double *calib_val;            // [win][4] CalibHessian::value
    const double *calib_zero;     // [win][4] value_zero
    const double *cprior;         // [win][4] cPrior
    const int *add_priors;        // [win]
    const double *x;              // [vec]
    float *precalc;               // [pairs][LDSO_BA_PRECALC_STRIDE]
    double *prior;                // [vec][2]: HL diagonal, bL
    // ldso_ba_optimize's loop exits (FullSystem.cc:922, 968-969): windows with it >= stop[w] skip;
    // canbreak at it >= min_its sets stop[w] = it + 1 (the pass after this step still runs)
    int *stop, *status;
    const double *win_nid;  // [win][2]: sumNID, numID of the idepths the step starts from (point_nid)
    int it, min_its;
    float th;  // setting_thOptIterations
    float aff_a, aff_b;  // setting_affineOptModeA / B: the affine priors of takeData (getPrior)
};
// one window's step: a whole 256-thread block (blk = the window)
__device__ __forceinline__ void frame_step_block(const FrameStepParams &P, int blk) {
    __shared__ double poses[LDSO_BA_MAX_FRAMES][4][7];  // ev, ev^-1, cur, cur^-1: quaternion (4), t (3)
    __shared__ float calib[4];
    // the stop flag and the window's descriptor in one round trip, then the exit
    const int stop_it = P.stop ? P.stop[blk] : INT_MAX;
    WinDev &W = P.wins[blk];
    const int N = W.N, tid = threadIdx.x;
    const double *xw = P.x + W.vec_base;
    if (P.it >= stop_it) return;  // lost in this iteration's solve, or stopped earlier
    if (P.stop && tid == 128 && P.it >= P.min_its &&
        step_canbreak(N, xw, (float)P.win_nid[2 * blk], (float)P.win_nid[2 * blk + 1], P.th)) {
        P.stop[blk] = P.it + 1;
        P.status[blk] = LDSO_BA_OPT_CONVERGED;
    }
    ldso_ba_frame_state *fs = P.fstate + W.frame_base;
    if (tid < 64) {
        // frame_step_one's two exponentials in one SIMT pass of the same code: lane f forms
        // exp(step_f), lane 32 + f exp(state_f), handed to lane f by a shuffle (N <= 16 < 32)
        const int f = tid & 31, fc = f < N ? f : 0;
        const ldso_ba_frame_state in = fs[fc];
        double v[6];
        if (tid < 32)
            frame_step_tangent(xw + 4 + 8 * fc, v);
        else
            for (int i = 0; i < 6; i++) v[i] = in.state[i];
        const Pose ex = Pose::exp(v);
        Pose eb;
        for (int k = 0; k < 4; k++) eb.q[k] = __shfl(ex.q[k], fc + 32, 64);
        for (int k = 0; k < 3; k++) eb.t[k] = __shfl(ex.t[k], fc + 32, 64);
        if (tid < N) {
            ldso_ba_frame_state o;
            frame_step_finish(in, xw + 4 + 8 * tid, ex, eb, o);
            fs[tid] = o;
            const Pose e = eval_pose(o), c = current_pose(o);
            const Pose ps[4] = {e, e.inverse(), c, c.inverse()};
            for (int q = 0; q < 4; q++) {
                for (int k = 0; k < 4; k++) poses[tid][q][k] = ps[q].q[k];
                for (int k = 0; k < 3; k++) poses[tid][q][4 + k] = ps[q].t[k];
            }
        }
    } else if (tid == 64) {
        double *v = P.calib_val + 4 * blk;
        float cd[4];
        calib_step(v, xw, P.calib_zero + 4 * blk, calib, cd);
        for (int k = 0; k < 4; k++) {
            W.calib[k] = calib[k];
            W.cdelta[k] = cd[k];
        }
        const bool add = P.add_priors[blk] != 0;
        for (int k = 0; k < 4; k++) {  // calibration prior: cPrior, cPrior * cDeltaF (upload_priors)
            P.prior[2 * (W.vec_base + k)] = add ? P.cprior[4 * blk + k] : 0.0;
            P.prior[2 * (W.vec_base + k) + 1] = add ? P.cprior[4 * blk + k] * (double)cd[k] : 0.0;
        }
    }
    __syncthreads();
    auto pose = [&](int f, int q) {
        Pose p;
        for (int k = 0; k < 4; k++) p.q[k] = poses[f][q][k];
        for (int k = 0; k < 3; k++) p.t[k] = poses[f][q][4 + k];
        return p;
    };
    for (int e = tid; e < N * N; e += blockDim.x) {
        const int h = e % N, t = e / N;
        pair_precalc(pose(t, 0), pose(h, 1), pose(t, 2), pose(h, 3), calib, fs[h], fs[t],
                     P.precalc + (size_t)(W.pair_base + e) * LDSO_BA_PRECALC_STRIDE);
    }
    if (tid < N) {
        double pr[8], dp[8];
        frame_take_data_one(fs[tid], P.aff_a, P.aff_b, pr, nullptr, dp);
        const bool add = P.add_priors[blk] != 0;
        for (int i = 0; i < 8; i++) {
            const int q = W.vec_base + 4 + 8 * tid + i;
            P.prior[2 * q] = add ? pr[i] : 0.0;
            P.prior[2 * q + 1] = add ? pr[i] * dp[i] : 0.0;
        }
    }
}
// ldso_ba_optimize: the frame / calibration step (blocks [0, n_win)) and the resubstitution with
// the point step (the rest) in one launch; both read only x and xAd, which the solve wrote
__global__ __launch_bounds__(256) void k_step_resub(FrameStepParams F, ResubParams R, int n_win) {
    if ((int)blockIdx.x < n_win) frame_step_block(F, blockIdx.x);
    else resubstitute_one(R, ((int)blockIdx.x - n_win) * 256 + threadIdx.x);
}
// ldso_ba_optimize's energy history with a communicator (the window blocks of k_stitch write it
// otherwise): row s <- the all-reduced energies
__global__ __launch_bounds__(256) void k_energy_to_history(const double *src, double *hist, int s, int n2) {
    for (int i = threadIdx.x; i < n2; i += 256) hist[(size_t)s * n2 + i] = src[i];
}
// ldso_ba_update_points: [P][4] (idepth_scaled, idepth_zero_scaled, priorF, deltaF) of one window in
// its sorted point order into the point records (columns 2..5)
__global__ __launch_bounds__(256) void k_set_point_vals(const float4 *__restrict__ vals, float *pt_data, int n) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float4 v = vals[q];
    float *d = pt_data + (size_t)q * LDSO_BA_POINT_STRIDE;
    d[2] = v.x;
    d[3] = v.y;
    d[4] = v.z;
    d[5] = v.w;
}
// idepth of every resident point (point-data column 2), compacted for one small download
// up to kPackSegs device arrays (4-byte words) and optionally the idepth column of the point
// records into the mapped results buffer, one launch
constexpr int kPackSegs = 8;
struct PackOut {
    const unsigned *src[kPackSegs];
    unsigned *dst[kPackSegs];
    int words[kPackSegs];
    int n_seg;
    const float *pt_data;  // non-null: idepth of every point record into idepth_dst
    float *idepth_dst;
    int n_points;
};
__global__ __launch_bounds__(256) void k_pack_out(PackOut P) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    for (int s = 0; s < P.n_seg; s++)
        for (int e = tid; e < P.words[s]; e += nth) P.dst[s][e] = P.src[s][e];
    if (P.pt_data)
        for (int q = tid; q < P.n_points; q += nth) P.idepth_dst[q] = P.pt_data[(size_t)q * LDSO_BA_POINT_STRIDE + 2];
}
// resetOOB() over a residual range; optionally also the scratch copies of
// ldso_ba_linearize_residuals: centre "not projected" (all-ones NaN) and the flags copied
__global__ __launch_bounds__(256) void k_reset_oob(int8_t *state, int8_t *newstate, float *energy, float *newenergy,
                                                    int n, float *center = nullptr, long long cstride = 0,
                                                    uint8_t *flags = nullptr, const uint8_t *flags_src = nullptr) {
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        state[r] = LDSO_BA_RES_IN;
        newstate[r] = LDSO_BA_RES_OUTLIER;
        energy[r] = 0.f;
        newenergy[r] = 0.f;
        if (center) {
            const float q = __uint_as_float(0xFFFFFFFFu);
            for (int k = 0; k < 4; k++) center[k * cstride + r] = q;
            flags[r] = flags_src[r];
        }
    }
}
__global__ __launch_bounds__(256) void k_gather_idepth(const float *__restrict__ pt_data, float *out, int n) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q < n) out[q] = pt_data[(size_t)q * LDSO_BA_POINT_STRIDE + 2];
}

__global__ void k_intensity_image(const float *__restrict__ src, float *dst, int w, int h, int tpr8, int hp,
                                  int *mismatch) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int wp = tpr8 * 8;
    if (i >= wp * hp) return;
    const int x = i % wp, y = i / wp;
    float v = 0.f;
    if (x < w && y < h) {
        const float *p = src + 3 * ((size_t)y * w + x);
        v = p[0];
        if (x >= 1 && x <= w - 2 && y >= 1 && y <= h - 2) {
            const float dx = make_grad(p[3], p[-3]), dy = make_grad(p[3 * w], p[-3 * w]);
            if (__float_as_uint(dx) != __float_as_uint(p[1]) || __float_as_uint(dy) != __float_as_uint(p[2]))
                atomicOr(mismatch, 1);
        }
    }
    dst[band_offset(x, y, (unsigned)wp * 16u) >> 2] = v;
}

// image layout 1: FrameHessian::dI (AoS [I, dx, dy]) -> [I, dx, dy, 0] texels in 2x4 tiles
__global__ void k_tile_image(const float *__restrict__ src, float4 *dst, int w, int h, int tpr2, int hp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int wp = tpr2 * 2;
    if (i >= wp * hp) return;
    const int x = i % wp, y = i / wp;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (x < w && y < h) {
        const float *p = src + 3 * ((size_t)y * w + x);
        v = make_float4(p[0], p[1], p[2], 0.f);
    }
    dst[(((y >> 2) * tpr2 + (x >> 1)) << 3) + ((y & 3) << 1) + (x & 1)] = v;
}

template <bool kMarg>
void launch_linearize(int img_mode, int nb, hipStream_t st, const LinParams &L, hipEvent_t ev_start = nullptr,
                      hipEvent_t ev_stop = nullptr) {
    if (ev_start) {  // timed: the dispatch itself stamps the events (no separate event packets in the stream)
        if (img_mode == 3)
            hipExtLaunchKernelGGL(k_linearize<3, kMarg>, dim3(nb), dim3(256), kLinLdsBytes, st, ev_start, ev_stop, 0, L);
        else
            hipExtLaunchKernelGGL(k_linearize<1, kMarg>, dim3(nb), dim3(256), kLinLdsBytes, st, ev_start, ev_stop, 0, L);
        return;
    }
    if (img_mode == 3) k_linearize<3, kMarg><<<nb, 256, kLinLdsBytes, st>>>(L);
    else k_linearize<1, kMarg><<<nb, 256, kLinLdsBytes, st>>>(L);
}

// ============================================================================================
// host side
// ============================================================================================
// bumped by every device (re)allocation: a captured graph is valid while it is unchanged
std::atomic<unsigned long long> g_alloc_gen{1};
template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    int alloc(size_t count) {
        g_alloc_gen.fetch_add(1);
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (count == 0) return 0;
        hipError_t e = hipMalloc(&p, count * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            return fail(-3, std::string("hipMalloc failed: ") + hipGetErrorString(e));
        }
        n = count;  // only a successful allocation counts as capacity
        return 0;
    }
    int ensure(size_t count) { return n >= count && p ? 0 : alloc(count); }  // keeps the pointer if it fits
    void release() {
        g_alloc_gen.fetch_add(1);
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
    std::vector<int> rs_slot;       // sorted residual -> record slot (global)
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
    // inside ldso_ba_optimize: the index of the pass being issued (0 = the initial linearizeAll,
    // k = the pass after step k-1), else -1.  Passes then write row opt_pass of the energy history,
    // the window blocks sumNID / numID, and every launch honours the per-window loop exits (d_stop)
    int opt_pass = -1;
    int opt_it = 0;
    // captured launch sequences: ldso_ba_optimize's GN iterations [projection][last pass][ns given]
    // and ldso_ba_iterate's pass + solve + resubstitution [projection]
    // a cached graph and everything fixed at its capture, compared field by field (no packing into
    // one word: a collision would replay a graph whose launch parameters differ)
    struct Graph {
        hipGraphExec_t exec = nullptr;
        unsigned long long gen = 0;
        std::vector<unsigned long long> key;
    };
    Graph opt_graph[2], it_graph[2];  // ldso_ba_optimize's whole call (without / with nullspaces)
    bool opt_warm = false;            // an optimize call ran directly on this context
    int item_order = 0;  // k_linearize chunk order: 0 target-major, 1 host-major, 2 target-major banded
    // the reference's settings this context runs with (ldso_ba_set_settings; always checked)
    ldso_ba_opt_settings settings = LDSO_BA_OPT_SETTINGS_INIT;
    int n_win = 0, width = 0, height = 0, npix = 0;
    std::vector<WinHost> wh;
    std::vector<WinDev> wd;
    int n_top_items = 0, n_sc_items = 0, n_pairs = 0, n_frames = 0, P_tot = 0, R_tot = 0, max_frames = 0;
    DevBuf<WinDev> d_wins;
    DevBuf<float4> d_img;
    DevBuf<ldso_ct_immature> d_act_in;  // point activation staging (ldso_ba_activate_points)
    DevBuf<ldso_ba_activation> d_act_out;
    int tiles_per_row = 0, padded_h = 0;
    long long frame_stride = 0;
    DevBuf<float> d_precalc, d_frame_th, d_pt_data, d_pt_out, d_pt_step;
    DevBuf<double> d_adH, d_adT;
    DevBuf<int> d_rs_slot, d_pt_nres, d_pair_win, d_frame_win, d_pt_host;
    DevBuf<unsigned long long> d_pt_tgt;
    DevBuf<uint8_t> d_rs_tgt, d_rs_flags;
    DevBuf<int8_t> d_rs_state, d_rs_newstate;
    DevBuf<float> d_rs_energy, d_rs_newenergy, d_rs_energy_wo;
    DevBuf<float4> d_rs_center, d_rec_a;
    DevBuf<float2> d_rec_b;
    DevBuf<float> d_geo_snap;  // [pairs][kGeoSnap] (LinParams::geo_snap)
    DevBuf<int4> d_top_items, d_sc_items;
    DevBuf<int2> d_pair_items, d_host_items;
    DevBuf<float> d_top_slab, d_sc_slab;
    // d_sys = the exchange buffer: every window's packed system [sys_n], then the linearizeAll
    // energy / #IN pairs [n_win][2] (win_energy()), then doStepFromBackup's sumNID / numID
    // [n_win][2] (win_nid(), double: the ranks' float partials summed) -- contiguous, so that the
    // multi-GPU exchange reduces all three in ONE collective
    DevBuf<double> d_item_energy, d_sys, d_stage;
    size_t sys_n = 0;
    double *win_energy() const { return d_sys.p + sys_n; }
    double *win_nid() const { return d_sys.p + sys_n + 2 * (size_t)n_win; }
    DevBuf<int2> d_sum_blocks;  // k_stitch_sum: {window, first packed element} per 256-thread block
    int n_sum_blocks = 0;
    // in-library multi-GPU exchange (ldso_ba_comm_init): RCCL communicator over this context's
    // device, the newest-frame energy slot stride (max over ranks, set at the first exchange
    // after a load) and its staging buffers
    ncclComm_t comm = nullptr;
    int comm_rank = 0, comm_world = 1;
    int64_t x_stride = 0;
    int64_t x_prun = 0;  // |idepth| run length per window slot (max local points over windows and ranks)
    DevBuf<float> d_x_local, d_x_gathered;
    // device GN loop (ldso_ba_optimize): frame states, CalibHessian::value / value_zero and the
    // prior switches per window, the energy history
    DevBuf<ldso_ba_frame_state> d_fstate;
    DevBuf<double> d_calib_val, d_calib_zero, d_cprior, d_ehist;
    DevBuf<int> d_stop, d_status;  // ldso_ba_optimize: per window, see FrameStepParams
    DevBuf<int> d_add_priors;
    DevBuf<float> d_xad;            // [win][kXadStride]
    DevBuf<double> d_prior, d_x, d_ns;  // per-window (8N+4)-vectors: priors (HL diag, bL), x, nullspaces
    DevBuf<double> d_ns_nm, d_ns_g;     // k_ortho_prep's Nm [7 vec] and per-window G | G^-1 | fast
    std::vector<double> ns_cache;       // the nullspaces k_ortho_prep last prepared (host copy) ...
    int ns_cache_null = -1;             // ... and their count; -1: nothing prepared
    DevBuf<int> d_pt_win;
    // marginalisation context (ldso_ba_load_marginalization): images borrowed from the parent
    // context's window, addPoint<2> sums, no prior shift in the SC pass
    bool marg = false;
    bool host_stitch = false;
    int n_cu = 256;  // compute units (k_stitch_host splits its blocks when the grid fits at once)  // k_stitch_host + k_stitch_host_sum (every window <= kHostStitchMaxN keyframes)
    const float4 *img_ext = nullptr;
    DevBuf<float> d_adhtd;  // [pairs][8] adHTdeltaF
    int vec_total = 0;
    size_t sc_smem_max = 0;
    bool timing = false;
    unsigned timing_mask = ~0u;  // kernel slots bracketed by events when timing is on
    int top_chunk = 0;  // residuals per k_linearize wave (0 = automatic); LDSO_BA_TUNE_TOP_CHUNK
    int solve_exact = 0;  // LDSO_BA_TUNE_SOLVE_EXACT: 1 = the pivoted k_solve_reg / k_solve (bit-identical to the host)
    int img_mode = 3;   // 3 intensity only (band_offset), 1 [I, dx, dy, 0] 2x4 tiles (LDSO_BA_TUNE_TILED_IMAGES)
    std::vector<PendingEv> pending;
    std::vector<hipEvent_t> ev_pool;
    double kms[kNumKernels] = {0};
    long long kcount[kNumKernels] = {0};
    std::vector<double> sys_host;  // last downloaded packed systems (per window, see sys_valid)
    std::vector<char> sys_valid;
    bool sys_host_valid = false;   // false => every window's host copy is stale
    // pinned staging for the per-iteration host round trips (system download, xAd upload,
    // point-step download): async copies with one synchronisation each
    double *pin_sys = nullptr;
    float *pin_xad = nullptr, *pin_step = nullptr;
    size_t pin_sys_n = 0, pin_step_n = 0;
    // pinned staging for the results of ldso_ba_iterate / ldso_ba_optimize: every download of
    // one call lands here, behind a single synchronisation
    char *pin_out = nullptr;
    size_t pin_out_n = 0;
    char *pin_map = nullptr, *pin_map_dev = nullptr;  // fine-grained pinned results buffer, written by k_pack_out
    size_t pin_map_n = 0;
    char *pin_in = nullptr, *pin_in_dev = nullptr;  // mapped staging of small uploads, read by k_pack_out
    size_t pin_in_n = 0;
    hipEvent_t pin_in_ev = nullptr;  // the last launch reading pin_in
    bool pin_in_busy = false;
    std::vector<double> energy_host;
    bool energy_valid = false;
    std::vector<float> th_host;  // d_frame_th as of the end of the last ldso_ba_optimize ...
    bool th_host_valid = false;  // ... until the next pass, update or threshold exchange
    // ldso_ba_linearize_residuals: k_linearize runs on copies of the residual state so that the
    // context's own state (and its records, read by resubstitution) stay untouched
    DevBuf<int8_t> d_sx_state, d_sx_newstate;
    DevBuf<uint8_t> d_sx_flags;
    DevBuf<float> d_sx_energy, d_sx_newenergy, d_sx_ewo;
    DevBuf<float4> d_sx_center, d_sx_rec_a, d_pt_vals;
    DevBuf<float2> d_sx_rec_b;
    DevBuf<float> d_sx_geo_snap, d_jp_out;
    DevBuf<double> d_sx_item;
};

namespace {

// LinParams::aff_fix of the context's settings: which of JabF[0] / JabF[1] linearize zeroes
inline int aff_fix_bits(const ldso_ba_ctx *c) {
    return (c->settings.affine_opt_mode_a < 0 ? 1 : 0) | (c->settings.affine_opt_mode_b < 0 ? 2 : 0);
}

// grow-only pinned host staging (the address is kept while it fits)
int pin_ensure(char *&p, size_t &cap, size_t bytes) {
    bytes = std::max<size_t>(bytes, 64);
    if (p && cap >= bytes) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    HIP_TRY(hipHostMalloc((void **)&p, bytes, hipHostMallocDefault));
    cap = bytes;
    return 0;
}

// the results buffer the device writes directly (coherent host memory: k_pack_out's stores are
// visible to the host once the stream has synchronised), so a call's results come back in one
// launch instead of one blit per array
int pin_map_ensure(ldso_ba_ctx *c, size_t bytes) {
    bytes = std::max<size_t>(bytes, 64);
    if (c->pin_map && c->pin_map_n >= bytes) return 0;
    if (c->pin_map) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        (void)hipHostFree(c->pin_map);
    }
    c->pin_map = c->pin_map_dev = nullptr;
    c->pin_map_n = 0;
    HIP_TRY(hipHostMalloc((void **)&c->pin_map, bytes, hipHostMallocCoherent | hipHostMallocMapped));
    void *d = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&d, c->pin_map, 0));
    c->pin_map_dev = static_cast<char *>(d);
    c->pin_map_n = bytes;
    return 0;
}

// Small host -> device uploads of one call gathered into the mapped staging buffer and written
// by ONE k_pack_out launch (pageable hipMemcpyAsync costs ~10 us of host time per array)
struct InBatch {
    struct Item {
        void *dst;
        const void *src;
        size_t bytes;
    };
    std::vector<Item> items;
    void add(void *dst, const void *src, size_t bytes) {
        if (bytes) items.push_back({dst, src, bytes});
    }
    int flush(ldso_ba_ctx *c);
};
int InBatch::flush(ldso_ba_ctx *c) {
    if (items.empty()) return 0;
    size_t total = 0;
    for (const Item &it : items) total += (it.bytes + 15) & ~(size_t)15;
    if (c->pin_in_busy) {  // the previous launch must have read the staging buffer
        HIP_TRY(hipEventSynchronize(c->pin_in_ev));
        c->pin_in_busy = false;
    }
    if (!c->pin_in || c->pin_in_n < total) {
        if (c->pin_in) (void)hipHostFree(c->pin_in);
        c->pin_in = c->pin_in_dev = nullptr;
        c->pin_in_n = 0;
        HIP_TRY(hipHostMalloc((void **)&c->pin_in, std::max<size_t>(total, 4096), hipHostMallocCoherent | hipHostMallocMapped));
        void *d = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&d, c->pin_in, 0));
        c->pin_in_dev = static_cast<char *>(d);
        c->pin_in_n = std::max<size_t>(total, 4096);
    }
    if (!c->pin_in_ev) HIP_TRY(hipEventCreateWithFlags(&c->pin_in_ev, hipEventDisableTiming));
    size_t off = 0;
    PackOut K{};
    for (size_t k = 0; k < items.size(); k++) {
        const Item &it = items[k];
        std::memcpy(c->pin_in + off, it.src, it.bytes);
        K.src[K.n_seg] = reinterpret_cast<const unsigned *>(c->pin_in_dev + off);
        K.dst[K.n_seg] = static_cast<unsigned *>(it.dst);
        K.words[K.n_seg++] = (int)(it.bytes / 4);
        off += (it.bytes + 15) & ~(size_t)15;
        if (K.n_seg == kPackSegs || k + 1 == items.size()) {
            k_pack_out<<<std::min(64, (int)(total / 1024) + 1), 256, 0, c->stream>>>(K);
            HIP_TRY(hipGetLastError());
            K = PackOut{};
        }
    }
    HIP_TRY(hipEventRecord(c->pin_in_ev, c->stream));
    c->pin_in_busy = true;
    items.clear();
    return 0;
}

hipEvent_t get_event(ldso_ba_ctx *c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    // timing-only events: no system-scope fence (its L2 write-back and invalidate would be timed,
    // and would slow the kernel after the start event)
    (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
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

// timed_launch for a launch that takes the events itself (hipExtLaunchKernelGGL's start / stop
// events, stamped by the dispatch): the stream carries no event packets around the kernel, which
// on this path cost ~5 us of idle GPU on each side of it
template <typename F>
int timed_launch_ext(ldso_ba_ctx *c, int slot, hipStream_t st, F &&launch) {
    hipEvent_t a = nullptr, b = nullptr;
    const bool timed = c->timing && ((c->timing_mask >> slot) & 1u);
    if (timed) {
        a = get_event(c);
        b = get_event(c);
    }
    launch(a, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(-2, std::string("launch ") + kKernelNames[slot] + ": " + hipGetErrorString(e));
    if (timed) c->pending.push_back({slot, a, b});
    (void)st;
    return 0;
}
template <typename F>
int timed_launch(ldso_ba_ctx *c, int slot, hipStream_t st, F &&launch) {
    hipEvent_t a = nullptr, b = nullptr;
    const bool timed = c->timing && ((c->timing_mask >> slot) & 1u);
    if (timed) {
        a = get_event(c);
        b = get_event(c);
        (void)hipEventRecord(a, st);
    }
    launch();
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(-2, std::string("launch ") + kKernelNames[slot] + ": " + hipGetErrorString(e));
    if (timed) {
        (void)hipEventRecord(b, st);
        c->pending.push_back({slot, a, b});
    }
    return 0;
}

int check_window(const ldso_ba_window &w, bool need_images = true) {
    if (w.n_frames < 2 || w.n_frames > LDSO_BA_MAX_FRAMES) return fail(-1, "n_frames out of range [2,16]");
    if (w.n_points < 0 || w.n_residuals < 0) return fail(-1, "negative counts");
    if ((need_images && !w.dI) || !w.frame_energy_th || !w.precalc || !w.ad_host || !w.ad_target || !w.c_prior || !w.c_delta ||
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

size_t sc_smem_bytes(int KP) {
    return ((size_t)kScPoints * (KP + 4) + (size_t)LDSO_BA_MAX_FRAMES * kPrePitch) * sizeof(float);
}

// frame geometry of the image layout (all strides in float4 units)
void image_geometry(ldso_ba_ctx *c) {
    c->padded_h = (c->height + 3) / 4 * 4;
    if (c->img_mode == 3) {
        c->tiles_per_row = (c->width + 7) / 8;
        c->frame_stride = (long long)c->tiles_per_row * 8 * c->padded_h / 4;
    } else {
        c->tiles_per_row = (c->width + 1) / 2;
        c->frame_stride = (long long)c->tiles_per_row * 2 * c->padded_h;
    }
}

int stage_images(ldso_ba_ctx *c, const ldso_ba_window *ws, int n_windows, int *mismatch) {
    float *stage = nullptr;
    int *flag = nullptr;
    HIP_TRY(hipMalloc(&stage, (size_t)c->npix * 3 * sizeof(float)));
    if (hipMalloc(&flag, sizeof(int)) != hipSuccess) {
        (void)hipFree(stage);
        return fail(-3, "hipMalloc failed");
    }
    hipError_t e = hipMemsetAsync(flag, 0, sizeof(int), c->stream);
    int fb = 0;
    for (int w = 0; w < n_windows && e == hipSuccess; w++)
        for (int f = 0; f < ws[w].n_frames && e == hipSuccess; f++, fb++) {
            e = hipMemcpyAsync(stage, ws[w].dI + (size_t)f * c->npix * 3, (size_t)c->npix * 3 * sizeof(float),
                               hipMemcpyHostToDevice, c->stream);
            if (e != hipSuccess) break;
            float4 *dst = c->d_img.p + (size_t)fb * c->frame_stride;
            if (c->img_mode == 3) {
                const long long n = (long long)c->tiles_per_row * 8 * c->padded_h;
                k_intensity_image<<<(int)((n + 255) / 256), 256, 0, c->stream>>>(
                    stage, reinterpret_cast<float *>(dst), c->width, c->height, c->tiles_per_row, c->padded_h, flag);
            } else {
                k_tile_image<<<(int)((c->frame_stride + 255) / 256), 256, 0, c->stream>>>(
                    stage, dst, c->width, c->height, c->tiles_per_row, c->padded_h);
            }
            e = hipGetLastError();
        }
    if (e == hipSuccess) e = hipMemcpyAsync(mismatch, flag, sizeof(int), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(stage);
    (void)hipFree(flag);
    if (e != hipSuccess) return fail(-2, std::string("image staging: ") + hipGetErrorString(e));
    return 0;
}

// HL diagonal and bL of one window (the priors accumulateLF_MT stitches, AccumulatedTopHessian.cc:
// 241-250) as the device solver reads them; zero on ranks other than 0 of a sharded window
void priors_vector(const ldso_ba_ctx *c, int win, std::vector<double> &pr) {
    const WinHost &H = c->wh[win];
    const WinDev &D = c->wd[win];
    pr.assign((size_t)2 * D.D, 0.0);
    if (H.add_priors) {
        for (int i = 0; i < 4; i++) {
            pr[2 * i] = H.c_prior[i];
            pr[2 * i + 1] = H.c_prior[i] * (double)H.c_delta[i];
        }
        for (int f = 0; f < H.N; f++)
            for (int i = 0; i < 8; i++) {
                const int q = 4 + 8 * f + i;
                pr[2 * q] = H.frame_prior[8 * f + i];
                pr[2 * q + 1] = H.frame_prior[8 * f + i] * H.frame_delta_prior[8 * f + i];
            }
    }
}
int upload_priors(ldso_ba_ctx *c, int win) {
    std::vector<double> pr;
    priors_vector(c, win, pr);
    HIP_TRY(hipMemcpyAsync(c->d_prior.p + (size_t)2 * c->wd[win].vec_base, pr.data(), pr.size() * sizeof(double),
                           hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

// where ldso_ba_optimize computes the step's sumNID: in extra blocks of k_solve_fast, beside the
// factorisation; with an exact solve mode in leading blocks of the pass's k_point_sc, or, with a
// communicator, in extra blocks of the exchange's k_frame_th
inline bool nid_in_solve(const ldso_ba_ctx *c) { return !c->solve_exact && !getenv_flag("LDSO_BA_SOLVE_LDS"); }
// the idepths the sumNID chain walks: the context's points, or with a communicator every rank's
// run of the window from the last exchange's all-gather (the runs concatenated in rank order are
// the unsharded host-frame order, so the chain is the single-GPU one bit for bit)
NidSrc nid_source(const ldso_ba_ctx *c) {
    NidSrc n{};
    n.pt_data = c->d_pt_data.p;
    if (c->comm) {
        n.gathered = c->d_x_gathered.p;
        n.slot = c->x_stride + c->x_prun;
        n.off = c->x_stride;
        n.n_ranks = c->comm_world;
        n.n_win = c->n_win;
        n.prun = (int)c->x_prun;
    }
    return n;
}
ResubParams resub_params(ldso_ba_ctx *c, int begin, int count, double lambda, bool apply_step) {
    ResubParams R{};
    R.pt_data = apply_step ? c->d_pt_data.p : nullptr;
    R.xad = c->d_xad.p;
    R.wins = c->d_wins.p;
    R.pt_win = c->d_pt_win.p;
    R.pt_nres = c->d_pt_nres.p;
    R.pt_tgt = c->d_pt_tgt.p;
    R.rec_a = c->d_rec_a.p;
    R.rec_b = c->d_rec_b.p;
    R.geo_snap = c->d_geo_snap.p;
    R.pt_geo = c->d_pt_data.p;
    R.pt_out = c->d_pt_out.p;
    R.pt_host = c->d_pt_host.p;
    R.pt_step = c->d_pt_step.p;
    R.begin = begin;
    R.count = count;
    R.lambda = (float)lambda;
    return R;
}
int launch_resubstitute(ldso_ba_ctx *c, int begin, int count, double lambda, bool apply_step = false) {
    const ResubParams R = resub_params(c, begin, count, lambda, apply_step);
    return timed_launch(c, 3, c->stream, [&] { k_resubstitute<<<(count + 255) / 256, 256, 0, c->stream>>>(R); });
}
// k_stitch dynamic LDS: max of the Top phase, the SC phase of the largest window, and the
// frame-threshold staging (at least 1024 candidates; more if the SC phase leaves room)
size_t stitch_smem_bytes(int KP, int N, int *th_cap) {
    const size_t top = (96 + 169 + 4 * 64) * sizeof(double);
    const size_t sc = (size_t)(kStTopLds + 8 * KP + 4 * (N - 1) * 64 + 20) * sizeof(double);
    const size_t th_fixed = th_fixed_bytes(kStThreads);
    size_t bytes = std::max(top, sc);
    bytes = std::max(bytes, th_fixed + 1024 * sizeof(unsigned));
    bytes = (bytes + 15) & ~(size_t)15;
    *th_cap = (int)((bytes - th_fixed) / sizeof(unsigned)) & ~3;
    return bytes;
}

// k_stitch_host dynamic LDS: the host block's staging for the largest window, at least the
// frame-threshold staging of 1024 candidates (more if the host phase leaves room)
size_t stitch_host_smem_bytes(int N, int *th_cap) {
    const size_t th_fixed = th_fixed_bytes(kHsThreads);
    size_t bytes = std::max(hs_lds_doubles(N) * sizeof(double), th_fixed + 1024 * sizeof(unsigned));
    bytes = (bytes + 15) & ~(size_t)15;
    *th_cap = (int)((bytes - th_fixed) / sizeof(unsigned)) & ~3;
    return bytes;
}

}  // namespace

namespace {
void shard_points(const ldso_ba_window &in, int rank, int count, std::vector<int> &out);
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
int ldso_ba_frame_take_data(int32_t n, const ldso_ba_frame_state *f, const ldso_ba_opt_settings *st, double *prior,
                            double *delta, double *dp) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !f) return fail(-1, "bad arguments");
    int rc;
    if ((rc = ldso_ba_check_settings(st))) return rc;
    const ldso_ba_opt_settings s = st ? *st : ldso_ba_opt_settings LDSO_BA_OPT_SETTINGS_INIT;
    return frame_take_data(n, f, s.affine_opt_mode_a, s.affine_opt_mode_b, prior, delta, dp);
}
int ldso_ba_nullspaces(int32_t n, const ldso_ba_frame_state *f, double *out) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !f || !out) return fail(-1, "bad arguments");
    return nullspaces(n, f, out);
}
int ldso_ba_solve_system(const ldso_ba_opt_settings *st, int32_t n, int32_t it, double lambda, const double *HA,
                         const double *bA, const double *HL, const double *bL, const double *HM, const double *bM,
                         const double *Hsc, const double *bsc, const double *ns, int32_t nn, double *x) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !HA || !bA || !HL || !bL || !Hsc || !bsc || !x)
        return fail(-1, "bad arguments");
    int rc;
    if ((rc = ldso_ba_check_settings(st))) return rc;  // the default solver mode only, no inertial terms
    // without SOLVER_ORTHOGONALIZE_X_LATER the solve never projects (EnergyFunctional.cc:428-432)
    if (st && !(st->solver_mode & LDSO_BA_SOLVER_ORTHOGONALIZE_X_LATER)) nn = 0;
    return solve_system(n, it, lambda, HA, bA, HL, bL, HM, bM, Hsc, bsc, ns, nn, x);
}

int ldso_ba_marginalize_frame(int32_t n, int32_t idx, const double *HM, const double *bM, const double *prior,
                              const double *delta_prior, double *HM_out, double *bM_out) {
    if (n < 2 || n > LDSO_BA_MAX_FRAMES || idx < 0 || idx >= n || !HM || !bM || !prior || !delta_prior || !HM_out ||
        !bM_out)
        return fail(-1, "bad arguments");
    return marginalize_frame(n, idx, HM, bM, prior, delta_prior, HM_out, bM_out);
}

int ldso_ba_ad_ht_delta(int32_t n, const double *delta, const double *adH, const double *adT, float *out) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !delta || !adH || !adT || !out) return fail(-1, "bad arguments");
    return ad_ht_delta(n, delta, adH, adT, out);
}
int ldso_ba_calc_m_energy(int32_t n, const double *HM, const double *bM, const float *c_delta, const double *delta,
                          double *out) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !HM || !bM || !c_delta || !delta || !out) return fail(-1, "bad arguments");
    *out = calc_m_energy(n, HM, bM, c_delta, delta);
    return 0;
}
int ldso_ba_calc_l_energy(int32_t n, const double *prior, const double *delta_prior, const double *c_prior,
                          const float *c_delta, int32_t n_points, const float *deltaF, const float *priorF,
                          double *out) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !prior || !delta_prior || !c_prior || !c_delta || n_points < 0 ||
        (n_points > 0 && (!deltaF || !priorF)) || !out)
        return fail(-1, "bad arguments");
    *out = calc_l_energy(n, prior, delta_prior, c_prior, c_delta, n_points, deltaF, priorF);
    return 0;
}

int ldso_ba_shard_points(const ldso_ba_window *w, int32_t rank, int32_t count, int32_t *points_out,
                         int32_t *n_out) {
    if (!w || !n_out || count < 1 || rank < 0 || rank >= count) return fail(-1, "bad arguments");
    if (int rc = check_window(*w, false)) return rc;
    std::vector<int> pts;
    shard_points(*w, rank, count, pts);
    if (points_out) std::memcpy(points_out, pts.data(), pts.size() * sizeof(int32_t));
    *n_out = (int32_t)pts.size();
    return 0;
}

int ldso_ba_pack_upper(int32_t dim, const double *HA, const double *bA, const double *Hsc, const double *bsc,
                        double *packed) {
    if (dim < 1 || !HA || !bA || !Hsc || !bsc || !packed) return fail(-1, "bad arguments");
    const long long pl = packed_len(dim);
    long long q = 0;
    for (int r = 0; r < dim; r++)
        for (int c = r; c < dim; c++, q++) {
            packed[q] = HA[(size_t)r * dim + c];
            packed[pl + dim + q] = Hsc[(size_t)r * dim + c];
        }
    for (int r = 0; r < dim; r++) {
        packed[pl + r] = bA[r];
        packed[2 * pl + dim + r] = bsc[r];
    }
    return 0;
}

int ldso_ba_unpack_upper(int32_t dim, const double *packed, double *HA, double *bA, double *Hsc, double *bsc) {
    if (dim < 1 || !packed) return fail(-1, "bad arguments");
    const long long pl = packed_len(dim);
    long long q = 0;
    for (int r = 0; r < dim; r++)
        for (int c = r; c < dim; c++, q++) {
            if (HA) HA[(size_t)r * dim + c] = HA[(size_t)c * dim + r] = packed[q];
            if (Hsc) Hsc[(size_t)r * dim + c] = Hsc[(size_t)c * dim + r] = packed[pl + dim + q];
        }
    for (int r = 0; r < dim; r++) {
        if (bA) bA[r] = packed[pl + r];
        if (bsc) bsc[r] = packed[2 * pl + dim + r];
    }
    return 0;
}

// setNewFrameEnergyTH (FullSystem.cc:2078-2109) over gathered NewEnergyWithOutlier values (< 0:
// padding, skipped): the host form of k_frame_th, for callers that gather the slots themselves
int ldso_ba_frame_threshold(const float *values, int64_t n, float *th_out) {
    if (!th_out || n < 0 || (n > 0 && !values)) return fail(-1, "bad arguments");
    std::vector<float> v;
    v.reserve((size_t)n);
    for (int64_t i = 0; i < n; i++)
        if (values[i] >= 0) v.push_back(values[i]);
    if (v.empty()) {
        *th_out = 12 * 12 * LDSO_BA_PATTERN_NUM;
        return 0;
    }
    const int nth = (int)(kFrameEnergyTHN * (float)v.size());
    std::nth_element(v.begin(), v.begin() + nth, v.end());
    const float x = sqrtf(v[nth]);
    float th = x * kFrameEnergyTHFacMedian;
    th = 26.0f * kFrameEnergyTHConstWeight + th * (1 - kFrameEnergyTHConstWeight);
    th = th * th;
    th *= kOverallEnergyTHWeight * kOverallEnergyTHWeight;
    *th_out = th;
    return 0;
}

int ldso_ba_validate_window(const ldso_ba_window *w) {
    if (!w) return fail(-1, "null window");
    return check_window(*w);
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
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->n_cu <= 0)
        c->n_cu = 256;
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
    for (auto &g : c->opt_graph)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    for (auto &g : c->it_graph)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    drain_events(c);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->pin_sys) (void)hipHostFree(c->pin_sys);
    if (c->pin_xad) (void)hipHostFree(c->pin_xad);
    if (c->pin_step) (void)hipHostFree(c->pin_step);
    if (c->pin_out) (void)hipHostFree(c->pin_out);
    if (c->pin_map) (void)hipHostFree(c->pin_map);
    if (c->pin_in) (void)hipHostFree(c->pin_in);
    if (c->pin_in_ev) (void)hipEventDestroy(c->pin_in_ev);
    c->d_wins.release();
    c->d_img.release();
    c->d_act_in.release();
    c->d_act_out.release();
    c->d_precalc.release();
    c->d_frame_th.release();
    c->d_pt_data.release();
    c->d_pt_out.release();
    c->d_pt_step.release();
    c->d_adH.release();
    c->d_adT.release();
    c->d_rs_slot.release();
    c->d_pt_nres.release();
    c->d_pt_tgt.release();
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
    c->d_rec_a.release();
    c->d_rec_b.release();
    c->d_geo_snap.release();
    c->d_top_items.release();
    c->d_sc_items.release();
    c->d_adhtd.release();
    c->d_pair_items.release();
    c->d_host_items.release();
    c->d_top_slab.release();
    c->d_sc_slab.release();
    c->d_item_energy.release();
    c->d_sys.release();
    c->d_stage.release();
    c->d_sum_blocks.release();
    c->d_x_local.release();
    c->d_x_gathered.release();
    c->d_fstate.release();
    c->d_calib_val.release();
    c->d_calib_zero.release();
    c->d_cprior.release();
    c->d_ehist.release();
    c->d_stop.release();
    c->d_status.release();
    c->d_add_priors.release();
    if (c->comm) (void)ncclCommDestroy(c->comm);
    c->d_xad.release();
    c->d_sx_state.release();
    c->d_sx_newstate.release();
    c->d_sx_flags.release();
    c->d_sx_energy.release();
    c->d_sx_newenergy.release();
    c->d_sx_ewo.release();
    c->d_sx_center.release();
    c->d_sx_rec_a.release();
    c->d_sx_rec_b.release();
    c->d_sx_geo_snap.release();
    c->d_jp_out.release();
    c->d_pt_vals.release();
    c->d_sx_item.release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

void *ldso_ba_stream(ldso_ba_ctx *c) { return c ? (void *)c->stream : nullptr; }

}  // extern "C"

namespace {
// SURVEY.md §8e's partition: points in host-frame order, cut into shard_count contiguous runs of
// (as nearly as possible) equal residual counts, so a shard holds whole host frames except at
// its two ends (a host is split only where a cut falls inside it, e.g. when shards outnumber
// hosts).  Rank r owns the points whose first residual lies in [r T / G, (r + 1) T / G).
void shard_points(const ldso_ba_window &in, int rank, int count, std::vector<int> &out) {
    out.clear();
    // the device point order: host frames in window order, each host's points in features order
    // (point_rank; the caller's order without it)
    std::vector<int> order;
    order.reserve(in.n_points);
    for (int f = 0; f < in.n_frames; f++) {
        const size_t b = order.size();
        for (int p = 0; p < in.n_points; p++)
            if (in.point_host[p] == f) order.push_back(p);
        if (in.point_rank)
            std::stable_sort(order.begin() + b, order.end(),
                             [&](int a, int c) { return in.point_rank[a] < in.point_rank[c]; });
    }
    const long long T = in.n_residuals;
    long long acc = 0;
    for (int p : order) {
        const long long owner = T > 0 ? std::min<long long>(count - 1, acc * count / T) : p % count;
        if (owner == rank) out.push_back(p);
        acc += in.point_res_begin[p + 1] - in.point_res_begin[p];
    }
}

// parent != nullptr: a marginalisation context over `ws[0]` whose frames are the parent's window
// parent_win (images borrowed, not uploaded; priorF scaled by setting_idepthFixPriorMargFac)
int load_impl(ldso_ba_ctx *c, int32_t n_windows, const ldso_ba_window *ws, int32_t shard_rank, int32_t shard_count,
              const ldso_ba_ctx *parent, int parent_win) {
    if (!c || n_windows < 1 || !ws) return fail(-1, "bad arguments");
    if (shard_count < 1 || shard_rank < 0 || shard_rank >= shard_count) return fail(-1, "bad shard");
    c->th_host_valid = false;
    for (int w = 0; w < n_windows; w++) {
        int rc = check_window(ws[w], parent == nullptr);
        if (rc) return rc;
        if (ws[w].width != ws[0].width || ws[w].height != ws[0].height)
            return fail(-1, "all windows of a context must share the image size");
    }
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->n_win = n_windows;
    c->x_stride = 0;
    c->x_prun = 0;
    c->width = ws[0].width;
    c->height = ws[0].height;
    c->npix = c->width * c->height;
    c->marg = parent != nullptr;
    c->img_ext = nullptr;
    if (parent) {
        c->img_mode = parent->img_mode;
        c->tiles_per_row = parent->tiles_per_row;
        c->padded_h = parent->padded_h;
        c->frame_stride = parent->frame_stride;
        c->img_ext = parent->d_img.p + (size_t)parent->wd[parent_win].frame_base * parent->frame_stride;
    } else {
        image_geometry(c);
    }
    c->wh.assign(n_windows, WinHost());
    c->wd.assign(n_windows, WinDev());
    c->sys_host_valid = false;
    c->energy_valid = false;

    // host-side layout
    std::vector<int4> top_items, sc_items;
    std::vector<int2> pair_items, host_items;
    std::vector<int> pair_win, frame_win, rs_slot, pt_nres, pt_host;
    std::vector<unsigned long long> pt_tgt;
    int rec_base = 0;
    std::vector<uint8_t> rs_tgt, rs_flags;
    std::vector<int8_t> rs_state;
    std::vector<float> rs_energy, pt_data, precalc, frame_th;
    std::vector<double> adH, adT;
    long long sc_slab_total = 0, sys_total = 0, stage_total = 0;
    int vec_total = 0;
    std::vector<int> pt_win;
    // residuals per k_linearize wave: 64 when the grid is large anyway; small workloads (one
    // window) use shorter chunks so more waves start at once (latency, not throughput, bound)
    long long r_est = 0;
    for (int w = 0; w < n_windows; w++) r_est += ws[w].n_residuals;
    r_est /= shard_count;
    const int chunk = c->top_chunk ? c->top_chunk : r_est >= 64LL * 4096 ? 64 : r_est >= 32LL * 2048 ? 32 : 16;
    // k_point_sc points per block: 64 for large loads; a small load (one window: 32 blocks of 64
    // points on 256 CUs) takes 16-point blocks, whose SYRK chains are a quarter as long (one S7
    // window's pass 30 -> 28 us; optimize unchanged: its sumNID block is the longest there)
    const int sc_chunk = r_est < 64LL * 4096 ? 16 : kScPoints;
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
        // the priors (HL, bL) are not part of the reduced packed system: every rank adds them in
        // its own (redundant) solve, so every shard keeps them
        H.add_priors = true;
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
        // points of this shard (host-frame partition, shard_points)
        shard_points(in, shard_rank, shard_count, H.pt_orig);
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
        // item order 2: inside each bucket the residuals are ranked by their projection into the
        // target (row, then column) and dealt round robin, in groups of 8 consecutive ranks (one
        // phase-A step of a wavefront), over the bucket's chunks: every chunk of a bucket sweeps the
        // target image top to bottom and the concurrent chunks of one target are at the same band
        // at the same step (the target's live lines: one band, not the frame).  Chunks stay
        // multiples of 8 but the last, so the phase-A steps are the same as in order 0.
        std::vector<int> bucket_nch(N * N, 0);
        std::vector<int> chunk_len;  // item order 2: residuals per chunk, bucket by bucket
        if (c->item_order == 2) {
            std::vector<std::pair<std::pair<float, float>, int>> key;
            for (int b = 0; b < N * N; b++) {
                const int n = bucket_cnt[b];
                if (n == 0) continue;
                const float *pre = in.precalc + (size_t)b * LDSO_BA_PRECALC_STRIDE;  // PRE_KRKiTll, PRE_KtTll
                key.clear();
                for (int pos = bucket_start[b]; pos < bucket_start[b + 1]; pos++) key.push_back({{0.f, 0.f}, H.rs_orig[pos]});
                for (auto &e : key) {
                    const int k = e.second;  // its point: point_res_begin is sorted
                    const int p = (int)(std::upper_bound(in.point_res_begin, in.point_res_begin + in.n_points + 1, k) -
                                        in.point_res_begin) - 1;
                    const float *d = in.point_data + (size_t)p * LDSO_BA_POINT_STRIDE;
                    float q[3];
                    for (int i = 0; i < 3; i++) q[i] = pre[3 * i] * d[0] + pre[3 * i + 1] * d[1] + pre[3 * i + 2] + pre[9 + i] * d[2];
                    const float y = q[1] / q[2], x = q[0] / q[2];
                    e.first = {std::isfinite(y) ? y : 0.f, std::isfinite(x) ? x : 0.f};
                }
                std::sort(key.begin(), key.end());
                const int G = (n + 7) / 8, nch = (n + chunk - 1) / chunk;
                bucket_nch[b] = nch;
                std::vector<int> start(nch + 1, 0);
                for (int cc = 0; cc < nch; cc++) {
                    const int groups = (G - cc + nch - 1) / nch;  // groups cc, cc + nch, ...
                    int len = 8 * groups;
                    if ((G - 1) % nch == cc) len -= 8 * G - n;  // the last (short) group ends this chunk
                    start[cc + 1] = start[cc] + len;
                    chunk_len.push_back(len);
                }
                for (int i = 0; i < n; i++) {
                    const int g = i / 8, cc = g % nch;
                    const int pos = bucket_start[b] + start[cc] + 8 * (g / nch) + (i & 7);
                    H.rs_orig[pos] = key[i].second;
                    res_pos_of[key[i].second] = pos;
                }
            }
        }
        // per-residual arrays (global, sorted)
        for (int pos = 0; pos < R; pos++) {
            const int k = H.rs_orig[pos];
            rs_tgt.push_back((uint8_t)in.res_target[k]);
            rs_flags.push_back(in.res_flags[k]);
            rs_state.push_back(in.res_state[k]);
            rs_energy.push_back(in.res_energy[k]);
            rs_slot.push_back(0);
        }
        H.rs_slot.assign(R, 0);
        // per-point arrays
        H.pt_host.resize(P);
        for (int q = 0; q < P; q++) {
            const int p = H.pt_orig[q];
            H.pt_host[q] = in.point_host[p];
            pt_host.push_back(in.point_host[p]);
            pt_data.insert(pt_data.end(), in.point_data + (size_t)p * LDSO_BA_POINT_STRIDE,
                           in.point_data + (size_t)(p + 1) * LDSO_BA_POINT_STRIDE);
            if (c->marg)  // marginalizePointsF: p->priorF *= setting_idepthFixPriorMargFac (EnergyFunctional.cc:216)
                pt_data[pt_data.size() - LDSO_BA_POINT_STRIDE + 4] *= kIdepthFixPriorMargFac;
            const int b = in.point_res_begin[p], e = in.point_res_begin[p + 1];
            pt_nres.push_back(e - b);
            unsigned long long tg = 0;
            for (int k = 0; k < e - b; k++) {
                const int pos = res_pos_of[b + k];
                const int tgk = in.res_target[b + k], hk = in.point_host[p];
                const int slot = rec_base + (tgk < hk ? tgk : tgk - 1) * P + q;
                rs_slot[res_base + pos] = slot;
                H.rs_slot[pos] = slot;
                tg |= (unsigned long long)in.res_target[b + k] << (4 * k);
            }
            pt_tgt.push_back(tg);
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
        for (int i = 0; i < 4; i++) D.cdelta[i] = in.c_delta[i];
        D.p_all = in.n_points;  // numID counts every shard's points
        D.K = 8 * (N - 1) + 5;
        D.KP = (D.K + 3) / 4 * 4;
        const int nt = D.KP / 4;
        D.ntiles = nt * (nt + 1) / 2;
        smem_max = std::max(smem_max, sc_smem_bytes(D.KP));
        // top items: chunks of `chunk` residuals of one bucket (one wave each)
        D.top_item_base = (int)top_items.size();
        const size_t pi0 = pair_items.size();
        pair_items.resize(pi0 + (size_t)N * N);
        std::vector<int> chunk_off(N * N + 1, 0);  // item order 2: first chunk_len entry of each bucket
        for (int b = 0; b < N * N; b++) chunk_off[b + 1] = chunk_off[b] + bucket_nch[b];
        for (int bb = 0; bb < N * N; bb++) {
            // bucket b = h + N t; chunks in target-major order (the N-1 buckets reading one target
            // image run together) or host-major (the buckets of one host's points run together)
            const int b = c->item_order == 1 ? (bb / N) + N * (bb % N) : bb;
            const int first = (int)top_items.size();
            if (bucket_nch[b] > 0) {  // item order 2: the chunks dealt above
                int s0 = bucket_start[b];
                for (int cc = 0; cc < bucket_nch[b]; cc++) {
                    const int len = chunk_len[chunk_off[b] + cc];
                    top_items.push_back(make_int4(res_base + s0, len | (cc == 0 ? 1 << 16 : 0), pair_base + b, w));
                    s0 += len;
                }
            } else {
                for (int s = bucket_start[b]; s < bucket_start[b + 1]; s += chunk)  // bit 16: the pair's first chunk
                    top_items.push_back(make_int4(res_base + s, std::min(chunk, bucket_start[b + 1] - s) | (s == bucket_start[b] ? 1 << 16 : 0),
                                                  pair_base + b, w));
            }
            pair_items[pi0 + b] = make_int2(first, (int)top_items.size() - first);
        }
        for (int b = 0; b < N * N; b++) pair_win.push_back(w);
        D.n_top_items = (int)top_items.size() - D.top_item_base;
        // sc items: chunks of kScPoints points of one host
        D.sc_item_base = (int)sc_items.size();
        {
            int q = 0;
            for (int f = 0; f < N; f++) {
                const int first = (int)sc_items.size();
                int q0 = q;
                while (q < P && H.pt_host[q] == f) q++;
                for (int s = q0; s < q; s += sc_chunk)
                    sc_items.push_back(make_int4(point_base + s, std::min(sc_chunk, q - s), f, w));
                host_items.push_back(make_int2(first, (int)sc_items.size() - first));
                frame_win.push_back(w);
            }
        }
        D.n_sc_items = (int)sc_items.size() - D.sc_item_base;
        D.sc_slab_base = sc_slab_total;
        sc_slab_total += (long long)D.n_sc_items * D.ntiles * 16;
        D.sys_base = sys_total;
        sys_total += sys_len(D.D);
        D.stage_base = stage_total;
        // k_stitch's per-pair records, or k_stitch_host's per-host partial systems
        stage_total += std::max<long long>((long long)N * N * stage_rec(N), (long long)N * sys_len(D.D));
        D.newest_begin = res_base + bucket_start[N * (N - 1)];
        D.newest_end = res_base + bucket_start[N * N];
        D.rec_base = rec_base;
        D.vec_base = vec_total;
        vec_total += D.D;
        pt_win.insert(pt_win.end(), P, w);
        // frame-level inputs
        precalc.insert(precalc.end(), in.precalc, in.precalc + (size_t)N * N * LDSO_BA_PRECALC_STRIDE);
        adH.insert(adH.end(), in.ad_host, in.ad_host + (size_t)N * N * 64);
        adT.insert(adT.end(), in.ad_target, in.ad_target + (size_t)N * N * 64);
        frame_th.insert(frame_th.end(), in.frame_energy_th, in.frame_energy_th + N);
        frame_base += N;
        pair_base += N * N;
        point_base += P;
        rec_base += P * (N - 1);
        res_base += R;
    }
    c->n_top_items = (int)top_items.size();
    c->n_sc_items = (int)sc_items.size();
    c->n_pairs = pair_base;
    c->n_frames = frame_base;
    c->max_frames = 0;
    for (int w = 0; w < n_windows; w++) c->max_frames = std::max(c->max_frames, ws[w].n_frames);
    c->host_stitch = c->max_frames <= kHostStitchMaxN && !getenv_flag("LDSO_BA_STITCH_RECORDS");
    c->P_tot = point_base;
    c->vec_total = vec_total;
    c->R_tot = res_base;
    c->sc_smem_max = smem_max;

    int rc = 0;
#define ALLOC(buf, n)                   \
    do {                                \
        rc = (buf).alloc(n);            \
        if (rc) return rc;              \
    } while (0)
    ALLOC(c->d_wins, n_windows);
    if (c->marg) c->d_img.release();
    else ALLOC(c->d_img, (size_t)c->n_frames * c->frame_stride);
    if (c->marg) ALLOC(c->d_adhtd, (size_t)c->n_pairs * 8);
    ALLOC(c->d_precalc, precalc.size());
    ALLOC(c->d_frame_th, frame_th.size());
    ALLOC(c->d_pt_data, std::max<size_t>(1, pt_data.size()));
    ALLOC(c->d_pt_out, std::max<size_t>(1, (size_t)c->P_tot * 12));
    ALLOC(c->d_pt_step, std::max<size_t>(1, (size_t)c->P_tot));
    ALLOC(c->d_pt_host, std::max<size_t>(1, pt_host.size()));
    ALLOC(c->d_adH, adH.size());
    ALLOC(c->d_adT, adT.size());
    ALLOC(c->d_pt_nres, std::max<size_t>(1, pt_nres.size()));
    ALLOC(c->d_rs_slot, std::max<size_t>(1, rs_slot.size()));
    ALLOC(c->d_pt_tgt, std::max<size_t>(1, pt_tgt.size()));
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
    ALLOC(c->d_rec_a, std::max<size_t>(1, (size_t)rec_base));
    ALLOC(c->d_rec_b, std::max<size_t>(1, (size_t)rec_base));
    ALLOC(c->d_geo_snap, std::max<size_t>(1, (size_t)pair_base * kGeoSnap));
    ALLOC(c->d_top_items, std::max<size_t>(1, top_items.size()));
    ALLOC(c->d_sc_items, std::max<size_t>(1, sc_items.size()));
    ALLOC(c->d_pair_items, pair_items.size());
    ALLOC(c->d_host_items, host_items.size());
    ALLOC(c->d_top_slab, std::max<size_t>(1, top_items.size() * kTopVals));
    ALLOC(c->d_sc_slab, std::max<size_t>(1, (size_t)sc_slab_total));
    ALLOC(c->d_item_energy, std::max<size_t>(1, top_items.size() * 2));
    ALLOC(c->d_sys, (size_t)sys_total + 4 * (size_t)n_windows);  // + win_energy() + win_nid()
    c->sys_n = (size_t)sys_total;
    ALLOC(c->d_stage, (size_t)std::max<long long>(1, stage_total));
    {
        std::vector<int2> sb;
        for (int w = 0; w < n_windows; w++) {
            const long long n_el = sys_len(c->wd[w].D);
            for (long long e0 = 0; e0 < n_el; e0 += 256) sb.push_back(make_int2(w, (int)e0));
        }
        c->n_sum_blocks = (int)sb.size();
        ALLOC(c->d_sum_blocks, sb.size());
        HIP_TRY(hipMemcpyAsync(c->d_sum_blocks.p, sb.data(), sb.size() * sizeof(int2), hipMemcpyHostToDevice, c->stream));
    }
    ALLOC(c->d_xad, (size_t)n_windows * kXadStride);
    ALLOC(c->d_prior, (size_t)2 * vec_total);
    ALLOC(c->d_x, (size_t)vec_total);
    ALLOC(c->d_ns, (size_t)7 * vec_total);
    ALLOC(c->d_ns_nm, (size_t)7 * vec_total);
    ALLOC(c->d_ns_g, (size_t)kPrepGStride * n_windows);
    c->ns_cache.clear();
    c->ns_cache_null = -1;
    ALLOC(c->d_pt_win, std::max<size_t>(1, pt_win.size()));
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
    UP(c->d_pt_nres, pt_nres);
    UP(c->d_rs_slot, rs_slot);
    UP(c->d_pt_tgt, pt_tgt);
    UP(c->d_pt_win, pt_win);
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
    HIP_TRY(hipMemsetAsync(c->d_rec_a.p, 0, c->d_rec_a.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_rec_b.p, 0xFF, c->d_rec_b.bytes(), c->stream));  // NaN: not active
    HIP_TRY(hipMemsetAsync(c->d_geo_snap.p, 0, c->d_geo_snap.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_pt_out.p, 0, c->d_pt_out.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_pt_step.p, 0, c->d_pt_step.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_sys.p, 0, c->d_sys.bytes(), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_rs_newstate.p, LDSO_BA_RES_OUTLIER, c->d_rs_newstate.bytes(), c->stream));
    {
        std::vector<float> neg(rs_energy.size(), -1.0f);
        rc = up(c->d_rs_energy_wo.p, neg.data(), neg.size() * sizeof(float));
        if (rc) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    // images: per frame through a float3 staging buffer, repacked on the device; the
    // intensity-only layout falls back to 2x4 float4 tiles if the caller's gradients are not
    // makeImages' (then recomputing them would not be exact)
    if (!c->marg) {
        int mismatch = 0;
        rc = stage_images(c, ws, n_windows, &mismatch);
        if (rc) return rc;
        if (c->img_mode == 3 && mismatch) {
            c->img_mode = 1;
            image_geometry(c);
            rc = c->d_img.alloc((size_t)c->n_frames * c->frame_stride);
            if (rc) return rc;
            rc = stage_images(c, ws, n_windows, &mismatch);
            if (rc) return rc;
        }
    }
    if (c->sc_smem_max > 64 * 1024) {
        HIP_TRY(hipFuncSetAttribute((const void *)k_point_sc, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)c->sc_smem_max));
    }
    for (int w = 0; w < n_windows; w++) {
        rc = upload_priors(c, w);
        if (rc) return rc;
    }
    return 0;
}
}  // namespace

extern "C" {

int ldso_ba_load(ldso_ba_ctx *c, int32_t n_windows, const ldso_ba_window *ws, int32_t shard_rank,
                 int32_t shard_count) {
    return load_impl(c, n_windows, ws, shard_rank, shard_count, nullptr, 0);
}

int ldso_ba_load_marginalization(ldso_ba_ctx *marg, const ldso_ba_ctx *parent, int32_t parent_win,
                                 const ldso_ba_window *points) {
    if (!marg || !parent || !points || marg == parent) return fail(-1, "bad arguments");
    if (parent_win < 0 || parent_win >= parent->n_win) return fail(-1, "parent window out of range");
    if (marg->device != parent->device) return fail(-1, "contexts on different devices");
    const WinDev &pw = parent->wd[parent_win];
    if (points->n_frames != pw.N || points->width != pw.width || points->height != pw.height)
        return fail(-1, "marginalisation window does not match the parent window's frames");
    marg->settings = parent->settings;  // the parent's affine modes shape res_toZeroF and Jab_r
    return load_impl(marg, 1, points, 0, 1, parent, parent_win);
}

int ldso_ba_update(ldso_ba_ctx *c, int32_t win, const ldso_ba_window *w) {
    if (!c || !w || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    c->th_host_valid = false;
    WinHost &H = c->wh[win];
    WinDev &D = c->wd[win];
    if (w->n_frames != H.N || w->n_points != H.P_all || w->n_residuals != H.R_all)
        return fail(-1, "update() cannot change the window structure; call ldso_ba_load");
    const int N = H.N;
    HIP_TRY(hipSetDevice(c->device));
    for (int i = 0; i < 4; i++) D.calib[i] = w->calib[i];
    H.c_prior.assign(w->c_prior, w->c_prior + 4);
    H.c_delta.assign(w->c_delta, w->c_delta + 4);
    H.frame_prior.assign(w->frame_prior, w->frame_prior + 8 * N);
    H.frame_delta_prior.assign(w->frame_delta_prior, w->frame_delta_prior + 8 * N);
    for (size_t k = 0; k < H.adHF.size(); k++) {
        H.adHF[k] = (float)w->ad_host[k];
        H.adTF[k] = (float)w->ad_target[k];
    }
    std::vector<float> pd(w->point_data ? (size_t)H.P * LDSO_BA_POINT_STRIDE : 0);
    if (w->point_data)
        for (int q = 0; q < H.P; q++)
            std::memcpy(&pd[(size_t)q * LDSO_BA_POINT_STRIDE],
                        w->point_data + (size_t)H.pt_orig[q] * LDSO_BA_POINT_STRIDE, LDSO_BA_POINT_STRIDE * sizeof(float));
    std::vector<double> pr;
    priors_vector(c, win, pr);
    // every array of the update through the mapped staging buffer in one launch, stream-ordered
    // (the caller's arrays are copied before this returns; no synchronisation)
    InBatch B;
    B.add(c->d_wins.p + win, &D, sizeof(WinDev));
    B.add(c->d_precalc.p + (size_t)D.pair_base * LDSO_BA_PRECALC_STRIDE, w->precalc,
          (size_t)N * N * LDSO_BA_PRECALC_STRIDE * sizeof(float));
    B.add(c->d_adH.p + (size_t)D.pair_base * 64, w->ad_host, (size_t)N * N * 64 * sizeof(double));
    B.add(c->d_adT.p + (size_t)D.pair_base * 64, w->ad_target, (size_t)N * N * 64 * sizeof(double));
    B.add(c->d_frame_th.p + D.frame_base, w->frame_energy_th, N * sizeof(float));
    B.add(c->d_prior.p + (size_t)2 * D.vec_base, pr.data(), pr.size() * sizeof(double));
    if (H.P && w->point_data)
        B.add(c->d_pt_data.p + (size_t)D.point_base * LDSO_BA_POINT_STRIDE, pd.data(), pd.size() * sizeof(float));
    c->sys_host_valid = false;
    return B.flush(c);
}

int ldso_ba_update_points(ldso_ba_ctx *c, int32_t win, const float *vals) {
    if (!c || win < 0 || win >= c->n_win || (!vals && c->wh[win].P_all > 0)) return fail(-1, "bad arguments");
    const WinHost &H = c->wh[win];
    const WinDev &D = c->wd[win];
    if (H.P == 0) return 0;
    HIP_TRY(hipSetDevice(c->device));
    int rc = c->d_pt_vals.ensure((size_t)c->P_tot);
    if (rc) return rc;
    if ((rc = pin_ensure(c->pin_out, c->pin_out_n, (size_t)H.P * sizeof(float4)))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));  // pin_out may feed an earlier copy
    float4 *st = reinterpret_cast<float4 *>(c->pin_out);
    for (int q = 0; q < H.P; q++) {
        const float *v = vals + 4 * (size_t)H.pt_orig[q];
        st[q] = make_float4(v[0], v[1], v[2], v[3]);
    }
    HIP_TRY(hipMemcpyAsync(c->d_pt_vals.p + D.point_base, st, (size_t)H.P * sizeof(float4), hipMemcpyHostToDevice,
                           c->stream));
    k_set_point_vals<<<(H.P + 255) / 256, 256, 0, c->stream>>>(c->d_pt_vals.p + D.point_base,
                                                              c->d_pt_data.p + (size_t)D.point_base * LDSO_BA_POINT_STRIDE, H.P);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int ldso_ba_update_residuals(ldso_ba_ctx *c, int32_t win, const int8_t *state, const float *state_energy,
                             const float *new_energy, const uint8_t *flags) {
    if (!c || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    const WinHost &H = c->wh[win];
    const WinDev &D = c->wd[win];
    if (D.R == 0) return 0;
    if (!state || !state_energy || !new_energy || !flags) return fail(-1, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const size_t R = (size_t)D.R;
    int rc = pin_ensure(c->pin_out, c->pin_out_n, R * (2 * sizeof(float) + 2));
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    float *se = reinterpret_cast<float *>(c->pin_out), *ne = se + R;
    int8_t *st = reinterpret_cast<int8_t *>(ne + R);
    uint8_t *fl = reinterpret_cast<uint8_t *>(st + R);
    for (size_t pos = 0; pos < R; pos++) {
        const int k = H.rs_orig[pos];
        se[pos] = state_energy[k];
        ne[pos] = new_energy[k];
        st[pos] = state[k];
        fl[pos] = flags[k];
    }
    HIP_TRY(hipMemcpyAsync(c->d_rs_energy.p + D.res_base, se, R * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_rs_newenergy.p + D.res_base, ne, R * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_rs_state.p + D.res_base, st, R, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_rs_flags.p + D.res_base, fl, R, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int ldso_ba_reset_oob(ldso_ba_ctx *c, int32_t win) {
    if (!c || win >= c->n_win) return fail(-1, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    // resetOOB(): state_NewEnergy = state_energy = 0; state_NewState = OUTLIER; state_state = IN,
    // for the windows' residual range (contiguous: windows back to back) in one launch instead of
    // four fills per window
    const int w0 = win < 0 ? 0 : win, w1 = win < 0 ? c->n_win : win + 1;
    const long long r0 = c->wd[w0].res_base, r1 = c->wd[w1 - 1].res_base + c->wd[w1 - 1].R;
    if (r1 <= r0) return 0;
    const int n = (int)(r1 - r0);
    k_reset_oob<<<std::min(1024, (n + 255) / 256), 256, 0, c->stream>>>(
        c->d_rs_state.p + r0, c->d_rs_newstate.p + r0, c->d_rs_energy.p + r0, c->d_rs_newenergy.p + r0, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"

namespace {
#define NCCL_TRY(expr)                                                                            \
    do {                                                                                          \
        ncclResult_t r_ = (expr);                                                                 \
        if (r_ != ncclSuccess) return fail(-2, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// SURVEY.md §8e's exchange, stream-ordered after k_stitch on the context stream (no host
// synchronisation): one fp64 sum all-reduce of every window's packed {HA, bA, Hsc, bsc} (the priors
// are not in it: every rank adds its own copy in the solve) and of the linearizeAll energy / #IN
// pairs, then an all-gather of per-window slots -- the newest-frame NewEnergyWithOutlier values,
// after which k_frame_th re-selects the exact setNewFrameEnergyTH threshold on every rank, and,
// inside ldso_ba_optimize, the rank's run of |idepth|, from which every rank walks the window's
// whole sumNID chain (doStepFromBackup's float sum in the unsharded order: nid_source).
int comm_exchange(ldso_ba_ctx *c, bool accumulate) {
    hipStream_t st = c->stream;
    if (c->x_stride == 0) {  // first exchange since the load: agree on the slot stride and run length
        int64_t m[2] = {1, 0};
        for (const WinDev &D : c->wd) {
            m[0] = std::max<int64_t>(m[0], D.newest_end - D.newest_begin);
            m[1] = std::max<int64_t>(m[1], D.P);
        }
        m[1] = (m[1] + 3) & ~(int64_t)3;  // the chain reads float4s of one rank's run
        DevBuf<int64_t> t;
        if (int rc = t.alloc(2)) return rc;
        HIP_TRY(hipMemcpyAsync(t.p, m, sizeof(m), hipMemcpyHostToDevice, st));
        NCCL_TRY(ncclAllReduce(t.p, t.p, 2, ncclInt64, ncclMax, c->comm, st));
        HIP_TRY(hipMemcpyAsync(m, t.p, sizeof(m), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        t.release();
        c->x_stride = m[0];
        c->x_prun = m[1];
        const size_t slot_max = (size_t)(m[0] + m[1]);
        if (int rc = c->d_x_local.alloc((size_t)c->n_win * slot_max)) return rc;
        if (int rc = c->d_x_gathered.alloc((size_t)c->comm_world * c->n_win * slot_max)) return rc;
    }
    const size_t nw2 = (size_t)2 * c->n_win;
    double *xb = accumulate ? c->d_sys.p : c->win_energy();
    const size_t xn = (accumulate ? c->sys_n : 0) + nw2;
    NCCL_TRY(ncclAllReduce(xb, xb, xn, ncclFloat64, ncclSum, c->comm, st));
    // inside optimize() an accumulating pass also ships the idepth runs of the next step's sumNID
    const bool nid = c->opt_pass >= 0 && accumulate;
    const long long stride = c->x_stride, prun = nid ? c->x_prun : 0, slot = stride + prun;
    const dim3 grid((unsigned)std::min<long long>((slot + 255) / 256, 64), (unsigned)c->n_win);
    k_export_newest<<<grid, 256, 0, st>>>(c->d_wins.p, c->d_rs_energy_wo.p, c->d_x_local.p, stride, slot,
                                          c->d_pt_data.p, (int)prun);
    HIP_TRY(hipGetLastError());
    NCCL_TRY(ncclAllGather(c->d_x_local.p, c->d_x_gathered.p, (size_t)c->n_win * slot, ncclFloat32, c->comm, st));
    // the chains run here when the solve does not host them (exact solve modes)
    const bool chain_here = nid && !nid_in_solve(c);
    NidSrc src = chain_here ? nid_source(c) : NidSrc{};
    const int* stop = c->opt_pass >= 0 ? c->d_stop.p : nullptr;
    return timed_launch(c, 4, st, [&] {
        k_frame_th<<<c->n_win * (chain_here ? 2 : 1), kStThreads, 0, st>>>(
            c->d_wins.p, c->d_x_gathered.p, c->comm_world, c->n_win, stride, slot, c->d_frame_th.p, src,
            chain_here ? c->win_nid() : nullptr, stop, c->opt_pass);
    });
}
}  // namespace

extern "C" {

int ldso_ba_comm_unique_id(uint8_t *id_out) {
    if (!id_out) return fail(-1, "null id");
    static_assert(sizeof(ncclUniqueId) == LDSO_BA_COMM_ID_BYTES, "RCCL unique id size");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return 0;
}

int ldso_ba_comm_init(ldso_ba_ctx *c, const uint8_t *id_in, int32_t rank, int32_t world) {
    if (!c || !id_in || world < 1 || rank < 0 || rank >= world) return fail(-1, "bad arguments");
    if (c->comm) return fail(-1, "communicator already initialised");
    HIP_TRY(hipSetDevice(c->device));
    ncclUniqueId id;
    std::memcpy(&id, id_in, sizeof(id));
    NCCL_TRY(ncclCommInitRank(&c->comm, world, id, rank));
    c->comm_rank = rank;
    c->comm_world = world;
    c->x_stride = 0;
    c->x_prun = 0;
    return 0;
}

int ldso_ba_linearize(ldso_ba_ctx *c, int32_t fix, int32_t accumulate) {
    if (!c || c->n_win == 0) return fail(-1, "no windows loaded");
    int rc;
    if ((rc = ldso_ba_check_settings(&c->settings))) return rc;
    HIP_TRY(hipSetDevice(c->device));
    c->sys_host_valid = false;
    c->energy_valid = false;
    c->th_host_valid = false;
    LinParams L{};
    L.items = c->d_top_items.p;
    L.wins = c->d_wins.p;
    L.img = c->img_ext ? c->img_ext : c->d_img.p;
    L.ad_ht_delta = c->marg ? c->d_adhtd.p : nullptr;
    L.precalc = c->d_precalc.p;
    L.frame_th = c->d_frame_th.p;
    L.rs_slot = c->d_rs_slot.p;
    L.pt_data = c->d_pt_data.p;
    L.rs_state = c->d_rs_state.p;
    L.rs_newstate = c->d_rs_newstate.p;
    L.rs_flags = c->d_rs_flags.p;
    L.rs_energy = c->d_rs_energy.p;
    L.rs_newenergy = c->d_rs_newenergy.p;
    L.rs_energy_wo = c->d_rs_energy_wo.p;
    L.rs_center = reinterpret_cast<float *>(c->d_rs_center.p);
    L.center_stride = c->R_tot;
    L.rec_a = c->d_rec_a.p;
    L.rec_b = c->d_rec_b.p;
    L.geo_snap = c->d_geo_snap.p;
    L.top_slab = c->d_top_slab.p;
    L.item_energy = c->d_item_energy.p;
    L.frame_stride = c->frame_stride;
    L.tiles_per_row = c->tiles_per_row;
    L.fix = fix;
    L.accumulate = accumulate;
    L.aff_fix = aff_fix_bits(c);
    L.item_base = 0;
    L.n_items = c->n_top_items;
    L.n_blocks = (L.n_items + 3) / 4;
    PointParams Pp{};
    Pp.items = c->d_sc_items.p;
    Pp.wins = c->d_wins.p;
    Pp.pt_data = c->d_pt_data.p;
    Pp.pt_nres = c->d_pt_nres.p;
    Pp.pt_tgt = c->d_pt_tgt.p;
    Pp.rec_a = c->d_rec_a.p;
    Pp.rec_b = c->d_rec_b.p;
    Pp.precalc = c->d_precalc.p;
    Pp.pt_out = c->d_pt_out.p;
    Pp.sc_slab = c->d_sc_slab.p;
    Pp.shift_prior = c->marg ? 0 : 1;
    Pp.item_base = 0;
    Pp.n_items = c->n_sc_items;
    StitchParams Sp{};
    Sp.wins = c->d_wins.p;
    Sp.pair_win = c->d_pair_win.p;
    Sp.e_wo = c->d_rs_energy_wo.p;
    Sp.frame_th = c->d_frame_th.p;
    Sp.pair_items = c->d_pair_items.p;
    Sp.top_slab = c->d_top_slab.p;
    Sp.item_energy = c->d_item_energy.p;
    Sp.host_items = c->d_host_items.p;
    Sp.sc_slab = c->d_sc_slab.p;
    Sp.adH = c->d_adH.p;
    Sp.adT = c->d_adT.p;
    Sp.sys = c->d_sys.p;
    Sp.stage = c->d_stage.p;
    Sp.win_energy = c->win_energy();
    const bool in_opt = c->opt_pass >= 0;
    Sp.ehist = in_opt && !c->comm ? c->d_ehist.p : nullptr;  // with RCCL: after the exchange
    Sp.pass = c->opt_pass;
    Sp.stop = in_opt ? c->d_stop.p : nullptr;
    L.stop = Sp.stop;
    L.pass = c->opt_pass;
    Pp.stop = Sp.stop;
    Pp.pass = c->opt_pass;
    const size_t sc_smem = std::max<size_t>(c->sc_smem_max, 4096);  // point_nid stages >= 1024 idepths
    if (in_opt && accumulate && !nid_in_solve(c) && !c->comm) {  // the next step's sumNID / numID (its backup idepths are this pass's)
        Pp.win_nid = c->win_nid();
        Pp.n_nid = c->n_win;
        Pp.nid_chunk = (int)std::min<size_t>(1024, (sc_smem / sizeof(float)) & ~(size_t)3);
    }
    Sp.accumulate = accumulate;
    Sp.pair_base = 0;
    Sp.win_base = 0;
    Sp.n_win = c->n_win;
    int kp_max = 0, n_max = 2;
    for (const WinDev &D : c->wd) {
        kp_max = std::max(kp_max, D.KP);
        n_max = std::max(n_max, D.N);
    }
    Sp.frame_win = c->d_frame_win.p;
    Sp.frame_base = 0;
    // two 512-thread blocks fit a CU: split the host blocks when the doubled grid still runs at once
    Sp.hs_split = Sp.n_win + 2 * c->n_frames <= 2 * c->n_cu ? 1 : 0;
    if (const char *e = std::getenv("LDSO_BA_HS_SPLIT")) Sp.hs_split = e[0] == '1';  // tests: force either
    const size_t st_smem = c->host_stitch ? stitch_host_smem_bytes(n_max, &Sp.th_cap)
                                          : stitch_smem_bytes(kp_max, n_max, &Sp.th_cap);
    hipStream_t st = c->stream;
    if (L.n_items > 0) {
        rc = timed_launch_ext(c, 0, st, [&](hipEvent_t a, hipEvent_t b) {
            if (c->marg) launch_linearize<true>(c->img_mode, L.n_blocks, st, L, a, b);
            else launch_linearize<false>(c->img_mode, L.n_blocks, st, L, a, b);
        });
        if (rc) return rc;
    }
    if (accumulate && Pp.n_nid + Pp.n_items > 0) {
        rc = timed_launch(c, 1, st,
                          [&] { k_point_sc<<<Pp.n_nid + Pp.n_items, kScThreads, sc_smem, st>>>(Pp); });
        if (rc) return rc;
    }
    if (c->host_stitch) {
        static std::once_flag once;
        std::call_once(once, [] {
            int th;
            (void)hipFuncSetAttribute((const void *)k_stitch_host, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)stitch_host_smem_bytes(kHostStitchMaxN, &th));
        });
        rc = timed_launch(c, 2, st, [&] { k_stitch_host<<<Sp.n_win + (Sp.hs_split ? 2 : 1) * c->n_frames, kHsThreads, st_smem, st>>>(Sp);
        });
        if (!rc && accumulate)
            rc = timed_launch(c, 7, st, [&] {
                k_stitch_host_sum<<<c->n_sum_blocks, 256, 0, st>>>(c->d_wins.p, c->d_sum_blocks.p, c->d_stage.p,
                                                                   c->d_sys.p);
            });
    } else {
        rc = timed_launch(c, 2, st, [&] { k_stitch<<<Sp.n_win + c->n_pairs, kStThreads, st_smem, st>>>(Sp); });
        if (!rc && accumulate)
            rc = timed_launch(c, 7, st, [&] {
                k_stitch_sum<<<c->n_sum_blocks, 256, 0, st>>>(c->d_wins.p, c->d_sum_blocks.p, c->d_stage.p, c->d_sys.p);
            });
    }
    if (rc || !c->comm) return rc;
    rc = comm_exchange(c, accumulate != 0);
    if (!rc && in_opt) {  // the reduced energies into the optimize() history
        k_energy_to_history<<<1, 256, 0, st>>>(c->win_energy(), c->d_ehist.p, c->opt_pass, 2 * c->n_win);
        HIP_TRY(hipGetLastError());
    }
    return rc;
}

// k_record_jpjdf into d_jp_out and down to the host: [R][8] in device order
int record_jpjdf(ldso_ba_ctx *c, int win, const float4 *rec_a, const float2 *rec_b, const float *geo_snap,
                 std::vector<float> &out) {
    const WinDev &D = c->wd[win];
    int rc = c->d_jp_out.ensure((size_t)D.R * 8);
    if (rc) return rc;
    k_record_jpjdf<<<(D.R + 255) / 256, 256, 0, c->stream>>>(c->d_wins.p, win, c->d_rs_slot.p, c->d_pt_host.p,
                                                            c->d_pt_data.p, rec_a, rec_b, geo_snap, c->d_jp_out.p);
    HIP_TRY(hipGetLastError());
    out.resize((size_t)D.R * 8);
    HIP_TRY(hipMemcpyAsync(out.data(), c->d_jp_out.p, out.size() * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    return 0;
}

int ldso_ba_linearize_residuals(ldso_ba_ctx *c, int32_t win, int8_t *new_state, float *new_energy,
                                float *new_energy_wo, float *center, uint8_t *center_ok, float *jpjdf) {
    if (!c || win < 0 || win >= c->n_win) return fail(-1, "bad arguments");
    if (c->marg) return fail(-1, "not on a marginalisation context");
    const WinDev &D = c->wd[win];
    const WinHost &H = c->wh[win];
    // every caller slot is written: a sharded window holds only its run of the residuals
    if (H.R_all != D.R) return fail(-1, "ldso_ba_linearize_residuals: the window is sharded (single-shard only)");
    HIP_TRY(hipSetDevice(c->device));
    const size_t R = (size_t)D.R;
    if (R == 0 || D.n_top_items == 0) return 0;  // no residuals: nothing to write
    int rc;
    const size_t Rt = (size_t)c->R_tot, slots = c->d_rec_a.n;
    if ((rc = c->d_sx_state.ensure(Rt)) || (rc = c->d_sx_newstate.ensure(Rt)) || (rc = c->d_sx_flags.ensure(Rt)) ||
        (rc = c->d_sx_energy.ensure(Rt)) || (rc = c->d_sx_newenergy.ensure(Rt)) || (rc = c->d_sx_ewo.ensure(Rt)) ||
        (rc = c->d_sx_center.ensure(Rt)) || (rc = c->d_sx_rec_a.ensure(slots)) || (rc = c->d_sx_rec_b.ensure(slots)) ||
        (rc = c->d_sx_geo_snap.ensure(c->d_geo_snap.n)) ||
        (rc = c->d_sx_item.ensure((size_t)2 * c->n_top_items)))
        return rc;
    hipStream_t st = c->stream;
    const size_t b = (size_t)D.res_base;
    // resetOOB() of every residual of the window on the copies: state IN, NewState OUTLIER,
    // energies 0; the centre marked "not projected" (NaN) so a failed centre projection shows
    if (R) {  // one launch for the five fills and the flag copy
        k_reset_oob<<<std::min<int>(1024, (int)((R + 255) / 256)), 256, 0, st>>>(
            c->d_sx_state.p + b, c->d_sx_newstate.p + b, c->d_sx_energy.p + b, c->d_sx_newenergy.p + b, (int)R,
            reinterpret_cast<float *>(c->d_sx_center.p) + b, (long long)Rt, c->d_sx_flags.p + b, c->d_rs_flags.p + b);
        HIP_TRY(hipGetLastError());
    }
    LinParams L{};
    L.aff_fix = aff_fix_bits(c);
    L.items = c->d_top_items.p;
    L.wins = c->d_wins.p;
    L.img = c->img_ext ? c->img_ext : c->d_img.p;
    L.ad_ht_delta = nullptr;
    L.precalc = c->d_precalc.p;
    L.frame_th = c->d_frame_th.p;
    L.rs_slot = c->d_rs_slot.p;
    L.pt_data = c->d_pt_data.p;
    L.rs_state = c->d_sx_state.p;
    L.rs_newstate = c->d_sx_newstate.p;
    L.rs_flags = c->d_sx_flags.p;
    L.rs_energy = c->d_sx_energy.p;
    L.rs_newenergy = c->d_sx_newenergy.p;
    L.rs_energy_wo = c->d_sx_ewo.p;
    L.rs_center = reinterpret_cast<float *>(c->d_sx_center.p);
    L.center_stride = (long long)Rt;
    L.rec_a = c->d_sx_rec_a.p;
    L.rec_b = c->d_sx_rec_b.p;
    L.geo_snap = c->d_sx_geo_snap.p;
    L.top_slab = nullptr;
    L.item_energy = c->d_sx_item.p;
    L.frame_stride = c->frame_stride;
    L.tiles_per_row = c->tiles_per_row;
    L.fix = 0;
    L.accumulate = 0;
    L.item_base = D.top_item_base;
    L.n_items = D.n_top_items;
    L.n_blocks = (L.n_items + 3) / 4;
    rc = timed_launch(c, 0, st, [&] {
        if (c->marg) launch_linearize<true>(c->img_mode, L.n_blocks, st, L);
        else launch_linearize<false>(c->img_mode, L.n_blocks, st, L);
    });
    if (rc) return rc;
    std::vector<int8_t> ns(R);
    std::vector<float> ne(R), ew(R);
    std::vector<float4> ce(R);
    HIP_TRY(hipMemcpyAsync(ns.data(), c->d_sx_newstate.p + b, R, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(ne.data(), c->d_sx_newenergy.p + b, R * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(ew.data(), c->d_sx_ewo.p + b, R * sizeof(float), hipMemcpyDeviceToHost, st));
    for (int k = 0; k < 4; k++)  // the planes back into (x, y, z, relBS) per residual
        HIP_TRY(hipMemcpy2DAsync(reinterpret_cast<float *>(ce.data()) + k, sizeof(float4),
                                 reinterpret_cast<const float *>(c->d_sx_center.p) + (size_t)k * Rt + b, sizeof(float),
                                 sizeof(float), R, hipMemcpyDeviceToHost, st));
    std::vector<float> jp;
    if (jpjdf && (rc = record_jpjdf(c, win, c->d_sx_rec_a.p, c->d_sx_rec_b.p, c->d_sx_geo_snap.p, jp))) return rc;
    if ((rc = ldso_ba_sync(c))) return rc;
    for (size_t pos = 0; pos < R; pos++) {
        const int k = H.rs_orig[pos];
        const bool cok = !std::isnan(ce[pos].x);
        if (new_state) new_state[k] = ns[pos];
        if (new_energy) new_energy[k] = ne[pos];
        if (new_energy_wo) new_energy_wo[k] = ew[pos];
        if (center_ok) center_ok[k] = cok ? 1 : 0;
        if (center) {
            center[3 * k] = cok ? ce[pos].x : 0.f;
            center[3 * k + 1] = cok ? ce[pos].y : 0.f;
            center[3 * k + 2] = cok ? ce[pos].z : 0.f;
        }
        if (jpjdf) {
            float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (ns[pos] == LDSO_BA_RES_IN) std::memcpy(v, &jp[8 * pos], sizeof(v));
            std::memcpy(jpjdf + 8 * (size_t)k, v, sizeof(v));
        }
    }
    return 0;
}

int ldso_ba_activate_points(ldso_ba_ctx *c, int32_t win, int32_t n, const ldso_ct_immature *pts, int32_t min_obs,
                            ldso_ba_activation *out) {
    if (!c || win < 0 || win >= c->n_win || n < 0 || (n > 0 && (!pts || !out))) return fail(-1, "bad arguments");
    const int N = c->wh[win].N;
    for (int k = 0; k < n; k++)
        if (pts[k].host < 0 || pts[k].host >= N) return fail(-1, "immature point host index outside the window");
    if (n == 0) return 0;
    HIP_TRY(hipSetDevice(c->device));
    if ((size_t)n > c->d_act_in.n || (size_t)n > c->d_act_out.n || !c->d_act_in.p || !c->d_act_out.p) {
        int rc = c->d_act_in.alloc(n);
        if (!rc) rc = c->d_act_out.alloc(n);
        if (rc) return rc;
    }
    HIP_TRY(hipMemcpyAsync(c->d_act_in.p, pts, (size_t)n * sizeof(ldso_ct_immature), hipMemcpyHostToDevice, c->stream));
    ActParams A;
    A.wins = c->d_wins.p;
    A.img = c->img_ext ? c->img_ext : c->d_img.p;
    A.precalc = c->d_precalc.p;
    A.pts = c->d_act_in.p;
    A.out = c->d_act_out.p;
    A.frame_stride = c->frame_stride;
    A.tpr = c->tiles_per_row;
    A.img_mode = c->img_mode;
    A.win = win;
    A.n = n;
    A.min_obs = min_obs;
    int rc = timed_launch(c, 6, c->stream, [&] { k_activate<<<(n + 3) / 4, 256, 0, c->stream>>>(A); });
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, c->d_act_out.p, (size_t)n * sizeof(ldso_ba_activation), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int ldso_ba_marginalize_points(ldso_ba_ctx *c, const float *ad_ht_delta, double *H, double *b) {
    if (!c || !ad_ht_delta || !H || !b) return fail(-1, "bad arguments");
    if (!c->marg || c->n_win != 1) return fail(-1, "not a marginalisation context (ldso_ba_load_marginalization)");
    HIP_TRY(hipSetDevice(c->device));
    const WinDev &D = c->wd[0];
    HIP_TRY(hipMemcpyAsync(c->d_adhtd.p, ad_ht_delta, (size_t)D.N * D.N * 8 * sizeof(float), hipMemcpyHostToDevice,
                           c->stream));
    int rc = ldso_ba_reset_oob(c, 0);
    if (rc) return rc;
    rc = ldso_ba_linearize(c, 0, 1);
    if (rc) return rc;
    const int n = D.D;
    std::vector<double> Hsc((size_t)n * n), bsc(n);
    rc = ldso_ba_get_system(c, 0, H, b, nullptr, nullptr, Hsc.data(), bsc.data());
    if (rc) return rc;
    for (size_t i = 0; i < (size_t)n * n; i++) H[i] -= Hsc[i];  // EnergyFunctional.cc:242-243
    for (int i = 0; i < n; i++) b[i] -= bsc[i];
    return 0;
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
    HIP_TRY(hipMemcpy(e, c->win_energy() + 2 * win, sizeof(e), hipMemcpyDeviceToHost));
    out[0] = e[0];
    out[1] = 0;
    out[2] = e[1];
    return 0;
}

// download one window's packed system (through pinned staging) unless the host copy is fresh
static int fetch_sys(ldso_ba_ctx *c, int win) {
    if (!c->sys_host_valid) {
        c->sys_valid.assign(c->n_win, 0);
        c->sys_host.resize(c->sys_n);
        c->sys_host_valid = true;
    }
    if (c->sys_valid[win]) return 0;
    const WinDev &D = c->wd[win];
    const size_t n = (size_t)sys_len(D.D);
    if (c->pin_sys_n < n) {
        if (c->pin_sys) (void)hipHostFree(c->pin_sys);
        c->pin_sys = nullptr;
        HIP_TRY(hipHostMalloc(&c->pin_sys, n * sizeof(double), hipHostMallocDefault));
        c->pin_sys_n = n;
    }
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(c->pin_sys, c->d_sys.p + D.sys_base, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    int rc = ldso_ba_sync(c);
    if (rc) return rc;
    std::memcpy(c->sys_host.data() + D.sys_base, c->pin_sys, n * sizeof(double));
    c->sys_valid[win] = 1;
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
    int rc = fetch_sys(c, win);
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
    return ldso_ba_solve_system(&c->settings, c->wh[win].N, iteration, lambda, HA.data(), bA.data(), HL.data(),
                                bL.data(), nullptr, nullptr, Hsc.data(), bsc.data(), ns, n_null, x_out);
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
    // only the arrays the caller asked for cross PCIe (a NULL output costs nothing)
    std::vector<int8_t> ns(new_state ? R : 0), st(state ? R : 0);
    std::vector<uint8_t> fl(flags ? R : 0);
    std::vector<float> se(state_energy ? R : 0), ew(new_energy_wo ? R : 0);
    std::vector<float4> ce(center || rel_bs ? R : 0);
    if (new_state) HIP_TRY(hipMemcpy(ns.data(), c->d_rs_newstate.p + D.res_base, R, hipMemcpyDeviceToHost));
    if (state) HIP_TRY(hipMemcpy(st.data(), c->d_rs_state.p + D.res_base, R, hipMemcpyDeviceToHost));
    if (flags) HIP_TRY(hipMemcpy(fl.data(), c->d_rs_flags.p + D.res_base, R, hipMemcpyDeviceToHost));
    if (state_energy)
        HIP_TRY(hipMemcpy(se.data(), c->d_rs_energy.p + D.res_base, R * sizeof(float), hipMemcpyDeviceToHost));
    if (new_energy_wo)
        HIP_TRY(hipMemcpy(ew.data(), c->d_rs_energy_wo.p + D.res_base, R * sizeof(float), hipMemcpyDeviceToHost));
    for (int k = 0; k < 4 && (center || rel_bs); k++) {  // the planes back into (x, y, z, relBS) per residual
        if ((k < 3 && !center) || (k == 3 && !rel_bs)) continue;
        HIP_TRY(hipMemcpy2D(reinterpret_cast<float *>(ce.data()) + k, sizeof(float4),
                            reinterpret_cast<const float *>(c->d_rs_center.p) + (size_t)k * c->R_tot + D.res_base,
                            sizeof(float), sizeof(float), R, hipMemcpyDeviceToHost));
    }
    std::vector<float> jp;
    if (jpjdf) {
        if ((rc = record_jpjdf(c, win, c->d_rec_a.p, c->d_rec_b.p, c->d_geo_snap.p, jp))) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
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
        if (jpjdf) std::memcpy(jpjdf + 8 * (size_t)k, &jp[8 * (size_t)pos], 8 * sizeof(float));
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
    if (c->th_host_valid) {  // ldso_ba_optimize brought it back with its other results
        std::memcpy(th, c->th_host.data() + c->wd[win].frame_base, c->wd[win].N * sizeof(float));
        return 0;
    }
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
    const size_t nx = (size_t)N * N * 8 + 4;
    if (!c->pin_xad)
        HIP_TRY(hipHostMalloc(&c->pin_xad, ((size_t)LDSO_BA_MAX_FRAMES * LDSO_BA_MAX_FRAMES * 8 + 4) * sizeof(float),
                              hipHostMallocDefault));
    HIP_TRY(hipStreamSynchronize(c->stream));  // a previous upload from pin_xad has completed
    std::vector<float> xF(D.D);
    float *host = c->pin_xad;
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
    HIP_TRY(hipMemcpyAsync(c->d_xad.p + (size_t)win * kXadStride, host, nx * sizeof(float), hipMemcpyHostToDevice,
                           c->stream));
    if (D.P > 0) {
        int rc = launch_resubstitute(c, D.point_base, D.P, lambda);
        if (rc) return rc;
    }
    if (point_step_out) {
        if (c->pin_step_n < (size_t)D.P) {
            if (c->pin_step) (void)hipHostFree(c->pin_step);
            c->pin_step = nullptr;
            HIP_TRY(hipHostMalloc(&c->pin_step, std::max<size_t>(1, D.P) * sizeof(float), hipHostMallocDefault));
            c->pin_step_n = D.P;
        }
        if (D.P)
            HIP_TRY(hipMemcpyAsync(c->pin_step, c->d_pt_step.p + D.point_base, D.P * sizeof(float),
                                   hipMemcpyDeviceToHost, c->stream));
        int rc = ldso_ba_sync(c);
        if (rc) return rc;
        for (int q = 0; q < D.P; q++) point_step_out[H.pt_orig[q]] = c->pin_step[q];
    }
    return 0;
}

// ---- device-side solve / resubstitute ----------------------------------
}  // extern "C"
namespace {
// The caller's nullspaces (every window's [7][D] back to back) to d_ns and k_ortho_prep's
// normalised Nm, G and G^-1 for n_null of them; skipped when they equal the last prepared ones.
int upload_nullspaces(ldso_ba_ctx *c, const double *ns, int n_null) {
    const size_t cnt = (size_t)7 * c->vec_total;
    if (c->ns_cache_null == n_null && c->ns_cache.size() == cnt &&
        std::memcmp(c->ns_cache.data(), ns, cnt * sizeof(double)) == 0)
        return 0;
    HIP_TRY(hipMemcpyAsync(c->d_ns.p, ns, cnt * sizeof(double), hipMemcpyHostToDevice, c->stream));
    int dmax = 0;
    for (const WinDev &D : c->wd) dmax = std::max(dmax, D.D);
    if (dmax > kSolveMaxDim) return fail(-1, "device solve supports windows of up to 11 keyframes");
    SolveParams S{};
    S.wins = c->d_wins.p;
    S.ns = c->d_ns.p;
    S.iteration = 2;
    S.n_null = n_null;
    const size_t smem = solve_smem_bytes(dmax) + 16 + (size_t)7 * dmax * sizeof(double);
    static std::once_flag once;
    std::call_once(once, [] {
        (void)hipFuncSetAttribute((const void *)k_ortho_prep, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(solve_smem_bytes(kSolveMaxDim) + 16 + (size_t)7 * kSolveMaxDim * sizeof(double)));
    });
    k_ortho_prep<<<c->n_win, 64, smem, c->stream>>>(S, c->d_ns_nm.p, c->d_ns_g.p);
    HIP_TRY(hipGetLastError());
    c->ns_cache.assign(ns, ns + cnt);
    c->ns_cache_null = n_null;
    return 0;
}
// SOLVER_ORTHOGONALIZE_X_LATER in the context's solver mode: the solve projects x from iteration 2
// (EnergyFunctional.cc:428-432); without it the nullspaces are ignored
inline bool ortho_x_later(const ldso_ba_ctx *c) {
    return (c->settings.solver_mode & LDSO_BA_SOLVER_ORTHOGONALIZE_X_LATER) != 0;
}
// k_solve_fast (or the exact k_solve_reg / k_solve) for every loaded window; n_null > 0 projects
// with the nullspaces upload_nullspaces prepared (iteration >= 2), n_null == 0 does not project
int solve_device_launch(ldso_ba_ctx *c, int iteration, int n_null) {
    int dmax = 0;
    for (const WinDev &D : c->wd) dmax = std::max(dmax, D.D);
    if (dmax > kSolveMaxDim) return fail(-1, "device solve supports windows of up to 11 keyframes");
    SolveParams S{};
    S.wins = c->d_wins.p;
    S.sys = c->d_sys.p;
    S.prior = c->d_prior.p;
    S.ns = c->d_ns.p;
    S.x = c->d_x.p;
    S.adH = c->d_adH.p;
    S.adT = c->d_adT.p;
    S.xad = c->d_xad.p;  // the resubstitution's xAd comes with x (k_xad after the LDS kernel)
    S.prep_nm = c->d_ns_nm.p;
    S.prep_g = c->d_ns_g.p;
    S.iteration = iteration;
    S.n_null = iteration >= 2 ? n_null : 0;
    if (c->opt_pass >= 0) {  // inside ldso_ba_optimize: the per-window loop exits
        S.stop = c->d_stop.p;
        S.status = c->d_status.p;
    }
    static std::once_flag once;
    std::call_once(once, [] {
        (void)hipFuncSetAttribute((const void *)k_solve, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)solve_smem_bytes(kSolveMaxDim));
        (void)hipFuncSetAttribute((const void *)k_solve_reg, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)solve_reg_smem_bytes(kSolveRegDim));
        (void)hipFuncSetAttribute((const void *)k_solve_fast, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)solve_fast_smem_bytes(kSolveMaxDim));
    });
    if (!c->solve_exact && !getenv_flag("LDSO_BA_SOLVE_LDS")) {  // the default: unpivoted, xAd fused
        const size_t smem = solve_fast_smem_bytes(dmax);
        int grid = c->n_win;
        if (c->opt_pass >= 0 && nid_in_solve(c)) {  // the step's sumNID chains in blocks of their own
            S.win_nid = c->win_nid();
            S.nid_src = nid_source(c);
            S.n_win = c->n_win;
            S.nid_chunk = (int)std::min<size_t>(1024, (smem / sizeof(float)) & ~(size_t)3);
            grid *= 2;
        }
        return timed_launch(c, 5, c->stream, [&] { k_solve_fast<<<grid, kSolveFastThreads, smem, c->stream>>>(S); });
    }
    // exact mode: windows of up to 7 keyframes (n <= 64) the register factorisation, larger the LDS one
    const bool reg = dmax <= kSolveRegDim && !getenv_flag("LDSO_BA_SOLVE_LDS");
    const size_t smem = reg ? solve_reg_smem_bytes(dmax) : solve_smem_bytes(dmax);
    int rc = timed_launch(c, 5, c->stream, [&] {
        if (reg)
            k_solve_reg<<<c->n_win, kSolveRegThreads, smem, c->stream>>>(S);
        else
            k_solve<<<c->n_win, kSolveThreads, smem, c->stream>>>(S);
    });
    if (rc) return rc;
    if (!reg) {
        k_xad<<<c->n_win, 256, 0, c->stream>>>(c->d_wins.p, c->d_x.p, c->d_adH.p, c->d_adT.p, c->d_xad.p);
        HIP_TRY(hipGetLastError());
    }
    return 0;
}
}  // namespace
extern "C" {

// The projection (iteration >= 2) uses the nullspaces passed in THIS call; without them the
// solve does not project, exactly as the host solver (ldso_ba_solve / ldso_ba_solve_system).
int ldso_ba_solve_device(ldso_ba_ctx *c, int32_t iteration, double lambda, const double *ns, int32_t n_null,
                         double *x_out) {
    (void)lambda;  // SOLVER_FIX_LAMBDA, as the host solver
    if (!c || c->n_win == 0) return fail(-1, "no windows loaded");
    if (n_null < 0 || n_null > 7) return fail(-1, "n_null must be in [0, 7]");
    int rc;
    if ((rc = ldso_ba_check_settings(&c->settings))) return rc;
    HIP_TRY(hipSetDevice(c->device));
    const bool project = iteration >= 2 && ns && n_null > 0 && ortho_x_later(c);
    if (project && (rc = upload_nullspaces(c, ns, n_null))) return rc;
    rc = solve_device_launch(c, iteration, project ? n_null : 0);
    if (rc) return rc;
    if (x_out) {
        HIP_TRY(hipMemcpyAsync(x_out, c->d_x.p, (size_t)c->vec_total * sizeof(double), hipMemcpyDeviceToHost,
                               c->stream));
        rc = ldso_ba_sync(c);
        if (rc) return rc;
    }
    return 0;
}

int ldso_ba_resubstitute_device(ldso_ba_ctx *c, double lambda, float *point_step_out) {
    if (!c || c->n_win == 0) return fail(-1, "no windows loaded");
    HIP_TRY(hipSetDevice(c->device));
    k_xad<<<c->n_win, 256, 0, c->stream>>>(c->d_wins.p, c->d_x.p, c->d_adH.p, c->d_adT.p, c->d_xad.p);
    HIP_TRY(hipGetLastError());
    if (c->P_tot > 0) {
        int rc = launch_resubstitute(c, 0, c->P_tot, lambda);
        if (rc) return rc;
    }
    if (point_step_out) {
        if (c->pin_step_n < (size_t)c->P_tot) {
            if (c->pin_step) (void)hipHostFree(c->pin_step);
            c->pin_step = nullptr;
            HIP_TRY(hipHostMalloc(&c->pin_step, std::max<size_t>(1, c->P_tot) * sizeof(float), hipHostMallocDefault));
            c->pin_step_n = c->P_tot;
        }
        if (c->P_tot)
            HIP_TRY(hipMemcpyAsync(c->pin_step, c->d_pt_step.p, c->P_tot * sizeof(float), hipMemcpyDeviceToHost,
                                   c->stream));
        int rc = ldso_ba_sync(c);
        if (rc) return rc;
        long long out_base = 0;  // windows back to back, each in its caller point order
        for (int w = 0; w < c->n_win; w++) {
            const WinDev &D = c->wd[w];
            const WinHost &H = c->wh[w];
            for (int q = 0; q < D.P; q++) point_step_out[out_base + H.pt_orig[q]] = c->pin_step[D.point_base + q];
            out_base += H.P_all;
        }
    }
    return 0;
}

}  // extern "C"
namespace {
// The launch parameters a captured pass / solve sequence depends on besides the call's own
// arguments: the solve kernel (exact or fast), the stitch split, and every setting the kernels read.
std::vector<unsigned long long> capture_key(const ldso_ba_ctx *c) {
    const char *hs = std::getenv("LDSO_BA_HS_SPLIT");
    unsigned a, b, th;
    std::memcpy(&a, &c->settings.affine_opt_mode_a, 4);
    std::memcpy(&b, &c->settings.affine_opt_mode_b, 4);
    std::memcpy(&th, &c->settings.th_opt_iterations, 4);
    return {(unsigned long long)c->solve_exact, (unsigned long long)getenv_flag("LDSO_BA_SOLVE_LDS"),
            (unsigned long long)(hs ? (hs[0] == '1' ? 1 : 2) : 0), (unsigned long long)(unsigned)c->settings.solver_mode,
            (unsigned long long)(unsigned)c->settings.min_opt_iterations, a, b, th};
}
// Launch a captured sequence: replay g if it was captured under the current allocation
// generation and key, else capture `body`'s launches on the context stream, instantiate, cache.
template <typename F>
int launch_cached_graph(ldso_ba_ctx *c, ldso_ba_ctx::Graph &g, const std::vector<unsigned long long> &key, F &&body) {
    const unsigned long long gen = g_alloc_gen.load();
    if (g.exec && (g.gen != gen || g.key != key)) {
        (void)hipGraphExecDestroy(g.exec);
        g.exec = nullptr;
    }
    if (!g.exec) {
        hipGraph_t gr = nullptr;
        HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        const int rcap = body();
        const hipError_t ecap = hipStreamEndCapture(c->stream, &gr);
        if (rcap || ecap != hipSuccess) {
            if (gr) (void)hipGraphDestroy(gr);
            return rcap ? rcap : fail(-2, std::string("graph capture: ") + hipGetErrorString(ecap));
        }
        const hipError_t ei = hipGraphInstantiate(&g.exec, gr, nullptr, nullptr, 0);
        (void)hipGraphDestroy(gr);
        if (ei != hipSuccess) {
            g.exec = nullptr;
            return fail(-2, std::string("graph instantiate: ") + hipGetErrorString(ei));
        }
        g.gen = gen;
        g.key = key;
    }
    const hipError_t el = hipGraphLaunch(g.exec, c->stream);
    if (el != hipSuccess) return fail(-2, std::string("graph launch: ") + hipGetErrorString(el));
    // a replay skips the host side of the captured calls: invalidate what their passes would
    c->sys_host_valid = false;
    c->energy_valid = false;
    c->th_host_valid = false;
    return 0;
}
}  // namespace
extern "C" {

int ldso_ba_iterate(ldso_ba_ctx *c, int32_t iteration, double lambda, const double *ns, int32_t n_null, double *x_out,
                    float *point_step_out, double *energy_out) {
    if (!c || c->n_win == 0) return fail(-1, "no windows loaded");
    if (n_null < 0 || n_null > 7) return fail(-1, "n_null must be in [0, 7]");
    int rc;
    if ((rc = ldso_ba_check_settings(&c->settings))) return rc;
    HIP_TRY(hipSetDevice(c->device));
    // the projection uses the nullspaces of THIS call (as ldso_ba_solve_device)
    const bool project = iteration >= 2 && n_null > 0 && ns && ortho_x_later(c);
    if (project && (rc = upload_nullspaces(c, ns, n_null)))  // before (outside) the captured sequence
        return rc;
    // pass + solve + resubstitution (LDSO_BA_ITERATE_GRAPH=1: one captured graph per (projection,
    // lambda, n_null) without a communicator or kernel timing); the downloads stay outside it
    auto body = [&]() -> int {
        int r;
        if ((r = ldso_ba_linearize(c, 0, 1))) return r;
        if ((r = solve_device_launch(c, project ? 2 : 0, project ? n_null : 0))) return r;
        return c->P_tot > 0 ? launch_resubstitute(c, 0, c->P_tot, lambda) : 0;
    };
    // direct launches by default: for this six-launch sequence hipGraphLaunch costs more host
    // time than it saves (one S7 window: 89 vs 95 us per call, tools/iter_probe.py)
    if (!c->comm && !c->timing && getenv_flag("LDSO_BA_ITERATE_GRAPH") && !getenv_flag("LDSO_BA_NO_GRAPH")) {
        unsigned long long lb;
        std::memcpy(&lb, &lambda, sizeof(lb));
        // keyed by everything fixed at capture: lambda, n_null, the solve kernel, the stitch split,
        // the settings the pass reads
        std::vector<unsigned long long> key = capture_key(c);
        key.push_back(lb);
        key.push_back((unsigned long long)n_null);
        rc = launch_cached_graph(c, c->it_graph[project ? 1 : 0], key, body);
    } else {
        rc = body();
    }
    if (rc) return rc;
    // x, the energies and the point steps into the mapped results buffer (one launch), one
    // synchronisation
    const size_t xb = (size_t)c->vec_total * sizeof(double), eb = (size_t)2 * c->n_win * sizeof(double),
                 sb = (size_t)c->P_tot * sizeof(float);
    if ((rc = pin_map_ensure(c, xb + eb + sb))) return rc;
    const double *px = reinterpret_cast<const double *>(c->pin_map), *pe = px + c->vec_total;
    const float *ps = reinterpret_cast<const float *>(pe + 2 * c->n_win);
    {
        PackOut K{};
        auto seg = [&](const void *src, size_t off, size_t bytes) {
            K.src[K.n_seg] = static_cast<const unsigned *>(src);
            K.dst[K.n_seg] = reinterpret_cast<unsigned *>(c->pin_map_dev + off);
            K.words[K.n_seg++] = (int)(bytes / 4);
        };
        if (x_out) seg(c->d_x.p, 0, xb);
        if (energy_out) seg(c->win_energy(), xb, eb);
        if (point_step_out && sb) seg(c->d_pt_step.p, xb + eb, sb);
        if (K.n_seg) {
            k_pack_out<<<std::min(64, (int)((xb + eb + sb) / 1024) + 1), 256, 0, c->stream>>>(K);
            HIP_TRY(hipGetLastError());
        }
    }
    if ((rc = ldso_ba_sync(c))) return rc;
    if (x_out) std::memcpy(x_out, px, xb);
    if (point_step_out) {
        long long out_base = 0;  // windows back to back, each in its caller point order
        for (int w = 0; w < c->n_win; w++) {
            const WinDev &D = c->wd[w];
            const WinHost &H = c->wh[w];
            for (int q = 0; q < D.P; q++) point_step_out[out_base + H.pt_orig[q]] = ps[D.point_base + q];
            out_base += H.P_all;
        }
    }
    if (energy_out)
        for (int w = 0; w < c->n_win; w++) {
            energy_out[3 * w] = pe[2 * w];
            energy_out[3 * w + 1] = 0;
            energy_out[3 * w + 2] = pe[2 * w + 1];
        }
    return 0;
}

int ldso_ba_check_settings(const ldso_ba_opt_settings *s) {
    if (!s) return 0;
    static const struct {
        int bit;
        const char *name, *where;
    } kUnsupported[] = {
        {LDSO_BA_SOLVER_SVD, "SOLVER_SVD", "EnergyFunctional.cc:383-411"},
        {LDSO_BA_SOLVER_ORTHOGONALIZE_SYSTEM, "SOLVER_ORTHOGONALIZE_SYSTEM", "EnergyFunctional.cc:325"},
        {LDSO_BA_SOLVER_ORTHOGONALIZE_POINTMARG, "SOLVER_ORTHOGONALIZE_POINTMARG", "EnergyFunctional.cc:245"},
        {LDSO_BA_SOLVER_ORTHOGONALIZE_FULL, "SOLVER_ORTHOGONALIZE_FULL", "EnergyFunctional.cc:257"},
        {LDSO_BA_SOLVER_SVD_CUT7, "SOLVER_SVD_CUT7", "EnergyFunctional.cc:404"},
        {LDSO_BA_SOLVER_REMOVE_POSEPRIOR, "SOLVER_REMOVE_POSEPRIOR", "FrameHessian.h:147"},
        {LDSO_BA_SOLVER_USE_GN, "SOLVER_USE_GN", "EnergyFunctional.cc:282"},
        {LDSO_BA_SOLVER_ORTHOGONALIZE_X, "SOLVER_ORTHOGONALIZE_X", "EnergyFunctional.cc:428"},
        {LDSO_BA_SOLVER_MOMENTUM, "SOLVER_MOMENTUM", "FullSystem.cc:1840-1867"},
        {LDSO_BA_SOLVER_STEPMOMENTUM, "SOLVER_STEPMOMENTUM", "FullSystem.cc:913-920"},
    };
    for (const auto &u : kUnsupported)
        if (s->solver_mode & u.bit)
            return fail(-1, std::string("setting_solverMode: ") + u.name + " (" + u.where + ") is not implemented");
    if (s->solver_mode & ~(LDSO_BA_SOLVER_DEFAULT | 0xFFF))
        return fail(-1, "setting_solverMode: unknown bits");
    if (!(s->solver_mode & LDSO_BA_SOLVER_FIX_LAMBDA))
        return fail(-1, "setting_solverMode without SOLVER_FIX_LAMBDA (the LM lambda, EnergyFunctional.cc:283) is not "
                        "implemented");
    if (!s->force_accept_step)
        return fail(-1, "setting_forceAceptStep = false (the accept / reject branch with loadStateBackup, "
                        "FullSystem.cc:935-966) is not implemented");
    if (s->min_opt_iterations < 0) return fail(-1, "setting_minOptIterations < 0");
    if (s->vi_enable)
        return fail(-1, "setting_vi_enable = true: the inertial terms (combineInertialHessians and H_I / b_I in "
                        "solveSystemF, EnergyFunctional.cc:307-376; linearizeInertial, FullSystem.cc:879-926; the "
                        "inertial step and canbreak terms of doStepFromBackup, FullSystem.cc:1871-1931) are not "
                        "implemented: run visual-only (setting_vi_enable = false)");
    if (!std::isfinite(s->affine_opt_mode_a) || !std::isfinite(s->affine_opt_mode_b))
        return fail(-1, "setting_affineOptModeA / B must be finite");
    if (s->reserved_ != 0) return fail(-1, "ldso_ba_opt_settings.reserved_ must be 0");
    return 0;
}

void ldso_ba_default_settings(ldso_ba_opt_settings *s) {
    if (s) *s = ldso_ba_opt_settings LDSO_BA_OPT_SETTINGS_INIT;
}

int ldso_ba_set_settings(ldso_ba_ctx *c, const ldso_ba_opt_settings *s) {
    if (!c) return fail(-1, "bad arguments");
    int rc;
    if ((rc = ldso_ba_check_settings(s))) return rc;
    c->settings = s ? *s : ldso_ba_opt_settings LDSO_BA_OPT_SETTINGS_INIT;
    return 0;
}

int ldso_ba_get_settings(ldso_ba_ctx *c, ldso_ba_opt_settings *out) {
    if (!c || !out) return fail(-1, "bad arguments");
    *out = c->settings;
    return 0;
}

// The loop's first pass and solve use the priors the caller loaded (ldso_ba_window::frame_prior); every
// later step recomputes them on the device from the settings (k_step_resub, getPrior).  In the
// reference both come from the same setting_affineOptModeA / B, so a window whose loaded affine priors
// do not follow the settings the loop runs with is refused rather than run half with each.
static int check_affine_priors(const ldso_ba_ctx *c, const ldso_ba_frame_state *frames,
                               const ldso_ba_opt_settings &st) {
    for (int w = 0; w < c->n_win; w++) {
        const WinHost &H = c->wh[w];
        for (int f = 0; f < H.N; f++) {
            double p[8];
            frame_take_data_one(frames[c->wd[w].frame_base + f], st.affine_opt_mode_a, st.affine_opt_mode_b, p,
                                nullptr, nullptr);
            if (H.frame_prior[8 * f + 6] != p[6] || H.frame_prior[8 * f + 7] != p[7])
                return fail(-1, "window " + std::to_string(w) + " frame " + std::to_string(f) +
                                    ": the loaded affine priors (frame_prior[6..7]) do not follow the settings' "
                                    "setting_affineOptModeA / B; load the window with priors from "
                                    "ldso_ba_frame_take_data under the same settings");
        }
    }
    return 0;
}

int ldso_ba_optimize(ldso_ba_ctx *c, int32_t n_its, const ldso_ba_opt_settings *settings,
                     const ldso_ba_frame_state *frames, const double *calib_value, const double *calib_value_zero,
                     const double *ns, double *energy_out, ldso_ba_frame_state *frames_out, double *calib_out,
                     float *idepth_out, int32_t *iterations_out, int32_t *status_out) {
    if (!c || c->n_win == 0) return fail(-1, "no windows loaded");
    if (n_its < 0 || !frames || !calib_value || !calib_value_zero) return fail(-1, "bad arguments");
    if (c->marg) return fail(-1, "not on a marginalisation context");
    int rc;
    if (settings && (rc = ldso_ba_check_settings(settings))) return rc;
    if ((rc = check_affine_priors(c, frames, settings ? *settings : c->settings))) return rc;
    if (settings && (rc = ldso_ba_set_settings(c, settings))) return rc;  // checked, then installed
    const ldso_ba_opt_settings st = c->settings;
    // without SOLVER_ORTHOGONALIZE_X_LATER the solve never projects (EnergyFunctional.cc:428-432)
    if (!ortho_x_later(c)) ns = nullptr;
    HIP_TRY(hipSetDevice(c->device));
    const int nw = c->n_win;
    // ensure(): the buffers keep their addresses across calls, so cached graphs stay valid
    if ((rc = c->d_fstate.ensure(c->n_frames)) || (rc = c->d_calib_val.ensure((size_t)4 * nw)) ||
        (rc = c->d_calib_zero.ensure((size_t)4 * nw)) || (rc = c->d_cprior.ensure((size_t)4 * nw)) ||
        (rc = c->d_add_priors.ensure(nw)) || (rc = c->d_ehist.ensure((size_t)2 * nw * (n_its + 1))) ||
        (rc = c->d_stop.ensure(nw)) || (rc = c->d_status.ensure(nw)))
        return rc;
    std::vector<double> cp((size_t)4 * nw);
    std::vector<int> ap(nw);
    for (int w = 0; w < nw; w++) {
        for (int k = 0; k < 4; k++) cp[4 * w + k] = c->wh[w].c_prior[k];
        ap[w] = c->wh[w].add_priors ? 1 : 0;
    }
    {  // the call's inputs in one staged launch
        InBatch B;
        B.add(c->d_fstate.p, frames, (size_t)c->n_frames * sizeof(ldso_ba_frame_state));
        B.add(c->d_calib_val.p, calib_value, (size_t)4 * nw * sizeof(double));
        B.add(c->d_calib_zero.p, calib_value_zero, (size_t)4 * nw * sizeof(double));
        B.add(c->d_cprior.p, cp.data(), cp.size() * sizeof(double));
        B.add(c->d_add_priors.p, ap.data(), ap.size() * sizeof(int));
        if ((rc = B.flush(c))) return rc;
    }
    if (ns && (rc = upload_nullspaces(c, ns, 7)))  // evalPT is fixed during optimize(): valid for every iteration
        return rc;
    FrameStepParams F{};
    F.wins = c->d_wins.p;
    F.fstate = c->d_fstate.p;
    F.calib_val = c->d_calib_val.p;
    F.calib_zero = c->d_calib_zero.p;
    F.cprior = c->d_cprior.p;
    F.add_priors = c->d_add_priors.p;
    F.x = c->d_x.p;
    F.precalc = c->d_precalc.p;
    F.prior = c->d_prior.p;
    F.stop = c->d_stop.p;
    F.status = c->d_status.p;
    F.win_nid = c->win_nid();
    F.min_its = st.min_opt_iterations;
    F.th = st.th_opt_iterations;
    F.aff_a = st.affine_opt_mode_a;
    F.aff_b = st.affine_opt_mode_b;
    // one GN iteration: solveSystemF (a NaN x: the window is lost), resubstituteF_MT,
    // doStepFromBackup + setPrecalcValues (canbreak), linearizeAll + applyRes (+ the accumulation
    // the next solve uses); windows that left the loop skip every launch
    auto gn_iteration = [&](int it) -> int {
        int r;
        if ((r = solve_device_launch(c, it, ns ? 7 : 0))) return r;
        // the frame / calibration step + FrameFramePrecalc and the resubstitution with the point
        // step applied in place, in one launch (the solve wrote x and xAd)
        FrameStepParams Fi = F;
        Fi.it = it;
        ResubParams R = resub_params(c, 0, c->P_tot, 1e-5, true);
        R.stop = c->d_stop.p;
        R.it = it;
        if ((r = timed_launch(c, 3, c->stream, [&] {
                 k_step_resub<<<nw + (c->P_tot + 255) / 256, 256, 0, c->stream>>>(Fi, R, nw);
             })))
            return r;
        c->opt_pass = it + 1;
        return ldso_ba_linearize(c, 0, it + 1 < n_its ? 1 : 0);
    };
    // FullSystem::optimize (FullSystem.cc:853-976) with setting_forceAceptStep: resetOOB, then
    // linearizeAll + applyRes, then the GN iterations.  Every launch argument of the whole
    // sequence is fixed by (n_its, nullspaces or not), so without a communicator or kernel timing
    // the calls after the first replay ONE captured HIP graph of it (graph launches are
    // separated by ~9 us on the GPU; one per call instead of one per iteration), cached in the
    // context and re-captured after a device (re)allocation or when anything fixed at capture
    // changes: n_its, the settings, the solve kernel (exact or not), the stitch split.
    auto body = [&]() -> int {
        int r;
        // every window in the loop: stop = INT_MAX-ish (0x7f7f7f7f), status LDSO_BA_OPT_RAN_ALL
        HIP_TRY(hipMemsetAsync(c->d_stop.p, 0x7f, (size_t)nw * sizeof(int), c->stream));
        HIP_TRY(hipMemsetAsync(c->d_status.p, 0, (size_t)nw * sizeof(int), c->stream));
        c->opt_pass = 0;  // every pass of this call writes its energies into the history too
        if ((r = ldso_ba_reset_oob(c, -1)) || (r = ldso_ba_linearize(c, 0, n_its > 0 ? 1 : 0))) return r;
        for (int it = 0; it < n_its; it++)
            if ((r = gn_iteration(it))) return r;
        return 0;
    };
    const bool use_graph = !c->comm && !c->timing && !getenv_flag("LDSO_BA_NO_GRAPH");
    if (use_graph && c->opt_warm) {
        std::vector<unsigned long long> key = capture_key(c);  // the settings were installed above
        key.push_back((unsigned long long)(unsigned)n_its);
        rc = launch_cached_graph(c, c->opt_graph[ns ? 1 : 0], key, body);
    } else {
        rc = body();  // the first call runs directly (one-time setup stays out of any capture)
        c->opt_warm = rc == 0;
    }
    c->opt_pass = -1;
    if (rc) return rc;
    // every result into one pinned buffer (energy history, frame states, calibration, the window
    // descriptors, the idepth column), one synchronisation
    const size_t hb = (size_t)2 * nw * (n_its + 1) * sizeof(double),
                 fb = (size_t)c->n_frames * sizeof(ldso_ba_frame_state), cb = (size_t)4 * nw * sizeof(double),
                 wb = (size_t)nw * sizeof(WinDev), ib = (size_t)c->P_tot * sizeof(float),
                 tb = (size_t)c->n_frames * sizeof(float), sb = (size_t)nw * sizeof(int);
    auto up16 = [](size_t v) { return (v + 15) & ~(size_t)15; };
    const size_t o_f = up16(hb), o_c = o_f + up16(fb), o_w = o_c + up16(cb), o_t = o_w + up16(wb), o_s = o_t + up16(tb),
                 o_u = o_s + up16(sb), o_i = o_u + up16(sb);
    if ((rc = pin_map_ensure(c, o_i + ib))) return rc;
    char *po = c->pin_map, *pd = c->pin_map_dev;
    {  // one launch writes every result into the mapped buffer (the idepth column only)
        PackOut K{};
        auto seg = [&](const void *src, size_t off, size_t bytes) {
            K.src[K.n_seg] = static_cast<const unsigned *>(src);
            K.dst[K.n_seg] = reinterpret_cast<unsigned *>(pd + off);
            K.words[K.n_seg++] = (int)(bytes / 4);
        };
        if (energy_out) seg(c->d_ehist.p, 0, hb);
        if (frames_out) seg(c->d_fstate.p, o_f, fb);
        if (calib_out) seg(c->d_calib_val.p, o_c, cb);
        seg(c->d_wins.p, o_w, wb);  // the host mirror of WinDev (calibration, cDeltaF) follows the device
        seg(c->d_frame_th.p, o_t, tb);  // setNewFrameEnergyTH of the last pass (ldso_ba_get_frame_energy_th)
        seg(c->d_stop.p, o_s, sb);      // the loop exits
        seg(c->d_status.p, o_u, sb);
        if (idepth_out && c->P_tot) {
            K.pt_data = c->d_pt_data.p;
            K.idepth_dst = reinterpret_cast<float *>(pd + o_i);
            K.n_points = c->P_tot;
        }
        k_pack_out<<<std::min(64, (int)((o_i + ib) / 1024) + 1), 256, 0, c->stream>>>(K);
        HIP_TRY(hipGetLastError());
    }
    if ((rc = ldso_ba_sync(c))) return rc;
    {
        const int *stop = reinterpret_cast<const int *>(po + o_s), *status = reinterpret_cast<const int *>(po + o_u);
        for (int w = 0; w < nw; w++) {
            // lost at iteration k: stop = k and k + 1 solves ran; converged at k: stop = k + 1
            const int its = status[w] == LDSO_BA_OPT_LOST ? stop[w] + 1 : std::min(stop[w], n_its);
            if (iterations_out) iterations_out[w] = its;
            if (status_out) status_out[w] = status[w];
        }
    }
    if (energy_out) {
        const double *e = reinterpret_cast<const double *>(po);
        for (int s = 0; s <= n_its; s++)
            for (int w = 0; w < nw; w++) {
                double *o = energy_out + ((size_t)s * nw + w) * 3;
                o[0] = e[(size_t)2 * (s * nw + w)];
                o[1] = 0;
                o[2] = e[(size_t)2 * (s * nw + w) + 1];
            }
    }
    if (frames_out) std::memcpy(frames_out, po + o_f, fb);
    if (calib_out) std::memcpy(calib_out, po + o_c, cb);
    std::memcpy(c->wd.data(), po + o_w, wb);
    c->th_host.assign(reinterpret_cast<const float *>(po + o_t), reinterpret_cast<const float *>(po + o_t) + c->n_frames);
    c->th_host_valid = true;
    if (idepth_out) {
        const float *id = reinterpret_cast<const float *>(po + o_i);
        long long out_base = 0;  // windows back to back, each in its caller point order
        for (int w = 0; w < nw; w++) {
            const WinDev &D = c->wd[w];
            const WinHost &H = c->wh[w];
            for (int q = 0; q < D.P; q++) idepth_out[out_base + H.pt_orig[q]] = id[D.point_base + q];
            out_base += H.P_all;
        }
    }
    c->sys_host_valid = false;
    c->energy_valid = false;
    return 0;
}

int ldso_ba_frame_step(int32_t n, const ldso_ba_frame_state *in, const double *x, ldso_ba_frame_state *out,
                       double *calib_value, const double *calib_value_zero, float *calib_scaled_out,
                       float *c_delta_out) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !in || !x || !out) return fail(-1, "bad arguments");
    for (int f = 0; f < n; f++) frame_step_one(in[f], x + 4 + 8 * f, out[f]);
    if (calib_value) {
        float sf[4], cd[4];
        const double zero[4] = {0, 0, 0, 0};
        calib_step(calib_value, x, calib_value_zero ? calib_value_zero : zero, sf, cd);
        for (int k = 0; k < 4; k++) {
            if (calib_scaled_out) calib_scaled_out[k] = sf[k];
            if (c_delta_out) c_delta_out[k] = cd[k];
        }
    }
    return 0;
}

int ldso_ba_step_canbreak(int32_t n, const double *x, float sum_nid, float num_id, float th, int32_t *out) {
    if (n < 1 || n > LDSO_BA_MAX_FRAMES || !x || !out) return fail(-1, "bad arguments");
    *out = step_canbreak(n, x, sum_nid, num_id, th) ? 1 : 0;
    return 0;
}

int ldso_ba_packed_system(ldso_ba_ctx *c, void **dev_ptr, int64_t *n_doubles, int64_t *stride) {
    if (!c || !dev_ptr) return fail(-1, "bad arguments");
    *dev_ptr = c->d_sys.p;
    if (n_doubles) *n_doubles = (int64_t)c->sys_n;
    if (stride) *stride = c->n_win ? (int64_t)sys_len(c->wd[0].D) : 0;
    return 0;
}

int ldso_ba_unpack_system(ldso_ba_ctx *c) {
    if (!c) return fail(-1, "null ctx");
    c->sys_host_valid = false;  // get_system re-reads the (externally reduced) device buffer
    return 0;
}

int ldso_ba_copy_packed(ldso_ba_ctx *c, void *buf, int64_t n, int32_t direction) {
    if (!c || !buf || n != (int64_t)c->sys_n) return fail(-1, "bad arguments (size must equal the packed system)");
    HIP_TRY(hipSetDevice(c->device));
    if (direction == 0)
        HIP_TRY(hipMemcpyAsync(buf, c->d_sys.p, c->sys_n * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    else
        HIP_TRY(hipMemcpyAsync(c->d_sys.p, buf, c->sys_n * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->sys_host_valid = false;
    return 0;
}

int ldso_ba_newest_stride(ldso_ba_ctx *c, int64_t *stride) {
    if (!c || !stride) return fail(-1, "bad arguments");
    int64_t m = 0;
    for (const WinDev &D : c->wd) m = std::max<int64_t>(m, D.newest_end - D.newest_begin);
    *stride = m;
    return 0;
}

int ldso_ba_export_newest(ldso_ba_ctx *c, float *dev_buf, int64_t stride) {
    if (!c || !dev_buf || c->n_win == 0 || stride < 1) return fail(-1, "bad arguments");
    for (const WinDev &D : c->wd)
        if (D.newest_end - D.newest_begin > stride) return fail(-1, "stride smaller than a newest-frame segment");
    HIP_TRY(hipSetDevice(c->device));
    const dim3 grid((unsigned)std::min<int64_t>((stride + 255) / 256, 64), (unsigned)c->n_win);
    k_export_newest<<<grid, 256, 0, c->stream>>>(c->d_wins.p, c->d_rs_energy_wo.p, dev_buf, (long long)stride,
                                                 (long long)stride, nullptr, 0);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int ldso_ba_frame_threshold_gathered(ldso_ba_ctx *c, const float *dev_buf, int32_t n_ranks, int64_t stride) {
    if (!c || !dev_buf || c->n_win == 0 || n_ranks < 1 || stride < 1) return fail(-1, "bad arguments");
    if ((int64_t)n_ranks * stride > INT32_MAX) return fail(-1, "too many candidates");
    HIP_TRY(hipSetDevice(c->device));
    c->th_host_valid = false;
    int rc = timed_launch(c, 4, c->stream, [&] {
        k_frame_th<<<c->n_win, kStThreads, 0, c->stream>>>(c->d_wins.p, dev_buf, n_ranks, c->n_win, (long long)stride,
                                                           (long long)stride, c->d_frame_th.p, NidSrc{}, nullptr,
                                                           nullptr, 0);
    });
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int ldso_ba_set_tuning(ldso_ba_ctx *c, int32_t key, int32_t value) {
    if (!c) return fail(-1, "null ctx");
    if (key == LDSO_BA_TUNE_TILED_IMAGES) {
        if (c->n_win) return fail(-1, "image layout must be chosen before ldso_ba_load");
        if (value != 1 && value != 3) return fail(-1, "image layout must be 1 or 3");
        c->img_mode = value;
        return 0;
    }
    if (key == LDSO_BA_TUNE_ITEM_ORDER) {
        if (c->n_win) return fail(-1, "item order must be chosen before ldso_ba_load");
        if (value < 0 || value > 2) return fail(-1, "item order must be 0, 1 or 2");
        c->item_order = value;
        return 0;
    }
    if (key == LDSO_BA_TUNE_SOLVE_EXACT) {
        if (value != 0 && value != 1) return fail(-1, "solve mode must be 0 (fast) or 1 (exact)");
        c->solve_exact = value;
        return 0;
    }
    if (key == LDSO_BA_TUNE_TIMING_MASK) {
        c->timing_mask = (unsigned)value;
        return 0;
    }
    if (key == LDSO_BA_TUNE_TOP_CHUNK) {
        if (value < 0 || value > 64 || value % 8) return fail(-1, "chunk must be 0 or a multiple of 8 up to 64");
        if (c->n_win) return fail(-1, "chunk size must be chosen before ldso_ba_load");
        c->top_chunk = value;
        return 0;
    }
    return fail(-1, "unknown tuning key");
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
    // the events the timed launches will take, created now: hipEventCreate is a host call of tens of
    // us, which inside a timed loop would stall the launches (kept in the pool across calls)
    while (c->timing && c->ev_pool.size() < 256) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) break;
        c->ev_pool.push_back(e);
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
        *device_bytes = (int64_t)(c->d_img.bytes() + c->d_precalc.bytes() + c->d_pt_data.bytes() + c->d_rec_a.bytes() + c->d_rec_b.bytes() +
                                  c->d_top_slab.bytes() + c->d_sc_slab.bytes() + c->d_sys.bytes());
    if (n_points) *n_points = c->P_tot;
    if (n_residuals) *n_residuals = c->R_tot;
    return 0;
}

}  // extern "C"
