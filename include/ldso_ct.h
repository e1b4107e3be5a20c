/*
 * ldso_ct.h -- C ABI of the MI355X-native coarse tracker.
 *
 * It replaces, for the GPU, the per-frame direct image alignment LDSO runs on every incoming
 * frame (reference paths relative to n-lalanne/LDSO):
 *
 *   FrameHessian::makeImages            src/internal/FrameHessian.cc:59-115  -> ldso_ct_set_new_frame
 *   CoarseTracker::makeK                src/frontend/CoarseTracker.cc:312-339 -> ldso_ct_make_k
 *   CoarseTracker::calcRes              src/frontend/CoarseTracker.cc:540-673 -> ldso_ct_calc_res
 *                                                                              (+ _batch: many poses)
 *   CoarseTracker::calcGSSSE            src/frontend/CoarseTracker.cc:675-741 -> ldso_ct_calc_gs
 *     with Accumulator9                 include/internal/OptimizationBackend/MatrixAccumulators.h:1104-1643
 *
 * The reference frame's point cloud (pc_u/pc_v/pc_idepth/pc_color per pyramid level, the output
 * of CoarseTracker::makeCoarseDepthL0, CoarseTracker.cc:357-538) is handed over by
 * ldso_ct_set_reference; trackNewestCoarse's LM loop (CoarseTracker.cc:61-310) stays with the
 * caller and calls these entry points exactly where it calls calcRes / calcGSSSE.
 *
 * Conventions: poses are SE3 refToNew as a row-major 3x4 double matrix [R | t]
 * (Sophus::SE3::matrix3x4()); affine brightness parameters are AffLight (a, b) pairs;
 * exposures are FrameHessian::ab_exposure.  Outputs are the reference's types: calcRes returns
 * the Vec6 {E, numTermsInE, shiftT, 0, shiftRT, saturated fraction}; calcGSSSE the 8x8 H and
 * 8-vector b (row-major doubles) with the SCALE_* factors applied.
 *
 * Error convention as ldso_ba.h: 0 on success, < 0 on failure with ldso_ba_last_error() set.
 * A context is bound to one HIP device and stream; entry points are not re-entrant.
 */
#ifndef LDSO_CT_H_
#define LDSO_CT_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDSO_CT_MAX_LEVELS 6 /* PYR_LEVELS, NumTypes.h */

typedef struct ldso_ct_ctx ldso_ct_ctx;

/* CoarseTracker::CoarseTracker(w, h): level-0 size; the level count follows GlobalCalib's rule
 * (halve while both sides stay even and w*h > 5000, at most LDSO_CT_MAX_LEVELS;
 * src/internal/GlobalCalib.cc:20-30).  n_levels_out may be NULL. */
int ldso_ct_create(int32_t device, int32_t width, int32_t height, ldso_ct_ctx **out, int32_t *n_levels_out);
void ldso_ct_destroy(ldso_ct_ctx *ctx);

/* CoarseTracker::makeK (CoarseTracker.cc:312-339) from the level-0 fxl, fyl, cxl, cyl.
 * k_out (may be NULL): per level {fx, fy, cx, cy, Ki[9] row-major} = 13 floats. */
int ldso_ct_make_k(ldso_ct_ctx *ctx, const float calib[4], float *k_out);

/* FrameHessian::makeImages of the new frame on the device: level-0 intensities `color`
 * [height*width] -> dIp[lvl] = [I, dx, dy] and absSquaredGrad[lvl] for every level.
 * b_response: CalibHessian::B[256] for setting_gammaWeightsPixelSelect (NULL = identity,
 * i.e. no photometric calibration loaded).  ab_exposure: FrameHessian::ab_exposure. */
int ldso_ct_set_new_frame(ldso_ct_ctx *ctx, const float *color, double ab_exposure, const float *b_response);
/* read back level lvl of the new frame: dI [wl*hl][3], abs_sq_grad [wl*hl] (either may be NULL) */
int ldso_ct_get_frame_level(ldso_ct_ctx *ctx, int32_t lvl, float *dI, float *abs_sq_grad);

/* setCoarseTrackingRef's outputs: for each level, pc_n[lvl] points with pc_u, pc_v, pc_idepth,
 * pc_color (arrays of pointers, one per level), the reference frame's ab_exposure and
 * lastRef_aff_g2l (a, b). */
int ldso_ct_set_reference(ldso_ct_ctx *ctx, const int32_t *pc_n, const float *const *pc_u,
                          const float *const *pc_v, const float *const *pc_idepth,
                          const float *const *pc_color, double ref_ab_exposure, double ref_aff_a,
                          double ref_aff_b);

/* CoarseTracker::calcRes(lvl, refToNew, aff_g2l, cutoffTH) -> rs_out[6]; also keeps the warped
 * buffers on the device for the next ldso_ct_calc_gs (as the reference keeps buf_warped_*). */
int ldso_ct_calc_res(ldso_ct_ctx *ctx, int32_t lvl, const double ref_to_new[12], double aff_a, double aff_b,
                     float cutoff_th, double rs_out[6]);
/* calcRes for n_hyp poses at once (the motion hypotheses of FullSystem::trackNewCoarse,
 * FullSystem.cc:282-386): rs_out [n_hyp][6]; does not touch the warped buffers. */
int ldso_ct_calc_res_batch(ldso_ct_ctx *ctx, int32_t lvl, int32_t n_hyp, const double *ref_to_new,
                           const double *aff_ab, float cutoff_th, double *rs_out);
/* CoarseTracker::calcGSSSE(lvl, H, b, refToNew, aff_g2l) over the warped buffers of the last
 * ldso_ct_calc_res at this level.  H_out [8][8], b_out [8]. */
int ldso_ct_calc_gs(ldso_ct_ctx *ctx, int32_t lvl, const double ref_to_new[12], double aff_a, double aff_b,
                    double *H_out, double *b_out);
/* calcRes followed by calcGSSSE at the same pose (what trackNewestCoarse does at the start of
 * each level and for every LM step, CoarseTracker.cc:90-105, 218-245; a rejected step simply
 * ignores H and b): both launches
 * back to back on the context stream and one round trip; results equal the two separate calls. */
int ldso_ct_calc_res_gs(ldso_ct_ctx *ctx, int32_t lvl, const double ref_to_new[12], double aff_a, double aff_b,
                        float cutoff_th, double rs_out[6], double *H_out, double *b_out);
/* the warped buffers of the last calcRes, compacted in point order and zero-padded to a multiple
 * of 4 exactly as buf_warped_* / buf_warped_n: out [n][8] = {idepth, u, v, dx, dy, residual,
 * weight, refColor}; *n_out = buf_warped_n.  out may be NULL to query n. */
int ldso_ct_get_warped(ldso_ct_ctx *ctx, int32_t *n_out, float *out, int32_t capacity);

/* ---- immature points: point creation and epipolar tracing ----------
 *
 *   ImmaturePoint::ImmaturePoint        src/internal/ImmaturePoint.cc:14-39   -> ldso_ct_make_immature
 *   ImmaturePoint::traceOn over all     src/internal/ImmaturePoint.cc:47-317  -> ldso_ct_trace
 *     immature points of all frames,    (FullSystem::traceNewCoarse,
 *     with the new frame                 src/frontend/FullSystem.cc:1157-1194)
 *
 * One record per ImmaturePoint (ImmaturePoint.h:101-121), 128 bytes.  `host` indexes the per-host
 * tables of ldso_ct_trace (traceNewCoarse's per-frame KRKi, Kt, aff).  The traced frame is the
 * context's new frame (ldso_ct_set_new_frame, level 0); ldso_ct_make_immature samples the same
 * frame, as makeNewTraces creates the points of the keyframe that was just made
 * (FullSystem.cc:1425-1475).  Where the reference would read outside the image (a rotated
 * pattern tap past the border: undefined behaviour there), both this path and the oracle clamp
 * the tap to the last interpolable texel. */
typedef struct ldso_ct_immature {
    float u, v;                  /* feature->uv */
    float idepth_min, idepth_max;
    float quality;
    float energy_th;             /* energyTH (NaN: a pattern colour was not finite) */
    float color[8];              /* pattern order: staticPattern[8], Setting.cc:275 */
    float weights[8];
    float grad_h[4];             /* gradH, row-major 2x2 */
    int32_t host;                /* index into ldso_ct_trace's host tables */
    int32_t last_status;         /* ImmaturePointStatus: GOOD 0, OOB 1, OUTLIER 2, SKIPPED 3,
                                    BADCONDITION 4, UNINITIALIZED 5 */
    float last_uv[2];            /* lastTraceUV */
    float last_interval;         /* lastTracePixelInterval */
    float type;                  /* my_type */
} ldso_ct_immature;

#define LDSO_CT_IPS_GOOD 0
#define LDSO_CT_IPS_OOB 1
#define LDSO_CT_IPS_OUTLIER 2
#define LDSO_CT_IPS_SKIPPED 3
#define LDSO_CT_IPS_BADCONDITION 4
#define LDSO_CT_IPS_UNINITIALIZED 5

/* new ImmaturePoint(newFrame, feat, type, HCalib) for n features at uv [n][2] on the context's
 * new frame: colour, weights, gradH and energyTH; idepth_min 0, idepth_max NaN, quality 10000,
 * status UNINITIALIZED, host = `host` for all n.  out: host memory [n]. */
int ldso_ct_make_immature(ldso_ct_ctx *ctx, int32_t n, const float *uv, float type, int32_t host,
                          ldso_ct_immature *out);
/* make the n records resident on the device (replaces the previous set) / read them back */
int ldso_ct_immature_upload(ldso_ct_ctx *ctx, int32_t n, const ldso_ct_immature *pts);
int ldso_ct_immature_download(ldso_ct_ctx *ctx, int32_t n, ldso_ct_immature *pts);
/* traceNewCoarse: traceOn of every resident record with the context's new frame.
 * krki [n_hosts][9] row-major, kt [n_hosts][3], aff [n_hosts][2] (AffLight::fromToVecExposure
 * host -> new frame), as traceNewCoarse builds them per host frame.
 * counts_out (may be NULL): [6] records per lastTraceStatus after the call (trace_good,
 * trace_oob, trace_out, trace_skip, trace_badcondition, trace_uninitialized). */
int ldso_ct_trace(ldso_ct_ctx *ctx, int32_t n_hosts, const float *krki, const float *kt, const float *aff,
                  int32_t *counts_out);

/* kernel timing of the tracker's launches (same slots mechanism as ldso_ba) */
int ldso_ct_set_kernel_timing(ldso_ct_ctx *ctx, int32_t enable);
int ldso_ct_get_kernel_times(ldso_ct_ctx *ctx, double *ms, int64_t *counts, int32_t n);
const char *ldso_ct_kernel_name(int32_t i);
int32_t ldso_ct_num_kernels(void);

#ifdef __cplusplus
}
#endif

#endif
