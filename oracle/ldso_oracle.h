/*
 * ldso_oracle.h -- C API of the CPU restatement of LDSO's photometric-BA hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library, and only as the checker / CPU baseline, never as the product.
 *
 * Parity status: the reference (n-lalanne/LDSO) ships no golden vectors, KATs or fixtures for
 * this path and cannot be built in this image (Eigen3, glog, OpenCV, g2o, DBoW3, Boost absent;
 * SURVEY.md §8c), so this restatement is "parity unpinned" by the reference.  It is pinned
 * instead by independent known-answer tests (finite-difference Jacobians, dense J^T W J and
 * explicit Schur complements computed from first principles in tests/test_oracle_kat.py).
 *
 * Every function follows a reference file:line (see ldso_oracle.cpp).  Float arithmetic is
 * compiled with -ffp-contract=off so that each statement rounds in the reference's source
 * order (the reference itself, built with -march=native, lets GCC contract FMAs).
 */
#ifndef LDSO_ORACLE_H_
#define LDSO_ORACLE_H_

#include "../include/ldso_ba.h"
#include "../include/ldso_ct.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_window oracle_window;

/* Number of IndexThreadReduce workers (reference NUM_THREADS = 6, Settings.h:11).
 * 0 selects the reference's multiThreading=false path (single thread, tid = -1 stitch). */
void oracle_set_threads(int n);
int oracle_get_threads(void);

oracle_window *oracle_create(const ldso_ba_window *w);
void oracle_destroy(oracle_window *ow);

/* per-iteration refresh (same fields as ldso_ba_update) */
int oracle_update(oracle_window *ow, const ldso_ba_window *w);
void oracle_reset_oob(oracle_window *ow);

/* FullSystem::linearizeAll(fix) incl. setNewFrameEnergyTH; out[3] = {E, 0, nIN} */
int oracle_linearize_all(oracle_window *ow, int fix, double *out);
/* FullSystem::applyRes_Reductor(true) over all residuals */
void oracle_apply_res(oracle_window *ow);
/* accumulateAF_MT + accumulateLF_MT + accumulateSCF_MT (with stitches); any output may be NULL */
int oracle_accumulate(oracle_window *ow, double *HA, double *bA, double *HL, double *bL,
                      double *Hsc, double *bsc);
/* one full hot-path GN pass, as the GPU's ldso_ba_linearize(fix=0, accumulate=1) */
int oracle_iteration(oracle_window *ow, double *energy_out);

void oracle_get_residuals(oracle_window *ow, int8_t *new_state, int8_t *state, float *state_energy,
                          float *new_energy_wo, float *center, uint8_t *flags, float *jpjdf,
                          float *rel_bs);
/* RawResidualJacobian dump per residual: resF[8], Jpdxi[2][6], Jpdc[2][4], Jpdd[2], JIdx[2][8],
 * JabF[2][8], JIdx2[4], JabJIdx[4], Jab2[4]  (= 78 floats) */
void oracle_get_jacobians(oracle_window *ow, float *out78);
void oracle_get_points(oracle_window *ow, float *HdiF, float *bdSumF, float *idepth_hessian,
                       float *Hdd_acc, float *bd_acc, float *Hcd_acc);
void oracle_get_frame_energy_th(oracle_window *ow, float *th);

int oracle_solve_system(int n_frames, int iteration, double lambda, const double *HA,
                        const double *bA, const double *HL, const double *bL, const double *HM,
                        const double *bM, const double *Hsc, const double *bsc,
                        const double *nullspaces, int n_null, double *x_out);
void oracle_resubstitute(oracle_window *ow, const double *x, double lambda, float *point_step);

/* host-side restatements of FrameFramePrecalc::Set, setAdjointsF, takeData, getNullspaces */
int oracle_frame_precalc(int n_frames, const ldso_ba_frame_state *frames, const float calib[4],
                         float *precalc_out);
int oracle_set_adjoints(int n_frames, const ldso_ba_frame_state *frames, double *ad_host,
                        double *ad_target, double *c_prior);
void oracle_set_affine_opt_modes(float a, float b);
void oracle_get_affine_opt_modes(float *a, float *b);
int oracle_frame_take_data(int n_frames, const ldso_ba_frame_state *frames, double *prior,
                           double *delta, double *delta_prior);
/* FrameHessian::setStateZero nullspaces + FullSystem::getNullspaces (pose x6, scale x1):
 * out [7][8N+4] in the order orthogonalize() stacks them. */
int oracle_nullspaces(int n_frames, const ldso_ba_frame_state *frames, double *out);
/* FullSystem::doStepFromBackup (FullSystem.cc:1826-1931; non-momentum, step factors 1, no inertial
 * terms) for one window: frames / calibration / point idepths stepped from their backups by the
 * solve's x and the resubstituted point steps; returns canbreak (0 / 1) or -1. */
int oracle_do_step_from_backup(int n_frames, const ldso_ba_frame_state *backup, const double *x, double *calib_value,
                               const double *calib_value_zero, int n_points, const int *point_host,
                               const float *idepth_backup, const float *point_step, float th_opt_iterations,
                               ldso_ba_frame_state *out, float *idepth_out, float *calib_scaled_out,
                               float *c_delta_out);

/* Point marginalisation of the points pts[n] (flagPointsForRemoval's relinearisation +
 * fixLinearizationF, then marginalizePointsF's addPoint<2> / SC addPoint(p, false) / stitch):
 * H = M - Msc [(8N+4)^2], b = Mb - Mbsc.  adHTdeltaF [N*N][8].  Mutates the points' residuals and
 * priorF as the reference does. */
int oracle_marginalize_points(oracle_window *ow, int n, const int *pts, const float *adHTdeltaF, double *H,
                              double *b);

/* EnergyFunctional::setDeltaF's adHTdeltaF, calcMEnergyF and calcLEnergyF_MT (the prior terms). */
int oracle_ad_ht_delta(int n_frames, const double *delta, const double *ad_host, const double *ad_target, float *out);
double oracle_calc_m_energy(int n_frames, const double *HM, const double *bM, const float *c_delta,
                            const double *delta);
double oracle_calc_l_energy(int n_frames, const double *prior, const double *delta_prior, const double *c_prior,
                            const float *c_delta, int n_points, const float *deltaF, const float *priorF);

/* ---- coarse tracker (ldso_oracle_tracker.cpp; the checker of include/ldso_ct.h) ---------- */
int oracle_ct_levels(int w, int h);
/* per level 13 floats {fx, fy, cx, cy, Ki[9]} */
void oracle_ct_make_k(const float calib[4], int w, int h, int levels, float *out);
/* dIp: all levels concatenated, [wl*hl][3] each; absg: [wl*hl] each; B: response (NULL = none) */
void oracle_make_images(const float *color, int w, int h, int levels, const float *B, float *dIp, float *absg);
/* aff6 = {ref exposure, new exposure, ref a, ref b, new a, new b}; T = refToNew 3x4 row-major */
int oracle_ct_calc_res(int lvl, int wl, int hl, const float *kl, const float *dI, int n, const float *pc_u,
                       const float *pc_v, const float *pc_idepth, const float *pc_color, const double *T,
                       const double *aff6, float cutoffTH, double *rs, float *warped_out, int *n_warped);
int oracle_ct_calc_gs(int n, const float *warped, float fxl, float fyl, const double *aff6, double *H_out,
                      double *b_out);

/* ImmaturePoint constructor over n features uv [n][2] of the level-0 frame dI [w*h][3] */
void oracle_ip_make(const float *dI, int w, int h, int n, const float *uv, float type, int host,
                    ldso_ct_immature *out);
/* traceNewCoarse: traceOn of every record against dI with its host's krki/kt/aff; counts [6] */
void oracle_ip_trace(const float *dI, int w, int h, const float *krki, const float *kt, const float *aff, int n,
                     ldso_ct_immature *pts, int *counts);

/* FullSystem::optimizeImmaturePoint for n immature points hosted in the window (pts[k].host) */
int oracle_activate_points(oracle_window *ow, int n, const ldso_ct_immature *pts, int min_obs,
                           ldso_ba_activation *out);

/* CPU-baseline timing: run `iters` oracle_iteration passes, return wall seconds. */
double oracle_time_iterations(oracle_window *ow, int iters);

#ifdef __cplusplus
}
#endif

#endif
