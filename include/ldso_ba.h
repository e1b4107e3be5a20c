/*
 * ldso_ba.h -- C ABI of the MI355X-native LDSO photometric bundle-adjustment hot path.
 *
 * This header is the drop-in boundary.  It replaces, for the GPU, the C++ class surface
 * the LDSO frontend drives once per Gauss-Newton iteration (reference paths are relative to
 * n-lalanne/LDSO):
 *
 *   PointFrameResidual::linearize / applyRes / resetOOB      src/internal/Residuals.cc:15-217,
 *                                                            include/internal/Residuals.h:61-88
 *   FullSystem::linearizeAll(_Reductor), setNewFrameEnergyTH src/frontend/FullSystem.cc:1716-1823, 2078-2109
 *   AccumulatedTopHessianSSE::addPoint<0> / stitchDoubleMT  src/internal/OptimizationBackend/AccumulatedTopHessian.cc:8-255
 *   AccumulatedSCHessianSSE::addPoint / stitchDoubleMT      src/internal/OptimizationBackend/AccumulatedSCHessian.cc:9-177
 *   EnergyFunctional::accumulate{AF,LF,SCF}_MT, solveSystemF, resubstituteF_MT
 *                                                            src/internal/OptimizationBackend/EnergyFunctional.cc:280-471, 611-749
 *   FrameFramePrecalc::Set, EnergyFunctional::setAdjointsF  src/internal/FrameFramePrecalc.cc:6-35,
 *                                                            src/internal/OptimizationBackend/EnergyFunctional.cc:551-609
 *   FullSystem::optimizeImmaturePoint with                   src/frontend/FullSystem.cc:1035-1156,
 *     ImmaturePoint::linearizeResidual (point activation)    src/internal/ImmaturePoint.cc:319-389
 *
 * Conventions (mirroring the reference):
 *   - frame-pair index            pair = h + N*t      (AccumulatedTopHessian.cc:38)
 *   - Hessian column blocks       [0,4) intrinsics, 4+8f+[0,6) xi_f, 4+8f+6 a_f, 4+8f+7 b_f
 *   - residual states             IN = 0, OOB = 1, OUTLIER = 2 (Residuals.h:33)
 *   - every matrix is row-major, every H is (8N+4)x(8N+4) double, every b is (8N+4) double.
 *
 * Error convention: every entry point returns 0 on success and a negative code on failure
 * (never throws); ldso_ba_last_error() gives a message.  Non-finite numbers pass through as
 * values, exactly as in the reference (the caller turns them into isLost).
 * Threading: a context is bound to one HIP device and one HIP stream; entry points are not
 * re-entrant (the reference runs them under FullSystem::mapMutex).
 */
#ifndef LDSO_BA_H_
#define LDSO_BA_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDSO_BA_ABI_VERSION 6

#define LDSO_BA_PATTERN_NUM 8      /* patternNum, Settings.h:225 (staticPattern[8])     */
#define LDSO_BA_CPARS 4            /* CPARS, NumTypes.h:25                              */
#define LDSO_BA_MAX_FRAMES 16      /* window size supported by one context              */
#define LDSO_BA_PRECALC_STRIDE 48  /* floats per FrameFramePrecalc record (see below)   */
#define LDSO_BA_POINT_STRIDE 24    /* floats per PointHessian record (see below)        */

/* Residual states, Residuals.h:33 */
#define LDSO_BA_RES_IN 0
#define LDSO_BA_RES_OOB 1
#define LDSO_BA_RES_OUTLIER 2

/* Residual flag bits */
#define LDSO_BA_FLAG_ACTIVE 1u     /* PointFrameResidual::isActiveAndIsGoodNEW */
#define LDSO_BA_FLAG_NEW 2u        /* PointFrameResidual::isNew                 */

/*
 * FrameFramePrecalc record (FrameFramePrecalc.h:35-44), LDSO_BA_PRECALC_STRIDE floats:
 *   [0..8]  PRE_KRKiTll (3x3 row-major)   [9..11]  PRE_KtTll
 *   [12..20] PRE_RTll_0 (3x3 row-major)   [21..23] PRE_tTll_0
 *   [24..25] PRE_aff_mode                 [26]     PRE_b0_mode
 *   [27..35] PRE_RTll (3x3 row-major)     [36..38] PRE_tTll        [39..47] unused
 * PRE_RTll_0 / PRE_tTll_0 come from the evaluation points (worldToCam_evalPT) and feed the FEJ
 * Jacobians of PointFrameResidual::linearize; PRE_RTll / PRE_tTll come from the current poses
 * (PRE_worldToCam) and feed ImmaturePoint::linearizeResidual (ImmaturePoint.cc:336-337).
 *
 * PointHessian record (PointHessian.h:83-131), LDSO_BA_POINT_STRIDE floats:
 *   [0] u  [1] v  [2] idepth_scaled  [3] idepth_zero_scaled  [4] priorF  [5] deltaF
 *   [6..7] unused  [8..15] color[8]  [16..23] weights[8]
 */

/* One sliding window (= one FullSystem / EnergyFunctional).  All pointers are host memory. */
typedef struct ldso_ba_window {
    int32_t n_frames;              /* N, 2 <= N <= LDSO_BA_MAX_FRAMES                        */
    int32_t n_points;              /* P: EnergyFunctional::allPoints (makeIDX order)         */
    int32_t n_residuals;           /* R: sum of PointHessian::residuals sizes                */
    int32_t width, height;         /* wG[0], hG[0]                                           */
    float calib[4];                /* CalibHessian::value_scaledf: fxl, fyl, cxl, cyl        */
    const float *dI;               /* [N][height*width][3]: FrameHessian::dI = [I, dx, dy]   */
    const float *frame_energy_th;  /* [N]: FrameHessian::frameEnergyTH                       */
    const float *precalc;          /* [N*N][LDSO_BA_PRECALC_STRIDE], index h + N*t           */
    const double *ad_host;         /* [N*N][64]: EnergyFunctional::adHost                    */
    const double *ad_target;       /* [N*N][64]: EnergyFunctional::adTarget                  */
    const double *c_prior;         /* [4]: EnergyFunctional::cPrior                          */
    const float *c_delta;          /* [4]: EnergyFunctional::cDeltaF                         */
    const double *frame_prior;     /* [N][8]: FrameHessian::prior                            */
    const double *frame_delta_prior; /* [N][8]: FrameHessian::delta_prior                    */
    const int32_t *point_host;     /* [P]: host frame index (FrameHessian::idx)              */
    const float *point_data;       /* [P][LDSO_BA_POINT_STRIDE]                              */
    const int32_t *point_res_begin;/* [P+1]: residuals of point p are [begin[p], begin[p+1]) */
    const int32_t *res_target;     /* [R]: target frame index (PointFrameResidual::targetIDX)*/
    const int8_t *res_state;       /* [R]: state_state                                       */
    const float *res_energy;       /* [R]: state_energy                                      */
    const uint8_t *res_flags;      /* [R]: LDSO_BA_FLAG_*                                    */
    /* [P] or NULL: the point's rank among its host frame's points in the order of the host
     * Frame's features vector.  The library keeps each host's points in this order (NULL: the
     * caller's order), which is the order doStepFromBackup sums sumNID in (frames -> features,
     * FullSystem.cc:1899-1909) and so decides the canbreak exit bit for bit.                  */
    const int32_t *point_rank;
} ldso_ba_window;

/* Per-frame state needed by FrameFramePrecalc::Set / setAdjointsF / takeData. */
typedef struct ldso_ba_frame_state {
    double world_to_cam_evalpt[12]; /* FrameHessian::worldToCam_evalPT: R (3x3 row-major), t */
    double state[10];               /* FrameHessian::state                                   */
    double state_zero[10];          /* FrameHessian::state_zero                              */
    double ab_exposure;             /* FrameHessian::ab_exposure                             */
    int32_t is_first_frame;         /* frame->id == 0 (FrameHessian::getPrior)              */
    int32_t pad_;
} ldso_ba_frame_state;

typedef struct ldso_ba_ctx ldso_ba_ctx;
struct ldso_ba_opt_settings; /* defined with ldso_ba_check_settings below */

/* ---- host-side helpers (no GPU needed) ---------------------------------------------- */

int ldso_ba_abi_version(void);
const char *ldso_ba_last_error(void);

/* FrameFramePrecalc::Set for every (h,t) pair and the per-frame PRE_worldToCam.
 * precalc_out: [N*N][LDSO_BA_PRECALC_STRIDE] (index h + N*t).              FrameFramePrecalc.cc:6-35 */
int ldso_ba_frame_precalc(int32_t n_frames, const ldso_ba_frame_state *frames, const float calib[4],
                          float *precalc_out);

/* EnergyFunctional::setAdjointsF (EnergyFunctional.cc:551-609): adHost/adTarget [N*N][64] and
 * cPrior [4] (= setting_initialCalibHessian). */
int ldso_ba_set_adjoints(int32_t n_frames, const ldso_ba_frame_state *frames, double *ad_host,
                         double *ad_target, double *c_prior);

/* FrameHessian::takeData (FrameHessian.cc:131-135): prior, delta, delta_prior [N][8].  The prior
 * (getPrior, FrameHessian.h:142-170) follows settings->affine_opt_mode_a / _b (NULL: the defaults);
 * settings are checked (ldso_ba_check_settings). */
int ldso_ba_frame_take_data(int32_t n_frames, const ldso_ba_frame_state *frames, const struct ldso_ba_opt_settings *settings,
                            double *prior, double *delta, double *delta_prior);

/* Solve assembly + Jacobi-scaled LDLT + optional nullspace projection, the non-VI branch of
 * EnergyFunctional::solveSystemF (EnergyFunctional.cc:280-471) in the default solver mode
 * (FIX_LAMBDA | ORTHOGONALIZE_X_LATER).  settings (NULL: the defaults) are checked first: another
 * solver mode or vi_enable returns < 0.  Inputs are the stitched blocks; HM/bM may be NULL (no
 * marginalisation prior).  nullspaces: [n_null][8N+4] column vectors (getNullspaces order) used when
 * (iteration >= 2), may be NULL.  x_out: [8N+4]. */
int ldso_ba_solve_system(const struct ldso_ba_opt_settings *settings, int32_t n_frames, int32_t iteration,
                         double lambda, const double *HA, const double *bA, const double *HL, const double *bL,
                         const double *HM, const double *bM, const double *Hsc, const double *bsc,
                         const double *nullspaces, int32_t n_null, double *x_out);

/* FrameHessian::setStateZero nullspaces + FullSystem::getNullspaces (FullSystem.cc:2027-2076):
 * out [7][8N+4] = the 6 pose nullspaces then the scale nullspace, the vectors
 * EnergyFunctional::orthogonalize stacks (EnergyFunctional.cc:811-813). */
int ldso_ba_nullspaces(int32_t n_frames, const ldso_ba_frame_state *frames, double *out);

/* Validate a window description without a GPU (what ldso_ba_load checks first): counts,
 * pointers, host/target ranges, residual lists (no duplicate or self targets, <= N-1 per
 * point).  Returns 0 or a negative code with ldso_ba_last_error() set. */
int ldso_ba_validate_window(const ldso_ba_window *w);

/* EnergyFunctional::marginalizeFrame (EnergyFunctional.cc:109-191), the dense part: frame idx's
 * 8 rows/columns of HM, bM (dimension 8N+4, row-major) are moved to the end, its prior
 * (FrameHessian::prior, delta_prior [8]) added, the block Schur-complemented out after
 * Jacobi scaling with MatrixInverter::invertPosDef (pseudo-inverse) and the result symmetrised.
 * Outputs HM_out (8(N-1)+4)^2 and bM_out 8(N-1)+4. */
int ldso_ba_marginalize_frame(int32_t n_frames, int32_t idx, const double *HM, const double *bM,
                              const double *prior, const double *delta_prior, double *HM_out,
                              double *bM_out);

/* EnergyFunctional::setDeltaF's adHTdeltaF (EnergyFunctional.cc:523-533): [N*N][8] float (index
 * h + N t) = delta_h^T adHostF + delta_t^T adTargetF, from the frames' delta [N][8]
 * (ldso_ba_frame_take_data) and the adjoints of ldso_ba_set_adjoints. */
int ldso_ba_ad_ht_delta(int32_t n_frames, const double *delta, const double *ad_host, const double *ad_target,
                        float *out);

/* EnergyFunctional::calcMEnergyF (EnergyFunctional.cc:473-479): out = d^T (2 bM + HM d), d =
 * [cDeltaF; delta of every frame] (getStitchedDeltaF), HM row-major (8N+4)^2. */
int ldso_ba_calc_m_energy(int32_t n_frames, const double *HM, const double *bM, const float *c_delta,
                          const double *delta, double *out);

/* EnergyFunctional::calcLEnergyF_MT (EnergyFunctional.cc:481-498, calcLEnergyPt :751-806): frame
 * priors (prior, delta_prior [N][8]), calibration prior (cPrior [4], cDeltaF [4]) and every
 * point's deltaF^2 priorF (Accumulator11 over 50-point chunks).  The linearised-residual term is
 * empty in this library (residuals are linearised only inside ldso_ba_marginalize_points, which
 * consumes their points). */
int ldso_ba_calc_l_energy(int32_t n_frames, const double *prior, const double *delta_prior, const double *c_prior,
                          const float *c_delta, int32_t n_points, const float *deltaF, const float *priorF,
                          double *out);

/* ---- multi-GPU -------------------------------------------------------
 * Points are sharded by host frame: in host-frame order the window's points are cut into
 * `count` contiguous runs of equal residual counts (ldso_ba_load keeps run `rank`); a host is
 * split only where a cut falls inside it.  points_out (may be NULL) receives the caller indices
 * of run `rank`, *n_out their number. */
int ldso_ba_shard_points(const ldso_ba_window *w, int32_t rank, int32_t count, int32_t *points_out,
                         int32_t *n_out);
/* The packed layout the ranks reduce (ldso_ba_packed_system): upper triangles, row-major,
 * [HA (dim(dim+1)/2), bA (dim), Hsc (dim(dim+1)/2), bsc (dim)]; unpack_upper mirrors to full. */
int ldso_ba_pack_upper(int32_t dim, const double *HA, const double *bA, const double *Hsc, const double *bsc,
                        double *packed);
int ldso_ba_unpack_upper(int32_t dim, const double *packed, double *HA, double *bA, double *Hsc, double *bsc);
/* setNewFrameEnergyTH over gathered newest-frame NewEnergyWithOutlier values (< 0 = padding). */
int ldso_ba_frame_threshold(const float *values, int64_t n, float *th_out);

/* ---- device context --------------------------------------------------------------- */

/* Create a context on HIP device `device` with its own non-blocking stream. */
int ldso_ba_create(int32_t device, ldso_ba_ctx **out);
void ldso_ba_destroy(ldso_ba_ctx *ctx);

/* The HIP stream (hipStream_t) every kernel of this context is launched on. */
void *ldso_ba_stream(ldso_ba_ctx *ctx);

/* In-library exchange over RCCL (xGMI): rank 0 makes the id, the caller hands it to every rank
 * (any channel), each rank attaches its context.  From then on every ldso_ba_linearize ends,
 * stream-ordered and without a host synchronisation, with the exchange of SURVEY §8e in TWO
 * collectives: ONE sum all-reduce (fp64) of a contiguous buffer holding the packed systems (with
 * accumulate) and the energy / #IN pairs; then an all-gather of per-window slots -- the newest-frame
 * energies, followed by the exact threshold re-selection, and inside ldso_ba_optimize each rank's
 * run of |idepth|, from which every rank walks doStepFromBackup's whole sumNID chain.  Load each
 * rank with ldso_ba_load(ctx, n, windows, rank, world).
 * Exactness: the system and energies of a sharded pass are those of the unsharded pass up to the
 * reassociation of float sums the block tolerance already allows; the threshold and sumNID / numID
 * are the single-GPU ones bit for bit (the runs concatenated in rank order are the unsharded
 * host-frame order, FullSystem.cc:1899-1909's one float chain), so a sharded window's canbreak
 * exit is decided on the same sumNID as on one GPU. */
#define LDSO_BA_COMM_ID_BYTES 128
int ldso_ba_comm_unique_id(uint8_t *id_out);
int ldso_ba_comm_init(ldso_ba_ctx *ctx, const uint8_t *id, int32_t rank, int32_t world);

/* (Re)build the device mirror of n_windows windows (EnergyFunctional::insertFrame /
 * insertResidual / dropResidual / makeIDX all end here).  shard_count > 1 keeps only run
 * shard_rank of the host-frame partition (ldso_ba_shard_points: the points in host-frame order
 * cut into shard_count contiguous runs of equal residual counts), for multi-GPU sharding.  The
 * priors (HL, bL) are not part of the reduced packed system, so every shard keeps them and every
 * rank's (redundant) solve sees them.  Every window must share width/height. */
int ldso_ba_load(ldso_ba_ctx *ctx, int32_t n_windows, const ldso_ba_window *windows,
                 int32_t shard_rank, int32_t shard_count);

/* Refresh per-iteration state of window `win` after doStepFromBackup / setPrecalcValues:
 * precalc, adjoints, priors, cDeltaF, frame_energy_th and point_data (all 24 floats per point;
 * w->point_data == NULL leaves the points as they are, see ldso_ba_update_points).
 * Structure (points, residual lists) must be unchanged. */
int ldso_ba_update(ldso_ba_ctx *ctx, int32_t win, const ldso_ba_window *w);

/* The per-step point values only (PointHessian::setIdepth / setIdepthZero, priorF, deltaF after
 * doStepFromBackup / setDeltaF; EnergyFunctional.cc:523-549): vals [P][4] in the caller's point
 * order = (idepth_scaled, idepth_zero_scaled, priorF, deltaF).  16 B per point instead of the 96-B
 * record of ldso_ba_update. */
int ldso_ba_update_points(ldso_ba_ctx *ctx, int32_t win, const float *vals);

/* Residual states edited on the host (PointFrameResidual::resetOOB / applyRes / setState,
 * Residuals.h:63-88) into the device mirror, caller order [R]: state_state, state_energy,
 * state_NewEnergy, flags (LDSO_BA_FLAG_*). */
int ldso_ba_update_residuals(ldso_ba_ctx *ctx, int32_t win, const int8_t *state, const float *state_energy,
                             const float *new_energy, const uint8_t *flags);

/* PointFrameResidual::linearize (Residuals.cc:15-217) of every residual of window win as it returns
 * right after the residual's resetOOB() -- FullSystem::flagPointsForRemoval's per-residual
 * relinearisation (FullSystem.cc:1390-1398) -- in one device pass, without applyRes,
 * setNewFrameEnergyTH or accumulation: the context's residual states, records and system are left
 * as they were.  Outputs in caller order (any may be NULL): new_state [R] (state_NewState),
 * new_energy [R] (state_NewEnergy = the returned energy unless new_state is OOB), new_energy_wo [R]
 * (state_NewEnergyWithOutlier, -1 when OOB), center [R][3] and center_ok [R] (centerProjectedTo;
 * 0: the centre projection failed and the reference leaves centerProjectedTo unchanged), jpjdf
 * [R][8] (the JpJdF applyRes(true)'s takeData forms from this linearisation, where new_state is
 * IN; 0 elsewhere).  A residual whose state is OOB returns state_energy in the reference without
 * any computation; the caller keeps that branch.  Single-shard windows only (a sharded window
 * holds only its run of the residuals: -1), not on a marginalisation context (-1). */
int ldso_ba_linearize_residuals(ldso_ba_ctx *ctx, int32_t win, int8_t *new_state, float *new_energy,
                                float *new_energy_wo, float *center, uint8_t *center_ok, float *jpjdf);

/* PointFrameResidual::resetOOB for every residual of window win (win < 0: all windows). */
int ldso_ba_reset_oob(ldso_ba_ctx *ctx, int32_t win);

/* Point marginalisation.  `marg` is a context of its own whose single
 * window holds the points being marginalised (FullSystem::flagPointsForRemoval's MARGINALIZED
 * points, FullSystem.cc:1384-1404) and their residuals; its frames are window parent_win of
 * `parent`, whose device images are borrowed (points->dI may be NULL; the parent must stay
 * loaded while marg is used).  priorF is scaled by setting_idepthFixPriorMargFac at load
 * (EnergyFunctional.cc:216). */
int ldso_ba_load_marginalization(ldso_ba_ctx *marg, const ldso_ba_ctx *parent, int32_t parent_win,
                                 const ldso_ba_window *points);
/* For every residual: resetOOB, linearize, applyRes(true) and, if active, fixLinearizationF
 * (FullSystem.cc:1390-1398, Residuals.cc:219-245); then AccumulatedTopHessianSSE::addPoint<2> and
 * AccumulatedSCHessianSSE::addPoint(p, false) with both stitches (EnergyFunctional.cc:226-243).
 * ad_ht_delta: EnergyFunctional::adHTdeltaF [N*N][8] (float, index h + N t).  Outputs
 * H = M - Msc ((8N+4)^2, full symmetric) and b = Mb - Mbsc; the caller adds
 * setting_margWeightFac * (H, b) to (HM, bM) (EnergyFunctional.cc:254-255).  Residual states and
 * points of `marg` are readable with get_residuals / get_points as after a pass. */
int ldso_ba_marginalize_points(ldso_ba_ctx *marg, const float *ad_ht_delta, double *H, double *b);

/* ---- point activation ----
 * FullSystem::optimizeImmaturePoint(point, min_obs, residuals) (FullSystem.cc:1035-1156) for n
 * immature points of window `win`: ImmaturePoint::linearizeResidual (ImmaturePoint.cc:319-389)
 * against every other frame of the window in window order, from idepth (min + max) / 2, then
 * setting_GNItsOnPointActivation LM steps on the inverse depth.  pts: ldso_ct_immature records
 * (include/ldso_ct.h; u, v, idepth_min/max, energy_th, color, weights, host = frame index in the
 * window).  Uses the context's images, FrameFramePrecalc (PRE_RTll, PRE_tTll, PRE_aff_mode) and
 * calibration as last loaded / set.  activatePointsMT calls it with min_obs = 1. */
struct ldso_ct_immature;
typedef struct ldso_ba_activation {
    float idepth;      /* currentIdepth at return                                              */
    int32_t status;    /* 0: a PointHessian is created (setIdepth(idepth)); 1: nullptr (idepth not
                          finite, or fewer than min_obs IN residuals); 2: 0 (energy not finite or
                          Hdd < setting_minIdepthH_act)                                        */
    uint32_t in_mask;  /* status 0: bit f set = the residual to window frame f is IN and moves
                          into the new point (lastResiduals follow from frames N-1, N-2)       */
    float energy;      /* lastEnergy at return                                                 */
} ldso_ba_activation;
int ldso_ba_activate_points(ldso_ba_ctx *ctx, int32_t win, int32_t n, const struct ldso_ct_immature *pts,
                            int32_t min_obs, ldso_ba_activation *out);

/* One hot-path pass over all loaded windows, asynchronous on the context stream:
 *   linearizeAll(fix) + applyRes(true) + setNewFrameEnergyTH, and if accumulate != 0
 *   accumulateAF_MT + accumulateLF_MT + accumulateSCF_MT with both stitches.
 * Mode-0 (active) accumulation uses the Jacobians of this same pass, exactly as the
 * reference's solveSystemF uses those of the preceding linearizeAll + applyRes. */
int ldso_ba_linearize(ldso_ba_ctx *ctx, int32_t fix, int32_t accumulate);

int ldso_ba_sync(ldso_ba_ctx *ctx);

/* Results of the last ldso_ba_linearize for window win (synchronising). */
/* energy_out[3] = {sum of linearize() energies (double), 0, number of NewState == IN}.     */
int ldso_ba_get_energy(ldso_ba_ctx *ctx, int32_t win, double *energy_out);
/* Any output pointer may be NULL.  Sizes (8N+4)^2 and (8N+4). */
int ldso_ba_get_system(ldso_ba_ctx *ctx, int32_t win, double *HA, double *bA, double *HL,
                       double *bL, double *Hsc, double *bsc);
/* Per residual, in the caller's point-major order. Any pointer may be NULL.
 *   new_state/state [R], state_energy/new_energy_wo [R], center [R][3] (centerProjectedTo),
 *   flags [R], jpjdf [R][8] (JpJdF of the last pass, formed from the pass's record and geometry;
 *   0 where that pass left the residual inactive -- the reference keeps a stale JpJdF there, which
 *   nothing reads), rel_bs [R] (linearizeAll_Reductor relBS, fix pass). */
int ldso_ba_get_residuals(ldso_ba_ctx *ctx, int32_t win, int8_t *new_state, int8_t *state,
                          float *state_energy, float *new_energy_wo, float *center,
                          uint8_t *flags, float *jpjdf, float *rel_bs);
/* Per point (caller order): HdiF, bdSumF, idepth_hessian, Hdd_accAF, bd_accAF, Hcd_accAF[4].
 * Points with no active residual report HdiF = bdSumF = idepth_hessian = 0. */
int ldso_ba_get_points(ldso_ba_ctx *ctx, int32_t win, float *HdiF, float *bdSumF,
                       float *idepth_hessian, float *Hdd_acc, float *bd_acc, float *Hcd_acc);
int ldso_ba_get_frame_energy_th(ldso_ba_ctx *ctx, int32_t win, float *th);

/* solveSystemF on the stitched system of the last pass (get_system + ldso_ba_solve_system):
 * priors come from the window's frame_prior / c_prior, HM = bM = 0. x_out [8N+4]. */
int ldso_ba_solve(ldso_ba_ctx *ctx, int32_t win, int32_t iteration, double lambda,
                  const double *nullspaces, int32_t n_null, double *x_out);

/* EnergyFunctional::resubstituteF_MT (EnergyFunctional.cc:611-667) on the device for window
 * win: x [8N+4], point_step_out [P] (PointHessian::step; NULL keeps it on the device). */
int ldso_ba_resubstitute(ldso_ba_ctx *ctx, int32_t win, const double *x, double lambda,
                         float *point_step_out);

/* Device pointer of the packed per-window partial system used for multi-GPU all-reduce:
 * [n_windows][sys_len] doubles, sys_len = 2*((8N+4)*(8N+5)/2 + (8N+4)) laid out as
 * {HA upper-tri, bA, Hsc upper-tri, bsc}.  After an external all-reduce (sum) call
 * ldso_ba_unpack_system so that get_system / solve read the reduced values. */
int ldso_ba_packed_system(ldso_ba_ctx *ctx, void **dev_ptr, int64_t *n_doubles, int64_t *stride);
int ldso_ba_unpack_system(ldso_ba_ctx *ctx);
/* Device-to-device copy of the packed partial systems to (direction 0) or from (direction 1)
 * a caller-owned device buffer of n_doubles (e.g. a torch tensor handed to RCCL); synchronises
 * the context stream.  Direction 1 also invalidates cached host copies.  The copy runs on the
 * context stream: work the caller queued on another stream that writes dev_buf (direction 1) or
 * reads it must be ordered by the caller (e.g. synchronise that stream before the call). */
int ldso_ba_copy_packed(ldso_ba_ctx *ctx, void *dev_buf, int64_t n_doubles, int32_t direction);

/* Sharded setNewFrameEnergyTH (FullSystem.cc:2078-2109 over activeResiduals that target the
 * newest frame).  With points sharded, each rank holds part of the newest frame's
 * NewEnergyWithOutlier values; the exact nth_element needs all of them:
 *   newest_stride       max over this context's windows of its newest-frame residual count
 *                       (static after load; ranks agree on max-over-ranks as the slot size)
 *   export_newest       writes [n_windows][stride] floats into a caller device buffer (-1 pads)
 *   frame_threshold_gathered  takes the all-gathered [n_ranks][n_windows][stride] buffer and
 *                       re-selects every window's newest-frame threshold on the device.
 * All three synchronise the context stream (buffers the caller fills on another stream must be
 * complete before the call).  Unsharded contexts never need them. */
int ldso_ba_newest_stride(ldso_ba_ctx *ctx, int64_t *stride);
int ldso_ba_export_newest(ldso_ba_ctx *ctx, float *dev_buf, int64_t stride);
int ldso_ba_frame_threshold_gathered(ldso_ba_ctx *ctx, const float *dev_buf, int32_t n_ranks, int64_t stride);

/* Device-side solve and resubstitution, every loaded window at once:
 *   solve_device         EnergyFunctional::solveSystemF on the GPU, one workgroup per window, for
 *                        windows of up to 11 keyframes: by default the unpivoted blocked LDL^T
 *                        (k_solve_fast); with LDSO_BA_TUNE_SOLVE_EXACT = 1 statement for statement
 *                        ldso_ba_solve with its diagonal pivoting (k_solve_reg: 5 wavefronts, up to 7
 *                        keyframes; k_solve: 4 wavefronts, up to 11; x bit-identical).  ns: every window's [7][8N+4] nullspaces back to back; the projection
 *                        (iteration >= 2) uses the nullspaces of THIS call and is skipped when ns is
 *                        NULL, as in the host solver.  x_out: every window's x back to back (or NULL:
 *                        x stays on the device for resubstitute_device).
 *   resubstitute_device  resubstituteF_MT from the device x; point_step_out (or NULL): every
 *                        window's points back to back, each in its caller order.
 *   iterate              linearize(fix=0, accumulate=1) + solve_device + resubstitute_device with
 *                        one synchronisation; energy_out: [n_windows][3] as ldso_ba_get_energy. */
int ldso_ba_solve_device(ldso_ba_ctx *ctx, int32_t iteration, double lambda, const double *ns, int32_t n_null,
                         double *x_out);
int ldso_ba_resubstitute_device(ldso_ba_ctx *ctx, double lambda, float *point_step_out);
int ldso_ba_iterate(ldso_ba_ctx *ctx, int32_t iteration, double lambda, const double *ns, int32_t n_null,
                    double *x_out, float *point_step_out, double *energy_out);

/* setting_solverMode bits (Settings.h:14-25).  The library implements the reference's default
 * mode, SOLVER_FIX_LAMBDA | SOLVER_ORTHOGONALIZE_X_LATER (Setting.cc:23); every other bit is
 * rejected (ldso_ba_check_settings) rather than silently run as the default. */
#define LDSO_BA_SOLVER_SVD 1
#define LDSO_BA_SOLVER_ORTHOGONALIZE_SYSTEM 2
#define LDSO_BA_SOLVER_ORTHOGONALIZE_POINTMARG 4
#define LDSO_BA_SOLVER_ORTHOGONALIZE_FULL 8
#define LDSO_BA_SOLVER_SVD_CUT7 16
#define LDSO_BA_SOLVER_REMOVE_POSEPRIOR 32
#define LDSO_BA_SOLVER_USE_GN 64
#define LDSO_BA_SOLVER_FIX_LAMBDA 128
#define LDSO_BA_SOLVER_ORTHOGONALIZE_X 256
#define LDSO_BA_SOLVER_MOMENTUM 512
#define LDSO_BA_SOLVER_STEPMOMENTUM 1024
#define LDSO_BA_SOLVER_ORTHOGONALIZE_X_LATER 2048
#define LDSO_BA_SOLVER_DEFAULT (LDSO_BA_SOLVER_FIX_LAMBDA | LDSO_BA_SOLVER_ORTHOGONALIZE_X_LATER)

/* The reference's global settings (src/Setting.cc) that change this path's arithmetic or control
 * flow.  A caller copies its globals into this struct and hands it to
 * ldso_ba_set_settings (per context), ldso_ba_optimize, ldso_ba_frame_take_data and
 * ldso_ba_solve_system; every one of them runs ldso_ba_check_settings first, so a setting this
 * library does not implement is refused (< 0 and a message) instead of silently run as the default.
 * Start from LDSO_BA_OPT_SETTINGS_INIT (or ldso_ba_default_settings) so that fields added later
 * keep their defaults. */
typedef struct ldso_ba_opt_settings {
    int32_t solver_mode;         /* setting_solverMode (LDSO_BA_SOLVER_DEFAULT, Setting.cc:23)     */
    int32_t force_accept_step;   /* setting_forceAceptStep (1, :73); 0 is rejected                  */
    int32_t min_opt_iterations;  /* setting_minOptIterations (1, :37)                               */
    float th_opt_iterations;     /* setting_thOptIterations (1.2f, :38)                             */
    /* setting_affineOptModeA / B (1e12 / 1e8, Setting.cc:65-66; the KITTI / EuRoC drivers set 0 / 0,
     * run_dso_kitti.cc:299-300, run_dso_euroc.cc:291-292; TUM-Mono mode 2 sets -1 / -1):
     *   >= 0  the affine parameter is optimised with this value as its prior (FrameHessian::getPrior,
     *         FrameHessian.h:154-165; 0 = no prior);
     *   <  0  it is fixed: prior setting_initialAffA/BPrior (1e14) and JabF[0] / JabF[1] zeroed after
     *         the pattern sums (Residuals.cc:186-187), which removes it from Jab_r (the Top block's
     *         b rows of a / b) and from fixLinearizationF's res_toZeroF (Residuals.cc:239-240).
     * Must be finite. */
    float affine_opt_mode_a;
    float affine_opt_mode_b;
    /* setting_vi_enable (Setting.cc:152: true in the reference; its drivers do not turn it off).
     * The inertial terms (combineInertialHessians, H_I / b_I in solveSystemF, linearizeInertial,
     * the inertial step of doStepFromBackup: EnergyFunctional.cc:307-376, FullSystem.cc:879-926,
     * 1871-1931) are not implemented: 1 is refused.  Visual-only LDSO runs with 0. */
    int32_t vi_enable;
    int32_t reserved_;           /* 0 */
} ldso_ba_opt_settings;

#define LDSO_BA_OPT_SETTINGS_INIT {LDSO_BA_SOLVER_DEFAULT, 1, 1, 1.2f, 1e12f, 1e8f, 0, 0}

/* Writes the defaults above (the reference's Setting.cc values, vi_enable = 0) into *s. */
void ldso_ba_default_settings(ldso_ba_opt_settings *s);

/* 0 when the settings are what this library runs, else -1 with a message naming the first
 * unsupported setting (SVD / SVD_CUT7 / ORTHOGONALIZE_SYSTEM / USE_GN / MOMENTUM / STEPMOMENTUM /
 * ... , force_accept_step == 0, whose accept / reject branch FullSystem.cc:935-966 is absent,
 * vi_enable != 0, a non-finite affine mode).  NULL means the defaults (accepted). */
int ldso_ba_check_settings(const ldso_ba_opt_settings *s);

/* Install settings into a context (NULL: the defaults; a new context starts with the defaults).
 * Checked first: a rejected set returns < 0 and leaves the context's settings unchanged, so a
 * context never holds settings the library does not implement.  Every entry point that runs the
 * path on the context reads them: ldso_ba_linearize (JabF zeroing), ldso_ba_marginalize_points
 * (res_toZeroF; a marginalisation context takes its parent's settings at
 * ldso_ba_load_marginalization), ldso_ba_solve / _solve_device / _iterate (solver mode) and
 * ldso_ba_optimize (all of them; its frame step forms the affine priors from them). */
int ldso_ba_set_settings(ldso_ba_ctx *ctx, const ldso_ba_opt_settings *s);
int ldso_ba_get_settings(ldso_ba_ctx *ctx, ldso_ba_opt_settings *out);

/* Per-window outcome of ldso_ba_optimize (status_out). */
#define LDSO_BA_OPT_RAN_ALL 0      /* n_its iterations, no early exit                            */
#define LDSO_BA_OPT_CONVERGED 1    /* doStepFromBackup's canbreak after >= min_opt_iterations    */
#define LDSO_BA_OPT_LOST 2         /* lastX had a NaN norm: FullSystem.cc:907-911 isLost = true  */

/* FullSystem::optimize (FullSystem.cc:844-970) on the device for every loaded window, with
 * setting_forceAceptStep (the default) and the non-momentum doStepFromBackup: resetOOB, one
 * linearizeAll + applyRes, then up to n_its times {solveSystemF (k_solve; orthogonalize with ns
 * from iteration 2), resubstituteF_MT, doStepFromBackup (FullSystem.cc:1826-1931: frame states by
 * log(exp(step) exp(state)), CalibHessian::setValue, point setIdepth / setIdepthZero) +
 * setPrecalcValues (FrameFramePrecalc::Set for every pair, the prior vector), linearizeAll +
 * applyRes}, all on the context stream with no host round trip; one synchronisation at the end.
 * Each window leaves the loop on its own, as the reference's loop does:
 *   - lost (FullSystem.cc:907-911): the solve's x has a NaN element (isnan(lastX.norm())): no
 *     step is applied in that iteration and the window stops (status LDSO_BA_OPT_LOST; the
 *     reference returns DBL_MAX and sets isLost);
 *   - converged (FullSystem.cc:968-969): doStepFromBackup's canbreak -- sqrtf of the frame-averaged
 *     squared a, b, rotation and translation steps (the translation term times the mean
 *     |idepth_backup| of the window's points, summed in the window's point order, hosts in
 *     window order) below 5e-4 / 5e-5 x th_opt_iterations (FullSystem.cc:1914-1931) -- once
 *     iteration >= min_opt_iterations: the pass after that step still runs, then the window stops.
 * A stopped window's later launches are no-ops inside the same (captured) sequence.
 *   settings: NULL = the context's settings (ldso_ba_set_settings); otherwise they are checked and
 *   installed into the context first, exactly as ldso_ba_set_settings does (anything
 *   ldso_ba_check_settings rejects returns -1 and runs nothing).
 *   frames [sum N]: the windows' frame states back to back; calib_value / calib_value_zero
 *   [n_windows][4]: CalibHessian::value / value_zero (unscaled: value_scaled = 50 value);
 *   ns: [7][sum (8N+4)] nullspaces (ldso_ba_nullspaces per window, back to back) or NULL.
 * Outputs (any may be NULL): energy_out [n_its + 1][n_windows][3] = (E, 0, #IN) of the initial
 * and every iteration's linearizeAll (rows after a window stopped repeat its last pass, the
 * reference's lastEnergy); frames_out / calib_out the stepped states; idepth_out [sum P] the
 * points' idepth, caller order; iterations_out [n_windows] the loop iterations entered (solves
 * run); status_out [n_windows] LDSO_BA_OPT_*.  Afterwards the context's precalc, calibration,
 * priors and point data are the stepped ones (ldso_ba_update overrides them as before).  The
 * reference's iteration-count override for windows of 2-3 frames (FullSystem.cc:846-851) is the
 * caller's (the C++ face applies it). */
int ldso_ba_optimize(ldso_ba_ctx *ctx, int32_t n_its, const ldso_ba_opt_settings *settings,
                     const ldso_ba_frame_state *frames, const double *calib_value, const double *calib_value_zero,
                     const double *ns, double *energy_out, ldso_ba_frame_state *frames_out, double *calib_out,
                     float *idepth_out, int32_t *iterations_out, int32_t *status_out);

/* doStepFromBackup's frame and calibration step on the host (the same se3.h statements as the
 * device loop): out[f] = in[f] stepped by -x[4 + 8f ..]; calib_value (if not NULL) += -x[0..3],
 * with value_scaledf and cDeltaF = value - value_zero returned if the pointers are not NULL. */
int ldso_ba_frame_step(int32_t n_frames, const ldso_ba_frame_state *in, const double *x, ldso_ba_frame_state *out,
                       double *calib_value, const double *calib_value_zero, float *calib_scaled_out,
                       float *c_delta_out);

/* doStepFromBackup's canbreak (FullSystem.cc:1894-1931, visual-only, stepfac 1) on the host, the
 * statements the device loop evaluates (se3.h step_canbreak): from the window's x [8N+4] (step = -x),
 * sumNID (the float sum of |idepth_backup| over the window's points in frames -> features order;
 * with sharded points the same chain over the gathered runs), numID and setting_thOptIterations.
 * *canbreak_out = 1 or 0. */
int ldso_ba_step_canbreak(int32_t n_frames, const double *x, float sum_nid, float num_id, float th_opt_iterations,
                          int32_t *canbreak_out);

/* Per-kernel HIP-event timing (bench/profiling).  When enabled every kernel launch of
 * ldso_ba_linearize is bracketed by events; get returns summed ms and launch counts for
 * n_kernels <= 16 slots in the order of ldso_ba_kernel_name(i). */
int ldso_ba_set_kernel_timing(ldso_ba_ctx *ctx, int32_t enable);

/* Tuning knobs (defaults are the measured best):
 *   LDSO_BA_TUNE_TILED_IMAGES  frame layout: 3 (default) intensity only, band-interleaved, the
 *                              gradients recomputed with makeImages' rule (falls back to 1 when the
 *                              caller's dI gradients are not makeImages'); 1 [I, dx, dy, 0]
 *                              texels in 2x4 tiles; set before ldso_ba_load
 *   LDSO_BA_TUNE_TOP_CHUNK     residuals per k_linearize wavefront: a multiple of 8 up to 64, or 0 = automatic
 *                              (64 for large batches, shorter for a single window); set before
 *                              ldso_ba_load
 *   LDSO_BA_TUNE_TIMING_MASK   bit i: bracket kernel slot i with events when timing is enabled
 *                              (default all; each event pair costs the stream a few us)
 *   LDSO_BA_TUNE_ITEM_ORDER    k_linearize chunk order: 0 (default) target-major, 1 host-major, 2
 *                              target-major with each bucket's residuals ranked by their projection
 *                              into the target and dealt over its chunks in groups of 8 (fewer L2
 *                              re-reads, slower: DESIGN.md 5e); set before ldso_ba_load
 *   LDSO_BA_TUNE_SOLVE_EXACT   device solve (solve_device / iterate / optimize): 0 (default) the
 *                              unpivoted blocked LDL^T (k_solve_fast: the Jacobi-scaled, damped system
 *                              is positive definite; x within rounding of the pivoted solve); 1 the
 *                              pivoted factorisation of the host solver (k_solve_reg / k_solve,
 *                              x bit-identical to ldso_ba_solve)
 * Keys 1, 3, 4, 5, 8, 9, 11 and 14 named experiment variants that measured slower and were removed
 * (DESIGN.md §5 keeps their numbers); setting them returns -1. */
#define LDSO_BA_TUNE_TILED_IMAGES 2
#define LDSO_BA_TUNE_TOP_CHUNK 6
#define LDSO_BA_TUNE_TIMING_MASK 7
#define LDSO_BA_TUNE_ITEM_ORDER 10
#define LDSO_BA_TUNE_SOLVE_EXACT 12
int ldso_ba_set_tuning(ldso_ba_ctx *ctx, int32_t key, int32_t value);
int ldso_ba_get_kernel_times(ldso_ba_ctx *ctx, double *ms, int64_t *counts, int32_t n);
const char *ldso_ba_kernel_name(int32_t i);
int32_t ldso_ba_num_kernels(void);

/* Size of the device-resident data for the loaded windows (bytes) and total counts. */
int ldso_ba_stats(ldso_ba_ctx *ctx, int64_t *device_bytes, int64_t *n_points,
                  int64_t *n_residuals);

#ifdef __cplusplus
}
#endif

#endif /* LDSO_BA_H_ */
