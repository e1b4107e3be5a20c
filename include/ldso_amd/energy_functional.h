/*
 * energy_functional.h -- C++ host face of the MI355X bundle-adjustment hot path.
 *
 * The class surface LDSO's FullSystem drives (names, members, argument order and shared_ptr /
 * weak_ptr ownership of the reference; paths relative to n-lalanne/LDSO):
 *
 *   EnergyFunctional     include/internal/OptimizationBackend/EnergyFunctional.h:55-186
 *                        insertResidual / insertFrame / dropResidual / marginalizeFrame /
 *                        removePoint / marginalizePointsF / dropPointsF / solveSystemF /
 *                        calcMEnergyF / calcLEnergyF_MT / makeIDX / setDeltaF / setAdjointsF /
 *                        resubstituteF_MT; public frames, nPoints, nFrames, nResiduals, HM, bM,
 *                        resInA/L/M, lastX, lastNullspaces_*, connectivityMap
 *   PointFrameResidual   include/internal/Residuals.h:42-131 (linearize, resetOOB, applyRes,
 *                        setState, isActive, fixLinearizationF, takeData's JpJdF, state_*)
 *   FrameHessian         include/internal/FrameHessian.h (state, state_zero, step, prior, delta,
 *                        delta_prior, idx, frameID, frameEnergyTH, flaggedForMarginalization, dI)
 *   PointHessian         include/internal/PointHessian.h (u, v, idepth*, color, weights, priorF,
 *                        deltaF, residuals, HdiF, bdSumF, idepth_hessian, step, setIdepth*)
 *   CalibHessian         include/internal/CalibHessian.h (value_scaledf, value_minus_value_zero, step)
 *   + linearizeAll(fix)  FullSystem::linearizeAll (FullSystem.cc:1716-1769) with applyRes and
 *                        setNewFrameEnergyTH, and the accumulate{AF,LF,SCF} of the next solve
 *
 * It lives in namespace ldso_amd, not ldso::internal: the reference's own FrameHessian /
 * PointHessian carry the frontend's state (images, pyramids, features) and stay where they are;
 * INTEGRATION.md §3 gives the literal forwarding bodies that make the reference's
 * EnergyFunctional.cc / Residuals.cc methods call these.  Eigen's VecX / MatXX are mirrored by
 * the small row-major VecX / MatXX below (this header needs no Eigen).
 *
 * Every number comes from the HIP path or from the library's host helpers through the C ABI of
 * include/ldso_ba.h; nothing here computes except packing.  Like the reference, nothing throws:
 * failures leave ok() false and lastError() set.
 */
#ifndef LDSO_AMD_ENERGY_FUNCTIONAL_H_
#define LDSO_AMD_ENERGY_FUNCTIONAL_H_

#include <array>
#include <cmath>
#include <cstdint>
#include <cstddef>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../ldso_ba.h"

namespace ldso_amd {

using std::shared_ptr;
using std::weak_ptr;

constexpr int CPARS = 4;                  // NumTypes.h:25
constexpr float SCALE_IDEPTH = 1.0f;      // Settings.h:28
using Vec3 = std::array<double, 3>;

// Eigen::VectorXd stand-in (the members the reference's callers use)
struct VecX {
    std::vector<double> v;
    VecX() = default;
    explicit VecX(int n, double x = 0.0) : v((size_t)n, x) {}
    static VecX Zero(int n) { return VecX(n); }
    static VecX Constant(int n, double x) { return VecX(n, x); }
    int size() const { return (int)v.size(); }
    double &operator[](int i) { return v[(size_t)i]; }
    double operator[](int i) const { return v[(size_t)i]; }
    double &operator()(int i) { return v[(size_t)i]; }
    double operator()(int i) const { return v[(size_t)i]; }
    double *data() { return v.data(); }
    const double *data() const { return v.data(); }
    double dot(const VecX &o) const {
        double s = 0;
        for (size_t i = 0; i < v.size(); i++) s += v[i] * o.v[i];
        return s;
    }
    double norm() const { return std::sqrt(dot(*this)); }
};

// Eigen::MatrixXd stand-in, row-major
struct MatXX {
    int r = 0, c = 0;
    std::vector<double> a;
    MatXX() = default;
    MatXX(int rows, int cols) : r(rows), c(cols), a((size_t)rows * cols, 0.0) {}
    static MatXX Zero(int rows, int cols) { return MatXX(rows, cols); }
    int rows() const { return r; }
    int cols() const { return c; }
    double &operator()(int i, int j) { return a[(size_t)i * c + j]; }
    double operator()(int i, int j) const { return a[(size_t)i * c + j]; }
    double *data() { return a.data(); }
    const double *data() const { return a.data(); }
};

enum ResState { IN = 0, OOB, OUTLIER };  // Residuals.h:33
// Point::PointStatus (include/Point.h): the states EnergyFunctional reads through frame->features
// in makeIDX / marginalizePointsF / dropPointsF; here a field of the PointHessian itself
enum class PointStatus { ACTIVE = 0, OUTLIER, OUT, MARGINALIZED };

struct CalibHessian {
    int wG0 = 0, hG0 = 0;                             // level-0 image size (GlobalCalib wG[0], hG[0])
    double value[4] = {0, 0, 0, 0};                   // CalibHessian::value (value_scaled = SCALE_F/C * value)
    double value_zero[4] = {0, 0, 0, 0};              // CalibHessian::value_zero
    float value_scaledf[4] = {0, 0, 0, 0};            // fxl, fyl, cxl, cyl
    double value_minus_value_zero[4] = {0, 0, 0, 0};  // cDeltaF source (setDeltaF)
    double step[4] = {0, 0, 0, 0};                    // resubstituteF_MT: -x.head<CPARS>()
    // CalibHessian::setValue (CalibHessian.h): value, value_scaledf and value_minus_value_zero
    void setValue(const double v[4]) {
        const double sc[4] = {50.0, 50.0, 50.0, 50.0};  // SCALE_F, SCALE_F, SCALE_C, SCALE_C (Settings.h:28-35)
        for (int i = 0; i < 4; i++) {
            value[i] = v[i];
            value_scaledf[i] = (float)(sc[i] * v[i]);
            value_minus_value_zero[i] = value[i] - value_zero[i];
        }
    }
};

struct FrameHessian {
    int idx = 0;                       // position in the window (makeIDX)
    void *user = nullptr;              // the caller's back-pointer (e.g. the reference object), untouched
    int frameID = 0;                   // keyframe id: 0 carries getPrior()'s strong pose prior
    bool flaggedForMarginalization = false;
    double worldToCam_evalPT[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};  // [R | t], row-major
    double state[10] = {0};            // FrameHessian::state (xi, a, b, ...)
    double state_zero[10] = {0};       // FrameHessian::state_zero
    double step[10] = {0};             // resubstituteF_MT: -x.segment<8>(CPARS + 8 idx)
    double ab_exposure = 1;
    const float *dI = nullptr;         // level-0 [I, dx, dy] per pixel (FrameHessian::dI)
    float frameEnergyTH = 8 * 8 * 8;   // written back for the newest frame by linearizeAll
    double prior[8] = {0}, delta[8] = {0}, delta_prior[8] = {0};  // takeData / setDeltaF
    // FrameHessian::takeData (FrameHessian.cc:131-135): prior, delta, delta_prior; the prior
    // (getPrior, FrameHessian.h:142-170) follows settings' affine modes (NULL: the defaults).  The
    // EnergyFunctional calls it with its own settings (setSettings).
    void takeData(const ldso_ba_opt_settings *settings = nullptr);
};

class EnergyFunctional;
struct PointFrameResidual;

struct PointHessian {
    weak_ptr<FrameHessian> host;
    float u = 0, v = 0;
    float idepth = 0, idepth_zero = 0, idepth_scaled = 0, idepth_zero_scaled = 0;
    float color[8] = {0}, weights[8] = {0};
    float priorF = 0, deltaF = 0;
    std::vector<shared_ptr<PointFrameResidual>> residuals;
    // written back by linearizeAll / resubstituteF_MT
    float HdiF = 0, bdSumF = 0, idepth_hessian = 0, step = 0;
    PointStatus status = PointStatus::ACTIVE;
    bool alreadyRemoved = false;
    int idxInPoints = -1;
    // the point's index in its host Frame's features vector (set by the caller at insert): the
    // library keeps each host's points in this order, the order doStepFromBackup sums sumNID in
    // (FullSystem.cc:1899-1909).  -1 on any point: each host's points in insertion order.
    int featureRank = -1;
    void *user = nullptr;  // the caller's back-pointer (e.g. the reference object), untouched
    // PointHessian::setIdepth / setIdepthZero (PointHessian.h)
    void setIdepth(float x) {
        idepth = x;
        idepth_scaled = SCALE_IDEPTH * x;
    }
    void setIdepthZero(float x) {
        idepth_zero = x;
        idepth_zero_scaled = SCALE_IDEPTH * x;
    }
};

struct PointFrameResidual {
    PointFrameResidual() = default;
    PointFrameResidual(shared_ptr<PointHessian> point_, shared_ptr<FrameHessian> host_,
                       shared_ptr<FrameHessian> target_)
        : point(point_), host(host_), target(target_) {
        resetOOB();
    }

    // Residuals.cc:15-217: this residual's own linearisation.  The device relinearises the
    // EnergyFunctional's whole window in ONE pass (ldso_ba_linearize_residuals) the first time a
    // residual asks after the window changed, and every later call until the next change reads
    // its entry: FullSystem::flagPointsForRemoval's per-residual loop (FullSystem.cc:1390-1398)
    // costs one device pass, not one per residual.  Sets state_NewState, state_NewEnergy,
    // state_NewEnergyWithOutlier, centerProjectedTo and the Jacobian applyRes(true) takes; like the
    // reference it changes neither state_state nor the frame thresholds.
    double linearize(shared_ptr<CalibHessian> &HCalib);
    void resetOOB();                       // Residuals.h:63-68
    void applyRes(bool copyJacobians);     // Residuals.h:70-88 (takeData: JpJdF = J_JpJdF)
    void setState(ResState s);
    bool isActive() const { return isActiveAndIsGoodNEW; }
    // Residuals.cc:219-245: marks the residual linearised; its res_toZeroF is formed on the
    // device by marginalizePointsF (ldso_ba_marginalize_points), the only consumer.
    void fixLinearizationF(shared_ptr<EnergyFunctional> ef);

    ResState state_state = OUTLIER;
    double state_energy = 0;
    ResState state_NewState = OUTLIER;
    double state_NewEnergy = 0;
    double state_NewEnergyWithOutlier = 0;
    weak_ptr<PointHessian> point;
    weak_ptr<FrameHessian> host;
    weak_ptr<FrameHessian> target;
    bool isNew = true;
    float centerProjectedTo[3] = {0, 0, 0};
    float relBS = 0;                  // linearizeAll_Reductor's maxRelBaseline term (fix pass)
    int hostIDX = 0, targetIDX = 0;
    float JpJdF[8] = {0};
    // takeData's JpJdF of this residual's last linearisation: what the reference derives from
    // its RawResidualJacobian J (Residuals.h:120-129); applyRes(true) copies it into JpJdF
    float J_JpJdF[8] = {0};
    bool isLinearized = false;
    bool isActiveAndIsGoodNEW = false;
    EnergyFunctional *ef = nullptr;   // set by EnergyFunctional::insertResidual, cleared on removal
    void *user = nullptr;             // the caller's back-pointer (e.g. the reference object), untouched
    int mirrorIdx = -1;               // position in the EnergyFunctional's device mirror
};

class EnergyFunctional : public std::enable_shared_from_this<EnergyFunctional> {
public:
    explicit EnergyFunctional(int device = 0);
    ~EnergyFunctional();
    EnergyFunctional(const EnergyFunctional &) = delete;
    EnergyFunctional &operator=(const EnergyFunctional &) = delete;

    bool ok() const { return err_.empty(); }
    const std::string &lastError() const { return err_; }

    // The reference's settings globals this window runs with (src/Setting.cc: setting_solverMode,
    // setting_forceAceptStep, setting_min/thOptIterations, setting_affineOptModeA / B,
    // setting_vi_enable), copied in by the caller before the first pass and whenever a driver
    // changes them.  Checked by the library (ldso_ba_set_settings): an
    // unsupported value returns false with lastError() set and keeps the previous settings.
    // Every later entry point runs with them: linearizeAll / optimize (JabF zeroing, priors, solver
    // mode), solveSystemF (checked again on every call), takeData's affine priors.
    bool setSettings(const ldso_ba_opt_settings &s);
    const ldso_ba_opt_settings &settings() const { return settings_; }

    // ---- EnergyFunctional.h:55-186 -------------------------------------------------------
    void insertResidual(shared_ptr<PointFrameResidual> r);
    void insertFrame(shared_ptr<FrameHessian> fh, shared_ptr<CalibHessian> Hcalib);
    void dropResidual(shared_ptr<PointFrameResidual> r);
    void marginalizeFrame(shared_ptr<FrameHessian> fh);
    void removePoint(shared_ptr<PointHessian> ph);
    // every allPoints entry with status MARGINALIZED: FullSystem::flagPointsForRemoval's
    // resetOOB / linearize / applyRes / fixLinearizationF of its residuals and the addPoint<2> +
    // SC addPoint(p, false) + stitch of marginalizePointsF, in one device call; then
    // HM += margWeightFac H, bM += margWeightFac b, removePoint, makeIDX
    void marginalizePointsF();
    void dropPointsF();  // removes the points with status OUTLIER or OUT
    // the non-VI branch (setting_vi_enable = false is the only setting setSettings accepts): the
    // reference's fourth argument, the InertialHessian, has no counterpart here and must be null
    void solveSystemF(int iteration, double lambda, shared_ptr<CalibHessian> HCalib);
    void solveSystemF(int iteration, double lambda, shared_ptr<CalibHessian> HCalib, std::nullptr_t /*HInertial*/) {
        solveSystemF(iteration, lambda, HCalib);
    }
    double calcMEnergyF();
    double calcLEnergyF_MT();
    void makeIDX();
    void setDeltaF(shared_ptr<CalibHessian> HCalib);
    void setAdjointsF(shared_ptr<CalibHessian> Hcalib);
    void resubstituteF_MT(const VecX &x, shared_ptr<CalibHessian> HCalib, bool MT = true);

    // ---- FullSystem-side passes served by the device ---------------------------------------
    // PointHessian activation (FullSystem::activatePointsMT adds it to its host's features,
    // which makeIDX then collects)
    void insertPoint(shared_ptr<PointHessian> ph);
    // PointFrameResidual::resetOOB for every active residual (FullSystem.cc:866-869)
    void resetOOB();
    // FullSystem::linearizeAll(fix) + applyRes + setNewFrameEnergyTH; with fix = false also the
    // accumulation of the stitched system for the following solveSystemF.  Returns (E, 0, #IN).
    Vec3 linearizeAll(bool fixLinearization);

    // FullSystem::optimize(mnumOptIts) (FullSystem.cc:844-970) with setting_forceAceptStep on the
    // device (ldso_ba_optimize): the iteration-count override for 2-3 frames (:846-851), resetOOB,
    // linearizeAll, then up to n_its x {solveSystemF (the pose / scale nullspaces of getNullspaces
    // from iteration 2), resubstituteF_MT, doStepFromBackup + setPrecalcValues, linearizeAll},
    // with no host round trip, leaving the loop on the reference's exits: canbreak once
    // iteration >= setting_minOptIterations (:968-969), or *isLost = true when the solution has a
    // NaN norm (:907-911; the reference then returns DBL_MAX).  Afterwards the frames' states,
    // HCalib's value and the points' idepth / idepth_zero hold the stepped values and setDeltaF
    // has run, as after the reference loop.  The residual fields (state_*, JpJdF,
    // centerProjectedTo) and the points' HdiF / bdSumF / idepth_hessian are written back lazily:
    // by the linearizeAll(true) FullSystem::optimize runs next, by syncResiduals(), or before any
    // PointFrameResidual method call.  energies (optional): (E, 0, #IN) of the first pass and of
    // every iteration's (after an exit: repeats of the last); iterations: the iterations entered;
    // settings: NULL = this window's settings (setSettings); otherwise they are installed first as
    // by setSettings (a rejected set fails the call).  Returns the last pass's energies.
    Vec3 optimize(int n_its, shared_ptr<CalibHessian> HCalib, std::vector<Vec3> *energies = nullptr,
                  bool *isLost = nullptr, int *iterations = nullptr, const ldso_ba_opt_settings *settings = nullptr);
    // the residual and point fields of the device's last pass, if the host copies are stale
    void syncResiduals();

    // FullSystem::linearizeAll(true)'s per-residual bookkeeping (FullSystem.cc:1771-1822), in compact
    // form, from the device arrays of the last linearizeAll(true): the residuals applyRes left
    // inactive (the reductor's toRemove, for ef->dropResidual), and per point (allPoints order) the
    // largest relBS of its active residuals and their number (p->maxRelBaseline / numGoodResiduals;
    // LDSO never clears isNew, so every active new residual contributes).  A forwarding shim applies
    // these instead of copying every field of every residual back into the reference's objects.
    // lastState[2q + i]: state_state of point q's residual to the newest (i = 0) / second-newest
    // (i = 1) keyframe, -1 without one -- p->lastResiduals[i].second (FullSystem.cc:1776-1782;
    // makeKeyFrame puts the residual to the new keyframe in lastResiduals[0] and shifts the
    // previous one to [1] for every point, FullSystem.cc:1247-1262)
    struct FixPassResult {
        std::vector<PointFrameResidual *> toRemove;
        std::vector<float> maxRelBS;
        std::vector<int> numGood;
        std::vector<int8_t> lastState;
    };
    const FixPassResult &fixPassResult() const { return fix_; }
    // the last pass's state_state / centerProjectedTo of residual mirrorIdx (PointFrameResidual::
    // mirrorIdx), for the consumers that read a few residuals after linearizeAll(true) --
    // lastResiduals' states (FullSystem.cc:1776-1782), CoarseTracker::makeCoarseDepthL0's
    // centerProjectedTo (CoarseTracker.cc:369-375) -- without a full write-back; downloaded once per
    // pass on first use
    ResState residualState(int mirrorIdx);
    const float *residualCenter(int mirrorIdx);
    // device linearisation passes run so far (linearizeAll, the per-residual relinearisation,
    // every pass of optimize): one per call site
    long devicePasses() const { return passes_; }

    // called by PointFrameResidual: make the host copy current before a residual method reads
    // it (device newer -> download), record a host-side edit (uploaded before the next pass),
    // and serve linearize() from the window's relinearisation pass
    void residualTouched() {
        if (resSync_ == ResSync::DeviceNewer) syncResiduals();
    }
    void residualEdited() { resSync_ = ResSync::HostNewer; }
    double linearizeResidual(PointFrameResidual &r);

    std::vector<shared_ptr<FrameHessian>> frames;
    int nPoints = 0, nFrames = 0, nResiduals = 0;
    MatXX HM = MatXX::Zero(CPARS, CPARS);  // marginalisation prior H
    VecX bM = VecX::Zero(CPARS);           // marginalisation prior b
    int resInA = 0, resInL = 0, resInM = 0;
    VecX lastX;
    std::vector<VecX> lastNullspaces_forLogging, lastNullspaces_pose, lastNullspaces_scale, lastNullspaces_affA,
        lastNullspaces_affB;
    // (host frameID << 32) + target frameID -> {active residuals, marginalised residuals}
    std::map<uint64_t, std::array<int, 2>> connectivityMap;
    std::vector<shared_ptr<PointHessian>> allPoints;
    std::vector<shared_ptr<PointHessian>> allPointsToMarg;
    // setDeltaF / setAdjointsF results (adHTdeltaF [N*N][8] float, index h + N t)
    std::vector<float> adHTdeltaF;
    float cDeltaF[4] = {0, 0, 0, 0};
    std::vector<double> adHost, adTarget;  // [N*N][64]
    double cPrior[4] = {0, 0, 0, 0};
    // the stitched blocks of the last solveSystemF (row-major (8N+4)^2 / (8N+4))
    MatXX HA_top, HL_top, H_sc;
    VecX bA_top, bL_top, b_sc;

    ldso_ba_ctx *context() { return ctx_; }

private:
    enum class ResSync { Synced, HostNewer, DeviceNewer };
    bool upload();
    bool uploadFrameTerms();
    bool runRelinearization();
    bool readBack(bool points_and_th);
    bool readPassSummary(bool fix);
    void fail(const char *what);
    void packFrames(std::vector<ldso_ba_frame_state> &fs) const;
    ldso_ba_ctx *ctx_ = nullptr;
    ldso_ba_ctx *margCtx_ = nullptr;
    std::vector<shared_ptr<PointHessian>> registry_;  // every inserted point not yet removed
    int device_ = 0;
    double currentLambda_ = 0;  // EnergyFunctional::currentLambda (set by solveSystemF)
    ldso_ba_opt_settings settings_ = LDSO_BA_OPT_SETTINGS_INIT;
    CalibHessian calib_;
    bool dirty_ = true;
    std::string err_;
    // SoA mirror (ldso_ba_window) of the loaded window
    std::vector<ldso_ba_frame_state> fs_;
    std::vector<float> dI_, frameTH_, precalc_, pointData_, resEnergy_;
    std::vector<double> adH_, adT_, cPrior_, fPrior_, fDelta_, fDeltaPrior_;
    std::vector<int32_t> pointHost_, resBegin_, resTarget_, pointRank_;
    bool pointRanked_ = false;
    std::vector<int8_t> resState_;
    std::vector<uint8_t> resFlags_;
    std::vector<PointFrameResidual *> resPtr_;
    std::vector<PointHessian *> ptPtr_, resPoint_;
    std::vector<float> pointVals_;  // [P][4] uploaded (idepth_scaled, idepth_zero_scaled, priorF, deltaF)
    std::vector<ldso_ba_frame_state> fsUp_;  // frame states / calibration / thresholds last uploaded
    float calibUp_[4] = {0, 0, 0, 0};
    float cDeltaUp_[4] = {0, 0, 0, 0};  // cDeltaF as last uploaded (it feeds the bL prior)
    std::vector<float> thUp_;
    int width_ = 0, height_ = 0;
    ResSync resSync_ = ResSync::Synced;
    long passes_ = 0;
    // the per-residual relinearisation (linearizeResidual): valid while epoch_ is unchanged and
    // the residual's point still has the snapshot's coordinates and inverse depths
    uint64_t epoch_ = 1, cacheEpoch_ = 0;
    // the last pass's compact outputs (readPassSummary) and their lazily downloaded companions
    FixPassResult fix_;
    std::vector<int8_t> outState_;
    std::vector<float> outCenter_;
    long outStatePass_ = -1, outCenterPass_ = -1;
    std::vector<int8_t> cNewState_;
    std::vector<uint8_t> cCenterOk_;
    std::vector<float> cNewEnergy_, cEwo_, cCenter_, cJp_, cSnap_;
};

}  // namespace ldso_amd

#endif  // LDSO_AMD_ENERGY_FUNCTIONAL_H_
