/*
 * energy_functional.h -- C++ host face of the MI355X bundle-adjustment hot path.
 *
 * Mirrors the class surface LDSO's FullSystem drives once per Gauss-Newton iteration (names,
 * fields and call order of the reference; paths relative to n-lalanne/LDSO):
 *
 *   FrameHessian         include/internal/FrameHessian.h      (state, state_zero, dI, frameEnergyTH)
 *   PointHessian         include/internal/PointHessian.h      (u, v, idepth, color, weights, residuals)
 *   PointFrameResidual   include/internal/Residuals.h:42-131   (state_*, centerProjectedTo, JpJdF)
 *   CalibHessian         include/internal/CalibHessian.h       (value_scaledf)
 *   EnergyFunctional     include/internal/OptimizationBackend/EnergyFunctional.h:55-149
 *                        insertFrame / insertPoint / insertResidual / dropResidual / removePoint /
 *                        makeIDX / solveSystemF / resubstituteF_MT / lastX
 *   + linearizeAll(fix)  FullSystem::linearizeAll (FullSystem.cc:1716-1769) with applyRes and
 *                        setNewFrameEnergyTH, and the accumulate{AF,LF,SCF} of the next solve
 *
 * Every call goes through the C ABI of include/ldso_ba.h into the HIP kernels; nothing here
 * computes on the CPU except packing.  Objects are owned by the caller (the reference holds
 * them in shared_ptr; here raw pointers that must outlive their EnergyFunctional membership).
 * Like the reference, nothing throws: failures leave ok() false and lastError() set.
 */
#ifndef LDSO_AMD_ENERGY_FUNCTIONAL_H_
#define LDSO_AMD_ENERGY_FUNCTIONAL_H_

#include <array>
#include <string>
#include <vector>

#include "../ldso_ba.h"

namespace ldso_amd {

using Vec3 = std::array<double, 3>;

enum ResState { IN = 0, OOB = 1, OUTLIER = 2 };  // Residuals.h:33

struct CalibHessian {
    int wG0 = 0, hG0 = 0;                            // level-0 image size (GlobalCalib wG[0], hG[0])
    float value_scaledf[4] = {0, 0, 0, 0};           // fxl, fyl, cxl, cyl
    float value_minus_value_zero[4] = {0, 0, 0, 0};  // cDeltaF source (EnergyFunctional::setDeltaF)
};

struct FrameHessian {
    int idx = -1;                      // position in the window (EnergyFunctional::makeIDX)
    double worldToCam_evalPT[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};  // [R | t], row-major
    double state[10] = {0};            // FrameHessian::state (xi, a, b, ...)
    double state_zero[10] = {0};       // FrameHessian::state_zero
    double ab_exposure = 1;
    bool isFirstFrame = false;         // frame->id == 0: the strong priors of getPrior()
    const float *dI = nullptr;         // level-0 [I, dx, dy] per pixel (FrameHessian::dI)
    float frameEnergyTH = 8 * 8 * 8;   // FrameHessian::frameEnergyTH (written back for the newest frame)
};

struct PointFrameResidual;

struct PointHessian {
    FrameHessian *host = nullptr;
    float u = 0, v = 0;
    float idepth_scaled = 0, idepth_zero_scaled = 0;
    float color[8] = {0}, weights[8] = {0};
    float priorF = 0, deltaF = 0;
    std::vector<PointFrameResidual *> residuals;
    // written back by linearizeAll / resubstituteF_MT
    float HdiF = 0, bdSumF = 0, idepth_hessian = 0, step = 0;
    int idxInPoints = -1;
};

struct PointFrameResidual {
    PointHessian *point = nullptr;
    FrameHessian *host = nullptr, *target = nullptr;
    ResState state_state = IN, state_NewState = OUTLIER;
    float state_energy = 0, state_NewEnergy = 0, state_NewEnergyWithOutlier = 0;
    float centerProjectedTo[3] = {0, 0, 0};
    float relBS = 0;                  // linearizeAll_Reductor's maxRelBaseline term (fix pass)
    bool isNew = true;
    bool isActiveAndIsGoodNEW = false;
    float JpJdF[8] = {0};
};

class EnergyFunctional {
public:
    explicit EnergyFunctional(int device = 0);
    ~EnergyFunctional();
    EnergyFunctional(const EnergyFunctional &) = delete;
    EnergyFunctional &operator=(const EnergyFunctional &) = delete;

    bool ok() const { return err_.empty(); }
    const std::string &lastError() const { return err_; }

    // structure (EnergyFunctional.cc:45-108, 500-521); any change re-uploads the window
    void insertFrame(FrameHessian *fh, const CalibHessian &Hcalib);
    void insertPoint(PointHessian *ph);
    void insertResidual(PointFrameResidual *r);
    void dropResidual(PointFrameResidual *r);
    void removePoint(PointHessian *p);
    void makeIDX();
    void setCalib(const CalibHessian &Hcalib);

    // PointFrameResidual::resetOOB for every residual (FullSystem.cc:876-879)
    void resetOOB();
    // FullSystem::linearizeAll(fix) + applyRes + setNewFrameEnergyTH; with fix = false also the
    // accumulation of the stitched system for the following solveSystemF.  Returns (E, 0, #IN).
    Vec3 linearizeAll(bool fixLinearization);
    // EnergyFunctional::solveSystemF (non-VI, FIX_LAMBDA, ORTHOGONALIZE_X_LATER): fills lastX
    void solveSystemF(int iteration, double lambda);
    // EnergyFunctional::resubstituteF_MT: frame steps are -lastX, point steps go to p->step
    void resubstituteF_MT(const std::vector<double> &x, double lambda);

    int nFrames = 0, nPoints = 0, nResiduals = 0;
    std::vector<FrameHessian *> frames;
    std::vector<PointHessian *> allPoints;
    std::vector<double> lastX;
    // last stitched system (row-major (8N+4)^2 / (8N+4)), as accumulateAF/LF/SCF leave them
    std::vector<double> HA_top, bA_top, HL_top, bL_top, H_sc, b_sc;

    ldso_ba_ctx *context() { return ctx_; }

private:
    bool upload();
    void fail(const char *what);
    ldso_ba_ctx *ctx_ = nullptr;
    CalibHessian calib_;
    bool dirty_ = true;
    std::string err_;
    // SoA mirror (ldso_ba_window)
    std::vector<ldso_ba_frame_state> fs_;
    std::vector<float> dI_, frameTH_, precalc_, pointData_, resEnergy_, cDelta_;
    std::vector<double> adH_, adT_, cPrior_, fPrior_, fDelta_, fDeltaPrior_;
    std::vector<int32_t> pointHost_, resBegin_, resTarget_;
    std::vector<int8_t> resState_;
    std::vector<uint8_t> resFlags_;
    std::vector<PointFrameResidual *> resPtr_;
    int width_ = 0, height_ = 0;
};

}  // namespace ldso_amd

#endif  // LDSO_AMD_ENERGY_FUNCTIONAL_H_
