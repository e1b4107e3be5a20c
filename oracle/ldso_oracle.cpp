// ldso_oracle.cpp -- CPU restatement of LDSO's sliding-window photometric BA hot path.
//
// TEST INFRASTRUCTURE ONLY (see ldso_oracle.h).  "Parity unpinned" by the reference: the
// reference has no golden vectors for this path and is unbuildable here; this restatement is
// pinned by the independent KATs in tests/test_oracle_kat.py.
//
// Each function cites the n-lalanne/LDSO file:line it restates.  Eigen fixed-size expressions
// are written out in Eigen's evaluation order (coefficient-wise, left to right); the file is
// compiled with -ffp-contract=off so every statement rounds as written.
#include "ldso_oracle.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace {

// ---- constants: include/Settings.h:28-35, src/Setting.cc ----------------------------------
constexpr int patternNum = 8;
const int patternP[8][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0},
                            {0, 0},  {2, 0},   {-1, 1}, {0, 2}};  // Setting.cc:275 (pattern 8)
constexpr int CPARS = 4;
constexpr float SCALE_IDEPTH = 1.0f;
constexpr float SCALE_XI_ROT = 1.0f;
constexpr float SCALE_XI_TRANS = 0.5f;
constexpr float SCALE_F = 50.0f;
constexpr float SCALE_C = 50.0f;
constexpr float SCALE_A = 10.0f;
constexpr float SCALE_B = 1000.0f;
constexpr float SCALE_XI_ROT_INVERSE = 1.0f / SCALE_XI_ROT;
constexpr float SCALE_XI_TRANS_INVERSE = 1.0f / SCALE_XI_TRANS;
constexpr float SCALE_A_INVERSE = 1.0f / SCALE_A;
constexpr float SCALE_B_INVERSE = 1.0f / SCALE_B;
float setting_outlierTHSumComponent = 50 * 50;  // Setting.cc:41
float setting_huberTH = 9;                      // Setting.cc:76
float setting_affineOptModeA = 1e12;            // Setting.cc:65
float setting_affineOptModeB = 1e8;             // Setting.cc:66
float setting_frameEnergyTHN = 0.7f;            // Setting.cc:79
float setting_frameEnergyTHConstWeight = 0.5;   // Setting.cc:77
float setting_frameEnergyTHFacMedian = 1.5;     // Setting.cc:81
float setting_overallEnergyTHWeight = 1;        // Setting.cc:82
float setting_initialCalibHessian = 5e9;        // Setting.cc:22
float setting_initialRotPrior = 1e11;           // Setting.cc:18
float setting_initialTransPrior = 1e10;         // Setting.cc:19
float setting_initialAffBPrior = 1e14;          // Setting.cc:20
float setting_initialAffAPrior = 1e14;          // Setting.cc:21
double setting_solverModeDelta = 0.00001;       // Setting.cc:24
constexpr int NUM_THREADS_MAX = 64;

enum ResState { IN = 0, OOB = 1, OUTLIER = 2 };

// ---- IndexThreadReduce<Vec10> (include/internal/IndexThreadReduce.h:26-170) ---------------
struct Vec10 {
    double v[10];
};
class IndexThreadReduce {
public:
    explicit IndexThreadReduce(int n) : n_(n) {
        for (int i = 0; i < n_; i++) {
            isDone_[i] = false;
            gotOne_[i] = true;
            workers_.emplace_back(&IndexThreadReduce::workerLoop, this, i);
        }
    }
    ~IndexThreadReduce() {
        {
            std::unique_lock<std::mutex> l(ex_);
            running_ = false;
            todo_.notify_all();
        }
        for (auto &t : workers_) t.join();
    }
    // reduce(): IndexThreadReduce.h:56-96
    void reduce(std::function<void(int, int, Vec10 *, int)> fn, int first, int end, int stepSize) {
        std::memset(&stats, 0, sizeof(stats));
        if (stepSize == 0) stepSize = ((end - first) + n_ - 1) / n_;
        std::unique_lock<std::mutex> lock(ex_);
        fn_ = fn;
        next_ = first;
        max_ = end;
        step_ = stepSize;
        for (int i = 0; i < n_; i++) {
            isDone_[i] = false;
            gotOne_[i] = false;
        }
        todo_.notify_all();
        while (true) {
            done_.wait(lock);
            bool all = true;
            for (int i = 0; i < n_; i++) all = all && isDone_[i];
            if (all) break;
        }
        next_ = 0;
        max_ = 0;
    }
    int n() const { return n_; }
    Vec10 stats;

private:
    // workerLoop(): IndexThreadReduce.h:125-166
    void workerLoop(int idx) {
        std::unique_lock<std::mutex> lock(ex_);
        while (running_) {
            int todo = 0;
            bool got = false;
            if (next_ < max_) {
                todo = next_;
                next_ += step_;
                got = true;
            }
            if (got) {
                lock.unlock();
                Vec10 s;
                std::memset(&s, 0, sizeof(s));
                fn_(todo, std::min(todo + step_, max_), &s, idx);
                gotOne_[idx] = true;
                lock.lock();
                for (int k = 0; k < 10; k++) stats.v[k] += s.v[k];
            } else {
                if (!gotOne_[idx]) {
                    lock.unlock();
                    Vec10 s;
                    std::memset(&s, 0, sizeof(s));
                    fn_(0, 0, &s, idx);
                    gotOne_[idx] = true;
                    lock.lock();
                    for (int k = 0; k < 10; k++) stats.v[k] += s.v[k];
                }
                isDone_[idx] = true;
                done_.notify_all();
                todo_.wait(lock);
            }
        }
    }
    int n_;
    std::vector<std::thread> workers_;
    bool isDone_[NUM_THREADS_MAX];
    bool gotOne_[NUM_THREADS_MAX];
    std::mutex ex_;
    std::condition_variable todo_, done_;
    int next_ = 0, max_ = 0, step_ = 1;
    bool running_ = true;
    std::function<void(int, int, Vec10 *, int)> fn_;
};

int g_threads = 6;  // NUM_THREADS, Settings.h:11

// ---- accumulators (include/internal/OptimizationBackend/MatrixAccumulators.h) ------------
// AccumulatorXX<i,j>: MatrixAccumulators.h:20-66
template <int I, int J>
struct AccumulatorXX {
    float A[I * J], A1k[I * J], A1m[I * J];
    size_t num;
    float numIn1, numIn1k, numIn1m;
    void initialize() {
        std::memset(A, 0, sizeof(A));
        std::memset(A1k, 0, sizeof(A1k));
        std::memset(A1m, 0, sizeof(A1m));
        num = 0;
        numIn1 = numIn1k = numIn1m = 0;
    }
    void finish() {
        shiftUp(true);
        num = (size_t)(numIn1 + numIn1k + numIn1m);
    }
    void update(const float *L, const float *R, float w) {
        for (int i = 0; i < I; i++) {
            float wl = w * L[i];
            for (int j = 0; j < J; j++) A[i * J + j] += wl * R[j];
        }
        numIn1++;
        shiftUp(false);
    }
    void shiftUp(bool force) {
        if (numIn1 > 1000 || force) {
            for (int k = 0; k < I * J; k++) A1k[k] += A[k];
            std::memset(A, 0, sizeof(A));
            numIn1k += numIn1;
            numIn1 = 0;
        }
        if (numIn1k > 1000 || force) {
            for (int k = 0; k < I * J; k++) A1m[k] += A1k[k];
            std::memset(A1k, 0, sizeof(A1k));
            numIn1m += numIn1k;
            numIn1k = 0;
        }
    }
};

// AccumulatorX<i>: MatrixAccumulators.h:145-197
template <int I>
struct AccumulatorX {
    float A[I], A1k[I], A1m[I];
    size_t num;
    float numIn1, numIn1k, numIn1m;
    void initialize() {
        std::memset(A, 0, sizeof(A));
        std::memset(A1k, 0, sizeof(A1k));
        std::memset(A1m, 0, sizeof(A1m));
        num = 0;
        numIn1 = numIn1k = numIn1m = 0;
    }
    void finish() {
        shiftUp(true);
        num = (size_t)(numIn1 + numIn1k + numIn1m);
    }
    void update(const float *L, float w) {
        for (int i = 0; i < I; i++) A[i] += w * L[i];
        numIn1++;
        shiftUp(false);
    }
    void shiftUp(bool force) {
        if (numIn1 > 1000 || force) {
            for (int k = 0; k < I; k++) A1k[k] += A[k];
            std::memset(A, 0, sizeof(A));
            numIn1k += numIn1;
            numIn1 = 0;
        }
        if (numIn1k > 1000 || force) {
            for (int k = 0; k < I; k++) A1m[k] += A1k[k];
            std::memset(A1k, 0, sizeof(A1k));
            numIn1m += numIn1k;
            numIn1k = 0;
        }
    }
};

// AccumulatorApprox: MatrixAccumulators.h:749-1101 (13x13: [0:4) C, [4:10) xi, 10 a, 11 b, 12 r)
struct AccumulatorApprox {
    double H[13][13];  // finish() output (stored as the float values, widened)
    size_t num;
    float Data[60], Data1k[60], Data1m[60];
    float TR[32], TR1k[32], TR1m[32];
    float BR[8], BR1k[8], BR1m[8];
    float numIn1, numIn1k, numIn1m;
    float Hf[13][13];
    void initialize() {
        std::memset(Data, 0, sizeof(Data));
        std::memset(Data1k, 0, sizeof(Data1k));
        std::memset(Data1m, 0, sizeof(Data1m));
        std::memset(TR, 0, sizeof(TR));
        std::memset(TR1k, 0, sizeof(TR1k));
        std::memset(TR1m, 0, sizeof(TR1m));
        std::memset(BR, 0, sizeof(BR));
        std::memset(BR1k, 0, sizeof(BR1k));
        std::memset(BR1m, 0, sizeof(BR1m));
        num = 0;
        numIn1 = numIn1k = numIn1m = 0;
    }
    // finish(): MatrixAccumulators.h:771-800
    void finish() {
        std::memset(Hf, 0, sizeof(Hf));
        shiftUp(true);
        int idx = 0;
        for (int r = 0; r < 10; r++)
            for (int c = r; c < 10; c++) {
                Hf[r][c] = Hf[c][r] = Data1m[idx];
                idx++;
            }
        idx = 0;
        for (int r = 0; r < 10; r++)
            for (int c = 0; c < 3; c++) {
                Hf[r][c + 10] = Hf[c + 10][r] = TR1m[idx];
                idx++;
            }
        Hf[10][10] = BR1m[0];
        Hf[10][11] = Hf[11][10] = BR1m[1];
        Hf[10][12] = Hf[12][10] = BR1m[2];
        Hf[11][11] = BR1m[3];
        Hf[11][12] = Hf[12][11] = BR1m[4];
        Hf[12][12] = BR1m[5];
        num = (size_t)(numIn1 + numIn1k + numIn1m);
    }
    // update(x4,x6,y4,y6,a,b,c): MatrixAccumulators.h:893-979.  x = [x4, x6], y = [y4, y6];
    // Data[idx(r,c)] += a*x[c]*x[r] + c*y[c]*y[r] + b*(x[c]*y[r] + y[c]*x[r]), c >= r.
    void update(const float *x4, const float *x6, const float *y4, const float *y6, float a,
                float b, float c) {
        float x[10], y[10];
        for (int i = 0; i < 4; i++) {
            x[i] = x4[i];
            y[i] = y4[i];
        }
        for (int i = 0; i < 6; i++) {
            x[4 + i] = x6[i];
            y[4 + i] = y6[i];
        }
        int idx = 0;
        for (int r = 0; r < 10; r++)
            for (int cc = r; cc < 10; cc++) {
                Data[idx] += a * x[cc] * x[r] + c * y[cc] * y[r] + b * (x[cc] * y[r] + y[cc] * x[r]);
                idx++;
            }
        num++;
        numIn1++;
        shiftUp(false);
    }
    // updateTopRight: MatrixAccumulators.h:982-1030
    void updateTopRight(const float *x4, const float *x6, const float *y4, const float *y6,
                        float TR00, float TR10, float TR01, float TR11, float TR02, float TR12) {
        float x[10], y[10];
        for (int i = 0; i < 4; i++) {
            x[i] = x4[i];
            y[i] = y4[i];
        }
        for (int i = 0; i < 6; i++) {
            x[4 + i] = x6[i];
            y[4 + i] = y6[i];
        }
        for (int r = 0; r < 10; r++) {
            TR[r * 3 + 0] += x[r] * TR00 + y[r] * TR10;
            TR[r * 3 + 1] += x[r] * TR01 + y[r] * TR11;
            TR[r * 3 + 2] += x[r] * TR02 + y[r] * TR12;
        }
    }
    // updateBotRight: MatrixAccumulators.h:1032-1045
    void updateBotRight(float a00, float a01, float a02, float a11, float a12, float a22) {
        BR[0] += a00;
        BR[1] += a01;
        BR[2] += a02;
        BR[3] += a11;
        BR[4] += a12;
        BR[5] += a22;
    }
    // shiftUp: MatrixAccumulators.h:1065-1100
    void shiftUp(bool force) {
        if (numIn1 > 1000 || force) {
            for (int i = 0; i < 60; i++) Data1k[i] += Data[i];
            for (int i = 0; i < 32; i++) TR1k[i] += TR[i];
            for (int i = 0; i < 8; i++) BR1k[i] += BR[i];
            numIn1k += numIn1;
            numIn1 = 0;
            std::memset(Data, 0, sizeof(Data));
            std::memset(TR, 0, sizeof(TR));
            std::memset(BR, 0, sizeof(BR));
        }
        if (numIn1k > 1000 || force) {
            for (int i = 0; i < 60; i++) Data1m[i] += Data1k[i];
            for (int i = 0; i < 32; i++) TR1m[i] += TR1k[i];
            for (int i = 0; i < 8; i++) BR1m[i] += BR1k[i];
            numIn1m += numIn1k;
            numIn1k = 0;
            std::memset(Data1k, 0, sizeof(Data1k));
            std::memset(TR1k, 0, sizeof(TR1k));
            std::memset(BR1k, 0, sizeof(BR1k));
        }
    }
};

// ---- state containers ----------------------------------------------------------------
// RawResidualJacobian: include/internal/RawResidualJacobian.h:13-39
struct RawResidualJacobian {
    float resF[8];
    float Jpdxi[2][6];
    float Jpdc[2][4];
    float Jpdd[2];
    float JIdx[2][8];
    float JabF[2][8];
    float JIdx2[2][2];
    float JabJIdx[2][2];
    float Jab2[2][2];
};

// PointFrameResidual: include/internal/Residuals.h:42-131
struct Residual {
    int state_state = OUTLIER;
    double state_energy = 0;
    int state_NewState = OUTLIER;
    double state_NewEnergy = 0;
    double state_NewEnergyWithOutlier = 0;
    int point = 0, hostIDX = 0, targetIDX = 0;
    RawResidualJacobian J;
    bool isNew = true;
    float projectedTo[8][2];
    float centerProjectedTo[3] = {0, 0, 0};
    float res_toZeroF[8];
    float JpJdF[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    bool isLinearized = false;
    bool isActiveAndIsGoodNEW = false;
    float relBS = 0;
    // Residuals.h:120-129
    void takeData() {
        float JI_JI_Jd[2];
        JI_JI_Jd[0] = J.JIdx2[0][0] * J.Jpdd[0] + J.JIdx2[0][1] * J.Jpdd[1];
        JI_JI_Jd[1] = J.JIdx2[1][0] * J.Jpdd[0] + J.JIdx2[1][1] * J.Jpdd[1];
        for (int i = 0; i < 6; i++) JpJdF[i] = J.Jpdxi[0][i] * JI_JI_Jd[0] + J.Jpdxi[1][i] * JI_JI_Jd[1];
        JpJdF[6] = J.JabJIdx[0][0] * J.Jpdd[0] + J.JabJIdx[0][1] * J.Jpdd[1];
        JpJdF[7] = J.JabJIdx[1][0] * J.Jpdd[0] + J.JabJIdx[1][1] * J.Jpdd[1];
    }
    // Residuals.h:63-67
    void resetOOB() {
        state_NewEnergy = state_energy = 0;
        state_NewState = OUTLIER;
        state_state = IN;
    }
    // Residuals.h:70-88
    void applyRes(bool copyJacobians) {
        if (copyJacobians) {
            if (state_state == OOB) return;
            if (state_NewState == IN) {
                isActiveAndIsGoodNEW = true;
                takeData();
            } else {
                isActiveAndIsGoodNEW = false;
            }
        }
        state_state = state_NewState;
        state_energy = state_NewEnergy;
    }
    bool isActive() const { return isActiveAndIsGoodNEW; }
};

// PointHessian: include/internal/PointHessian.h:83-131
struct PointH {
    float u = 0, v = 0, idepth_scaled = 0, idepth_zero_scaled = 0, priorF = 0, deltaF = 0;
    float color[8], weights[8];
    int host = 0;
    std::vector<int> residuals;
    float bdSumF = 0, HdiF = 0, Hdd_accLF = 0, Hcd_accLF[4] = {0, 0, 0, 0}, bd_accLF = 0;
    float Hdd_accAF = 0, Hcd_accAF[4] = {0, 0, 0, 0}, bd_accAF = 0;
    float idepth_hessian = 0, maxRelBaseline = 0, step = 0;
    int numGoodResiduals = 0;
};

struct FrameH {
    float frameEnergyTH = 8 * 8 * patternNum;
    double prior[8], delta_prior[8];
};

}  // namespace

struct oracle_window {
    int N = 0, w = 0, h = 0;
    float calib[4];
    float wM3G = 0, hM3G = 0;
    std::vector<float> dI;
    std::vector<float> precalc;
    std::vector<double> adHost, adTarget;
    std::vector<float> adHostF, adTargetF;
    double cPrior[4];
    float cDeltaF[4];
    std::vector<FrameH> frames;
    std::vector<PointH> points;
    std::vector<Residual> res;
    float currentLambda = 0;
    // accumulators: AccumulatedTopHessian.h:107-109, AccumulatedSCHessian.h:100-105
    std::vector<std::vector<AccumulatorApprox>> accTop;
    std::vector<int> nres;
    std::vector<std::vector<AccumulatorXX<8, 4>>> accE;
    std::vector<std::vector<AccumulatorX<8>>> accEB;
    std::vector<std::vector<AccumulatorXX<8, 8>>> accD;
    std::vector<AccumulatorXX<4, 4>> accHcc;
    std::vector<AccumulatorX<4>> accbc;
    IndexThreadReduce *red = nullptr;
    ~oracle_window() { delete red; }
    float fxl() const { return calib[0]; }
    float fyl() const { return calib[1]; }
    float cxl() const { return calib[2]; }
    float cyl() const { return calib[3]; }
    float fxli() const { return 1.0f / calib[0]; }  // CalibHessian::setValueScaled
    float fyli() const { return 1.0f / calib[1]; }
};

namespace {

void load_update(oracle_window *ow, const ldso_ba_window *w, bool structure) {
    const int N = w->n_frames;
    if (structure) {
        ow->N = N;
        ow->w = w->width;
        ow->h = w->height;
        ow->wM3G = (float)(w->width - 3);  // GlobalCalib.cc:40-41
        ow->hM3G = (float)(w->height - 3);
        ow->dI.assign(w->dI, w->dI + (size_t)N * w->width * w->height * 3);
        ow->frames.assign(N, FrameH());
        ow->points.assign(w->n_points, PointH());
        ow->res.assign(w->n_residuals, Residual());
        for (int p = 0; p < w->n_points; p++) {
            PointH &ph = ow->points[p];
            ph.host = w->point_host[p];
            for (int k = w->point_res_begin[p]; k < w->point_res_begin[p + 1]; k++) {
                ph.residuals.push_back(k);
                Residual &r = ow->res[k];
                r.point = p;
                r.hostIDX = ph.host;
                r.targetIDX = w->res_target[k];
                r.state_state = w->res_state[k];
                r.state_energy = w->res_energy[k];
                r.isActiveAndIsGoodNEW = (w->res_flags[k] & LDSO_BA_FLAG_ACTIVE) != 0;
                r.isNew = (w->res_flags[k] & LDSO_BA_FLAG_NEW) != 0;
                std::memset(&r.J, 0, sizeof(r.J));
            }
        }
    }
    for (int i = 0; i < 4; i++) {
        ow->calib[i] = w->calib[i];
        ow->cPrior[i] = w->c_prior[i];
        ow->cDeltaF[i] = w->c_delta[i];
    }
    ow->precalc.assign(w->precalc, w->precalc + (size_t)N * N * LDSO_BA_PRECALC_STRIDE);
    ow->adHost.assign(w->ad_host, w->ad_host + (size_t)N * N * 64);
    ow->adTarget.assign(w->ad_target, w->ad_target + (size_t)N * N * 64);
    ow->adHostF.resize(ow->adHost.size());
    ow->adTargetF.resize(ow->adTarget.size());
    for (size_t i = 0; i < ow->adHost.size(); i++) {  // EnergyFunctional.cc:598-602
        ow->adHostF[i] = (float)ow->adHost[i];
        ow->adTargetF[i] = (float)ow->adTarget[i];
    }
    for (int f = 0; f < N; f++) {
        ow->frames[f].frameEnergyTH = w->frame_energy_th[f];
        for (int k = 0; k < 8; k++) {
            ow->frames[f].prior[k] = w->frame_prior[f * 8 + k];
            ow->frames[f].delta_prior[k] = w->frame_delta_prior[f * 8 + k];
        }
    }
    for (int p = 0; p < w->n_points; p++) {
        const float *d = w->point_data + (size_t)p * LDSO_BA_POINT_STRIDE;
        PointH &ph = ow->points[p];
        ph.u = d[0];
        ph.v = d[1];
        ph.idepth_scaled = d[2];
        ph.idepth_zero_scaled = d[3];
        ph.priorF = d[4];
        ph.deltaF = d[5];
        for (int i = 0; i < 8; i++) {
            ph.color[i] = d[8 + i];
            ph.weights[i] = d[16 + i];
        }
    }
}

// getInterpolatedElement33: include/internal/GlobalFuncs.h:89-103
inline void interp33(const float *mat, float x, float y, int width, float out[3]) {
    int ix = (int)x;
    int iy = (int)y;
    float dx = x - ix;
    float dy = y - iy;
    float dxdy = dx * dy;
    const float *bp = mat + 3 * ((size_t)ix + (size_t)iy * width);
    const float *p11 = bp + 3 * (1 + width), *p01 = bp + 3 * width, *p10 = bp + 3, *p00 = bp;
    float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
    for (int c = 0; c < 3; c++) out[c] = w11 * p11[c] + w01 * p01[c] + w10 * p10[c] + w00 * p00[c];
}

// PointFrameResidual::linearize: src/internal/Residuals.cc:15-217
double linearize(oracle_window *ow, Residual &r) {
    r.state_NewEnergyWithOutlier = -1;
    if (r.state_state == OOB) {
        r.state_NewState = OOB;
        return r.state_energy;
    }
    const int N = ow->N;
    const PointH &p = ow->points[r.point];
    const FrameH &fh = ow->frames[r.hostIDX];
    const FrameH &ft = ow->frames[r.targetIDX];
    const float *pre = ow->precalc.data() + (size_t)(r.hostIDX + N * r.targetIDX) * LDSO_BA_PRECALC_STRIDE;
    const float *KRKi = pre + 0;   // PRE_KRKiTll
    const float *Kt = pre + 9;     // PRE_KtTll
    const float *R0 = pre + 12;    // PRE_RTll_0
    const float *t0 = pre + 21;    // PRE_tTll_0
    const float affLL[2] = {pre[24], pre[25]};
    const float b0 = pre[26];
    const float *dIl = ow->dI.data() + (size_t)r.targetIDX * ow->w * ow->h * 3;
    float energyLeft = 0;
    const float *color = p.color, *weights = p.weights;
    RawResidualJacobian &J = r.J;

    float d_xi_x[6], d_xi_y[6], d_C_x[4], d_C_y[4], d_d_x, d_d_y;
    {
        // projectPoint (full): include/internal/ResidualProjections.h:57-84
        float KliP[3] = {(p.u + 0 - ow->cxl()) * ow->fxli(), (p.v + 0 - ow->cyl()) * ow->fyli(), 1};
        float ptp[3];
        for (int i = 0; i < 3; i++)
            ptp[i] = (R0[3 * i + 0] * KliP[0] + R0[3 * i + 1] * KliP[1] + R0[3 * i + 2] * KliP[2]) + t0[i] * p.idepth_zero_scaled;
        float drescale = 1.0f / ptp[2];
        float new_idepth = p.idepth_zero_scaled * drescale;
        if (!(drescale > 0)) {
            r.state_NewState = OOB;
            return r.state_energy;
        }
        float u = ptp[0] * drescale;
        float v = ptp[1] * drescale;
        float Ku = u * ow->fxl() + ow->cxl();
        float Kv = v * ow->fyl() + ow->cyl();
        if (!(Ku > 1.1f && Kv > 1.1f && Ku < ow->wM3G && Kv < ow->hM3G)) {
            r.state_NewState = OOB;
            return r.state_energy;
        }
        r.centerProjectedTo[0] = Ku;
        r.centerProjectedTo[1] = Kv;
        r.centerProjectedTo[2] = new_idepth;

        // Residuals.cc:69-106
        d_d_x = drescale * (t0[0] - t0[2] * u) * SCALE_IDEPTH * ow->fxl();
        d_d_y = drescale * (t0[1] - t0[2] * v) * SCALE_IDEPTH * ow->fyl();
        d_C_x[2] = drescale * (R0[6] * u - R0[0]);
        d_C_x[3] = ow->fxl() * drescale * (R0[7] * u - R0[1]) * ow->fyli();
        d_C_x[0] = KliP[0] * d_C_x[2];
        d_C_x[1] = KliP[1] * d_C_x[3];
        d_C_y[2] = ow->fyl() * drescale * (R0[6] * v - R0[3]) * ow->fxli();
        d_C_y[3] = drescale * (R0[7] * v - R0[4]);
        d_C_y[0] = KliP[0] * d_C_y[2];
        d_C_y[1] = KliP[1] * d_C_y[3];
        d_C_x[0] = (d_C_x[0] + u) * SCALE_F;
        d_C_x[1] *= SCALE_F;
        d_C_x[2] = (d_C_x[2] + 1) * SCALE_C;
        d_C_x[3] *= SCALE_C;
        d_C_y[0] *= SCALE_F;
        d_C_y[1] = (d_C_y[1] + v) * SCALE_F;
        d_C_y[2] *= SCALE_C;
        d_C_y[3] = (d_C_y[3] + 1) * SCALE_C;
        d_xi_x[0] = new_idepth * ow->fxl();
        d_xi_x[1] = 0;
        d_xi_x[2] = -new_idepth * u * ow->fxl();
        d_xi_x[3] = -u * v * ow->fxl();
        d_xi_x[4] = (1 + u * u) * ow->fxl();
        d_xi_x[5] = -v * ow->fxl();
        d_xi_y[0] = 0;
        d_xi_y[1] = new_idepth * ow->fyl();
        d_xi_y[2] = -new_idepth * v * ow->fyl();
        d_xi_y[3] = -(1 + v * v) * ow->fyl();
        d_xi_y[4] = u * v * ow->fyl();
        d_xi_y[5] = u * ow->fyl();
    }
    // Residuals.cc:109-120
    for (int i = 0; i < 6; i++) {
        J.Jpdxi[0][i] = d_xi_x[i];
        J.Jpdxi[1][i] = d_xi_y[i];
    }
    for (int i = 0; i < 4; i++) {
        J.Jpdc[0][i] = d_C_x[i];
        J.Jpdc[1][i] = d_C_y[i];
    }
    J.Jpdd[0] = d_d_x;
    J.Jpdd[1] = d_d_y;

    float JIdxJIdx_00 = 0, JIdxJIdx_11 = 0, JIdxJIdx_10 = 0;
    float JabJIdx_00 = 0, JabJIdx_01 = 0, JabJIdx_10 = 0, JabJIdx_11 = 0;
    float JabJab_00 = 0, JabJab_01 = 0, JabJab_11 = 0;
    float wJI2_sum = 0;

    // Residuals.cc:128-190
    for (int idx = 0; idx < patternNum; idx++) {
        // projectPoint (simple): ResidualProjections.h:24-33
        float upt = p.u + patternP[idx][0], vpt = p.v + patternP[idx][1];
        float ptp[3];
        for (int i = 0; i < 3; i++)
            ptp[i] = (KRKi[3 * i + 0] * upt + KRKi[3 * i + 1] * vpt + KRKi[3 * i + 2] * 1.0f) + Kt[i] * p.idepth_scaled;
        float Ku = ptp[0] / ptp[2];
        float Kv = ptp[1] / ptp[2];
        if (!(Ku > 1.1f && Kv > 1.1f && Ku < ow->wM3G && Kv < ow->hM3G)) {
            r.state_NewState = OOB;
            return r.state_energy;
        }
        r.projectedTo[idx][0] = Ku;
        r.projectedTo[idx][1] = Kv;

        float hitColor[3];
        interp33(dIl, Ku, Kv, ow->w, hitColor);
        float residual = hitColor[0] - (float)(affLL[0] * color[idx] + affLL[1]);
        float drdA = (color[idx] - b0);
        if (!std::isfinite((float)hitColor[0])) {
            r.state_NewState = OOB;
            return r.state_energy;
        }
        float w = sqrtf(setting_outlierTHSumComponent /
                        (setting_outlierTHSumComponent + (hitColor[1] * hitColor[1] + hitColor[2] * hitColor[2])));
        w = 0.5f * (w + weights[idx]);
        float hw = fabsf(residual) < setting_huberTH ? 1 : setting_huberTH / fabsf(residual);
        energyLeft += w * w * hw * residual * residual * (2 - hw);
        {
            if (hw < 1) hw = sqrtf(hw);
            hw = hw * w;
            hitColor[1] *= hw;
            hitColor[2] *= hw;
            J.resF[idx] = residual * hw;
            J.JIdx[0][idx] = hitColor[1];
            J.JIdx[1][idx] = hitColor[2];
            J.JabF[0][idx] = drdA * hw;
            J.JabF[1][idx] = hw;
            JIdxJIdx_00 += hitColor[1] * hitColor[1];
            JIdxJIdx_11 += hitColor[2] * hitColor[2];
            JIdxJIdx_10 += hitColor[1] * hitColor[2];
            JabJIdx_00 += drdA * hw * hitColor[1];
            JabJIdx_01 += drdA * hw * hitColor[2];
            JabJIdx_10 += hw * hitColor[1];
            JabJIdx_11 += hw * hitColor[2];
            JabJab_00 += drdA * drdA * hw * hw;
            JabJab_01 += drdA * hw * hw;
            JabJab_11 += hw * hw;
            wJI2_sum += hw * hw * (hitColor[1] * hitColor[1] + hitColor[2] * hitColor[2]);
            if (setting_affineOptModeA < 0) J.JabF[0][idx] = 0;
            if (setting_affineOptModeB < 0) J.JabF[1][idx] = 0;
        }
    }
    // Residuals.cc:192-216
    J.JIdx2[0][0] = JIdxJIdx_00;
    J.JIdx2[0][1] = JIdxJIdx_10;
    J.JIdx2[1][0] = JIdxJIdx_10;
    J.JIdx2[1][1] = JIdxJIdx_11;
    J.JabJIdx[0][0] = JabJIdx_00;
    J.JabJIdx[0][1] = JabJIdx_01;
    J.JabJIdx[1][0] = JabJIdx_10;
    J.JabJIdx[1][1] = JabJIdx_11;
    J.Jab2[0][0] = JabJab_00;
    J.Jab2[0][1] = JabJab_01;
    J.Jab2[1][0] = JabJab_01;
    J.Jab2[1][1] = JabJab_11;
    r.state_NewEnergyWithOutlier = energyLeft;
    float th = std::max<float>(fh.frameEnergyTH, ft.frameEnergyTH);
    if (energyLeft > th || wJI2_sum < 2) {
        energyLeft = th;
        r.state_NewState = OUTLIER;
    } else {
        r.state_NewState = IN;
    }
    r.state_NewEnergy = energyLeft;
    return energyLeft;
}

// FullSystem::setNewFrameEnergyTH: src/frontend/FullSystem.cc:2078-2109
void setNewFrameEnergyTH(oracle_window *ow) {
    std::vector<float> all;
    const int newest = ow->N - 1;
    for (auto &r : ow->res)
        if (r.state_NewEnergyWithOutlier >= 0 && r.targetIDX == newest)
            all.push_back((float)r.state_NewEnergyWithOutlier);
    FrameH &nf = ow->frames[newest];
    if (all.empty()) {
        nf.frameEnergyTH = 12 * 12 * patternNum;
        return;
    }
    int nthIdx = setting_frameEnergyTHN * all.size();
    std::nth_element(all.begin(), all.begin() + nthIdx, all.end());
    float nthElement = sqrtf(all[nthIdx]);
    nf.frameEnergyTH = nthElement * setting_frameEnergyTHFacMedian;
    nf.frameEnergyTH = 26.0f * setting_frameEnergyTHConstWeight + nf.frameEnergyTH * (1 - setting_frameEnergyTHConstWeight);
    nf.frameEnergyTH = nf.frameEnergyTH * nf.frameEnergyTH;
    nf.frameEnergyTH *= setting_overallEnergyTHWeight * setting_overallEnergyTHWeight;
}

// FullSystem::linearizeAll_Reductor: src/frontend/FullSystem.cc:1771-1823
void linearizeAll_Reductor(oracle_window *ow, bool fix, int min, int max, Vec10 *stats) {
    for (int k = min; k < max; k++) {
        Residual &r = ow->res[k];
        stats->v[0] += linearize(ow, r);
        if (r.state_NewState == IN) stats->v[1] += 1;
        if (fix) {
            r.applyRes(true);
            if (r.isActive()) {
                if (r.isNew) {
                    const PointH &p = ow->points[r.point];
                    const float *pre = ow->precalc.data() + (size_t)(r.hostIDX + ow->N * r.targetIDX) * LDSO_BA_PRECALC_STRIDE;
                    float ptp_inf[3], ptp[3];
                    for (int i = 0; i < 3; i++) {
                        ptp_inf[i] = pre[3 * i + 0] * p.u + pre[3 * i + 1] * p.v + pre[3 * i + 2] * 1.0f;
                        ptp[i] = ptp_inf[i] + pre[9 + i] * p.idepth_scaled;
                    }
                    float dx = ptp_inf[0] / ptp_inf[2] - ptp[0] / ptp[2];
                    float dy = ptp_inf[1] / ptp_inf[2] - ptp[1] / ptp[2];
                    float relBS = 0.01f * sqrtf(dx * dx + dy * dy);
                    r.relBS = relBS;
                    PointH &pm = ow->points[r.point];
                    if (relBS > pm.maxRelBaseline) pm.maxRelBaseline = relBS;
                    pm.numGoodResiduals++;
                }
            }
        }
    }
}

// ---- Top accumulation (AccumulatedTopHessian.cc) --------------------------------------
// addPoint<mode>: AccumulatedTopHessian.cc:8-118
template <int mode>
void topAddPoint(oracle_window *ow, PointH &p, int tid) {
    const int N = ow->N;
    const float *dc = ow->cDeltaF;
    float dd = p.deltaF;
    float bd_acc = 0, Hdd_acc = 0, Hcd_acc[4] = {0, 0, 0, 0};
    for (int ri : p.residuals) {
        Residual &r = ow->res[ri];
        if (mode == 0) {
            if (r.isLinearized || !r.isActive()) continue;
        }
        if (mode == 1) {
            if (!r.isLinearized || !r.isActive()) continue;
        }
        if (mode == 2) {
            if (!r.isActive()) continue;
        }
        const RawResidualJacobian &rJ = r.J;
        int htIDX = r.hostIDX + r.targetIDX * N;
        float resApprox[8];
        if (mode == 0)
            for (int i = 0; i < 8; i++) resApprox[i] = rJ.resF[i];
        if (mode == 2)
            for (int i = 0; i < 8; i++) resApprox[i] = r.res_toZeroF[i];
        if (mode == 1) {
            // adHTdeltaF is only non-zero with linearized residuals (marginalisation path); the
            // hot path never has them (FullSystem.cc:854-875 gathers !isLinearized residuals).
            for (int i = 0; i < 8; i++) resApprox[i] = r.res_toZeroF[i];
            (void)dc;
            (void)dd;
        }
        float JI_r[2] = {0, 0}, Jab_r[2] = {0, 0}, rr = 0;
        for (int i = 0; i < patternNum; i++) {
            JI_r[0] += resApprox[i] * rJ.JIdx[0][i];
            JI_r[1] += resApprox[i] * rJ.JIdx[1][i];
            Jab_r[0] += resApprox[i] * rJ.JabF[0][i];
            Jab_r[1] += resApprox[i] * rJ.JabF[1][i];
            rr += resApprox[i] * resApprox[i];
        }
        AccumulatorApprox &acc = ow->accTop[tid][htIDX];
        acc.update(rJ.Jpdc[0], rJ.Jpdxi[0], rJ.Jpdc[1], rJ.Jpdxi[1], rJ.JIdx2[0][0], rJ.JIdx2[0][1], rJ.JIdx2[1][1]);
        acc.updateBotRight(rJ.Jab2[0][0], rJ.Jab2[0][1], Jab_r[0], rJ.Jab2[1][1], Jab_r[1], rr);
        acc.updateTopRight(rJ.Jpdc[0], rJ.Jpdxi[0], rJ.Jpdc[1], rJ.Jpdxi[1], rJ.JabJIdx[0][0],
                           rJ.JabJIdx[0][1], rJ.JabJIdx[1][0], rJ.JabJIdx[1][1], JI_r[0], JI_r[1]);
        float Ji2_Jpdd[2];
        Ji2_Jpdd[0] = rJ.JIdx2[0][0] * rJ.Jpdd[0] + rJ.JIdx2[0][1] * rJ.Jpdd[1];
        Ji2_Jpdd[1] = rJ.JIdx2[1][0] * rJ.Jpdd[0] + rJ.JIdx2[1][1] * rJ.Jpdd[1];
        bd_acc += JI_r[0] * rJ.Jpdd[0] + JI_r[1] * rJ.Jpdd[1];
        Hdd_acc += Ji2_Jpdd[0] * rJ.Jpdd[0] + Ji2_Jpdd[1] * rJ.Jpdd[1];
        for (int i = 0; i < 4; i++) Hcd_acc[i] += rJ.Jpdc[0][i] * Ji2_Jpdd[0] + rJ.Jpdc[1][i] * Ji2_Jpdd[1];
        ow->nres[tid]++;
    }
    if (mode == 0) {
        p.Hdd_accAF = Hdd_acc;
        p.bd_accAF = bd_acc;
        for (int i = 0; i < 4; i++) p.Hcd_accAF[i] = Hcd_acc[i];
    }
    if (mode == 1 || mode == 2) {
        p.Hdd_accLF = Hdd_acc;
        p.bd_accLF = bd_acc;
        for (int i = 0; i < 4; i++) p.Hcd_accLF[i] = Hcd_acc[i];
    }
    if (mode == 2) {
        for (int i = 0; i < 4; i++) p.Hcd_accAF[i] = 0;
        p.Hdd_accAF = 0;
        p.bd_accAF = 0;
    }
}

inline int dimH(int N) { return 8 * N + CPARS; }

// y(8x8) = A * B * C^T   (double)
void sandwich(const double *A, const double *B, const double *C, double *out) {
    double T[64];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            double s = 0;
            for (int k = 0; k < 8; k++) s += A[i * 8 + k] * B[k * 8 + j];
            T[i * 8 + j] = s;
        }
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            double s = 0;
            for (int k = 0; k < 8; k++) s += T[i * 8 + k] * C[j * 8 + k];
            out[i * 8 + j] = s;
        }
}

// AccumulatedTopHessianSSE::stitchDoubleInternal: AccumulatedTopHessian.cc:193-253
void topStitchInternal(oracle_window *ow, std::vector<double> &H, std::vector<double> &b,
                       bool usePrior, int min, int max, int tid) {
    int toAggregate = (int)ow->accTop.size();
    if (tid == -1) {
        toAggregate = 1;
        tid = 0;
    }
    if (min == max) return;
    const int N = ow->N, D = dimH(N);
    for (int k = min; k < max; k++) {
        int h = k % N, t = k / N;
        int hIdx = CPARS + h * 8, tIdx = CPARS + t * 8;
        int aidx = h + N * t;
        double accH[13][13];
        std::memset(accH, 0, sizeof(accH));
        for (int tid2 = 0; tid2 < toAggregate; tid2++) {
            AccumulatorApprox &a = ow->accTop[tid2][aidx];
            a.finish();
            if (a.num == 0) continue;
            for (int i = 0; i < 13; i++)
                for (int j = 0; j < 13; j++) accH[i][j] += (double)a.Hf[i][j];
        }
        double A88[64], A8C[32], A8r[8];
        for (int i = 0; i < 8; i++) {
            for (int j = 0; j < 8; j++) A88[i * 8 + j] = accH[CPARS + i][CPARS + j];
            for (int j = 0; j < 4; j++) A8C[i * 4 + j] = accH[CPARS + i][j];
            A8r[i] = accH[CPARS + i][CPARS + 8];
        }
        const double *AH = &ow->adHost[(size_t)aidx * 64], *AT = &ow->adTarget[(size_t)aidx * 64];
        double blk[64];
        sandwich(AH, A88, AH, blk);
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 8; j++) H[(size_t)(hIdx + i) * D + hIdx + j] += blk[i * 8 + j];
        sandwich(AT, A88, AT, blk);
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 8; j++) H[(size_t)(tIdx + i) * D + tIdx + j] += blk[i * 8 + j];
        sandwich(AH, A88, AT, blk);
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 8; j++) H[(size_t)(hIdx + i) * D + tIdx + j] += blk[i * 8 + j];
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 4; j++) {
                double sh = 0, st = 0;
                for (int k2 = 0; k2 < 8; k2++) {
                    sh += AH[i * 8 + k2] * A8C[k2 * 4 + j];
                    st += AT[i * 8 + k2] * A8C[k2 * 4 + j];
                }
                H[(size_t)(hIdx + i) * D + j] += sh;
                H[(size_t)(tIdx + i) * D + j] += st;
            }
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) H[(size_t)i * D + j] += accH[i][j];
        for (int i = 0; i < 8; i++) {
            double sh = 0, st = 0;
            for (int k2 = 0; k2 < 8; k2++) {
                sh += AH[i * 8 + k2] * A8r[k2];
                st += AT[i * 8 + k2] * A8r[k2];
            }
            b[hIdx + i] += sh;
            b[tIdx + i] += st;
        }
        for (int i = 0; i < 4; i++) b[i] += accH[i][CPARS + 8];
    }
    if (min == 0 && usePrior) {
        for (int i = 0; i < 4; i++) {
            H[(size_t)i * D + i] += ow->cPrior[i];
            b[i] += ow->cPrior[i] * (double)ow->cDeltaF[i];
        }
        for (int h = 0; h < N; h++)
            for (int i = 0; i < 8; i++) {
                int c = CPARS + h * 8 + i;
                H[(size_t)c * D + c] += ow->frames[h].prior[i];
                b[c] += ow->frames[h].prior[i] * ow->frames[h].delta_prior[i];
            }
    }
}

// AccumulatedTopHessianSSE::stitchDoubleMT: AccumulatedTopHessian.h:64-105
void topStitchMT(oracle_window *ow, std::vector<double> &H, std::vector<double> &b, bool usePrior,
                 bool MT) {
    const int N = ow->N, D = dimH(N);
    if (MT) {
        int nt = ow->red->n();
        std::vector<std::vector<double>> Hs(nt, std::vector<double>((size_t)D * D, 0.0));
        std::vector<std::vector<double>> bs(nt, std::vector<double>(D, 0.0));
        ow->red->reduce([&](int mn, int mx, Vec10 *, int tid) { topStitchInternal(ow, Hs[tid], bs[tid], usePrior, mn, mx, tid); },
                        0, N * N, 0);
        H = Hs[0];
        b = bs[0];
        for (int i = 1; i < nt; i++) {
            for (size_t k = 0; k < H.size(); k++) H[k] += Hs[i][k];
            for (int k = 0; k < D; k++) b[k] += bs[i][k];
            ow->nres[0] += ow->nres[i];
        }
    } else {
        H.assign((size_t)D * D, 0.0);
        b.assign(D, 0.0);
        topStitchInternal(ow, H, b, usePrior, 0, N * N, -1);
    }
    for (int h = 0; h < N; h++) {
        int hIdx = CPARS + h * 8;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 8; j++) H[(size_t)i * D + hIdx + j] = H[(size_t)(hIdx + j) * D + i];
        for (int t = h + 1; t < N; t++) {
            int tIdx = CPARS + t * 8;
            for (int i = 0; i < 8; i++)
                for (int j = 0; j < 8; j++) H[(size_t)(hIdx + i) * D + tIdx + j] += H[(size_t)(tIdx + j) * D + hIdx + i];
            for (int i = 0; i < 8; i++)
                for (int j = 0; j < 8; j++) H[(size_t)(tIdx + i) * D + hIdx + j] = H[(size_t)(hIdx + j) * D + tIdx + i];
        }
    }
}

// ---- Schur complement (AccumulatedSCHessian.cc) ---------------------------------------
// addPoint: AccumulatedSCHessian.cc:9-51
void scAddPoint(oracle_window *ow, PointH &p, bool shiftPriorToZero, int tid) {
    int ngoodres = 0;
    for (int ri : p.residuals)
        if (ow->res[ri].isActive()) ngoodres++;
    if (ngoodres == 0) {
        p.HdiF = 0;
        p.bdSumF = 0;
        p.idepth_hessian = 0;
        p.maxRelBaseline = 0;
        return;
    }
    float H = p.Hdd_accAF + p.Hdd_accLF + p.priorF;
    if (H < 1e-10) H = 1e-10;
    p.idepth_hessian = H;
    p.HdiF = 1.0 / H;
    p.bdSumF = p.bd_accAF + p.bd_accLF;
    if (shiftPriorToZero) p.bdSumF += p.priorF * p.deltaF;
    float Hcd[4];
    for (int i = 0; i < 4; i++) Hcd[i] = p.Hcd_accAF[i] + p.Hcd_accLF[i];
    ow->accHcc[tid].update(Hcd, Hcd, p.HdiF);
    ow->accbc[tid].update(Hcd, p.bdSumF * p.HdiF);
    const int N = ow->N, nFrames2 = N * N;
    for (int r1i : p.residuals) {
        Residual &r1 = ow->res[r1i];
        if (!r1.isActive()) continue;
        int r1ht = r1.hostIDX + r1.targetIDX * N;
        for (int r2i : p.residuals) {
            Residual &r2 = ow->res[r2i];
            if (!r2.isActive()) continue;
            ow->accD[tid][r1ht + r2.targetIDX * nFrames2].update(r1.JpJdF, r2.JpJdF, p.HdiF);
        }
        ow->accE[tid][r1ht].update(r1.JpJdF, Hcd, p.HdiF);
        ow->accEB[tid][r1ht].update(r1.JpJdF, p.HdiF * p.bdSumF);
    }
}

// stitchDoubleInternal: AccumulatedSCHessian.cc:53-119
void scStitchInternal(oracle_window *ow, std::vector<double> &H, std::vector<double> &b, int min,
                      int max, int tid) {
    int toAggregate = (int)ow->accE.size();
    if (tid == -1) {
        toAggregate = 1;
        tid = 0;
    }
    if (min == max) return;
    const int nf = ow->N, nframes2 = nf * nf, D = dimH(nf);
    for (int k = min; k < max; k++) {
        int i = k % nf, j = k / nf;
        int iIdx = CPARS + i * 8, jIdx = CPARS + j * 8;
        int ijIdx = i + nf * j;
        double Hpc[32], bp[8];
        std::memset(Hpc, 0, sizeof(Hpc));
        std::memset(bp, 0, sizeof(bp));
        for (int tid2 = 0; tid2 < toAggregate; tid2++) {
            ow->accE[tid2][ijIdx].finish();
            ow->accEB[tid2][ijIdx].finish();
            for (int q = 0; q < 32; q++) Hpc[q] += (double)ow->accE[tid2][ijIdx].A1m[q];
            for (int q = 0; q < 8; q++) bp[q] += (double)ow->accEB[tid2][ijIdx].A1m[q];
        }
        const double *AHij = &ow->adHost[(size_t)ijIdx * 64], *ATij = &ow->adTarget[(size_t)ijIdx * 64];
        for (int r = 0; r < 8; r++) {
            for (int c = 0; c < 4; c++) {
                double sh = 0, st = 0;
                for (int q = 0; q < 8; q++) {
                    sh += AHij[r * 8 + q] * Hpc[q * 4 + c];
                    st += ATij[r * 8 + q] * Hpc[q * 4 + c];
                }
                H[(size_t)(iIdx + r) * D + c] += sh;
                H[(size_t)(jIdx + r) * D + c] += st;
            }
            double sh = 0, st = 0;
            for (int q = 0; q < 8; q++) {
                sh += AHij[r * 8 + q] * bp[q];
                st += ATij[r * 8 + q] * bp[q];
            }
            b[iIdx + r] += sh;
            b[jIdx + r] += st;
        }
        for (int kk = 0; kk < nf; kk++) {
            int kIdx = CPARS + kk * 8;
            int ijkIdx = ijIdx + kk * nframes2;
            int ikIdx = i + nf * kk;
            double accDM[64];
            std::memset(accDM, 0, sizeof(accDM));
            for (int tid2 = 0; tid2 < toAggregate; tid2++) {
                ow->accD[tid2][ijkIdx].finish();
                if (ow->accD[tid2][ijkIdx].num == 0) continue;
                for (int q = 0; q < 64; q++) accDM[q] += (double)ow->accD[tid2][ijkIdx].A1m[q];
            }
            const double *AHik = &ow->adHost[(size_t)ikIdx * 64], *ATik = &ow->adTarget[(size_t)ikIdx * 64];
            double blk[64];
            sandwich(AHij, accDM, AHik, blk);
            for (int r = 0; r < 8; r++)
                for (int c = 0; c < 8; c++) H[(size_t)(iIdx + r) * D + iIdx + c] += blk[r * 8 + c];
            sandwich(ATij, accDM, ATik, blk);
            for (int r = 0; r < 8; r++)
                for (int c = 0; c < 8; c++) H[(size_t)(jIdx + r) * D + kIdx + c] += blk[r * 8 + c];
            sandwich(ATij, accDM, AHik, blk);
            for (int r = 0; r < 8; r++)
                for (int c = 0; c < 8; c++) H[(size_t)(jIdx + r) * D + iIdx + c] += blk[r * 8 + c];
            sandwich(AHij, accDM, ATik, blk);
            for (int r = 0; r < 8; r++)
                for (int c = 0; c < 8; c++) H[(size_t)(iIdx + r) * D + kIdx + c] += blk[r * 8 + c];
        }
    }
    if (min == 0) {
        for (int tid2 = 0; tid2 < toAggregate; tid2++) {
            ow->accHcc[tid2].finish();
            ow->accbc[tid2].finish();
            for (int r = 0; r < 4; r++) {
                for (int c = 0; c < 4; c++) H[(size_t)r * D + c] += (double)ow->accHcc[tid2].A1m[r * 4 + c];
                b[r] += (double)ow->accbc[tid2].A1m[r];
            }
        }
    }
}

// stitchDoubleMT: AccumulatedSCHessian.h:64-98
void scStitchMT(oracle_window *ow, std::vector<double> &H, std::vector<double> &b, bool MT) {
    const int N = ow->N, D = dimH(N);
    if (MT) {
        int nt = ow->red->n();
        std::vector<std::vector<double>> Hs(nt, std::vector<double>((size_t)D * D, 0.0));
        std::vector<std::vector<double>> bs(nt, std::vector<double>(D, 0.0));
        ow->red->reduce([&](int mn, int mx, Vec10 *, int tid) { scStitchInternal(ow, Hs[tid], bs[tid], mn, mx, tid); },
                        0, N * N, 0);
        H = Hs[0];
        b = bs[0];
        for (int i = 1; i < nt; i++) {
            for (size_t k = 0; k < H.size(); k++) H[k] += Hs[i][k];
            for (int k = 0; k < D; k++) b[k] += bs[i][k];
        }
    } else {
        H.assign((size_t)D * D, 0.0);
        b.assign(D, 0.0);
        scStitchInternal(ow, H, b, 0, N * N, -1);
    }
    for (int h = 0; h < N; h++) {
        int hIdx = CPARS + h * 8;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 8; j++) H[(size_t)i * D + hIdx + j] = H[(size_t)(hIdx + j) * D + i];
    }
}

void ensure_pool(oracle_window *ow) {
    int nt = g_threads > 0 ? g_threads : 1;
    if (g_threads > 0 && (!ow->red || ow->red->n() != nt)) {
        delete ow->red;
        ow->red = new IndexThreadReduce(nt);
    }
    const int N = ow->N;
    if ((int)ow->accTop.size() != nt || (ow->accTop.size() && (int)ow->accTop[0].size() != N * N)) {
        ow->accTop.assign(nt, std::vector<AccumulatorApprox>(N * N));
        ow->accE.assign(nt, std::vector<AccumulatorXX<8, 4>>(N * N));
        ow->accEB.assign(nt, std::vector<AccumulatorX<8>>(N * N));
        ow->accD.assign(nt, std::vector<AccumulatorXX<8, 8>>(N * N * N));
        ow->accHcc.assign(nt, AccumulatorXX<4, 4>());
        ow->accbc.assign(nt, AccumulatorX<4>());
        ow->nres.assign(nt, 0);
    }
}

// EnergyFunctional::accumulateAF_MT / LF_MT / SCF_MT: EnergyFunctional.cc:670-749
void accumulateAll(oracle_window *ow, std::vector<double> &HA, std::vector<double> &bA,
                   std::vector<double> &HL, std::vector<double> &bL, std::vector<double> &Hsc,
                   std::vector<double> &bsc) {
    ensure_pool(ow);
    const bool MT = g_threads > 0;
    const int N = ow->N;
    const int P = (int)ow->points.size();
    auto setZeroTop = [&](int tid) {
        for (auto &a : ow->accTop[tid]) a.initialize();
        ow->nres[tid] = 0;
    };
    auto setZeroSC = [&](int tid) {
        ow->accHcc[tid].initialize();
        ow->accbc[tid].initialize();
        for (auto &a : ow->accE[tid]) a.initialize();
        for (auto &a : ow->accEB[tid]) a.initialize();
        for (auto &a : ow->accD[tid]) a.initialize();
    };
    (void)N;
    // A (mode 0)
    if (MT) {
        ow->red->reduce([&](int, int, Vec10 *, int tid) { setZeroTop(tid); }, 0, 0, 0);
        ow->red->reduce([&](int mn, int mx, Vec10 *, int tid) {
            for (int i = mn; i < mx; i++) topAddPoint<0>(ow, ow->points[i], tid);
        }, 0, P, 50);
    } else {
        setZeroTop(0);
        for (int i = 0; i < P; i++) topAddPoint<0>(ow, ow->points[i], 0);
    }
    topStitchMT(ow, HA, bA, false, MT);
    // L (mode 1, with priors)
    if (MT) {
        ow->red->reduce([&](int, int, Vec10 *, int tid) { setZeroTop(tid); }, 0, 0, 0);
        ow->red->reduce([&](int mn, int mx, Vec10 *, int tid) {
            for (int i = mn; i < mx; i++) topAddPoint<1>(ow, ow->points[i], tid);
        }, 0, P, 50);
    } else {
        setZeroTop(0);
        for (int i = 0; i < P; i++) topAddPoint<1>(ow, ow->points[i], 0);
    }
    topStitchMT(ow, HL, bL, true, MT);
    // SC
    if (MT) {
        ow->red->reduce([&](int, int, Vec10 *, int tid) { setZeroSC(tid); }, 0, 0, 0);
        ow->red->reduce([&](int mn, int mx, Vec10 *, int tid) {
            for (int i = mn; i < mx; i++) scAddPoint(ow, ow->points[i], true, tid);
        }, 0, P, 50);
    } else {
        setZeroSC(0);
        for (int i = 0; i < P; i++) scAddPoint(ow, ow->points[i], true, 0);
    }
    scStitchMT(ow, Hsc, bsc, MT);
}

double linearizeAllImpl(oracle_window *ow, bool fix, double *out) {
    ensure_pool(ow);
    const int R = (int)ow->res.size();
    double E = 0, num = 0;
    if (g_threads > 0) {
        ow->red->reduce([&](int mn, int mx, Vec10 *st, int) { linearizeAll_Reductor(ow, fix, mn, mx, st); }, 0, R, 0);
        E = ow->red->stats.v[0];
        num = ow->red->stats.v[1];
    } else {
        Vec10 st;
        std::memset(&st, 0, sizeof(st));
        linearizeAll_Reductor(ow, fix, 0, R, &st);
        E = st.v[0];
        num = st.v[1];
    }
    setNewFrameEnergyTH(ow);
    if (out) {
        out[0] = E;
        out[1] = 0;
        out[2] = num;
    }
    return E;
}

void applyResAll(oracle_window *ow) {
    const int R = (int)ow->res.size();
    if (g_threads > 0) {
        ensure_pool(ow);
        ow->red->reduce([&](int mn, int mx, Vec10 *, int) {
            for (int k = mn; k < mx; k++) ow->res[k].applyRes(true);
        }, 0, R, 50);
    } else {
        for (int k = 0; k < R; k++) ow->res[k].applyRes(true);
    }
}

// ---- dense double helpers (host side) -------------------------------------------------
// Sophus SE3 (thirdparty/Sophus/sophus/se3.hpp, so3.hpp) as Sophus stores it: a unit quaternion
// (Eigen coeffs() order x, y, z, w) and a translation.  Every operation below restates Sophus's
// code in its statement order (Eigen's fixed-size sums as its packet code adds them; no FMA).
struct SE3d {
    double q[4];  // x, y, z, w
    double t[3];
};
void hat(const double w[3], double M[9]) {
    M[0] = 0; M[1] = -w[2]; M[2] = w[1];
    M[3] = w[2]; M[4] = 0; M[5] = -w[0];
    M[6] = -w[1]; M[7] = w[0]; M[8] = 0;
}
void mm3(const double *A, const double *B, double *C) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}
void mv3(const double *A, const double *v, double *out) {
    for (int i = 0; i < 3; i++) out[i] = A[i * 3] * v[0] + A[i * 3 + 1] * v[1] + A[i * 3 + 2] * v[2];
}
// SO3Base::normalize (so3.hpp:289-295): Eigen's 4-vector norm sums (x^2 + z^2) + (y^2 + w^2)
void quat_normalize(double q[4]) {
    const double len = std::sqrt((q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]));
    for (int i = 0; i < 4; i++) q[i] /= len;
}
// Eigen Quaternion::toRotationMatrix (SO3::matrix, so3.hpp:302-304)
void quat_matrix(const double q[4], double R[9]) {
    const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
// the SO3 action on a point (so3.hpp:341-347)
void quat_rotate(const double q[4], const double p[3], double out[3]) {
    double uv[3] = {q[1] * p[2] - q[2] * p[1], q[2] * p[0] - q[0] * p[2], q[0] * p[1] - q[1] * p[0]};
    for (int i = 0; i < 3; i++) uv[i] += uv[i];
    const double c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2], q[0] * uv[1] - q[1] * uv[0]};
    for (int i = 0; i < 3; i++) out[i] = p[i] + q[3] * uv[i] + c[i];
}
// Sophus::SE3::exp (se3.hpp:765-786), tangent = [upsilon, omega], through SO3::expAndTheta
// (so3.hpp:577-605: imaginary factor sin(theta / 2) / theta, real factor cos(theta / 2))
SE3d se3_exp(const double a[6]) {
    const double *up = a, *w = a + 3;
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const double th = std::sqrt(th2);
    double im, re;
    if (th < 1e-10) {
        const double th4 = th2 * th2;
        im = 0.5 - (1.0 / 48.0) * th2 + (1.0 / 3840.0) * th4;
        re = 1 - (1.0 / 8.0) * th2 + (1.0 / 384.0) * th4;
    } else {
        im = std::sin(0.5 * th) / th;
        re = std::cos(0.5 * th);
    }
    SE3d T;
    T.q[0] = im * w[0];
    T.q[1] = im * w[1];
    T.q[2] = im * w[2];
    T.q[3] = re;
    double V[9];
    if (th < 1e-10) {
        quat_matrix(T.q, V);
    } else {
        double W[9], W2[9];
        hat(w, W);
        mm3(W, W, W2);
        const double B = (1 - std::cos(th)) / th2, C = (th - std::sin(th)) / (th2 * th);
        for (int i = 0; i < 9; i++) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + B * W[i] + C * W2[i];
    }
    mv3(V, up, T.t);
    return T;
}
// Sophus::SE3::log (se3.hpp:220-253): SO3::logAndTheta (so3.hpp:239-283, atan form) on the
// quaternion, V^-1 with theta cos(theta/2) / (2 sin(theta/2)); epsilon 1e-10
void se3_log(const SE3d &T, double out[6]) {
    const double *q = T.q;
    const double squared_n = q[0] * q[0] + q[1] * q[1] + q[2] * q[2];
    const double n = std::sqrt(squared_n), w = q[3];
    double two_atan_nbyw_by_n;
    if (n < 1e-10) two_atan_nbyw_by_n = 2.0 / w - 2.0 * squared_n / (w * (w * w));
    else if (std::fabs(w) < 1e-10) two_atan_nbyw_by_n = (w > 0 ? M_PI : -M_PI) / n;
    else two_atan_nbyw_by_n = 2.0 * std::atan(n / w) / n;
    const double theta = two_atan_nbyw_by_n * n;
    double w3[3] = {two_atan_nbyw_by_n * q[0], two_atan_nbyw_by_n * q[1], two_atan_nbyw_by_n * q[2]};
    double W[9], W2[9];
    hat(w3, W);
    mm3(W, W, W2);
    double D;
    if (std::fabs(theta) < 1e-10) D = 1.0 / 12.0;
    else D = (1.0 - theta * std::cos(0.5 * theta) / (2.0 * std::sin(0.5 * theta))) / (theta * theta);
    double Vi[9];
    for (int i = 0; i < 9; i++) Vi[i] = ((i % 4 == 0) ? 1.0 : 0.0) - 0.5 * W[i] + D * W2[i];
    mv3(Vi, T.t, out);
    for (int i = 0; i < 3; i++) out[3 + i] = w3[i];
}
// SE3 product (se3.hpp:305-309): the quaternion product (so3.hpp:320-326), normalised by the
// SO3(quaternion) constructor (so3.hpp:475-481), and t_A + R_A t_B through the quaternion action
SE3d se3_mul(const SE3d &A, const SE3d &B) {
    const double *a = A.q, *b = B.q;
    SE3d C;
    C.q[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    C.q[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    C.q[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    C.q[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    quat_normalize(C.q);
    double r[3];
    quat_rotate(A.q, B.t, r);
    for (int i = 0; i < 3; i++) C.t[i] = A.t[i] + r[i];
    return C;
}
// SE3::inverse (se3.hpp:205-208): SO3(conjugate) (normalised) applied to -t
SE3d se3_inv(const SE3d &A) {
    SE3d C;
    C.q[0] = -A.q[0];
    C.q[1] = -A.q[1];
    C.q[2] = -A.q[2];
    C.q[3] = A.q[3];
    quat_normalize(C.q);
    const double mt[3] = {A.t[0] * -1.0, A.t[1] * -1.0, A.t[2] * -1.0};
    quat_rotate(C.q, mt, C.t);
    return C;
}
// Sophus SE3::Adj = [R, hat(t) R; 0, R] (se3.hpp:100-108)
void se3_adj(const SE3d &T, double Adj[36]) {
    std::memset(Adj, 0, 36 * sizeof(double));
    double R[9], tx[9], tR[9];
    quat_matrix(T.q, R);
    hat(T.t, tx);
    mm3(tx, R, tR);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            Adj[i * 6 + j] = R[i * 3 + j];
            Adj[i * 6 + 3 + j] = tR[i * 3 + j];
            Adj[(3 + i) * 6 + 3 + j] = R[i * 3 + j];
        }
}
// worldToCam_evalPT from the ABI's matrix3x4(): SE3(Matrix3, t) -> SO3(R) = Eigen's
// Quaternion(Matrix3) (Quaternion.h, quaternionbase_assign_impl)
SE3d frame_evalpt(const ldso_ba_frame_state &f) {
    const double *R = f.world_to_cam_evalpt;
    SE3d T;
    double *q = T.q;
    const double tr = R[0] + R[4] + R[8];
    if (tr > 0) {
        double t = std::sqrt(tr + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (R[7] - R[5]) * t;
        q[1] = (R[2] - R[6]) * t;
        q[2] = (R[3] - R[1]) * t;
    } else {
        int i = 0;
        if (R[4] > R[0]) i = 1;
        if (R[8] > R[i * 4]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double t = std::sqrt(R[i * 4] - R[j * 4] - R[k * 4] + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (R[k * 3 + j] - R[j * 3 + k]) * t;
        q[j] = (R[j * 3 + i] + R[i * 3 + j]) * t;
        q[k] = (R[k * 3 + i] + R[i * 3 + k]) * t;
    }
    for (int i = 0; i < 3; i++) T.t[i] = f.world_to_cam_evalpt[9 + i];
    return T;
}
// FrameHessian::setState: PRE_worldToCam = exp(w2c_leftEps) * evalPT (FrameHessian.h:95-114)
SE3d frame_pre_w2c(const ldso_ba_frame_state &f) {
    double eps[6];
    for (int i = 0; i < 3; i++) eps[i] = SCALE_XI_TRANS * f.state[i];
    for (int i = 3; i < 6; i++) eps[i] = SCALE_XI_ROT * f.state[i];
    return se3_mul(se3_exp(eps), frame_evalpt(f));
}
}  // namespace

// AffLight::fromToVecExposure: include/AffLight.h:27-35 (exp of a float, as expf)
namespace {
void fromToVecExposure2(float exposureF, float exposureT, float g2Fa, float g2Fb, float g2Ta,
                        float g2Tb, double out[2]) {
    if (exposureF == 0 || exposureT == 0) exposureT = exposureF = 1;
    float a = std::exp(g2Ta - g2Fa) * exposureT / exposureF;
    float b = g2Tb - a * g2Fb;
    out[0] = a;
    out[1] = b;
}
}  // namespace

// ---- LDLT with diagonal pivoting (Eigen::LDLT semantics) -------------------------------
static bool ldlt_solve(int n, std::vector<double> A, std::vector<double> b, std::vector<double> &x) {
    std::vector<int> perm(n);
    for (int i = 0; i < n; i++) perm[i] = i;
    // A is full symmetric; in-place LDL^T with symmetric pivoting on max |diag|
    for (int k = 0; k < n; k++) {
        int piv = k;
        double best = std::fabs(A[(size_t)k * n + k]);
        for (int i = k + 1; i < n; i++)
            if (std::fabs(A[(size_t)i * n + i]) > best) {
                best = std::fabs(A[(size_t)i * n + i]);
                piv = i;
            }
        if (piv != k) {
            std::swap(perm[k], perm[piv]);
            for (int j = 0; j < n; j++) std::swap(A[(size_t)k * n + j], A[(size_t)piv * n + j]);
            for (int j = 0; j < n; j++) std::swap(A[(size_t)j * n + k], A[(size_t)j * n + piv]);
        }
        double d = A[(size_t)k * n + k];
        // trailing update A(i,j) -= A(i,k) A(j,k) / d with the UNSCALED column k, then L(i,k) = A(i,k) / d
        std::vector<double> col(n, 0.0);
        for (int i = k + 1; i < n; i++) col[i] = A[(size_t)i * n + k];
        for (int i = k + 1; i < n; i++) {
            double l = (d != 0) ? col[i] / d : 0.0;
            for (int j = k + 1; j <= i; j++) A[(size_t)i * n + j] -= l * col[j];
            A[(size_t)i * n + k] = l;
        }
        for (int i = k + 1; i < n; i++)
            for (int j = k + 1; j < i; j++) A[(size_t)j * n + i] = A[(size_t)i * n + j];
    }
    std::vector<double> y(n);
    for (int i = 0; i < n; i++) y[i] = b[perm[i]];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < i; j++) y[i] -= A[(size_t)i * n + j] * y[j];
    for (int i = 0; i < n; i++) {
        double d = A[(size_t)i * n + i];
        y[i] = (d != 0) ? y[i] / d : 0.0;
    }
    for (int i = n - 1; i >= 0; i--)
        for (int j = i + 1; j < n; j++) y[i] -= A[(size_t)j * n + i] * y[j];
    x.assign(n, 0.0);
    for (int i = 0; i < n; i++) x[perm[i]] = y[i];
    return true;
}

// Jacobi eigen-decomposition of a small symmetric matrix (for the nullspace projector).
static void jacobi_eig(int n, std::vector<double> A, std::vector<double> &evals, std::vector<double> &V) {
    V.assign((size_t)n * n, 0.0);
    for (int i = 0; i < n; i++) V[(size_t)i * n + i] = 1;
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) off += A[(size_t)p * n + q] * A[(size_t)p * n + q];
        if (off < 1e-30) break;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) {
                double apq = A[(size_t)p * n + q];
                if (std::fabs(apq) < 1e-300) continue;
                double app = A[(size_t)p * n + p], aqq = A[(size_t)q * n + q];
                double theta = (aqq - app) / (2 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
                double c = 1 / std::sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < n; k++) {
                    double akp = A[(size_t)k * n + p], akq = A[(size_t)k * n + q];
                    A[(size_t)k * n + p] = c * akp - s * akq;
                    A[(size_t)k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; k++) {
                    double apk = A[(size_t)p * n + k], aqk = A[(size_t)q * n + k];
                    A[(size_t)p * n + k] = c * apk - s * aqk;
                    A[(size_t)q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; k++) {
                    double vkp = V[(size_t)k * n + p], vkq = V[(size_t)k * n + q];
                    V[(size_t)k * n + p] = c * vkp - s * vkq;
                    V[(size_t)k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    evals.resize(n);
    for (int i = 0; i < n; i++) evals[i] = A[(size_t)i * n + i];
}

// EnergyFunctional::orthogonalize (x only): EnergyFunctional.cc:809-841
static void orthogonalize_x(int n, const double *ns, int k, std::vector<double> &x) {
    std::vector<double> Nm((size_t)n * k);
    for (int c = 0; c < k; c++) {
        double nrm = 0;
        for (int i = 0; i < n; i++) nrm += ns[(size_t)c * n + i] * ns[(size_t)c * n + i];
        nrm = std::sqrt(nrm);
        for (int i = 0; i < n; i++) Nm[(size_t)i * k + c] = ns[(size_t)c * n + i] / nrm;
    }
    std::vector<double> G((size_t)k * k, 0.0);
    for (int a = 0; a < k; a++)
        for (int b2 = 0; b2 < k; b2++) {
            double s = 0;
            for (int i = 0; i < n; i++) s += Nm[(size_t)i * k + a] * Nm[(size_t)i * k + b2];
            G[(size_t)a * k + b2] = s;
        }
    std::vector<double> ev, V;
    jacobi_eig(k, G, ev, V);
    double maxSv = 0;
    for (int i = 0; i < k; i++) maxSv = std::max(maxSv, std::sqrt(std::max(ev[i], 0.0)));
    // projector P = N V diag(1/ev or 0) V^T N^T  (= NNpiTS)
    std::vector<double> Ginv((size_t)k * k, 0.0);
    for (int e = 0; e < k; e++) {
        double sv = std::sqrt(std::max(ev[e], 0.0));
        if (!(sv > setting_solverModeDelta * maxSv)) continue;
        for (int a = 0; a < k; a++)
            for (int b2 = 0; b2 < k; b2++) Ginv[(size_t)a * k + b2] += V[(size_t)a * k + e] * V[(size_t)b2 * k + e] / ev[e];
    }
    std::vector<double> Ntx(k, 0.0), c(k, 0.0);
    for (int a = 0; a < k; a++)
        for (int i = 0; i < n; i++) Ntx[a] += Nm[(size_t)i * k + a] * x[i];
    for (int a = 0; a < k; a++)
        for (int b2 = 0; b2 < k; b2++) c[a] += Ginv[(size_t)a * k + b2] * Ntx[b2];
    for (int i = 0; i < n; i++) {
        double s = 0;
        for (int a = 0; a < k; a++) s += Nm[(size_t)i * k + a] * c[a];
        x[i] -= s;
    }
}

extern "C" {

void oracle_set_threads(int n) { g_threads = std::max(0, std::min(n, NUM_THREADS_MAX)); }
// setting_affineOptModeA / B as a driver sets them before the system starts (run_dso_kitti.cc:299-300,
// run_dso_euroc.cc:291-292, run_dso_tum_mono.cc:284-292): read by linearize (Residuals.cc:186-187)
// and takeData's getPrior (FrameHessian.h:154-165) as the reference reads its globals
void oracle_set_affine_opt_modes(float a, float b) {
    setting_affineOptModeA = a;
    setting_affineOptModeB = b;
}
void oracle_get_affine_opt_modes(float *a, float *b) {
    *a = setting_affineOptModeA;
    *b = setting_affineOptModeB;
}
int oracle_get_threads(void) { return g_threads; }

oracle_window *oracle_create(const ldso_ba_window *w) {
    if (!w || w->n_frames < 2 || w->n_frames > LDSO_BA_MAX_FRAMES) return nullptr;
    oracle_window *ow = new oracle_window();
    load_update(ow, w, true);
    return ow;
}
void oracle_destroy(oracle_window *ow) { delete ow; }
int oracle_update(oracle_window *ow, const ldso_ba_window *w) {
    if (!ow || !w || w->n_frames != ow->N) return -1;
    load_update(ow, w, false);
    return 0;
}
void oracle_reset_oob(oracle_window *ow) {
    for (auto &r : ow->res) r.resetOOB();
}
int oracle_linearize_all(oracle_window *ow, int fix, double *out) {
    linearizeAllImpl(ow, fix != 0, out);
    return 0;
}
void oracle_apply_res(oracle_window *ow) { applyResAll(ow); }

int oracle_accumulate(oracle_window *ow, double *HA, double *bA, double *HL, double *bL,
                      double *Hsc, double *bsc) {
    std::vector<double> vHA, vbA, vHL, vbL, vHsc, vbsc;
    accumulateAll(ow, vHA, vbA, vHL, vbL, vHsc, vbsc);
    auto cp = [](const std::vector<double> &v, double *o) {
        if (o) std::memcpy(o, v.data(), v.size() * sizeof(double));
    };
    cp(vHA, HA);
    cp(vbA, bA);
    cp(vHL, HL);
    cp(vbL, bL);
    cp(vHsc, Hsc);
    cp(vbsc, bsc);
    return 0;
}

int oracle_iteration(oracle_window *ow, double *energy_out) {
    linearizeAllImpl(ow, false, energy_out);
    applyResAll(ow);
    std::vector<double> HA, bA, HL, bL, Hsc, bsc;
    accumulateAll(ow, HA, bA, HL, bL, Hsc, bsc);
    return 0;
}

void oracle_get_residuals(oracle_window *ow, int8_t *new_state, int8_t *state, float *state_energy,
                          float *new_energy_wo, float *center, uint8_t *flags, float *jpjdf,
                          float *rel_bs) {
    for (size_t k = 0; k < ow->res.size(); k++) {
        const Residual &r = ow->res[k];
        if (new_state) new_state[k] = (int8_t)r.state_NewState;
        if (state) state[k] = (int8_t)r.state_state;
        if (state_energy) state_energy[k] = (float)r.state_energy;
        if (new_energy_wo) new_energy_wo[k] = (float)r.state_NewEnergyWithOutlier;
        if (center)
            for (int i = 0; i < 3; i++) center[3 * k + i] = r.centerProjectedTo[i];
        if (flags) flags[k] = (r.isActiveAndIsGoodNEW ? LDSO_BA_FLAG_ACTIVE : 0) | (r.isNew ? LDSO_BA_FLAG_NEW : 0);
        if (jpjdf)
            for (int i = 0; i < 8; i++) jpjdf[8 * k + i] = r.JpJdF[i];
        if (rel_bs) rel_bs[k] = r.relBS;
    }
}

void oracle_get_jacobians(oracle_window *ow, float *out) {
    for (size_t k = 0; k < ow->res.size(); k++) {
        const RawResidualJacobian &J = ow->res[k].J;
        float *o = out + 78 * k;
        int q = 0;
        for (int i = 0; i < 8; i++) o[q++] = J.resF[i];
        for (int a = 0; a < 2; a++)
            for (int i = 0; i < 6; i++) o[q++] = J.Jpdxi[a][i];
        for (int a = 0; a < 2; a++)
            for (int i = 0; i < 4; i++) o[q++] = J.Jpdc[a][i];
        o[q++] = J.Jpdd[0];
        o[q++] = J.Jpdd[1];
        for (int a = 0; a < 2; a++)
            for (int i = 0; i < 8; i++) o[q++] = J.JIdx[a][i];
        for (int a = 0; a < 2; a++)
            for (int i = 0; i < 8; i++) o[q++] = J.JabF[a][i];
        for (int a = 0; a < 2; a++)
            for (int i = 0; i < 2; i++) o[q++] = J.JIdx2[a][i];
        for (int a = 0; a < 2; a++)
            for (int i = 0; i < 2; i++) o[q++] = J.JabJIdx[a][i];
        for (int a = 0; a < 2; a++)
            for (int i = 0; i < 2; i++) o[q++] = J.Jab2[a][i];
    }
}

void oracle_get_points(oracle_window *ow, float *HdiF, float *bdSumF, float *idepth_hessian,
                       float *Hdd_acc, float *bd_acc, float *Hcd_acc) {
    for (size_t p = 0; p < ow->points.size(); p++) {
        const PointH &ph = ow->points[p];
        if (HdiF) HdiF[p] = ph.HdiF;
        if (bdSumF) bdSumF[p] = ph.bdSumF;
        if (idepth_hessian) idepth_hessian[p] = ph.idepth_hessian;
        if (Hdd_acc) Hdd_acc[p] = ph.Hdd_accAF;
        if (bd_acc) bd_acc[p] = ph.bd_accAF;
        if (Hcd_acc)
            for (int i = 0; i < 4; i++) Hcd_acc[4 * p + i] = ph.Hcd_accAF[i];
    }
}

void oracle_get_frame_energy_th(oracle_window *ow, float *th) {
    for (int f = 0; f < ow->N; f++) th[f] = ow->frames[f].frameEnergyTH;
}

// EnergyFunctional::solveSystemF, non-VI, !SOLVER_ORTHOGONALIZE_SYSTEM branch:
// EnergyFunctional.cc:282-283, 310, 342-378, 413-432
int oracle_solve_system(int n_frames, int iteration, double lambda, const double *HA,
                        const double *bA, const double *HL, const double *bL, const double *HM,
                        const double *bM, const double *Hsc, const double *bsc,
                        const double *nullspaces, int n_null, double *x_out) {
    const int n = 8 * n_frames + CPARS;
    lambda = 1e-5;  // SOLVER_FIX_LAMBDA (setting_solverMode = FIX_LAMBDA | ORTHOGONALIZE_X_LATER)
    std::vector<double> Hf((size_t)n * n, 0.0), bf(n, 0.0);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            size_t q = (size_t)i * n + j;
            Hf[q] = HL[q] + (HM ? HM[q] : 0.0) + HA[q];
        }
    for (int i = 0; i < n; i++)
        bf[i] = bL[i] + (bM ? bM[i] : 0.0) + bA[i] - bsc[i] / (1 + lambda);
    for (int i = 0; i < n; i++) Hf[(size_t)i * n + i] *= (1 + lambda);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) Hf[(size_t)i * n + j] -= Hsc[(size_t)i * n + j] * (1.0f / (1 + lambda));
    for (int i = 0; i < n; i++)
        for (int j = 0; j < i; j++) Hf[(size_t)i * n + j] = Hf[(size_t)j * n + i];
    std::vector<double> S(n);
    for (int i = 0; i < n; i++) S[i] = 1.0 / std::sqrt(Hf[(size_t)i * n + i] + 10);
    std::vector<double> Hs((size_t)n * n), bs(n), x;
    for (int i = 0; i < n; i++) {
        bs[i] = S[i] * bf[i];
        for (int j = 0; j < n; j++) Hs[(size_t)i * n + j] = S[i] * Hf[(size_t)i * n + j] * S[j];
    }
    ldlt_solve(n, Hs, bs, x);
    for (int i = 0; i < n; i++) x[i] *= S[i];
    if (iteration >= 2 && nullspaces && n_null > 0) orthogonalize_x(n, nullspaces, n_null, x);
    std::memcpy(x_out, x.data(), n * sizeof(double));
    return 0;
}

// EnergyFunctional::resubstituteF_MT / resubstituteFPt: EnergyFunctional.cc:611-667
void oracle_resubstitute(oracle_window *ow, const double *x, double lambda, float *point_step) {
    const int N = ow->N;
    ow->currentLambda = (float)lambda;
    std::vector<float> xF(8 * N + CPARS);
    for (size_t i = 0; i < xF.size(); i++) xF[i] = (float)x[i];
    std::vector<float> xAd((size_t)N * N * 8);
    for (int h = 0; h < N; h++)
        for (int t = 0; t < N; t++) {
            const float *AH = &ow->adHostF[(size_t)(h + N * t) * 64], *AT = &ow->adTargetF[(size_t)(h + N * t) * 64];
            for (int c = 0; c < 8; c++) {
                float s = 0, s2 = 0;
                for (int k = 0; k < 8; k++) s += xF[CPARS + 8 * h + k] * AH[k * 8 + c];
                for (int k = 0; k < 8; k++) s2 += xF[CPARS + 8 * t + k] * AT[k * 8 + c];
                xAd[(size_t)(N * h + t) * 8 + c] = s + s2;
            }
        }
    for (size_t p = 0; p < ow->points.size(); p++) {
        PointH &ph = ow->points[p];
        int ngood = 0;
        for (int ri : ph.residuals)
            if (ow->res[ri].isActive()) ngood++;
        if (ngood == 0) {
            ph.step = 0;
            if (point_step) point_step[p] = 0;
            continue;
        }
        float b = ph.bdSumF;
        float dotc = 0;
        for (int i = 0; i < 4; i++) dotc += xF[i] * (ph.Hcd_accAF[i] + ph.Hcd_accLF[i]);
        b -= dotc;
        for (int ri : ph.residuals) {
            const Residual &r = ow->res[ri];
            if (!r.isActive()) continue;
            float d = 0;
            for (int i = 0; i < 8; i++) d += xAd[(size_t)(r.hostIDX * N + r.targetIDX) * 8 + i] * r.JpJdF[i];
            b -= d;
        }
        ph.step = -b * ph.HdiF / (1 + ow->currentLambda);
        if (point_step) point_step[p] = ph.step;
    }
    ow->currentLambda = 0;
}

// FrameFramePrecalc::Set: src/internal/FrameFramePrecalc.cc:6-35
int oracle_frame_precalc(int N, const ldso_ba_frame_state *frames, const float calib[4], float *out) {
    for (int h = 0; h < N; h++)
        for (int t = 0; t < N; t++) {
            float *o = out + (size_t)(h + N * t) * LDSO_BA_PRECALC_STRIDE;
            std::memset(o, 0, LDSO_BA_PRECALC_STRIDE * sizeof(float));
            SE3d l2l0 = se3_mul(frame_evalpt(frames[t]), se3_inv(frame_evalpt(frames[h])));
            SE3d l2l = se3_mul(frame_pre_w2c(frames[t]), se3_inv(frame_pre_w2c(frames[h])));
            double l2l0R[9], l2lR[9];  // rotationMatrix()
            quat_matrix(l2l0.q, l2l0R);
            quat_matrix(l2l.q, l2lR);
            float RTll[9], tTll[3];
            for (int i = 0; i < 9; i++) {
                o[12 + i] = (float)l2l0R[i];          // PRE_RTll_0
                o[27 + i] = RTll[i] = (float)l2lR[i];  // PRE_RTll
            }
            for (int i = 0; i < 3; i++) {
                o[21 + i] = (float)l2l0.t[i];          // PRE_tTll_0
                o[36 + i] = tTll[i] = (float)l2l.t[i];  // PRE_tTll
            }
            float K[9] = {calib[0], 0, calib[2], 0, calib[1], calib[3], 0, 0, 1};
            // K.inverse(): Eigen's 3x3 cofactor inverse (Eigen/src/LU/InverseImpl.h,
            // compute_inverse<...,3>) specialised to K = [fx 0 cx; 0 fy cy; 0 0 1]
            float det = calib[1] * calib[0];
            float invdet = 1.0f / det;
            float Ki[9] = {calib[1] * invdet, 0 * invdet, (0 * calib[3] - calib[2] * calib[1]) * invdet,
                           0 * invdet, calib[0] * invdet, (calib[2] * 0 - calib[0] * calib[3]) * invdet,
                           0 * invdet, 0 * invdet, (calib[0] * calib[1] - 0 * 0) * invdet};
            float KR[9], KRKi[9];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) KR[i * 3 + j] = K[i * 3] * RTll[j] + K[i * 3 + 1] * RTll[3 + j] + K[i * 3 + 2] * RTll[6 + j];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) KRKi[i * 3 + j] = KR[i * 3] * Ki[j] + KR[i * 3 + 1] * Ki[3 + j] + KR[i * 3 + 2] * Ki[6 + j];
            for (int i = 0; i < 9; i++) o[i] = KRKi[i];
            for (int i = 0; i < 3; i++) o[9 + i] = K[i * 3] * tTll[0] + K[i * 3 + 1] * tTll[1] + K[i * 3 + 2] * tTll[2];
            const ldso_ba_frame_state &H = frames[h], &T = frames[t];
            double aff[2];
            fromToVecExposure2((float)H.ab_exposure, (float)T.ab_exposure, (float)(SCALE_A * H.state[6]),
                               (float)(SCALE_B * H.state[7]), (float)(SCALE_A * T.state[6]), (float)(SCALE_B * T.state[7]), aff);
            o[24] = (float)aff[0];
            o[25] = (float)aff[1];
            o[26] = (float)(H.state_zero[7] * SCALE_B);
        }
    return 0;
}

// EnergyFunctional::setAdjointsF: EnergyFunctional.cc:551-609
int oracle_set_adjoints(int N, const ldso_ba_frame_state *frames, double *ad_host, double *ad_target,
                        double *c_prior) {
    for (int h = 0; h < N; h++)
        for (int t = 0; t < N; t++) {
            SE3d h2t = se3_mul(frame_evalpt(frames[t]), se3_inv(frame_evalpt(frames[h])));
            double Adj[36];
            se3_adj(h2t, Adj);
            double AH[64], AT[64];
            std::memset(AH, 0, sizeof(AH));
            std::memset(AT, 0, sizeof(AT));
            for (int i = 0; i < 8; i++) AH[i * 8 + i] = AT[i * 8 + i] = 1;
            for (int i = 0; i < 6; i++)
                for (int j = 0; j < 6; j++) {
                    AH[i * 8 + j] = -Adj[j * 6 + i];
                    AT[i * 8 + j] = (i == j) ? 1 : 0;
                }
            const ldso_ba_frame_state &H = frames[h], &T = frames[t];
            double aff[2];
            fromToVecExposure2((float)H.ab_exposure, (float)T.ab_exposure, (float)(H.state_zero[6] * SCALE_A),
                               (float)(H.state_zero[7] * SCALE_B), (float)(T.state_zero[6] * SCALE_A),
                               (float)(T.state_zero[7] * SCALE_B), aff);
            float affLL0 = (float)aff[0];
            AT[6 * 8 + 6] = -affLL0;
            AH[6 * 8 + 6] = affLL0;
            AT[7 * 8 + 7] = -1;
            AH[7 * 8 + 7] = affLL0;
            for (int r = 0; r < 8; r++) {
                double s = r < 3 ? SCALE_XI_TRANS : r < 6 ? SCALE_XI_ROT : r == 6 ? SCALE_A : SCALE_B;
                for (int c = 0; c < 8; c++) {
                    AH[r * 8 + c] *= s;
                    AT[r * 8 + c] *= s;
                }
            }
            std::memcpy(ad_host + (size_t)(h + t * N) * 64, AH, sizeof(AH));
            std::memcpy(ad_target + (size_t)(h + t * N) * 64, AT, sizeof(AT));
        }
    for (int i = 0; i < 4; i++) c_prior[i] = setting_initialCalibHessian;
    return 0;
}

// FrameHessian::takeData / getPrior / get_state_minus_stateZero: FrameHessian.h:59-70, 142-174,
// FrameHessian.cc:131-135
int oracle_frame_take_data(int N, const ldso_ba_frame_state *frames, double *prior, double *delta,
                           double *delta_prior) {
    for (int f = 0; f < N; f++) {
        const ldso_ba_frame_state &F = frames[f];
        double p[10];
        std::memset(p, 0, sizeof(p));
        if (F.is_first_frame) {
            for (int i = 0; i < 3; i++) p[i] = setting_initialTransPrior;
            for (int i = 3; i < 6; i++) p[i] = setting_initialRotPrior;
            p[6] = setting_initialAffAPrior;
            p[7] = setting_initialAffBPrior;
        } else {
            p[6] = setting_affineOptModeA < 0 ? setting_initialAffAPrior : setting_affineOptModeA;
            p[7] = setting_affineOptModeB < 0 ? setting_initialAffBPrior : setting_affineOptModeB;
        }
        for (int i = 0; i < 8; i++) prior[f * 8 + i] = p[i];
        double mz[6], z[6];
        for (int i = 0; i < 6; i++) {
            mz[i] = -F.state_zero[i];
            z[i] = F.state[i];
        }
        double lg[6];
        se3_log(se3_mul(se3_exp(mz), se3_exp(z)), lg);
        for (int i = 0; i < 8; i++) delta[f * 8 + i] = i < 6 ? lg[i] : F.state[i] - F.state_zero[i];
        se3_log(se3_exp(z), lg);  // getPriorZero() == 0
        for (int i = 0; i < 8; i++) delta_prior[f * 8 + i] = i < 6 ? lg[i] : F.state[i];
    }
    return 0;
}

// FrameHessian::setStateZero (FrameHessian.cc:26-57) + FullSystem::getNullspaces
// (FullSystem.cc:2027-2076); orthogonalize() stacks pose (6) then scale (1).
int oracle_nullspaces(int N, const ldso_ba_frame_state *frames, double *out) {
    const int n = 8 * N + CPARS;
    std::memset(out, 0, sizeof(double) * 7 * n);
    for (int f = 0; f < N; f++) {
        SE3d E = frame_evalpt(frames[f]), Ei = se3_inv(E);
        for (int i = 0; i < 6; i++) {
            double eps[6] = {0, 0, 0, 0, 0, 0}, meps[6];
            eps[i] = 1e-3;
            for (int k = 0; k < 6; k++) meps[k] = -eps[k];
            double lp[6], lm[6];
            se3_log(se3_mul(se3_mul(E, se3_exp(eps)), Ei), lp);
            se3_log(se3_mul(se3_mul(E, se3_exp(meps)), Ei), lm);
            for (int k = 0; k < 6; k++) {
                double v = (lp[k] - lm[k]) / (2e-3);
                v *= (k < 3) ? (double)SCALE_XI_TRANS_INVERSE : (double)SCALE_XI_ROT_INVERSE;
                out[(size_t)i * n + CPARS + 8 * f + k] = v;
            }
        }
        SE3d P = E, M = E;
        for (int k = 0; k < 3; k++) {
            P.t[k] *= 1.00001;
            M.t[k] /= 1.00001;
        }
        double lp[6], lm[6];
        se3_log(se3_mul(P, Ei), lp);
        se3_log(se3_mul(M, Ei), lm);
        for (int k = 0; k < 6; k++) {
            double v = (lp[k] - lm[k]) / (2e-3);
            v *= (k < 3) ? (double)SCALE_XI_TRANS_INVERSE : (double)SCALE_XI_ROT_INVERSE;
            out[(size_t)6 * n + CPARS + 8 * f + k] = v;
        }
    }
    (void)SCALE_A_INVERSE;
    (void)SCALE_B_INVERSE;
    return 0;
}

// FullSystem::doStepFromBackup (FullSystem.cc:1826-1931), the branch without SOLVER_MOMENTUM
// (:1868-1912) with every step factor 1 (optimize() passes stepsize = 1 unless
// SOLVER_STEPMOMENTUM), on the visual-only path (the inertial x_step / x_backup stay zero, so
// sumI = sumIH = 0).  The steps are those resubstituteF_MT leaves (EnergyFunctional.cc:611-622):
// HCalib->step = -x.head<4>(), fh->step.head<8>() = -x.segment<8>(4 + 8 idx), tail 0; the point
// steps come from the caller (oracle_resubstitute).  Float sums exactly as written: sumA etc. are
// float accumulators fed double products (float += double), sumNID a float sum of fabsf over the
// window's active points in frames -> features order (here: host frames in window order, each
// host's points in the window's point order).  Returns canbreak (0 / 1).
int oracle_do_step_from_backup(int N, const ldso_ba_frame_state *backup, const double *x, double *calib_value,
                               const double *calib_value_zero, int n_points, const int *point_host,
                               const float *idepth_backup, const float *point_step, float th_opt_iterations,
                               ldso_ba_frame_state *out, float *idepth_out, float *calib_scaled_out,
                               float *c_delta_out) {
    if (N < 1 || !backup || !x || !calib_value || !out || n_points < 0 ||
        (n_points > 0 && (!point_host || !idepth_backup || !point_step || !idepth_out)))
        return -1;
    const float stepfacC = 1, stepfacT = 1, stepfacR = 1, stepfacA = 1, stepfacD = 1;
    double pstepfac[10];
    for (int i = 0; i < 3; i++) pstepfac[i] = stepfacT;
    for (int i = 3; i < 6; i++) pstepfac[i] = stepfacR;
    for (int i = 6; i < 10; i++) pstepfac[i] = stepfacA;
    float sumA = 0, sumB = 0, sumT = 0, sumR = 0, sumID = 0, numID = 0;
    float sumNID = 0;
    double sumI = 0, sumIH = 0;
    // Hcalib->mpCH->setValue(value_backup + stepfacC * step)  (CalibHessian.h:71-85)
    for (int k = 0; k < CPARS; k++) calib_value[k] = calib_value[k] + stepfacC * (-x[k]);
    if (calib_scaled_out)
        for (int k = 0; k < CPARS; k++) calib_scaled_out[k] = (float)((k < 2 ? SCALE_F : SCALE_C) * calib_value[k]);
    if (c_delta_out && calib_value_zero)
        for (int k = 0; k < CPARS; k++) c_delta_out[k] = (float)(calib_value[k] - calib_value_zero[k]);
    for (int f = 0; f < N; f++) {
        const ldso_ba_frame_state &B = backup[f];
        double step[10];
        for (int i = 0; i < 10; i++) step[i] = i < 8 ? -x[CPARS + 8 * f + i] : 0.0;
        ldso_ba_frame_state &O = out[f];
        O = B;
        // Vec10 step = state_backup + pstepfac .* step; head<6> = log(exp(pstepfac .* step) exp(state_backup))
        double a[6], bk[6], lg[6];
        for (int i = 0; i < 6; i++) {
            a[i] = pstepfac[i] * step[i];
            bk[i] = B.state[i];
        }
        se3_log(se3_mul(se3_exp(a), se3_exp(bk)), lg);
        for (int i = 0; i < 10; i++) O.state[i] = i < 6 ? lg[i] : B.state[i] + pstepfac[i] * step[i];
        sumA += step[6] * step[6];
        sumB += step[7] * step[7];
        sumT += (step[0] * step[0] + step[1] * step[1]) + step[2] * step[2];
        sumR += (step[3] * step[3] + step[4] * step[4]) + step[5] * step[5];
        for (int p = 0; p < n_points; p++) {
            if (point_host[p] != f) continue;
            const float ib = idepth_backup[p], st = point_step[p];
            idepth_out[p] = ib + stepfacD * st;  // setIdepth / setIdepthZero (the same value)
            sumID += st * st;
            sumNID += fabsf(ib);
            numID++;
        }
    }
    sumA /= N;
    sumB /= N;
    sumR /= N;
    sumT /= N;
    sumID /= numID;
    sumNID /= numID;
    sumI /= N;
    const double th = th_opt_iterations;
    return sqrtf(sumA) < 0.0005 * th && sqrtf(sumB) < 0.00005 * th && sqrtf(sumR) < 0.00005 * th &&
           sqrtf(sumT) * sumNID < 0.00005 * th && std::sqrt(sumI) < 0.00005 * th && std::sqrt(sumIH) < 0.00005 * th;
}

// ---- point marginalisation --------------------------------------
// FullSystem::flagPointsForRemoval's per-residual part for the MARGINALIZED points
// (FullSystem.cc:1390-1398) with PointFrameResidual::fixLinearizationF (Residuals.cc:219-245;
// the Eigen dot products taken left to right), then EnergyFunctional::marginalizePointsF
// (EnergyFunctional.cc:205-243): priorF *= setting_idepthFixPriorMargFac, addPoint<2>,
// SC addPoint(p, false), single-threaded stitchDouble of both; H = M - Msc, b = Mb - Mbsc.
int oracle_marginalize_points(oracle_window *ow, int n, const int *pts, const float *adHTdeltaF, double *H,
                              double *b) {
    if (!ow || n < 0 || (n > 0 && !pts) || !adHTdeltaF || !H || !b) return -1;
    const int N = ow->N, D = dimH(N);
    for (int k = 0; k < n; k++)
        if (pts[k] < 0 || pts[k] >= (int)ow->points.size()) return -1;
    for (int k = 0; k < n; k++) {
        PointH &p = ow->points[pts[k]];
        for (int ri : p.residuals) {
            Residual &r = ow->res[ri];
            r.resetOOB();
            linearize(ow, r);
            r.isLinearized = false;
            r.applyRes(true);
            if (!r.isActive()) continue;
            // fixLinearizationF
            const RawResidualJacobian &J = r.J;
            const float *dp = adHTdeltaF + (size_t)(r.hostIDX + N * r.targetIDX) * 8;
            float x6 = 0, y6 = 0, x4 = 0, y4 = 0;
            for (int i = 0; i < 6; i++) {
                x6 += J.Jpdxi[0][i] * dp[i];
                y6 += J.Jpdxi[1][i] * dp[i];
            }
            for (int i = 0; i < 4; i++) {
                x4 += J.Jpdc[0][i] * ow->cDeltaF[i];
                y4 += J.Jpdc[1][i] * ow->cDeltaF[i];
            }
            const float Jp_delta_x = x6 + x4 + J.Jpdd[0] * p.deltaF;
            const float Jp_delta_y = y6 + y4 + J.Jpdd[1] * p.deltaF;
            const float delta_a = dp[6], delta_b = dp[7];
            for (int i = 0; i < patternNum; i++) {
                float rtz = J.resF[i];
                rtz = rtz - J.JIdx[0][i] * Jp_delta_x;
                rtz = rtz - J.JIdx[1][i] * Jp_delta_y;
                rtz = rtz - J.JabF[0][i] * delta_a;
                rtz = rtz - J.JabF[1][i] * delta_b;
                r.res_toZeroF[i] = rtz;
            }
            r.isLinearized = true;
        }
    }
    ensure_pool(ow);
    for (int k = 0; k < n; k++) ow->points[pts[k]].priorF *= 600.0f * 600.0f;  // setting_idepthFixPriorMargFac
    for (auto &a : ow->accTop[0]) a.initialize();
    ow->nres[0] = 0;
    ow->accHcc[0].initialize();
    ow->accbc[0].initialize();
    for (auto &a : ow->accE[0]) a.initialize();
    for (auto &a : ow->accEB[0]) a.initialize();
    for (auto &a : ow->accD[0]) a.initialize();
    for (int k = 0; k < n; k++) {
        topAddPoint<2>(ow, ow->points[pts[k]], 0);
        scAddPoint(ow, ow->points[pts[k]], false, 0);
    }
    std::vector<double> M, Mb, Msc, Mbsc;
    topStitchMT(ow, M, Mb, false, false);
    scStitchMT(ow, Msc, Mbsc, false);
    for (size_t i = 0; i < (size_t)D * D; i++) H[i] = M[i] - Msc[i];
    for (int i = 0; i < D; i++) b[i] = Mb[i] - Mbsc[i];
    return 0;
}

double oracle_time_iterations(oracle_window *ow, int iters) {
    ensure_pool(ow);
    auto t0 = std::chrono::steady_clock::now();
    double e[3];
    for (int i = 0; i < iters; i++) oracle_iteration(ow, e);
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}


// ---- point activation ------------------------------------------------
// ImmaturePoint::linearizeResidual (ImmaturePoint.cc:319-389) with projectPoint / derive_idepth
// (ResidualProjections.h:12-18, 57-84), inside FullSystem::optimizeImmaturePoint
// (FullSystem.cc:1035-1156): residuals to every other frame in window order.
namespace {
struct IpTmpRes {  // ImmaturePointTemporaryResidual (ImmaturePoint.h:18-26)
    int state_state;
    double state_energy;
    int state_NewState;
    double state_NewEnergy;
    int target;
};
double ip_linearize_residual(const oracle_window *ow, const ldso_ct_immature &ip, int host, float outlierTHSlack,
                             IpTmpRes &r, float &Hdd, float &bd, float idepth) {
    if (r.state_state == OOB) {
        r.state_NewState = OOB;
        return r.state_energy;
    }
    const int N = ow->N;
    const float *pre = ow->precalc.data() + (size_t)(host + N * r.target) * LDSO_BA_PRECALC_STRIDE;
    const float *R = pre + 27, *t = pre + 36;  // PRE_RTll, PRE_tTll (current poses, ImmaturePoint.cc:336-337)
    const float aff0 = pre[24], aff1 = pre[25];  // PRE_aff_mode
    const float *dIl = ow->dI.data() + (size_t)r.target * ow->w * ow->h * 3;
    float energyLeft = 0;
    for (int idx = 0; idx < patternNum; idx++) {
        const int dx = patternP[idx][0], dy = patternP[idx][1];
        const float K0 = (ip.u + dx - ow->cxl()) * ow->fxli(), K1 = (ip.v + dy - ow->cyl()) * ow->fyli();
        float ptp[3];
        for (int i = 0; i < 3; i++) ptp[i] = (R[3 * i] * K0 + R[3 * i + 1] * K1 + R[3 * i + 2] * 1.0f) + t[i] * idepth;
        const float drescale = 1.0f / ptp[2];
        if (!(drescale > 0)) {
            r.state_NewState = OOB;
            return r.state_energy;
        }
        const float u = ptp[0] * drescale, v = ptp[1] * drescale;
        const float Ku = u * ow->fxl() + ow->cxl(), Kv = v * ow->fyl() + ow->cyl();
        if (!(Ku > 1.1f && Kv > 1.1f && Ku < ow->wM3G && Kv < ow->hM3G)) {
            r.state_NewState = OOB;
            return r.state_energy;
        }
        float hitColor[3];
        interp33(dIl, Ku, Kv, ow->w, hitColor);
        if (!std::isfinite(hitColor[0])) {
            r.state_NewState = OOB;
            return r.state_energy;
        }
        const float residual = hitColor[0] - (aff0 * ip.color[idx] + aff1);
        float hw = std::fabs(residual) < setting_huberTH ? 1 : setting_huberTH / std::fabs(residual);
        energyLeft += ip.weights[idx] * ip.weights[idx] * hw * residual * residual * (2 - hw);
        const float dxInterp = hitColor[1] * ow->fxl();
        const float dyInterp = hitColor[2] * ow->fyl();
        const float d_idepth = (dxInterp * drescale * (t[0] - t[2] * u) + dyInterp * drescale * (t[1] - t[2] * v)) * 1.0f;
        hw *= ip.weights[idx] * ip.weights[idx];
        Hdd += (hw * d_idepth) * d_idepth;
        bd += (hw * residual) * d_idepth;
    }
    if (energyLeft > ip.energy_th * outlierTHSlack) {
        energyLeft = ip.energy_th * outlierTHSlack;
        r.state_NewState = OUTLIER;
    } else {
        r.state_NewState = IN;
    }
    r.state_NewEnergy = energyLeft;
    return energyLeft;
}
}  // namespace

int oracle_activate_points(oracle_window *ow, int n, const ldso_ct_immature *pts, int min_obs,
                           ldso_ba_activation *out) {
    constexpr float setting_minIdepthH_act = 100;    // Setting.cc:25
    constexpr int setting_GNItsOnPointActivation = 3;  // Setting.cc:47
    const int N = ow->N;
    for (int k = 0; k < n; k++) {
        const ldso_ct_immature &ip = pts[k];
        ldso_ba_activation &o = out[k];
        const int host = ip.host;
        if (host < 0 || host >= N) return -1;
        IpTmpRes res[LDSO_BA_MAX_FRAMES];
        int nres = 0;
        for (int f = 0; f < N; f++)
            if (f != host) res[nres++] = IpTmpRes{IN, 0.0, OUTLIER, 0.0, f};
        float lastEnergy = 0, lastHdd = 0, lastbd = 0;
        float currentIdepth = (ip.idepth_max + ip.idepth_min) * 0.5f;
        o.status = 0;
        o.in_mask = 0;
        for (int i = 0; i < nres; i++) {
            lastEnergy += ip_linearize_residual(ow, ip, host, 1000, res[i], lastHdd, lastbd, currentIdepth);
            res[i].state_state = res[i].state_NewState;
            res[i].state_energy = res[i].state_NewEnergy;
        }
        o.energy = lastEnergy;
        o.idepth = currentIdepth;
        if (!std::isfinite(lastEnergy) || lastHdd < setting_minIdepthH_act) {
            o.status = 2;
            continue;
        }
        float lambda = 0.1f;
        bool zero = false;
        for (int iteration = 0; iteration < setting_GNItsOnPointActivation; iteration++) {
            float H = lastHdd;
            H *= 1 + lambda;
            const float step = (1.0 / H) * lastbd;
            const float newIdepth = currentIdepth - step;
            float newHdd = 0, newbd = 0, newEnergy = 0;
            for (int i = 0; i < nres; i++)
                newEnergy += ip_linearize_residual(ow, ip, host, 1, res[i], newHdd, newbd, newIdepth);
            if (!std::isfinite(lastEnergy) || newHdd < setting_minIdepthH_act) {
                zero = true;
                break;
            }
            if (newEnergy < lastEnergy) {
                currentIdepth = newIdepth;
                lastHdd = newHdd;
                lastbd = newbd;
                lastEnergy = newEnergy;
                for (int i = 0; i < nres; i++) {
                    res[i].state_state = res[i].state_NewState;
                    res[i].state_energy = res[i].state_NewEnergy;
                }
                lambda *= 0.5;
            } else {
                lambda *= 5;
            }
            if (std::fabs(step) < 0.0001 * currentIdepth) break;
        }
        o.energy = lastEnergy;
        o.idepth = currentIdepth;
        if (zero) {
            o.status = 2;
            continue;
        }
        if (!std::isfinite(currentIdepth)) {
            o.status = 1;
            continue;
        }
        int numGoodRes = 0;
        for (int i = 0; i < nres; i++)
            if (res[i].state_state == IN) {
                numGoodRes++;
                o.in_mask |= 1u << res[i].target;
            }
        if (numGoodRes < min_obs) {
            o.status = 1;
            o.in_mask = 0;
        }
    }
    return 0;
}

// EnergyFunctional::setDeltaF (EnergyFunctional.cc:523-533): adHTdeltaF[h + t N] =
// frames[h]->delta^T (float) * adHostF + frames[t]->delta^T * adTargetF, Mat18f row times Mat88f
// (each output column a k-ascending float dot product).
int oracle_ad_ht_delta(int N, const double *delta, const double *adH, const double *adT, float *out) {
    for (int h = 0; h < N; h++)
        for (int t = 0; t < N; t++) {
            const int idx = h + t * N;
            for (int j = 0; j < 8; j++) {
                float lh = 0.f, lt = 0.f;
                for (int k = 0; k < 8; k++) lh += (float)delta[8 * h + k] * (float)adH[(size_t)idx * 64 + k * 8 + j];
                for (int k = 0; k < 8; k++) lt += (float)delta[8 * t + k] * (float)adT[(size_t)idx * 64 + k * 8 + j];
                out[(size_t)idx * 8 + j] = lh + lt;
            }
        }
    return 0;
}

// EnergyFunctional::calcMEnergyF (EnergyFunctional.cc:473-479): delta.dot(2 * bM + HM * delta),
// delta = getStitchedDeltaF() (EnergyFunctional.h:192-198: cDeltaF then each frame's delta).
double oracle_calc_m_energy(int N, const double *HM, const double *bM, const float *cDeltaF, const double *delta) {
    const int n = 8 * N + 4;
    std::vector<double> d(n), Hd(n, 0.0);
    for (int i = 0; i < 4; i++) d[i] = (double)cDeltaF[i];
    for (int f = 0; f < N; f++)
        for (int k = 0; k < 8; k++) d[4 + 8 * f + k] = delta[8 * f + k];
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++) Hd[r] += HM[(size_t)r * n + c] * d[c];
    double e = 0.0;
    for (int r = 0; r < n; r++) e += d[r] * (2 * bM[r] + Hd[r]);
    return e;
}

// EnergyFunctional::calcLEnergyF_MT (EnergyFunctional.cc:481-498) with calcLEnergyPt (:751-806)
// over IndexThreadReduce chunks of 50 points (red->reduce(..., 50)), one Accumulator11
// (MatrixAccumulators.h:68-123) per chunk, chunk totals summed into stats[0] in order.  Only the
// per-point prior term: no residual of an optimised window is linearised (see ldso_ba.h).
double oracle_calc_l_energy(int N, const double *prior, const double *delta_prior, const double *cPrior,
                            const float *cDeltaF, int n_points, const float *deltaF, const float *priorF) {
    double E = 0;
    for (int f = 0; f < N; f++) {
        double dot = 0;
        for (int k = 0; k < 8; k++) dot += (delta_prior[8 * f + k] * prior[8 * f + k]) * delta_prior[8 * f + k];
        E += dot;
    }
    float cdot = 0.f;
    for (int k = 0; k < 4; k++) cdot += (cDeltaF[k] * (float)cPrior[k]) * cDeltaF[k];
    E += cdot;
    double stat0 = 0;
    for (int lo = 0; lo < n_points; lo += 50) {
        float sse[4] = {0, 0, 0, 0}, sse1k[4] = {0, 0, 0, 0}, sse1m[4] = {0, 0, 0, 0};
        const int hi = std::min(n_points, lo + 50);
        for (int q = lo; q < hi; q++) sse[0] += deltaF[q] * deltaF[q] * priorF[q];  // updateSingle
        for (int k = 0; k < 4; k++) sse1k[k] += sse[k];                           // finish(): shiftUp(true)
        for (int k = 0; k < 4; k++) sse1m[k] += sse1k[k];
        stat0 += sse1m[0] + sse1m[1] + sse1m[2] + sse1m[3];
    }
    return E + stat0;
}

}  // extern "C"
