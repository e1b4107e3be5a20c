// energy_functional.cpp -- the C++ host face (include/ldso_amd/energy_functional.h) packed onto
// the C ABI of include/ldso_ba.h.  Packing only: every number is computed by the HIP path or by
// the library's host helpers (precalc, adjoints, priors, nullspaces, solve).
#include "../../include/ldso_amd/energy_functional.h"

#include <algorithm>
#include <cstring>

namespace ldso_amd {

EnergyFunctional::EnergyFunctional(int device) {
    if (ldso_ba_create(device, &ctx_) != 0) {
        ctx_ = nullptr;
        fail("ldso_ba_create");
    }
}

EnergyFunctional::~EnergyFunctional() {
    if (ctx_) ldso_ba_destroy(ctx_);
}

void EnergyFunctional::fail(const char *what) {
    err_ = std::string(what) + ": " + ldso_ba_last_error();
}

void EnergyFunctional::setCalib(const CalibHessian &Hcalib) {
    calib_ = Hcalib;
    width_ = Hcalib.wG0;
    height_ = Hcalib.hG0;
}

void EnergyFunctional::insertFrame(FrameHessian *fh, const CalibHessian &Hcalib) {
    setCalib(Hcalib);
    fh->idx = (int)frames.size();
    frames.push_back(fh);
    nFrames = (int)frames.size();
    dirty_ = true;
}

void EnergyFunctional::insertPoint(PointHessian *ph) {
    allPoints.push_back(ph);
    nPoints = (int)allPoints.size();
    dirty_ = true;
}

void EnergyFunctional::insertResidual(PointFrameResidual *r) {
    r->point->residuals.push_back(r);
    nResiduals++;
    dirty_ = true;
}

void EnergyFunctional::dropResidual(PointFrameResidual *r) {
    auto &v = r->point->residuals;
    auto it = std::find(v.begin(), v.end(), r);
    if (it != v.end()) {
        v.erase(it);
        nResiduals--;
        dirty_ = true;
    }
}

void EnergyFunctional::removePoint(PointHessian *p) {
    auto it = std::find(allPoints.begin(), allPoints.end(), p);
    if (it != allPoints.end()) {
        nResiduals -= (int)p->residuals.size();
        allPoints.erase(it);
        nPoints = (int)allPoints.size();
        dirty_ = true;
    }
}

// EnergyFunctional::makeIDX (EnergyFunctional.cc:500-521): frame indices, points in host-frame order
void EnergyFunctional::makeIDX() {
    for (size_t i = 0; i < frames.size(); i++) frames[i]->idx = (int)i;
    std::stable_sort(allPoints.begin(), allPoints.end(),
                     [](const PointHessian *a, const PointHessian *b) { return a->host->idx < b->host->idx; });
    for (size_t i = 0; i < allPoints.size(); i++) allPoints[i]->idxInPoints = (int)i;
    dirty_ = true;
}

bool EnergyFunctional::upload() {
    if (!ctx_) return false;
    const int N = nFrames;
    if (N < 2) {
        err_ = "need at least two frames";
        return false;
    }
    // frame-level terms from the current states (setPrecalcValues, setAdjointsF, takeData)
    fs_.resize(N);
    for (int f = 0; f < N; f++) {
        const FrameHessian &F = *frames[f];
        ldso_ba_frame_state &S = fs_[f];
        std::memset(&S, 0, sizeof(S));
        std::memcpy(S.world_to_cam_evalpt, F.worldToCam_evalPT, sizeof(S.world_to_cam_evalpt));
        std::memcpy(S.state, F.state, sizeof(S.state));
        std::memcpy(S.state_zero, F.state_zero, sizeof(S.state_zero));
        S.ab_exposure = F.ab_exposure;
        S.is_first_frame = F.isFirstFrame ? 1 : 0;
    }
    precalc_.assign((size_t)N * N * LDSO_BA_PRECALC_STRIDE, 0.f);
    adH_.assign((size_t)N * N * 64, 0.0);
    adT_.assign((size_t)N * N * 64, 0.0);
    cPrior_.assign(4, 0.0);
    fPrior_.assign((size_t)N * 8, 0.0);
    fDelta_.assign((size_t)N * 8, 0.0);
    fDeltaPrior_.assign((size_t)N * 8, 0.0);
    cDelta_.assign(calib_.value_minus_value_zero, calib_.value_minus_value_zero + 4);
    if (ldso_ba_frame_precalc(N, fs_.data(), calib_.value_scaledf, precalc_.data()) ||
        ldso_ba_set_adjoints(N, fs_.data(), adH_.data(), adT_.data(), cPrior_.data()) ||
        ldso_ba_frame_take_data(N, fs_.data(), fPrior_.data(), fDelta_.data(), fDeltaPrior_.data())) {
        fail("frame terms");
        return false;
    }
    frameTH_.resize(N);
    for (int f = 0; f < N; f++) frameTH_[f] = frames[f]->frameEnergyTH;
    // points and residuals in makeIDX order
    const int P = nPoints;
    pointHost_.resize(P);
    pointData_.assign((size_t)P * LDSO_BA_POINT_STRIDE, 0.f);
    resBegin_.assign(P + 1, 0);
    resTarget_.clear();
    resState_.clear();
    resEnergy_.clear();
    resFlags_.clear();
    resPtr_.clear();
    for (int q = 0; q < P; q++) {
        const PointHessian &p = *allPoints[q];
        pointHost_[q] = p.host->idx;
        float *d = &pointData_[(size_t)q * LDSO_BA_POINT_STRIDE];
        d[0] = p.u;
        d[1] = p.v;
        d[2] = p.idepth_scaled;
        d[3] = p.idepth_zero_scaled;
        d[4] = p.priorF;
        d[5] = p.deltaF;
        std::memcpy(d + 8, p.color, sizeof(p.color));
        std::memcpy(d + 16, p.weights, sizeof(p.weights));
        for (PointFrameResidual *r : p.residuals) {
            resTarget_.push_back(r->target->idx);
            resState_.push_back((int8_t)r->state_state);
            resEnergy_.push_back(r->state_energy);
            resFlags_.push_back((uint8_t)((r->isActiveAndIsGoodNEW ? LDSO_BA_FLAG_ACTIVE : 0u) |
                                          (r->isNew ? LDSO_BA_FLAG_NEW : 0u)));
            resPtr_.push_back(r);
        }
        resBegin_[q + 1] = (int32_t)resTarget_.size();
    }
    nResiduals = (int)resPtr_.size();
    ldso_ba_window w;
    std::memset(&w, 0, sizeof(w));
    w.n_frames = N;
    w.n_points = P;
    w.n_residuals = nResiduals;
    w.width = width_;
    w.height = height_;
    std::memcpy(w.calib, calib_.value_scaledf, sizeof(w.calib));
    if (dirty_) {  // images are only uploaded on a structural change
        dI_.resize((size_t)N * width_ * height_ * 3);
        for (int f = 0; f < N; f++)
            std::memcpy(&dI_[(size_t)f * width_ * height_ * 3], frames[f]->dI,
                        (size_t)width_ * height_ * 3 * sizeof(float));
    }
    w.dI = dI_.data();
    w.frame_energy_th = frameTH_.data();
    w.precalc = precalc_.data();
    w.ad_host = adH_.data();
    w.ad_target = adT_.data();
    w.c_prior = cPrior_.data();
    w.c_delta = cDelta_.data();
    w.frame_prior = fPrior_.data();
    w.frame_delta_prior = fDeltaPrior_.data();
    w.point_host = pointHost_.data();
    w.point_data = pointData_.data();
    w.point_res_begin = resBegin_.data();
    w.res_target = resTarget_.data();
    w.res_state = resState_.data();
    w.res_energy = resEnergy_.data();
    w.res_flags = resFlags_.data();
    const int rc = dirty_ ? ldso_ba_load(ctx_, 1, &w, 0, 1) : ldso_ba_update(ctx_, 0, &w);
    if (rc) {
        fail(dirty_ ? "ldso_ba_load" : "ldso_ba_update");
        return false;
    }
    dirty_ = false;
    return true;
}

void EnergyFunctional::resetOOB() {
    for (PointHessian *p : allPoints)
        for (PointFrameResidual *r : p->residuals) {  // Residuals.h:63-68
            r->state_NewEnergy = r->state_energy = 0;
            r->state_NewState = OUTLIER;
            r->state_state = IN;
        }
    if (!dirty_ && ctx_ && ldso_ba_reset_oob(ctx_, 0)) fail("ldso_ba_reset_oob");
}

Vec3 EnergyFunctional::linearizeAll(bool fixLinearization) {
    Vec3 out = {0, 0, 0};
    if (!upload()) return out;
    if (ldso_ba_linearize(ctx_, fixLinearization ? 1 : 0, fixLinearization ? 0 : 1)) {
        fail("ldso_ba_linearize");
        return out;
    }
    double e[3];
    if (ldso_ba_get_energy(ctx_, 0, e)) {
        fail("ldso_ba_get_energy");
        return out;
    }
    const int R = nResiduals, P = nPoints, N = nFrames;
    std::vector<int8_t> ns(R), st(R);
    std::vector<float> se(R), ewo(R), ctr((size_t)3 * R), jp((size_t)8 * R), rb(R);
    std::vector<uint8_t> fl(R);
    if (R && ldso_ba_get_residuals(ctx_, 0, ns.data(), st.data(), se.data(), ewo.data(), ctr.data(), fl.data(),
                                   jp.data(), rb.data())) {
        fail("ldso_ba_get_residuals");
        return out;
    }
    for (int k = 0; k < R; k++) {
        PointFrameResidual &r = *resPtr_[k];
        r.state_NewState = (ResState)ns[k];
        r.state_state = (ResState)st[k];
        r.state_energy = se[k];
        r.state_NewEnergy = se[k];
        r.state_NewEnergyWithOutlier = ewo[k];
        std::memcpy(r.centerProjectedTo, &ctr[(size_t)3 * k], 3 * sizeof(float));
        r.isActiveAndIsGoodNEW = (fl[k] & LDSO_BA_FLAG_ACTIVE) != 0;
        if (r.isActiveAndIsGoodNEW) std::memcpy(r.JpJdF, &jp[(size_t)8 * k], 8 * sizeof(float));
        r.relBS = rb[k];
    }
    std::vector<float> hdi(P), bds(P), ih(P), th(N);
    if (P && ldso_ba_get_points(ctx_, 0, hdi.data(), bds.data(), ih.data(), nullptr, nullptr, nullptr)) {
        fail("ldso_ba_get_points");
        return out;
    }
    for (int q = 0; q < P; q++) {
        allPoints[q]->HdiF = hdi[q];
        allPoints[q]->bdSumF = bds[q];
        allPoints[q]->idepth_hessian = ih[q];
    }
    if (ldso_ba_get_frame_energy_th(ctx_, 0, th.data()) == 0)
        for (int f = 0; f < N; f++) frames[f]->frameEnergyTH = th[f];
    out = {e[0], e[1], e[2]};
    return out;
}

void EnergyFunctional::solveSystemF(int iteration, double lambda) {
    const int n = 8 * nFrames + 4;
    HA_top.assign((size_t)n * n, 0.0);
    bA_top.assign(n, 0.0);
    HL_top.assign((size_t)n * n, 0.0);
    bL_top.assign(n, 0.0);
    H_sc.assign((size_t)n * n, 0.0);
    b_sc.assign(n, 0.0);
    if (ldso_ba_get_system(ctx_, 0, HA_top.data(), bA_top.data(), HL_top.data(), bL_top.data(), H_sc.data(),
                           b_sc.data())) {
        fail("ldso_ba_get_system");
        return;
    }
    std::vector<double> ns((size_t)7 * n);
    if (ldso_ba_nullspaces(nFrames, fs_.data(), ns.data())) {
        fail("ldso_ba_nullspaces");
        return;
    }
    lastX.assign(n, 0.0);
    if (ldso_ba_solve(ctx_, 0, iteration, lambda, ns.data(), 7, lastX.data())) fail("ldso_ba_solve");
}

void EnergyFunctional::resubstituteF_MT(const std::vector<double> &x, double lambda) {
    std::vector<float> step(nPoints);
    if (ldso_ba_resubstitute(ctx_, 0, x.data(), lambda, step.data())) {
        fail("ldso_ba_resubstitute");
        return;
    }
    for (int q = 0; q < nPoints; q++) allPoints[q]->step = step[q];
}

}  // namespace ldso_amd
