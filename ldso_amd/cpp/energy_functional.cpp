// energy_functional.cpp -- the C++ host face (include/ldso_amd/energy_functional.h) on the C ABI
// of include/ldso_ba.h.  Packing and bookkeeping only: every number is computed by the HIP path
// or by the library's host helpers (precalc, adjoints, priors, deltas, energies, nullspaces,
// solve, frame marginalisation).
#include "../../include/ldso_amd/energy_functional.h"

#include <algorithm>
#include <cstring>

namespace ldso_amd {

namespace {

constexpr float kIdepthFixPriorMargFac = 600.0f * 600.0f;  // setting_idepthFixPriorMargFac (Setting.cc:17)
constexpr double kMargWeightFac = 0.5 * 0.5;                // setting_margWeightFac (Setting.cc:45)

uint64_t conn_key(const PointFrameResidual &r) {
    return ((uint64_t)r.host.lock()->frameID << 32) + (uint64_t)r.target.lock()->frameID;
}

void frame_state(const FrameHessian &F, ldso_ba_frame_state &S) {
    std::memset(&S, 0, sizeof(S));
    std::memcpy(S.world_to_cam_evalpt, F.worldToCam_evalPT, sizeof(S.world_to_cam_evalpt));
    std::memcpy(S.state, F.state, sizeof(S.state));
    std::memcpy(S.state_zero, F.state_zero, sizeof(S.state_zero));
    S.ab_exposure = F.ab_exposure;
    S.is_first_frame = F.frameID == 0 ? 1 : 0;
}

// points + residuals of one ldso_ba_window (caller point order = the order given)
struct PointPack {
    std::vector<int32_t> host, begin, target, rank;
    bool ranked = true;  // every point carries its featureRank
    std::vector<float> data, energy;
    std::vector<int8_t> state;
    std::vector<uint8_t> flags;
    std::vector<PointFrameResidual *> res;
    void build(const std::vector<PointHessian *> &pts) {
        host.assign(pts.size(), 0);
        rank.assign(pts.size(), 0);
        ranked = true;
        data.assign(pts.size() * LDSO_BA_POINT_STRIDE, 0.f);
        begin.assign(pts.size() + 1, 0);
        target.clear();
        energy.clear();
        state.clear();
        flags.clear();
        res.clear();
        for (size_t q = 0; q < pts.size(); q++) {
            const PointHessian &p = *pts[q];
            host[q] = p.host.lock()->idx;
            rank[q] = p.featureRank;
            ranked = ranked && p.featureRank >= 0;
            float *d = &data[q * LDSO_BA_POINT_STRIDE];
            d[0] = p.u;
            d[1] = p.v;
            d[2] = p.idepth_scaled;
            d[3] = p.idepth_zero_scaled;
            d[4] = p.priorF;
            d[5] = p.deltaF;
            std::memcpy(d + 8, p.color, sizeof(p.color));
            std::memcpy(d + 16, p.weights, sizeof(p.weights));
            for (const shared_ptr<PointFrameResidual> &r : p.residuals) {
                target.push_back(r->target.lock()->idx);
                state.push_back((int8_t)r->state_state);
                energy.push_back((float)r->state_energy);
                flags.push_back((uint8_t)((r->isActiveAndIsGoodNEW ? LDSO_BA_FLAG_ACTIVE : 0u) |
                                          (r->isNew ? LDSO_BA_FLAG_NEW : 0u)));
                res.push_back(r.get());
            }
            begin[q + 1] = (int32_t)target.size();
        }
    }
    void into(ldso_ba_window &w) {
        w.n_points = (int32_t)host.size();
        w.n_residuals = (int32_t)target.size();
        w.point_host = host.data();
        w.point_data = data.data();
        w.point_res_begin = begin.data();
        w.res_target = target.data();
        w.res_state = state.data();
        w.res_energy = energy.data();
        w.res_flags = flags.data();
        w.point_rank = ranked ? rank.data() : nullptr;
    }
};

// write a device pass's per-residual results back into the residual objects
bool read_residuals(ldso_ba_ctx *ctx, const std::vector<PointFrameResidual *> &res) {
    const size_t R = res.size();
    if (!R) return true;
    std::vector<int8_t> ns(R), st(R);
    std::vector<float> se(R), ewo(R), ctr(3 * R), jp(8 * R), rb(R);
    std::vector<uint8_t> fl(R);
    if (ldso_ba_get_residuals(ctx, 0, ns.data(), st.data(), se.data(), ewo.data(), ctr.data(), fl.data(), jp.data(),
                              rb.data()))
        return false;
    for (size_t k = 0; k < R; k++) {
        PointFrameResidual &r = *res[k];
        r.state_NewState = (ResState)ns[k];
        r.state_state = (ResState)st[k];
        r.state_energy = se[k];
        r.state_NewEnergy = se[k];
        r.state_NewEnergyWithOutlier = ewo[k];
        std::memcpy(r.centerProjectedTo, &ctr[3 * k], 3 * sizeof(float));
        r.isActiveAndIsGoodNEW = (fl[k] & LDSO_BA_FLAG_ACTIVE) != 0;
        if (r.isActiveAndIsGoodNEW) {
            std::memcpy(r.JpJdF, &jp[8 * k], 8 * sizeof(float));
            std::memcpy(r.J_JpJdF, &jp[8 * k], 8 * sizeof(float));
        }
        r.relBS = rb[k];
    }
    return true;
}

}  // namespace

void FrameHessian::takeData(const ldso_ba_opt_settings *settings) {
    ldso_ba_frame_state S;
    frame_state(*this, S);
    ldso_ba_frame_take_data(1, &S, settings, prior, delta, delta_prior);
}

// Residuals.cc:15-217 (see the header): the OOB early return here, the rest from the window's
// relinearisation pass
double PointFrameResidual::linearize(shared_ptr<CalibHessian> &HCalib) {
    (void)HCalib;  // the window's calibration is its EnergyFunctional's (insertFrame / setAdjointsF)
    if (!ef) return state_energy;
    ef->residualTouched();
    state_NewEnergyWithOutlier = -1;
    if (state_state == OOB) {
        state_NewState = OOB;
        return state_energy;
    }
    return ef->linearizeResidual(*this);
}

// Residuals.h:63-68
void PointFrameResidual::resetOOB() {
    if (ef) ef->residualTouched();
    const bool same = state_NewEnergy == 0 && state_energy == 0 && state_NewState == OUTLIER && state_state == IN;
    state_NewEnergy = state_energy = 0;
    state_NewState = OUTLIER;
    state_state = IN;
    if (ef && !same) ef->residualEdited();
}

// Residuals.h:70-88; takeData (Residuals.h:120-129) is the JpJdF of the last linearisation
void PointFrameResidual::applyRes(bool copyJacobians) {
    if (ef) ef->residualTouched();
    const ResState s0 = state_state;
    const double e0 = state_energy;
    const bool a0 = isActiveAndIsGoodNEW;
    if (copyJacobians) {
        if (state_state == OOB) return;
        if (state_NewState == IN) {
            isActiveAndIsGoodNEW = true;
            std::memcpy(JpJdF, J_JpJdF, sizeof(JpJdF));
        } else {
            isActiveAndIsGoodNEW = false;
        }
    }
    state_state = state_NewState;
    state_energy = state_NewEnergy;
    if (ef && (s0 != state_state || e0 != state_energy || a0 != isActiveAndIsGoodNEW)) ef->residualEdited();
}

void PointFrameResidual::setState(ResState s) {
    if (ef) ef->residualTouched();
    if (ef && s != state_state) ef->residualEdited();
    state_state = s;
}

void PointFrameResidual::fixLinearizationF(shared_ptr<EnergyFunctional> e) {
    (void)e;
    isLinearized = true;
}

EnergyFunctional::EnergyFunctional(int device) : device_(device) {
    if (ldso_ba_create(device, &ctx_) != 0) {
        ctx_ = nullptr;
        fail("ldso_ba_create");
    }
}

EnergyFunctional::~EnergyFunctional() {
    for (const shared_ptr<PointHessian> &p : registry_)
        for (const shared_ptr<PointFrameResidual> &r : p->residuals)
            if (r->ef == this) r->ef = nullptr;
    if (margCtx_) ldso_ba_destroy(margCtx_);
    if (ctx_) ldso_ba_destroy(ctx_);
}

void EnergyFunctional::fail(const char *what) { err_ = std::string(what) + ": " + ldso_ba_last_error(); }

bool EnergyFunctional::setSettings(const ldso_ba_opt_settings &s) {
    if (!ctx_) return false;
    if (ldso_ba_set_settings(ctx_, &s) || (margCtx_ && ldso_ba_set_settings(margCtx_, &s))) {
        fail("ldso_ba_set_settings");
        return false;
    }
    const bool priors_change = s.affine_opt_mode_a != settings_.affine_opt_mode_a ||
                               s.affine_opt_mode_b != settings_.affine_opt_mode_b;
    settings_ = s;
    if (priors_change) {  // takeData's priors follow the affine modes: recompute and re-upload them
        for (const shared_ptr<FrameHessian> &f : frames) f->takeData(&settings_);
        fsUp_.clear();
        epoch_++;
    }
    return true;
}

void EnergyFunctional::packFrames(std::vector<ldso_ba_frame_state> &fs) const {
    fs.resize(frames.size());
    for (size_t f = 0; f < frames.size(); f++) frame_state(*frames[f], fs[f]);
}

// EnergyFunctional.cc:45-49 (the caller has pushed r into its point's residuals)
void EnergyFunctional::insertResidual(shared_ptr<PointFrameResidual> r) {
    residualTouched();  // before any structural change: the mirror's residuals may not outlive it
    r->ef = this;
    r->mirrorIdx = -1;
    connectivityMap[conn_key(*r)][0]++;
    nResiduals++;
    dirty_ = true;
    epoch_++;
}

// EnergyFunctional.cc:51-98 (the non-VI part): HM, bM grow by the frame's 8 zero rows/columns
void EnergyFunctional::insertFrame(shared_ptr<FrameHessian> fh, shared_ptr<CalibHessian> Hcalib) {
    residualTouched();
    fh->takeData(&settings_);
    frames.push_back(fh);
    fh->idx = (int)frames.size();
    nFrames++;
    const int n = 8 * nFrames + CPARS;
    MatXX H2(n, n);
    VecX b2(n);
    for (int i = 0; i < HM.rows(); i++) {
        b2[i] = bM[i];
        for (int j = 0; j < HM.cols(); j++) H2(i, j) = HM(i, j);
    }
    HM = H2;
    bM = b2;
    calib_ = *Hcalib;
    width_ = Hcalib->wG0;
    height_ = Hcalib->hG0;
    setAdjointsF(Hcalib);
    makeIDX();
    for (const shared_ptr<FrameHessian> &fh2 : frames) {
        connectivityMap[((uint64_t)fh->frameID << 32) + (uint64_t)fh2->frameID] = {0, 0};
        if (fh2 != fh) connectivityMap[((uint64_t)fh2->frameID << 32) + (uint64_t)fh->frameID] = {0, 0};
    }
    dirty_ = true;
    epoch_++;
}

void EnergyFunctional::insertPoint(shared_ptr<PointHessian> ph) {
    residualTouched();
    ph->status = PointStatus::ACTIVE;
    ph->alreadyRemoved = false;
    registry_.push_back(ph);
    allPoints.push_back(ph);
    nPoints++;
    dirty_ = true;
    epoch_++;
}

// EnergyFunctional.cc:100-107
void EnergyFunctional::dropResidual(shared_ptr<PointFrameResidual> r) {
    residualTouched();
    shared_ptr<PointHessian> p = r->point.lock();
    if (p) {
        auto &v = p->residuals;
        auto it = std::find(v.begin(), v.end(), r);
        if (it != v.end()) v.erase(it);
    }
    connectivityMap[conn_key(*r)][0]--;
    nResiduals--;
    if (r->ef == this) r->ef = nullptr;
    r->mirrorIdx = -1;
    dirty_ = true;
    epoch_++;
}

// EnergyFunctional.cc:109-191: the dense reorder / prior / Schur step on the host
// (ldso_ba_marginalize_frame), then the frame leaves the window
void EnergyFunctional::marginalizeFrame(shared_ptr<FrameHessian> fh) {
    residualTouched();
    const int no = 8 * nFrames + CPARS, nn = no - 8;
    MatXX Ho(nn, nn);
    VecX bo(nn);
    if (ldso_ba_marginalize_frame(nFrames, fh->idx, HM.data(), bM.data(), fh->prior, fh->delta_prior, Ho.data(),
                                  bo.data())) {
        fail("ldso_ba_marginalize_frame");
        return;
    }
    HM = Ho;
    bM = bo;
    for (size_t i = (size_t)fh->idx; i + 1 < frames.size(); i++) {
        frames[i] = frames[i + 1];
        frames[i]->idx = (int)i;
    }
    frames.pop_back();
    nFrames--;
    makeIDX();
    dirty_ = true;
    epoch_++;
}

// EnergyFunctional.cc:193-203
void EnergyFunctional::removePoint(shared_ptr<PointHessian> ph) {
    residualTouched();
    for (const shared_ptr<PointFrameResidual> &r : ph->residuals) {
        connectivityMap[conn_key(*r)][0]--;
        nResiduals--;
        if (r->ef == this) r->ef = nullptr;
        r->mirrorIdx = -1;
    }
    ph->residuals.clear();
    if (!ph->alreadyRemoved) nPoints--;
    ph->alreadyRemoved = true;
    dirty_ = true;
    epoch_++;
}

// EnergyFunctional.cc:205-262 with FullSystem.cc:1384-1404 (see the header)
void EnergyFunctional::marginalizePointsF() {
    epoch_++;
    residualTouched();
    allPointsToMarg.clear();
    for (const shared_ptr<PointHessian> &p : registry_)
        if (p->status == PointStatus::MARGINALIZED && !p->alreadyRemoved) allPointsToMarg.push_back(p);
    if (allPointsToMarg.empty()) return;
    if (!upload()) return;  // current frame terms; the parent window lends its device images
    if (!margCtx_ && ldso_ba_create(device_, &margCtx_)) {
        margCtx_ = nullptr;
        fail("ldso_ba_create (marginalisation)");
        return;
    }
    // the parent window as loaded holds every point still flagged ACTIVE before this call
    std::vector<PointHessian *> pts;
    for (const shared_ptr<PointHessian> &p : allPointsToMarg) pts.push_back(p.get());
    PointPack pk;
    pk.build(pts);
    ldso_ba_window w;
    std::memset(&w, 0, sizeof(w));
    w.n_frames = nFrames;
    w.width = width_;
    w.height = height_;
    std::memcpy(w.calib, calib_.value_scaledf, sizeof(w.calib));
    w.frame_energy_th = frameTH_.data();
    w.precalc = precalc_.data();
    w.ad_host = adH_.data();
    w.ad_target = adT_.data();
    w.c_prior = cPrior_.data();
    w.c_delta = cDeltaF;
    w.frame_prior = fPrior_.data();
    w.frame_delta_prior = fDeltaPrior_.data();
    pk.into(w);
    const int n = 8 * nFrames + CPARS;
    std::vector<double> H((size_t)n * n), b(n);
    if (ldso_ba_load_marginalization(margCtx_, ctx_, 0, &w) ||
        ldso_ba_marginalize_points(margCtx_, adHTdeltaF.data(), H.data(), b.data())) {
        fail("ldso_ba_marginalize_points");
        return;
    }
    if (!read_residuals(margCtx_, pk.res)) {
        fail("ldso_ba_get_residuals (marginalisation)");
        return;
    }
    passes_++;
    int nres = 0;
    for (PointFrameResidual *r : pk.res) {
        if (r->isActive()) {
            r->isLinearized = true;  // fixLinearizationF
            connectivityMap[conn_key(*r)][1]++;
            nres++;
        }
    }
    for (const shared_ptr<PointHessian> &p : allPointsToMarg) p->priorF *= kIdepthFixPriorMargFac;
    resInM += nres;
    for (int i = 0; i < n; i++) {
        bM[i] += kMargWeightFac * b[i];
        for (int j = 0; j < n; j++) HM(i, j) += kMargWeightFac * H[(size_t)i * n + j];
    }
    for (const shared_ptr<PointHessian> &p : allPointsToMarg) removePoint(p);
    makeIDX();
}

// EnergyFunctional.cc:264-278
void EnergyFunctional::dropPointsF() {
    residualTouched();
    for (const shared_ptr<PointHessian> &p : registry_)
        if ((p->status == PointStatus::OUTLIER || p->status == PointStatus::OUT) && !p->alreadyRemoved) removePoint(p);
    makeIDX();
}

// EnergyFunctional.cc:500-521: frame indices; the active, not removed points in host-frame order
// (the reference walks its frames' features; registry_ is that list)
void EnergyFunctional::makeIDX() {
    residualTouched();
    epoch_++;
    for (size_t i = 0; i < frames.size(); i++) frames[i]->idx = (int)i;
    std::vector<shared_ptr<PointHessian>> keep, live;
    for (const shared_ptr<PointHessian> &p : registry_) {
        if (p->alreadyRemoved) continue;
        live.push_back(p);
        if (p->status == PointStatus::ACTIVE) keep.push_back(p);
    }
    registry_.swap(live);
    std::stable_sort(keep.begin(), keep.end(), [](const shared_ptr<PointHessian> &a, const shared_ptr<PointHessian> &b) {
        return a->host.lock()->idx < b->host.lock()->idx;
    });
    allPoints.swap(keep);
    for (size_t i = 0; i < allPoints.size(); i++) {
        allPoints[i]->idxInPoints = (int)i;
        for (const shared_ptr<PointFrameResidual> &r : allPoints[i]->residuals) {
            r->hostIDX = r->host.lock()->idx;
            r->targetIDX = r->target.lock()->idx;
        }
    }
    dirty_ = true;
}

// EnergyFunctional.cc:551-609 (ldso_ba_set_adjoints)
void EnergyFunctional::setAdjointsF(shared_ptr<CalibHessian> Hcalib) {
    (void)Hcalib;
    epoch_++;
    std::vector<ldso_ba_frame_state> fs;
    packFrames(fs);
    adHost.assign((size_t)nFrames * nFrames * 64, 0.0);
    adTarget.assign((size_t)nFrames * nFrames * 64, 0.0);
    if (nFrames && ldso_ba_set_adjoints(nFrames, fs.data(), adHost.data(), adTarget.data(), cPrior))
        fail("ldso_ba_set_adjoints");
}

// EnergyFunctional.cc:523-549: frames' delta / delta_prior, adHTdeltaF, cDeltaF, points' deltaF
void EnergyFunctional::setDeltaF(shared_ptr<CalibHessian> HCalib) {
    epoch_++;
    for (int k = 0; k < 4; k++) cDeltaF[k] = (float)HCalib->value_minus_value_zero[k];
    std::vector<double> delta((size_t)8 * nFrames);
    for (int f = 0; f < nFrames; f++) {
        frames[f]->takeData(&settings_);
        std::memcpy(&delta[(size_t)8 * f], frames[f]->delta, 8 * sizeof(double));
    }
    adHTdeltaF.assign((size_t)nFrames * nFrames * 8, 0.f);
    if (nFrames && ldso_ba_ad_ht_delta(nFrames, delta.data(), adHost.data(), adTarget.data(), adHTdeltaF.data()))
        fail("ldso_ba_ad_ht_delta");
    for (const shared_ptr<PointHessian> &p : allPoints) p->deltaF = p->idepth - p->idepth_zero;
    calib_ = *HCalib;
}

// EnergyFunctional.cc:473-479
double EnergyFunctional::calcMEnergyF() {
    std::vector<double> delta((size_t)8 * nFrames);
    for (int f = 0; f < nFrames; f++) std::memcpy(&delta[(size_t)8 * f], frames[f]->delta, 8 * sizeof(double));
    double e = 0;
    if (ldso_ba_calc_m_energy(nFrames, HM.data(), bM.data(), cDeltaF, delta.data(), &e)) fail("ldso_ba_calc_m_energy");
    return e;
}

// EnergyFunctional.cc:481-498
double EnergyFunctional::calcLEnergyF_MT() {
    std::vector<double> prior((size_t)8 * nFrames), dprior((size_t)8 * nFrames);
    for (int f = 0; f < nFrames; f++) {
        std::memcpy(&prior[(size_t)8 * f], frames[f]->prior, 8 * sizeof(double));
        std::memcpy(&dprior[(size_t)8 * f], frames[f]->delta_prior, 8 * sizeof(double));
    }
    std::vector<float> dd(allPoints.size()), pf(allPoints.size());
    for (size_t q = 0; q < allPoints.size(); q++) {
        dd[q] = allPoints[q]->deltaF;
        pf[q] = allPoints[q]->priorF;
    }
    double e = 0;
    if (ldso_ba_calc_l_energy(nFrames, prior.data(), dprior.data(), cPrior, cDeltaF, (int32_t)dd.size(), dd.data(),
                              pf.data(), &e))
        fail("ldso_ba_calc_l_energy");
    return e;
}

// Frame-level terms (setPrecalcValues, setAdjointsF, takeData) from the current frame states,
// uploaded only when a frame state, the calibration or a threshold changed since the last upload
bool EnergyFunctional::uploadFrameTerms() {
    const int N = nFrames;
    packFrames(fs_);
    frameTH_.resize(N);
    for (int f = 0; f < N; f++) frameTH_[f] = frames[f]->frameEnergyTH;
    const bool same = fsUp_.size() == fs_.size() && thUp_ == frameTH_ &&
                      std::memcmp(fsUp_.data(), fs_.data(), fs_.size() * sizeof(ldso_ba_frame_state)) == 0 &&
                      std::memcmp(calibUp_, calib_.value_scaledf, sizeof(calibUp_)) == 0 &&
                      std::memcmp(cDeltaUp_, cDeltaF, sizeof(cDeltaUp_)) == 0;  // the bL calibration prior
    if (same && !dirty_) return true;
    precalc_.assign((size_t)N * N * LDSO_BA_PRECALC_STRIDE, 0.f);
    adH_.assign((size_t)N * N * 64, 0.0);
    adT_.assign((size_t)N * N * 64, 0.0);
    cPrior_.assign(4, 0.0);
    fPrior_.assign((size_t)N * 8, 0.0);
    fDelta_.assign((size_t)N * 8, 0.0);
    fDeltaPrior_.assign((size_t)N * 8, 0.0);
    if (ldso_ba_frame_precalc(N, fs_.data(), calib_.value_scaledf, precalc_.data()) ||
        ldso_ba_set_adjoints(N, fs_.data(), adH_.data(), adT_.data(), cPrior_.data()) ||
        ldso_ba_frame_take_data(N, fs_.data(), &settings_, fPrior_.data(), fDelta_.data(), fDeltaPrior_.data())) {
        fail("frame terms");
        return false;
    }
    if (!dirty_) {  // structure unchanged: the frame terms alone (ldso_ba_update without point data)
        ldso_ba_window w;
        std::memset(&w, 0, sizeof(w));
        w.n_frames = N;
        w.n_points = (int32_t)ptPtr_.size();
        w.n_residuals = (int32_t)resPtr_.size();
        w.width = width_;
        w.height = height_;
        std::memcpy(w.calib, calib_.value_scaledf, sizeof(w.calib));
        w.frame_energy_th = frameTH_.data();
        w.precalc = precalc_.data();
        w.ad_host = adH_.data();
        w.ad_target = adT_.data();
        w.c_prior = cPrior_.data();
        w.c_delta = cDeltaF;
        w.frame_prior = fPrior_.data();
        w.frame_delta_prior = fDeltaPrior_.data();
        if (ldso_ba_update(ctx_, 0, &w)) {
            fail("ldso_ba_update");
            return false;
        }
    }
    fsUp_ = fs_;
    thUp_ = frameTH_;
    std::memcpy(calibUp_, calib_.value_scaledf, sizeof(calibUp_));
    std::memcpy(cDeltaUp_, cDeltaF, sizeof(cDeltaUp_));
    return true;
}

// The persistent SoA mirror of the window (ldso_ba_window).  A structural change (insert / drop /
// remove / makeIDX / marginalisation) rebuilds and reloads it; otherwise only what changed goes
// up: the frame terms, the points' four per-step values (ldso_ba_update_points, 16 B a point,
// read through the mirror's raw pointers) and residual states edited on the host.
bool EnergyFunctional::upload() {
    if (!ctx_) return false;
    const int N = nFrames;
    if (N < 2) {
        err_ = "need at least two frames";
        return false;
    }
    if (!dirty_) {
        if (!uploadFrameTerms()) return false;
        const size_t P = ptPtr_.size();
        std::vector<float> pv(4 * P);
        for (size_t q = 0; q < P; q++) {
            const PointHessian &p = *ptPtr_[q];
            pv[4 * q] = p.idepth_scaled;
            pv[4 * q + 1] = p.idepth_zero_scaled;
            pv[4 * q + 2] = p.priorF;
            pv[4 * q + 3] = p.deltaF;
        }
        if (P && std::memcmp(pv.data(), pointVals_.data(), pv.size() * sizeof(float)) != 0) {
            if (ldso_ba_update_points(ctx_, 0, pv.data())) {
                fail("ldso_ba_update_points");
                return false;
            }
            pointVals_.swap(pv);
        }
        if (resSync_ == ResSync::HostNewer) {
            const size_t R = resPtr_.size();
            std::vector<int8_t> st(R);
            std::vector<float> se(R), ne(R);
            std::vector<uint8_t> fl(R);
            for (size_t k = 0; k < R; k++) {
                const PointFrameResidual &r = *resPtr_[k];
                st[k] = (int8_t)r.state_state;
                se[k] = (float)r.state_energy;
                ne[k] = (float)r.state_NewEnergy;
                fl[k] = (uint8_t)((r.isActiveAndIsGoodNEW ? LDSO_BA_FLAG_ACTIVE : 0u) | (r.isNew ? LDSO_BA_FLAG_NEW : 0u));
            }
            if (ldso_ba_update_residuals(ctx_, 0, st.data(), se.data(), ne.data(), fl.data())) {
                fail("ldso_ba_update_residuals");
                return false;
            }
            resSync_ = ResSync::Synced;
        }
        return true;
    }
    // structural change: rebuild the mirror (the only place the weak_ptr graph is walked)
    residualTouched();
    if (!uploadFrameTerms()) return false;
    ptPtr_.clear();
    for (const shared_ptr<PointHessian> &p : allPoints) ptPtr_.push_back(p.get());
    PointPack pk;
    pk.build(ptPtr_);
    pointHost_ = pk.host;
    pointRank_ = pk.rank;
    pointRanked_ = pk.ranked;
    pointData_ = pk.data;
    resBegin_ = pk.begin;
    resTarget_ = pk.target;
    resState_ = pk.state;
    resEnergy_ = pk.energy;
    resFlags_ = pk.flags;
    resPtr_ = pk.res;
    nResiduals = (int)resPtr_.size();
    resPoint_.resize(resPtr_.size());
    for (size_t q = 0; q < ptPtr_.size(); q++)
        for (int k = resBegin_[q]; k < resBegin_[q + 1]; k++) {
            resPtr_[k]->mirrorIdx = k;
            resPoint_[k] = ptPtr_[q];
        }
    pointVals_.resize(4 * ptPtr_.size());
    for (size_t q = 0; q < ptPtr_.size(); q++) {
        pointVals_[4 * q] = pointData_[q * LDSO_BA_POINT_STRIDE + 2];
        pointVals_[4 * q + 1] = pointData_[q * LDSO_BA_POINT_STRIDE + 3];
        pointVals_[4 * q + 2] = pointData_[q * LDSO_BA_POINT_STRIDE + 4];
        pointVals_[4 * q + 3] = pointData_[q * LDSO_BA_POINT_STRIDE + 5];
    }
    ldso_ba_window w;
    std::memset(&w, 0, sizeof(w));
    w.n_frames = N;
    w.n_points = (int32_t)pointHost_.size();
    w.n_residuals = nResiduals;
    w.width = width_;
    w.height = height_;
    std::memcpy(w.calib, calib_.value_scaledf, sizeof(w.calib));
    dI_.resize((size_t)N * width_ * height_ * 3);
    for (int f = 0; f < N; f++)
        std::memcpy(&dI_[(size_t)f * width_ * height_ * 3], frames[f]->dI, (size_t)width_ * height_ * 3 * sizeof(float));
    w.dI = dI_.data();
    w.frame_energy_th = frameTH_.data();
    w.precalc = precalc_.data();
    w.ad_host = adH_.data();
    w.ad_target = adT_.data();
    w.c_prior = cPrior_.data();
    w.c_delta = cDeltaF;
    w.frame_prior = fPrior_.data();
    w.frame_delta_prior = fDeltaPrior_.data();
    w.point_host = pointHost_.data();
    w.point_data = pointData_.data();
    w.point_res_begin = resBegin_.data();
    w.res_target = resTarget_.data();
    w.res_state = resState_.data();
    w.res_energy = resEnergy_.data();
    w.res_flags = resFlags_.data();
    w.point_rank = pointRanked_ ? pointRank_.data() : nullptr;
    if (ldso_ba_load(ctx_, 1, &w, 0, 1)) {
        fail("ldso_ba_load");
        return false;
    }
    // the device's state_NewEnergy starts as state_energy (ldso_ba_load); the host's may differ
    bool ne_differs = false;
    for (size_t k = 0; k < resPtr_.size() && !ne_differs; k++)
        ne_differs = (float)resPtr_[k]->state_NewEnergy != resEnergy_[k];
    resSync_ = ne_differs ? ResSync::HostNewer : ResSync::Synced;
    dirty_ = false;
    if (resSync_ == ResSync::HostNewer) return upload();
    return true;
}

void EnergyFunctional::resetOOB() {
    residualTouched();
    for (const shared_ptr<PointHessian> &p : allPoints)
        for (const shared_ptr<PointFrameResidual> &r : p->residuals)
            if (!r->isLinearized) {  // FullSystem.cc:866-869 (the mirror follows below)
                r->state_NewEnergy = r->state_energy = 0;
                r->state_NewState = OUTLIER;
                r->state_state = IN;
            }
    if (!dirty_ && ctx_) {
        if (ldso_ba_reset_oob(ctx_, 0)) fail("ldso_ba_reset_oob");
        else if (resSync_ == ResSync::DeviceNewer) resSync_ = ResSync::Synced;
    }
}

// every per-residual / per-point result of the device's last pass into the objects
bool EnergyFunctional::readBack(bool points_and_th) {
    if (!read_residuals(ctx_, resPtr_)) {
        fail("ldso_ba_get_residuals");
        return false;
    }
    resSync_ = ResSync::Synced;
    if (!points_and_th) return true;
    const int P = (int)ptPtr_.size(), N = nFrames;
    std::vector<float> hdi(P), bds(P), ih(P), th(N);
    if (P && ldso_ba_get_points(ctx_, 0, hdi.data(), bds.data(), ih.data(), nullptr, nullptr, nullptr)) {
        fail("ldso_ba_get_points");
        return false;
    }
    for (int q = 0; q < P; q++) {
        ptPtr_[q]->HdiF = hdi[q];
        ptPtr_[q]->bdSumF = bds[q];
        ptPtr_[q]->idepth_hessian = ih[q];
    }
    if (ldso_ba_get_frame_energy_th(ctx_, 0, th.data()) == 0) {
        for (int f = 0; f < N; f++) frames[f]->frameEnergyTH = th[f];
        thUp_ = th;  // the device holds these already
        frameTH_ = th;
    }
    return true;
}

// linearizeAll's read-back of what its callers need at once: the frame thresholds, the points'
// HdiF / bdSumF / idepth_hessian, the residual states and, on the fix pass, FixPassResult from the
// flags and relBS; every other residual field stays on the device until a consumer asks
// (syncResiduals, a residual method, residualCenter)
bool EnergyFunctional::readPassSummary(bool fix) {
    const size_t R = resPtr_.size(), P = ptPtr_.size();
    const int N = nFrames;
    std::vector<uint8_t> fl(R);
    std::vector<float> rb(fix ? R : 0);
    outState_.resize(R);
    if (R && ldso_ba_get_residuals(ctx_, 0, nullptr, outState_.data(), nullptr, nullptr, nullptr, fl.data(), nullptr,
                                   fix ? rb.data() : nullptr)) {
        fail("ldso_ba_get_residuals");
        return false;
    }
    outStatePass_ = passes_;
    std::vector<float> hdi(P), bds(P), ih(P), th(N);
    if (P && ldso_ba_get_points(ctx_, 0, hdi.data(), bds.data(), ih.data(), nullptr, nullptr, nullptr)) {
        fail("ldso_ba_get_points");
        return false;
    }
    for (size_t q = 0; q < P; q++) {
        ptPtr_[q]->HdiF = hdi[q];
        ptPtr_[q]->bdSumF = bds[q];
        ptPtr_[q]->idepth_hessian = ih[q];
    }
    if (ldso_ba_get_frame_energy_th(ctx_, 0, th.data()) == 0) {
        for (int f = 0; f < N; f++) frames[f]->frameEnergyTH = th[f];
        thUp_ = th;  // the device holds these already
        frameTH_ = th;
    }
    if (fix) {
        fix_.toRemove.clear();
        fix_.maxRelBS.assign(P, 0.f);
        fix_.numGood.assign(P, 0);
        fix_.lastState.assign(2 * P, -1);
        for (size_t q = 0; q < P; q++)
            for (int k = resBegin_[q]; k < resBegin_[q + 1]; k++) {
                const int t = resTarget_[k];
                if (t >= N - 2) fix_.lastState[2 * q + (N - 1 - t)] = outState_[k];
                if (!(fl[k] & LDSO_BA_FLAG_ACTIVE)) {
                    fix_.toRemove.push_back(resPtr_[k]);
                } else if (fl[k] & LDSO_BA_FLAG_NEW) {  // FullSystem.cc:1799-1813
                    fix_.maxRelBS[q] = std::max(fix_.maxRelBS[q], rb[k]);
                    fix_.numGood[q]++;
                }
            }
    }
    return true;
}

ResState EnergyFunctional::residualState(int k) {
    if (outStatePass_ != passes_ || resSync_ != ResSync::DeviceNewer) {  // not from the last pass
        if (resSync_ == ResSync::DeviceNewer && ldso_ba_get_residuals(ctx_, 0, nullptr, outState_.data(), nullptr,
                                                                      nullptr, nullptr, nullptr, nullptr, nullptr) == 0)
            outStatePass_ = passes_;
        else
            return resPtr_[k]->state_state;  // the host copy is current
    }
    return (ResState)outState_[k];
}

const float *EnergyFunctional::residualCenter(int k) {
    if (resSync_ != ResSync::DeviceNewer) return resPtr_[k]->centerProjectedTo;  // the host copy is current
    if (outCenterPass_ != passes_) {
        outCenter_.resize(3 * resPtr_.size());
        if (ldso_ba_get_residuals(ctx_, 0, nullptr, nullptr, nullptr, nullptr, outCenter_.data(), nullptr, nullptr,
                                  nullptr)) {
            fail("ldso_ba_get_residuals");
            return resPtr_[k]->centerProjectedTo;
        }
        outCenterPass_ = passes_;
    }
    return &outCenter_[3 * (size_t)k];
}

void EnergyFunctional::syncResiduals() {
    if (resSync_ != ResSync::DeviceNewer || !ctx_ || dirty_) return;
    resSync_ = ResSync::Synced;  // before the reads: the residual setters called below see it synced
    readBack(true);
}

Vec3 EnergyFunctional::linearizeAll(bool fixLinearization) {
    Vec3 out = {0, 0, 0};
    epoch_++;
    if (!upload()) return out;
    if (ldso_ba_linearize(ctx_, fixLinearization ? 1 : 0, fixLinearization ? 0 : 1)) {
        fail("ldso_ba_linearize");
        return out;
    }
    passes_++;
    double e[3];
    if (ldso_ba_get_energy(ctx_, 0, e)) {
        fail("ldso_ba_get_energy");
        return out;
    }
    if (!readPassSummary(fixLinearization)) return out;
    resSync_ = ResSync::DeviceNewer;  // the residual objects' fields follow on demand (syncResiduals)
    if (!fixLinearization) resInA = (int)e[2];
    out = {e[0], e[1], e[2]};
    return out;
}

// One device pass (ldso_ba_linearize_residuals) relinearising every residual of the window from
// resetOOB; the entries serve PointFrameResidual::linearize until the next change of the window
bool EnergyFunctional::runRelinearization() {
    if (!upload()) return false;
    const size_t R = resPtr_.size();
    cNewState_.assign(R, 0);
    cCenterOk_.assign(R, 0);
    cNewEnergy_.assign(R, 0.f);
    cEwo_.assign(R, 0.f);
    cCenter_.assign(3 * R, 0.f);
    cJp_.assign(8 * R, 0.f);
    if (R && ldso_ba_linearize_residuals(ctx_, 0, cNewState_.data(), cNewEnergy_.data(), cEwo_.data(), cCenter_.data(),
                                         cCenterOk_.data(), cJp_.data())) {
        fail("ldso_ba_linearize_residuals");
        return false;
    }
    passes_++;
    cSnap_.resize(4 * R);
    for (size_t k = 0; k < R; k++) {
        const PointHessian &p = *resPoint_[k];
        cSnap_[4 * k] = p.u;
        cSnap_[4 * k + 1] = p.v;
        cSnap_[4 * k + 2] = p.idepth_scaled;
        cSnap_[4 * k + 3] = p.idepth_zero_scaled;
    }
    cacheEpoch_ = epoch_;
    return true;
}

double EnergyFunctional::linearizeResidual(PointFrameResidual &r) {
    auto fresh = [&]() {
        if (dirty_ || cacheEpoch_ != epoch_ || r.mirrorIdx < 0 || (size_t)r.mirrorIdx >= cNewState_.size() ||
            resPtr_[r.mirrorIdx] != &r)
            return false;
        const PointHessian &p = *resPoint_[r.mirrorIdx];
        const float *sn = &cSnap_[4 * (size_t)r.mirrorIdx];
        if (!(sn[0] == p.u && sn[1] == p.v && sn[2] == p.idepth_scaled && sn[3] == p.idepth_zero_scaled)) return false;
        // the frame terms the pass used: the residual's host and target as uploaded (state,
        // evaluation point, exposure, threshold) and the calibration -- a direct edit of either
        // without setDeltaF / setAdjointsF / linearizeAll in between is seen here
        if (std::memcmp(calibUp_, calib_.value_scaledf, sizeof(calibUp_)) != 0) return false;
        for (const auto &wf : {r.host, r.target}) {
            const auto f = wf.lock();
            if (!f) return false;
            const size_t i = (size_t)f->idx;
            if (i >= fsUp_.size() || i >= frames.size() || frames[i].get() != f.get()) return false;
            ldso_ba_frame_state fsn;
            frame_state(*f, fsn);
            if (std::memcmp(&fsn, &fsUp_[i], sizeof(fsn)) != 0 || f->frameEnergyTH != thUp_[i]) return false;
        }
        return true;
    };
    if (!fresh() && (!runRelinearization() || !fresh())) return r.state_energy;
    const size_t k = (size_t)r.mirrorIdx;
    const ResState ns = (ResState)cNewState_[k];
    r.state_NewState = ns;
    if (cCenterOk_[k]) std::memcpy(r.centerProjectedTo, &cCenter_[3 * k], 3 * sizeof(float));
    if (ns == OOB) return r.state_energy;  // Residuals.cc:59-63, 131-146: state_energy, NewEnergy kept
    r.state_NewEnergyWithOutlier = cEwo_[k];
    if (r.state_NewEnergy != (double)cNewEnergy_[k]) residualEdited();  // the device's NewEnergy follows
    r.state_NewEnergy = cNewEnergy_[k];
    if (ns == IN) std::memcpy(r.J_JpJdF, &cJp_[8 * k], sizeof(r.J_JpJdF));
    return r.state_NewEnergy;
}

// FullSystem::optimize's loop (FullSystem.cc:844-970) on the device; see the header
Vec3 EnergyFunctional::optimize(int n_its, shared_ptr<CalibHessian> HCalib, std::vector<Vec3> *energies,
                                bool *isLost, int *iterations, const ldso_ba_opt_settings *settings) {
    Vec3 out = {0, 0, 0};
    if (isLost) *isLost = false;
    if (iterations) *iterations = 0;
    if (nFrames < 2) return out;   // FullSystem.cc:846-851
    if (nFrames < 3) n_its = 20;
    if (nFrames < 4) n_its = 15;
    if (settings && !setSettings(*settings)) return out;
    epoch_++;
    calib_ = *HCalib;
    if (!upload()) return out;
    const int N = nFrames, n = 8 * N + CPARS, P = (int)ptPtr_.size();
    std::vector<double> ns((size_t)7 * n), e((size_t)3 * (n_its + 1));
    if (ldso_ba_nullspaces(N, fs_.data(), ns.data())) {
        fail("ldso_ba_nullspaces");
        return out;
    }
    std::vector<ldso_ba_frame_state> fo(N);
    std::vector<float> idepth(P);
    double calib_out[4];
    int32_t its = 0, status = 0;
    if (ldso_ba_optimize(ctx_, n_its, &settings_, fs_.data(), HCalib->value, HCalib->value_zero, ns.data(), e.data(),
                         fo.data(), calib_out, idepth.data(), &its, &status)) {
        fail("ldso_ba_optimize");
        return out;
    }
    // the loop's exits: lost (FullSystem.cc:907-911) after its iterations (the state is that of
    // the step before), canbreak (:968-969); the passes the device ran: the first + one per step
    passes_ += 1 + (status == LDSO_BA_OPT_LOST ? its - 1 : its);
    if (isLost) *isLost = status == LDSO_BA_OPT_LOST;
    if (iterations) *iterations = its;
    // doStepFromBackup's results (FullSystem.cc:1843-1922) into the objects: frame states, the
    // calibration, every point's setIdepth / setIdepthZero
    for (int f = 0; f < N; f++) std::memcpy(frames[f]->state, fo[f].state, sizeof(fo[f].state));
    HCalib->setValue(calib_out);
    calib_ = *HCalib;
    for (int q = 0; q < P; q++) {
        ptPtr_[q]->setIdepth(idepth[q]);
        ptPtr_[q]->setIdepthZero(idepth[q]);
    }
    // setNewFrameEnergyTH of the loop's passes (the device holds it; the next frame-term upload
    // must not overwrite it with the old value)
    std::vector<float> th(N);
    if (ldso_ba_get_frame_energy_th(ctx_, 0, th.data())) {
        fail("ldso_ba_get_frame_energy_th");
        return out;
    }
    for (int f = 0; f < N; f++) frames[f]->frameEnergyTH = th[f];
    setDeltaF(HCalib);  // setPrecalcValues' setDeltaF after the last step: points' deltaF = 0
    // The frame terms are NOT marked uploaded: the next pass uses the host's FrameFramePrecalc /
    // takeData of the stepped states (the reference's setPrecalcValues), which differ from the
    // device's in libm's last ulp; upload() re-sends them in one staged launch.
    for (int q = 0; q < P; q++) {
        pointVals_[4 * q] = ptPtr_[q]->idepth_scaled;
        pointVals_[4 * q + 1] = ptPtr_[q]->idepth_zero_scaled;
        pointVals_[4 * q + 3] = ptPtr_[q]->deltaF;
    }
    resSync_ = ResSync::DeviceNewer;
    resInA = (int)e[3 * n_its + 2];
    if (energies)
        for (int s = 0; s <= n_its; s++) energies->push_back({e[3 * s], e[3 * s + 1], e[3 * s + 2]});
    out = {e[3 * n_its], e[3 * n_its + 1], e[3 * n_its + 2]};
    return out;
}

// EnergyFunctional.cc:280-471, non-VI branch: the stitched blocks of the last linearizeAll,
// HM / bM, the pose and scale nullspaces (FullSystem::getNullspaces) and the host LDL^T
void EnergyFunctional::solveSystemF(int iteration, double lambda, shared_ptr<CalibHessian> HCalib) {
    (void)HCalib;
    if (ldso_ba_check_settings(&settings_)) {  // the solver mode / vi_enable this branch implements
        fail("solveSystemF");
        return;
    }
    currentLambda_ = lambda;
    const int n = 8 * nFrames + CPARS;
    HA_top = MatXX(n, n);
    HL_top = MatXX(n, n);
    H_sc = MatXX(n, n);
    bA_top = VecX(n);
    bL_top = VecX(n);
    b_sc = VecX(n);
    if (ldso_ba_get_system(ctx_, 0, HA_top.data(), bA_top.data(), HL_top.data(), bL_top.data(), H_sc.data(),
                           b_sc.data())) {
        fail("ldso_ba_get_system");
        return;
    }
    std::vector<ldso_ba_frame_state> fs;
    packFrames(fs);
    std::vector<double> ns((size_t)7 * n);
    if (ldso_ba_nullspaces(nFrames, fs.data(), ns.data())) {
        fail("ldso_ba_nullspaces");
        return;
    }
    lastNullspaces_pose.assign(6, VecX(n));
    lastNullspaces_scale.assign(1, VecX(n));
    for (int k = 0; k < 7; k++)
        std::memcpy((k < 6 ? lastNullspaces_pose[k] : lastNullspaces_scale[0]).data(), &ns[(size_t)k * n],
                    n * sizeof(double));
    lastNullspaces_forLogging = lastNullspaces_pose;
    lastNullspaces_forLogging.push_back(lastNullspaces_scale[0]);
    lastX = VecX(n);
    if (ldso_ba_solve_system(&settings_, nFrames, iteration, lambda, HA_top.data(), bA_top.data(), HL_top.data(),
                             bL_top.data(), HM.data(), bM.data(), H_sc.data(), b_sc.data(), ns.data(), 7, lastX.data()))
        fail("ldso_ba_solve_system");
}

// EnergyFunctional.cc:611-667: calibration and frame steps are -x, point steps from the device
void EnergyFunctional::resubstituteF_MT(const VecX &x, shared_ptr<CalibHessian> HCalib, bool MT) {
    (void)MT;
    for (int k = 0; k < CPARS; k++) HCalib->step[k] = -x[k];
    for (const shared_ptr<FrameHessian> &h : frames) {
        for (int k = 0; k < 8; k++) h->step[k] = -x[CPARS + 8 * h->idx + k];
        h->step[8] = h->step[9] = 0;
    }
    std::vector<float> step(ptPtr_.size());
    if (ldso_ba_resubstitute(ctx_, 0, x.data(), currentLambda_, step.data())) {
        fail("ldso_ba_resubstitute");
        return;
    }
    for (size_t q = 0; q < ptPtr_.size(); q++) ptPtr_[q]->step = step[q];
}

}  // namespace ldso_amd
