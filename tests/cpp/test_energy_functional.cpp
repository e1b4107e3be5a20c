// test_energy_functional.cpp -- the C++ host face (include/ldso_amd/energy_functional.h) driven
// through a whole keyframe cycle the way FullSystem drives LDSO's EnergyFunctional, each device
// result checked against the CPU oracle (oracle/, test infrastructure) on the same inputs:
//
//   insertFrame / insertPoint / insertResidual / makeIDX / setAdjointsF / setDeltaF
//   optimize x3: resetOOB, linearizeAll (+applyRes, accumulate), solveSystemF, resubstituteF_MT,
//                the step (test harness: additive frame states, point setIdepth/setIdepthZero),
//                setDeltaF, calcLEnergyF_MT / calcMEnergyF
//   flagPointsForRemoval (frame 0's points + every 7th point MARGINALIZED, some OUT) with the
//   reference's per-residual loop (resetOOB, linearize, applyRes, fixLinearizationF): every
//   residual against the oracle, and ONE device pass for the whole loop,
//   marginalizePointsF, dropPointsF, marginalizeFrame(frame 0) + dropResidual of its
//   observations, setAdjointsF / setDeltaF
//   optimize x2 with the marginalisation prior HM / bM in the solve
//   EnergyFunctional::optimize (the device GN loop) against ldso_ba_optimize on the same window,
//   the lazy write-back of the residual fields, then linearizeAll(true) against the oracle
//
//   test_energy_functional --cpu   bookkeeping and the no-device error path
//   test_energy_functional         the GPU cycle
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <unordered_map>
#include <vector>

#include "../../include/ldso_amd/energy_functional.h"
#include "../../ldso_amd/csrc/synth.h"
#include "../../oracle/ldso_oracle.h"

using namespace ldso_amd;

static int g_fail = 0;
#define CHECK(cond, ...)                                     \
    do {                                                     \
        if (!(cond)) {                                       \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);                        \
            std::printf("\n");                               \
            g_fail++;                                        \
        }                                                    \
    } while (0)

struct Synth {
    int N, P, R, w, h;
    std::vector<ldso_ba_frame_state> fs;
    std::vector<float> dI, th, pd, re;
    float calib[4];
    std::vector<int32_t> ph, rb, rt;
    std::vector<int8_t> rs;
    std::vector<uint8_t> rf;
    Synth(int N_, int P_, int w_, int h_, uint64_t seed) : N(N_), P(P_), R(P_ * (N_ - 1)), w(w_), h(h_) {
        fs.resize(N);
        dI.resize((size_t)N * w * h * 3);
        th.resize(N);
        pd.resize((size_t)P * LDSO_BA_POINT_STRIDE);
        ph.resize(P);
        rb.resize(P + 1);
        rt.resize(R);
        rs.resize(R);
        re.resize(R);
        rf.resize(R);
        ldso_synth_params prm = {N, P, w, h, seed, 0.05f, 0.01f, 1e-3f, 0.04f};
        ldso_synth_fill(&prm, fs.data(), dI.data(), calib, th.data(), ph.data(), pd.data(), rb.data(), rt.data(),
                        rs.data(), re.data(), rf.data());
    }
};

// the LDSO object graph of a synthetic window (shared_ptr ownership, as the reference)
struct Graph {
    shared_ptr<CalibHessian> calib = std::make_shared<CalibHessian>();
    std::vector<shared_ptr<FrameHessian>> frames;
    std::vector<shared_ptr<PointHessian>> points;
    explicit Graph(const Synth &S) {
        calib->wG0 = S.w;
        calib->hG0 = S.h;
        std::memcpy(calib->value_scaledf, S.calib, sizeof(S.calib));
        for (int k = 0; k < 4; k++) calib->value[k] = calib->value_zero[k] = (double)S.calib[k] * (1.0 / 50.0);
        for (int f = 0; f < S.N; f++) {
            auto F = std::make_shared<FrameHessian>();
            F->frameID = f;
            std::memcpy(F->worldToCam_evalPT, S.fs[f].world_to_cam_evalpt, sizeof(F->worldToCam_evalPT));
            std::memcpy(F->state, S.fs[f].state, sizeof(F->state));
            std::memcpy(F->state_zero, S.fs[f].state_zero, sizeof(F->state_zero));
            F->ab_exposure = S.fs[f].ab_exposure;
            F->dI = &S.dI[(size_t)f * S.w * S.h * 3];
            F->frameEnergyTH = S.th[f];
            frames.push_back(F);
        }
        for (int p = 0; p < S.P; p++) {
            auto Pt = std::make_shared<PointHessian>();
            const float *d = &S.pd[(size_t)p * LDSO_BA_POINT_STRIDE];
            Pt->host = frames[S.ph[p]];
            Pt->u = d[0];
            Pt->v = d[1];
            Pt->setIdepth(d[2]);
            Pt->setIdepthZero(d[3]);
            Pt->priorF = d[4];
            Pt->deltaF = d[5];
            std::memcpy(Pt->color, d + 8, sizeof(Pt->color));
            std::memcpy(Pt->weights, d + 16, sizeof(Pt->weights));
            for (int k = S.rb[p]; k < S.rb[p + 1]; k++) {
                auto r = std::make_shared<PointFrameResidual>(Pt, frames[S.ph[p]], frames[S.rt[k]]);
                r->state_state = (ResState)S.rs[k];
                r->state_energy = S.re[k];
                r->isNew = (S.rf[k] & LDSO_BA_FLAG_NEW) != 0;
                r->isActiveAndIsGoodNEW = (S.rf[k] & LDSO_BA_FLAG_ACTIVE) != 0;
                Pt->residuals.push_back(r);
            }
            points.push_back(Pt);
        }
    }
    void insertInto(EnergyFunctional &ef) {
        for (auto &F : frames) ef.insertFrame(F, calib);
        for (auto &P : points) {
            ef.insertPoint(P);
            for (auto &r : P->residuals) ef.insertResidual(r);
        }
        ef.makeIDX();
        ef.setAdjointsF(calib);
        ef.setDeltaF(calib);
    }
};

// The oracle's window built from the EnergyFunctional's current objects (makeIDX order)
struct OracleWin {
    std::vector<int32_t> ph, rb, rt;
    std::vector<float> pd, re, precalc, th, dI, cdelta;
    std::vector<int8_t> rs;
    std::vector<uint8_t> rf;
    std::vector<double> adH, adT, cp, fp, fd, fdp;
    std::vector<ldso_ba_frame_state> fs;
    std::vector<PointFrameResidual *> order;
    ldso_ba_window w;
    // calib: CalibHessian::value_scaledf of the pass (the synthetic one unless a device loop stepped it)
    OracleWin(const Synth &S, EnergyFunctional &ef, const float *calib = nullptr) {
        if (!calib) calib = S.calib;
        const int N = ef.nFrames;
        fs.resize(N);
        dI.resize((size_t)N * S.w * S.h * 3);
        for (int f = 0; f < N; f++) {
            const FrameHessian &F = *ef.frames[f];
            std::memset(&fs[f], 0, sizeof(fs[f]));
            std::memcpy(fs[f].world_to_cam_evalpt, F.worldToCam_evalPT, sizeof(F.worldToCam_evalPT));
            std::memcpy(fs[f].state, F.state, sizeof(F.state));
            std::memcpy(fs[f].state_zero, F.state_zero, sizeof(F.state_zero));
            fs[f].ab_exposure = F.ab_exposure;
            fs[f].is_first_frame = F.frameID == 0;
            std::memcpy(&dI[(size_t)f * S.w * S.h * 3], F.dI, (size_t)S.w * S.h * 3 * sizeof(float));
            th.push_back(F.frameEnergyTH);
        }
        precalc.resize((size_t)N * N * LDSO_BA_PRECALC_STRIDE);
        adH.resize((size_t)N * N * 64);
        adT.resize((size_t)N * N * 64);
        cp.resize(4);
        fp.resize(8 * N);
        fd.resize(8 * N);
        fdp.resize(8 * N);
        cdelta.assign(ef.cDeltaF, ef.cDeltaF + 4);
        oracle_frame_precalc(N, fs.data(), calib, precalc.data());
        oracle_set_adjoints(N, fs.data(), adH.data(), adT.data(), cp.data());
        oracle_frame_take_data(N, fs.data(), fp.data(), fd.data(), fdp.data());
        rb.push_back(0);
        for (auto &p : ef.allPoints) {
            ph.push_back(p->host.lock()->idx);
            float d[LDSO_BA_POINT_STRIDE] = {p->u, p->v, p->idepth_scaled, p->idepth_zero_scaled, p->priorF, p->deltaF};
            std::memcpy(d + 8, p->color, sizeof(p->color));
            std::memcpy(d + 16, p->weights, sizeof(p->weights));
            pd.insert(pd.end(), d, d + LDSO_BA_POINT_STRIDE);
            for (auto &r : p->residuals) {
                rt.push_back(r->target.lock()->idx);
                rs.push_back((int8_t)r->state_state);
                re.push_back((float)r->state_energy);
                rf.push_back((r->isActiveAndIsGoodNEW ? 1 : 0) | (r->isNew ? 2 : 0));
                order.push_back(r.get());
            }
            rb.push_back((int32_t)rt.size());
        }
        std::memset(&w, 0, sizeof(w));
        w.n_frames = N;
        w.n_points = (int)ph.size();
        w.n_residuals = (int)rt.size();
        w.width = S.w;
        w.height = S.h;
        std::memcpy(w.calib, calib, sizeof(w.calib));
        w.dI = dI.data();
        w.frame_energy_th = th.data();
        w.precalc = precalc.data();
        w.ad_host = adH.data();
        w.ad_target = adT.data();
        w.c_prior = cp.data();
        w.c_delta = cdelta.data();
        w.frame_prior = fp.data();
        w.frame_delta_prior = fdp.data();
        w.point_host = ph.data();
        w.point_data = pd.data();
        w.point_res_begin = rb.data();
        w.res_target = rt.data();
        w.res_state = rs.data();
        w.res_energy = re.data();
        w.res_flags = rf.data();
    }
};

static double rel(const double *a, const double *b, size_t n) {
    double num = 0, den = 0;
    for (size_t i = 0; i < n; i++) {
        num += (a[i] - b[i]) * (a[i] - b[i]);
        den += b[i] * b[i];
    }
    return std::sqrt(num / (den > 0 ? den : 1));
}

// worst per 8x8-block relative Frobenius error (blocks: calibration, then frames)
static double block_err(const MatXX &G, const MatXX &O) {
    const int n = O.rows(), nb = (n - 4) / 8 + 1;
    auto lo = [](int k) { return k == 0 ? 0 : 4 + 8 * (k - 1); };
    auto hi = [](int k) { return k == 0 ? 4 : 4 + 8 * k; };
    double scale = 0;
    for (double v : O.a) scale += v * v;
    scale = std::sqrt(scale);
    double worst = 0;
    for (int a = 0; a < nb; a++)
        for (int b = 0; b < nb; b++) {
            double num = 0, den = 0;
            for (int i = lo(a); i < hi(a); i++)
                for (int j = lo(b); j < hi(b); j++) {
                    num += (G(i, j) - O(i, j)) * (G(i, j) - O(i, j));
                    den += O(i, j) * O(i, j);
                }
            worst = std::fmax(worst, std::sqrt(num) / std::fmax(std::sqrt(den), 1e-9 * scale + 1e-300));
        }
    return worst;
}

static int cpu_tests() {
    Synth S(4, 60, 160, 120, 3);
    Graph G(S);
    auto ef = std::make_shared<EnergyFunctional>(1 << 20);  // no such device: reported, never thrown
    CHECK(!ef->ok(), "creating a context on a missing device must fail");
    CHECK(!ef->lastError().empty(), "error message expected");
    G.insertInto(*ef);
    CHECK(ef->nFrames == 4 && ef->nPoints == 60 && ef->nResiduals == 180, "counts %d %d %d", ef->nFrames,
          ef->nPoints, ef->nResiduals);
    CHECK(ef->HM.rows() == 8 * 4 + CPARS && ef->bM.size() == 8 * 4 + CPARS, "HM / bM grow with insertFrame");
    for (size_t i = 1; i < ef->allPoints.size(); i++)
        CHECK(ef->allPoints[i - 1]->host.lock()->idx <= ef->allPoints[i]->host.lock()->idx, "makeIDX host order");
    int conn = 0;
    for (auto &kv : ef->connectivityMap) conn += kv.second[0];
    CHECK(conn == 180, "connectivity map counts %d", conn);
    auto r0 = G.points[0]->residuals[0];
    ef->dropResidual(r0);
    CHECK(ef->nResiduals == 179 && G.points[0]->residuals.size() == 2, "dropResidual");
    ef->removePoint(G.points[1]);
    CHECK(ef->nPoints == 59 && ef->nResiduals == 176, "removePoint");
    G.points[2]->status = PointStatus::OUT;
    ef->dropPointsF();
    CHECK(ef->nPoints == 58 && (int)ef->allPoints.size() == 58, "dropPointsF");
    const double eL = ef->calcLEnergyF_MT(), eM = ef->calcMEnergyF();
    CHECK(std::isfinite(eL) && eM == 0.0, "host energies without a device: %g %g", eL, eM);
    const Vec3 e = ef->linearizeAll(false);
    CHECK(e[0] == 0 && !ef->ok(), "linearize without a device reports an error");
    return 0;
}

struct Cycle {
    const Synth &S;
    EnergyFunctional &ef;
    MatXX HMo;
    VecX bMo;
    std::unique_ptr<OracleWin> Op;
    oracle_window *ow = nullptr;
    Cycle(const Synth &S_, EnergyFunctional &ef_) : S(S_), ef(ef_), HMo(ef_.HM), bMo(ef_.bM) {}
    ~Cycle() {
        if (ow) oracle_destroy(ow);
    }

    // reload: the face re-uploads the window (structure changed) and the oracle is created anew;
    // otherwise both keep their residual states and take the new frame / point values
    void iteration(int it, const shared_ptr<CalibHessian> &calib, bool reload) {
        const int N = ef.nFrames, n = 8 * N + 4;
        Op.reset(new OracleWin(S, ef));  // the inputs this pass sees
        OracleWin &O = *Op;
        oracle_set_threads(0);
        if (reload || !ow) {
            if (ow) oracle_destroy(ow);
            ow = oracle_create(&O.w);
        } else {
            CHECK(oracle_update(ow, &O.w) == 0, "oracle_update");
        }
        CHECK(ow != nullptr, "oracle window");
        if (!ow) return;
        const Vec3 e = ef.linearizeAll(false);
        CHECK(ef.ok(), "it %d linearizeAll: %s", it, ef.lastError().c_str());
        double eo[3];
        oracle_linearize_all(ow, 0, eo);
        oracle_apply_res(ow);
        std::vector<double> HA(n * n), bA(n), HL(n * n), bL(n), Hsc(n * n), bsc(n);
        oracle_accumulate(ow, HA.data(), bA.data(), HL.data(), bL.data(), Hsc.data(), bsc.data());
        CHECK(e[2] == eo[2], "it %d: #IN %g vs %g", it, e[2], eo[2]);
        CHECK(std::fabs(e[0] - eo[0]) <= 1e-9 * std::fabs(eo[0]), "it %d: energy %.17g vs %.17g", it, e[0], eo[0]);
        CHECK(ef.resInA == (int)eo[2], "it %d: resInA", it);
        const int R = (int)O.order.size();
        std::vector<int8_t> ns(R), st(R);
        std::vector<float> se(R), ewo(R), ctr(3 * R), jp(8 * R), rbs(R);
        std::vector<uint8_t> fl(R);
        oracle_get_residuals(ow, ns.data(), st.data(), se.data(), ewo.data(), ctr.data(), fl.data(), jp.data(),
                             rbs.data());
        // the compact per-pass outputs before any write-back: states and centres by mirror index
        int bad_lazy = 0;
        for (int k = 0; k < R; k++) {
            const PointFrameResidual &r = *O.order[k];
            bad_lazy += ef.residualState(r.mirrorIdx) != st[k];
            bad_lazy += std::memcmp(ef.residualCenter(r.mirrorIdx), &ctr[3 * k], 12) != 0;
        }
        CHECK(bad_lazy == 0, "it %d: %d residualState / residualCenter values differ from the oracle", it, bad_lazy);
        ef.syncResiduals();  // linearizeAll leaves the residual objects' fields on the device until asked
        int bad = 0, why[7] = {0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < R; k++) {
            const PointFrameResidual &r = *O.order[k];
            const bool d[7] = {r.state_NewState != ns[k], r.state_state != st[k], (float)r.state_energy != se[k],
                               (float)r.state_NewEnergyWithOutlier != ewo[k],
                               r.isActiveAndIsGoodNEW != ((fl[k] & 1) != 0),
                               std::memcmp(r.centerProjectedTo, &ctr[3 * k], 12) != 0,
                               r.isActiveAndIsGoodNEW && std::memcmp(r.JpJdF, &jp[8 * k], 32) != 0};
            bool any = false;
            for (int q = 0; q < 7; q++) {
                why[q] += d[q];
                any = any || d[q];
            }
            bad += any;
        }
        CHECK(bad == 0, "it %d: %d of %d residuals differ from the oracle (new_state %d state %d energy %d e_wo %d "
              "active %d centre %d JpJdF %d)", it, bad, R, why[0], why[1], why[2], why[3], why[4], why[5], why[6]);
        std::vector<float> th(N);
        oracle_get_frame_energy_th(ow, th.data());
        for (int f = 0; f < N; f++) CHECK(ef.frames[f]->frameEnergyTH == th[f], "it %d: frameEnergyTH[%d]", it, f);

        ef.solveSystemF(it, 1e-5, calib);
        CHECK(ef.ok(), "it %d solveSystemF: %s", it, ef.lastError().c_str());
        CHECK(rel(ef.HA_top.data(), HA.data(), n * n) < 1e-5 && rel(ef.H_sc.data(), Hsc.data(), n * n) < 1e-5 &&
                  rel(ef.bA_top.data(), bA.data(), n) < 1e-5 && rel(ef.b_sc.data(), bsc.data(), n) < 1e-5,
              "it %d: stitched system %.2e %.2e", it, rel(ef.HA_top.data(), HA.data(), n * n),
              rel(ef.H_sc.data(), Hsc.data(), n * n));
        // the solver on the same system and marginalisation prior as the oracle's
        std::vector<double> ns7((size_t)7 * n), xo(n);
        oracle_nullspaces(N, O.fs.data(), ns7.data());
        oracle_solve_system(N, it, 1e-5, ef.HA_top.data(), ef.bA_top.data(), ef.HL_top.data(), ef.bL_top.data(),
                            ef.HM.data(), ef.bM.data(), ef.H_sc.data(), ef.b_sc.data(), ns7.data(), 7, xo.data());
        CHECK(rel(ef.lastX.data(), xo.data(), n) < 1e-9, "it %d: solve %.2e", it, rel(ef.lastX.data(), xo.data(), n));
        CHECK((int)ef.lastNullspaces_pose.size() == 6 && (int)ef.lastNullspaces_scale.size() == 1 &&
                  rel(ef.lastNullspaces_pose[0].data(), ns7.data(), n) == 0.0,
              "it %d: lastNullspaces", it);

        ef.resubstituteF_MT(ef.lastX, calib);
        CHECK(ef.ok(), "it %d resubstituteF_MT: %s", it, ef.lastError().c_str());
        std::vector<float> so(ef.allPoints.size());
        oracle_resubstitute(ow, ef.lastX.data(), 1e-5, so.data());
        double num = 0, den = 0;
        for (size_t q = 0; q < so.size(); q++) {
            num += (ef.allPoints[q]->step - so[q]) * (double)(ef.allPoints[q]->step - so[q]);
            den += (double)so[q] * so[q];
        }
        CHECK(std::sqrt(num) <= 1e-3 * std::sqrt(den) + 1e-12, "it %d: resubstitute", it);
        CHECK(calib->step[0] == -ef.lastX[0] && ef.frames[N - 1]->step[0] == -ef.lastX[4 + 8 * (N - 1)],
              "it %d: calibration / frame steps", it);

        // doStepFromBackup (test harness) + setPrecalcValues' setDeltaF
        for (auto &F : ef.frames)
            for (int k = 0; k < 8; k++) F->state[k] += F->step[k];
        for (auto &p : ef.allPoints) {
            p->setIdepth(p->idepth + p->step);
            p->setIdepthZero(p->idepth);
        }
        ef.setDeltaF(calib);
        energies(it);
    }

    void energies(int it) {
        const int N = ef.nFrames;
        std::vector<double> prior(8 * N), dprior(8 * N), delta(8 * N);
        for (int f = 0; f < N; f++) {
            std::memcpy(&prior[8 * f], ef.frames[f]->prior, 64);
            std::memcpy(&dprior[8 * f], ef.frames[f]->delta_prior, 64);
            std::memcpy(&delta[8 * f], ef.frames[f]->delta, 64);
        }
        std::vector<float> dd, pf;
        for (auto &p : ef.allPoints) {
            dd.push_back(p->deltaF);
            pf.push_back(p->priorF);
        }
        const double eL = ef.calcLEnergyF_MT();
        const double eLo = oracle_calc_l_energy(N, prior.data(), dprior.data(), ef.cPrior, ef.cDeltaF, (int)dd.size(),
                                                dd.data(), pf.data());
        CHECK(eL == eLo, "it %d: calcLEnergyF_MT %.17g vs %.17g", it, eL, eLo);
        const double eM = ef.calcMEnergyF();
        const double eMo = oracle_calc_m_energy(N, HMo.data(), bMo.data(), ef.cDeltaF, delta.data());
        CHECK(std::fabs(eM - eMo) <= 1e-4 * std::fabs(eMo) + 1e-12, "it %d: calcMEnergyF %.17g vs %.17g", it, eM, eMo);
    }
};

static int gpu_tests() {
    Synth S(6, 800, 320, 240, 21);
    Graph G(S);
    auto ef = std::make_shared<EnergyFunctional>(0);
    CHECK(ef->ok(), "context: %s", ef->lastError().c_str());
    if (!ef->ok()) return 1;
    G.insertInto(*ef);
    Cycle C(S, *ef);
    // FullSystem::optimize: resetOOB of every active residual, then GN iterations
    ef->resetOOB();
    for (int it = 0; it < 3; it++) C.iteration(it, G.calib, it == 0);

    // flagPointsForRemoval: frame 0 leaves; its points and every 7th point are marginalised, a few
    // points are dropped (OUT)
    auto f0 = ef->frames[0];
    f0->flaggedForMarginalization = true;
    int k = 0, nmarg = 0, nout = 0;
    for (auto &p : ef->allPoints) {
        if (p->host.lock() == f0 || k % 7 == 0) {
            p->status = PointStatus::MARGINALIZED;
            nmarg++;
        } else if (k % 29 == 3) {
            p->status = PointStatus::OUT;
            nout++;
        }
        k++;
    }
    {
        // FullSystem::flagPointsForRemoval's per-residual loop (FullSystem.cc:1390-1398) on the
        // MARGINALIZED points, against the oracle's fresh linearisation of the same window state
        OracleWin O(S, *ef);
        oracle_window *ow = oracle_create(&O.w);
        oracle_reset_oob(ow);
        double eo[3];
        oracle_linearize_all(ow, 0, eo);
        const int R = (int)O.order.size();
        std::vector<int8_t> ns(R), st(R);
        std::vector<float> se(R), ewo(R), ctr(3 * R), jp(8 * R), rbs(R);
        std::vector<uint8_t> fl(R);
        oracle_get_residuals(ow, ns.data(), st.data(), se.data(), ewo.data(), ctr.data(), fl.data(), jp.data(),
                             rbs.data());
        oracle_apply_res(ow);
        std::vector<float> se2(R), jp2(8 * R);
        oracle_get_residuals(ow, nullptr, nullptr, se2.data(), nullptr, nullptr, nullptr, jp2.data(), nullptr);
        oracle_destroy(ow);
        std::unordered_map<const PointFrameResidual *, int> idx;
        for (int k = 0; k < R; k++) idx[O.order[k]] = k;
        const long passes0 = ef->devicePasses();
        int checked = 0, bad = 0, ngood = 0;
        for (auto &p : ef->allPoints) {
            if (p->status != PointStatus::MARGINALIZED) continue;
            for (auto &r : p->residuals) {
                r->resetOOB();
                const double e = r->linearize(G.calib);
                r->isLinearized = false;
                r->applyRes(true);
                if (r->isActive()) {
                    r->fixLinearizationF(ef);
                    ngood++;
                }
                const int k = idx.at(r.get());
                const bool oob = ns[k] == LDSO_BA_RES_OOB;
                const double e_ref = oob ? 0.0 : (double)se2[k];
                bool ok = r->state_NewState == ns[k] && e == e_ref && (float)r->state_NewEnergyWithOutlier == ewo[k] &&
                          r->isActiveAndIsGoodNEW == (ns[k] == LDSO_BA_RES_IN);
                if (!oob) ok = ok && std::memcmp(r->centerProjectedTo, &ctr[3 * k], 12) == 0;
                if (r->isActive()) ok = ok && std::memcmp(r->JpJdF, &jp2[8 * k], 32) == 0;
                bad += !ok;
                checked++;
            }
        }
        CHECK(checked > 0 && bad == 0, "flagPointsForRemoval loop: %d of %d residuals differ from the oracle", bad,
              checked);
        CHECK(ngood > 0, "no active residual among the marginalised points");
        CHECK(ef->devicePasses() == passes0 + 1, "per-residual linearize: %ld device passes for one call site",
              ef->devicePasses() - passes0);
        CHECK(ef->ok(), "per-residual linearize: %s", ef->lastError().c_str());
    }
    {
        OracleWin O(S, *ef);
        oracle_window *ow = oracle_create(&O.w);  // marginalisation relinearises from resetOOB
        std::vector<int> pts;
        for (size_t q = 0; q < ef->allPoints.size(); q++)
            if (ef->allPoints[q]->status == PointStatus::MARGINALIZED) pts.push_back((int)q);
        const int n = 8 * ef->nFrames + 4;
        std::vector<double> H((size_t)n * n), b(n);
        oracle_marginalize_points(ow, (int)pts.size(), pts.data(), ef->adHTdeltaF.data(), H.data(), b.data());
        for (int i = 0; i < n; i++) {
            C.bMo[i] += 0.25 * b[i];
            for (int j = 0; j < n; j++) C.HMo(i, j) += 0.25 * H[(size_t)i * n + j];
        }
        oracle_destroy(ow);
    }
    const int pts_before = ef->nPoints;
    ef->marginalizePointsF();
    CHECK(ef->ok(), "marginalizePointsF: %s", ef->lastError().c_str());
    CHECK(ef->nPoints == pts_before - nmarg && ef->resInM > 0, "marginalizePointsF removed %d of %d points",
          pts_before - ef->nPoints, nmarg);
    CHECK(block_err(ef->HM, C.HMo) < 1e-4, "HM after marginalizePointsF: %.2e", block_err(ef->HM, C.HMo));
    CHECK(rel(ef->bM.data(), C.bMo.data(), ef->bM.size()) < 1e-4, "bM after marginalizePointsF");
    ef->dropPointsF();
    CHECK(ef->nPoints == pts_before - nmarg - nout, "dropPointsF");

    // FullSystem::marginalizeFrame: the Schur step, then every observation of frame 0 dropped
    {
        const int N = ef->nFrames, n = 8 * N + 4;
        ldso_ba_frame_state s0;
        std::memset(&s0, 0, sizeof(s0));
        std::memcpy(s0.world_to_cam_evalpt, f0->worldToCam_evalPT, sizeof(f0->worldToCam_evalPT));
        std::memcpy(s0.state, f0->state, sizeof(f0->state));
        std::memcpy(s0.state_zero, f0->state_zero, sizeof(f0->state_zero));
        s0.ab_exposure = f0->ab_exposure;
        s0.is_first_frame = 1;
        double pr[8], dl[8], dp[8];
        oracle_frame_take_data(1, &s0, pr, dl, dp);
        MatXX Ho(n - 8, n - 8);
        VecX bo(n - 8);
        ldso_ba_marginalize_frame(N, f0->idx, C.HMo.data(), C.bMo.data(), pr, dp, Ho.data(), bo.data());
        C.HMo = Ho;
        C.bMo = bo;
    }
    ef->marginalizeFrame(f0);
    CHECK(ef->ok() && ef->nFrames == S.N - 1 && ef->HM.rows() == 8 * (S.N - 1) + 4, "marginalizeFrame: %s",
          ef->lastError().c_str());
    CHECK(block_err(ef->HM, C.HMo) < 1e-4, "HM after marginalizeFrame: %.2e", block_err(ef->HM, C.HMo));
    for (auto &p : std::vector<shared_ptr<PointHessian>>(ef->allPoints)) {
        const auto rs = p->residuals;
        for (auto &r : rs)
            if (r->target.lock() == f0) ef->dropResidual(r);
    }
    ef->makeIDX();
    ef->setAdjointsF(G.calib);
    ef->setDeltaF(G.calib);
    for (auto &p : ef->allPoints)
        for (auto &r : p->residuals) CHECK(r->target.lock() != f0 && r->host.lock() != f0, "stale observation");

    // optimize again on the 5-frame window, HM / bM in the solve
    ef->resetOOB();
    for (int it = 0; it < 2; it++) C.iteration(3 + it, G.calib, it == 0);
    return 0;
}

// EnergyFunctional::optimize (FullSystem::optimize's loop on the device) against the C ABI's
// ldso_ba_optimize on the same window, bit for bit; then the lazily written-back residual fields
// and a FullSystem-style linearizeAll(true) against the oracle
static int gpu_optimize_tests() {
    Synth S(6, 800, 320, 240, 22);
    Graph G(S);
    auto ef = std::make_shared<EnergyFunctional>(0);
    CHECK(ef->ok(), "context: %s", ef->lastError().c_str());
    if (!ef->ok()) return 1;
    G.insertInto(*ef);
    // the same window through the C ABI, caller order = the synthetic point order
    const int N = S.N, n = 8 * N + 4;
    std::vector<float> precalc((size_t)N * N * LDSO_BA_PRECALC_STRIDE);
    std::vector<double> adH((size_t)N * N * 64), adT((size_t)N * N * 64), cp(4), fp(8 * N), fd(8 * N), fdp(8 * N);
    ldso_ba_frame_precalc(N, S.fs.data(), S.calib, precalc.data());
    ldso_ba_set_adjoints(N, S.fs.data(), adH.data(), adT.data(), cp.data());
    ldso_ba_frame_take_data(N, S.fs.data(), nullptr, fp.data(), fd.data(), fdp.data());
    const float cdelta[4] = {0, 0, 0, 0};
    ldso_ba_window w;
    std::memset(&w, 0, sizeof(w));
    w.n_frames = N;
    w.n_points = S.P;
    w.n_residuals = S.R;
    w.width = S.w;
    w.height = S.h;
    std::memcpy(w.calib, S.calib, sizeof(w.calib));
    w.dI = S.dI.data();
    w.frame_energy_th = S.th.data();
    w.precalc = precalc.data();
    w.ad_host = adH.data();
    w.ad_target = adT.data();
    w.c_prior = cp.data();
    w.c_delta = cdelta;
    w.frame_prior = fp.data();
    w.frame_delta_prior = fdp.data();
    w.point_host = S.ph.data();
    w.point_data = S.pd.data();
    w.point_res_begin = S.rb.data();
    w.res_target = S.rt.data();
    w.res_state = S.rs.data();
    w.res_energy = S.re.data();
    w.res_flags = S.rf.data();
    ldso_ba_ctx *raw = nullptr;
    CHECK(ldso_ba_create(0, &raw) == 0 && ldso_ba_load(raw, 1, &w, 0, 1) == 0, "raw context: %s", ldso_ba_last_error());
    std::vector<double> ns((size_t)7 * n), e_raw(3 * 4), cv(4), cz(4), co(4);
    ldso_ba_nullspaces(N, S.fs.data(), ns.data());
    for (int k = 0; k < 4; k++) cv[k] = cz[k] = G.calib->value[k];
    std::vector<ldso_ba_frame_state> fo(N);
    std::vector<float> id(S.P);
    int32_t its_raw = -1, status_raw = -1;
    CHECK(ldso_ba_optimize(raw, 3, nullptr, S.fs.data(), cv.data(), cz.data(), ns.data(), e_raw.data(), fo.data(),
                           co.data(), id.data(), &its_raw, &status_raw) == 0,
          "ldso_ba_optimize: %s", ldso_ba_last_error());

    std::vector<Vec3> e_face;
    const long passes0 = ef->devicePasses();
    bool lost = true;
    int its_face = -1;
    const Vec3 last = ef->optimize(3, G.calib, &e_face, &lost, &its_face);
    CHECK(ef->ok(), "EnergyFunctional::optimize: %s", ef->lastError().c_str());
    CHECK(!lost && status_raw != LDSO_BA_OPT_LOST, "optimize reported lost");
    CHECK(its_face == its_raw && its_raw >= 1 && its_raw <= 3, "iterations: face %d, C ABI %d", its_face, its_raw);
    CHECK(ef->devicePasses() == passes0 + 1 + its_raw, "optimize(3) ran %ld passes", ef->devicePasses() - passes0);
    CHECK(e_face.size() == 4, "energy history size %zu", e_face.size());
    for (size_t s2 = 0; s2 < e_face.size() && s2 < 4; s2++)
        CHECK(e_face[s2][0] == e_raw[3 * s2] && e_face[s2][2] == e_raw[3 * s2 + 2], "optimize energy %zu: %.17g vs %.17g",
              s2, e_face[s2][0], e_raw[3 * s2]);
    CHECK(last[0] == e_raw[9] && ef->resInA == (int)e_raw[11], "optimize return value");
    for (int f = 0; f < N; f++)
        CHECK(std::memcmp(G.frames[f]->state, fo[f].state, sizeof(fo[f].state)) == 0, "frame %d state after optimize", f);
    for (int k = 0; k < 4; k++) CHECK(G.calib->value[k] == co[k], "calibration after optimize");
    int badp = 0;
    for (int p = 0; p < S.P; p++)
        badp += !(G.points[p]->idepth == id[p] && G.points[p]->idepth_zero == id[p] && G.points[p]->deltaF == 0.f);
    CHECK(badp == 0, "%d points' idepth differ after optimize", badp);

    // lazy write-back: the residual fields equal the C ABI context's after the same loop
    ef->syncResiduals();
    {
        std::vector<int8_t> rns(S.R), rst(S.R);
        std::vector<float> rse(S.R), rew(S.R), rctr(3 * S.R), rjp(8 * S.R);
        std::vector<uint8_t> rfl(S.R);
        ldso_ba_get_residuals(raw, 0, rns.data(), rst.data(), rse.data(), rew.data(), rctr.data(), rfl.data(), rjp.data(),
                              nullptr);
        int bad = 0, k = 0;
        for (int p = 0; p < S.P; p++)
            for (auto &r : G.points[p]->residuals) {
                bad += !(r->state_state == rst[k] && r->state_NewState == rns[k] && (float)r->state_energy == rse[k] &&
                         (float)r->state_NewEnergyWithOutlier == rew[k] &&
                         r->isActiveAndIsGoodNEW == ((rfl[k] & LDSO_BA_FLAG_ACTIVE) != 0) &&
                         std::memcmp(r->centerProjectedTo, &rctr[3 * k], 12) == 0 &&
                         (!r->isActiveAndIsGoodNEW || std::memcmp(r->JpJdF, &rjp[8 * k], 32) == 0));
                k++;
            }
        CHECK(bad == 0, "%d residuals differ from ldso_ba_optimize's after syncResiduals", bad);
        std::vector<float> th(N);
        ldso_ba_get_frame_energy_th(raw, 0, th.data());
        for (int f = 0; f < N; f++) CHECK(G.frames[f]->frameEnergyTH == th[f], "frameEnergyTH[%d] after optimize", f);
    }
    ldso_ba_destroy(raw);

    // FullSystem::optimize's tail: linearizeAll(true) on the stepped state, against the oracle
    OracleWin O(S, *ef, G.calib->value_scaledf);  // optimize stepped the calibration too
    oracle_window *ow = oracle_create(&O.w);
    double eo[3];
    oracle_linearize_all(ow, 1, eo);
    const Vec3 ef_fix = ef->linearizeAll(true);
    CHECK(ef->ok(), "linearizeAll(true): %s", ef->lastError().c_str());
    CHECK(ef_fix[2] == eo[2] && std::fabs(ef_fix[0] - eo[0]) <= 1e-9 * std::fabs(eo[0]), "fix pass energy %.17g vs %.17g",
          ef_fix[0], eo[0]);
    const int R = (int)O.order.size();
    std::vector<int8_t> ons(R), ost(R);
    std::vector<float> ose(R), oew(R), octr(3 * R), ojp(8 * R), orb(R);
    std::vector<uint8_t> ofl(R);
    oracle_get_residuals(ow, ons.data(), ost.data(), ose.data(), oew.data(), octr.data(), ofl.data(), ojp.data(),
                         orb.data());
    {   // FixPassResult against the oracle's reductor bookkeeping (FullSystem.cc:1799-1822)
        const auto &fx = ef->fixPassResult();
        std::map<const PointFrameResidual *, int> idx;
        for (int k = 0; k < R; k++) idx[O.order[k]] = k;
        int n_inactive = 0, bad_rm = 0;
        for (int k = 0; k < R; k++) n_inactive += !(ofl[k] & 1);
        for (const PointFrameResidual *r : fx.toRemove) bad_rm += (ofl[idx.at(r)] & 1) != 0;
        CHECK(bad_rm == 0 && (int)fx.toRemove.size() == n_inactive, "toRemove: %zu listed, %d inactive, %d wrong",
              fx.toRemove.size(), n_inactive, bad_rm);
        int bad_pt = 0, bad_last = 0;
        for (size_t q = 0; q < ef->allPoints.size(); q++) {
            float mx = 0;
            int cnt = 0;
            int last[2] = {-1, -1};  // lastResiduals[0] / [1]: the residuals to frames N-1 / N-2
            for (const auto &r : ef->allPoints[q]->residuals) {
                const int k = idx.at(r.get());
                if ((ofl[k] & 1) && r->isNew) {
                    mx = std::max(mx, orb[k]);
                    cnt++;
                }
                const int t = r->target.lock()->idx;
                if (t >= N - 2) last[N - 1 - t] = ost[k];
            }
            bad_pt += fx.maxRelBS[q] != mx || fx.numGood[q] != cnt;
            bad_last += fx.lastState[2 * q] != last[0] || fx.lastState[2 * q + 1] != last[1];
        }
        CHECK(bad_pt == 0, "maxRelBS / numGood of %d points differ from the oracle", bad_pt);
        CHECK(bad_last == 0, "lastResiduals' states of %d points differ from the oracle", bad_last);
    }
    ef->syncResiduals();
    int bad = 0;
    for (int k = 0; k < R; k++) {
        const PointFrameResidual &r = *O.order[k];
        // an OOB residual returns at once (Residuals.cc:19-23): its centre / relBS are the previous
        // pass's, which a freshly created oracle window does not have
        const bool oob = ons[k] == LDSO_BA_RES_OOB;
        bad += !(r.state_NewState == ons[k] && r.state_state == ost[k] && (float)r.state_energy == ose[k] &&
                 (float)r.state_NewEnergyWithOutlier == oew[k] && (oob || r.relBS == orb[k]) &&
                 (oob || std::memcmp(r.centerProjectedTo, &octr[3 * k], 12) == 0));
    }
    CHECK(bad == 0, "linearizeAll(true) after optimize: %d of %d residuals differ from the oracle", bad, R);
    oracle_destroy(ow);
    return 0;
}

int main(int argc, char **argv) {
    const bool cpu = argc > 1 && std::strcmp(argv[1], "--cpu") == 0;
    if (cpu) {
        cpu_tests();
    } else {
        gpu_tests();
        gpu_optimize_tests();
    }
    std::printf("%s: %d failure(s)\n", cpu ? "cpu" : "gpu", g_fail);
    return g_fail ? 1 : 0;
}
