// test_energy_functional.cpp -- the C++ host face (include/ldso_amd/energy_functional.h) driven
// the way FullSystem::optimize drives LDSO's EnergyFunctional, checked against the CPU oracle
// (oracle/, test infrastructure) on the same seeded synthetic window.
//
//   test_energy_functional --cpu   structure bookkeeping and the no-device error path
//   test_energy_functional         GPU parity over two GN iterations (load, then update path)
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/ldso_amd/energy_functional.h"
#include "../../ldso_amd/csrc/synth.h"
#include "../../oracle/ldso_oracle.h"

using namespace ldso_amd;

static int g_fail = 0;
#define CHECK(cond, ...)                                  \
    do {                                                  \
        if (!(cond)) {                                    \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);                     \
            std::printf("\n");                            \
            g_fail++;                                     \
        }                                                 \
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

// the LDSO object graph of a synthetic window
struct Graph {
    CalibHessian calib;
    std::vector<std::unique_ptr<FrameHessian>> frames;
    std::vector<std::unique_ptr<PointHessian>> points;
    std::vector<std::unique_ptr<PointFrameResidual>> res;
    explicit Graph(const Synth &S) {
        calib.wG0 = S.w;
        calib.hG0 = S.h;
        std::memcpy(calib.value_scaledf, S.calib, sizeof(S.calib));
        for (int f = 0; f < S.N; f++) {
            auto F = std::make_unique<FrameHessian>();
            std::memcpy(F->worldToCam_evalPT, S.fs[f].world_to_cam_evalpt, sizeof(F->worldToCam_evalPT));
            std::memcpy(F->state, S.fs[f].state, sizeof(F->state));
            std::memcpy(F->state_zero, S.fs[f].state_zero, sizeof(F->state_zero));
            F->ab_exposure = S.fs[f].ab_exposure;
            F->isFirstFrame = S.fs[f].is_first_frame != 0;
            F->dI = &S.dI[(size_t)f * S.w * S.h * 3];
            F->frameEnergyTH = S.th[f];
            frames.push_back(std::move(F));
        }
        for (int p = 0; p < S.P; p++) {
            auto Pt = std::make_unique<PointHessian>();
            const float *d = &S.pd[(size_t)p * LDSO_BA_POINT_STRIDE];
            Pt->host = frames[S.ph[p]].get();
            Pt->u = d[0];
            Pt->v = d[1];
            Pt->idepth_scaled = d[2];
            Pt->idepth_zero_scaled = d[3];
            Pt->priorF = d[4];
            Pt->deltaF = d[5];
            std::memcpy(Pt->color, d + 8, sizeof(Pt->color));
            std::memcpy(Pt->weights, d + 16, sizeof(Pt->weights));
            points.push_back(std::move(Pt));
        }
        for (int p = 0; p < S.P; p++)
            for (int k = S.rb[p]; k < S.rb[p + 1]; k++) {
                auto r = std::make_unique<PointFrameResidual>();
                r->point = points[p].get();
                r->host = points[p]->host;
                r->target = frames[S.rt[k]].get();
                r->state_state = (ResState)S.rs[k];
                r->state_energy = S.re[k];
                r->isNew = (S.rf[k] & LDSO_BA_FLAG_NEW) != 0;
                r->isActiveAndIsGoodNEW = (S.rf[k] & LDSO_BA_FLAG_ACTIVE) != 0;
                res.push_back(std::move(r));
            }
    }
    void insertInto(EnergyFunctional &ef) {
        for (auto &F : frames) ef.insertFrame(F.get(), calib);
        for (auto &P : points) ef.insertPoint(P.get());
        for (auto &r : res) ef.insertResidual(r.get());
        ef.makeIDX();
    }
};

// The oracle's window in the EnergyFunctional's (makeIDX) point order.
struct OracleWin {
    std::vector<int32_t> ph, rb, rt;
    std::vector<float> pd, re, precalc, th;
    std::vector<int8_t> rs;
    std::vector<uint8_t> rf;
    std::vector<double> adH, adT, cp, fp, fd, fdp;
    std::vector<float> cdelta;
    std::vector<ldso_ba_frame_state> fs;
    std::vector<PointFrameResidual *> order;
    ldso_ba_window w;
    OracleWin(const Synth &S, EnergyFunctional &ef) {
        const int N = S.N;
        fs.resize(N);
        for (int f = 0; f < N; f++) {
            const FrameHessian &F = *ef.frames[f];
            std::memset(&fs[f], 0, sizeof(fs[f]));
            std::memcpy(fs[f].world_to_cam_evalpt, F.worldToCam_evalPT, sizeof(F.worldToCam_evalPT));
            std::memcpy(fs[f].state, F.state, sizeof(F.state));
            std::memcpy(fs[f].state_zero, F.state_zero, sizeof(F.state_zero));
            fs[f].ab_exposure = F.ab_exposure;
            fs[f].is_first_frame = F.isFirstFrame;
        }
        precalc.resize((size_t)N * N * LDSO_BA_PRECALC_STRIDE);
        adH.resize((size_t)N * N * 64);
        adT.resize((size_t)N * N * 64);
        cp.resize(4);
        fp.resize(8 * N);
        fd.resize(8 * N);
        fdp.resize(8 * N);
        cdelta.assign(4, 0.f);
        oracle_frame_precalc(N, fs.data(), S.calib, precalc.data());
        oracle_set_adjoints(N, fs.data(), adH.data(), adT.data(), cp.data());
        oracle_frame_take_data(N, fs.data(), fp.data(), fd.data(), fdp.data());
        th = S.th;
        rb.push_back(0);
        for (PointHessian *p : ef.allPoints) {
            ph.push_back(p->host->idx);
            float d[LDSO_BA_POINT_STRIDE] = {p->u, p->v, p->idepth_scaled, p->idepth_zero_scaled, p->priorF, p->deltaF};
            std::memcpy(d + 8, p->color, sizeof(p->color));
            std::memcpy(d + 16, p->weights, sizeof(p->weights));
            pd.insert(pd.end(), d, d + LDSO_BA_POINT_STRIDE);
            for (PointFrameResidual *r : p->residuals) {
                rt.push_back(r->target->idx);
                rs.push_back((int8_t)r->state_state);
                re.push_back(r->state_energy);
                rf.push_back((r->isActiveAndIsGoodNEW ? 1 : 0) | (r->isNew ? 2 : 0));
                order.push_back(r);
            }
            rb.push_back((int32_t)rt.size());
        }
        std::memset(&w, 0, sizeof(w));
        w.n_frames = N;
        w.n_points = (int)ph.size();
        w.n_residuals = (int)rt.size();
        w.width = S.w;
        w.height = S.h;
        std::memcpy(w.calib, S.calib, sizeof(w.calib));
        w.dI = S.dI.data();
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

static int cpu_tests() {
    Synth S(4, 60, 160, 120, 3);
    Graph G(S);
    EnergyFunctional ef(1 << 20);  // no such device: reported, never thrown
    CHECK(!ef.ok(), "creating a context on a missing device must fail");
    CHECK(!ef.lastError().empty(), "error message expected");
    G.insertInto(ef);
    CHECK(ef.nFrames == 4 && ef.nPoints == 60 && ef.nResiduals == 180, "counts %d %d %d", ef.nFrames, ef.nPoints,
          ef.nResiduals);
    for (size_t i = 1; i < ef.allPoints.size(); i++)
        CHECK(ef.allPoints[i - 1]->host->idx <= ef.allPoints[i]->host->idx, "makeIDX host order");
    ef.dropResidual(G.res[0].get());
    CHECK(ef.nResiduals == 179 && G.points[0]->residuals.size() == 2, "dropResidual");
    ef.removePoint(G.points[1].get());
    CHECK(ef.nPoints == 59 && ef.nResiduals == 176, "removePoint");
    const Vec3 e = ef.linearizeAll(false);
    CHECK(e[0] == 0 && !ef.ok(), "linearize without a device reports an error");
    return 0;
}

static double rel(const std::vector<double> &a, const std::vector<double> &b) {
    double num = 0, den = 0;
    for (size_t i = 0; i < a.size(); i++) {
        num += (a[i] - b[i]) * (a[i] - b[i]);
        den += b[i] * b[i];
    }
    return std::sqrt(num / (den > 0 ? den : 1));
}

static void compare_iteration(const Synth &S, EnergyFunctional &ef, oracle_window *ow, OracleWin &O, const Vec3 &e,
                              int it) {
    double eo[3];
    const int R = ef.nResiduals, N = ef.nFrames, n = 8 * N + 4;
    std::vector<double> HA(n * n), bA(n), HL(n * n), bL(n), Hsc(n * n), bsc(n);
    oracle_linearize_all(ow, 0, eo);  // the pass ldso_ba_linearize(0, 1) runs
    oracle_apply_res(ow);
    oracle_accumulate(ow, HA.data(), bA.data(), HL.data(), bL.data(), Hsc.data(), bsc.data());
    CHECK(e[2] == eo[2], "it %d: #IN %g vs %g", it, e[2], eo[2]);
    CHECK(std::fabs(e[0] - eo[0]) <= 1e-9 * std::fabs(eo[0]), "it %d: energy %.17g vs %.17g", it, e[0], eo[0]);
    std::vector<int8_t> ns(R), st(R);
    std::vector<float> se(R), ewo(R), ctr(3 * R), jp(8 * R), rb(R);
    std::vector<uint8_t> fl(R);
    oracle_get_residuals(ow, ns.data(), st.data(), se.data(), ewo.data(), ctr.data(), fl.data(), jp.data(), rb.data());
    int bad = 0;
    for (int k = 0; k < R; k++) {
        const PointFrameResidual &r = *O.order[k];
        bad += r.state_NewState != ns[k] || r.state_state != st[k] || r.state_energy != se[k] ||
               r.state_NewEnergyWithOutlier != ewo[k] || r.isActiveAndIsGoodNEW != ((fl[k] & 1) != 0) ||
               std::memcmp(r.centerProjectedTo, &ctr[3 * k], 12) != 0 ||
               (r.isActiveAndIsGoodNEW && std::memcmp(r.JpJdF, &jp[8 * k], 32) != 0);
    }
    CHECK(bad == 0, "it %d: %d residuals differ from the oracle", it, bad);
    std::vector<float> th(N);
    oracle_get_frame_energy_th(ow, th.data());
    for (int f = 0; f < N; f++) CHECK(ef.frames[f]->frameEnergyTH == th[f], "it %d: frameEnergyTH[%d]", it, f);
    // system (tolerance: reassociated float partial sums), solve on the same system, resubstitute
    ef.solveSystemF(it, 1e-5);
    CHECK(ef.ok(), "solveSystemF: %s", ef.lastError().c_str());
    CHECK(rel(ef.HA_top, HA) < 1e-5 && rel(ef.H_sc, Hsc) < 1e-5 && rel(ef.bA_top, bA) < 1e-5 &&
              rel(ef.b_sc, bsc) < 1e-5,
          "it %d: stitched system %.2e %.2e", it, rel(ef.HA_top, HA), rel(ef.H_sc, Hsc));
    std::vector<double> ns7((size_t)7 * n), xo(n);
    oracle_nullspaces(N, O.fs.data(), ns7.data());
    oracle_solve_system(N, it, 1e-5, ef.HA_top.data(), ef.bA_top.data(), ef.HL_top.data(), ef.bL_top.data(), nullptr,
                        nullptr, ef.H_sc.data(), ef.b_sc.data(), ns7.data(), 7, xo.data());
    CHECK(rel(ef.lastX, xo) < 1e-9, "it %d: solve %.2e", it, rel(ef.lastX, xo));
    ef.resubstituteF_MT(ef.lastX, 1e-5);
    std::vector<float> so(ef.nPoints);
    oracle_resubstitute(ow, ef.lastX.data(), 1e-5, so.data());
    double num = 0, den = 0;
    for (int q = 0; q < ef.nPoints; q++) {
        num += (ef.allPoints[q]->step - so[q]) * (double)(ef.allPoints[q]->step - so[q]);
        den += (double)so[q] * so[q];
    }
    CHECK(std::sqrt(num) <= 1e-3 * std::sqrt(den) + 1e-12, "it %d: resubstitute", it);
    (void)S;
}

static int gpu_tests() {
    Synth S(6, 800, 320, 240, 21);
    Graph G(S);
    EnergyFunctional ef(0);
    CHECK(ef.ok(), "context: %s", ef.lastError().c_str());
    if (!ef.ok()) return 1;
    G.insertInto(ef);
    OracleWin O(S, ef);
    oracle_set_threads(0);
    oracle_window *ow = oracle_create(&O.w);
    // iteration 0: FullSystem::optimize's resetOOB + linearizeAll(false) + solve + resubstitute
    ef.resetOOB();
    oracle_reset_oob(ow);
    Vec3 e = ef.linearizeAll(false);
    CHECK(ef.ok(), "linearizeAll: %s", ef.lastError().c_str());
    compare_iteration(S, ef, ow, O, e, 0);
    // iteration 1: a step on the newest frame (the update path, no structural change)
    FrameHessian *nf = ef.frames.back();
    nf->state[0] += 1e-4;
    nf->state[4] -= 2e-4;
    OracleWin O2(S, ef);
    oracle_update(ow, &O2.w);
    e = ef.linearizeAll(false);
    CHECK(ef.ok(), "linearizeAll (update): %s", ef.lastError().c_str());
    compare_iteration(S, ef, ow, O2, e, 2);
    oracle_destroy(ow);
    return 0;
}

int main(int argc, char **argv) {
    const bool cpu = argc > 1 && std::strcmp(argv[1], "--cpu") == 0;
    if (cpu) cpu_tests();
    else gpu_tests();
    std::printf("%s: %d failure(s)\n", cpu ? "cpu" : "gpu", g_fail);
    return g_fail ? 1 : 0;
}
