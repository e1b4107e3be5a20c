// face_bench.cpp -- times the C++ host face (include/ldso_amd/energy_functional.h) the way LDSO's
// FullSystem drives it, on one synthetic S7 window (7 keyframes, 2000 points, 640x480), beside
// the C ABI's ldso_ba_optimize on the same window in the same process.  Run by bench.py
// (cpp_face); prints one JSON object.
//
//   optimize        EnergyFunctional::optimize(6) with the early exit off (th_opt_iterations = 0:
//                   all 6 iterations, so per-iteration times compare across calls and with the C
//                   ABI): FullSystem::optimize's GN loop on the device plus the face's write-back
//                   (frame states, calibration, point idepths, setDeltaF), host clock per call;
//                   iterations_default: what the reference's exits (canbreak) leave of the 6
//   shim            INTEGRATION.md §3's reference-side forwarding around one FullSystem::optimize
//                   (copy-in, optimize, copy-back, linearizeAll(true), residual / point copy-out)
//                   on stand-ins for the reference's heap objects: the copy loops alone, through
//                   std::unordered_map (as §3 wrote it in round 3) and by walking the face's own
//                   containers with the objects' `user` back-pointers (§3 now)
//   optimize_full   the same + setAdjointsF + setDeltaF + linearizeAll(true) with the complete
//                   residual / point write-back: everything FullSystem::optimize asks of the
//                   backend after the frontend's setEvalPT
//   c_abi_optimize  ldso_ba_optimize(6) on a context loaded with the same window (no face)
//   flag_loop       FullSystem::flagPointsForRemoval's per-residual resetOOB / linearize /
//                   applyRes over every residual of 10 % of the points (one device pass)
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <random>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/ldso_amd/energy_functional.h"
#include "../csrc/synth.h"

using namespace ldso_amd;
using Clock = std::chrono::steady_clock;

static double ms_since(Clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

int main(int argc, char **argv) {
    const int N = 7, P = 2000, W = 640, H = 480, n_its = 6;
    const int reps = argc > 1 ? std::atoi(argv[1]) : 10;
    const int R = P * (N - 1);
    std::vector<ldso_ba_frame_state> fs(N);
    std::vector<float> dI((size_t)N * W * H * 3), th(N), pd((size_t)P * LDSO_BA_POINT_STRIDE), re(R);
    std::vector<int32_t> ph(P), rb(P + 1), rt(R);
    std::vector<int8_t> rs(R);
    std::vector<uint8_t> rf(R);
    float calib[4];
    ldso_synth_params prm = {N, P, W, H, 1, 0.05f, 0.01f, 1e-3f, 0.04f};
    if (ldso_synth_fill(&prm, fs.data(), dI.data(), calib, th.data(), ph.data(), pd.data(), rb.data(), rt.data(),
                        rs.data(), re.data(), rf.data())) {
        std::printf("{\"error\": \"synth\"}\n");
        return 1;
    }
    // the LDSO object graph (shared_ptr ownership, as the reference)
    auto HCalib = std::make_shared<CalibHessian>();
    HCalib->wG0 = W;
    HCalib->hG0 = H;
    std::memcpy(HCalib->value_scaledf, calib, sizeof(calib));
    for (int k = 0; k < 4; k++) HCalib->value[k] = HCalib->value_zero[k] = (double)calib[k] * (1.0 / 50.0);
    std::vector<shared_ptr<FrameHessian>> frames;
    std::vector<shared_ptr<PointHessian>> points;
    for (int f = 0; f < N; f++) {
        auto F = std::make_shared<FrameHessian>();
        F->frameID = f;
        std::memcpy(F->worldToCam_evalPT, fs[f].world_to_cam_evalpt, sizeof(F->worldToCam_evalPT));
        std::memcpy(F->state, fs[f].state, sizeof(F->state));
        std::memcpy(F->state_zero, fs[f].state_zero, sizeof(F->state_zero));
        F->ab_exposure = fs[f].ab_exposure;
        F->dI = &dI[(size_t)f * W * H * 3];
        F->frameEnergyTH = th[f];
        frames.push_back(F);
    }
    auto ef = std::make_shared<EnergyFunctional>(0);
    if (!ef->ok()) {
        std::printf("{\"error\": \"%s\"}\n", ef->lastError().c_str());
        return 1;
    }
    for (auto &F : frames) ef->insertFrame(F, HCalib);
    for (int p = 0; p < P; p++) {
        auto Pt = std::make_shared<PointHessian>();
        const float *d = &pd[(size_t)p * LDSO_BA_POINT_STRIDE];
        Pt->host = frames[ph[p]];
        Pt->u = d[0];
        Pt->v = d[1];
        Pt->setIdepth(d[2]);
        Pt->setIdepthZero(d[3]);
        std::memcpy(Pt->color, d + 8, sizeof(Pt->color));
        std::memcpy(Pt->weights, d + 16, sizeof(Pt->weights));
        for (int k = rb[p]; k < rb[p + 1]; k++) {
            auto r = std::make_shared<PointFrameResidual>(Pt, frames[ph[p]], frames[rt[k]]);
            r->isNew = true;
            Pt->residuals.push_back(r);
        }
        points.push_back(Pt);
        ef->insertPoint(Pt);
        for (auto &r : Pt->residuals) ef->insertResidual(r);
    }
    ef->makeIDX();
    ef->setAdjointsF(HCalib);
    ef->setDeltaF(HCalib);

    // the reference's exits on the first call (the window as synthesised)
    int its_default = 0;
    {
        bool lost = false;
        ef->optimize(n_its, HCalib, nullptr, &lost, &its_default);
    }
    // EnergyFunctional::optimize(6), all iterations
    ldso_ba_opt_settings all_its = LDSO_BA_OPT_SETTINGS_INIT;
    all_its.th_opt_iterations = 0.0f;
    for (int i = 0; i < 2; i++) ef->optimize(n_its, HCalib, nullptr, nullptr, nullptr, &all_its);
    auto t0 = Clock::now();
    for (int i = 0; i < reps; i++) ef->optimize(n_its, HCalib, nullptr, nullptr, nullptr, &all_its);
    const double ms_opt = ms_since(t0) / reps;
    // + FullSystem::optimize's tail on the backend: setAdjointsF, setDeltaF, linearizeAll(true)
    auto full = [&] {
        ef->optimize(n_its, HCalib, nullptr, nullptr, nullptr, &all_its);
        ef->setAdjointsF(HCalib);
        ef->setDeltaF(HCalib);
        ef->linearizeAll(true);
    };
    for (int i = 0; i < 2; i++) full();
    t0 = Clock::now();
    for (int i = 0; i < reps; i++) full();
    const double ms_full = ms_since(t0) / reps;
    // flagPointsForRemoval's per-residual loop over 10 % of the points
    const long passes0 = ef->devicePasses();
    t0 = Clock::now();
    int nres = 0;
    for (size_t q = 0; q < ef->allPoints.size(); q += 10)
        for (auto &r : ef->allPoints[q]->residuals) {
            r->resetOOB();
            r->linearize(HCalib);
            r->applyRes(true);
            nres++;
        }
    const double ms_flag = ms_since(t0);
    const long flag_passes = ef->devicePasses() - passes0;

    // INTEGRATION.md §3's forwarding shim, timed: stand-ins for the reference's objects, each its
    // own heap allocation in the reference's creation order (frames, then per point the point and
    // its residuals), mapped to the face's objects either by std::unordered_map keyed by the
    // reference pointer (mf / mp / mr, as §3 writes it) or by index vectors filled in the same
    // order (the replacement)
    struct RefFrame {
        double state[10], state_zero[10], ab_exposure;
        float frameEnergyTH;
        char other[512];  // the rest of a FrameHessian
    };
    struct RefResidual;
    struct RefPoint {
        float idepth, idepth_zero, HdiF, bdSumF, idepth_hessian, step;
        float maxRelBaseline;
        int numGoodResiduals;
        std::pair<RefResidual *, int> lastResiduals[2];
        char other[128];
    };
    struct RefResidual {
        int state_state, state_NewState;
        double state_energy, state_NewEnergy, state_NewEnergyWithOutlier;
        float centerProjectedTo[3], JpJdF[8];
        bool isActiveAndIsGoodNEW;
        int mirrorIdx;  // the face's index, copied at makeIDX as hostIDX / targetIDX are
        char other[92];
    };
    std::vector<std::unique_ptr<RefFrame>> rframes;
    std::vector<std::unique_ptr<RefPoint>> rpoints;
    std::vector<std::unique_ptr<RefResidual>> rres;
    std::unordered_map<RefFrame *, FrameHessian *> mf;
    std::unordered_map<RefPoint *, PointHessian *> mp;
    std::unordered_map<RefResidual *, PointFrameResidual *> mr;
    for (auto &F : ef->frames) {
        rframes.emplace_back(new RefFrame());
        mf[rframes.back().get()] = F.get();
        F->user = rframes.back().get();
    }
    for (auto &Pt : ef->allPoints) {
        rpoints.emplace_back(new RefPoint());
        mp[rpoints.back().get()] = Pt.get();
        Pt->user = rpoints.back().get();
        for (auto &r : Pt->residuals) {
            rres.emplace_back(new RefResidual());
            mr[rres.back().get()] = r.get();
            r->user = rres.back().get();
            rres.back()->mirrorIdx = r->mirrorIdx;
        }
        // lastResiduals: the point's residuals to the two newest keyframes (FullSystem.cc:566-567)
        RefPoint &rp = *rpoints.back();
        rp.lastResiduals[0] = rp.lastResiduals[1] = {nullptr, 0};
        for (auto &r : Pt->residuals) {
            const int t = r->target.lock()->idx;
            if (t == N - 1) rp.lastResiduals[0].first = (RefResidual *)r->user;
            if (t == N - 2) rp.lastResiduals[1].first = (RefResidual *)r->user;
        }
    }
    // the replacement: walk the face's own containers (frames, allPoints, each point's residuals:
    // contiguous, in the device's order) and reach the reference object through `user`
    struct FaceFrames {
        EnergyFunctional &e;
        struct It {
            std::vector<shared_ptr<FrameHessian>>::iterator i;
            std::pair<RefFrame *, FrameHessian *> operator*() const { return {(RefFrame *)(*i)->user, i->get()}; }
            It &operator++() { ++i; return *this; }
            bool operator!=(const It &o) const { return i != o.i; }
        };
        It begin() { return {e.frames.begin()}; }
        It end() { return {e.frames.end()}; }
    } vf{*ef};
    struct FacePoints {
        EnergyFunctional &e;
        struct It {
            std::vector<shared_ptr<PointHessian>>::iterator i;
            std::pair<RefPoint *, PointHessian *> operator*() const { return {(RefPoint *)(*i)->user, i->get()}; }
            It &operator++() { ++i; return *this; }
            bool operator!=(const It &o) const { return i != o.i; }
        };
        It begin() { return {e.allPoints.begin()}; }
        It end() { return {e.allPoints.end()}; }
    } vp{*ef};
    std::vector<std::pair<RefResidual *, PointFrameResidual *>> vr;  // rebuilt at makeIDX in a real shim
    for (auto &Pt : ef->allPoints)
        for (auto &r : Pt->residuals) vr.emplace_back((RefResidual *)r->user, r.get());
    // the copy loops of one FullSystem::optimize through the shim (§3: "replaces
    // FullSystem.cc:853-970" and FullSystem::linearizeAll), without the face calls themselves
    auto shim_loops = [&](auto &F, auto &Pm, auto &Rm) {
        for (auto kv : F) std::memcpy(kv.second->state, kv.first->state, sizeof(kv.first->state));  // copyIn
        for (auto kv : Pm) {
            kv.second->setIdepth(kv.first->idepth);
            kv.second->setIdepthZero(kv.first->idepth_zero);
        }
        // ... gpu->optimize(...) ...
        for (auto kv : F) std::memcpy(kv.first->state, kv.second->state, sizeof(kv.first->state));
        for (auto kv : Pm) {
            kv.first->idepth = kv.second->idepth;
            kv.first->idepth_zero = kv.second->idepth_zero;
        }
        // FullSystem::linearizeAll(true): copy-in, gpu->linearizeAll, copy-out
        for (auto kv : F) std::memcpy(kv.second->state, kv.first->state, sizeof(kv.first->state));
        for (auto kv : Pm) kv.second->setIdepth(kv.first->idepth);
        auto copy_out = [](RefResidual &r, const PointFrameResidual &g) {
            r.state_state = (int)g.state_state;
            r.state_NewState = (int)g.state_NewState;
            r.state_energy = g.state_energy;
            r.state_NewEnergy = g.state_NewEnergy;
            r.state_NewEnergyWithOutlier = g.state_NewEnergyWithOutlier;
            std::memcpy(r.centerProjectedTo, g.centerProjectedTo, sizeof(r.centerProjectedTo));
            r.isActiveAndIsGoodNEW = g.isActiveAndIsGoodNEW;
            std::memcpy(r.JpJdF, g.JpJdF, sizeof(r.JpJdF));
        };
        if constexpr (std::is_same_v<std::decay_t<decltype(Rm)>, std::vector<std::pair<RefResidual *, PointFrameResidual *>>>) {
            // the objects are scattered on the heap: prefetch a few residuals ahead
            const size_t n = Rm.size();
            for (size_t k = 0; k < n; k++) {
                if (k + 8 < n) {
                    __builtin_prefetch(Rm[k + 8].first, 1);
                    __builtin_prefetch(Rm[k + 8].second, 0);
                }
                copy_out(*Rm[k].first, *Rm[k].second);
            }
        } else {
            for (auto kv : Rm) copy_out(*kv.first, *kv.second);
        }
        for (auto kv : Pm) {
            kv.first->HdiF = kv.second->HdiF;
            kv.first->bdSumF = kv.second->bdSumF;
            kv.first->idepth_hessian = kv.second->idepth_hessian;
        }
    };
    // the round-5 protocol: copy back only what the reference's consumers read.
    // After optimize: the frames' states and the points' idepths.  After linearizeAll(true): the
    // points' HdiF / idepth_hessian (CoarseTracker, flagPointsForRemoval), maxRelBaseline /
    // numGoodResiduals and lastResiduals' states from the face's per-point FixPassResult (allPoints
    // order: no residual object is touched), and the toRemove list for dropResidual.  centerProjectedTo stays with the face: its one
    // consumer per keyframe (CoarseTracker::makeCoarseDepthL0) reads gpu->residualCenter(mirrorIdx).
    std::vector<RefResidual *> toRemove;
    auto shim_digest = [&]() {
        for (auto &F : ef->frames)
            std::memcpy(((RefFrame *)F->user)->state, F->state, sizeof(F->state));
        // the face's own containers in order; FixPassResult is indexed like allPoints
        const auto &fx = ef->fixPassResult();
        const size_t P = ef->allPoints.size();
        for (size_t q = 0; q < P; q++) {
            if (q + 8 < P) __builtin_prefetch(ef->allPoints[q + 8]->user, 1);
            const PointHessian &g = *ef->allPoints[q];
            RefPoint &p = *(RefPoint *)g.user;
            p.idepth = g.idepth;
            p.idepth_zero = g.idepth_zero;
            p.HdiF = g.HdiF;
            p.idepth_hessian = g.idepth_hessian;
            if (fx.numGood.size() == P) {
                p.maxRelBaseline = std::max(p.maxRelBaseline, fx.maxRelBS[q]);
                p.numGoodResiduals += fx.numGood[q];
            }
            if (fx.lastState.size() == 2 * P)
                for (int i = 0; i < 2; i++)
                    if (p.lastResiduals[i].first) p.lastResiduals[i].second = fx.lastState[2 * q + i];
        }
        toRemove.clear();
        for (PointFrameResidual *g : fx.toRemove) toRemove.push_back((RefResidual *)g->user);
    };
    auto time_shim = [&](auto &&loops) {
        // between calls the frontend touches other memory (tracking, images): evict the caches
        std::vector<char> evict((size_t)64 << 20, 1);
        double tot = 0;
        for (int i = 0; i < reps; i++) {
            for (size_t k = 0; k < evict.size(); k += 64) evict[k]++;
            auto t1 = Clock::now();
            loops();
            tot += ms_since(t1);
        }
        return tot / reps;
    };
    // the face state after FullSystem::optimize: optimize, then linearizeAll(true) (its FixPassResult)
    ef->optimize(n_its, HCalib, nullptr, nullptr, nullptr, &all_its);
    ef->linearizeAll(true);
    (void)ef->residualState(0);  // states of the pass downloaded once (as the first consumer would)
    const double ms_shim_digest = time_shim(shim_digest);
    ef->syncResiduals();  // the round-4 per-field loops read every residual object
    const double ms_shim_map = time_shim([&] { shim_loops(mf, mp, mr); });
    const double ms_shim_vec = time_shim([&] { shim_loops(vf, vp, vr); });
    const bool ok = ef->ok();

    // the C ABI alone on a context of the same window
    std::vector<float> precalc((size_t)N * N * LDSO_BA_PRECALC_STRIDE);
    std::vector<double> adH((size_t)N * N * 64), adT((size_t)N * N * 64), cp(4), fp(8 * N), fd(8 * N), fdp(8 * N);
    ldso_ba_frame_precalc(N, fs.data(), calib, precalc.data());
    ldso_ba_set_adjoints(N, fs.data(), adH.data(), adT.data(), cp.data());
    ldso_ba_frame_take_data(N, fs.data(), nullptr, fp.data(), fd.data(), fdp.data());
    const float cdelta[4] = {0, 0, 0, 0};
    ldso_ba_window w;
    std::memset(&w, 0, sizeof(w));
    w.n_frames = N;
    w.n_points = P;
    w.n_residuals = R;
    w.width = W;
    w.height = H;
    std::memcpy(w.calib, calib, sizeof(calib));
    w.dI = dI.data();
    w.frame_energy_th = th.data();
    w.precalc = precalc.data();
    w.ad_host = adH.data();
    w.ad_target = adT.data();
    w.c_prior = cp.data();
    w.c_delta = cdelta;
    w.frame_prior = fp.data();
    w.frame_delta_prior = fdp.data();
    w.point_host = ph.data();
    w.point_data = pd.data();
    w.point_res_begin = rb.data();
    w.res_target = rt.data();
    w.res_state = rs.data();
    w.res_energy = re.data();
    w.res_flags = rf.data();
    ldso_ba_ctx *raw = nullptr;
    double ms_raw = -1;
    if (ldso_ba_create(0, &raw) == 0 && ldso_ba_load(raw, 1, &w, 0, 1) == 0) {
        const int n = 8 * N + 4;
        std::vector<double> ns((size_t)7 * n), e((size_t)3 * (n_its + 1)), cv(4), co(4);
        std::vector<ldso_ba_frame_state> fo(N);
        std::vector<float> id(P);
        for (int k = 0; k < 4; k++) cv[k] = HCalib->value_zero[k];
        ldso_ba_nullspaces(N, fs.data(), ns.data());
        for (int i = 0; i < 2; i++)
            ldso_ba_optimize(raw, n_its, &all_its, fs.data(), cv.data(), cv.data(), ns.data(), e.data(), fo.data(),
                             co.data(), id.data(), nullptr, nullptr);
        t0 = Clock::now();
        for (int i = 0; i < reps; i++)
            ldso_ba_optimize(raw, n_its, &all_its, fs.data(), cv.data(), cv.data(), ns.data(), e.data(), fo.data(),
                             co.data(), id.data(), nullptr, nullptr);
        ms_raw = ms_since(t0) / reps;
        ldso_ba_destroy(raw);
    }
    std::printf(
        "{\"window\": \"S7 (7 KF, 2000 pts, 640x480, seed 1)\", \"n_its\": %d, \"reps\": %d, \"ok\": %s, "
        "\"optimize\": {\"ms_per_optimize\": %.6f, \"ms_per_gn_iteration\": %.6f, \"iterations\": %d, "
        "\"iterations_default\": %d}, "
        "\"shim\": {\"what\": \"INTEGRATION.md 3 reference-side copy loops of one FullSystem::optimize, %d residuals, "
        "%d points, caches evicted between calls: the consumers' fields only (FixPassResult incl. lastResiduals' "
        "states by point; digest_ms, the protocol of 3) vs every residual field through back-pointers / "
        "unordered_map (round 4)\", \"digest_ms\": %.6f, \"per_field_back_pointer_ms\": %.6f, "
        "\"unordered_map_ms\": %.6f, \"shim_ms_per_gn_iteration\": %.6f, "
        "\"frac_of_face_gn_iteration\": %.4f, \"per_field_frac_of_face_gn_iteration\": %.4f, "
        "\"to_remove\": %zu}, "
        "\"optimize_full\": {\"ms\": %.6f, \"what\": \"optimize(6) + setAdjointsF + setDeltaF + linearizeAll(true) "
        "with the residual / point write-back\"}, "
        "\"c_abi_optimize\": {\"ms_per_optimize\": %.6f, \"ms_per_gn_iteration\": %.6f}, "
        "\"flag_loop\": {\"residuals\": %d, \"ms\": %.6f, \"device_passes\": %ld}}\n",
        n_its, reps, ok ? "true" : "false", ms_opt, ms_opt / n_its, n_its, its_default, (int)vr.size(), (int)ef->allPoints.size(),
        ms_shim_digest, ms_shim_vec, ms_shim_map, ms_shim_digest / n_its, ms_shim_digest / ms_opt, ms_shim_vec / ms_opt,
        toRemove.size(),
        ms_full, ms_raw, ms_raw / n_its, nres, ms_flag, flag_passes);
    return ok ? 0 : 1;
}
