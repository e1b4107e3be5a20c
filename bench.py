"""Headline benchmark: point-residuals/sec per GN iteration on synthetic 7-keyframe windows.

A *step* is one hot-path pass over every window resident on the GPU: linearizeAll + applyRes +
setNewFrameEnergyTH + accumulate{AF,LF,SCF} + both stitches (one ldso_ba_linearize call,
seven kernels on the context's stream).  Each GPU holds `--windows` independent S7 windows
(7 keyframes, 2000 active points, 640x480, distinct seeds), so per-GPU work is fixed as GPUs
are added ("scaling": "weak"; no collective is needed between independent windows).

roofline: dominant kernel k_linearize, algorithmic bytes per residual
          = 276 B (23 unique 12-B texels) + 8 B state + 88 B/(N-1) point data, times the
          residuals that do gather (not OOB before the pass), / its mean HIP-event duration
          over the timed region (the event pair on every EVENT_EVERY-th timed step);
          frac_step: the same bytes over the sum of the pass's kernel durations (k_linearize,
          k_point_sc, k_stitch, k_stitch_sum: §8d's step-level definition), frac_step_wall over the
          step's wall clock.
value  = residuals that gather in the pass (R_active: not OOB going in, OOB being sticky within
          optimize()) of all ranks per step / max-over-ranks step time.
cpu_baseline: the oracle restatement (oracle/cpu_baseline.py) compiled -O3 -march=native on the
          box: the headline's own workload (the same 64 S7 windows, one single-threaded window pass
          per worker process pinned one per physical core of socket 0), the like-for-like figure
          behind speedup_vs_cpu; beside it one S7 window with (ii) one pinned worker per physical
          core of socket 0 (SURVEY §8d's "single-socket" figure, compared with the GPU's
          single-window rate) and (i) 6 threads as the reference's IndexThreadReduce.
cpp_face: the C++ host face (include/ldso_amd/energy_functional.h) timed as FullSystem drives it
          (ldso_amd/lib/ldso_face_bench, one S7 window) beside the C ABI's ldso_ba_optimize.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--windows B] [--mode replicas|shard]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "point-residuals/sec per GN iter (7-KF window) + ms/solve; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
EVENT_EVERY = 5  # timed steps whose k_linearize the roofline's HIP event pair brackets: every 5th


def algo_bytes_per_residual(n_frames):
    return 276.0 + 8.0 + 88.0 / (n_frames - 1)


def world_from_env(gpus, env=None):
    """(world, launched_by_a_launcher).  Under torchrun (WORLD_SIZE set) --gpus must equal
    WORLD_SIZE: a mismatch is an error, not a silently different measurement."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world} (the launcher started {world} ranks)")
        return world, True
    return 1, False


def free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, cmd, env=None, poll_s=0.5):
    """`bench.py --gpus N` without a launcher: start N fresh child processes of `cmd` (one per
    GPU, RANK = LOCAL_RANK = i, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free MASTER_PORT)
    before this process touches the GPU, forward rank 0's stdout (the JSON line), and return
    the first non-zero exit code (0 when every rank succeeded).  If a rank fails the others are
    stopped (they would wait in a collective forever)."""
    import subprocess

    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n))
        # rank 0's stdout is this process's (the one JSON line); the others' goes to stderr
        procs.append(subprocess.Popen(cmd, env=e, stdout=None if r == 0 else sys.stderr))
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


def load_pmc(workload):
    """HBM traffic per k_linearize launch from the committed rocprofv3 --pmc summary
    (profiles/pmc_k_linearize.json, written by tools/pmc_traffic.py in separate counter passes), if
    it exists for this exact workload -> (bytes, provenance), else (None, reason).  It is NOT measured
    in this run: the provenance names the file, the session that measured it and whether the
    library build it measured is this run's (sha256 of the library's sources, _lib.source_sha256:
    the .so is relinked wherever the tests build it, so its bytes are no build identity)."""
    rel = os.path.join("profiles", "pmc_k_linearize.json")
    try:
        with open(os.path.join(ROOT, rel)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, {"file": rel, "note": "no committed PMC summary"}
    if d.get("workload") != workload:
        return None, {"file": rel, "note": "committed PMC summary is for another workload"}
    from ldso_amd import _lib

    mine = _lib.source_sha256()
    prov = {"file": rel, "measured_in_this_run": False, "session": d.get("session"),
            "source_sha256": d.get("source_sha256"),
            "same_build_as_this_run": bool(mine and mine == d.get("source_sha256")),
            "method": "rocprofv3 --pmc, separate passes: 2 x FETCH_SIZE + WRITE_SIZE per launch (tools/pmc_traffic.py)",
            "fetch_x2_calibration": "profiles/r6/fetch_probe: 16-B pieces of random 128-B lines (1, 2, 4 or 8 per line, "
                                    "tools/gather_probe_pieces.hip) -- one TCC_EA0_RDREQ per touched line whatever its "
                                    "used bytes, FETCH_SIZE = exactly half of the whole-line bytes: the x2 applies"}
    return d.get("hbm_bytes_per_launch"), prov


def L_PATH():
    from ldso_amd import _lib

    return _lib.LIB_PATH


def cpp_face_leg():
    """ldso_amd/lib/ldso_face_bench in a child process (its own HIP context): EnergyFunctional::
    optimize(6) on one S7 window, host clock, beside ldso_ba_optimize(6) on the same window."""
    import subprocess

    exe = os.path.join(ROOT, "ldso_amd", "lib", "ldso_face_bench")
    try:
        p = subprocess.run([exe], cwd=ROOT, capture_output=True, text=True, timeout=300)
        d = json.loads(p.stdout.strip().splitlines()[-1])
    except (OSError, subprocess.SubprocessError, ValueError, IndexError) as e:
        return {"error": str(e)}
    d["ms_per_gn_iteration"] = d["optimize"]["ms_per_gn_iteration"]
    if "shim" in d:  # INTEGRATION.md §3's forwarding loops per GN iteration (index vectors)
        d["shim_ms_per_gn_iteration"] = d["shim"]["shim_ms_per_gn_iteration"]
    return d


def cpu_baseline(seconds=10.0):
    """oracle/cpu_baseline.py in a child process (it pins its own threads): the restatement built
    -O3 -march=native on this host, (i) 6 threads as the reference's IndexThreadReduce, (ii) one
    worker per physical core of socket 0 within the job's CPU share, pinned.  None on failure."""
    import subprocess

    try:
        p = subprocess.run([sys.executable, "-m", "oracle.cpu_baseline", "--seconds", str(seconds)], cwd=ROOT,
                           capture_output=True, text=True, timeout=600)
        return json.loads(p.stdout.strip().splitlines()[-1]) if p.returncode == 0 else None
    except (subprocess.SubprocessError, ValueError, IndexError):
        return None


def time_optimize(ctx, nss, n_its=6, reps=10, settings=None):
    """ms per ldso_ba_optimize(n_its) call (host clock) and per GN iteration it ran.  With the
    default settings every window leaves the loop on the reference's exits (canbreak after
    setting_minOptIterations, FullSystem.cc:968-969), so the iterations run are reported;
    settings with th_opt_iterations = 0 never break and run all n_its."""
    for _ in range(2):
        r = ctx.optimize(n_its, nullspaces=nss, settings=settings)
    t = time.perf_counter()
    for _ in range(reps):
        ctx.optimize(n_its, nullspaces=nss, settings=settings)
    ms = 1e3 * (time.perf_counter() - t) / reps
    its, status = np.asarray(r[4]), np.asarray(r[5])
    out = {"n_its": n_its, "ms_per_optimize": ms, "windows": len(nss),
           "iterations_run": int(its[0]) if len(its) == 1 else
           {"min": int(its.min()), "max": int(its.max()), "mean": float(its.mean())},
           "converged_windows": int((status == 1).sum()), "lost_windows": int((status == 2).sum())}
    if settings is not None and settings.th_opt_iterations == 0.0:
        out["ms_per_iteration"] = ms / n_its  # every window runs all n_its iterations
    else:
        # a window that left the loop still has every later kernel of the captured sequence launched
        # (it returns at once): the call's time is not per iteration run, so none is derived from it
        out["ms_per_iteration"] = None
        out["note"] = ("early exits skip work, not launches: per-iteration cost only from optimize_all_its")
    return out


def secondary_s11(device, windows=8, steps=20):
    """BASELINE config[3]'s window shape (11 keyframes, 8000 points, 640x480) on ONE GPU, batched
    like the headline (a parity/scaling case in BASELINE.json, reported beside the headline, not
    as `value`): denser windows share more texel lines between residuals."""
    from ldso_amd import BAContext, synth

    ws = [synth.make_window(**synth.S11, seed=5000 + i) for i in range(windows)]
    ctx = BAContext(device)
    ctx.load(ws)
    for w in ws:
        w.dI = None
    R = ctx.stats()["residuals"]
    for _ in range(3):
        ctx.linearize()
    ctx.sync()
    ctx.set_tuning(7, 1)
    ctx.set_kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.linearize()
    ctx.sync()
    el = time.perf_counter() - t0
    kt = ctx.kernel_times()
    ctx.set_kernel_timing(False)
    n_gather = sum(int((ctx.residuals(i)["state"] != 1).sum()) for i in range(len(ws)))  # same every pass
    ctx.close()
    k_ms, k_n = kt["k_linearize"]
    k_s = k_ms / max(1, k_n) / 1e3
    ach = n_gather * algo_bytes_per_residual(11) / k_s / 1e9
    return {"workload": f"{windows} x S11 synthetic windows (11 KF, 8000 pts, 640x480)", "residuals_per_step": R,
            "ms_per_step": 1e3 * el / steps, "point_residuals_per_s": R * steps / el,
            "k_linearize_us": k_s * 1e6, "roofline_frac": ach / HBM_PEAK_GBS, "achieved_GBps": ach}


def tracker_leg(device, reps=50, n_hyp=32, cpu_seconds=2.0, with_cpu=True):
    """Coarse tracker (include/ldso_ct.h) on a 640x480 frame with the
    reference point clouds of synth.make_tracker_scene (8000 level-0 points):
    * lm_iteration: one calcRes + calcGSSSE at level 0, what each LM iteration of
      CoarseTracker::trackNewestCoarse calls (CoarseTracker.cc:61-310), host clock, results on
      the host;
    * hypotheses: calcRes of n_hyp motion hypotheses in one launch (FullSystem::trackNewCoarse's
      tries, FullSystem.cc:282-386), point-evaluations/s;
    * k_ct_calc_res roofline: 48 B (4 bilinear taps x 12-B [I, dx, dy]) per point-evaluation
      + 16 B per point per launch, over its mean HIP-event duration;
    * cpu: the oracle's calcRes + calcGSSSE (single thread, as the reference's tracker) on the
      same level-0 cloud."""
    from ldso_amd import synth
    from ldso_amd.tracker import CoarseTracker

    w, h = 640, 480
    calib = np.array([384.0, 432.0, 319.5, 239.5], np.float32)
    color, make_pc = synth.make_tracker_scene(w, h, seed=0)
    ct = CoarseTracker(w, h, device)
    ct.make_k(calib)
    ct.set_new_frame(color, 1.0)
    pcs = make_pc([ct.frame_level(l)[0][:, 0] for l in range(ct.levels)])
    ct.set_reference([(p["u"], p["v"], p["idepth"], p["color"]) for p in pcs], 1.0, (0.02, 3.0))
    rng = np.random.default_rng(3)
    Ts = np.stack([synth.se3_matrix(rng.normal(0, 2e-3, 3), rng.normal(0, 1e-2, 3)) for _ in range(n_hyp)])
    ab = np.tile([0.05, 1.0], (n_hyp, 1))
    n0 = int(pcs[0]["u"].size)
    for _ in range(5):
        ct.calc_res(0, Ts[0], ab[0])
        ct.calc_gs(0, Ts[0], ab[0])
        ct.calc_res_batch(0, Ts, ab)
    t0 = time.perf_counter()
    for i in range(reps):
        ct.calc_res(0, Ts[i % n_hyp], ab[0])
        ct.calc_gs(0, Ts[i % n_hyp], ab[0])
    lm_ms = 1e3 * (time.perf_counter() - t0) / reps
    for _ in range(5):
        ct.calc_res_gs(0, Ts[0], ab[0])
    t0 = time.perf_counter()
    for i in range(reps):
        ct.calc_res_gs(0, Ts[i % n_hyp], ab[0])
    lm_fused_ms = 1e3 * (time.perf_counter() - t0) / reps
    ct.set_kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        ct.calc_res_batch(0, Ts, ab)
    hyp_ms = 1e3 * (time.perf_counter() - t0) / reps
    kt = ct.kernel_times()
    ct.set_kernel_timing(False)
    k_ms, k_n = kt["k_ct_calc_res"]
    k_s = k_ms / max(1, k_n) / 1e3
    algo = n_hyp * n0 * 48.0 + n0 * 16.0
    out = {
        "frame": "640x480, 4 levels", "points_level0": n0,
        "lm_iteration": {"ms": lm_fused_ms, "calls": "calcRes + calcGSSSE, level 0, one round trip (ldso_ct_calc_res_gs)",
                         "ms_two_calls": lm_ms},
        "hypotheses": {"n_hyp": n_hyp, "ms_per_launch_host": hyp_ms,
                       "point_evals_per_s": n_hyp * n0 / (hyp_ms / 1e3)},
        "k_ct_calc_res": {"avg_launch_us": k_s * 1e6, "algo_bytes_per_launch": algo,
                          "achieved_GBps": algo / k_s / 1e9 if k_s > 0 else None,
                          "frac_of_hbm_peak": algo / k_s / 1e9 / HBM_PEAK_GBS if k_s > 0 else None},
    }
    ct.close()
    if with_cpu:
        import oracle

        lv = oracle.make_images(color, w, h)
        K = oracle.ct_make_k(calib, w, h)
        aff6 = (1.0, 1.0, 0.02, 3.0, 0.05, 1.0)
        pc = (pcs[0]["u"], pcs[0]["v"], pcs[0]["idepth"], pcs[0]["color"])
        n, el = 0, 0.0
        while el < cpu_seconds:
            t0 = time.perf_counter()
            rs, warped = oracle.ct_calc_res(0, w, h, K[0], lv[0][0], pc, Ts[n % n_hyp], aff6, 20.0)
            oracle.ct_calc_gs(warped, K[0, 0], K[0, 1], aff6)
            el += time.perf_counter() - t0
            n += 1
        out["cpu_lm_iteration"] = {"ms": 1e3 * el / n, "cores": 1, "kind": "port",
                                   "sample": f"{n} oracle calcRes + calcGSSSE at level 0 ({n0} points)"}
        out["lm_iteration_speedup_vs_cpu"] = out["cpu_lm_iteration"]["ms"] / lm_fused_ms
    return out


def activation_leg(device, reps=20, cpu_seconds=2.0, with_cpu=True):
    """Point activation (ldso_ba_activate_points): optimizeImmaturePoint for
    the 2000 points of an S7 window (inverse-depth interval +-10 %), against every other frame
    (6 residuals x 8 pixels x 4 evaluations per point).  Host-clock ms per call (upload, k_activate,
    download), k_activate's mean HIP-event duration, and the oracle's single-thread loop (the
    reference's activatePointsMT runs on 6 threads; its per-point work is this loop)."""
    from ldso_amd import BAContext, synth

    w = synth.make_window(**synth.S7, seed=1)
    pts = synth.immature_from_window(w)
    ctx = BAContext(device).load([w])
    for _ in range(3):
        ctx.activate_points(0, pts)
    ctx.set_kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        out = ctx.activate_points(0, pts)
    ms = 1e3 * (time.perf_counter() - t0) / reps
    kt = ctx.kernel_times()
    ctx.close()
    k_ms, k_n = kt["k_activate"]
    k_us = 1e3 * k_ms / max(1, k_n)
    res = {"points": int(pts.size), "window": "S7 (7 KF, 640x480)", "activated": int((out["status"] == 0).sum()),
           "ms_per_call": ms, "k_activate_us": k_us,
           "point_activations_per_s": pts.size / (k_us / 1e6) if k_us > 0 else None}
    if with_cpu:
        import oracle

        ow = oracle.OracleWindow(synth.make_window(**synth.S7, seed=1), threads=0)
        m, el = 0, 0.0
        while el < cpu_seconds:
            t0 = time.perf_counter()
            ow.activate_points(pts)
            el += time.perf_counter() - t0
            m += 1
        ow.close()
        res["cpu"] = {"ms": 1e3 * el / m, "cores": 1, "kind": "port", "sample": f"{m} oracle calls over {pts.size} points"}
        res["kernel_speedup_vs_cpu"] = res["cpu"]["ms"] / (k_us / 1e3) if k_us > 0 else None
    return res


def trace_leg(device, reps=50, cpu_seconds=2.0, with_cpu=True):
    """traceNewCoarse (ldso_ct_trace): ImmaturePoint::traceOn of 7 hosts x
    1500 immature points (setting_desiredImmatureDensity) against a 640x480 new frame, records
    resident on the device.  Reported: host-clock ms per traceNewCoarse (launch + counters + one
    round trip), the k_ct_trace kernel's mean HIP-event duration and point traces/s, and the
    oracle's single-thread traceNewCoarse (the reference runs it on one thread under mapMutex,
    FullSystem.cc:1157-1194) on the same records.  The 4.9 MB level-0 frame stays in L2 / MALL:
    the kernel is latency bound (dependent bilinear taps), not an HBM stream."""
    from ldso_amd import synth
    from ldso_amd.tracker import CoarseTracker

    w, h = 640, 480
    host, new, uv, krki, kt, aff = synth.make_trace_scene(w, h)
    n_hosts, per = uv.shape[0], uv.shape[1]
    ct = CoarseTracker(w, h, device)
    ct.set_new_frame(host, 1.0)
    pts = np.concatenate([ct.make_immature(uv[i], 1.0, i) for i in range(n_hosts)])
    ct.set_new_frame(new, 1.0)
    for _ in range(3):
        ct.immature_upload(pts)
        ct.trace(krki, kt, aff)
    ct.set_kernel_timing(True)
    total = 0.0
    counts = None
    for _ in range(reps):
        ct.immature_upload(pts)  # every rep traces the same freshly created records
        t0 = time.perf_counter()
        counts = ct.trace(krki, kt, aff)
        total += time.perf_counter() - t0
    kt_ = ct.kernel_times()
    ct.close()
    k_ms, k_n = kt_["k_ct_trace"]
    k_us = 1e3 * k_ms / max(1, k_n)
    n = pts.size
    out = {"points": int(n), "hosts": int(n_hosts), "frame": f"{w}x{h}",
           "status_counts": dict(zip(("good", "oob", "outlier", "skipped", "badcondition", "uninitialized"),
                                     [int(x) for x in counts])),
           "ms_per_trace_new_coarse": 1e3 * total / reps, "k_ct_trace_us": k_us,
           "point_traces_per_s": n / (k_us / 1e6) if k_us > 0 else None}
    if with_cpu:
        import oracle

        dN = oracle.make_images(new, w, h)[0][0]
        m, el = 0, 0.0
        while el < cpu_seconds:
            ref = pts.copy()
            t0 = time.perf_counter()
            oracle.ip_trace(dN, w, h, krki, kt, aff, ref)
            el += time.perf_counter() - t0
            m += 1
        out["cpu_trace_new_coarse"] = {"ms": 1e3 * el / m, "cores": 1, "kind": "port",
                                       "sample": f"{m} oracle traceNewCoarse calls over the same {n} records"}
        out["kernel_speedup_vs_cpu"] = out["cpu_trace_new_coarse"]["ms"] / (k_us / 1e3) if k_us > 0 else None
    return out


def sharded_window_leg(dist, rank, world, device, coll_dev, steps=20):
    """BASELINE config[3]'s split on the job's ranks: ONE S11 window (11 KF, 8000
    points) with its points sharded by host frame over the ranks, every pass ending with the
    library's own RCCL exchange (ldso_ba_comm_init: all-reduce of the packed systems and energies,
    all-gather of the newest-frame slots, the threshold re-selected on every rank).  Timed like
    the headline (barriers, max over ranks); rank 0 checks the reduced system against the same
    window unsharded on its own GPU (worst block ||G - O||_F / ||O||_F, energies, the newest
    frame's threshold bit for bit) and times that unsharded pass beside it.  Every phase ends
    with a status all-reduce, so a rank that fails is reported instead of leaving the others
    waiting inside a collective."""
    import torch

    from ldso_amd import BAContext, synth
    from ldso_amd import dist as ldist

    out = {"workload": "1 x S11 synthetic window (11 KF, 8000 pts, 640x480), points sharded over the ranks",
           "ranks": world, "exchange": "in-library RCCL (ldso_ba_comm_init)"}
    cfg = dict(synth.S11, seed=7001)
    state = {"err": None}

    def phase(fn):
        if state["err"] is None:
            try:
                fn()
            except Exception as ex:  # reported, the other ranks told below
                state["err"] = f"rank {rank}: {ex!r}"[:400]
        t = torch.tensor([0.0 if state["err"] is None else 1.0], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t)
        if t.item() != 0 and state["err"] is None:
            state["err"] = "another rank failed"
        return state["err"] is None

    ctxs = {}

    def build():
        ctxs["w"] = synth.make_window(**cfg)
        ctxs["c"] = BAContext(device)

    def attach():
        ldist.attach_rccl(ctxs["c"], dist)
        ctxs["c"].load([ctxs["w"]], shard_rank=rank, shard_count=world)

    times = {}

    def run():
        c = ctxs["c"]
        for _ in range(3):
            c.linearize()
        c.sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            c.linearize()
        c.sync()
        dist.barrier()
        times["el"] = time.perf_counter() - t0
        times["points"] = c.stats()["points"]

    ok = phase(build) and phase(attach) and phase(run)
    if ok:
        t = torch.tensor([times["el"], times["points"]], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0].item())
        pts = torch.tensor([times["points"]], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(pts)
        out["ms_per_pass"] = 1e3 * el / steps
        out["points_total"] = int(pts.item())
        if rank == 0:
            c = ctxs["c"]
            f = BAContext(device).load([synth.make_window(**cfg)])
            for _ in range(3 + steps):  # the sharded context's pass count
                f.linearize()
            s, sf = c.system(0), f.system(0)
            N = cfg["n_frames"]
            edges = [0, 4] + [4 + 8 * (k + 1) for k in range(N)]
            worst = 0.0
            for key in ("HA", "Hsc"):
                G, O = s[key], sf[key]
                scale = np.linalg.norm(O)
                for a in range(len(edges) - 1):
                    for b in range(a, len(edges) - 1):
                        g = G[edges[a]:edges[a + 1], edges[b]:edges[b + 1]]
                        o = O[edges[a]:edges[a + 1], edges[b]:edges[b + 1]]
                        if a == b:
                            g, o = np.triu(g), np.triu(o)
                        den = max(np.linalg.norm(o), 1e-12 * scale, 1e-300)
                        worst = max(worst, float(np.linalg.norm(g - o) / den))
            e, ef = c.energy(0), f.energy(0)
            th_equal = bool(np.array_equal(c.frame_energy_th(0)[-1], f.frame_energy_th(0)[-1]))
            f.sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                f.linearize()
            f.sync()
            out["ms_per_pass_unsharded_one_gpu"] = 1e3 * (time.perf_counter() - t0) / steps
            out["parity"] = {
                "max_block_rel_err": worst,
                "block_tol": 1e-4,
                "energy_rel_err": float(abs(e[0] - ef[0]) / max(abs(ef[0]), 1e-300)),
                "n_in_equal": bool(e[2] == ef[2]),
                "newest_threshold_bitwise": th_equal,
            }
            out["parity"]["ok"] = bool(worst < 1e-4 and out["parity"]["energy_rel_err"] <= 1e-9
                                       and out["parity"]["n_in_equal"] and out["parity"]["newest_threshold_bitwise"])
            f.close()
    if state["err"] is not None:
        out["error"] = state["err"]
    if "c" in ctxs:
        ctxs["c"].close()
    dist.barrier()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--windows", type=int, default=64, help="S7 windows per GPU")
    ap.add_argument("--frames", type=int, default=7)
    ap.add_argument("--points", type=int, default=2000)
    ap.add_argument("--mode", choices=["replicas", "shard"], default="replicas")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-tracker", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the S11 line")
    ap.add_argument("--no-shard-leg", action="store_true", help="N > 1: skip the sharded S11 window")
    args = ap.parse_args()

    world, launched = world_from_env(args.gpus)
    if not launched and args.gpus > 1:  # no launcher: start the ranks here, before any GPU call
        sys.exit(launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    # stdout carries exactly one line, the JSON: everything else written to fd 1 (RCCL's init
    # banner, library prints) goes to stderr
    json_out = os.fdopen(os.dup(1), "w", buffering=1)
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 path on a one-GPU box: LDSO_BENCH_SHARE_GPU=1 puts every rank on
    # device 0 and the timing collectives on gloo (the driver's multi-GPU runs use neither)
    share_gpu = os.environ.get("LDSO_BENCH_SHARE_GPU") == "1"
    if share_gpu:
        local_rank = 0
    backend = "gloo" if share_gpu else "nccl"
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist

        torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend)
        dist = tdist
    import torch
    coll_dev = "cpu" if backend == "gloo" else "cuda"

    # torch's bundled HIP runtime must initialise before the one libldso_ba.so links
    torch.cuda.set_device(local_rank)
    from ldso_amd import _lib as L
    from ldso_amd import BAContext, synth

    B, N, P = args.windows, args.frames, args.points
    if args.mode == "replicas":
        seeds = [1000 + rank * B + i for i in range(B)]  # independent windows per rank
        shard = (0, 1)
    else:
        seeds = [1000 + i for i in range(B)]  # same windows on every rank, points sharded
        shard = (rank, world)
    windows = [synth.make_window(n_frames=N, n_points=P, seed=s) for s in seeds]
    ctx = BAContext(local_rank)
    if args.mode == "shard" and dist is not None:
        from ldso_amd import dist as ldist

        ldist.attach_rccl(ctx, dist)  # the library's own RCCL exchange ends every pass
    ctx.load(windows, shard_rank=shard[0], shard_count=shard[1])
    for w in windows:
        w.dI = None  # images now live in HBM only
    R_rank = ctx.stats()["residuals"]

    def step():
        ctx.linearize(fix=False, accumulate=True)

    for _ in range(args.warmup):
        step()
    ctx.sync()
    torch.cuda.synchronize()

    # HIP events bracket only the dominant kernel inside the timed region, on every EVENT_EVERY-th
    # step (each event pair costs the stream ~4-6 us; the sampled launches are the same kernel on
    # the same inputs); the per-kernel breakdown is taken afterwards
    ctx.set_kernel_timing(True)
    if dist is not None:
        dist.barrier()
    ctx.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        ctx.set_tuning(7, 1 if s % EVENT_EVERY == 0 else 0)  # LDSO_BA_TUNE_TIMING_MASK: slot 0 = k_linearize
        step()
    ctx.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    ktimes = ctx.kernel_times()
    # residuals that gather texels in a pass (the same in every pass after the first: the inputs do
    # not change between the passes and OOB is sticky), counted after the timed region so that no
    # host-side download leaves the GPU idle between the warmup and the timed steps
    n_gather = sum(int((ctx.residuals(i)["state"] != 1).sum()) for i in range(len(windows)))
    ctx.set_kernel_timing(False)
    # the same steps without the roofline's event pair (each costs the stream ~5 us of idle GPU on
    # either side of k_linearize): reported beside the headline, never as it
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    ms_step_no_events = 1e3 * (time.perf_counter() - t0) / args.steps
    ctx.set_tuning(7, -1)
    ctx.set_kernel_timing(True)  # breakdown of every kernel, outside the timed region
    for _ in range(min(args.steps, 20)):
        step()
    ctx.sync()
    kall = ctx.kernel_times()
    ctx.set_kernel_timing(False)
    # every resident window through a full device GN iteration (pass + solve + resubstitute)
    gn = None
    if args.mode == "replicas" and max(w.n_frames for w in windows) <= 11:
        nss = [w.nullspaces() for w in windows]
        for _ in range(3):
            ctx.iterate(2, 1e-5, nss, fetch_steps=False)
        ctx.sync()
        t1 = time.perf_counter()
        it_reps = min(args.steps, 20)
        for _ in range(it_reps):
            ctx.iterate(2, 1e-5, nss, fetch_steps=False)
        gn_ms = 1e3 * (time.perf_counter() - t1) / it_reps
        gn = {"ms_per_iteration": gn_ms, "windows": B, "windows_per_s": B / (gn_ms / 1e3)}
        gn["optimize"] = time_optimize(ctx, nss, n_its=6, reps=3)
        gn["optimize_all_its"] = time_optimize(ctx, nss, n_its=6, reps=3,
                                               settings=L.OptSettings.default(th_opt_iterations=0.0))

    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        tot = torch.tensor([R_rank, n_gather], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tot)
        R_total, G_total = float(tot[0].item()), float(tot[1].item())
    else:
        R_total, G_total = float(R_rank), float(n_gather)
    if args.mode == "shard":
        R_job = float(sum(w.n_residuals for w in windows))  # each residual counted once
    else:
        R_job = R_total
    ms_step = 1e3 * el / args.steps
    value = G_total * args.steps / el  # R_active: residuals that gather (OOB ones return at once)

    klin_ms, klin_n = ktimes["k_linearize"]
    klin_avg_s = klin_ms / max(1, klin_n) / 1e3
    bytes_per_launch = n_gather * algo_bytes_per_residual(N)
    achieved = bytes_per_launch / klin_avg_s / 1e9 if klin_avg_s > 0 else 0.0
    workload = f"{B} x S7 synthetic windows/GPU ({N} KF, {P} pts, 640x480)" if (N, P) == (7, 2000) else \
        f"{B} x synthetic windows/GPU ({N} KF, {P} pts, 640x480)"
    traffic, traffic_source = load_pmc(workload)

    # N > 1: one S11 window sharded over every rank, the library's RCCL exchange in each pass
    sharded = None
    if dist is not None and not args.no_shard_leg:
        sharded = sharded_window_leg(dist, rank, world, local_rank, coll_dev, steps=min(args.steps, 20))

    # one window: pass alone, and a GN iteration with the solve on the host (stitched-system
    # download + LDLT + resubstitute) or on the device (ldso_ba_iterate), host clock
    single = None
    if rank == 0:
        sw = synth.make_window(n_frames=N, n_points=P, seed=1)
        ns = sw.nullspaces()
        c1 = BAContext(local_rank)
        c1.load([sw])
        for i in range(5):
            c1.linearize()
            x = c1.solve(0, i, 1e-5, ns)
            c1.resubstitute(0, x, 1e-5, fetch=True)
        reps = 30
        c1.sync()
        t1 = time.perf_counter()
        for i in range(reps):
            c1.linearize()
            x = c1.solve(0, 2, 1e-5, ns)
            c1.resubstitute(0, x, 1e-5, fetch=True)
        ms_solve = 1e3 * (time.perf_counter() - t1) / reps
        c1.sync()
        t1 = time.perf_counter()
        for i in range(reps):
            c1.linearize()
        c1.sync()
        sw_ms = 1e3 * (time.perf_counter() - t1) / reps
        # the same GN iteration with the solve and resubstitution on the device (ldso_ba_iterate:
        # pass + solve + resubstitute, x and point steps back on the host, one synchronisation)
        for i in range(5):
            c1.iterate(2, 1e-5, [ns])
        t1 = time.perf_counter()
        for i in range(reps):
            c1.iterate(2, 1e-5, [ns])
        ms_solve_dev = 1e3 * (time.perf_counter() - t1) / reps
        # GN iteration = pass + solve + resubstitute with x and the point steps on the host
        sw_active = int((c1.residuals(0)["state"] != 1).sum())  # R_active, as the headline counts
        single = {"ms_per_pass": sw_ms, "residuals": sw.n_residuals, "residuals_active": sw_active,
                  "point_residuals_per_s": sw_active / (sw_ms / 1e3),
                  "ms_per_gn_iteration_host_solve": ms_solve, "ms_per_gn_iteration_device_solve": ms_solve_dev}
        # FullSystem::optimize(setting_maxOptIterations = 6) entirely on the device (ldso_ba_optimize:
        # resetOOB + linearizeAll, then 6 x {solve, resubstitute, doStepFromBackup + setPrecalcValues,
        # linearizeAll}; one synchronisation), host clock around the call
        single["optimize"] = time_optimize(c1, [ns], n_its=6)
        # the same call with the early exit disabled (th_opt_iterations = 0): all 6 iterations
        single["optimize_all_its"] = time_optimize(c1, [ns], n_its=6, settings=L.OptSettings.default(th_opt_iterations=0.0))
        c1.close()

    s11 = None
    if rank == 0 and args.mode == "replicas" and not args.no_secondary:
        s11 = secondary_s11(local_rank)

    tracker = None
    if rank == 0 and not args.no_tracker:
        tracker = tracker_leg(local_rank, with_cpu=(world == 1 and not args.no_cpu))
        tracker["trace_new_coarse"] = trace_leg(local_rank, with_cpu=(world == 1 and not args.no_cpu))
        tracker["activate_points"] = activation_leg(local_rank, with_cpu=(world == 1 and not args.no_cpu))

    face = cpp_face_leg() if rank == 0 else None

    cpu = cpu1 = cpu6 = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cb = cpu_baseline(args.cpu_seconds)
        if cb:
            cpu, cpu1, cpu6 = cb.get("batched"), cb["socket_pinned"], cb["six_threads"]

    # SURVEY §8d's step-level roofline: Achieved = R_active * B_res / (the sum of the pass's kernel
    # durations), beside the dominant kernel's fraction (`frac`); and the same bytes over the step's
    # wall clock (every launch gap included)
    kms = {k: v[0] / max(1, v[1]) for k, v in kall.items() if v[1]}
    step_kernels = [k for k in ("k_linearize", "k_point_sc", "k_stitch", "k_stitch_sum") if k in kms]
    step_kernel_ms = sum(kms[k] for k in step_kernels)
    frac_step = bytes_per_launch / (step_kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if step_kernel_ms > 0 else None
    frac_step_wall = bytes_per_launch / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS if ms_step > 0 else None

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "point-residuals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "replicas" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded textured-plane windows, photo-consistent; no dataset)",
            "config": {
                "workload": workload,
                "n_frames": N,
                "points_per_window": P,
                "windows_per_gpu": B,
                "residuals_per_step": int(R_job),
                "residuals_active_per_step": int(G_total),
                "image": "640x480",
                "parallelism": f"{args.mode}{world}" if world > 1 else "single",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_source,
                "kernel": "k_linearize",
                "avg_launch_us": klin_avg_s * 1e6,
                "event_launches": int(klin_n),
                "event_every": EVENT_EVERY,
                "algo_bytes_per_launch": bytes_per_launch,
                "algo_bytes_per_residual": algo_bytes_per_residual(N),
                "frac_step": frac_step,
                "frac_step_kernels": step_kernels,
                "step_kernel_ms": step_kernel_ms,
                "frac_step_wall": frac_step_wall,
            },
            "kernel_ms_per_step": kms,
            "ms_per_step_without_kernel_events": ms_step_no_events,
            "gn_iteration_batched": gn,
            "single_window": single,
            "s11": s11,
            "sharded_window": sharded,
            "tracker": tracker,
            "cpp_face": face,
            "cpu_baseline": cpu,
            "cpu_baseline_single_window": cpu1,
            "cpu_baseline_six_threads": cpu6,
        }
        if face and single and "optimize" in face:  # both with all 6 iterations
            face["vs_c_abi_single_window_optimize"] = (face["ms_per_gn_iteration"] /
                                                       single["optimize_all_its"]["ms_per_iteration"])
        if cpu is not None:  # like for like: the same 64-window workload on both sides
            out["speedup_vs_cpu"] = value / cpu["value"]
            out["speedup_vs_cpu_workload"] = f"{B} x S7 windows: GPU step vs {cpu['workers']} pinned CPU workers"
        if cpu1 is not None and single is not None:  # one window on each side
            out["speedup_single_window_vs_cpu"] = single["point_residuals_per_s"] / cpu1["value"]
        if cpu6 is not None:
            out["speedup_vs_cpu_six_threads"] = value / cpu6["value"]
        print(json.dumps(out), file=json_out, flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
