"""GPU parity: the HIP path (through the C ABI) against the CPU restatement (oracle/) on the
same seeded windows.

Bars (SURVEY.md §7 "Hard parts", BASELINE.json north_star):
  * per-residual arithmetic (states, energies, centerProjectedTo, JpJdF, per-point Hdd/bd/Hcd,
    HdiF, frameEnergyTH) is bit-exact: both sides round every statement in the reference's
    order with FMA contraction off;
  * linearizeAll energy: relative 1e-12 (double sums, different order);
  * stitched H, b (float accumulation reassociated on the GPU, then double): per 8x8 block
    relative Frobenius error <= 1e-4 (the north star's tolerance is 1e-4 on the energy);
  * solve: the product's solver matches the oracle's on the same system to 1e-9; end to end, x
    stays within 20x the system's float-rounding sensitivity envelope (see sensitivity());
  * resubstituted point steps: relative 1e-3 on the step vector.
"""
import numpy as np
import pytest

import oracle
from ldso_amd import BAContext, synth

pytestmark = pytest.mark.gpu

BLOCK_TOL = 1e-4


def block_errors(G, O, N):
    """max over the upper-triangle blocks of ||G-O||_F / ||O||_F (blocks: calib, frames)."""
    edges = [0, 4] + [4 + 8 * (f + 1) for f in range(N)]
    scale = np.linalg.norm(O)
    worst = 0.0
    for a in range(len(edges) - 1):
        for b in range(a, len(edges) - 1):
            g = G[edges[a]:edges[a + 1], edges[b]:edges[b + 1]]
            o = O[edges[a]:edges[a + 1], edges[b]:edges[b + 1]]
            if a == b:
                g, o = np.triu(g), np.triu(o)
            den = max(np.linalg.norm(o), 1e-12 * scale, 1e-300)
            worst = max(worst, np.linalg.norm(g - o) / den)
    return worst


def vec_block_errors(g, o, N):
    edges = [0, 4] + [4 + 8 * (f + 1) for f in range(N)]
    scale = np.linalg.norm(o)
    worst = 0.0
    for a in range(len(edges) - 1):
        gg, oo = g[edges[a]:edges[a + 1]], o[edges[a]:edges[a + 1]]
        worst = max(worst, np.linalg.norm(gg - oo) / max(np.linalg.norm(oo), 1e-12 * scale, 1e-300))
    return worst


def sensitivity(N, it, sysm, ns, x0, eps=2.0 ** -20, trials=3):
    rng = np.random.default_rng(0)
    worst = 0.0
    for _ in range(trials):
        pert = {}
        for k, v in sysm.items():
            if k in ("HA", "Hsc"):
                E = rng.standard_normal(v.shape)
                pert[k] = v * (1 + eps * (E + E.T) / 2)
            elif k in ("bA", "bsc"):
                pert[k] = v * (1 + eps * rng.standard_normal(v.shape))
            else:
                pert[k] = v
        x = oracle.solve_system(N, it, 1e-5, pert, nullspaces=ns)
        worst = max(worst, np.linalg.norm(x - x0) / np.linalg.norm(x0))
    return worst


def compare_pass(ctx, ow, win_idx, e_cpu, s_cpu, check_system=True):
    N = ow.window.n_frames
    rg, rc = ctx.residuals(win_idx), ow.residuals()
    assert np.array_equal(rg["new_state"], rc["new_state"])
    assert np.array_equal(rg["state"], rc["state"])
    assert np.array_equal(rg["flags"], rc["flags"])
    assert np.array_equal(rg["state_energy"], rc["state_energy"])
    assert np.array_equal(rg["new_energy_wo"], rc["new_energy_wo"])
    assert np.array_equal(rg["center"], rc["center"])
    act = (rc["flags"] & 1).astype(bool)
    assert np.array_equal(rg["jpjdf"][act], rc["jpjdf"][act])
    e_gpu = ctx.energy(win_idx)
    assert e_gpu[2] == e_cpu[2]
    assert abs(e_gpu[0] - e_cpu[0]) <= 1e-12 * abs(e_cpu[0]) + 1e-9
    np.testing.assert_array_equal(ctx.frame_energy_th(win_idx), ow.frame_energy_th())
    if not check_system:
        return
    pg, pc = ctx.points(win_idx), ow.points()
    for k in ("Hdd", "bd", "Hcd", "HdiF", "bdSumF", "idepth_hessian"):
        np.testing.assert_array_equal(pg[k], pc[k], err_msg=k)
    s_gpu = ctx.system(win_idx)
    errs = {k: block_errors(s_gpu[k], s_cpu[k], N) for k in ("HA", "Hsc")}
    errs.update({k: vec_block_errors(s_gpu[k], s_cpu[k], N) for k in ("bA", "bsc")})
    print("max block rel errors:", {k: f"{v:.2e}" for k, v in errs.items()})
    assert block_errors(s_gpu["HA"], s_cpu["HA"], N) < BLOCK_TOL
    assert block_errors(s_gpu["Hsc"], s_cpu["Hsc"], N) < BLOCK_TOL
    assert vec_block_errors(s_gpu["bA"], s_cpu["bA"], N) < BLOCK_TOL
    assert vec_block_errors(s_gpu["bsc"], s_cpu["bsc"], N) < BLOCK_TOL
    np.testing.assert_array_equal(s_gpu["HL"], s_cpu["HL"])
    np.testing.assert_array_equal(s_gpu["bL"], s_cpu["bL"])
    return s_gpu


@pytest.fixture(scope="module")
def ctx(built):
    c = BAContext(0)
    yield c
    c.close()


@pytest.mark.parametrize("cfg", [dict(n_frames=3, n_points=64, seed=11), dict(n_frames=5, n_points=400, seed=3),
                                 dict(synth.S7, seed=1)], ids=["N3P64", "N5P400", "S7"])
def test_single_pass_parity(ctx, cfg):
    w = synth.make_window(**cfg)
    ctx.load([w])
    ctx.linearize(fix=False, accumulate=True)
    ow = oracle.OracleWindow(synth.make_window(**cfg), threads=0)
    e_cpu, s_cpu = ow.iteration()
    s_gpu = compare_pass(ctx, ow, 0, e_cpu, s_cpu)
    # solveSystemF and resubstituteF on both sides
    ns = w.nullspaces()
    for it in (0, 2):
        xg = ctx.solve(0, it, 1e-5, ns)
        # the product's solver on the GPU system == the oracle's solver on the same system
        xo = oracle.solve_system(w.n_frames, it, 1e-5, s_gpu, nullspaces=ns)
        assert np.linalg.norm(xg - xo) <= 1e-9 * np.linalg.norm(xo)
        # end to end: float reassociation of H (~1e-6 relative) is amplified by the system's
        # conditioning.  Bar: within 20x the shift of x under a random 2^-20 relative
        # perturbation of the oracle's own H and b (its float-rounding sensitivity envelope).
        xc = oracle.solve_system(w.n_frames, it, 1e-5, s_cpu, nullspaces=ns)
        env = sensitivity(w.n_frames, it, s_cpu, ns, xc)
        rel = np.linalg.norm(xg - xc) / np.linalg.norm(xc)
        print(f"solve it={it}: |xg-xc|/|xc|={rel:.3e} envelope={env:.3e}")
        assert rel <= max(1e-6, 20 * env)
    xc = oracle.solve_system(w.n_frames, 0, 1e-5, s_cpu, nullspaces=ns)
    stg = ctx.resubstitute(0, xc, 1e-5)
    stc = ow.resubstitute(xc, 1e-5)
    assert np.linalg.norm(stg - stc) <= 1e-3 * np.linalg.norm(stc) + 1e-12


@pytest.mark.parametrize("stitch", ["split", "whole", "records"])
def test_stitch_paths_agree(built, monkeypatch, stitch):
    """The three stitch paths -- k_stitch_host with the Top / Schur halves in separate blocks
    (small grids), with one block per host (large grids: the bench's 64 windows), and k_stitch's
    per-pair records (windows over 11 keyframes) -- against the oracle on the same windows; the
    two host-stitch modes are the same arithmetic, so their systems are bitwise equal."""
    cfgs = [dict(n_frames=7, n_points=600, seed=81), dict(n_frames=4, n_points=200, seed=82),
            dict(n_frames=11, n_points=900, seed=83)]
    if stitch == "records":
        monkeypatch.setenv("LDSO_BA_STITCH_RECORDS", "1")
    else:
        monkeypatch.setenv("LDSO_BA_HS_SPLIT", "1" if stitch == "split" else "0")
    c = BAContext(0).load([synth.make_window(**cf) for cf in cfgs])
    c.linearize(fix=False, accumulate=True)
    systems = [c.system(i) for i in range(len(cfgs))]
    for i, cf in enumerate(cfgs):
        ow = oracle.OracleWindow(synth.make_window(**cf), threads=0)
        e_cpu, s_cpu = ow.iteration()
        compare_pass(c, ow, i, e_cpu, s_cpu)
    c.close()
    if stitch != "records":
        monkeypatch.setenv("LDSO_BA_HS_SPLIT", "0" if stitch == "split" else "1")
        c2 = BAContext(0).load([synth.make_window(**cf) for cf in cfgs])
        c2.linearize(fix=False, accumulate=True)
        for i in range(len(cfgs)):
            s2 = c2.system(i)
            for k in ("HA", "Hsc", "bA", "bsc"):
                np.testing.assert_array_equal(systems[i][k], s2[k], err_msg=k)
        c2.close()


def test_caller_point_order_does_not_matter(built):
    """The same window with each host's points in image row order (as LDSO's pixel selection emits
    them) instead of random order: every per-residual and per-point result is the same value for
    the same residual / point (bit for bit), the system within the block tolerance (the chunks hold
    other residuals, so the Top partial sums reassociate), #IN equal."""
    cfg = dict(n_frames=6, n_points=700, seed=91)
    w = synth.make_window(**cfg)
    o = synth.in_image_order(synth.make_window(**cfg))
    c1, c2 = BAContext(0).load([w]), BAContext(0).load([o])
    for c in (c1, c2):
        c.linearize()
    r1, r2 = c1.residuals(0), c2.residuals(0)
    for k in r1:
        np.testing.assert_array_equal(r2[k], np.asarray(r1[k])[o.res_order], err_msg=k)
    p1, p2 = c1.points(0), c2.points(0)
    for k in p1:
        np.testing.assert_array_equal(p2[k], np.asarray(p1[k])[o.point_order], err_msg=k)
    e1, e2 = c1.energy(0), c2.energy(0)
    assert e1[2] == e2[2] and abs(e1[0] - e2[0]) <= 1e-12 * abs(e1[0])
    s1, s2 = c1.system(0), c2.system(0)
    N = cfg["n_frames"]
    for k in ("HA", "Hsc"):
        assert block_errors(s2[k], s1[k], N) < BLOCK_TOL, k
    for k in ("bA", "bsc"):
        assert vec_block_errors(s2[k], s1[k], N) < BLOCK_TOL, k
    c1.close()
    c2.close()


def test_repeated_passes_and_oob_stickiness(ctx):
    """OOB is sticky inside optimize(): later passes return the stored state_energy."""
    cfg = dict(n_frames=6, n_points=800, seed=5, baseline=0.12)
    ctx.load([synth.make_window(**cfg)])
    ow = oracle.OracleWindow(synth.make_window(**cfg), threads=0)
    for _ in range(3):
        ctx.linearize(fix=False, accumulate=True)
        e_cpu, s_cpu = ow.iteration()
        compare_pass(ctx, ow, 0, e_cpu, s_cpu)
    ctx.reset_oob()
    ow.reset_oob()
    ctx.linearize(fix=True, accumulate=False)
    e_cpu = ow.linearize_all(True)
    compare_pass(ctx, ow, 0, e_cpu, None, check_system=False)
    rg, rc = ctx.residuals(0), ow.residuals()
    np.testing.assert_array_equal(rg["rel_bs"], rc["rel_bs"])


def test_stitched_system_is_bitwise_repeatable(ctx):
    """k_stitch writes one record per (pair, block) and k_stitch_sum adds them in a fixed order:
    repeated passes over the same state give the same system to the bit (FullSystem's
    accumulateAF_MT/accumulateSCF_MT reduce in a fixed order too; the GPU order differs from the
    CPU's, hence the block tolerance against the oracle in compare_pass)."""
    cfgs = [dict(n_frames=7, n_points=900, seed=13), dict(n_frames=3, n_points=200, seed=14)]
    ctx.load([synth.make_window(**c) for c in cfgs])
    ref = None
    for _ in range(4):
        ctx.linearize(fix=False, accumulate=True)
        sy = [ctx.system(i) for i in range(len(cfgs))]
        if ref is None:
            ref = sy
            continue
        for a, b in zip(ref, sy):
            for k in ("HA", "Hsc", "bA", "bsc"):
                np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    for i, c in enumerate(cfgs):
        ow = oracle.OracleWindow(synth.make_window(**c), threads=0)
        e_cpu, s_cpu = ow.iteration()
        compare_pass(ctx, ow, i, e_cpu, s_cpu)


def test_multi_window_batch(ctx):
    cfgs = [dict(n_frames=7, n_points=500, seed=s) for s in (21, 22)] + [dict(n_frames=4, n_points=300, seed=23)]
    ctx.load([synth.make_window(**c) for c in cfgs])
    ctx.linearize(fix=False, accumulate=True)
    for i, c in enumerate(cfgs):
        ow = oracle.OracleWindow(synth.make_window(**c), threads=0)
        e_cpu, s_cpu = ow.iteration()
        compare_pass(ctx, ow, i, e_cpu, s_cpu)


def test_state_update_between_passes(ctx):
    """doStepFromBackup -> setPrecalcValues -> ldso_ba_update, then a fresh pass."""
    cfg = dict(n_frames=5, n_points=600, seed=31)
    w = synth.make_window(**cfg)
    ctx.load([w])
    ctx.linearize()
    w2 = synth.make_window(**cfg)
    w2.frames["state"][2, :6] += 2e-3
    w2.point_data[:, 2] *= 1.01
    w2.refresh_frame_terms()
    ctx.update(0, w2)
    ctx.linearize()
    ow = oracle.OracleWindow(synth.make_window(**cfg), threads=0)
    ow.iteration()
    ow.update(w2)
    e_cpu, s_cpu = ow.iteration()
    compare_pass(ctx, ow, 0, e_cpu, s_cpu)


def test_shards_sum_to_full(built):
    """Host-frame contiguous sharding: per-shard systems sum to the full system; every shard
    keeps the priors (HL, bL are not reduced: each rank adds them in its own solve)."""
    cfg = dict(n_frames=7, n_points=900, seed=41)
    full = BAContext(0).load([synth.make_window(**cfg)])
    full.linearize()
    s_full = full.system(0)
    parts = []
    for r in range(3):
        c = BAContext(0).load([synth.make_window(**cfg)], shard_rank=r, shard_count=3)
        c.linearize()
        parts.append(c.system(0))
        c.close()
    N = cfg["n_frames"]
    for k in ("HA", "Hsc"):
        tot = sum(p[k] for p in parts)
        assert block_errors(tot, s_full[k], N) < BLOCK_TOL
    for k in ("bA", "bsc"):
        assert vec_block_errors(sum(p[k] for p in parts), s_full[k], N) < BLOCK_TOL
    for p in parts:
        np.testing.assert_array_equal(p["HL"], s_full["HL"])
        np.testing.assert_array_equal(p["bL"], s_full["bL"])
    full.close()


def test_s11_split_over_four_contexts(built):
    """BASELINE config 4's split as far as one GPU allows: the S11 window (11 keyframes, 8000
    points) loaded as 4 contexts with shard_count = 4 (the host-frame partition of SURVEY §8e).
    The four partial systems sum to the unsharded one within BLOCK_TOL, the four energy / #IN
    pairs sum to the unsharded ones, and ldso_ba_frame_threshold_gathered over the four exported
    newest-frame slots re-selects the unsharded setNewFrameEnergyTH threshold on every shard."""
    import ctypes as C

    import torch

    from ldso_amd import _lib as L

    cfg = dict(synth.S11, seed=2)
    world = 4
    full = BAContext(0).load([synth.make_window(**cfg)])
    full.linearize()
    s_full, e_full, th_full = full.system(0), full.energy(0), full.frame_energy_th(0)
    full.close()
    shards = [BAContext(0).load([synth.make_window(**cfg)], shard_rank=r, shard_count=world) for r in range(world)]
    parts, strides = [], []
    for c in shards:
        c.linearize()
        parts.append((c.system(0), c.energy(0)))
        st = C.c_int64()
        L.check(c._lib.ldso_ba_newest_stride(c._h, C.byref(st)))
        strides.append(st.value)
    assert sum(c.stats()["residuals"] for c in shards) == synth.make_window(**cfg).n_residuals
    N = cfg["n_frames"]
    for k in ("HA", "Hsc"):
        assert block_errors(sum(p[0][k] for p in parts), s_full[k], N) < BLOCK_TOL, k
    for k in ("bA", "bsc"):
        assert vec_block_errors(sum(p[0][k] for p in parts), s_full[k], N) < BLOCK_TOL, k
    assert sum(p[1][2] for p in parts) == e_full[2]
    assert abs(sum(p[1][0] for p in parts) - e_full[0]) <= 1e-9 * abs(e_full[0])
    stride = max(strides)
    gathered = torch.empty(world * stride, dtype=torch.float32, device="cuda")
    for r, c in enumerate(shards):
        L.check(c._lib.ldso_ba_export_newest(c._h, gathered[r * stride:].data_ptr(), stride))
    torch.cuda.synchronize()
    for c in shards:
        L.check(c._lib.ldso_ba_frame_threshold_gathered(c._h, gathered.data_ptr(), world, stride))
        np.testing.assert_array_equal(c.frame_energy_th(0)[-1], th_full[-1])
        c.close()


def test_s11_window(ctx):
    cfg = dict(synth.S11, seed=2)
    ctx.load([synth.make_window(**cfg)])
    ctx.linearize()
    ow = oracle.OracleWindow(synth.make_window(**cfg), threads=0)
    e_cpu, s_cpu = ow.iteration()
    compare_pass(ctx, ow, 0, e_cpu, s_cpu)


def _zoomed_window(seed, dz, angle):
    """A synthetic window whose newest keyframe moved dz toward the plane and rolled by angle
    (radians) about its optical axis: patterns projected into it spread over more pixels."""
    w = synth.make_window(n_frames=4, n_points=600, seed=seed, finalize=False)
    T = w.frames["world_to_cam_evalpt"][-1]
    R, t = T[:9].reshape(3, 3), T[9:].copy()
    c, s = np.cos(angle), np.sin(angle)
    Rz = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])
    T[:9] = (Rz @ R).reshape(-1)
    T[9:] = Rz @ t - np.array([0, 0, dz])
    w.frames["world_to_cam_evalpt"][-1] = T
    return w.refresh_frame_terms()


def _pattern_spreads(w):
    """max - min of floor(projected x) and of floor(y) over each residual's 8 pattern pixels
    (float64 host projection with the window's precalc), for residuals with all pixels in view."""
    pat = np.array([[0, -2], [-1, -1], [1, -1], [-2, 0], [0, 0], [2, 0], [-1, 1], [0, 2]], np.float64)
    N, out = w.n_frames, []
    for p in range(w.point_data.shape[0]):
        h = w.point_host[p]
        u, v, idz = w.point_data[p, 0], w.point_data[p, 1], w.point_data[p, 2]
        for r in range(w.point_res_begin[p], w.point_res_begin[p + 1]):
            pre = w.precalc[w.res_target[r] * N + h].astype(np.float64)
            q = np.stack([u + pat[:, 0], v + pat[:, 1], np.ones(8)], 1) @ pre[:9].reshape(3, 3).T + pre[9:12] * idz
            if np.any(q[:, 2] <= 0):
                continue
            x, y = q[:, 0] / q[:, 2], q[:, 1] / q[:, 2]
            if x.min() > 2 and y.min() > 2 and x.max() < w.width - 4 and y.max() < w.height - 4:
                out.append((np.ptp(np.floor(x)), np.ptp(np.floor(y))))
    return np.array(out)


@pytest.mark.parametrize("dz,angle", [(0.0, 0.0), (0.6, 0.3), (1.0, 0.8)], ids=["plain", "zoom1.4", "zoom2"])
def test_wide_pattern_footprints(ctx, dz, angle):
    """k_linearize loads each residual's tap footprint into a 3-band x 9-column box; residuals
    whose projected pattern spreads more (zoom, roll) gather per lane.  Both paths, in one
    window, are bit-exact against the oracle."""
    w = _zoomed_window(5, dz, angle)
    sp = _pattern_spreads(w)
    wide = np.mean((sp[:, 0] > 5) | (sp[:, 1] > 5))
    print(f"dz={dz} angle={angle}: {len(sp)} residuals in view, {wide:.1%} with spread > 5")
    if dz > 0:
        assert 0.03 < wide < 0.5  # both paths exercised in one pass
    ctx.load([w])
    ctx.linearize()
    ow = oracle.OracleWindow(_zoomed_window(5, dz, angle), threads=0)
    e_cpu, s_cpu = ow.iteration()
    compare_pass(ctx, ow, 0, e_cpu, s_cpu)


def test_sharded_frame_threshold_exchange(built):
    """ldso_ba_export_newest + ldso_ba_frame_threshold_gathered: three shards' newest-frame
    slots concatenated as an all-gather would lay them out re-select the unsharded threshold,
    for a batch of windows (also one whose newest segment exceeds the LDS staging size)."""
    import ctypes as C

    import torch

    from ldso_amd import _lib as L

    cfgs = [dict(n_frames=7, n_points=900, seed=43), dict(n_frames=5, n_points=12000, seed=44),
            dict(n_frames=4, n_points=30, seed=45)]
    full = BAContext(0).load([synth.make_window(**c) for c in cfgs])
    full.linearize()
    th_full = [full.frame_energy_th(i) for i in range(len(cfgs))]
    world = 3
    ctxs = [BAContext(0).load([synth.make_window(**c) for c in cfgs], shard_rank=r, shard_count=world)
            for r in range(world)]
    strides = []
    for c in ctxs:
        c.linearize()
        s = C.c_int64()
        L.check(c._lib.ldso_ba_newest_stride(c._h, C.byref(s)))
        strides.append(s.value)
    stride = max(strides)
    nw = len(cfgs)
    gathered = torch.empty(world * nw * stride, dtype=torch.float32, device="cuda")
    for r, c in enumerate(ctxs):
        L.check(c._lib.ldso_ba_export_newest(c._h, gathered[r * nw * stride:].data_ptr(), stride))
    torch.cuda.synchronize()
    for c in ctxs:
        L.check(c._lib.ldso_ba_frame_threshold_gathered(c._h, gathered.data_ptr(), world, stride))
        for i in range(nw):
            np.testing.assert_array_equal(c.frame_energy_th(i), th_full[i])
        c.close()
    full.close()


@pytest.mark.parametrize("layout", [1, 3])
def test_image_layouts_agree(built, layout):
    """k_linearize on both frame layouts (2x4 tiles of [I, dx, dy, 0] texels; intensity only,
    band-interleaved, with the gradients recomputed) is bit-exact on the per-residual outputs."""
    cfg = dict(n_frames=6, n_points=700, seed=23)
    c = BAContext(0)
    c.set_tuning(2, layout)  # LDSO_BA_TUNE_TILED_IMAGES, before load
    c.load([synth.make_window(**cfg)])
    c.linearize(fix=False, accumulate=True)
    ow = oracle.OracleWindow(synth.make_window(**cfg), threads=0)
    e_cpu, s_cpu = ow.iteration()
    compare_pass(c, ow, 0, e_cpu, s_cpu)
    c.close()


@pytest.mark.parametrize("key,value", [(1, 3), (2, 0), (2, 2), (8, 2), (11, 1), (10, 3), (14, 1)])
def test_removed_tuning_variants_are_rejected(built, key, value):
    c = BAContext(0)
    with pytest.raises(RuntimeError):
        c.set_tuning(key, value)
    c.close()


def test_intensity_layout_falls_back_when_gradients_are_not_makeimages(built):
    """Layout 3 recomputes gradients with makeImages' rule; a caller whose dI gradients differ
    (here: every dx nudged) must still get results from ITS gradients."""
    cfg = dict(n_frames=4, n_points=300, seed=29)
    w = synth.make_window(**cfg)
    w.dI = w.dI.copy()
    w.dI[:, :, 1] += np.float32(0.125)
    c = BAContext(0)
    c.set_tuning(2, 3)
    c.load([w])
    c.linearize()
    w2 = synth.make_window(**cfg)
    w2.dI = w.dI.copy()
    ow = oracle.OracleWindow(w2, threads=0)
    e_cpu, s_cpu = ow.iteration()
    compare_pass(c, ow, 0, e_cpu, s_cpu)
    c.close()


@pytest.mark.parametrize("chunk", [16, 32, 64])
def test_chunk_sizes_agree(built, chunk):
    cfg = dict(n_frames=5, n_points=500, seed=37)
    c = BAContext(0)
    c.set_tuning(6, chunk)  # LDSO_BA_TUNE_TOP_CHUNK
    c.load([synth.make_window(**cfg)])
    c.linearize()
    ow = oracle.OracleWindow(synth.make_window(**cfg), threads=0)
    e_cpu, s_cpu = ow.iteration()
    compare_pass(c, ow, 0, e_cpu, s_cpu)
    c.close()


@pytest.mark.parametrize("order", [1, 2])
@pytest.mark.parametrize("chunk", [16, 64])
def test_item_orders_agree(built, order, chunk):
    """k_linearize's chunk orders (LDSO_BA_TUNE_ITEM_ORDER: 1 host-major; 2 each bucket ranked by
    the projection into its target and dealt over balanced chunks) hold other residuals per chunk,
    so against the oracle: per-residual / per-point outputs bit for bit, the system within
    BLOCK_TOL, over two windows batched (one with one-residual buckets) and two passes."""
    cfgs = [dict(n_frames=7, n_points=900, seed=41), dict(n_frames=3, n_points=40, seed=42)]
    c = BAContext(0)
    c.set_tuning(6, chunk)   # LDSO_BA_TUNE_TOP_CHUNK
    c.set_tuning(10, order)  # LDSO_BA_TUNE_ITEM_ORDER
    c.load([synth.make_window(**cf) for cf in cfgs])
    ows = [oracle.OracleWindow(synth.make_window(**cf), threads=0) for cf in cfgs]
    for _ in range(2):
        c.linearize()
        for i, ow in enumerate(ows):
            e_cpu, s_cpu = ow.iteration()
            compare_pass(c, ow, i, e_cpu, s_cpu)
    c.close()


@pytest.mark.parametrize("cfg", [dict(n_frames=2, n_points=90, seed=81), dict(n_frames=3, n_points=33, seed=82),
                                 dict(n_frames=8, n_points=700, seed=83), dict(n_frames=16, n_points=300, seed=84)])
def test_window_sizes_over_two_passes(built, cfg):
    """Windows from 2 to 16 keyframes (one-residual buckets, partial chunks, the widest Schur
    block) match the oracle over two passes: per-residual and per-point outputs bit for bit, the
    system within BLOCK_TOL."""
    c = BAContext(0)
    c.load([synth.make_window(**cfg)])
    ow = oracle.OracleWindow(synth.make_window(**cfg), threads=0)
    for _ in range(2):
        c.linearize()
        e_cpu, s_cpu = ow.iteration()
        compare_pass(c, ow, 0, e_cpu, s_cpu)
    c.close()


def test_windows_of_different_sizes_in_one_context(built):
    """Five windows of different sizes in one context give the same per-window results."""
    cfgs = [dict(n_frames=4 + (i % 3), n_points=150 + 40 * i, seed=60 + i) for i in range(5)]
    c = BAContext(0)
    c.load([synth.make_window(**cf) for cf in cfgs])
    c.linearize()
    c.linearize()
    for i, cf in enumerate(cfgs):
        ow = oracle.OracleWindow(synth.make_window(**cf), threads=0)
        ow.iteration()
        e_cpu, s_cpu = ow.iteration()
        compare_pass(c, ow, i, e_cpu, s_cpu)
    c.close()


@pytest.mark.parametrize("kernel", ["reg", "lds", "lds_forced"])
def test_device_solve_and_resubstitute_match_host_path(built, kernel, monkeypatch):
    """ldso_ba_solve_device / resubstitute_device reproduce the host solver and the host-staged
    resubstitution bit for bit, for a batch of windows of different sizes, at iteration 0 (no
    orthogonalisation) and 2 (nullspace projection: the Cholesky path, and the Jacobi path for a
    rank-deficient nullspace set).  Both factorisations: k_solve_reg (every window <= 7
    keyframes) and k_solve (a window of 11 keyframes in the batch, or LDSO_BA_SOLVE_LDS=1)."""
    cfgs = [dict(n_frames=3, n_points=120, seed=70), dict(n_frames=7, n_points=900, seed=71),
            dict(n_frames=11, n_points=1200, seed=72), dict(n_frames=5, n_points=400, seed=73)]
    if kernel != "lds":
        cfgs = [cf for cf in cfgs if cf["n_frames"] <= 7] + [dict(n_frames=7, n_points=300, seed=75, baseline=0.2)]
    if kernel == "lds_forced":
        monkeypatch.setenv("LDSO_BA_SOLVE_LDS", "1")
    ws = [synth.make_window(**cf) for cf in cfgs]
    ns = [w.nullspaces() for w in ws]
    c = BAContext(0)
    c.set_tuning(12, 1)  # LDSO_BA_TUNE_SOLVE_EXACT: the pivoted factorisation
    c.load(ws)
    c.linearize()
    for it in (0, 2):
        xd = c.solve_device(it, 1e-5, ns)
        for i in range(len(ws)):
            xh = c.solve(i, it, 1e-5, ns[i])
            np.testing.assert_array_equal(xd[i], xh)
        sd = c.resubstitute_device(1e-5)
        for i in range(len(ws)):
            sh = c.resubstitute(i, xd[i], 1e-5)
            np.testing.assert_array_equal(sd[i], sh)
    # rank-deficient nullspaces: the Jacobi fallback of the projection, also bit for bit
    ns_deg = [a.copy() for a in ns]
    for a in ns_deg:
        a[6] = a[5]
    xd = c.solve_device(2, 1e-5, ns_deg)
    for i in range(len(ws)):
        np.testing.assert_array_equal(xd[i], c.solve(i, 2, 1e-5, ns_deg[i]))
    # fused iteration == the separate calls, bit for bit: the stitch sums every packed element
    # in a fixed pair order (k_stitch_sum), so a new pass over the same state rebuilds the
    # same system
    c.linearize()
    xs_ref = c.solve_device(2, 1e-5, ns)
    st_ref = c.resubstitute_device(1e-5)
    e_ref = [c.energy(i) for i in range(len(ws))]
    e, xs, sts = c.iterate(2, 1e-5, ns)
    for i in range(len(ws)):
        np.testing.assert_array_equal(xs[i], xs_ref[i])
        np.testing.assert_array_equal(sts[i], st_ref[i])
        assert e[i][2] == e_ref[i][2] and abs(e[i][0] - e_ref[i][0]) <= 1e-12 * abs(e_ref[i][0])
    c.close()


@pytest.mark.parametrize("it", [0, 2])
def test_fast_device_solve_matches_host_within_rounding(built, it):
    """The default device solve (k_solve_fast: unpivoted blocked LDL^T on the Jacobi-scaled,
    damped, positive definite system) against the host's pivoted solver on the same stitched
    system: x within 20x the system's float-rounding sensitivity envelope (and 1e-9 relative at
    worst), for windows of 3 to 11 keyframes batched in one launch; then its resubstitution
    against the host-staged one from the same x."""
    cfgs = [dict(n_frames=3, n_points=120, seed=70), dict(n_frames=7, n_points=900, seed=71),
            dict(n_frames=11, n_points=1200, seed=72), dict(n_frames=5, n_points=400, seed=73),
            dict(n_frames=7, n_points=300, seed=75, baseline=0.2)]
    ws = [synth.make_window(**cf) for cf in cfgs]
    ns = [w.nullspaces() for w in ws]
    c = BAContext(0).load(ws)
    c.linearize()
    xd = c.solve_device(it, 1e-5, ns)
    for i, w in enumerate(ws):
        xh = c.solve(i, it, 1e-5, ns[i])
        env = sensitivity(w.n_frames, it, c.system(i), ns[i], xh)
        rel = np.linalg.norm(xd[i] - xh) / np.linalg.norm(xh)
        print(f"window {i} (N={w.n_frames}) it={it}: |x_fast - x_host|/|x_host| = {rel:.3e}, envelope {env:.3e}")
        assert rel <= max(1e-12, min(1e-9, 20 * env))
    sd = c.resubstitute_device(1e-5)
    for i in range(len(ws)):
        sh = c.resubstitute(i, xd[i], 1e-5)
        np.testing.assert_array_equal(sd[i], sh)
    c.close()


def test_prepared_nullspaces_follow_the_callers_nullspaces(built):
    """k_ortho_prep's normalised nullspaces and (N^T N)^-1 are kept across calls while the caller
    passes the same nullspaces, and redone when they change (other values or another count):
    exact-mode x stays bit-identical to the host solver with the nullspaces of each call."""
    cfg = dict(n_frames=5, n_points=400, seed=62)
    w = synth.make_window(**cfg)
    na = w.nullspaces()
    rng = np.random.default_rng(5)
    nb = na + 0.05 * rng.standard_normal(na.shape)
    c = BAContext(0).load([w])
    c.set_tuning(12, 1)
    c.linearize()
    for ns, k in ((na, 7), (na, 7), (nb, 7), (nb, 5), (na, 7)):
        xd = c.solve_device(2, 1e-5, [ns], n_null=k)[0]
        np.testing.assert_array_equal(xd, c.solve(0, 2, 1e-5, ns[:k]))
    c.close()


def test_iterate_replay_refreshes_host_copies_and_projects_only_with_this_calls_nullspaces(built, monkeypatch):
    """A replayed ldso_ba_iterate graph (LDSO_BA_ITERATE_GRAPH=1; direct launches are the default)
    invalidates the host copies of the system / energies (the replay skips the captured calls'
    host side), and a device solve projects only with the nullspaces passed in THAT call (none:
    no projection, as the host solver)."""
    monkeypatch.setenv("LDSO_BA_ITERATE_GRAPH", "1")
    cfg = dict(n_frames=5, n_points=400, seed=61)
    w = synth.make_window(**cfg)
    ns = [w.nullspaces()]
    c = BAContext(0).load([w])
    c.set_tuning(12, 1)  # exact mode: bit-identical to the host solver
    c.update_points(0, w.point_data[:, 2:6])  # allocates its staging now, so the graph below stays valid
    c.iterate(2, 1e-5, ns)  # captures the graph
    s0 = c.system(0)        # host copy cached
    vals = np.stack([w.point_data[:, 2] * 1.01, w.point_data[:, 3], w.point_data[:, 4], w.point_data[:, 5]], 1)
    c.update_points(0, vals)
    e, _, _ = c.iterate(2, 1e-5, ns)  # replays on the changed points
    s1 = c.system(0)
    w2 = synth.make_window(**cfg)
    w2.point_data[:, 2] = vals[:, 0]
    fresh = BAContext(0).load([w2])
    fresh.linearize()
    sf = fresh.system(0)
    for k in ("HA", "Hsc", "bA", "bsc"):
        np.testing.assert_array_equal(s1[k], sf[k], err_msg=k)
    assert not np.array_equal(s0["HA"], s1["HA"])
    assert e[0][2] == fresh.energy(0)[2]
    # projection only with this call's nullspaces
    x_ns = c.solve_device(2, 1e-5, ns)[0]
    x_none = c.solve_device(2, 1e-5, None)[0]
    np.testing.assert_array_equal(x_ns, c.solve(0, 2, 1e-5, ns[0]))
    np.testing.assert_array_equal(x_none, c.solve(0, 2, 1e-5, None))
    assert not np.array_equal(x_ns, x_none)
    fresh.close()
    c.close()


def test_device_solve_rejects_windows_above_eleven_keyframes(built):
    c = BAContext(0).load([synth.make_window(n_frames=12, n_points=200, seed=74)])
    c.linearize()
    with pytest.raises(RuntimeError, match="11 keyframes"):
        c.solve_device(0)
    c.close()


def test_rccl_world1_exchange_keeps_results(built):
    """ldso_ba_comm_init with one rank: every pass ends with the in-library RCCL exchange
    (all-reduce of the packed systems and energies, all-gather of the newest-frame energies and
    k_frame_th's re-selection) on the context stream; a single rank's results must equal those
    of a context without a communicator, bit for bit (the stitch is order-fixed)."""
    from ldso_amd import _lib as L

    cfg = dict(n_frames=6, n_points=700, seed=51)
    a = BAContext(0).load([synth.make_window(**cfg)])
    uid = np.zeros(128, np.uint8)
    L.check(L.lib().ldso_ba_comm_unique_id(uid.ctypes.data))
    b = BAContext(0).comm_init(uid.tobytes(), 0, 1).load([synth.make_window(**cfg)], shard_rank=0, shard_count=1)
    for _ in range(3):
        a.linearize(fix=False, accumulate=True)
        b.linearize(fix=False, accumulate=True)
    ra, rb = a.residuals(0), b.residuals(0)
    for k in ("new_state", "state", "state_energy", "new_energy_wo", "jpjdf"):
        np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)
    np.testing.assert_array_equal(a.frame_energy_th(0), b.frame_energy_th(0))
    np.testing.assert_array_equal(a.energy(0), b.energy(0))
    sa, sb = a.system(0), b.system(0)
    for k in ("HA", "Hsc", "bA", "bsc"):
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
    with pytest.raises(RuntimeError, match="already"):
        b.comm_init(uid.tobytes(), 0, 1)
    a.close()
    b.close()


@pytest.mark.parametrize("exact", [False, True])
def test_rccl_world1_optimize_keeps_results(built, exact):
    """ldso_ba_optimize on a context with a (world-1) communicator -- direct launches, the
    exchange after every pass, the energy history written after it, sumNID walked over the
    exchange's gathered |idepth| runs (in k_solve_fast's extra blocks, or with the exact solve in
    k_frame_th's) -- equals the same call on a context without one (graph replay), bit for bit:
    iteration counts and statuses included, so the canbreak exits saw the same sumNID."""
    from ldso_amd import _lib as L

    cfg = dict(n_frames=6, n_points=701, seed=52)  # a run length that is not a multiple of 4
    w = synth.make_window(**cfg)
    ns = [w.nullspaces()]
    a = BAContext(0).load([synth.make_window(**cfg)])
    uid = np.zeros(128, np.uint8)
    L.check(L.lib().ldso_ba_comm_unique_id(uid.ctypes.data))
    b = BAContext(0).comm_init(uid.tobytes(), 0, 1).load([synth.make_window(**cfg)], shard_rank=0, shard_count=1)
    if exact:
        a.set_tuning(12, 1)  # LDSO_BA_TUNE_SOLVE_EXACT
        b.set_tuning(12, 1)
    ra = a.optimize(4, nullspaces=ns)
    rb = b.optimize(4, nullspaces=ns)
    for x, y in zip(ra, rb):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    a.close()
    b.close()


def test_degenerate_windows_in_a_batch(built):
    """A window without points and a window whose residuals all start OOB, batched with a normal
    one: every window matches the oracle over two passes (the degenerate ones give zero energies
    and prior-only systems), and ldso_ba_optimize over the batch stays finite and leaves the
    normal window's result equal to optimising it alone."""
    cfgs = [dict(n_frames=4, n_points=200, seed=91), dict(n_frames=3, n_points=0, seed=92),
            dict(n_frames=5, n_points=60, seed=93)]

    def make(i):
        w = synth.make_window(**cfgs[i])
        if i == 2:
            w.res_state[:] = 1  # ResState::OOB: linearize returns the stored energy at once
        return w

    c = BAContext(0)
    c.load([make(i) for i in range(3)])
    ows = [oracle.OracleWindow(make(i), threads=0) for i in range(3)]
    for _ in range(2):
        c.linearize()
        for i, ow in enumerate(ows):
            e_cpu, s_cpu = ow.iteration()
            compare_pass(c, ow, i, e_cpu, s_cpu)
    assert c.energy(1)[2] == 0 and c.energy(2)[2] == 0
    c.close()

    ws = [make(i) for i in range(3)]
    both = BAContext(0).load(ws)
    e3, fr3, co3, id3 = both.optimize(3, nullspaces=[w.nullspaces() for w in ws])[:4]
    assert np.all(np.isfinite(e3)) and np.all(np.isfinite(fr3["state"])) and np.all(np.isfinite(co3))
    assert len(id3[1]) == 0 and np.all(np.isfinite(id3[2]))
    w0 = make(0)
    one = BAContext(0).load([w0])
    e1, fr1, _, id1 = one.optimize(3, nullspaces=[w0.nullspaces()])[:4]
    np.testing.assert_allclose(e3[:, 0, 0], e1[:, 0, 0], rtol=1e-9)
    np.testing.assert_allclose(fr3["state"][:w0.n_frames], fr1["state"], rtol=1e-9, atol=1e-15)
    np.testing.assert_allclose(id3[0], id1[0], rtol=1e-6)
    one.close()
    both.close()


def test_records_keep_the_pass_geometry(built):
    """The 24-B records hold (j0, j1) and the pass's idepth; JpJdF[0..5] is re-formed from the
    centre geometry of the pass (the per-pair snapshot), not from the live state: after the
    points' idepths and the frames' precalc change (ldso_ba_update_points, ldso_ba_update), the
    JpJdF read back and the resubstitution's point steps are bit for bit those of the pass, as the
    reference's stored JpJdF would give (Residuals.h:120-129, EnergyFunctional.cc:638-667)."""
    cfg = dict(n_frames=5, n_points=400, seed=63)
    w = synth.make_window(**cfg)
    c = BAContext(0).load([w])
    c.linearize()
    jp1 = c.residuals(0)["jpjdf"]
    x = np.random.default_rng(3).standard_normal(w.dim) * 1e-4
    st1 = c.resubstitute(0, x, 1e-5)
    w2 = synth.make_window(**cfg)
    fr = np.ascontiguousarray(w2.frames).copy()
    fr["state"][1, 0] += 1e-3  # another pose: another precalc
    w2.frames = fr
    w2.refresh_frame_terms()
    c.update(0, w2)
    vals = np.stack([w.point_data[:, 2] * 1.01, w.point_data[:, 3], w.point_data[:, 4], w.point_data[:, 5]], 1)
    c.update_points(0, vals)
    jp2 = c.residuals(0)["jpjdf"]
    st2 = c.resubstitute(0, x, 1e-5)
    np.testing.assert_array_equal(jp1, jp2)
    np.testing.assert_array_equal(st1, st2)
    c.linearize()  # a new pass takes the new state
    assert not np.array_equal(c.residuals(0)["jpjdf"], jp1)
    c.close()
