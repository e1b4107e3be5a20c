"""Randomised immature-point sweep: seeded draws of frame size, scene texture
(blob scale, pixel noise, NaN pixels), number of hosts (1-8) with random camera models, rotations
up to 0.15 rad about random axes, translations and affine brightness pairs, features anywhere in
the frame (borders included), pattern scales 1 or 2, and resident records whose previous statuses
and inverse-depth intervals are drawn at random -- through ldso_ct_make_immature and three
successive ldso_ct_trace calls against the oracle, record for record and byte for byte
(tests/test_immature.py's bar: NaN equals NaN), and the per-status counts exactly."""
import numpy as np
import pytest

import oracle
from ldso_amd import _lib as L
from test_immature import blob_image, differing

pytestmark = pytest.mark.gpu

SIZES = [(640, 480), (317, 203), (752, 480), (1242, 375), (160, 120)]


def pose_tables(rng, w, h, n_hosts):
    krki, kt, aff = [], [], []
    for _ in range(n_hosts):
        f = float(rng.uniform(0.5, 1.1)) * w
        K = np.array([[f, 0, (w - 1) / 2 + rng.uniform(-0.05, 0.05) * w],
                      [0, f * rng.uniform(0.95, 1.05), (h - 1) / 2 + rng.uniform(-0.05, 0.05) * h], [0, 0, 1]])
        axis = rng.standard_normal(3)
        axis /= np.linalg.norm(axis)
        ang = float(rng.uniform(0, 0.15))
        A = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
        R = np.eye(3) + np.sin(ang) * A + (1 - np.cos(ang)) * A @ A
        t = rng.standard_normal(3) * np.array([0.05, 0.05, 0.02]) * float(rng.choice([0.1, 1.0, 5.0]))
        krki.append((K @ R @ np.linalg.inv(K)).astype(np.float32))
        kt.append((K @ t).astype(np.float32))
        aff.append(np.array((rng.uniform(0.7, 1.4), rng.normal(0, 8)), np.float32))
    return np.stack(krki), np.stack(kt), np.stack(aff)


@pytest.mark.parametrize("case", range(10))
def test_random_trace_matches_oracle(built, case):
    from ldso_amd.tracker import CoarseTracker

    rng = np.random.default_rng(13000 + case)
    w, h = SIZES[rng.integers(len(SIZES))]
    n_hosts = int(rng.integers(1, 9))
    sig = [(1.0, 3.0), (2.0, 8.0), (4.0, 16.0)][rng.integers(3)]
    noise = float(rng.choice([0.0, 0.5, 3.0]))
    shift = float(rng.uniform(-12, 12))
    print(f"case {case}: {w}x{h}, {n_hosts} hosts, blobs {sig}, noise {noise}, shift {shift:.2f}")
    host = blob_image(w, h, seed=case, sigma=sig)
    new = blob_image(w, h, shift=shift, seed=case, sigma=sig, a=float(rng.uniform(0.8, 1.25)), b=float(rng.normal(0, 6)))
    host += (noise * rng.standard_normal(host.shape)).astype(np.float32)
    new += (noise * rng.standard_normal(new.shape)).astype(np.float32)
    if rng.random() < 0.5:  # a few NaN pixels (dead pixels of a real frame)
        for img in (host, new):
            img[rng.integers(0, h, 4), rng.integers(0, w, 4)] = np.nan
    krki, kt, aff = pose_tables(rng, w, h, n_hosts)
    ct = CoarseTracker(w, h)
    ct.set_new_frame(host)
    dH = oracle.make_images(host, w, h)[0][0]
    recs = []
    for i in range(n_hosts):
        n = int(rng.integers(0, 1500))
        m = int(rng.choice([3, 5, 10]))  # feature margin: down to the 4-pixel border the pattern reads
        uv = np.stack([rng.uniform(m, w - m - 1, n), rng.uniform(m, h - m - 1, n)], 1).astype(np.float32)
        typ = float(rng.choice([1.0, 2.0]))
        got = ct.make_immature(uv, typ, i)
        ref = oracle.ip_make(dH, w, h, uv, typ, i)
        assert differing(got, ref).size == 0, i
        recs.append(got)
    pts = np.concatenate(recs) if recs else np.zeros(0, L.IMMATURE_DTYPE)
    if len(pts):
        k = rng.random(len(pts))
        pts["last_status"][k < 0.3] = rng.integers(0, 6, int((k < 0.3).sum()))
        fin = rng.random(len(pts)) < 0.3
        lo = rng.uniform(0.0, 1.0, int(fin.sum())).astype(np.float32)
        pts["idepth_min"][fin], pts["idepth_max"][fin] = lo, lo + rng.uniform(0.01, 1.0, lo.size).astype(np.float32)
    ref = pts.copy()
    ct.set_new_frame(new)
    ct.immature_upload(pts)
    dN = oracle.make_images(new, w, h)[0][0]
    for t in range(3):
        c = ct.trace(krki, kt, aff)
        cr = oracle.ip_trace(dN, w, h, krki, kt, aff, ref)
        got = ct.immature_download()
        bad = differing(got, ref)
        print(f"  trace {t}: counts {c.tolist()}")
        assert bad.size == 0, (t, bad[:5], got[bad[:2]], ref[bad[:2]])
        np.testing.assert_array_equal(c, cr)
    ct.close()


ACT_SIZES = [(160, 120), (317, 203), (640, 480), (1242, 375)]


@pytest.mark.parametrize("case", range(10))
def test_random_activation_matches_oracle(built, case):
    """optimizeImmaturePoint (ldso_ba_activate_points) on random windows: 2-16 keyframes, the sizes,
    camera models, motions and outliers of tests/test_fuzz_parity.py, interval spreads 1-60 % with
    random offsets (true depth inside or outside), random colour offsets on a fraction of the
    points, non-finite and empty intervals, energy thresholds and min_obs drawn at random, both
    image layouts, and the activated window drawn from a context holding one to three windows:
    every record (idepth, status, residual mask, energy) bit for bit against the oracle."""
    from ldso_amd import BAContext, synth
    from test_activation import differing as act_differing

    rng = np.random.default_rng(17000 + case)
    W, H = ACT_SIZES[rng.integers(len(ACT_SIZES))]
    cfgs = []
    for _ in range(int(rng.integers(1, 4))):
        N = int(rng.integers(2, 17))
        calib = None
        if rng.random() < 0.5:
            f = float(rng.uniform(0.4, 1.2)) * W
            calib = [f, f * float(rng.uniform(0.95, 1.05)), W / 2 + float(rng.uniform(-0.1, 0.1)) * W,
                     H / 2 + float(rng.uniform(-0.1, 0.1)) * H]
        cfgs.append(dict(n_frames=N, n_points=int(rng.integers(1, 1200 if N <= 8 else 400)), width=W, height=H,
                         seed=int(rng.integers(1 << 30)), outlier_frac=float(rng.uniform(0.0, 0.3)),
                         motion=str(rng.choice(["sideways", "forward"])), calib=calib,
                         edge_frac=float(rng.choice([0.0, 0.2])), plane_depth=max(25.0, 2.5 * (N - 1))))
    k = int(rng.integers(len(cfgs)))
    layout = int(rng.choice([1, 3]))
    print(f"case {case}: layout {layout}, activating window {k} of {len(cfgs)}")
    for c in cfgs:
        print("  ", c)
    w = synth.make_window(**cfgs[k])
    pts = synth.immature_from_window(w, spread=float(rng.uniform(0.01, 0.6)), seed=case)
    P = len(pts)
    off = rng.uniform(-0.3, 0.3, P).astype(np.float32) * (rng.random(P) < 0.3)
    pts["idepth_min"] *= 1 + off
    pts["idepth_max"] *= 1 + off
    bad = rng.random(P) < 0.1
    pts["color"][bad] += rng.normal(0, 60, (int(bad.sum()), 1)).astype(np.float32)
    pts["idepth_max"][rng.random(P) < 0.03] = np.nan
    e = rng.random(P) < 0.03
    pts["idepth_min"][e] = pts["idepth_max"][e] = 0.0
    pts["energy_th"] = np.float32(rng.uniform(2, 12)) * np.float32(144)
    ctx = BAContext(0)
    ctx.set_tuning(2, layout)  # LDSO_BA_TUNE_TILED_IMAGES, before load
    ctx.load([synth.make_window(**c) for c in cfgs])
    ow = oracle.OracleWindow(synth.make_window(**cfgs[k]), threads=0)
    for min_obs in sorted({1, int(rng.integers(1, cfgs[k]["n_frames"] + 1))}):
        got = ctx.activate_points(k, pts, min_obs)
        ref = ow.activate_points(pts, min_obs)
        bad = act_differing(got, ref)
        print(f"  min_obs {min_obs}: statuses {np.bincount(ref['status'], minlength=3).tolist()}")
        assert bad.size == 0, (min_obs, bad[:5], got[bad[:3]], ref[bad[:3]])
    ow.close()
    ctx.close()
