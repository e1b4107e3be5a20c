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
