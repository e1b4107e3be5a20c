"""Immature points: ImmaturePoint::ImmaturePoint and ImmaturePoint::traceOn
over FullSystem::traceNewCoarse (src/internal/ImmaturePoint.cc:14-39, 47-317;
src/frontend/FullSystem.cc:1157-1194).

CPU tests pin the oracle restatement (oracle/ldso_oracle_tracker.cpp) with checks that do not
share its code: a numpy float32 restatement of the constructor (bit-exact), a scene with a known
depth (a textured fronto-parallel plane seen from a translated camera: traced intervals must
bracket the true inverse depth, also after a second trace), and hand-built records that drive
each early exit of traceOn (OOB, SKIPPED, BADCONDITION, OUTLIER -> OOB).  The reference ships
no fixtures for this path and cannot be built here: parity with the reference
itself is unpinned beyond these known answers.

GPU tests compare include/ldso_ct.h's ldso_ct_make_immature / ldso_ct_trace with the oracle
record for record, byte for byte (statuses, intervals, lastTraceUV, quality), over several hosts
with rotated poses and two successive traces."""
import numpy as np
import pytest

import oracle
from ldso_amd import _lib as L

W, H = 640, 480
FX = 384.0
RHO = 0.5     # inverse depth of the plane
SHIFT = 8.0   # its disparity in the new frame (pixels)
AFF = (1.1, -5.0)


def blob_image(w, h, shift=0.0, seed=0, a=1.0, b=0.0, sigma=(2.0, 8.0)):
    """Sum of Gaussian blobs evaluated at (x - shift, y): the host image, or the new image of a
    fronto-parallel plane after a camera translation along x, with affine brightness a, b."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    xx = xx - shift
    img = np.full((h, w), 90.0)
    for _ in range(int(w * h / 2000)):
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        s = rng.uniform(*sigma)
        A = rng.uniform(20, 80) * rng.choice([-1, 1])
        img += A * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * s * s))
    return (a * img + b).astype(np.float32)


def level0(img):
    return oracle.make_images(img, img.shape[1], img.shape[0])[0][0]


def scene_tables():
    """Host 0: the known-depth translation; hosts 1-2: rotated poses (exercise Rplane, clamps)."""
    tx = SHIFT / (FX * RHO)
    krki = [np.eye(3, dtype=np.float32)]
    kt = [np.array([FX * tx, 0, 0], np.float32)]
    aff = [np.array(AFF, np.float32)]
    for i, (ang, t) in enumerate([(0.02, (3.0, -1.0, 0.01)), (-0.05, (-6.0, 4.0, -0.02))]):
        c, s = np.cos(ang), np.sin(ang)
        K = np.array([[FX, 0, 319.5], [0, 432.0, 239.5], [0, 0, 1]])
        R = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
        krki.append((K @ R @ np.linalg.inv(K)).astype(np.float32))
        kt.append(np.array(t, np.float32))
        aff.append(np.array((1.0 + 0.1 * i, 2.0 * i), np.float32))
    return np.stack(krki), np.stack(kt), np.stack(aff)


def features(n, seed=1, margin=10):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(margin, W - 4 * margin, n), rng.uniform(margin, H - margin, n)], 1).astype(np.float32)


def np_make(dI, w, h, uv):
    """ImmaturePoint's constructor in numpy float32 (no shared code with the oracle)."""
    f = np.float32
    pat = [(0, -2), (-1, -1), (1, -1), (-2, 0), (0, 0), (2, 0), (-1, 1), (0, 2)]
    I = dI[:, 0]
    n = uv.shape[0]
    color = np.zeros((n, 8), f)
    wts = np.zeros((n, 8), f)
    G = np.zeros((n, 4), f)
    c = f(50 * 50)
    for k, (px, py) in enumerate(pat):
        x = (uv[:, 0] + f(px)).astype(f)
        y = (uv[:, 1] + f(py)).astype(f)
        ix, iy = x.astype(np.int32), y.astype(np.int32)
        dx, dy = (x - ix.astype(f)).astype(f), (y - iy.astype(f)).astype(f)
        b = ix + iy * w
        tl, tr, bl, br = I[b], I[b + 1], I[b + w], I[b + w + 1]
        one = f(1)
        top = dx * tr + (one - dx) * tl
        bot = dx * br + (one - dx) * bl
        left = dy * bl + (one - dy) * tl
        right = dy * br + (one - dy) * tr
        color[:, k] = dx * right + (one - dx) * left
        g0, g1 = right - left, bot - top
        G[:, 0] += g0 * g0
        G[:, 1] += g0 * g1
        G[:, 2] += g1 * g0
        G[:, 3] += g1 * g1
        wts[:, k] = np.sqrt(c / (c + (g0 * g0 + g1 * g1)))
    return color, wts, G


def bits(a):
    """records as raw 32-bit words"""
    return np.ascontiguousarray(a).view(np.uint32).reshape(-1, 32)


def differing(got, ref):
    """indices of records that differ in any word; NaN equals NaN whatever its sign / payload
    (x86's default NaN has the sign bit set, the GPU's does not: 0/0 of a textureless patch)"""
    a = np.ascontiguousarray(got).view(np.float32).reshape(-1, 32)
    b = np.ascontiguousarray(ref).view(np.float32).reshape(-1, 32)
    same = (bits(got) == bits(ref)) | (np.isnan(a) & np.isnan(b))
    return np.flatnonzero(~same.all(axis=1))


# ------------------------------------------------------------------------------------------
# CPU: the oracle against independent known answers
# ------------------------------------------------------------------------------------------
def test_record_layout_matches_oracle(built):
    assert L.IMMATURE_DTYPE == oracle.IMMATURE_DTYPE
    assert L.IMMATURE_DTYPE.itemsize == 128


def test_oracle_make_known_answer(built):
    img = blob_image(W, H, seed=4)
    dI = level0(img)
    uv = features(3000, seed=2)
    pts = oracle.ip_make(dI, W, H, uv, 2.0, 3)
    color, wts, G = np_make(dI, W, H, uv)
    np.testing.assert_array_equal(pts["color"], color)
    np.testing.assert_array_equal(pts["weights"], wts)
    np.testing.assert_array_equal(pts["grad_h"], G)
    assert np.all(pts["energy_th"] == np.float32(8 * 144))
    assert np.all(np.isnan(pts["idepth_max"])) and np.all(pts["idepth_min"] == 0)
    assert np.all(pts["last_status"] == 5) and np.all(pts["quality"] == 10000)
    assert np.all(pts["host"] == 3) and np.all(pts["type"] == 2.0)


def test_oracle_make_nonfinite_colour(built):
    img = blob_image(W, H, seed=4)
    img[100, 101] = np.nan
    pts = oracle.ip_make(level0(img), W, H, np.array([[100.0, 100.0], [300.0, 300.0]], np.float32))
    assert np.isnan(pts["energy_th"][0]) and pts["energy_th"][1] == np.float32(1152)


def test_oracle_trace_brackets_true_depth(built):
    host, new = blob_image(W, H, seed=0), blob_image(W, H, shift=SHIFT, seed=0, a=AFF[0], b=AFF[1])
    krki, kt, aff = scene_tables()
    pts = oracle.ip_make(level0(host), W, H, features(2000))
    dN = level0(new)
    c1 = oracle.ip_trace(dN, W, H, krki[:1], kt[:1], aff[:1], pts)
    assert c1.sum() == 2000 and c1[0] > 1200  # mostly GOOD from the uninitialised state
    g = pts["last_status"] == 0
    inside = (pts["idepth_min"][g] <= RHO) & (pts["idepth_max"][g] >= RHO)
    assert inside.mean() > 0.9
    # the traced position is the true match to within the stated interval
    err = np.abs(pts["last_uv"][g, 0] - (features(2000)[g, 0] + SHIFT))
    assert np.median(err) < 0.25
    c2 = oracle.ip_trace(dN, W, H, krki[:1], kt[:1], aff[:1], pts)
    assert c2[3] + c2[4] > 0  # finite intervals now: SKIPPED / BADCONDITION appear
    g2 = g & (pts["last_status"] == 0)  # re-traced inside the first pass's interval
    if g2.sum() > 20:
        assert ((pts["idepth_min"][g2] <= RHO) & (pts["idepth_max"][g2] >= RHO)).mean() > 0.9


def test_oracle_trace_early_exits(built):
    host = blob_image(W, H, seed=0)
    dI = level0(host)
    krki, kt, aff = scene_tables()
    pts = oracle.ip_make(dI, W, H, np.array([[2.0, 200.0], [300.0, 200.0], [300.0, 200.0], [300.0, 200.0],
                                              [300.0, 200.0]], np.float32))
    pts["last_status"][4] = 1  # already OOB: untouched
    pts["idepth_min"][1], pts["idepth_max"][1] = 0.5, 0.5005  # < 1.5 px apart: SKIPPED
    pts["idepth_min"][2], pts["idepth_max"][2] = 0.3, 0.7  # gradient perpendicular to the line
    pts["grad_h"][2] = (1e-6, 0, 0, 1e4)
    pts["last_status"][3] = 2  # an outlier again -> OOB (colours far from the new frame)
    pts["color"][3] = 1e4
    before = pts.copy()
    oracle.ip_trace(dI, W, H, krki[:1], kt[:1], aff[:1], pts)
    assert list(pts["last_status"]) == [1, 3, 4, 1, 1]
    assert np.all(pts["last_uv"][0] == -1) and pts["last_interval"][0] == 0
    assert bits(pts[4:5]).tolist() == bits(before[4:5]).tolist()


# ------------------------------------------------------------------------------------------
# GPU: include/ldso_ct.h against the oracle
# ------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def gpu_tracker(built):
    from ldso_amd.tracker import CoarseTracker
    t = CoarseTracker(W, H)
    yield t
    t.close()


@pytest.mark.gpu
def test_gpu_make_immature_parity(gpu_tracker):
    img = blob_image(W, H, seed=4)
    img[100, 101] = np.nan
    uv = np.concatenate([features(5000, seed=3), np.array([[100.0, 100.0], [3.0, 3.0]], np.float32)])
    gpu_tracker.set_new_frame(img)
    got = gpu_tracker.make_immature(uv, 2.0, 5)
    ref = oracle.ip_make(level0(img), W, H, uv, 2.0, 5)
    assert differing(got, ref).size == 0


@pytest.mark.gpu
def test_gpu_trace_parity(gpu_tracker):
    host, new = blob_image(W, H, seed=0), blob_image(W, H, shift=SHIFT, seed=0, a=AFF[0], b=AFF[1])
    krki, kt, aff = scene_tables()
    gpu_tracker.set_new_frame(host)
    recs = [gpu_tracker.make_immature(features(3000, seed=10 + i, margin=6), 1.0, i) for i in range(3)]
    pts = np.concatenate(recs)
    pts["last_status"][::97] = 1  # some already OOB
    pts["last_status"][5::89] = 2  # some outliers from a previous frame
    pts["idepth_min"][7::13], pts["idepth_max"][7::13] = 0.3, 0.8  # finite intervals
    ref = pts.copy()
    gpu_tracker.set_new_frame(new)
    gpu_tracker.immature_upload(pts)
    dN = level0(new)
    for _ in range(2):  # two successive traceNewCoarse calls on the resident records
        c = gpu_tracker.trace(krki, kt, aff)
        cr = oracle.ip_trace(dN, W, H, krki, kt, aff, ref)
        got = gpu_tracker.immature_download()
        bad = differing(got, ref)
        assert bad.size == 0, (bad[:5], got[bad[:2]], ref[bad[:2]])
        np.testing.assert_array_equal(c, cr)
    assert (cr[[0, 1, 2]] > 0).all()


@pytest.mark.gpu
def test_gpu_trace_edge_cases(gpu_tracker):
    img = blob_image(W, H, seed=0)
    gpu_tracker.set_new_frame(img)
    krki, kt, aff = scene_tables()
    gpu_tracker.immature_upload(np.zeros(0, L.IMMATURE_DTYPE))
    assert gpu_tracker.trace(krki, kt, aff).tolist() == [0] * 6
    pts = gpu_tracker.make_immature(features(10), 1.0, 2)
    gpu_tracker.immature_upload(pts)
    with pytest.raises(RuntimeError):
        gpu_tracker.trace(krki[:2], kt[:2], aff[:2])  # host index 2 >= n_hosts
    bad = pts.copy()
    bad["last_status"][0] = 9
    with pytest.raises(RuntimeError):
        gpu_tracker.immature_upload(bad)
