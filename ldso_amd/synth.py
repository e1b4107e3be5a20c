"""Seeded synthetic sliding windows for tests and the bench.

A window is ``n_frames`` keyframes of a textured tilted plane rendered with per-frame affine
brightness, so correctly placed points are photo-consistent (mostly inliers) as in a real DSO
window.  Generation runs in ``libldso_synth.so`` (ldso_amd/csrc/synth.cpp); frame-pair terms
(precalc, adjoints, priors) come from the product's host helpers.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .window import Window


class _Params(C.Structure):
    _fields_ = [
        ("n_frames", C.c_int32),
        ("n_points", C.c_int32),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("seed", C.c_uint64),
        ("outlier_frac", C.c_float),
        ("idepth_noise", C.c_float),
        ("newest_perturb", C.c_float),
        ("baseline", C.c_float),
        ("motion", C.c_int32),
        ("fx", C.c_float),
        ("fy", C.c_float),
        ("cx", C.c_float),
        ("cy", C.c_float),
        ("fwd_min", C.c_float),
        ("fwd_max", C.c_float),
        ("plane_depth", C.c_float),
        ("edge_frac", C.c_float),
    ]


def kitti_crop_calib(fx, fy, cx, cy, w_org, h_org, w, h):
    """The output pinhole of LDSO's "crop" undistortion for a distortion-free Pinhole input:
    Undistort::makeOptimalK_crop (src/frontend/Undistort.cc:558-668) with
    UndistortPinhole::distortCoordinates (:1103-1125) restated in float32 (the reference computes in
    float; the crop K is then stored as double and read back as float calibration).  Returns
    float32 [fx, fy, cx, cy] of the w x h output images."""
    f32 = np.float32
    fx, fy, cx, cy = f32(fx), f32(fy), f32(cx), f32(cy)
    w_lim, h_lim = f32(w_org - 1), f32(h_org - 1)

    def distort(x, y):  # K = identity while the crop is searched: ix = x, iy = y
        return fx * x + cx, fy * y + cy

    t = (np.arange(100000, dtype=np.int64).astype(f32) - f32(50000.0)) / f32(10000.0)
    # 1. stretch the centre lines: the first / last sample whose distorted coordinate is inside
    dx, _ = distort(t, np.zeros_like(t))
    inside = np.flatnonzero((dx > 0) & (dx < w_lim))
    min_x, max_x = t[inside[0]], t[inside[-1]]
    _, dy = distort(np.zeros_like(t), t)
    inside = np.flatnonzero((dy > 0) & (dy < h_lim))
    min_y, max_y = t[inside[0]], t[inside[-1]]
    min_x, max_x, min_y, max_y = (v * f32(1.01) for v in (min_x, max_x, min_y, max_y))
    # 2. shrink the side(s) with invalid border pixels by 0.995 until none is left
    ys = np.arange(h).astype(f32)
    xs = np.arange(w).astype(f32)
    for _ in range(501):
        ry = min_y + (max_y - min_y) * ys / (f32(h) - f32(1.0))
        lx, _ = distort(np.full(h, min_x, f32), ry)
        rx, _ = distort(np.full(h, max_x, f32), ry)
        oob_l, oob_r = bool(np.any(~((lx > 0) & (lx < w_lim)))), bool(np.any(~((rx > 0) & (rx < w_lim))))
        rxs = min_x + (max_x - min_x) * xs / (f32(w) - f32(1.0))
        _, ty = distort(rxs, np.full(w, min_y, f32))
        _, by = distort(rxs, np.full(w, max_y, f32))
        oob_t, oob_b = bool(np.any(~((ty > 0) & (ty < h_lim)))), bool(np.any(~((by > 0) & (by < h_lim))))
        if not (oob_l or oob_r or oob_t or oob_b):
            break
        if (oob_l or oob_r) and (oob_t or oob_b):
            if (max_x - min_x) > (max_y - min_y):
                oob_t = oob_b = False
            else:
                oob_l = oob_r = False
        if oob_l:
            min_x = min_x * f32(0.995)
        if oob_r:
            max_x = max_x * f32(0.995)
        if oob_t:
            min_y = min_y * f32(0.995)
        if oob_b:
            max_y = max_y * f32(0.995)
    else:
        raise ValueError("no valid crop")
    kfx = (f32(w) - f32(1.0)) / (max_x - min_x)
    kfy = (f32(h) - f32(1.0)) / (max_y - min_y)
    return np.array([kfx, kfy, -np.float64(min_x) * np.float64(kfx), -np.float64(min_y) * np.float64(kfy)], np.float32)


# configs of BASELINE.json used by tests and bench
S7 = dict(n_frames=7, n_points=2000, width=640, height=480)
S11 = dict(n_frames=11, n_points=8000, width=640, height=480)
# BASELINE config 3 (KITTI 00, preset 0: 7 keyframes, 2000 points): the output geometry of
# examples/Kitti/Kitti00-02.txt (1241 x 376 Pinhole 718.856 718.856 607.1928 185.2157, "crop" to
# 1232 x 368) and a car's forward travel of 0.5-1 m per keyframe down a street canyon (road, two walls,
# a facade 25 m ahead: depths from ~3 to 25 m, large
# scale changes, many pattern pixels leaving the image).  The KITTI driver fixes both affine modes to 0
# (run_dso_kitti.cc:299-300).
KITTI00_CALIB = kitti_crop_calib(718.856, 718.856, 607.1928, 185.2157, 1241, 376, 1232, 368)
KITTI00 = dict(n_frames=7, n_points=2000, width=1232, height=368, calib=KITTI00_CALIB, motion="forward")
# KITTI 03's raw frame (examples/Kitti/Kitti03.txt: 1242 x 375, Pinhole 721.5377 721.5377 609.5593
# 172.854) without the crop: a width that is not a multiple of 8 and a height not a multiple of 4.
KITTI03_RAW = dict(n_frames=7, n_points=2000, width=1242, height=375,
                   calib=np.array([721.5377, 721.5377, 609.5593, 172.854], np.float32), motion="forward")


def make_window(n_frames=7, n_points=2000, width=640, height=480, seed=0, outlier_frac=0.05, idepth_noise=0.01,
                newest_perturb=1e-3, baseline=0.04, finalize=True, calib=None, motion="sideways",
                fwd_step=(0.5, 1.0), plane_depth=25.0, edge_frac=0.0) -> Window:
    """calib: pinhole [fx, fy, cx, cy] of the output images (None: EuRoC-style 0.6w, 0.9h);
    motion: "sideways" (x travel of `baseline` per keyframe, the round-1 window) or "forward"
    (+z travel of U(fwd_step) m per keyframe down a street canyon whose far facade is `plane_depth` m ahead);
    edge_frac: the fraction of points drawn 4..9 px from the image border instead of in [8, w - 9]."""
    N, P = int(n_frames), int(n_points)
    k = np.zeros(4, np.float32) if calib is None else np.asarray(calib, np.float32)
    mot = {"sideways": 0, "forward": 1}[motion]
    R = P * (N - 1)
    frames = np.zeros(N, L.FRAME_STATE_DTYPE)
    dI = np.zeros((N, width * height, 3), np.float32)
    calib = np.zeros(4, np.float32)
    fth = np.zeros(N, np.float32)
    point_host = np.zeros(P, np.int32)
    point_data = np.zeros((P, L.POINT_STRIDE), np.float32)
    begin = np.zeros(P + 1, np.int32)
    res_target = np.zeros(R, np.int32)
    res_state = np.zeros(R, np.int8)
    res_energy = np.zeros(R, np.float32)
    res_flags = np.zeros(R, np.uint8)
    prm = _Params(N, P, width, height, int(seed), outlier_frac, idepth_noise, newest_perturb, baseline, mot,
                  float(k[0]), float(k[1]), float(k[2]), float(k[3]), float(fwd_step[0]), float(fwd_step[1]),
                  float(plane_depth), float(edge_frac))
    rc = L.synth_lib().ldso_synth_fill(
        C.byref(prm), frames.ctypes.data, L.ptr(dI, L.f32p), L.ptr(calib, L.f32p), L.ptr(fth, L.f32p),
        L.ptr(point_host, L.i32p), L.ptr(point_data, L.f32p), L.ptr(begin, L.i32p), L.ptr(res_target, L.i32p),
        L.ptr(res_state, L.i8p), L.ptr(res_energy, L.f32p), L.ptr(res_flags, L.u8p))
    if rc != 0:
        raise ValueError("ldso_synth_fill rejected the parameters")
    w = Window(n_frames=N, width=width, height=height, calib=calib, frames=frames, dI=dI, frame_energy_th=fth,
               point_host=point_host, point_data=point_data, point_res_begin=begin, res_target=res_target,
               res_state=res_state, res_energy=res_energy, res_flags=res_flags)
    if finalize:
        w.refresh_frame_terms()
    return w


def in_image_order(w: Window) -> Window:
    """The same window with each host frame's points in image row order (v, then u): the order in
    which LDSO's pixel selection emits them.  make_window's points are in random order."""
    return permute_points(w, np.lexsort((w.point_data[:, 0], np.floor(w.point_data[:, 1]), w.point_host)))


def permute_points(w: Window, order) -> Window:
    """The same window with its points (and their residual runs) in the order `order` (new index ->
    index in w); o.point_order / o.res_order map the new points / residuals back to w's."""
    import copy
    order = np.asarray(order)
    ridx = np.concatenate([np.arange(w.point_res_begin[p], w.point_res_begin[p + 1]) for p in order])
    o = copy.copy(w)
    o.point_host = np.ascontiguousarray(w.point_host[order])
    o.point_data = np.ascontiguousarray(w.point_data[order])
    # a point's features rank travels with it (ldso_ba_window::point_rank orders by it)
    o.point_rank = None if w.point_rank is None else np.ascontiguousarray(np.asarray(w.point_rank)[order])
    o.point_res_begin = np.concatenate([[0], np.cumsum(np.diff(w.point_res_begin)[order])]).astype(np.int32)
    for k in ("res_target", "res_state", "res_energy", "res_flags"):
        setattr(o, k, np.ascontiguousarray(getattr(w, k)[ridx]))
    o._keep = []
    o.point_order, o.res_order = order, ridx  # new index -> index in w
    return o


def make_tracker_scene(width=640, height=480, n_points=(8000, 4000, 2000, 1000, 500, 250), seed=0, blobs=64):
    """A coarse-tracking scene: a smooth textured reference image (sum of
    Gaussian blobs, [0, 255] float, the same family as §8d's frames) and per-level reference point
    clouds at integer pixel positions of that level, as CoarseTracker::makeCoarseDepthL0 emits
    them (CoarseTracker.cc:357-538), with the level's pyramid intensity as pc_color.  The caller
    supplies the level intensities (``level_images``, e.g. FrameHessian::makeImages' output) so
    pc_color is exact; idepth ~ U(0.3, 1.5).  Returns (color [h][w], make_pc(level_images))."""
    rng = np.random.default_rng(0x1D50 + int(seed))
    yy, xx = np.mgrid[0:height, 0:width].astype(np.float64)
    img = np.full((height, width), 90.0)
    for _ in range(int(blobs)):
        cx, cy = rng.uniform(0, width), rng.uniform(0, height)
        s = rng.uniform(4, 40) * width / 640
        a = rng.uniform(20, 120) * rng.choice([-1, 1])
        img += a * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * s * s))
    color = np.clip(img, 0, 255).astype(np.float32)

    def make_pc(level_images):
        pcs = []
        for l, I in enumerate(level_images):
            wl, hl = width >> l, height >> l
            n = min(int(n_points[min(l, len(n_points) - 1)]), (wl - 4) * (hl - 4))
            idx = rng.choice((wl - 4) * (hl - 4), size=n, replace=False)
            u = (idx % (wl - 4) + 2).astype(np.float32)
            v = (idx // (wl - 4) + 2).astype(np.float32)
            col = np.asarray(I, np.float32).reshape(-1)[(v.astype(np.int64) * wl + u.astype(np.int64))]
            idepth = rng.uniform(0.3, 1.5, n).astype(np.float32)
            pcs.append(dict(u=u, v=v, idepth=idepth, color=col))
        return pcs

    return color, make_pc


def se3_matrix(omega, upsilon):
    """Sophus::SE3::exp((upsilon, omega)).matrix3x4() (se3.hpp: translation first), in double."""
    w = np.asarray(omega, np.float64)
    th = np.linalg.norm(w)
    W = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-10:
        R = np.eye(3) + W
        V = np.eye(3) + 0.5 * W
    else:
        R = np.eye(3) + np.sin(th) / th * W + (1 - np.cos(th)) / th ** 2 * W @ W
        V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * W + (th - np.sin(th)) / th ** 3 * W @ W
    T = np.zeros((3, 4))
    T[:, :3] = R
    T[:, 3] = V @ np.asarray(upsilon, np.float64)
    return T


def make_trace_scene(width=640, height=480, n_hosts=7, points_per_host=1500, shift=8.0, seed=0):
    """traceNewCoarse workload: a blob-textured fronto-parallel plane at
    inverse depth 0.5 seen by n_hosts host keyframes translated along x, and the new frame.
    Host i sees the plane shifted by shift * (1 + i / n_hosts) pixels in the new frame.
    Returns (host_image, new_image, uv [n_hosts][points_per_host][2], krki [n][9], kt [n][3],
    aff [n][2]).  points_per_host defaults to setting_desiredImmatureDensity (Setting.cc)."""
    rng = np.random.default_rng(0x7ACE + int(seed))
    yy, xx = np.mgrid[0:height, 0:width].astype(np.float64)
    blobs = [(rng.uniform(0, width), rng.uniform(0, height), rng.uniform(2.0, 8.0),
              rng.uniform(20, 80) * rng.choice([-1, 1])) for _ in range(int(width * height / 2000))]

    def render(dx, a=1.0, b=0.0):
        img = np.full((height, width), 90.0)
        for cx, cy, s, A in blobs:
            img += A * np.exp(-((xx - dx - cx) ** 2 + (yy - cy) ** 2) / (2 * s * s))
        return (a * img + b).astype(np.float32)

    host, new = render(0.0), render(shift, 1.1, -5.0)
    fx, rho = 0.6 * width, 0.5
    krki = np.tile(np.eye(3, dtype=np.float32).reshape(1, 9), (n_hosts, 1))
    kt = np.zeros((n_hosts, 3), np.float32)
    kt[:, 0] = [shift * (1 + i / n_hosts) / rho for i in range(n_hosts)]
    aff = np.tile(np.array([1.1, -5.0], np.float32), (n_hosts, 1))
    uv = np.stack([rng.uniform(10, width - 50, (n_hosts, points_per_host)),
                   rng.uniform(10, height - 10, (n_hosts, points_per_host))], -1).astype(np.float32)
    del fx
    return host, new, uv, krki, kt, aff


def immature_from_window(w, spread=0.1, seed=0):
    """Point-activation workload: the window's points as ImmaturePoint
    records (include/ldso_ct.h) with the window's host, pixel, colour and weights and an
    inverse-depth interval of +-spread (jittered 3 %) around the stored inverse depth."""
    rng = np.random.default_rng(seed)
    P = w.point_data.shape[0]
    pts = np.zeros(P, L.IMMATURE_DTYPE)
    pd = w.point_data
    pts["u"], pts["v"] = pd[:, 0], pd[:, 1]
    idp = pd[:, 2]
    jitter = rng.uniform(-0.03, 0.03, P).astype(np.float32)
    pts["idepth_min"] = idp * np.float32(1 - spread) * (1 + jitter)
    pts["idepth_max"] = idp * np.float32(1 + spread) * (1 + jitter)
    pts["energy_th"] = np.float32(8 * 144)
    pts["color"] = pd[:, 8:16]
    pts["weights"] = pd[:, 16:24]
    pts["host"] = w.point_host
    pts["quality"] = 10000
    return pts
