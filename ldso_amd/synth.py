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
    ]


# configs of BASELINE.json used by tests and bench
S7 = dict(n_frames=7, n_points=2000, width=640, height=480)
S11 = dict(n_frames=11, n_points=8000, width=640, height=480)


def make_window(n_frames=7, n_points=2000, width=640, height=480, seed=0, outlier_frac=0.05, idepth_noise=0.01,
                newest_perturb=1e-3, baseline=0.04, finalize=True) -> Window:
    N, P = int(n_frames), int(n_points)
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
    prm = _Params(N, P, width, height, int(seed), outlier_frac, idepth_noise, newest_perturb, baseline)
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
