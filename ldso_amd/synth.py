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
