"""Host-side sliding window: the SoA mirror of LDSO's EnergyFunctional state that the C ABI
consumes (``ldso_ba_window``).

Field meanings follow the reference classes:
  FrameHessian (include/internal/FrameHessian.h), PointHessian (include/internal/PointHessian.h),
  PointFrameResidual (include/internal/Residuals.h), FrameFramePrecalc
  (include/internal/FrameFramePrecalc.h), EnergyFunctional::adHost/adTarget/cPrior/cDeltaF
  (include/internal/OptimizationBackend/EnergyFunctional.h:222-235).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L


@dataclass
class Window:
    n_frames: int
    width: int
    height: int
    calib: np.ndarray                 # f32[4]  fxl, fyl, cxl, cyl
    frames: np.ndarray                # FRAME_STATE_DTYPE[N]
    dI: np.ndarray                    # f32[N, h*w, 3]
    frame_energy_th: np.ndarray       # f32[N]
    point_host: np.ndarray            # i32[P]
    point_data: np.ndarray            # f32[P, 24]
    point_res_begin: np.ndarray       # i32[P+1]
    res_target: np.ndarray            # i32[R]
    res_state: np.ndarray             # i8[R]
    res_energy: np.ndarray            # f32[R]
    res_flags: np.ndarray             # u8[R]
    precalc: np.ndarray = None        # f32[N*N, LDSO_BA_PRECALC_STRIDE]
    ad_host: np.ndarray = None        # f64[N*N, 64]
    ad_target: np.ndarray = None      # f64[N*N, 64]
    c_prior: np.ndarray = None        # f64[4]
    c_delta: np.ndarray = None        # f32[4]
    frame_prior: np.ndarray = None    # f64[N, 8]
    frame_delta: np.ndarray = None    # f64[N, 8]
    frame_delta_prior: np.ndarray = None  # f64[N, 8]
    # the reference settings takeData's priors follow (setting_affineOptModeA / B): an L.OptSettings,
    # None = the defaults.  The context that runs the window must hold the same (BAContext.set_settings).
    settings: object = None
    # i32[P] or None: each point's rank in its host frame's features order (ldso_ba_window::point_rank)
    point_rank: np.ndarray = None
    _keep: list = field(default_factory=list, repr=False)

    @property
    def n_points(self) -> int:
        return int(self.point_host.shape[0])

    @property
    def n_residuals(self) -> int:
        return int(self.res_target.shape[0])

    @property
    def dim(self) -> int:
        return 8 * self.n_frames + 4

    def refresh_frame_terms(self):
        """setPrecalcValues + setAdjointsF + FrameHessian::takeData through the product's host
        helpers (FullSystem.cc:1667-1675, EnergyFunctional.cc:551-609, FrameHessian.cc:131-135)."""
        lib = L.lib()
        N = self.n_frames
        fr = np.ascontiguousarray(self.frames)
        self.precalc = np.zeros((N * N, L.PRECALC_STRIDE), np.float32)
        L.check(lib.ldso_ba_frame_precalc(N, fr.ctypes.data, L.ptr(self.calib, L.f32p), L.ptr(self.precalc, L.f32p)))
        self.ad_host = np.zeros((N * N, 64), np.float64)
        self.ad_target = np.zeros((N * N, 64), np.float64)
        self.c_prior = np.zeros(4, np.float64)
        L.check(lib.ldso_ba_set_adjoints(N, fr.ctypes.data, L.ptr(self.ad_host, L.f64p), L.ptr(self.ad_target, L.f64p),
                                         L.ptr(self.c_prior, L.f64p)))
        self.frame_prior = np.zeros((N, 8), np.float64)
        self.frame_delta = np.zeros((N, 8), np.float64)
        self.frame_delta_prior = np.zeros((N, 8), np.float64)
        sp = C.byref(self.settings) if self.settings is not None else None
        L.check(lib.ldso_ba_frame_take_data(N, fr.ctypes.data, sp, L.ptr(self.frame_prior, L.f64p),
                                            L.ptr(self.frame_delta, L.f64p), L.ptr(self.frame_delta_prior, L.f64p)))
        if self.c_delta is None:
            self.c_delta = np.zeros(4, np.float32)  # CalibHessian::value_minus_value_zero
        return self

    def nullspaces(self) -> np.ndarray:
        out = np.zeros((7, self.dim), np.float64)
        fr = np.ascontiguousarray(self.frames)
        L.check(L.lib().ldso_ba_nullspaces(self.n_frames, fr.ctypes.data, L.ptr(out, L.f64p)))
        return out

    def c_struct(self, with_images: bool = True) -> L.LdsoBaWindow:
        """with_images=False leaves dI NULL (a marginalisation window borrows its parent's)."""
        if self.precalc is None:
            self.refresh_frame_terms()
        arrs = dict(
            dI=np.ascontiguousarray(self.dI, np.float32) if with_images else None,
            frame_energy_th=np.ascontiguousarray(self.frame_energy_th, np.float32),
            precalc=np.ascontiguousarray(self.precalc, np.float32),
            ad_host=np.ascontiguousarray(self.ad_host, np.float64),
            ad_target=np.ascontiguousarray(self.ad_target, np.float64),
            c_prior=np.ascontiguousarray(self.c_prior, np.float64),
            c_delta=np.ascontiguousarray(self.c_delta, np.float32),
            frame_prior=np.ascontiguousarray(self.frame_prior, np.float64),
            frame_delta_prior=np.ascontiguousarray(self.frame_delta_prior, np.float64),
            point_host=np.ascontiguousarray(self.point_host, np.int32),
            point_data=np.ascontiguousarray(self.point_data, np.float32),
            point_res_begin=np.ascontiguousarray(self.point_res_begin, np.int32),
            res_target=np.ascontiguousarray(self.res_target, np.int32),
            res_state=np.ascontiguousarray(self.res_state, np.int8),
            res_energy=np.ascontiguousarray(self.res_energy, np.float32),
            res_flags=np.ascontiguousarray(self.res_flags, np.uint8),
            point_rank=None if self.point_rank is None else np.ascontiguousarray(self.point_rank, np.int32),
        )
        self._keep = [a for a in arrs.values() if a is not None]
        s = L.LdsoBaWindow()
        s.n_frames = self.n_frames
        s.n_points = self.n_points
        s.n_residuals = self.n_residuals
        s.width = self.width
        s.height = self.height
        s.calib[:] = [float(x) for x in self.calib]
        types = {np.float32: L.f32p, np.float64: L.f64p, np.int32: L.i32p, np.int8: L.i8p, np.uint8: L.u8p}
        for k, a in arrs.items():
            if a is not None:
                setattr(s, k, L.ptr(a, types[a.dtype.type]))
        return s

    def copy_state(self) -> "Window":
        """Deep copy of the mutable per-residual / per-point state."""
        import copy
        w = copy.copy(self)
        for k in ("point_data", "res_state", "res_energy", "res_flags", "frame_energy_th", "frames"):
            setattr(w, k, getattr(self, k).copy())
        w._keep = []
        return w
