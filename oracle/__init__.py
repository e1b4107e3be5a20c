"""CPU restatement of LDSO's photometric-BA hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker / CPU baseline.  The product path (ldso_amd) never touches it.

Parity status: "parity unpinned" by the reference (n-lalanne/LDSO ships no golden vectors for
this path and cannot be built here: Eigen3/glog/OpenCV/g2o/DBoW3 are absent).  The restatement
is pinned by independent known-answer tests (tests/test_oracle_kat.py).  See ldso_oracle.cpp
for the reference file:line of every function.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libldso_oracle.so")

i32p = C.POINTER(C.c_int32)
f32p = C.POINTER(C.c_float)
f64p = C.POINTER(C.c_double)
i8p = C.POINTER(C.c_int8)
u8p = C.POINTER(C.c_uint8)

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        Lb = C.CDLL(LIB_PATH)
        sig = {
            "oracle_set_threads": (None, [C.c_int]),
            "oracle_set_affine_opt_modes": (None, [C.c_float, C.c_float]),
            "oracle_get_affine_opt_modes": (None, [f32p, f32p]),
            "oracle_get_threads": (C.c_int, []),
            "oracle_create": (C.c_void_p, [C.c_void_p]),
            "oracle_destroy": (None, [C.c_void_p]),
            "oracle_update": (C.c_int, [C.c_void_p, C.c_void_p]),
            "oracle_reset_oob": (None, [C.c_void_p]),
            "oracle_linearize_all": (C.c_int, [C.c_void_p, C.c_int, f64p]),
            "oracle_apply_res": (None, [C.c_void_p]),
            "oracle_accumulate": (C.c_int, [C.c_void_p, f64p, f64p, f64p, f64p, f64p, f64p]),
            "oracle_iteration": (C.c_int, [C.c_void_p, f64p]),
            "oracle_get_residuals": (None, [C.c_void_p, i8p, i8p, f32p, f32p, f32p, u8p, f32p, f32p]),
            "oracle_get_jacobians": (None, [C.c_void_p, f32p]),
            "oracle_get_points": (None, [C.c_void_p, f32p, f32p, f32p, f32p, f32p, f32p]),
            "oracle_get_frame_energy_th": (None, [C.c_void_p, f32p]),
            "oracle_solve_system": (C.c_int, [C.c_int, C.c_int, C.c_double] + [f64p] * 9 + [C.c_int, f64p]),
            "oracle_resubstitute": (None, [C.c_void_p, f64p, C.c_double, f32p]),
            "oracle_frame_precalc": (C.c_int, [C.c_int, C.c_void_p, f32p, f32p]),
            "oracle_set_adjoints": (C.c_int, [C.c_int, C.c_void_p, f64p, f64p, f64p]),
            "oracle_frame_take_data": (C.c_int, [C.c_int, C.c_void_p, f64p, f64p, f64p]),
            "oracle_nullspaces": (C.c_int, [C.c_int, C.c_void_p, f64p]),
            "oracle_do_step_from_backup": (C.c_int, [C.c_int, C.c_void_p, f64p, f64p, f64p, C.c_int, i32p, f32p, f32p,
                                                     C.c_float, C.c_void_p, f32p, f32p, f32p]),
            "oracle_time_iterations": (C.c_double, [C.c_void_p, C.c_int]),
            "oracle_ad_ht_delta": (C.c_int, [C.c_int, f64p, f64p, f64p, f32p]),
            "oracle_calc_m_energy": (C.c_double, [C.c_int, f64p, f64p, f32p, f64p]),
            "oracle_calc_l_energy": (C.c_double, [C.c_int, f64p, f64p, f64p, f32p, C.c_int, f32p, f32p]),
            "oracle_marginalize_points": (C.c_int, [C.c_void_p, C.c_int, i32p, f32p, f64p, f64p]),
            "oracle_ct_levels": (C.c_int, [C.c_int, C.c_int]),
            "oracle_ct_make_k": (None, [f32p, C.c_int, C.c_int, C.c_int, f32p]),
            "oracle_make_images": (None, [f32p, C.c_int, C.c_int, C.c_int, f32p, f32p, f32p]),
            "oracle_ct_calc_res": (C.c_int, [C.c_int, C.c_int, C.c_int, f32p, f32p, C.c_int, f32p, f32p, f32p, f32p,
                                             f64p, f64p, C.c_float, f64p, f32p, i32p]),
            "oracle_ct_calc_gs": (C.c_int, [C.c_int, f32p, C.c_float, C.c_float, f64p, f64p, f64p]),
            "oracle_activate_points": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]),
            "oracle_ip_make": (None, [f32p, C.c_int, C.c_int, C.c_int, f32p, C.c_float, C.c_int, C.c_void_p]),
            "oracle_ip_trace": (None, [f32p, C.c_int, C.c_int, f32p, f32p, f32p, C.c_int, C.c_void_p, i32p]),
        }
        for k, (res, args) in sig.items():
            f = getattr(Lb, k)
            f.restype = res
            f.argtypes = args
        _lib = Lb
    return _lib


def _p(a, t):
    if a is None:
        return C.cast(None, t)
    # the C side reads and writes through this pointer at its own element size: a mismatched or
    # strided array would be overrun (a float32 calib_value handed as double* once corrupted the heap)
    assert a.flags["C_CONTIGUOUS"] and a.dtype == np.dtype(t._type_), (a.dtype, t)
    return a.ctypes.data_as(t)


def set_threads(n: int):
    lib().oracle_set_threads(int(n))


class OracleWindow:
    """EnergyFunctional + FullSystem::linearizeAll restated on the CPU for one window."""

    def __init__(self, window, threads=None):
        if threads is not None:
            set_threads(threads)
        self.window = window
        s = window.c_struct()
        self._h = lib().oracle_create(C.byref(s))
        if not self._h:
            raise ValueError("oracle_create rejected the window")
        window._keep = []

    def close(self):
        if self._h:
            lib().oracle_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def update(self, window):
        s = window.c_struct()
        rc = lib().oracle_update(self._h, C.byref(s))
        window._keep = []
        assert rc == 0

    def reset_oob(self):
        lib().oracle_reset_oob(self._h)

    def linearize_all(self, fix=False):
        out = np.zeros(3, np.float64)
        lib().oracle_linearize_all(self._h, int(bool(fix)), _p(out, f64p))
        return out

    def apply_res(self):
        lib().oracle_apply_res(self._h)

    def accumulate(self) -> dict:
        n = self.window.dim
        out = {k: np.zeros((n, n) if k.startswith("H") else n, np.float64) for k in ("HA", "bA", "HL", "bL", "Hsc", "bsc")}
        lib().oracle_accumulate(self._h, *[_p(out[k], f64p) for k in ("HA", "bA", "HL", "bL", "Hsc", "bsc")])
        return out

    def iteration(self):
        """linearizeAll(false) + applyRes + accumulate: the same pass as ldso_ba_linearize(0, 1)."""
        e = self.linearize_all(False)
        self.apply_res()
        sysm = self.accumulate()
        return e, sysm

    def residuals(self) -> dict:
        R = self.window.n_residuals
        o = dict(new_state=np.zeros(R, np.int8), state=np.zeros(R, np.int8), state_energy=np.zeros(R, np.float32),
                 new_energy_wo=np.zeros(R, np.float32), center=np.zeros((R, 3), np.float32),
                 flags=np.zeros(R, np.uint8), jpjdf=np.zeros((R, 8), np.float32), rel_bs=np.zeros(R, np.float32))
        lib().oracle_get_residuals(self._h, _p(o["new_state"], i8p), _p(o["state"], i8p), _p(o["state_energy"], f32p),
                                   _p(o["new_energy_wo"], f32p), _p(o["center"], f32p), _p(o["flags"], u8p),
                                   _p(o["jpjdf"], f32p), _p(o["rel_bs"], f32p))
        return o

    def jacobians(self) -> np.ndarray:
        out = np.zeros((self.window.n_residuals, 78), np.float32)
        lib().oracle_get_jacobians(self._h, _p(out, f32p))
        return out

    def points(self) -> dict:
        P = self.window.n_points
        o = dict(HdiF=np.zeros(P, np.float32), bdSumF=np.zeros(P, np.float32), idepth_hessian=np.zeros(P, np.float32),
                 Hdd=np.zeros(P, np.float32), bd=np.zeros(P, np.float32), Hcd=np.zeros((P, 4), np.float32))
        lib().oracle_get_points(self._h, *[_p(o[k], f32p) for k in ("HdiF", "bdSumF", "idepth_hessian", "Hdd", "bd", "Hcd")])
        return o

    def frame_energy_th(self):
        out = np.zeros(self.window.n_frames, np.float32)
        lib().oracle_get_frame_energy_th(self._h, _p(out, f32p))
        return out

    def resubstitute(self, x, lam=1e-5):
        step = np.zeros(self.window.n_points, np.float32)
        lib().oracle_resubstitute(self._h, _p(np.ascontiguousarray(x, np.float64), f64p), float(lam), _p(step, f32p))
        return step

    def marginalize_points(self, points, ad_ht_delta):
        """flagPointsForRemoval + marginalizePointsF for `points` -> (H, b) = (M - Msc, Mb - Mbsc)."""
        n = self.window.dim
        pts = np.ascontiguousarray(points, np.int32)
        adh = np.ascontiguousarray(ad_ht_delta, np.float32)
        H = np.zeros((n, n), np.float64)
        b = np.zeros(n, np.float64)
        rc = lib().oracle_marginalize_points(self._h, int(pts.size), _p(pts, i32p), _p(adh, f32p), _p(H, f64p),
                                             _p(b, f64p))
        assert rc == 0
        return H, b

    def activate_points(self, pts, min_obs=1):
        """FullSystem::optimizeImmaturePoint for immature-point records of this window."""
        assert pts.dtype == IMMATURE_DTYPE and pts.flags.c_contiguous
        out = np.zeros(pts.size, ACTIVATION_DTYPE)
        rc = lib().oracle_activate_points(self._h, int(pts.size), pts.ctypes.data, int(min_obs), out.ctypes.data)
        assert rc == 0
        return out

    def time_iterations(self, iters: int) -> float:
        return float(lib().oracle_time_iterations(self._h, int(iters)))


def get_affine_opt_modes():
    a, b = C.c_float(), C.c_float()
    lib().oracle_get_affine_opt_modes(C.byref(a), C.byref(b))
    return a.value, b.value


class affine_opt_modes:
    """with oracle.affine_opt_modes(a, b): setting_affineOptModeA / B for the oracle (process-wide
    globals, as in the reference), restored on exit."""

    def __init__(self, a, b):
        self.ab = (float(a), float(b))

    def __enter__(self):
        self.saved = get_affine_opt_modes()
        lib().oracle_set_affine_opt_modes(*self.ab)
        return self

    def __exit__(self, *exc):
        lib().oracle_set_affine_opt_modes(*self.saved)
        return False


def solve_system(n_frames, iteration, lam, sysm, HM=None, bM=None, nullspaces=None):
    n = 8 * n_frames + 4
    x = np.zeros(n, np.float64)
    ns = None if nullspaces is None else np.ascontiguousarray(nullspaces, np.float64)
    lib().oracle_solve_system(int(n_frames), int(iteration), float(lam), _p(sysm["HA"], f64p), _p(sysm["bA"], f64p),
                              _p(sysm["HL"], f64p), _p(sysm["bL"], f64p), _p(HM, f64p), _p(bM, f64p),
                              _p(sysm["Hsc"], f64p), _p(sysm["bsc"], f64p), _p(ns, f64p),
                              0 if ns is None else ns.shape[0], _p(x, f64p))
    return x


def frame_terms(window):
    """Oracle restatement of FrameFramePrecalc::Set / setAdjointsF / takeData / nullspaces."""
    N = window.n_frames
    fr = np.ascontiguousarray(window.frames)
    pre = np.zeros((N * N, 48), np.float32)  # LDSO_BA_PRECALC_STRIDE
    lib().oracle_frame_precalc(N, fr.ctypes.data, _p(np.ascontiguousarray(window.calib, np.float32), f32p), _p(pre, f32p))
    adH = np.zeros((N * N, 64))
    adT = np.zeros((N * N, 64))
    cp = np.zeros(4)
    lib().oracle_set_adjoints(N, fr.ctypes.data, _p(adH, f64p), _p(adT, f64p), _p(cp, f64p))
    prior = np.zeros((N, 8))
    delta = np.zeros((N, 8))
    dprior = np.zeros((N, 8))
    lib().oracle_frame_take_data(N, fr.ctypes.data, _p(prior, f64p), _p(delta, f64p), _p(dprior, f64p))
    ns = np.zeros((7, 8 * N + 4))
    lib().oracle_nullspaces(N, fr.ctypes.data, _p(ns, f64p))
    return dict(precalc=pre, ad_host=adH, ad_target=adT, c_prior=cp, frame_prior=prior, frame_delta=delta,
                frame_delta_prior=dprior, nullspaces=ns)


def do_step_from_backup(frames, x, calib_value, calib_value_zero, point_host, idepth_backup, point_step,
                        th_opt_iterations=1.2):
    """FullSystem::doStepFromBackup for one window -> (frames, calib_value, value_scaledf, cDeltaF,
    idepth, canbreak); calib_value is stepped in place as well."""
    fr = np.ascontiguousarray(frames)
    out = np.zeros_like(fr)
    P = int(np.asarray(point_host).size)
    ph = np.ascontiguousarray(point_host, np.int32)
    ib = np.ascontiguousarray(idepth_backup, np.float32)
    ps = np.ascontiguousarray(point_step, np.float32)
    idepth = np.zeros(P, np.float32)
    sf = np.zeros(4, np.float32)
    cd = np.zeros(4, np.float32)
    cz = np.ascontiguousarray(calib_value_zero, np.float64)
    cv = np.ascontiguousarray(calib_value, np.float64)  # a copy unless already float64 (stepped in place)
    rc = lib().oracle_do_step_from_backup(len(fr), fr.ctypes.data, _p(np.ascontiguousarray(x, np.float64), f64p),
                                          _p(cv, f64p), _p(cz, f64p), P, _p(ph, i32p), _p(ib, f32p),
                                          _p(ps, f32p), float(th_opt_iterations), out.ctypes.data, _p(idepth, f32p),
                                          _p(sf, f32p), _p(cd, f32p))
    assert rc >= 0
    if cv is not calib_value and isinstance(calib_value, np.ndarray) and calib_value.flags.writeable:
        calib_value[...] = cv
    return out, cv, sf, cd, idepth, bool(rc)


# ---- coarse tracker (ldso_oracle_tracker.cpp): the checker of include/ldso_ct.h -------------
def ct_levels(w, h):
    return int(lib().oracle_ct_levels(int(w), int(h)))


def ct_make_k(calib, w, h):
    L = ct_levels(w, h)
    out = np.zeros((L, 13), np.float32)
    lib().oracle_ct_make_k(_p(np.ascontiguousarray(calib, np.float32), f32p), int(w), int(h), L, _p(out, f32p))
    return out


def make_images(color, w, h, b_response=None):
    """FrameHessian::makeImages: per level (dI [wl*hl][3], absSquaredGrad [wl*hl])."""
    L = ct_levels(w, h)
    tot = sum((w >> l) * (h >> l) for l in range(L))
    dIp = np.zeros((tot, 3), np.float32)
    ag = np.zeros(tot, np.float32)
    B = None if b_response is None else np.ascontiguousarray(b_response, np.float32)
    lib().oracle_make_images(_p(np.ascontiguousarray(color, np.float32).reshape(-1), f32p), int(w), int(h), L,
                             _p(B, f32p), _p(dIp, f32p), _p(ag, f32p))
    out, off = [], 0
    for l in range(L):
        n = (w >> l) * (h >> l)
        out.append((dIp[off:off + n], ag[off:off + n]))
        off += n
    return out


def ct_calc_res(lvl, wl, hl, kl, dI, pc, T, aff6, cutoff_th):
    """CoarseTracker::calcRes -> (rs[6], warped [buf_warped_n][8])."""
    u, v, idp, col = [np.ascontiguousarray(a, np.float32).reshape(-1) for a in pc]
    n = u.size
    rs = np.zeros(6, np.float64)
    warped = np.zeros((n + 4, 8), np.float32)
    nw = C.c_int32()
    Tm = np.ascontiguousarray(np.asarray(T, np.float64)[:3, :4])
    lib().oracle_ct_calc_res(int(lvl), int(wl), int(hl), _p(np.ascontiguousarray(kl, np.float32), f32p),
                             _p(np.ascontiguousarray(dI, np.float32), f32p), n, _p(u, f32p), _p(v, f32p),
                             _p(idp, f32p), _p(col, f32p), _p(Tm, f64p),
                             _p(np.ascontiguousarray(aff6, np.float64), f64p), float(cutoff_th), _p(rs, f64p),
                             _p(warped, f32p), C.byref(nw))
    return rs, warped[:nw.value].copy()


def ct_calc_gs(warped, fxl, fyl, aff6):
    """CoarseTracker::calcGSSSE (Accumulator9 in SSE lane order) -> (H 8x8, b 8)."""
    H = np.zeros((8, 8), np.float64)
    b = np.zeros(8, np.float64)
    w = np.ascontiguousarray(warped, np.float32)
    rc = lib().oracle_ct_calc_gs(int(w.shape[0]), _p(w, f32p), float(fxl), float(fyl),
                                 _p(np.ascontiguousarray(aff6, np.float64), f64p), _p(H, f64p), _p(b, f64p))
    assert rc == 0
    return H, b


# ---- immature points (ldso_oracle_tracker.cpp): the checker of ldso_ct_make_immature / _trace --
# ldso_ct_immature (include/ldso_ct.h), 128 bytes
IMMATURE_DTYPE = np.dtype([("u", "<f4"), ("v", "<f4"), ("idepth_min", "<f4"), ("idepth_max", "<f4"),
                           ("quality", "<f4"), ("energy_th", "<f4"), ("color", "<f4", (8,)),
                           ("weights", "<f4", (8,)), ("grad_h", "<f4", (4,)), ("host", "<i4"),
                           ("last_status", "<i4"), ("last_uv", "<f4", (2,)), ("last_interval", "<f4"),
                           ("type", "<f4")])
assert IMMATURE_DTYPE.itemsize == 128
ACTIVATION_DTYPE = np.dtype([("idepth", "<f4"), ("status", "<i4"), ("in_mask", "<u4"), ("energy", "<f4")])


def ip_make(dI0, w, h, uv, type_=1.0, host=0):
    """new ImmaturePoint(frame, feat, type, HCalib) for features uv [n][2] on level-0 dI [w*h][3]."""
    uv = np.ascontiguousarray(uv, np.float32).reshape(-1, 2)
    out = np.zeros(uv.shape[0], IMMATURE_DTYPE)
    lib().oracle_ip_make(_p(np.ascontiguousarray(dI0, np.float32), f32p), int(w), int(h), int(uv.shape[0]),
                         _p(uv, f32p), float(type_), int(host), out.ctypes.data)
    return out


def ip_trace(dI0, w, h, krki, kt, aff, pts):
    """traceNewCoarse over the records pts (updated in place) -> status counts [6]."""
    assert pts.dtype == IMMATURE_DTYPE and pts.flags.c_contiguous
    counts = np.zeros(6, np.int32)
    lib().oracle_ip_trace(_p(np.ascontiguousarray(dI0, np.float32), f32p), int(w), int(h),
                          _p(np.ascontiguousarray(krki, np.float32), f32p),
                          _p(np.ascontiguousarray(kt, np.float32), f32p),
                          _p(np.ascontiguousarray(aff, np.float32), f32p), int(pts.size), pts.ctypes.data,
                          _p(counts, i32p))
    return counts


# ---- CPU baseline timing build (bench.py cpu_baseline leg only) -----------------------------
NATIVE_FLAGS = ["-O3", "-march=native", "-std=c++17", "-fPIC", "-shared"]


def build_timing_lib(out_path: str) -> str:
    """The same restatement compiled for speed the way the reference is (CMakeLists.txt:55-56:
    -O3 -march=native; FP contraction left at the compiler default, i.e. allowed).  Built on
    the machine that runs it; used for timing only, never as the checker."""
    src = [os.path.join(HERE, "ldso_oracle.cpp"), os.path.join(HERE, "ldso_oracle_tracker.cpp")]
    subprocess.run(["g++"] + NATIVE_FLAGS + ["-o", out_path] + src + ["-lpthread"], check=True, timeout=300)
    return out_path


class TimingWindow:
    """oracle_create / oracle_time_iterations through a separately loaded timing build."""

    def __init__(self, window, threads: int, lib_path: str):
        self._lib = C.CDLL(lib_path)
        self._lib.oracle_set_threads.argtypes = [C.c_int]
        self._lib.oracle_create.restype = C.c_void_p
        self._lib.oracle_create.argtypes = [C.c_void_p]
        self._lib.oracle_destroy.argtypes = [C.c_void_p]
        self._lib.oracle_time_iterations.restype = C.c_double
        self._lib.oracle_time_iterations.argtypes = [C.c_void_p, C.c_int]
        self._lib.oracle_set_threads(int(threads))
        s = window.c_struct()
        self._h = self._lib.oracle_create(C.byref(s))
        window._keep = []
        if not self._h:
            raise ValueError("oracle_create rejected the window")

    def time_iterations(self, iters: int) -> float:
        return float(self._lib.oracle_time_iterations(self._h, int(iters)))

    def close(self):
        if self._h:
            self._lib.oracle_destroy(self._h)
            self._h = None
