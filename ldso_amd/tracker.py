"""CoarseTracker face over the C ABI in include/ldso_ct.h.

Mirrors the reference class (src/frontend/CoarseTracker.cc) for the parts that run on the GPU:

    CoarseTracker(w, h)                   -> CoarseTracker(width, height)
    makeK(HCalib)                         -> make_k(calib)                     CoarseTracker.cc:312-339
    newFrame->makeImages(color, HCalib)   -> set_new_frame(color, exposure)    FrameHessian.cc:59-115
    setCoarseTrackingRef's pc_* outputs   -> set_reference(levels, ...)        CoarseTracker.cc:357-538
    calcRes(lvl, refToNew, aff, cutoff)   -> calc_res(lvl, T, aff, cutoff)     CoarseTracker.cc:540-673
    calcGSSSE(lvl, H, b, refToNew, aff)   -> calc_gs(lvl, T, aff)              CoarseTracker.cc:675-741
    calcRes + calcGSSSE at one pose       -> calc_res_gs(lvl, T, aff, cutoff)  CoarseTracker.cc:90-105, 218-245
    new ImmaturePoint(newFrame, feat, ..) -> make_immature(uv, type, host)     ImmaturePoint.cc:14-39
    traceNewCoarse -> ImmaturePoint::traceOn
                                          -> trace(krki, kt, aff)              FullSystem.cc:1157-1194,
                                             (records resident: immature_upload / immature_download)
                                                                               ImmaturePoint.cc:47-317

No numerical work happens here; every call goes to libldso_ba.so (no fallback).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def _f32(a):
    return np.ascontiguousarray(a, np.float32)


class CoarseTracker:
    def __init__(self, width: int, height: int, device: int = 0):
        lib = L.lib()
        h = C.c_void_p()
        nl = C.c_int32()
        L.check(lib.ldso_ct_create(int(device), int(width), int(height), C.byref(h), C.byref(nl)))
        self._h = h
        self.width, self.height, self.levels = int(width), int(height), int(nl.value)

    def close(self):
        if self._h and self._h.value:
            L.lib().ldso_ct_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def make_k(self, calib) -> np.ndarray:
        """Per level {fx, fy, cx, cy, Ki[9]} (13 floats)."""
        out = np.zeros((self.levels, 13), np.float32)
        L.check(L.lib().ldso_ct_make_k(self._h, L.ptr(_f32(calib), L.f32p), L.ptr(out, L.f32p)))
        return out

    def set_new_frame(self, color, ab_exposure: float = 1.0, b_response=None):
        color = _f32(color).reshape(-1)
        assert color.size == self.width * self.height
        B = None if b_response is None else _f32(b_response)
        assert B is None or B.size == 256
        L.check(L.lib().ldso_ct_set_new_frame(self._h, L.ptr(color, L.f32p), float(ab_exposure), L.ptr(B, L.f32p)))

    def frame_level(self, lvl: int):
        wl, hl = self.width >> lvl, self.height >> lvl
        dI = np.zeros((hl * wl, 3), np.float32)
        ag = np.zeros(hl * wl, np.float32)
        L.check(L.lib().ldso_ct_get_frame_level(self._h, int(lvl), L.ptr(dI, L.f32p), L.ptr(ag, L.f32p)))
        return dI, ag

    def set_reference(self, pc, ab_exposure: float = 1.0, aff_ab=(0.0, 0.0)):
        """pc: per level a dict/tuple (u, v, idepth, color) of equal-length float arrays."""
        assert len(pc) == self.levels
        keep = []
        n = np.zeros(self.levels, np.int32)
        arrs = [(L.f32p * self.levels)() for _ in range(4)]
        for l, lv in enumerate(pc):
            cols = [lv[k] for k in ("u", "v", "idepth", "color")] if isinstance(lv, dict) else list(lv)
            cols = [_f32(c).reshape(-1) for c in cols]
            n[l] = cols[0].size
            assert all(c.size == n[l] for c in cols)
            for j in range(4):
                keep.append(cols[j])
                arrs[j][l] = L.ptr(cols[j], L.f32p)
        L.check(L.lib().ldso_ct_set_reference(self._h, L.ptr(n, L.i32p), *arrs, float(ab_exposure),
                                              float(aff_ab[0]), float(aff_ab[1])))

    def calc_res(self, lvl: int, ref_to_new, aff_ab=(0.0, 0.0), cutoff_th: float = 20.0) -> np.ndarray:
        T = np.ascontiguousarray(np.asarray(ref_to_new, np.float64)[:3, :4])
        rs = np.zeros(6, np.float64)
        L.check(L.lib().ldso_ct_calc_res(self._h, int(lvl), L.ptr(T, L.f64p), float(aff_ab[0]), float(aff_ab[1]),
                                         float(cutoff_th), L.ptr(rs, L.f64p)))
        return rs

    def calc_res_batch(self, lvl: int, ref_to_new, aff_ab, cutoff_th: float = 20.0) -> np.ndarray:
        T = np.ascontiguousarray(np.asarray(ref_to_new, np.float64)[:, :3, :4])
        ab = np.ascontiguousarray(aff_ab, np.float64).reshape(-1, 2)
        assert ab.shape[0] == T.shape[0]
        rs = np.zeros((T.shape[0], 6), np.float64)
        L.check(L.lib().ldso_ct_calc_res_batch(self._h, int(lvl), int(T.shape[0]), L.ptr(T, L.f64p),
                                               L.ptr(ab, L.f64p), float(cutoff_th), L.ptr(rs, L.f64p)))
        return rs

    def calc_gs(self, lvl: int, ref_to_new, aff_ab=(0.0, 0.0)):
        T = np.ascontiguousarray(np.asarray(ref_to_new, np.float64)[:3, :4])
        H = np.zeros((8, 8), np.float64)
        b = np.zeros(8, np.float64)
        L.check(L.lib().ldso_ct_calc_gs(self._h, int(lvl), L.ptr(T, L.f64p), float(aff_ab[0]), float(aff_ab[1]),
                                        L.ptr(H, L.f64p), L.ptr(b, L.f64p)))
        return H, b

    def calc_res_gs(self, lvl: int, ref_to_new, aff_ab=(0.0, 0.0), cutoff_th: float = 20.0):
        """calcRes + calcGSSSE at the same pose in one round trip -> (rs[6], H 8x8, b 8).
        The LM loop calls this once per iteration: the pose and result buffers and their ctypes
        pointers are made once per tracker, the results returned as copies."""
        if not hasattr(self, "_lm"):
            bufs = (np.zeros((3, 4), np.float64), np.zeros(6, np.float64), np.zeros((8, 8), np.float64),
                    np.zeros(8, np.float64))
            self._lm = (bufs, tuple(L.ptr(x, L.f64p) for x in bufs), L.lib().ldso_ct_calc_res_gs)
        (T, rs, H, b), (pT, prs, pH, pb), fn = self._lm
        T[...] = np.asarray(ref_to_new, np.float64)[:3, :4]
        L.check(fn(self._h, int(lvl), pT, float(aff_ab[0]), float(aff_ab[1]), float(cutoff_th), prs, pH, pb))
        return rs.copy(), H.copy(), b.copy()

    def warped(self) -> np.ndarray:
        """buf_warped_* of the last calc_res as [n][8] {idepth, u, v, dx, dy, residual, weight, refColor}."""
        n = C.c_int32()
        lib = L.lib()
        L.check(lib.ldso_ct_get_warped(self._h, C.byref(n), L.ptr(None, L.f32p), 0))
        out = np.zeros((n.value, 8), np.float32)
        L.check(lib.ldso_ct_get_warped(self._h, C.byref(n), L.ptr(out, L.f32p), int(n.value)))
        return out

    def set_kernel_timing(self, on: bool):
        L.check(L.lib().ldso_ct_set_kernel_timing(self._h, int(bool(on))))

    def kernel_times(self) -> dict:
        lib = L.lib()
        k = lib.ldso_ct_num_kernels()
        ms = np.zeros(k, np.float64)
        cnt = np.zeros(k, np.int64)
        L.check(lib.ldso_ct_get_kernel_times(self._h, L.ptr(ms, L.f64p), L.ptr(cnt, L.i64p), int(k)))
        return {lib.ldso_ct_kernel_name(i).decode(): (float(ms[i]), int(cnt[i])) for i in range(k)}

    # ---- immature points ----
    def make_immature(self, uv, type_: float = 1.0, host: int = 0) -> np.ndarray:
        """ImmaturePoint(newFrame, feat, type) for features uv [n][2] on the new frame -> records."""
        uv = _f32(uv).reshape(-1, 2)
        out = np.zeros(uv.shape[0], L.IMMATURE_DTYPE)
        L.check(L.lib().ldso_ct_make_immature(self._h, int(uv.shape[0]), L.ptr(uv, L.f32p), float(type_), int(host),
                                              out.ctypes.data))
        return out

    def immature_upload(self, pts: np.ndarray):
        assert pts.dtype == L.IMMATURE_DTYPE and pts.flags.c_contiguous
        L.check(L.lib().ldso_ct_immature_upload(self._h, int(pts.size), pts.ctypes.data))
        self._ip_n = int(pts.size)

    def immature_download(self) -> np.ndarray:
        out = np.zeros(getattr(self, "_ip_n", 0), L.IMMATURE_DTYPE)
        L.check(L.lib().ldso_ct_immature_download(self._h, int(out.size), out.ctypes.data))
        return out

    def trace(self, krki, kt, aff, counts: bool = True):
        """traceNewCoarse over the resident records: per host KRKi [9], Kt [3], aff [2] -> counts [6]
        (GOOD, OOB, OUTLIER, SKIPPED, BADCONDITION, UNINITIALIZED) or None."""
        krki = _f32(krki).reshape(-1, 9)
        kt = _f32(kt).reshape(-1, 3)
        aff = _f32(aff).reshape(-1, 2)
        assert krki.shape[0] == kt.shape[0] == aff.shape[0]
        c = np.zeros(6, np.int32) if counts else None
        L.check(L.lib().ldso_ct_trace(self._h, int(krki.shape[0]), L.ptr(krki, L.f32p), L.ptr(kt, L.f32p),
                                      L.ptr(aff, L.f32p), L.ptr(c, L.i32p)))
        return c
