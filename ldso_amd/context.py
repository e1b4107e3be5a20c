"""Python face of the device context (one per FullSystem / group of windows).

Mirrors the reference's per-iteration call sequence (FullSystem::optimize, FullSystem.cc:844-1007):

    ctx.reset_oob()                         # PointFrameResidual::resetOOB for activeResiduals
    ctx.linearize(fix=False)                # linearizeAll(false) + applyRes + accumulate{AF,LF,SCF}
    x = ctx.solve(0, iteration, lam, ns)    # EnergyFunctional::solveSystemF (stitched system)
    ctx.resubstitute(0, x, lam)             # resubstituteF_MT
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .window import Window


class BAContext:
    def __init__(self, device: int = 0):
        self._lib = L.lib()
        h = C.c_void_p()
        L.check(self._lib.ldso_ba_create(int(device), C.byref(h)))
        self._h = h
        self.windows: list[Window] = []
        self._structs = None

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.ldso_ba_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- settings ----------------------------------------------------------------------
    def set_settings(self, settings=None):
        """ldso_ba_set_settings: the reference settings this context runs with (an L.OptSettings;
        None = the defaults).  Unsupported ones raise (the context keeps its previous settings)."""
        L.check(self._lib.ldso_ba_set_settings(self._h, C.byref(settings) if settings is not None else None))
        return self

    def settings(self) -> L.OptSettings:
        out = L.OptSettings()
        L.check(self._lib.ldso_ba_get_settings(self._h, C.byref(out)))
        return out

    # ---- structure ---------------------------------------------------------------------
    def load(self, windows, shard_rank: int = 0, shard_count: int = 1):
        if isinstance(windows, Window):
            windows = [windows]
        self.windows = list(windows)
        structs = (L.LdsoBaWindow * len(self.windows))(*[w.c_struct() for w in self.windows])
        L.check(self._lib.ldso_ba_load(self._h, len(self.windows), structs, int(shard_rank), int(shard_count)))
        self._structs = structs
        for w in self.windows:
            w._keep = []  # host copies are no longer referenced by the device
        return self

    def optimize(self, n_its: int, calib_value=None, calib_value_zero=None, nullspaces=None, settings=None):
        """FullSystem::optimize on the device (ldso_ba_optimize): up to n_its GN iterations of every
        loaded window with no host round trip; each window leaves the loop on the reference's
        exits (canbreak after setting_minOptIterations, or lost on a NaN solution).
        calib_value / calib_value_zero: [n_windows][4] CalibHessian::value / value_zero (default:
        each window's calib / 50, i.e. no calibration delta); settings: an L.OptSettings (None =
        the reference's defaults).  Returns (energies [n_its + 1][n_windows][3], frames,
        calib_value, idepths, iterations [n_windows], status [n_windows] (L.OPT_*)).  Non-None settings
        are installed into the context first (ldso_ba_set_settings)."""
        nw = len(self.windows)
        frames = np.ascontiguousarray(np.concatenate([np.ascontiguousarray(w.frames) for w in self.windows]))
        if calib_value is None:
            calib_value = np.stack([w.calib.astype(np.float64) * (1.0 / 50.0) for w in self.windows])
        calib_value = np.ascontiguousarray(calib_value, np.float64).reshape(nw, 4)
        cz = calib_value.copy() if calib_value_zero is None else np.ascontiguousarray(calib_value_zero, np.float64)
        ns = self._ns_all(nullspaces)
        e = np.zeros((n_its + 1, nw, 3), np.float64)
        fo = np.zeros_like(frames)
        co = np.zeros((nw, 4), np.float64)
        idep = np.zeros(sum(w.n_points for w in self.windows), np.float32)
        its = np.zeros(nw, np.int32)
        status = np.zeros(nw, np.int32)
        sp = C.byref(settings) if settings is not None else None
        L.check(self._lib.ldso_ba_optimize(self._h, int(n_its), sp, frames.ctypes.data, L.ptr(calib_value, L.f64p),
                                           L.ptr(cz, L.f64p), L.ptr(ns, L.f64p), L.ptr(e, L.f64p), fo.ctypes.data,
                                           L.ptr(co, L.f64p), L.ptr(idep, L.f32p), L.ptr(its, L.i32p),
                                           L.ptr(status, L.i32p)))
        return e, fo, co, self._split(idep, [w.n_points for w in self.windows]), its, status

    def comm_init(self, unique_id, rank: int, world: int):
        """Attach to an RCCL communicator (ldso_ba_comm_init); unique_id: 128 bytes from
        ldso_ba_comm_unique_id on rank 0.  See ldso_amd.dist.attach_rccl."""
        uid = np.frombuffer(bytes(unique_id), np.uint8).copy()
        L.check(self._lib.ldso_ba_comm_init(self._h, uid.ctypes.data, int(rank), int(world)))
        return self

    def load_marginalization(self, parent: "BAContext", parent_win: int, window: Window):
        """Make this context the marginalisation context of `parent`'s window `parent_win` for the
        points (and residuals) of `window` (ldso_ba_load_marginalization: images are borrowed)."""
        self.windows = [window]
        s = window.c_struct(with_images=False)
        L.check(self._lib.ldso_ba_load_marginalization(self._h, parent._h, int(parent_win), C.byref(s)))
        self._structs = s
        self._parent = parent  # the borrowed images must outlive this context
        window._keep = []
        return self

    def marginalize_points(self, ad_ht_delta):
        """ldso_ba_marginalize_points -> (H, b) = (M - Msc, Mb - Mbsc) (EnergyFunctional.cc:226-243)."""
        n = self.windows[0].dim
        H = np.zeros((n, n), np.float64)
        b = np.zeros(n, np.float64)
        adh = np.ascontiguousarray(ad_ht_delta, np.float32)
        L.check(self._lib.ldso_ba_marginalize_points(self._h, L.ptr(adh, L.f32p), L.ptr(H, L.f64p), L.ptr(b, L.f64p)))
        return H, b

    def update(self, win: int, window: Window):
        s = window.c_struct()
        L.check(self._lib.ldso_ba_update(self._h, int(win), C.byref(s)))

    def activate_points(self, win: int, pts: np.ndarray, min_obs: int = 1) -> np.ndarray:
        """FullSystem::optimizeImmaturePoint for ldso_ct_immature records hosted in window `win`
        (FullSystem.cc:1035-1156) -> ldso_ba_activation records {idepth, status, in_mask, energy}."""
        assert pts.dtype == L.IMMATURE_DTYPE and pts.flags.c_contiguous
        out = np.zeros(pts.size, L.ACTIVATION_DTYPE)
        L.check(self._lib.ldso_ba_activate_points(self._h, int(win), int(pts.size), pts.ctypes.data, int(min_obs),
                                                  out.ctypes.data))
        return out

    def update_points(self, win: int, vals: np.ndarray):
        """ldso_ba_update_points: [P][4] (idepth_scaled, idepth_zero_scaled, priorF, deltaF), caller order."""
        v = np.ascontiguousarray(vals, np.float32).reshape(-1, 4)
        L.check(self._lib.ldso_ba_update_points(self._h, int(win), L.ptr(v, L.f32p)))

    def reset_oob(self, win: int = -1):
        L.check(self._lib.ldso_ba_reset_oob(self._h, int(win)))

    # ---- hot path ----------------------------------------------------------------------
    def linearize(self, fix: bool = False, accumulate: bool = True):
        L.check(self._lib.ldso_ba_linearize(self._h, int(bool(fix)), int(bool(accumulate))))

    def sync(self):
        L.check(self._lib.ldso_ba_sync(self._h))

    @property
    def stream(self) -> int:
        return int(self._lib.ldso_ba_stream(self._h) or 0)

    # ---- results -----------------------------------------------------------------------
    def energy(self, win: int = 0):
        out = np.zeros(3, np.float64)
        L.check(self._lib.ldso_ba_get_energy(self._h, int(win), L.ptr(out, L.f64p)))
        return out

    def system(self, win: int = 0) -> dict:
        n = self.windows[win].dim
        out = {k: np.zeros((n, n) if k.startswith("H") else n, np.float64) for k in ("HA", "bA", "HL", "bL", "Hsc", "bsc")}
        L.check(self._lib.ldso_ba_get_system(self._h, int(win), *[L.ptr(out[k], L.f64p) for k in ("HA", "bA", "HL", "bL", "Hsc", "bsc")]))
        return out

    def residuals(self, win: int = 0) -> dict:
        R = self.windows[win].n_residuals
        o = dict(new_state=np.zeros(R, np.int8), state=np.zeros(R, np.int8), state_energy=np.zeros(R, np.float32),
                 new_energy_wo=np.zeros(R, np.float32), center=np.zeros((R, 3), np.float32),
                 flags=np.zeros(R, np.uint8), jpjdf=np.zeros((R, 8), np.float32), rel_bs=np.zeros(R, np.float32))
        L.check(self._lib.ldso_ba_get_residuals(
            self._h, int(win), L.ptr(o["new_state"], L.i8p), L.ptr(o["state"], L.i8p), L.ptr(o["state_energy"], L.f32p),
            L.ptr(o["new_energy_wo"], L.f32p), L.ptr(o["center"], L.f32p), L.ptr(o["flags"], L.u8p),
            L.ptr(o["jpjdf"], L.f32p), L.ptr(o["rel_bs"], L.f32p)))
        return o

    def points(self, win: int = 0) -> dict:
        P = self.windows[win].n_points
        o = dict(HdiF=np.zeros(P, np.float32), bdSumF=np.zeros(P, np.float32), idepth_hessian=np.zeros(P, np.float32),
                 Hdd=np.zeros(P, np.float32), bd=np.zeros(P, np.float32), Hcd=np.zeros((P, 4), np.float32))
        L.check(self._lib.ldso_ba_get_points(self._h, int(win), *[L.ptr(o[k], L.f32p) for k in
                                                                  ("HdiF", "bdSumF", "idepth_hessian", "Hdd", "bd", "Hcd")]))
        return o

    def frame_energy_th(self, win: int = 0):
        out = np.zeros(self.windows[win].n_frames, np.float32)
        L.check(self._lib.ldso_ba_get_frame_energy_th(self._h, int(win), L.ptr(out, L.f32p)))
        return out

    def solve(self, win: int = 0, iteration: int = 0, lam: float = 1e-5, nullspaces=None):
        x = np.zeros(self.windows[win].dim, np.float64)
        ns = None if nullspaces is None else np.ascontiguousarray(nullspaces, np.float64)
        L.check(self._lib.ldso_ba_solve(self._h, int(win), int(iteration), float(lam), L.ptr(ns, L.f64p),
                                        0 if ns is None else ns.shape[0], L.ptr(x, L.f64p)))
        return x

    def resubstitute(self, win: int, x, lam: float = 1e-5, fetch: bool = True):
        x = np.ascontiguousarray(x, np.float64)
        step = np.zeros(self.windows[win].n_points, np.float32) if fetch else None
        L.check(self._lib.ldso_ba_resubstitute(self._h, int(win), L.ptr(x, L.f64p), float(lam), L.ptr(step, L.f32p)))
        return step

    # ---- device-side solve ---------------------------------------------
    def _ns_all(self, nullspaces):
        if nullspaces is None:
            return None
        return np.ascontiguousarray(np.concatenate([np.asarray(n, np.float64).ravel() for n in nullspaces]))

    def _split(self, flat, sizes):
        out, o = [], 0
        for n in sizes:
            out.append(flat[o:o + n])
            o += n
        return out

    def solve_device(self, iteration: int = 0, lam: float = 1e-5, nullspaces=None, n_null: int = 7):
        """x of every window (solveSystemF on the GPU); nullspaces: list of [7][8N+4] arrays, of
        which the first n_null rows project."""
        ns = self._ns_all(nullspaces)
        x = np.zeros(sum(w.dim for w in self.windows), np.float64)
        L.check(self._lib.ldso_ba_solve_device(self._h, int(iteration), float(lam), L.ptr(ns, L.f64p),
                                               0 if ns is None else int(n_null), L.ptr(x, L.f64p)))
        return self._split(x, [w.dim for w in self.windows])

    def resubstitute_device(self, lam: float = 1e-5):
        """Point steps of every window from the device x (caller point order per window)."""
        st = np.zeros(sum(w.n_points for w in self.windows), np.float32)
        L.check(self._lib.ldso_ba_resubstitute_device(self._h, float(lam), L.ptr(st, L.f32p)))
        return self._split(st, [w.n_points for w in self.windows])

    def iterate(self, iteration: int = 0, lam: float = 1e-5, nullspaces=None, fetch_steps: bool = True):
        """One fused GN iteration on the device: pass + solve + resubstitute, one synchronisation."""
        ns = self._ns_all(nullspaces)
        x = np.zeros(sum(w.dim for w in self.windows), np.float64)
        st = np.zeros(sum(w.n_points for w in self.windows), np.float32) if fetch_steps else None
        e = np.zeros((len(self.windows), 3), np.float64)
        L.check(self._lib.ldso_ba_iterate(self._h, int(iteration), float(lam), L.ptr(ns, L.f64p),
                                          0 if ns is None else 7, L.ptr(x, L.f64p), L.ptr(st, L.f32p),
                                          L.ptr(e, L.f64p)))
        xs = self._split(x, [w.dim for w in self.windows])
        sts = self._split(st, [w.n_points for w in self.windows]) if fetch_steps else None
        return e, xs, sts

    # ---- multi-GPU / profiling -----------------------------------------------------------
    def packed_system(self):
        p = C.c_void_p()
        n = C.c_int64()
        s = C.c_int64()
        L.check(self._lib.ldso_ba_packed_system(self._h, C.byref(p), C.byref(n), C.byref(s)))
        return int(p.value or 0), int(n.value), int(s.value)

    def unpack_system(self):
        L.check(self._lib.ldso_ba_unpack_system(self._h))

    def set_tuning(self, key: int, value: int):
        L.check(self._lib.ldso_ba_set_tuning(self._h, int(key), int(value)))

    def set_kernel_timing(self, on: bool):
        L.check(self._lib.ldso_ba_set_kernel_timing(self._h, int(bool(on))))

    def kernel_times(self) -> dict:
        n = int(self._lib.ldso_ba_num_kernels())
        ms = np.zeros(n, np.float64)
        cnt = np.zeros(n, np.int64)
        L.check(self._lib.ldso_ba_get_kernel_times(self._h, L.ptr(ms, L.f64p), L.ptr(cnt, L.i64p), n))
        return {self._lib.ldso_ba_kernel_name(i).decode(): (float(ms[i]), int(cnt[i])) for i in range(n)}

    def stats(self):
        b, p, r = C.c_int64(), C.c_int64(), C.c_int64()
        L.check(self._lib.ldso_ba_stats(self._h, C.byref(b), C.byref(p), C.byref(r)))
        return dict(device_bytes=b.value, points=p.value, residuals=r.value)
