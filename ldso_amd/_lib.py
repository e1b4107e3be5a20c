"""ctypes bindings of the C ABI in include/ldso_ba.h.

The product path is the HIP library ``ldso_amd/lib/libldso_ba.so`` (built in-tree by
``__graft_entry__.build()``).  There is no CPU fallback: if the library is missing the import
fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.environ.get("LDSO_BA_LIB") or os.path.join(LIB_DIR, "libldso_ba.so")  # override: A/B builds only
SYNTH_PATH = os.path.join(LIB_DIR, "libldso_synth.so")

PATTERN_NUM = 8
CPARS = 4
MAX_FRAMES = 16
PRECALC_STRIDE = 48
POINT_STRIDE = 24
RES_IN, RES_OOB, RES_OUTLIER = 0, 1, 2
FLAG_ACTIVE, FLAG_NEW = 1, 2

i32p = C.POINTER(C.c_int32)
f32p = C.POINTER(C.c_float)
f64p = C.POINTER(C.c_double)
i8p = C.POINTER(C.c_int8)
u8p = C.POINTER(C.c_uint8)
i64p = C.POINTER(C.c_int64)

FRAME_STATE_DTYPE = np.dtype(
    [
        ("world_to_cam_evalpt", np.float64, (12,)),
        ("state", np.float64, (10,)),
        ("state_zero", np.float64, (10,)),
        ("ab_exposure", np.float64),
        ("is_first_frame", np.int32),
        ("pad_", np.int32),
    ],
    align=True,
)
assert FRAME_STATE_DTYPE.itemsize == 272


ABI_VERSION = 6

# setting_solverMode bits (Settings.h:14-25) and ldso_ba_optimize's per-window outcome
SOLVER_SVD, SOLVER_ORTHOGONALIZE_SYSTEM, SOLVER_ORTHOGONALIZE_POINTMARG, SOLVER_ORTHOGONALIZE_FULL = 1, 2, 4, 8
SOLVER_SVD_CUT7, SOLVER_REMOVE_POSEPRIOR, SOLVER_USE_GN, SOLVER_FIX_LAMBDA = 16, 32, 64, 128
SOLVER_ORTHOGONALIZE_X, SOLVER_MOMENTUM, SOLVER_STEPMOMENTUM, SOLVER_ORTHOGONALIZE_X_LATER = 256, 512, 1024, 2048
SOLVER_DEFAULT = SOLVER_FIX_LAMBDA | SOLVER_ORTHOGONALIZE_X_LATER
OPT_RAN_ALL, OPT_CONVERGED, OPT_LOST = 0, 1, 2


class OptSettings(C.Structure):
    """ldso_ba_opt_settings: setting_solverMode, setting_forceAceptStep, setting_minOptIterations,
    setting_thOptIterations, setting_affineOptModeA / B, setting_vi_enable (Setting.cc:23, 36-38, 65-66,
    73, 152)."""
    _fields_ = [("solver_mode", C.c_int32), ("force_accept_step", C.c_int32), ("min_opt_iterations", C.c_int32),
                ("th_opt_iterations", C.c_float), ("affine_opt_mode_a", C.c_float), ("affine_opt_mode_b", C.c_float),
                ("vi_enable", C.c_int32), ("reserved_", C.c_int32)]

    @classmethod
    def default(cls, **kw):
        s = cls(SOLVER_DEFAULT, 1, 1, 1.2, 1e12, 1e8, 0, 0)
        for k, v in kw.items():
            setattr(s, k, v)
        return s


# setting_affineOptModeA / B of the reference's drivers (the library default is Setting.cc:65-66)
AFFINE_MODES = {
    "default": (1e12, 1e8),     # Setting.cc:65-66
    "kitti_euroc": (0.0, 0.0),  # run_dso_kitti.cc:299-300, run_dso_euroc.cc:291-292, TUM-Mono mode 1
    "fixed": (-1.0, -1.0),      # run_dso_tum_mono.cc:291-292 (mode 2: a and b fixed)
}


class LdsoBaWindow(C.Structure):
    _fields_ = [
        ("n_frames", C.c_int32),
        ("n_points", C.c_int32),
        ("n_residuals", C.c_int32),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("calib", C.c_float * 4),
        ("dI", f32p),
        ("frame_energy_th", f32p),
        ("precalc", f32p),
        ("ad_host", f64p),
        ("ad_target", f64p),
        ("c_prior", f64p),
        ("c_delta", f32p),
        ("frame_prior", f64p),
        ("frame_delta_prior", f64p),
        ("point_host", i32p),
        ("point_data", f32p),
        ("point_res_begin", i32p),
        ("res_target", i32p),
        ("res_state", i8p),
        ("res_energy", f32p),
        ("res_flags", u8p),
        ("point_rank", i32p),
    ]


def source_sha256() -> str | None:
    """sha256 over the sources libldso_ba.so is built from (ldso_amd/csrc, include/ldso_ba.h): the
    identity of a build that survives a rebuild on another machine (the .so bytes do not)."""
    import glob
    import hashlib

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = sorted(glob.glob(os.path.join(root, "ldso_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(root, "ldso_amd", "csrc", "*.h")) +
                   glob.glob(os.path.join(root, "ldso_amd", "csrc", "*.cpp")) +
                   [os.path.join(root, "ldso_amd", "csrc", "Makefile"), os.path.join(root, "include", "ldso_ba.h")])
    h = hashlib.sha256()
    try:
        for f in files:
            h.update(os.path.relpath(f, root).encode())
            with open(f, "rb") as fh:
                h.update(hashlib.sha256(fh.read()).digest())
    except OSError:
        return None
    return h.hexdigest()


def ptr(a, t):
    if a is None:
        return C.cast(None, t)
    assert a.flags["C_CONTIGUOUS"], "arrays handed to the C ABI must be C-contiguous"
    assert a.dtype == np.dtype(t._type_), f"array of {a.dtype} handed as {t.__name__}"
    return a.ctypes.data_as(t)


# (name, restype, argtypes) of every entry point declared in include/ldso_ba.h
ABI = [
    ("ldso_ba_abi_version", C.c_int, []),
    ("ldso_ba_last_error", C.c_char_p, []),
    ("ldso_ba_frame_precalc", C.c_int, [C.c_int32, C.c_void_p, f32p, f32p]),
    ("ldso_ba_set_adjoints", C.c_int, [C.c_int32, C.c_void_p, f64p, f64p, f64p]),
    ("ldso_ba_frame_take_data", C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, f64p, f64p, f64p]),
    ("ldso_ba_solve_system", C.c_int,
     [C.c_void_p, C.c_int32, C.c_int32, C.c_double, f64p, f64p, f64p, f64p, f64p, f64p, f64p, f64p, f64p, C.c_int32,
      f64p]),
    ("ldso_ba_nullspaces", C.c_int, [C.c_int32, C.c_void_p, f64p]),
    ("ldso_ba_validate_window", C.c_int, [C.POINTER(LdsoBaWindow)]),
    ("ldso_ba_create", C.c_int, [C.c_int32, C.POINTER(C.c_void_p)]),
    ("ldso_ba_destroy", None, [C.c_void_p]),
    ("ldso_ba_stream", C.c_void_p, [C.c_void_p]),
    ("ldso_ba_load", C.c_int, [C.c_void_p, C.c_int32, C.POINTER(LdsoBaWindow), C.c_int32, C.c_int32]),
    ("ldso_ba_update", C.c_int, [C.c_void_p, C.c_int32, C.POINTER(LdsoBaWindow)]),
    ("ldso_ba_reset_oob", C.c_int, [C.c_void_p, C.c_int32]),
    ("ldso_ba_update_points", C.c_int, [C.c_void_p, C.c_int32, f32p]),
    ("ldso_ba_update_residuals", C.c_int, [C.c_void_p, C.c_int32, i8p, f32p, f32p, u8p]),
    ("ldso_ba_linearize_residuals", C.c_int, [C.c_void_p, C.c_int32, i8p, f32p, f32p, f32p, u8p, f32p]),
    ("ldso_ba_linearize", C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    ("ldso_ba_sync", C.c_int, [C.c_void_p]),
    ("ldso_ba_get_energy", C.c_int, [C.c_void_p, C.c_int32, f64p]),
    ("ldso_ba_get_system", C.c_int, [C.c_void_p, C.c_int32, f64p, f64p, f64p, f64p, f64p, f64p]),
    ("ldso_ba_get_residuals", C.c_int, [C.c_void_p, C.c_int32, i8p, i8p, f32p, f32p, f32p, u8p, f32p, f32p]),
    ("ldso_ba_get_points", C.c_int, [C.c_void_p, C.c_int32, f32p, f32p, f32p, f32p, f32p, f32p]),
    ("ldso_ba_get_frame_energy_th", C.c_int, [C.c_void_p, C.c_int32, f32p]),
    ("ldso_ba_solve", C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_double, f64p, C.c_int32, f64p]),
    ("ldso_ba_resubstitute", C.c_int, [C.c_void_p, C.c_int32, f64p, C.c_double, f32p]),
    ("ldso_ba_solve_device", C.c_int, [C.c_void_p, C.c_int32, C.c_double, f64p, C.c_int32, f64p]),
    ("ldso_ba_resubstitute_device", C.c_int, [C.c_void_p, C.c_double, f32p]),
    ("ldso_ba_iterate", C.c_int, [C.c_void_p, C.c_int32, C.c_double, f64p, C.c_int32, f64p, f32p, f64p]),
    ("ldso_ba_packed_system", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), i64p, i64p]),
    ("ldso_ba_unpack_system", C.c_int, [C.c_void_p]),
    ("ldso_ba_copy_packed", C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32]),
    ("ldso_ba_newest_stride", C.c_int, [C.c_void_p, i64p]),
    ("ldso_ba_export_newest", C.c_int, [C.c_void_p, C.c_void_p, C.c_int64]),
    ("ldso_ba_frame_threshold_gathered", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int64]),
    ("ldso_ba_shard_points", C.c_int, [C.c_void_p, C.c_int32, C.c_int32, i32p, i32p]),
    ("ldso_ba_pack_upper", C.c_int, [C.c_int32, f64p, f64p, f64p, f64p, f64p]),
    ("ldso_ba_unpack_upper", C.c_int, [C.c_int32, f64p, f64p, f64p, f64p, f64p]),
    ("ldso_ba_frame_threshold", C.c_int, [f32p, C.c_int64, f32p]),
    ("ldso_ba_comm_unique_id", C.c_int, [C.c_void_p]),
    ("ldso_ba_comm_init", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32]),
    ("ldso_ba_check_settings", C.c_int, [C.c_void_p]),
    ("ldso_ba_default_settings", None, [C.c_void_p]),
    ("ldso_ba_set_settings", C.c_int, [C.c_void_p, C.c_void_p]),
    ("ldso_ba_get_settings", C.c_int, [C.c_void_p, C.c_void_p]),
    ("ldso_ba_optimize", C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, f64p, f64p, f64p, f64p, C.c_void_p,
                                   f64p, f32p, i32p, i32p]),
    ("ldso_ba_frame_step", C.c_int, [C.c_int32, C.c_void_p, f64p, C.c_void_p, f64p, f64p, f32p, f32p]),
    ("ldso_ba_step_canbreak", C.c_int, [C.c_int32, f64p, C.c_float, C.c_float, C.c_float, i32p]),
    ("ldso_ba_set_kernel_timing", C.c_int, [C.c_void_p, C.c_int32]),
    ("ldso_ba_set_tuning", C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    ("ldso_ba_get_kernel_times", C.c_int, [C.c_void_p, f64p, i64p, C.c_int32]),
    ("ldso_ba_kernel_name", C.c_char_p, [C.c_int32]),
    ("ldso_ba_num_kernels", C.c_int32, []),
    ("ldso_ba_stats", C.c_int, [C.c_void_p, i64p, i64p, i64p]),
    ("ldso_ba_marginalize_frame", C.c_int, [C.c_int32, C.c_int32, f64p, f64p, f64p, f64p, f64p, f64p]),
    ("ldso_ba_ad_ht_delta", C.c_int, [C.c_int32, f64p, f64p, f64p, f32p]),
    ("ldso_ba_calc_m_energy", C.c_int, [C.c_int32, f64p, f64p, f32p, f64p, f64p]),
    ("ldso_ba_calc_l_energy", C.c_int, [C.c_int32, f64p, f64p, f64p, f32p, C.c_int32, f32p, f32p, f64p]),
    ("ldso_ba_load_marginalization", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(LdsoBaWindow)]),
    ("ldso_ba_marginalize_points", C.c_int, [C.c_void_p, f32p, f64p, f64p]),
    ("ldso_ba_activate_points", C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]),
]

f32pp = C.POINTER(f32p)

# ldso_ct_immature (include/ldso_ct.h): one ImmaturePoint, 128 bytes
IMMATURE_DTYPE = np.dtype([("u", "<f4"), ("v", "<f4"), ("idepth_min", "<f4"), ("idepth_max", "<f4"),
                           ("quality", "<f4"), ("energy_th", "<f4"), ("color", "<f4", (8,)),
                           ("weights", "<f4", (8,)), ("grad_h", "<f4", (4,)), ("host", "<i4"),
                           ("last_status", "<i4"), ("last_uv", "<f4", (2,)), ("last_interval", "<f4"),
                           ("type", "<f4")])
assert IMMATURE_DTYPE.itemsize == 128
# ldso_ba_activation (include/ldso_ba.h)
ACTIVATION_DTYPE = np.dtype([("idepth", "<f4"), ("status", "<i4"), ("in_mask", "<u4"), ("energy", "<f4")])
IPS_NAMES = ("GOOD", "OOB", "OUTLIER", "SKIPPED", "BADCONDITION", "UNINITIALIZED")  # ImmaturePoint.h:31-38

# (name, restype, argtypes) of every entry point declared in include/ldso_ct.h (coarse tracker)
CT_ABI = [
    ("ldso_ct_create", C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p), i32p]),
    ("ldso_ct_destroy", None, [C.c_void_p]),
    ("ldso_ct_make_k", C.c_int, [C.c_void_p, f32p, f32p]),
    ("ldso_ct_set_new_frame", C.c_int, [C.c_void_p, f32p, C.c_double, f32p]),
    ("ldso_ct_get_frame_level", C.c_int, [C.c_void_p, C.c_int32, f32p, f32p]),
    ("ldso_ct_set_reference", C.c_int,
     [C.c_void_p, i32p, f32pp, f32pp, f32pp, f32pp, C.c_double, C.c_double, C.c_double]),
    ("ldso_ct_calc_res", C.c_int, [C.c_void_p, C.c_int32, f64p, C.c_double, C.c_double, C.c_float, f64p]),
    ("ldso_ct_calc_res_batch", C.c_int, [C.c_void_p, C.c_int32, C.c_int32, f64p, f64p, C.c_float, f64p]),
    ("ldso_ct_calc_gs", C.c_int, [C.c_void_p, C.c_int32, f64p, C.c_double, C.c_double, f64p, f64p]),
    ("ldso_ct_calc_res_gs", C.c_int,
     [C.c_void_p, C.c_int32, f64p, C.c_double, C.c_double, C.c_float, f64p, f64p, f64p]),
    ("ldso_ct_get_warped", C.c_int, [C.c_void_p, i32p, f32p, C.c_int32]),
    ("ldso_ct_make_immature", C.c_int, [C.c_void_p, C.c_int32, f32p, C.c_float, C.c_int32, C.c_void_p]),
    ("ldso_ct_immature_upload", C.c_int, [C.c_void_p, C.c_int32, C.c_void_p]),
    ("ldso_ct_immature_download", C.c_int, [C.c_void_p, C.c_int32, C.c_void_p]),
    ("ldso_ct_trace", C.c_int, [C.c_void_p, C.c_int32, f32p, f32p, f32p, i32p]),
    ("ldso_ct_set_kernel_timing", C.c_int, [C.c_void_p, C.c_int32]),
    ("ldso_ct_get_kernel_times", C.c_int, [C.c_void_p, f64p, i64p, C.c_int32]),
    ("ldso_ct_kernel_name", C.c_char_p, [C.c_int32]),
    ("ldso_ct_num_kernels", C.c_int32, []),
]

_lib = None
_synth = None


def lib():
    """The product library.  Raises if it has not been built (no fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(make -C ldso_amd/csrc). The HIP path has no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        for name, res, args in ABI + CT_ABI:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.ldso_ba_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{LIB_PATH} has ABI {L.ldso_ba_abi_version()}, these bindings expect {ABI_VERSION}: "
                               "rebuild it (make -C ldso_amd/csrc)")
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise RuntimeError(f"ldso_ba error {rc}: {lib().ldso_ba_last_error().decode()}")
    return rc


def synth_lib():
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_PATH):
            raise RuntimeError(f"{SYNTH_PATH} missing: run make -C ldso_amd/csrc")
        S = C.CDLL(SYNTH_PATH)
        S.ldso_synth_fill.restype = C.c_int
        S.ldso_synth_fill.argtypes = [C.c_void_p, C.c_void_p, f32p, f32p, f32p, i32p, f32p, i32p, i32p, i8p, f32p, u8p]
        _synth = S
    return _synth
