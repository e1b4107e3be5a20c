"""C-ABI boundary checks that need no GPU: the library loads, exports every entry point that
include/ldso_ba.h declares, the host-side helpers (precalc, adjoints, priors, nullspaces,
solve) agree with the oracle's independent restatement, and errors follow the reference's
convention (negative status + message, never a crash)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
from ldso_amd import _lib as L
from ldso_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ldso_ba.h")
CT_HEADER = os.path.join(ROOT, "include", "ldso_ct.h")


def declared_symbols(header=HEADER, prefix="ldso_ba_"):
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(" + prefix + r"[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol(built):
    syms = declared_symbols()
    assert len(syms) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (ldso_ba_\w+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    bound = {name for name, _, _ in L.ABI}
    assert set(syms) == bound, set(syms) ^ bound
    lib = L.lib()
    assert lib.ldso_ba_abi_version() == L.ABI_VERSION == 6
    assert lib.ldso_ba_num_kernels() >= 3


def test_library_exports_every_tracker_symbol(built):
    syms = declared_symbols(CT_HEADER, "ldso_ct_")
    assert len(syms) >= 14
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (ldso_ct_\w+)", out))
    assert not [s for s in syms if s not in exported]
    assert set(syms) == {name for name, _, _ in L.CT_ABI}
    lib = L.lib()
    assert lib.ldso_ct_num_kernels() == 7 and lib.ldso_ct_kernel_name(2) == b"k_ct_calc_res"
    assert lib.ldso_ct_kernel_name(5) == b"k_ct_trace"
    h = C.c_void_p()
    assert lib.ldso_ct_create(0, 4, 4, C.byref(h), None) < 0 and b"small" in lib.ldso_ba_last_error()


def test_library_is_gfx950_only(built, tmp_path):
    import shutil

    lib = tmp_path / "libldso_ba.so"  # objdump --offloading extracts bundles next to its input
    shutil.copy(L.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)], capture_output=True,
                         text=True, cwd=tmp_path).stdout
    out += subprocess.run(["strings", L.LIB_PATH], capture_output=True, text=True).stdout
    assert "gfx950" in out
    assert not re.search(r"gfx9[0-4]\d\b|gfx1[01]\d\d", out.replace("gfx950", ""))


@pytest.mark.parametrize("cfg", [dict(n_frames=3, n_points=40, width=160, height=120, seed=5),
                                 dict(n_frames=7, n_points=100, width=320, height=240, seed=9)])
def test_host_helpers_match_oracle(built, cfg):
    w = synth.make_window(**cfg)
    ref = oracle.frame_terms(w)
    np.testing.assert_array_equal(w.precalc, ref["precalc"])
    np.testing.assert_allclose(w.ad_host, ref["ad_host"], rtol=0, atol=1e-12 * np.abs(ref["ad_host"]).max())
    np.testing.assert_allclose(w.ad_target, ref["ad_target"], rtol=0, atol=0)
    np.testing.assert_array_equal(w.c_prior, ref["c_prior"])
    np.testing.assert_array_equal(w.frame_prior, ref["frame_prior"])
    np.testing.assert_allclose(w.frame_delta, ref["frame_delta"], rtol=0, atol=1e-15)
    np.testing.assert_allclose(w.frame_delta_prior, ref["frame_delta_prior"], rtol=0, atol=1e-15)
    np.testing.assert_allclose(w.nullspaces(), ref["nullspaces"], rtol=0, atol=1e-9)


def test_solver_matches_oracle_solver(built):
    w = synth.make_window(n_frames=5, n_points=200, width=320, height=240, seed=3)
    ow = oracle.OracleWindow(w, threads=0)
    _, sysm = ow.iteration()
    ns = w.nullspaces()
    lib = L.lib()
    n = w.dim
    for it in (0, 3):
        x = np.zeros(n)
        args = [L.ptr(np.ascontiguousarray(sysm[k]), L.f64p) for k in ("HA", "bA", "HL", "bL")]
        rc = lib.ldso_ba_solve_system(None, w.n_frames, it, 1e-5, *args, L.ptr(None, L.f64p), L.ptr(None, L.f64p),
                                      L.ptr(np.ascontiguousarray(sysm["Hsc"]), L.f64p),
                                      L.ptr(np.ascontiguousarray(sysm["bsc"]), L.f64p), L.ptr(ns, L.f64p), 7,
                                      L.ptr(x, L.f64p))
        assert rc == 0
        xo = oracle.solve_system(w.n_frames, it, 1e-5, sysm, nullspaces=ns)
        assert np.linalg.norm(x - xo) <= 1e-9 * np.linalg.norm(xo)
    if True:  # orthogonalize(): x is orthogonal to the (normalised) gauge directions at it >= 2
        xo = oracle.solve_system(w.n_frames, 2, 1e-5, sysm, nullspaces=ns)
        Nn = ns / np.linalg.norm(ns, axis=1, keepdims=True)
        assert np.abs(Nn @ xo).max() <= 1e-9 * np.linalg.norm(xo)


def test_error_convention(built):
    lib = L.lib()
    assert lib.ldso_ba_frame_precalc(0, None, None, None) < 0
    assert b"bad arguments" in lib.ldso_ba_last_error()
    assert lib.ldso_ba_validate_window(None) < 0
    w = synth.make_window(n_frames=3, n_points=10, width=160, height=120, seed=1)
    s = w.c_struct()
    assert lib.ldso_ba_validate_window(C.byref(s)) == 0
    bad = w.copy_state()
    bad.res_target = w.res_target.copy()
    bad.res_target[0] = bad.point_host[0]  # a residual onto its own host
    sb = bad.c_struct()
    assert lib.ldso_ba_validate_window(C.byref(sb)) < 0
    assert b"host" in lib.ldso_ba_last_error()
    bad2 = w.copy_state()
    bad2.point_host = w.point_host.copy()
    bad2.point_host[1] = 7  # frame index out of range
    sb2 = bad2.c_struct()
    assert lib.ldso_ba_validate_window(C.byref(sb2)) < 0
    bad3 = w.copy_state()
    bad3.res_target = w.res_target.copy()
    b0, b1 = w.point_res_begin[0], w.point_res_begin[1]
    if b1 - b0 >= 2:
        bad3.res_target[b0 + 1] = bad3.res_target[b0]  # duplicate (point, target)
        sb3 = bad3.c_struct()
        assert lib.ldso_ba_validate_window(C.byref(sb3)) < 0
    h = C.c_void_p()
    rc = lib.ldso_ba_create(1 << 20, C.byref(h))  # no such device: error, not a crash
    assert rc < 0 and not h.value


def test_synthetic_generator_is_deterministic(built):
    a = synth.make_window(n_frames=4, n_points=50, width=160, height=120, seed=17)
    b = synth.make_window(n_frames=4, n_points=50, width=160, height=120, seed=17)
    c = synth.make_window(n_frames=4, n_points=50, width=160, height=120, seed=18)
    for k in ("dI", "point_data", "point_host", "res_target", "precalc"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k))
    assert not np.array_equal(a.dI, c.dI)
    # FrameHessian::makeImages gradients (FrameHessian.cc:96-105) hold on the generated images
    I = a.dI[0, :, 0].reshape(120, 160)
    gx = 0.5 * (np.roll(I.ravel(), -1) - np.roll(I.ravel(), 1)).reshape(120, 160).astype(np.float32)
    np.testing.assert_array_equal(a.dI[0, 160:160 * 119, 1], gx.ravel()[160:160 * 119])
    assert (a.point_res_begin[1:] - a.point_res_begin[:-1] == 3).all()


def test_product_solver_known_answer(built):
    """ldso_ba_solve_system on an SPD system that needs pivoting equals numpy's solve."""
    rng = np.random.default_rng(7)
    N = 4
    n = 8 * N + 4
    A = rng.standard_normal((n, n))
    D = np.diag(10.0 ** rng.uniform(-3, 6, n))
    H = np.ascontiguousarray(D @ (A @ A.T + n * np.eye(n)) @ D)
    b = rng.standard_normal(n)
    Z = np.zeros((n, n))
    z = np.zeros(n)
    x = np.zeros(n)
    lib = L.lib()
    rc = lib.ldso_ba_solve_system(None, N, 0, 1e-5, L.ptr(H, L.f64p), L.ptr(b, L.f64p), L.ptr(Z, L.f64p), L.ptr(z, L.f64p),
                                  L.ptr(None, L.f64p), L.ptr(None, L.f64p), L.ptr(Z, L.f64p), L.ptr(z, L.f64p),
                                  L.ptr(None, L.f64p), 0, L.ptr(x, L.f64p))
    assert rc == 0
    Hl = H.copy()
    Hl[np.diag_indices(n)] *= 1 + 1e-5
    xr = np.linalg.solve(Hl, b)
    assert np.linalg.norm(x - xr) <= 1e-9 * np.linalg.norm(xr)


@pytest.mark.parametrize("degenerate", [False, True])
def test_product_solver_projection_known_answer(built, degenerate):
    """Iteration >= 2 projects the step out of the nullspace span (EnergyFunctional::orthogonalize):
    x = (I - N N^+) x0.  Well-conditioned nullspaces take the Cholesky path; a rank-deficient set
    (two equal columns) takes the Jacobi path, whose cut drops the zero singular value."""
    rng = np.random.default_rng(8)
    N = 3
    n = 8 * N + 4
    A = rng.standard_normal((n, n))
    H = np.ascontiguousarray(A @ A.T + n * np.eye(n))
    b = rng.standard_normal(n)
    ns = rng.standard_normal((7, n))
    if degenerate:
        ns[6] = ns[5]
    ns = np.ascontiguousarray(ns)
    Z, z = np.zeros((n, n)), np.zeros(n)
    x0, x2 = np.zeros(n), np.zeros(n)
    lib = L.lib()
    for it, x in ((0, x0), (2, x2)):
        rc = lib.ldso_ba_solve_system(None, N, it, 1e-5, L.ptr(H, L.f64p), L.ptr(b, L.f64p), L.ptr(Z, L.f64p),
                                      L.ptr(z, L.f64p), L.ptr(None, L.f64p), L.ptr(None, L.f64p), L.ptr(Z, L.f64p),
                                      L.ptr(z, L.f64p), L.ptr(ns, L.f64p), 7, L.ptr(x, L.f64p))
        assert rc == 0
    Nm = (ns / np.linalg.norm(ns, axis=1, keepdims=True)).T
    xr = x0 - Nm @ (np.linalg.pinv(Nm, rcond=1e-10) @ x0)
    assert np.linalg.norm(x2 - xr) <= 1e-9 * np.linalg.norm(x0)
    assert np.abs(Nm.T @ x2).max() <= 1e-9 * np.linalg.norm(x0)


def test_precalc_current_pose_rotation_known_answer(built):
    """FrameFramePrecalc::Set (FrameFramePrecalc.cc:12-19): PRE_RTll / PRE_tTll (record slots
    27..38) come from the CURRENT poses PRE_worldToCam = exp(scaled state) * evalPT, while
    PRE_RTll_0 / PRE_tTll_0 (slots 12..23) come from the evaluation points.  A non-newest frame
    is moved away from its state_zero and the record is checked against the relative poses
    rebuilt here in numpy (ImmaturePoint::linearizeResidual reads slots 27..38)."""
    from ldso_amd.synth import se3_matrix

    w = synth.make_window(n_frames=5, n_points=50, width=160, height=120, seed=4)
    fr = w.frames
    fr["state"][2, :6] = [0.02, -0.01, 0.03, 0.004, -0.006, 0.002]  # frame 2 is not the newest
    w.refresh_frame_terms()
    N = w.n_frames

    def pose(f, current):
        T = np.eye(4)
        T[:3, :3] = fr["world_to_cam_evalpt"][f][:9].reshape(3, 3)
        T[:3, 3] = fr["world_to_cam_evalpt"][f][9:]
        if current:
            s = fr["state"][f]
            E = np.eye(4)
            E[:3] = se3_matrix(s[3:6] * 1.0, s[0:3] * 0.5)  # SCALE_XI_ROT = 1, SCALE_XI_TRANS = 0.5
            T = E @ T
        return T

    for h in range(N):
        for t in range(N):
            rec = w.precalc[h + N * t]
            for current, (ro, to) in ((True, (27, 36)), (False, (12, 21))):
                L2L = pose(t, current) @ np.linalg.inv(pose(h, current))
                np.testing.assert_allclose(rec[ro:ro + 9], L2L[:3, :3].ravel(), rtol=0, atol=1e-6)
                np.testing.assert_allclose(rec[to:to + 3], L2L[:3, 3], rtol=0, atol=1e-6)
    # the moved frame's pairs differ between the two pose sets, frame 0 <-> 1 (both at their
    # evaluation points) does not
    assert not np.array_equal(w.precalc[2 + N * 0][27:36], w.precalc[2 + N * 0][12:21])
    np.testing.assert_array_equal(w.precalc[0 + N * 1][27:39], w.precalc[0 + N * 1][12:24])
