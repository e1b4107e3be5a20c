"""Randomised solve sweep (solveSystemF / resubstituteF_MT on the device):
seeded batches of one to six windows (2-11 keyframes, 20-900 points, the fuzz frame sizes, camera
models, motions and baselines), a random damping lambda, iteration (0-1: no projection; >= 2:
nullspace projection) and count of projected nullspace rows (5-7, rank-deficient sets included).
The exact mode (LDSO_BA_TUNE_SOLVE_EXACT: k_solve_reg, or k_solve when the batch holds a window
above 7 keyframes) equals the host solver bit for bit; the default k_solve_fast is within 20x
the system's float-rounding envelope of it (tests/test_gpu_parity.py's bar, 1e-9 relative at
worst); both resubstitutions equal the host-staged one from the same x."""
import numpy as np
import pytest

import oracle
from ldso_amd import synth

pytestmark = pytest.mark.gpu

SIZES = [(160, 120), (317, 203), (640, 480), (1242, 375)]


def envelope(N, it, lam, sysm, ns, x0, eps=2.0 ** -20, trials=3):
    """largest |x' - x0| / |x0| over solves of the system with entries scaled by 1 + eps N(0, 1)"""
    rng = np.random.default_rng(0)
    worst = 0.0
    for _ in range(trials):
        pert = dict(sysm)
        for k in ("HA", "Hsc"):
            E = rng.standard_normal(sysm[k].shape)
            pert[k] = sysm[k] * (1 + eps * (E + E.T) / 2)
        for k in ("bA", "bsc"):
            pert[k] = sysm[k] * (1 + eps * rng.standard_normal(sysm[k].shape))
        x = oracle.solve_system(N, it, lam, pert, nullspaces=ns)
        worst = max(worst, np.linalg.norm(x - x0) / np.linalg.norm(x0))
    return worst


@pytest.mark.parametrize("case", range(12))
def test_random_device_solve_matches_host(built, case):
    from ldso_amd import BAContext

    rng = np.random.default_rng(19000 + case)
    W, H = SIZES[rng.integers(len(SIZES))]
    cfgs = [dict(n_frames=int(rng.integers(2, 12)), n_points=int(rng.integers(20, 900)), width=W, height=H,
                 seed=int(rng.integers(1 << 30)), motion=str(rng.choice(["sideways", "forward"])),
                 baseline=float(rng.choice([0.04, 0.2])), outlier_frac=float(rng.uniform(0, 0.2)))
            for _ in range(int(rng.integers(1, 7)))]
    lam = float(rng.choice([1e-5, 1e-3, 1e-1]))
    it = int(rng.choice([0, 1, 2, 5]))
    n_null = int(rng.choice([5, 6, 7]))
    deficient = bool(rng.random() < 0.3)
    print(f"case {case}: lambda {lam}, iteration {it}, n_null {n_null}, rank-deficient {deficient}")
    for c in cfgs:
        print("  ", c)
    ws = [synth.make_window(**c) for c in cfgs]
    ns = [w.nullspaces() for w in ws]
    if deficient:
        for a in ns:
            a[n_null - 1] = a[n_null - 2]
    for exact in (1, 0):
        ctx = BAContext(0)
        ctx.set_tuning(12, exact)  # LDSO_BA_TUNE_SOLVE_EXACT
        ctx.load(ws)
        ctx.linearize()
        xd = ctx.solve_device(it, lam, ns, n_null=n_null)
        for i, w in enumerate(ws):
            xh = ctx.solve(i, it, lam, ns[i][:n_null])
            if exact:
                np.testing.assert_array_equal(xd[i], xh, err_msg=f"window {i}")
            else:
                env = envelope(w.n_frames, it, lam, ctx.system(i), ns[i][:n_null], xh)
                rel = np.linalg.norm(xd[i] - xh) / np.linalg.norm(xh)
                print(f"  window {i} (N={w.n_frames}): fast {rel:.3e}, envelope {env:.3e}")
                assert rel <= max(1e-12, min(1e-9, 20 * env)), i
        sd = ctx.resubstitute_device(lam)
        for i in range(len(ws)):
            np.testing.assert_array_equal(sd[i], ctx.resubstitute(i, xd[i], lam), err_msg=f"window {i}")
        ctx.close()
