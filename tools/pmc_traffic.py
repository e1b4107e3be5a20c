"""Collect HBM traffic of k_linearize with rocprofv3 PMC counters (separate passes, as
MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes) and write
profiles/pmc_k_linearize.json.

  python tools/pmc_traffic.py [--windows 64] [--out gpurun_out/pmc]

FETCH_SIZE and WRITE_SIZE are in KiB (TCC_EA0_RDREQ/WRREQ x 64 B).  On gfx950 FETCH_SIZE
reads 1/2 of the bytes of a wide coalesced 16-B/lane stream; k_linearize's texel reads are
16-B/lane but scattered: tools/gather_probe_pieces.hip (profiles/r6/fetch_probe) calibrates exactly
that pattern -- 1, 2, 4 or 8 16-B pieces of random 128-B lines of a 1-GiB buffer -- and finds one
TCC_EA0_RDREQ per touched line and FETCH_SIZE exactly half of the whole-line bytes in every case
(the HBM delivers whole lines), so the x2-corrected read figure is the traffic; both are recorded."""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_sha256():
    sys.path.insert(0, ROOT)
    from ldso_amd import _lib

    return _lib.source_sha256()


def lib_sha256(path=os.path.join(ROOT, "ldso_amd", "lib", "libldso_ba.so")):
    import hashlib

    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def run_pass(counters, outdir, args):
    os.makedirs(outdir, exist_ok=True)
    cmd = ["rocprofv3", "--pmc"] + counters + ["--kernel-include-regex", "k_linearize", "-d", outdir, "-o", "run",
                                               "--output-format", "csv", "--", sys.executable,
                                               os.path.join(ROOT, "tools", "pmc_driver.py"), "--windows",
                                               str(args.windows), "--steps", str(args.steps)]
    env = dict(os.environ, TMPDIR="/tmp")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    if p.returncode != 0:
        sys.stderr.write(p.stdout[-3000:] + p.stderr[-3000:])
        raise SystemExit(f"rocprofv3 failed ({p.returncode})")
    n_gather = None
    for line in p.stdout.splitlines():
        if line.startswith("n_gather="):
            n_gather = int(line.split()[0].split("=")[1])
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if "k_linearize" not in row.get("Kernel_Name", ""):
                continue
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return vals, n_gather


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    ap.add_argument("--session", default=os.environ.get("LDSO_PMC_SESSION", ""),
                    help="the measurement session's name, recorded with the result (provenance)")
    args = ap.parse_args()
    res = {}
    n_gather = None
    for i, ctrs in enumerate([["FETCH_SIZE"], ["WRITE_SIZE"], ["TCC_HIT_sum", "TCC_MISS_sum"],
                              ["TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "TCP_PENDING_STALL_CYCLES_sum"]]):
        vals, ng = run_pass(ctrs, os.path.join(args.out, f"pass{i}"), args)
        n_gather = n_gather or ng
        for k, v in vals.items():
            steady = v[1:] if len(v) > 1 else v  # drop the first (cold) launch
            res[k] = sum(steady) / len(steady)
    fetch_kib = res.get("FETCH_SIZE", 0.0)
    write_kib = res.get("WRITE_SIZE", 0.0)
    B = args.windows
    out = {
        "workload": f"{B} x S7 synthetic windows/GPU (7 KF, 2000 pts, 640x480)",
        "kernel": "k_linearize",
        "launches_averaged": args.steps - 1,
        "n_gather_residuals": n_gather,
        "FETCH_SIZE_KiB_per_launch": fetch_kib,
        "WRITE_SIZE_KiB_per_launch": write_kib,
        "read_bytes_raw": fetch_kib * 1024,
        "read_bytes_corrected_x2": 2 * fetch_kib * 1024,
        "write_bytes": write_kib * 1024,
        "hbm_bytes_per_launch": 2 * fetch_kib * 1024 + write_kib * 1024,
        "hbm_bytes_per_gather_residual": (2 * fetch_kib * 1024 + write_kib * 1024) / n_gather if n_gather else None,
        "TCC_hit_rate": res["TCC_HIT_sum"] / (res["TCC_HIT_sum"] + res["TCC_MISS_sum"])
        if res.get("TCC_HIT_sum") is not None else None,
        "TCP_accesses_per_gather_residual": res["TCP_TOTAL_CACHE_ACCESSES_sum"] / n_gather
        if n_gather and res.get("TCP_TOTAL_CACHE_ACCESSES_sum") is not None else None,
        "TCP_TCC_read_requests_per_gather_residual": res["TCP_TCC_READ_REQ_sum"] / n_gather
        if n_gather and res.get("TCP_TCC_READ_REQ_sum") is not None else None,
        "counters": res,
        # provenance: the session that measured it and the exact library build it measured (bench.py
        # reports whether its own build is the same one)
        "session": args.session,
        "lib_sha256": lib_sha256(),
        "source_sha256": source_sha256(),
    }
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "pmc_k_linearize.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
