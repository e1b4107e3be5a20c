"""bench.py --gpus N without a launcher starts its own N ranks: one fresh child
process per GPU before any GPU call, torchrun's environment (RANK, LOCAL_RANK, WORLD_SIZE,
MASTER_ADDR/PORT), rank 0's JSON line forwarded, a failing rank failing the run.  Under a
launcher --gpus must equal WORLD_SIZE.  CPU only: the children here are small Python programs
(and, last, bench.py itself, whose ranks fail without a GPU)."""
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_world_from_env():
    assert bench.world_from_env(1, {}) == (1, False)
    assert bench.world_from_env(4, {}) == (1, False)  # no launcher: bench.py launches the 4 ranks itself
    assert bench.world_from_env(2, {"WORLD_SIZE": "2"}) == (2, True)
    with pytest.raises(SystemExit, match="--gpus 8 but WORLD_SIZE=2"):
        bench.world_from_env(8, {"WORLD_SIZE": "2"})


CHILD = ("import json, os, sys; r = int(os.environ['RANK']); "
         "print(json.dumps({k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', "
         "'MASTER_PORT')}), flush=True); sys.exit(int(os.environ.get('FAIL_RANK_' + str(r), '0')))")


def run_launcher(n, env_extra=None, child=CHILD):
    """launch_ranks in a fresh interpreter so that its stdout can be captured."""
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(%d, [sys.executable, '-c', %r]))" % (ROOT, n, child))
    env = dict(os.environ, **(env_extra or {}))
    t = time.time()
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    return p, time.time() - t


def test_launch_ranks_environment_and_forwarding():
    import json

    p, _ = run_launcher(3)
    assert p.returncode == 0, p.stderr
    lines = [json.loads(l) for l in p.stdout.strip().splitlines()]
    assert len(lines) == 1  # only rank 0's stdout reaches the caller
    d = lines[0]
    assert d["RANK"] == d["LOCAL_RANK"] == "0" and d["WORLD_SIZE"] == "3" and d["MASTER_ADDR"] == "127.0.0.1"
    assert 1024 <= int(d["MASTER_PORT"]) < 65536
    others = [json.loads(l) for l in p.stderr.strip().splitlines() if l.startswith("{")]
    assert sorted(o["RANK"] for o in others) == ["1", "2"]
    assert all(o["LOCAL_RANK"] == o["RANK"] and o["MASTER_PORT"] == d["MASTER_PORT"] for o in others)


def test_launch_ranks_failure_stops_the_others():
    hang = ("import os, sys, time; r = int(os.environ['RANK']); "
            "sys.exit(5) if r == 1 else time.sleep(600)")
    p, dt = run_launcher(3, child=hang)
    assert p.returncode == 5
    assert dt < 60  # the sleeping ranks were stopped, not waited for


def test_bench_gpus2_without_launcher_fails_loudly_without_gpu():
    """The real entry: `python bench.py --gpus 2` starts two ranks of itself; on this GPU-less
    host they fail at the first device call, and so does the run (non-zero, promptly)."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    t = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--windows", "1", "--no-cpu", "--no-tracker", "--no-secondary"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert p.returncode != 0
    assert p.stdout.strip() == ""
    assert time.time() - t < 240
