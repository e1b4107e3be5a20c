"""The C++ host face (include/ldso_amd/energy_functional.h: the EnergyFunctional.h:55-186 surface
with shared_ptr ownership, PointFrameResidual / FrameHessian / PointHessian / CalibHessian)
exercised by its own C++ test program, tests/cpp/test_energy_functional.cpp: a whole keyframe
cycle (insert, optimize x3, flag + marginalizePointsF, dropPointsF, marginalizeFrame, optimize x2
with HM / bM) against the oracle on the same inputs."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_energy_functional")


def run(*args):
    p = subprocess.run([BIN, *args], capture_output=True, text=True, timeout=600)
    print(p.stdout[-4000:], p.stderr[-2000:])
    return p


def test_cpp_host_structure_and_errors(built):
    p = run("--cpu")
    assert p.returncode == 0 and "0 failure(s)" in p.stdout


@pytest.mark.gpu
def test_cpp_host_keyframe_cycle_matches_oracle(built):
    p = run()
    assert p.returncode == 0 and "0 failure(s)" in p.stdout
