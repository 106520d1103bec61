"""The plan compiler (csrc/schedule.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer.

Host-only: builds tests/c/plan_sanitize.cpp with schedule.cpp (g++, no GPU) and
builds, checks and serialises every rank's plan for every ordered factorization
of P = 2..14 with 0..3 lonely ranks and the ring, sizes 0/1/P-1/ragged/2^20,
all four data-movement forms; malformed topologies must be rejected.  Any
memory error or UB aborts the binary (-fno-sanitize-recover=all).
"""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_plan_compiler_is_clean_under_asan_ubsan(tmp_path):
    exe = tmp_path / "plan_sanitize"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "allreduce-over-mpi_amd", "csrc"), "-I", "/opt/rocm/include",
           os.path.join(ROOT, "tests", "c", "plan_sanitize.cpp"),
           os.path.join(ROOT, "allreduce-over-mpi_amd", "csrc", "schedule.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    r = subprocess.run([str(exe), "14"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    stats = json.loads(r.stdout.strip().splitlines()[-1])
    assert stats["plans"] > 10_000 and stats["worlds"] > 500
