"""ASan + UBSan build of the engine's host code (band planner: band_plan.cpp; TSV writer: tsv_format.cpp), run
on CPU: tests/native/plan_tsv_check.cpp drives both on random and edge-case inputs and checks them against
brute-force restatements (see its header)."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

CSRC = os.path.join(REPO, "nldsc_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", CSRC, "sanitize"], check=True, capture_output=True, timeout=600)
    exe = os.path.join(CSRC, "build", "plan_tsv_check_asan")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "plan_tsv_check OK" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
