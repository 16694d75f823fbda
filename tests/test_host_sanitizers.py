"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU).

GPU sanitizers are not available on the MI355X pool; the host-side launch planning of the HIP
wrappers (csrc/kernels/host_plan.h: the weight-gradient split-K planner, the reduction slicer)
is plain C++ and is built here with ``-fsanitize=address,undefined -fno-sanitize-recover=all``
and exercised on the production shapes and degenerate inputs (any sanitizer report fails)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs a host C++ compiler")
def test_host_plan_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_plan_test"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "csrc", "kernels"),
           os.path.join(ROOT, "tests", "native", "host_plan_test.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert run.returncode == 0, run.stdout + run.stderr
    assert "host_plan_test: ok" in run.stdout
    assert "runtime error" not in run.stderr and "AddressSanitizer" not in run.stderr
