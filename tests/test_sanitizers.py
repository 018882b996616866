"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md section 5:
"build tests under -fsanitize=address,undefined for the CPU restatement"). GPU sanitizers
are not available on the pool; the kernels are covered by the parity suite instead.

tests/asan/asan_driver.c links the oracle and libbhrt's host C sources (device launchers
stubbed) and exercises frames of every configuration, edge rays, recorded paths, particle
creation/update, the context API, the no-GPU error paths and the spacetime helpers."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "raytracing-engine-in-c_amd", "csrc")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "asan_driver")
    srcs = [os.path.join(ROOT, "tests", "asan", "asan_driver.c"),
            os.path.join(ROOT, "oracle", "oracle.c"),
            os.path.join(CSRC, "bhrt_api.c"), os.path.join(CSRC, "particles.c"),
            os.path.join(CSRC, "kerr_helpers.c")]
    cmd = ["gcc", "-std=gnu11", "-O1", "-g", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-ffp-contract=off",
           "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include", "-I", os.path.join(ROOT, "include"),
           "-I", CSRC, "-I", os.path.join(ROOT, "oracle"), *srcs, "-L", "/opt/rocm/lib",
           "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-lm", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1", HIP_VISIBLE_DEVICES="-1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
