"""SURVEY §5 sanitizers row: the C ABI's host code (plan creation, flat parameter
layout, workspace sizing, saved-tensor lookups, rejection of malformed configs) under
AddressSanitizer + UndefinedBehaviorSanitizer on the CPU, for every BASELINE.json
shape (scripts/asan_build.sh builds the host half of every HIP translation unit with
-Xarch_host -fsanitize=address,undefined and links scripts/asan_plans.cpp; no GPU
call is made).  Skipped where the ROCm toolchain is absent."""
import os
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.timeout(900)
def test_abi_host_code_is_asan_ubsan_clean():
    if not (os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("hipcc")):
        pytest.skip("hipcc not available")
    r = subprocess.run(["bash", str(ROOT / "scripts" / "asan_build.sh"), "--run"],
                       capture_output=True, text=True, timeout=850)
    out = r.stdout + r.stderr
    print(out[-3000:])
    assert r.returncode == 0, out[-4000:]
    assert "asan_plans: ok" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out
    assert "ERROR: LeakSanitizer" not in out
