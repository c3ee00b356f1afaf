"""The variable-length record walk's fast path (walk program, ngz_internal.h)
agrees with the exact per-field walk on random records, truncations and
corruptions: same records, offsets and error keys (host build of the same
__host__ __device__ code the framing kernel runs)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fast_walk_matches_exact_walk(tmp_path):
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    exe = str(tmp_path / "vlen_walk_check")
    subprocess.check_call(["hipcc", "-O2", "-std=c++17", "-I" + os.path.join(HERE, "..", "include"),
                           os.path.join(HERE, "native", "vlen_walk_check.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout
    errors = int(out.stdout.split("errors ")[1].split()[0])
    assert errors > 500  # the error paths are exercised
