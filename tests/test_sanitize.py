"""The host library sources and the oracle under AddressSanitizer + UndefinedBehaviorSanitizer
(`make sanitize`, tools/sanitize/main.cpp): scene builds, both integrators over the Cornell box
and a scene with every texture kind, and the PNG / HDR / OBJ / MTL readers on truncated,
bit-flipped and mangled input.  Any sanitizer report aborts the driver.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _have_asan():
    if not shutil.which("g++"):
        return False
    r = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True)
    return r.returncode == 0 and os.path.isabs(r.stdout.strip())


@pytest.mark.skipif(not _have_asan(), reason="no g++ with libasan")
def test_host_and_oracle_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "sanitize"], cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "sanitize ok" in r.stdout
