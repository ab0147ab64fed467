"""Host-side ASan + UBSan build of the native trainer (CMake,
-DXFLOW_HOST_SANITIZE=ON) run over every model family and quirk mode
(scripts/sanitize_host.sh).  GPU sanitizers are unavailable on the MI355X
pool; device kernels are covered by the numerics tests."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake not installed")
def test_host_asan_ubsan_clean():
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "sanitize_host.sh")],
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "sanitize_host: clean" in r.stdout
