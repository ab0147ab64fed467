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


def test_device_assert_build_compiles(tmp_path):
    """The debug build's device-side bounds asserts (XF_DASSERT) compile for
    gfx950 (hipcc cross-compiles without a GPU)."""
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    for src in ("kernels_table.hip", "kernels_model.hip"):
        r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O1", "-std=c++17",
                            "-DXFLOW_DEVICE_ASSERT=1", "-I" + os.path.join(ROOT, "csrc", "include"),
                            "-I" + os.path.join(ROOT, "csrc", "hip"), "-c",
                            os.path.join(ROOT, "csrc", "hip", src), "-o", str(tmp_path / "k.o")],
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
