"""Native planner + JIT code generator under host AddressSanitizer/UBSan on random circuits
(GPU ASan/XNACK are unavailable on the GPU pool; the host C++ is where memory errors are hunted)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"), reason="needs g++ + ROCm headers")
def test_native_planner_codegen_asan_ubsan():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_host.sh"), "150"], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "native fuzz ok" in r.stdout
