"""Debug build of the native extension (QFEDX_DEBUG=1 -> qfedx_amd._qfedx_C_debug, csrc/qfx_check.h): the
device-side checks stay silent on a valid program and report the failing source line when an op record is
corrupted.  The corruption used (a group op's real-qubit count set to 5) only feeds a parity loop over the
record's own words, so the run stays memory-safe.  Runs in a child process: the loader picks the build once."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

CHILD = r"""
import torch
from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops._ext import ext
from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
C = ext()
assert C.__name__.endswith("_qfedx_C_debug"), C.__name__
dev = torch.device("cuda", 0)
spec = VQCSpec(12, 2, 3)
prog = HeaMfmaProgram(spec, dev, tile_bits=10)
x = torch.rand(2, 3, 12, device=dev) * 3
th = torch.randn(2, spec.n_theta, device=dev)
w = torch.randn(2, 3, 3, device=dev)
prog.vjp(x, th, w)
assert C.hea_check_status() == 0
ops = prog.passes[0][2][0]                    # first pass' adjoint op records (device int32 [nops, 128])
code = ops[:, 0].cpu()
row = int((code == 8).nonzero()[0])           # a BACK op
ops[row, 2] = 5
try:
    prog.vjp(x, th, w)
except RuntimeError as e:
    assert "device check failed at hea_mfma.hip:" in str(e), str(e)
    print("DETECTED", str(e).split(":")[-1])
else:
    raise SystemExit("corrupted record not detected")
"""


def test_debug_build_device_checks(cuda):
    env = dict(os.environ, QFEDX_DEBUG="1")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "DETECTED" in r.stdout
