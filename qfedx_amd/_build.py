"""In-tree build of the native extension ``qfedx_amd._qfedx_C`` for gfx950 (MI355X).

``QFEDX_DEBUG=1`` (or ``python -m qfedx_amd._build --debug``) builds the separate debug extension
``qfedx_amd._qfedx_C_debug`` with device-side bounds checks (``csrc/qfx_check.h``) into ``build/qfx_debug``;
``QFEDX_DEBUG=1`` at run time makes ``ops/_ext.py`` load it instead of the release one.  ``--stamps``
(``QFEDX_STAMPS=1``) likewise builds / loads ``qfedx_amd._qfedx_C_stamps``: the MFMA pass kernels with per-wave
s_memtime phase stamps (``-DQFX_HEA_STAMPS=1``, stall attribution: scripts/hea_stamps.py), never the release path.

Device code (``csrc/*.hip``) is compiled by ``hipcc --offload-arch=gfx950``; host bindings
(``csrc/*.cpp``: planner + pybind11/torch glue) by g++ against torch's headers; everything is linked
by hipcc into one shared object next to this file, so it travels with the repo snapshot to the GPU
box (no JIT cache, no site-packages install).  Incremental: objects are rebuilt only when a source
or header hash changes.  No hipify step: the sources are HIP/CDNA4 code to begin with.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import json
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ARCH = os.environ.get("QFEDX_ARCH", "gfx950")


def variant(debug=None) -> str:
    """release | debug | stamps (``debug``: True / False forces debug / release; None reads the environment)."""
    if debug is not None:
        return "debug" if debug else "release"
    if os.environ.get("QFEDX_DEBUG", "0") == "1":
        return "debug"
    if os.environ.get("QFEDX_STAMPS", "0") == "1":
        return "stamps"
    return "release"


_VARIANTS = {"release": ("qfx", "_qfedx_C", []), "debug": ("qfx_debug", "_qfedx_C_debug", ["-DQFX_DEVICE_CHECKS=1"]),
             "stamps": ("qfx_stamps", "_qfedx_C_stamps", ["-DQFX_HEA_STAMPS=1"])}


def _mode(debug):
    v = debug if isinstance(debug, str) else variant(debug)
    d, name, flags = _VARIANTS[v]
    return os.path.join(HERE, "..", "build", d), name, flags


def ext_path(debug=None) -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(HERE, _mode(debug)[1] + suffix)


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths(device_type="cuda") if "device_type" in ce.include_paths.__code__.co_varnames \
        else ce.include_paths(cuda=True)
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hash(paths) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()


def _local_includes(src: str) -> list:
    """Non-header sources ``src`` pulls in with #include "..." (hea_mfma_bf16.hip includes hea_mfma.hip): part of
    its rebuild key (the *.h headers are hashed for every object anyway)."""
    import re
    out = []
    with open(src) as f:
        for m in re.finditer(r'^\s*#include\s+"([^"]+)"', f.read(), re.M):
            p = os.path.join(os.path.dirname(src), m.group(1))
            if os.path.exists(p) and not p.endswith(".h"):
                out.append(p)
    return out


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


def build(verbose: bool = False, force: bool = False, debug=None) -> str:
    BUILD, EXT_NAME, checks = _mode(debug)
    os.makedirs(BUILD, exist_ok=True)
    extra = os.environ.get("QFEDX_EXTRA_HIPFLAGS", "").split()   # e.g. -DQFX_HEA_GATE_LO=0 (A/B builds)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    hips = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    cpps = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))
    stamp_path = os.path.join(BUILD, "stamp.json")
    stamps = {}
    if os.path.exists(stamp_path) and not force:
        with open(stamp_path) as f:
            stamps = json.load(f)
    inc, tlib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    import pybind11
    common_defs = ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    jobs = []
    objs = []
    hh = _hash(headers)
    for src in hips:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        key = _hash([src] + _local_includes(src)) + hh + ARCH + " ".join(extra)
        objs.append(obj)
        if stamps.get(obj) != key or not os.path.exists(obj):
            cmd = ["hipcc", "-c", "-fPIC", "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fno-gpu-rdc",
                   "-munsafe-fp-atomics", *checks, *extra, "-I", CSRC, src, "-o", obj]
            jobs.append((obj, key, cmd))
    for src in cpps:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        key = _hash([src]) + hh + str(abi)
        objs.append(obj)
        if stamps.get(obj) != key or not os.path.exists(obj):
            cmd = ["g++", "-c", "-fPIC", "-O2", "-std=c++17", *common_defs, *checks,
                   f"-DTORCH_EXTENSION_NAME={EXT_NAME}", "-DTORCH_API_INCLUDE_EXTENSION_H",
                   *[f"-I{p}" for p in inc], f"-I{py_inc}", f"-I{pybind11.get_include()}", "-I", CSRC,
                   src, "-o", obj]
            jobs.append((obj, key, cmd))
    if jobs:
        workers = min(len(jobs), int(os.environ.get("MAX_JOBS", "8")))
        with cf.ThreadPoolExecutor(workers) as ex:
            futs = {ex.submit(_run, cmd): (obj, key) for obj, key, cmd in jobs}
            for fu in cf.as_completed(futs):
                obj, key = futs[fu]
                fu.result()
                stamps[obj] = key
                if verbose:
                    print("compiled", os.path.basename(obj))
    out = ext_path(debug)
    link_key = _hash(objs) if all(os.path.exists(o) for o in objs) else ""
    if jobs or stamps.get("__link__") != link_key or not os.path.exists(out):
        cmd = ["hipcc", "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out + ".tmp",
               f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-ltorch_hip", "-lhiprtc",
               "-lamdhip64",
               f"-Wl,-rpath,{tlib}"]
        _run(cmd)
        os.replace(out + ".tmp", out)
        stamps["__link__"] = _hash(objs)
        if verbose:
            print("linked", out)
    with open(stamp_path, "w") as f:
        json.dump(stamps, f)
    return out


if __name__ == "__main__":
    v = "debug" if "--debug" in sys.argv else ("stamps" if "--stamps" in sys.argv else None)
    p = build(verbose=True, force="--force" in sys.argv, debug=v)
    print(p)
