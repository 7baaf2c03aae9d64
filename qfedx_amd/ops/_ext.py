"""Loader for the in-tree native extension ``qfedx_amd._qfedx_C``.

On a GPU box the HIP path is mandatory: if the extension cannot be imported, ``ext()`` raises
instead of silently falling back to the torch reference path.  ``QFEDX_AUTOBUILD=1`` builds it on
first use (hipcc, gfx950) when the shared object is missing.  ``QFEDX_DEBUG=1`` loads the debug build
``qfedx_amd._qfedx_C_debug`` (device-side bounds checks that raise after the failing launch; build it with
``python -m qfedx_amd._build --debug``); ``QFEDX_STAMPS=1`` the stall-attribution build ``_qfedx_C_stamps``.
"""
from __future__ import annotations

import importlib
import os

_EXT = None


def ext():
    global _EXT
    if _EXT is not None:
        return _EXT
    from .. import _build
    v = _build.variant()
    name = "qfedx_amd." + _build._VARIANTS[v][1]
    try:
        _EXT = importlib.import_module(name)
    except ImportError as e:
        if os.environ.get("QFEDX_AUTOBUILD", "0") == "1":
            _build.build(debug=v)
            _EXT = importlib.import_module(name)
        else:
            raise RuntimeError(
                "qfedx_amd native extension is not built (run `python -m qfedx_amd._build` or "
                "`python -c 'import __graft_entry__ as g; g.build()'`): " + str(e)) from e
    return _EXT


def available() -> bool:
    try:
        ext()
        return True
    except RuntimeError:
        return False
