"""Loader for the in-tree native extension ``qfedx_amd._qfedx_C``.

On a GPU box the HIP path is mandatory: if the extension cannot be imported, ``ext()`` raises
instead of silently falling back to the torch reference path.  ``QFEDX_AUTOBUILD=1`` builds it on
first use (hipcc, gfx950) when the shared object is missing.  ``QFEDX_DEBUG=1`` loads the debug build
``qfedx_amd._qfedx_C_debug`` (device-side bounds checks that raise after the failing launch; build it with
``python -m qfedx_amd._build --debug``).
"""
from __future__ import annotations

import importlib
import os

_EXT = None


def ext():
    global _EXT
    if _EXT is not None:
        return _EXT
    debug = os.environ.get("QFEDX_DEBUG", "0") == "1"
    name = "qfedx_amd._qfedx_C_debug" if debug else "qfedx_amd._qfedx_C"
    try:
        _EXT = importlib.import_module(name)
    except ImportError as e:
        if os.environ.get("QFEDX_AUTOBUILD", "0") == "1":
            from .. import _build
            _build.build(debug=debug)
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
