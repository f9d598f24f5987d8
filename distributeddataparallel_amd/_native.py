"""Loader for the native extension ``distributeddataparallel_amd._C``.

The extension is built in-tree (``python -m distributeddataparallel_amd._build``). On a GPU
box a missing extension is a hard error: GPU code paths must never silently fall back to
eager PyTorch. On CPU-only hosts the build is attempted on first import.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_C = None


def load():
    global _C
    if _C is not None:
        return _C
    with _lock:
        if _C is not None:
            return _C
        try:
            _C = importlib.import_module("distributeddataparallel_amd._C")
        except ImportError as first:
            if os.environ.get("XDDP_NO_AUTOBUILD") == "1":
                raise ImportError(
                    "distributeddataparallel_amd._C is not built; run "
                    "`python -m distributeddataparallel_amd._build`"
                ) from first
            from . import _build

            _build.build()
            _C = importlib.import_module("distributeddataparallel_amd._C")
        if os.environ.get("XDDP_NATIVE_BACKTRACE") == "1":
            _C.install_crash_handler()
    return _C
