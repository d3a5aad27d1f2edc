"""roctx ranges (visible in rocprofv3 --marker-trace) with a silent no-op fallback.

Enabled by DNN_ROCTX=1 so that production runs pay nothing; loads libroctx64 from
/opt/rocm via ctypes (no build dependency).
"""
from __future__ import annotations

import ctypes
import os

_lib = None
_enabled = os.environ.get("DNN_ROCTX", "0") == "1"


def _load():
    global _lib, _enabled
    if _lib is not None or not _enabled:
        return _lib
    for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            _lib = ctypes.CDLL(name)
            _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            return _lib
        except OSError:
            continue
    _enabled = False
    return None


def push(name: str) -> None:
    lib = _load()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def pop() -> None:
    lib = _load()
    if lib is not None:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _load()
    if lib is not None:
        lib.roctxMarkA(name.encode())
