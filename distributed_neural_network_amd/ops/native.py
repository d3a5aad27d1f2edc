"""Loader for the in-tree native extensions.

GPU code paths call :func:`hip` and get the compiled gfx950 kernel module or a loud
``RuntimeError``: there is no silent eager-PyTorch fallback on a GPU box.  The CPU
oracle engine exists for CPU-only hosts and tests, and is selected explicitly.
"""
from __future__ import annotations

import importlib
from types import ModuleType

from ..models.network import LAYOUT

_HIP: ModuleType | None = None
_IO: ModuleType | None = None

SLAB = 2872


def _import(name: str, build_fn) -> ModuleType:
    try:
        return importlib.import_module(f"{__package__}.{name}")
    except ImportError:
        build_fn()
        return importlib.import_module(f"{__package__}.{name}")


def hip() -> ModuleType:
    """The gfx950 kernel module (built in-tree on first use if missing)."""
    global _HIP
    if _HIP is None:
        from . import build

        try:
            mod = _import("_dnn_hip", build.build_hip)
        except Exception as e:  # pragma: no cover - exercised only on broken installs
            raise RuntimeError(
                "the gfx950 HIP extension _dnn_hip is missing and could not be built; "
                "run `python -m distributed_neural_network_amd.ops.build`") from e
        lay = mod.layout()
        for key, off in LAYOUT.offsets.items():
            if lay[key] != off:
                raise RuntimeError(f"arena layout mismatch for {key}: kernel {lay[key]} != python {off}")
        if lay["arena"] != LAYOUT.total or lay["slab"] != SLAB:
            raise RuntimeError("arena/slab size mismatch between kernels and python")
        _HIP = mod
    return _HIP


def io() -> ModuleType:
    """The native data runtime (CIFAR reader, synthetic data, permutations)."""
    global _IO
    if _IO is None:
        from . import build

        _IO = _import("_dnn_io", build.build_io)
    return _IO
