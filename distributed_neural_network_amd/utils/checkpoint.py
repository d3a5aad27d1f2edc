"""Checkpoint / resume.

The reference never writes a checkpoint (no torch.save anywhere); its
only serialized model is ``Network().state_dict()`` with 10 fp32 keys.  The checkpoint
format here IS that state_dict: ``torch.save(OrderedDict(conv1.weight, ..., fc3.bias))``
with the reference keys, shapes and dtypes, loadable by the reference
``models/model.py::Network.load_state_dict`` unmodified.

Resume state that the reference has no notion of (momentum arena, epoch, RNG/seed,
world size, sync mode) goes to a sidecar ``<path>.resume.pt`` next to it.  Both files
are written by rank 0 after a sync point (parameters are identical on every rank),
atomically (write to a temp name, then rename).
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Any

import torch

from ..models.network import LAYOUT, PARAM_SHAPES


def _atomic_save(obj: Any, path: str) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save(path: str, state_dict: "OrderedDict[str, torch.Tensor]", momentum: torch.Tensor | None = None,
         **meta: Any) -> None:
    """Write ``state_dict`` (all of its keys, in order: the reference 10 for the reference
    model; parameters + BatchNorm buffers for zoo models) + the resume sidecar."""
    sd = OrderedDict((k, v.detach().cpu().contiguous() if not v.is_floating_point()
                      else v.detach().float().cpu().contiguous()) for k, v in state_dict.items())
    _atomic_save(sd, path)
    side = {"format": "dnn-amd-resume-v1", "arena_total": int(momentum.numel()) if momentum is not None
            else LAYOUT.total, **meta}
    if momentum is not None:
        side["momentum"] = momentum.detach().float().cpu().clone()
    _atomic_save(side, path + ".resume.pt")


def load(path: str, expected: "list[tuple[str, tuple[int, ...]]] | None" = None
         ) -> tuple["OrderedDict[str, torch.Tensor]", dict]:
    """Load a checkpoint (weights_only: nothing from the file is executed) and check it
    against ``expected`` (key, shape) pairs - the reference Network's by default."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    for k, shape in (PARAM_SHAPES if expected is None else expected):
        if k not in sd:
            raise KeyError(f"{path}: missing {k}")
        if tuple(sd[k].shape) != tuple(shape):
            raise ValueError(f"{path}: {k} has shape {tuple(sd[k].shape)}, expected {tuple(shape)}")
    side = {}
    sp = path + ".resume.pt"
    if os.path.exists(sp):
        side = torch.load(sp, map_location="cpu", weights_only=True)
    return sd, side
