"""The CIFAR-10 CNN and its flat parameter layout.

Capability parity: the reference ``Network`` (``models/model.py:9-27`` in
dat-rohit/distributed-neural-network) is conv(3->6,5x5) -> ReLU -> maxpool2 ->
conv(6->16,5x5) -> ReLU -> maxpool2 -> flatten(400) -> fc 400->120 -> ReLU ->
fc 120->84 -> ReLU -> fc 84->10.  Its ``state_dict`` has 10 fp32 tensors in a
fixed key order; that key set/shape/dtype contract is the
checkpoint format of this framework.

MI355X-first design: the parameters do not live in ten separate tensors.  They
live in ONE flat fp32 arena (plus a gradient arena and a momentum arena of the
same layout), each tensor starting on a 256-byte boundary.  ``state_dict()``
tensors are views into it, a whole-model all-reduce is one collective on one
buffer, and the fused HIP kernels address every parameter by a constant offset.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

# (key, shape) in reference state_dict order (SURVEY.md §2.4 per-tensor table).
PARAM_SHAPES: List[Tuple[str, Tuple[int, ...]]] = [
    ("conv1.weight", (6, 3, 5, 5)),
    ("conv1.bias", (6,)),
    ("conv2.weight", (16, 6, 5, 5)),
    ("conv2.bias", (16,)),
    ("fc1.weight", (120, 400)),
    ("fc1.bias", (120,)),
    ("fc2.weight", (84, 120)),
    ("fc2.bias", (84,)),
    ("fc3.weight", (10, 84)),
    ("fc3.bias", (10,)),
]

NUM_CLASSES = 10
IMG_C, IMG_H, IMG_W = 3, 32, 32
IMG_BYTES = IMG_C * IMG_H * IMG_W
ALIGN_ELEMS = 64  # 256 B: every tensor starts on its own cache-line group


def _numel(shape: Tuple[int, ...]) -> int:
    n = 1
    for s in shape:
        n *= s
    return n


@dataclass(frozen=True)
class ArenaLayout:
    """Offsets (in fp32 elements) of every parameter inside the flat arena.

    The conv tensors come first and the MLP tensors second, so the two
    gradient buckets used for comm/compute overlap are contiguous ranges:
    ``conv_range`` and ``mlp_range``.
    """

    offsets: Dict[str, int]
    shapes: Dict[str, Tuple[int, ...]]
    total: int          # padded arena length (elements)
    num_params: int     # real parameter count (62,006)

    @staticmethod
    def build(param_shapes: "List[Tuple[str, Tuple[int, ...]]] | None" = None) -> "ArenaLayout":
        offsets, shapes = {}, {}
        cur = 0
        n = 0
        for key, shape in (PARAM_SHAPES if param_shapes is None else param_shapes):
            offsets[key] = cur
            shapes[key] = shape
            k = _numel(shape)
            n += k
            cur += (k + ALIGN_ELEMS - 1) // ALIGN_ELEMS * ALIGN_ELEMS
        return ArenaLayout(offsets, shapes, cur, n)

    def numel(self, key: str) -> int:
        return _numel(self.shapes[key])

    @property
    def conv_range(self) -> Tuple[int, int]:
        return 0, self.offsets["fc1.weight"]

    @property
    def mlp_range(self) -> Tuple[int, int]:
        return self.offsets["fc1.weight"], self.total

    def views(self, arena: torch.Tensor) -> "OrderedDict[str, torch.Tensor]":
        out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        for key, shape in self.shapes.items():
            o = self.offsets[key]
            out[key] = arena[o:o + _numel(shape)].view(shape)
        return out

    def pad_mask(self) -> torch.Tensor:
        """Boolean mask over the arena: True where a real parameter lives."""
        m = torch.zeros(self.total, dtype=torch.bool)
        for key, shape in self.shapes.items():
            o = self.offsets[key]
            m[o:o + _numel(shape)] = True
        return m


LAYOUT = ArenaLayout.build()


class Network(nn.Module):
    """nn.Module facade with the reference attribute names and state_dict keys.

    Used (a) as the fp32 oracle on CPU, (b) to draw PyTorch-default initial
    weights (kaiming-uniform a=sqrt(5), bias U(+-1/sqrt(fan_in))), and (c) as
    the load target of saved checkpoints.  The training hot path on MI355X
    never calls ``forward``; it runs the fused HIP kernels on the arena.
    """

    def __init__(self) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(IMG_C, 6, 5)
        self.pool = nn.MaxPool2d(2, 2)
        self.conv2 = nn.Conv2d(6, 16, 5)
        self.fc1 = nn.Linear(16 * 5 * 5, 120)
        self.fc2 = nn.Linear(120, 84)
        self.fc3 = nn.Linear(84, NUM_CLASSES)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = self.pool(F.relu(self.conv1(x)))
        h = self.pool(F.relu(self.conv2(h)))
        h = h.flatten(1)
        h = F.relu(self.fc1(h))
        h = F.relu(self.fc2(h))
        return self.fc3(h)


def init_arena(seed: int | None = None) -> torch.Tensor:
    """Fresh fp32 CPU arena holding a PyTorch-default-initialised Network."""
    if seed is not None:
        g_state = torch.random.get_rng_state()
        torch.manual_seed(seed)
    net = Network()
    if seed is not None:
        torch.random.set_rng_state(g_state)
    arena = torch.zeros(LAYOUT.total, dtype=torch.float32)
    load_state_dict_into(arena, net.state_dict())
    return arena


def load_state_dict_into(arena: torch.Tensor, sd) -> None:
    views = LAYOUT.views(arena)
    for key, _ in PARAM_SHAPES:
        if key not in sd:
            raise KeyError(f"state_dict is missing {key!r}")
        src = sd[key]
        if tuple(src.shape) != LAYOUT.shapes[key]:
            raise ValueError(f"{key}: shape {tuple(src.shape)} != {LAYOUT.shapes[key]}")
        views[key].copy_(src.detach().to(views[key].device, torch.float32))


def arena_state_dict(arena: torch.Tensor) -> "OrderedDict[str, torch.Tensor]":
    """Reference-format state_dict (CPU fp32 clones) from an arena on any device."""
    host = arena.detach().float().cpu()
    return OrderedDict((k, v.clone()) for k, v in LAYOUT.views(host).items())


def network_from_arena(arena: torch.Tensor) -> Network:
    net = Network()
    net.load_state_dict(arena_state_dict(arena))
    return net
