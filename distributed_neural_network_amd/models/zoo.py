"""Model zoo for the modular (layer-kernel) engine.

A model is a flat list of layer specs.  The same spec builds

* an ``nn.Module`` (``SpecNet``) - PyTorch-default initialisation, the fp32 CPU oracle,
  and the ``state_dict`` key set / checkpoint format (``conv1.weight``, ``bn1.running_mean``,
  ...; for ``lenet`` exactly the reference keys of ``models/model.py:13-18``), and
* the parameter arena layout (``ArenaLayout.build(param_shapes)``) + a buffer arena for
  BatchNorm running statistics, which the HIP layer engine (runtime/layer_engine.py)
  runs with the kernels of csrc/kernels/layers.hip.

Models:

``lenet``      the reference CNN (models/model.py:9-27) - also served by the fused engine.
``lenet-bn``   the reference CNN with BatchNorm2d after each convolution (the layer set
               the north star names: Conv2d, BatchNorm, ReLU, MaxPool, Linear).
``cifar-vgg``  a wider CIFAR-10 CNN (3x3 convs with padding, BatchNorm, 2 pooling stages)
               to show the layer engine is not LeNet-specific.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch
import torch.nn as nn

from .network import NUM_CLASSES, ArenaLayout


@dataclass(frozen=True)
class Conv:
    name: str
    cin: int
    cout: int
    k: int
    pad: int = 0


@dataclass(frozen=True)
class BN:
    name: str
    c: int
    eps: float = 1e-5
    momentum: float = 0.1


@dataclass(frozen=True)
class ReluPool:  # ReLU + 2x2 max-pool (stride 2), fused
    pass


@dataclass(frozen=True)
class Relu:
    pass


@dataclass(frozen=True)
class Flatten:
    pass


@dataclass(frozen=True)
class FC:
    name: str
    fin: int
    fout: int


MODELS: Dict[str, List[object]] = {
    "lenet": [Conv("conv1", 3, 6, 5), ReluPool(), Conv("conv2", 6, 16, 5), ReluPool(), Flatten(),
              FC("fc1", 400, 120), Relu(), FC("fc2", 120, 84), Relu(), FC("fc3", 84, NUM_CLASSES)],
    "lenet-bn": [Conv("conv1", 3, 6, 5), BN("bn1", 6), ReluPool(), Conv("conv2", 6, 16, 5), BN("bn2", 16),
                 ReluPool(), Flatten(), FC("fc1", 400, 120), Relu(), FC("fc2", 120, 84), Relu(),
                 FC("fc3", 84, NUM_CLASSES)],
    "cifar-vgg": [Conv("conv1", 3, 32, 3, 1), BN("bn1", 32), Relu(), Conv("conv2", 32, 32, 3, 1), BN("bn2", 32),
                  ReluPool(), Conv("conv3", 32, 64, 3, 1), BN("bn3", 64), Relu(), Conv("conv4", 64, 64, 3, 1),
                  BN("bn4", 64), ReluPool(), Flatten(), FC("fc1", 64 * 8 * 8, 256), Relu(),
                  FC("fc2", 256, NUM_CLASSES)],
}


def spec(name: str) -> List[object]:
    if name not in MODELS:
        raise ValueError(f"unknown model {name!r}; available: {sorted(MODELS)}")
    return MODELS[name]


def param_shapes(name: str) -> List[Tuple[str, Tuple[int, ...]]]:
    out: List[Tuple[str, Tuple[int, ...]]] = []
    for L in spec(name):
        if isinstance(L, Conv):
            out += [(f"{L.name}.weight", (L.cout, L.cin, L.k, L.k)), (f"{L.name}.bias", (L.cout,))]
        elif isinstance(L, BN):
            out += [(f"{L.name}.weight", (L.c,)), (f"{L.name}.bias", (L.c,))]
        elif isinstance(L, FC):
            out += [(f"{L.name}.weight", (L.fout, L.fin)), (f"{L.name}.bias", (L.fout,))]
    return out


def buffer_shapes(name: str) -> List[Tuple[str, Tuple[int, ...]]]:
    """fp32 buffers (BatchNorm running statistics) kept in a second flat arena."""
    out: List[Tuple[str, Tuple[int, ...]]] = []
    for L in spec(name):
        if isinstance(L, BN):
            out += [(f"{L.name}.running_mean", (L.c,)), (f"{L.name}.running_var", (L.c,))]
    return out


def layouts(name: str) -> Tuple[ArenaLayout, ArenaLayout]:
    return ArenaLayout.build(param_shapes(name)), ArenaLayout.build(buffer_shapes(name) or [("_none", (1,))])


class SpecNet(nn.Module):
    """nn.Module built from a spec: default init, CPU oracle, checkpoint key set."""

    def __init__(self, name: str) -> None:
        super().__init__()
        self.model_name = name
        self._order: List[Tuple[str, object]] = []
        for i, L in enumerate(spec(name)):
            if isinstance(L, Conv):
                self.add_module(L.name, nn.Conv2d(L.cin, L.cout, L.k, padding=L.pad))
                self._order.append((L.name, L))
            elif isinstance(L, BN):
                self.add_module(L.name, nn.BatchNorm2d(L.c, eps=L.eps, momentum=L.momentum))
                self._order.append((L.name, L))
            elif isinstance(L, FC):
                self.add_module(L.name, nn.Linear(L.fin, L.fout))
                self._order.append((L.name, L))
            else:
                self._order.append(("", L))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        for name, L in self._order:
            if isinstance(L, (Conv, BN, FC)):
                x = getattr(self, name)(x)
            elif isinstance(L, ReluPool):
                x = torch.nn.functional.max_pool2d(torch.relu(x), 2, 2)
            elif isinstance(L, Relu):
                x = torch.relu(x)
            elif isinstance(L, Flatten):
                x = x.flatten(1)
        return x


def init_arenas(name: str, seed: int | None = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(param arena, buffer arena) of a PyTorch-default-initialised model (CPU fp32)."""
    if seed is not None:
        g = torch.random.get_rng_state()
        torch.manual_seed(seed)
    net = SpecNet(name)
    if seed is not None:
        torch.random.set_rng_state(g)
    return arenas_from_state_dict(name, net.state_dict())


def arenas_from_state_dict(name: str, sd) -> Tuple[torch.Tensor, torch.Tensor]:
    play, blay = layouts(name)
    p = torch.zeros(play.total, dtype=torch.float32)
    b = torch.zeros(blay.total, dtype=torch.float32)
    for k, v in play.views(p).items():
        if k not in sd:
            raise KeyError(f"state_dict is missing {k!r}")
        if tuple(sd[k].shape) != tuple(v.shape):
            raise ValueError(f"{k}: shape {tuple(sd[k].shape)} != {tuple(v.shape)}")
        v.copy_(sd[k].detach().float())
    for k, v in blay.views(b).items():
        if k in sd:
            v.copy_(sd[k].detach().float())
    return p, b


def state_dict_from_arenas(name: str, params: torch.Tensor, buffers: torch.Tensor,
                           num_batches_tracked: int = 0) -> "OrderedDict[str, torch.Tensor]":
    """torch-compatible state_dict (loadable by SpecNet(name); for ``lenet`` by the
    reference ``Network``) in module registration order."""
    play, blay = layouts(name)
    pv = play.views(params.detach().float().cpu())
    bv = blay.views(buffers.detach().float().cpu())
    out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for L in spec(name):
        if isinstance(L, (Conv, FC)):
            out[f"{L.name}.weight"] = pv[f"{L.name}.weight"].clone()
            out[f"{L.name}.bias"] = pv[f"{L.name}.bias"].clone()
        elif isinstance(L, BN):
            out[f"{L.name}.weight"] = pv[f"{L.name}.weight"].clone()
            out[f"{L.name}.bias"] = pv[f"{L.name}.bias"].clone()
            out[f"{L.name}.running_mean"] = bv[f"{L.name}.running_mean"].clone()
            out[f"{L.name}.running_var"] = bv[f"{L.name}.running_var"].clone()
            out[f"{L.name}.num_batches_tracked"] = torch.tensor(int(num_batches_tracked), dtype=torch.long)
    return out


def checkpoint_keys(name: str) -> List[Tuple[str, Tuple[int, ...]]]:
    return param_shapes(name) + buffer_shapes(name)
