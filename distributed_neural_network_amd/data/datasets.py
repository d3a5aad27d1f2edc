"""Datasets: CIFAR-10 binary batches or learnable synthetic CIFAR-shaped data.

Capability parity: ``torchvision.datasets.CIFAR10(root='./data', train=...)``
(data_parallelism_train.py:69-71,89; model_replication_train.py:41,47;
single_proc_train.py:37-43).  There is no network on the target machines, so
nothing is downloaded: ``--data cifar10`` reads the standard binary distribution
(``<root>/cifar-10-batches-bin/{data_batch_1..5,test_batch}.bin``) with the native
reader, and ``--data synthetic`` (the benchmark input, BASELINE.json) generates
CIFAR-shaped uint8 images with a deterministic seed.  Either way a split is one
contiguous ``uint8 [N,3,32,32]`` tensor + ``int32 [N]`` labels, uploaded to HBM
once; the ToTensor/Normalize transform runs inside the fused HIP kernel.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

from ..ops import native

CIFAR_TRAIN = 50_000
CIFAR_TEST = 10_000


@dataclass
class Split:
    images: torch.Tensor  # uint8 [N,3,32,32]
    labels: torch.Tensor  # int32 [N]
    name: str = ""

    def __len__(self) -> int:
        return int(self.labels.shape[0])

    def to(self, device) -> "Split":
        if self.images.device == torch.device(device):
            return self
        return Split(self.images.to(device, non_blocking=False), self.labels.to(device), self.name)


def _cifar_dir(root: str | os.PathLike) -> Path:
    root = Path(root)
    for cand in (root / "cifar-10-batches-bin", root):
        if (cand / "test_batch.bin").exists():
            return cand
    raise FileNotFoundError(
        f"CIFAR-10 binary batches not found under {root} (expected cifar-10-batches-bin/*.bin); "
        "there is no network to download them - use --data synthetic")


def load_cifar10(root: str | os.PathLike, train: bool) -> Split:
    d = _cifar_dir(root)
    files = [d / f"data_batch_{i}.bin" for i in range(1, 6)] if train else [d / "test_batch.bin"]
    images, labels = native.io().read_cifar_bin([str(f) for f in files])
    return Split(torch.from_numpy(images), torch.from_numpy(labels), "cifar10-" + ("train" if train else "test"))


SYNTH_NOISE = 96       # default template + noise amplitude (learnable in about one epoch)
SYNTH_NOISE_HARD = 255  # maximal noise: accuracy climbs over several epochs (tools/convergence.py)


def synthetic(n: int, seed: int, train: bool = True, noise: int = SYNTH_NOISE) -> Split:
    images, labels = native.io().synthetic(int(n), int(seed), noise=int(noise), split=0 if train else 1)
    tag = "" if noise == SYNTH_NOISE else f"-noise{noise}"
    return Split(torch.from_numpy(images), torch.from_numpy(labels),
                 "synthetic" + tag + "-" + ("train" if train else "test"))


def get_splits(kind: str, root: str = "./data", n_train: int | None = None, n_test: int | None = None,
               seed: int = 0) -> tuple[Split, Split]:
    if kind == "cifar10":
        tr, te = load_cifar10(root, True), load_cifar10(root, False)
        if n_train is not None:
            tr = Split(tr.images[:n_train], tr.labels[:n_train], tr.name)
        if n_test is not None:
            te = Split(te.images[:n_test], te.labels[:n_test], te.name)
        return tr, te
    if kind in ("synthetic", "synthetic-hard"):
        noise = SYNTH_NOISE if kind == "synthetic" else SYNTH_NOISE_HARD
        return (synthetic(CIFAR_TRAIN if n_train is None else n_train, seed, True, noise),
                synthetic(CIFAR_TEST if n_test is None else n_test, seed, False, noise))
    raise ValueError(f"unknown dataset kind {kind!r} (expected 'synthetic', 'synthetic-hard' or 'cifar10')")


def write_cifar_bin(path: str | os.PathLike, images: np.ndarray, labels: np.ndarray) -> None:
    """Write a CIFAR-10 binary batch (label byte + 3072 CHW bytes per record)."""
    images = np.ascontiguousarray(images, dtype=np.uint8).reshape(len(labels), -1)
    rec = np.concatenate([np.asarray(labels, dtype=np.uint8)[:, None], images], axis=1)
    Path(path).parent.mkdir(parents=True, exist_ok=True)
    rec.tofile(str(path))
