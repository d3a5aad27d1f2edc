from .datasets import CIFAR_TEST, CIFAR_TRAIN, Split, get_splits, load_cifar10, synthetic, write_cifar_bin
from .partition import EpochSampler, shard_bounds

__all__ = ["CIFAR_TEST", "CIFAR_TRAIN", "Split", "get_splits", "load_cifar10", "synthetic", "write_cifar_bin",
           "EpochSampler", "shard_bounds"]
