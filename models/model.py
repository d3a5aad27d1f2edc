"""Reference-compatible import path: ``from models.model import Network``.

The reference keeps its CNN in ``models/model.py:9-27``; scripts and
checkpoints written against it keep working because this module re-exports
the framework's ``Network`` (same attribute names, same state_dict keys,
shapes and dtypes).
"""
from distributed_neural_network_amd.models.network import Network  # noqa: F401

__all__ = ["Network"]
