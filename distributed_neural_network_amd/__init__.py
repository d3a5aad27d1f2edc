"""MI355X-native data-parallel CNN training framework (see README.md)."""
from .hsa_env import apply as _apply_hsa_env

_apply_hsa_env()  # (before any GPU runtime initialisation in this process)
