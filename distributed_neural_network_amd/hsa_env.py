"""HSA runtime defaults of this framework, applied before the GPU runtime starts (ROCr reads them
once, when the process first initialises it; ``import torch`` alone does not).  A value already
in the environment wins, and ``DNN_HSA_DEFAULTS=0`` applies none.

- ``HSA_ALLOCATE_QUEUE_DEV_MEM=1``: AQL queue ring buffers in device memory, so the command
  processor fetches a dispatch packet from HBM instead of across the host link.  The persistent
  window is ONE dispatch, so that fetch sits on its critical path: 16.00 vs 16.14 us per step
  in the driver's 20/5 window (5 alternating pairs, profiles/r6/aql/queue_devmem/).
"""
import os

DEFAULTS = {"HSA_ALLOCATE_QUEUE_DEV_MEM": "1"}


def apply() -> None:
    if os.environ.get("DNN_HSA_DEFAULTS", "1") == "0":
        return
    for k, v in DEFAULTS.items():
        os.environ.setdefault(k, v)
