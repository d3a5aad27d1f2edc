"""HSA runtime defaults of this framework, applied before the GPU runtime starts (ROCr reads them
once, when the process first initialises it; ``import torch`` alone does not).  A value already
in the environment wins, and ``DNN_HSA_DEFAULTS=0`` applies none.

- ``HSA_ALLOCATE_QUEUE_DEV_MEM=1``: AQL queue ring buffers in device memory, so the command
  processor fetches a dispatch packet from HBM instead of across the host link.  The persistent
  window is ONE dispatch, so that fetch sits on its critical path: 16.00 vs 16.14 us per step
  in the driver's 20/5 window (5 alternating pairs, profiles/r6/aql/queue_devmem/).

Single-rank processes only: a rank of a multi-rank job (WORLD_SIZE > 1, or an MPI size) keeps the
runtime's defaults - its step is graph replays plus collectives, where the placement was not
measured, and RCCL / IPC over distinct GPUs has not run with it.  A self-launching parent that
applied them hands its ranks an environment without them (``strip``).
"""
import os

DEFAULTS = {"HSA_ALLOCATE_QUEUE_DEV_MEM": "1"}
_MARK = "DNN_HSA_DEFAULTED"  # the keys apply() set (not the user)
_SIZE_VARS = ("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS")


def _multi_rank(env) -> bool:
    for k in _SIZE_VARS:
        try:
            if int(env.get(k, "1")) > 1:
                return True
        except ValueError:
            pass
    return False


def apply() -> None:
    if os.environ.get("DNN_HSA_DEFAULTS", "1") == "0" or _multi_rank(os.environ):
        return
    set_here = [k for k in DEFAULTS if k not in os.environ]
    for k in set_here:
        os.environ[k] = DEFAULTS[k]
    if set_here:
        os.environ[_MARK] = ",".join(sorted(set(os.environ.get(_MARK, "").split(",") + set_here) - {""}))


def strip(env: dict) -> dict:
    """``env`` without the defaults apply() set in this process (for the ranks it launches)."""
    for k in env.pop(_MARK, "").split(","):
        if k:
            env.pop(k, None)
    return env
