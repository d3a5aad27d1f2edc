"""LDS hygiene: no kernel result may depend on what an earlier kernel left in a CU's LDS.

LDS is not cleared between kernels.  A kernel that reads LDS it did not write in the same launch
(a pad it assumes zero, a DMA'd tile read before the DMA landed) usually reads the identical
bytes its own previous launch left and passes every test - until another kernel ran on that CU
in between.  ``lds_poison`` (csrc/kernels/diag.hip) fills every CU's 160 KB with one pattern;
each run below starts from the same parameters after a different pattern and must end bit for
bit where the zero-pattern run ends."""
import time

import numpy as np
import pytest
import torch

from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.runtime import HipEngine

pytestmark = pytest.mark.gpu

PATTERNS = (0x00000000, 0xFFFFFFFF, 0x7FC07FC0, 0x3F803F80, 0x5A5A5A5A)


def _rows(dtype: str, B: int, pattern: int) -> dict:
    """One serial fused-kernel launch on B samples right after an LDS poison pass."""
    split = synthetic(300, seed=3)
    eng = HipEngine(batch=B, seed=1, use_graphs=False, dtype=dtype)
    eng.attach(split)
    eng.begin_epoch(np.arange(5, 5 + B, dtype=np.int32))
    torch.cuda.synchronize()
    eng.ext.lds_poison(pattern, eng._stream())
    eng._launch_step()
    torch.cuda.synchronize()
    return {k: getattr(eng, k).clone().cpu() for k in ("a0", "h1", "h2", "z1", "z2", "z3", "slab", "loss", "master")}


@pytest.mark.parametrize("dtype,B", [("bf16", 1), ("bf16", 13), ("bf16", 64), ("fp32", 1), ("fp32", 13)])
def test_serial_step_ignores_stale_lds(dtype, B):
    ref = _rows(dtype, B, 0)
    for pat in PATTERNS[1:]:
        got = _rows(dtype, B, pat)
        for k in ref:
            bad = int((ref[k] != got[k]).sum()) if ref[k].dtype.is_floating_point else 0
            assert torch.equal(ref[k], got[k]), f"{dtype} B={B} pattern {pat:#010x}: {k} differs at {bad} elements"


def _steps(dtype: str, pipeline: bool, persist: bool, pattern: int, steps: int = 24) -> tuple:
    data = synthetic(1024, 12)
    order = np.random.default_rng(4).permutation(1024).astype(np.int32)
    eng = HipEngine(batch=64, arena=init_arena(seed=6), graph_chunk=8, pipeline=pipeline, persist=persist, dtype=dtype)
    eng.attach(data)
    eng.begin_epoch(order)
    eng.prepare_graphs()
    torch.cuda.synchronize()
    eng.ext.lds_poison(pattern, eng._stream())
    eng.run_steps(steps)
    torch.cuda.synchronize()
    assert not eng.pipe_failed()
    return eng.master.cpu(), eng.mom.cpu(), eng.shadow.cpu()


@pytest.mark.parametrize("dtype,pipeline,persist", [("bf16", False, False), ("bf16", True, False), ("bf16", True, True),
                                                    ("fp32", False, False), ("fp32", False, True)])
def test_training_steps_ignore_stale_lds(dtype, pipeline, persist):
    ref = _steps(dtype, pipeline, persist, 0)
    for pat in PATTERNS[1:]:
        got = _steps(dtype, pipeline, persist, pat)
        for x, y, name in zip(ref, got, ("master", "momentum", "bf16 images")):
            assert torch.equal(x, y), f"{dtype} pipe={pipeline} pers={persist} pattern {pat:#010x}: {name} differs " \
                                      f"at {int((x != y).sum())} elements"


def _squat_run(dtype: str, pipeline: bool, persist: bool, squat_bytes: int, steps: int = 16):
    """The same training steps with (squat_bytes > 0) one-wave workgroups holding squat_bytes of
    LDS each resident on every CU while the engine's kernels run beside them on another stream."""
    data = synthetic(1024, 12)
    order = np.random.default_rng(4).permutation(1024).astype(np.int32)
    eng = HipEngine(batch=64, arena=init_arena(seed=6), graph_chunk=8, pipeline=pipeline, persist=persist, dtype=dtype)
    eng.attach(data)
    eng.begin_epoch(order)
    eng.prepare_graphs()
    bad = torch.zeros(1, dtype=torch.int32, device=eng.device)
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    if squat_bytes:
        cus = torch.cuda.get_device_properties(eng.device).multi_processor_count
        eng.ext.lds_squat(squat_bytes, 30000.0, 2 * cus, bad.data_ptr(), side.cuda_stream)
        time.sleep(0.003)  # (resident before the engine's first launch)
    eng.run_steps(steps)
    torch.cuda.synchronize()
    assert not eng.pipe_failed()
    return eng.master.cpu(), eng.mom.cpu(), int(bad.item())


@pytest.mark.parametrize("dtype,pipeline,persist", [("bf16", False, False), ("bf16", True, True), ("fp32", False, True)])
def test_kernels_share_cus_with_lds_holding_workgroups(dtype, pipeline, persist):
    """Workgroups of other kernels (other streams, other engines of the process - the in-process
    exchange harness runs two) may sit on the engine's CUs in the LDS its kernels leave free.
    Neither side may see the other's LDS: the squatters' LDS must be intact and the engine's
    parameters bit-identical to a run on an otherwise idle GPU."""
    ref = _squat_run(dtype, pipeline, persist, 0)
    for nbytes in (1024, 3072):
        got = _squat_run(dtype, pipeline, persist, nbytes)
        assert got[2] == 0, f"{nbytes} B squatters: {got[2]} LDS words overwritten under them"
        assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1]), \
            f"{nbytes} B squatters: master differs at {int((ref[0] != got[0]).sum())} elements"
