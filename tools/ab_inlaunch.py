"""Diagnostic: separate-kernel vs in-launch reduction, per-parameter max |diff| per step."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import synthetic  # noqa: E402
from distributed_neural_network_amd.models.network import LAYOUT, init_arena  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402

data = synthetic(1000, 7)
a = init_arena(seed=5)
e1 = HipEngine(batch=64, arena=a, in_launch_reduce=False, use_graphs=False)
e2 = HipEngine(batch=64, arena=a, in_launch_reduce=True, use_graphs=False)
for e in (e1, e2):
    e.attach(data)
    e.begin_epoch(np.arange(1000, dtype=np.int32))
for step in range(16):
    for e in (e1, e2):
        e.run_steps(1)
    torch.cuda.synchronize()
    rows = {k: float((getattr(e1, k) - getattr(e2, k)).abs().max()) for k in ["a0", "h1", "z1", "slab", "loss"]}
    d = {k: float((v1 - v2).abs().max()) for (k, v1), v2 in zip(LAYOUT.views(e1.master).items(),
                                                                 LAYOUT.views(e2.master).values())}
    bad = {k: v for k, v in d.items() if v}
    print(step, "rows", {k: v for k, v in rows.items() if v}, "params", bad, "sync", e2.sync.tolist())
