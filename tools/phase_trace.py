#!/usr/bin/env python3
"""Per-phase timeline of the fused training kernel (diagnostic).

Launches the fused kernel with its stamp buffer enabled: block 0 / thread 0 records
s_memrealtime (100 MHz) at each phase boundary.  Prints the median over repeats of
each phase's duration in microseconds, plus the whole-kernel wall time from events.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import synthetic  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402

PHASES = ["A ingest+staging", "B conv1 fwd", "C conv2 fwd", "D MLP fwd+CE", "D' MLP bwd",
          "E conv2 bwd", "F conv1 wgrad",
          "  C1 prefetch+R2 build", "  E1 dY2 build", "  E2 wgrad2+col2im", "  E3 dP1 gather",
          "  F1 dY1 + R1 rebuild"]


def main(reps: int = 50, batch: int = 64):
    tr = synthetic(4096, 0)
    eng = HipEngine(batch=batch, seed=0, use_graphs=False)
    eng.attach(tr)
    eng.begin_epoch(np.arange(4096, dtype=np.int32))
    stamps = torch.zeros(16, dtype=torch.int64, device=eng.device)
    rows = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    walls = []
    for r in range(reps):
        eng.begin_epoch(np.roll(np.arange(4096, dtype=np.int32), -64 * (r % 60)))
        ev0.record()
        eng.ext.fused_train(eng._p(eng.train.images), eng._p(eng.train.labels), eng._p(eng.batch_ids), eng.order_len,
                            eng.batch, eng._p(eng.state), eng._p(eng.master), eng._p(eng.shadow), eng._p(eng.a0),
                            eng._p(eng.h1), eng._p(eng.h2), eng._p(eng.z1), eng._p(eng.z2), eng._p(eng.z3),
                            eng._p(eng.slab), eng._p(eng.loss), eng._p(eng.correct), eng._stream(),
                            stamps=stamps.data_ptr())
        ev1.record()
        torch.cuda.synchronize()
        walls.append(ev0.elapsed_time(ev1) * 1000)
        s = stamps.cpu().numpy()
        rows.append(np.concatenate([np.diff(s[:8]), [s[11] - s[2], s[8] - s[5], s[9] - s[8], s[6] - s[9],
                                                      s[10] - s[6]]]) * 0.01)  # 100 MHz ticks -> us
    med = np.median(np.array(rows[5:]), axis=0)
    for name, v in zip(PHASES, med):
        print(f"{name:20s} {v:8.2f} us")
    print(f"{'sum (block 0)':20s} {med[:7].sum():8.2f} us")
    print(f"{'kernel wall (event)':20s} {np.median(walls[5:]):8.2f} us")


if __name__ == "__main__":
    main()
