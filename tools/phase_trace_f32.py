#!/usr/bin/env python3
"""Per-phase timeline of the fp32 fused training kernel (lenet_f32.hip), diagnostic.

Block 0 / thread 0 stamps s_memrealtime (100 MHz) after every workgroup barrier; prints the
median duration of each interval over repeats, plus the kernel wall time from events."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import synthetic  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402

NAMES = ["A ingest + weights", "B conv1 fwd", "C conv2 fwd (halves)", "C' conv2 epilogue + fc1 issue",
         "D fc1 fwd", "D fc2 fwd", "D fc3 + CE", "D' dh2", "D' dh1", "D' dA0 partials",
         "D' dA0 sum + rows + dY2/T2", "E dgrad || dW2 + XW copy", "E dgrad sum + T1 values", "F dW1 slices",
         "F dW1 sum + end"]


def main(reps: int = 50, batch: int = 64):
    tr = synthetic(4096, 0)
    eng = HipEngine(batch=batch, seed=0, use_graphs=False, dtype="fp32")
    eng.attach(tr)
    stamps = torch.zeros(56, dtype=torch.int64, device=eng.device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rows, walls, lanes, waves = [], [], [], []
    e = eng
    for r in range(reps):
        eng.begin_epoch(np.roll(np.arange(4096, dtype=np.int32), -64 * (r % 60)))
        ev0.record()
        e.ext.fused_train_f32(e._p(e.train.images), e._p(e.train.labels), e._p(e.batch_ids), e.order_len, e.batch,
                              e._p(e.state), e._p(e.master), e._p(e.a0), e._p(e.h1), e._p(e.h2), e._p(e.z1),
                              e._p(e.z2), e._p(e.z3), e._p(e.slab), e._p(e.loss), e._p(e.correct), e._stream(),
                              stamps=stamps.data_ptr())
        ev1.record()
        torch.cuda.synchronize()
        walls.append(ev0.elapsed_time(ev1) * 1000)
        st = stamps.cpu().numpy()
        rows.append(np.diff(st[:16]) * 0.01)
        lanes.append((st[16:21] - st[[11, 11, 11, 13, 13]]) * 0.01)
        waves.append(np.concatenate([st[24:40] - st[11], st[40:56] - st[13]]) * 0.01)
    med = np.median(np.array(rows[5:]), axis=0)
    for name, v in zip(NAMES, med):
        print(f"{name:30s} {v:8.2f} us")
    print(f"{'sum (block 0)':30s} {med.sum():8.2f} us")
    lm = np.median(np.array(lanes[5:]), axis=0)
    for name, v in zip(["E: dgrad lanes done", "E: dW2 lanes done", "E: + XW copy done", "F: db1 lanes done",
                        "F: dW1 lanes done"], lm):
        print(f"  {name:28s} {v:8.2f} us after the phase start")
    wm = np.median(np.array(waves[5:]), axis=0)
    print("  E: wave w at the barrier (us after the phase start):", " ".join(f"{x:.2f}" for x in wm[:16]))
    print("  F: wave w at the barrier (us after the phase start):", " ".join(f"{x:.2f}" for x in wm[16:]))
    print(f"{'kernel wall (event)':30s} {np.median(walls[5:]):8.2f} us")


if __name__ == "__main__":
    main()
