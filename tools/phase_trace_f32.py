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


def pers_main(reps: int = 30, batch: int = 64, steps: int = 8):
    """--pers: the fp32 persistent launch (lenet_f32.hip PERS): sample block 0's phases of the LAST
    step of an n-step launch (relative to that step's start), its per-step hand-off stamps, the
    reduction workgroups' last step, and the wall time per step for n = 8 and n = 64."""
    tr = synthetic(8192, 0)
    eng = HipEngine(batch=batch, seed=0, use_graphs=False, dtype="fp32", persist=True)
    eng.attach(tr)
    assert eng.persist, "persistent launch unavailable"
    nwg = eng.ext.persist_wg_f32()
    stamps = torch.zeros(6400 + 32 * nwg + 64, dtype=torch.int64, device=eng.device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    walls, rows, hand, red = {steps: [], 64: []}, [], [], []
    for r in range(reps):
        for n in (steps, 64):
            eng.begin_epoch(np.roll(np.arange(8192, dtype=np.int32), -64 * (r % 60)))
            eng._pipe_stamps = stamps.data_ptr() if n == steps else 0
            stamps.zero_()
            torch.cuda.synchronize()
            ev0.record()
            eng.run_steps(n)
            ev1.record()
            torch.cuda.synchronize()
            walls[n].append(1e3 * ev0.elapsed_time(ev1))
            if n != steps:
                continue
            st = stamps.cpu().numpy().astype(np.float64)
            start = st[2048:2048 + steps]
            rows.append(np.diff(st[:16]) * 0.01)
            # per step s >= 1: wait (start -> ready passed), MLP / conv arrival after the start
            hand.append(np.stack([(st[3072:3072 + steps] - start), (st[4096:4096 + steps] - start),
                                  (st[5120:5120 + steps] - start), np.r_[np.diff(start), np.nan]]) * 0.01)
            last = start[-1]
            rw = st[6144:6144 + 4 * nwg].reshape(nwg, 4)
            pw = st[6400:6400 + 32 * nwg].reshape(nwg, 16, 2)
            red.append(dict(wbody=(pw[:, :, 0] - last) * 0.01, wdrain=(pw[:, :, 1] - last) * 0.01,
                            seen=(rw[:, 0] - last) * 0.01, body=(rw[:, 1] - last) * 0.01,
                            ready=(rw[:, 2] - last) * 0.01, arrive=(st[5120 + steps - 1] - last) * 0.01))
    assert not eng.pipe_failed(), "a persistent-launch wait timed out"
    med = np.median(np.array(rows[3:]), axis=0)
    print("sample block 0, last step (us per phase):")
    for name, v in zip(NAMES, med):
        print(f"  {name:30s} {v:8.2f}")
    h = np.nanmedian(np.array(hand[3:]), axis=0)  # [4][steps]
    print("sample block 0 per step (us from the step's start; medians): ready passed / MLP arrival / "
          "conv arrival / step length")
    for s in range(steps):
        print(f"  step {s}: " + " ".join(f"{h[k][s]:7.2f}" for k in range(4)))
    m = lambda f: float(np.median([f(x) for x in red[3:]]))  # noqa: E731
    print(f"last step's reduction (us from that step's start; sample 0 stored its conv arrival at "
          f"{m(lambda x: x['arrive']):.2f}):")
    cw = eng.ext.persist_conv_wg_f32()
    for name, sl in ((f"conv WGs 0-{cw - 1}", slice(0, cw)), (f"MLP WGs {cw}-", slice(cw, nwg))):
        print(f"  {name:14s} rows seen med/max {m(lambda x: np.median(x['seen'][sl])):.2f}/"
              f"{m(lambda x: x['seen'][sl].max()):.2f}, body done {m(lambda x: np.median(x['body'][sl])):.2f}/"
              f"{m(lambda x: x['body'][sl].max()):.2f}, ready stored {m(lambda x: np.median(x['ready'][sl])):.2f}/"
              f"{m(lambda x: x['ready'][sl].max()):.2f}")
    print("per workgroup, the slowest wave (us from the last step's start): body done / drained")
    for w in range(nwg):
        print(f"  WG {w:2d}: {m(lambda x, w=w: x['wbody'][w].max()):6.2f} / {m(lambda x, w=w: x['wdrain'][w].max()):6.2f}"
              f"   (waves: " + " ".join(f"{m(lambda x, w=w, v=v: x['wbody'][w][v]):.2f}" for v in range(16)) + ")")
    w8, w64 = np.median(walls[steps][3:]), np.median(walls[64][3:])
    print(f"wall: {steps} steps {w8:.1f} us, 64 steps {w64:.1f} us -> steady step {(w64 - w8) / (64 - steps):.2f} us")


if __name__ == "__main__":
    if "--pers" in sys.argv:
        pers_main()
    else:
        main()
