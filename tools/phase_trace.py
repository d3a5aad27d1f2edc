#!/usr/bin/env python3
"""Per-phase timeline of the fused training kernel (diagnostic).

Launches the fused kernel (the image-staged variant unless DNN_STAGE_IMAGES=0) with its
stamp buffer enabled: block 0 / thread 0 records
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
          "  E1 dY2 records build", "  E2 dgrad + wgrad2", "  F1 dY1 + R1 rebuild", "  F2 conv1 wgrad",
          "  A1 image landed", "  A2 R1 build + weights landed", "  A3 fc1 DMA issue + barrier"]


def pipe_main(reps: int = 50, batch: int = 64):
    """--pipe: the pipelined step's merged launch (lenet_fused.hip PIPE): reduction workgroups
    (start / end), the samples' ready waits (conv1: before phase B; conv2 + MLP: mid-phase B, the
    MLP again after phase B if it was not complete then) and the sample phases, medians over repeats of 1-step chunks (launch 1 = reduction + samples)."""
    tr = synthetic(4096, 0)
    eng = HipEngine(batch=batch, seed=0, use_graphs=False, pipeline=True, persist=False)
    eng.attach(tr)
    stamps = torch.zeros(4096 + 64, dtype=torch.int64, device=eng.device)
    eng._pipe_stamps = stamps.data_ptr()
    nrw = (eng.ext.pipe_reduce_blocks() + 1) // 2
    recs = []
    for r in range(reps):
        eng.begin_epoch(np.roll(np.arange(4096, dtype=np.int32), -64 * (r % 60)))
        stamps.zero_()
        eng.run_steps(2)  # launches: [bookkeeping + S0] [R0 + S1] [R1]; stamps from the middle one
        torch.cuda.synchronize()
        s = stamps.cpu().numpy().astype(np.float64)
        nb = nrw + batch
        bl = s[16:16 + 4 * nb].reshape(nb, 4)
        t0 = bl[:, 0].min()
        recs.append(dict(red_body=(bl[:nrw, 1] - t0) * 0.01, red_add=(bl[:nrw, 3] - t0) * 0.01,
                         poll0=(s[14] - t0) * 0.01, polls=s[15],
                         red_start=(bl[:nrw, 0] - t0) * 0.01, red_end=(bl[:nrw, 2] - t0) * 0.01,
                         smp_start=(bl[nrw:, 0] - t0) * 0.01, smp_end=(bl[nrw:, 2] - t0) * 0.01,
                         conv_ready=(s[12] - t0) * 0.01, mlp_ready=(s[13] - t0) * 0.01,
                         poll_t=[(s[4096 + 2 * k] - t0) * 0.01 if s[4096 + 2 * k] else None for k in range(12)],
                         poll_v=[int(s[4097 + 2 * k]) for k in range(12)],
                         a_done=(s[1] - t0) * 0.01, b_done=(s[2] - t0) * 0.01, c_done=(s[3] - t0) * 0.01,
                         img=(s[9] - t0) * 0.01, end0=(s[7] - t0) * 0.01))
    rr = recs[5:]
    med = lambda f: float(np.median([f(x) for x in rr]))  # noqa: E731
    # reduction WG order: conv1 group blocks 0..7 (WGs 0..3), conv2 blocks 8..44 (WGs 4..22),
    # bookkeeping (WG 22 half 1), MLP (WGs 23..56)
    print(f"  conv1 WGs (0-3) add performed med {med(lambda x: np.median(x['red_add'][:4])):.2f} max {med(lambda x: x['red_add'][:4].max()):.2f}")
    print(f"reduction WGs start med {med(lambda x: np.median(x['red_start'])):.2f} max {med(lambda x: x['red_start'].max()):.2f} us")
    print(f"  conv WGs (0-22) end med {med(lambda x: np.median(x['red_end'][:23])):.2f} max {med(lambda x: x['red_end'][:23].max()):.2f}")
    print(f"  MLP WGs (23-56) end med {med(lambda x: np.median(x['red_end'][23:])):.2f} max {med(lambda x: x['red_end'][23:].max()):.2f}")
    print(f"  conv WGs body done med {med(lambda x: np.median(x['red_body'][:23])):.2f} max {med(lambda x: x['red_body'][:23].max()):.2f}"
          f"; add performed med {med(lambda x: np.median(x['red_add'][:23])):.2f} max {med(lambda x: x['red_add'][:23].max()):.2f}")
    print(f"  MLP WGs body done med {med(lambda x: np.median(x['red_body'][23:])):.2f} max {med(lambda x: x['red_body'][23:].max()):.2f}"
          f"; add performed med {med(lambda x: np.median(x['red_add'][23:])):.2f} max {med(lambda x: x['red_add'][23:].max()):.2f}")
    print(f"  sample block 0 first conv poll {med(lambda x: x['poll0']):.2f} us, polls {med(lambda x: x['polls']):.0f}")
    print(f"sample blocks start med {med(lambda x: np.median(x['smp_start'])):.2f} max {med(lambda x: x['smp_start'].max()):.2f}"
          f"  end med {med(lambda x: np.median(x['smp_end'])):.2f} max {med(lambda x: x['smp_end'].max()):.2f} us")
    last = rr[-1]
    print("  last rep: conv adds performed (sorted):", " ".join(f"{x:.2f}" for x in sorted(last["red_add"][:23])))
    print("  last rep: conv polls (t us, count):", " ".join(f"({t:.2f},{v})" for t, v in zip(last["poll_t"], last["poll_v"])
                                                        if t is not None))
    # conv_ready: thread 0 saw conv1's flag; mlp_ready: wave 0 past its end-of-phase-B MLP check
    for k in ("img", "conv_ready", "a_done", "b_done", "mlp_ready", "c_done", "end0"):
        print(f"  sample block 0 {k:10s} {med(lambda x: x[k]):8.2f} us")


def pers_main(reps: int = 30, batch: int = 64, steps: int = 8):
    """--pers: the persistent launch (lenet_fused.hip PERS): sample block 0's phase stamps of the
    LAST step of an n-step launch, relative to that step's start (= the end of its previous step),
    and the launch's wall time per step for n = 8 and n = 64 (event timing; the difference is the
    steady-state step)."""
    tr = synthetic(8192, 0)
    eng = HipEngine(batch=batch, seed=0, use_graphs=False, pipeline=True, persist=True)
    eng.attach(tr)
    assert eng.persist, "persistent launch unavailable"
    stamps = torch.zeros(4096 + 64, dtype=torch.int64, device=eng.device)
    keys = dict(img=9, conv_ready=12, a_done=1, b_r0=1000, b_wait=1001, b_issue=1002, b_r1=1003, mlp_ready=13,
                b_done=2, c_done=3, d_done=4, dp_done=5, e1_done=8, e_done=6, f1_done=10, end=7)
    recs, walls, tl = [], {steps: [], 64: []}, []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
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
            if n == steps:
                s = stamps.cpu().numpy().astype(np.float64)
                recs.append({k: (s[i] - s[0]) * 0.01 for k, i in keys.items()})
                for nm, base in (("w_r0", 1010), ("w_r1", 1020), ("w_wait", 1040), ("w_bar", 1050)):
                    recs[-1][nm] = (s[base:base + 8] - s[0]) * 0.01
                nrw = (eng.ext.pipe_reduce_blocks() + 1) // 2
                bl = s[16:16 + 4 * (nrw + batch)].reshape(nrw + batch, 4)
                t0 = bl[:, 0].min()
                last = s[2048 + steps - 1]  # the last step's start (sample block 0)
                rw = s[2400:2400 + 4 * nrw].reshape(nrw, 4)
                cw = s[2640:2640 + 16 * 4].reshape(4, 8, 2)  # conv1 WGs x waves x (body done, drained)
                tl.append(dict(c1_body=(cw[:, :, 0] - last) * 0.01, c1_drain=(cw[:, :, 1] - last) * 0.01,
                               red_seen=(rw[:, 0] - last) * 0.01, red_body=(rw[:, 1] - last) * 0.01,
                               red_ready=(rw[:, 2] - last) * 0.01, arrive0=(s[2398] - last) * 0.01,
                               steps=(s[2048:2048 + steps] - t0) * 0.01, smp_start=(bl[nrw:, 0] - t0) * 0.01,
                               red_start=(bl[:nrw, 0] - t0) * 0.01, smp_end=(bl[nrw:, 2] - t0) * 0.01,
                               red_end=(bl[:nrw, 2] - t0) * 0.01))
    assert not eng.pipe_failed(), "a persistent-launch wait timed out"
    rr = recs[3:]
    for k in keys:
        print(f"  sample block 0, last step: {k:10s} {float(np.median([x[k] for x in rr])):8.2f} us")
    for nm in ("w_r0", "w_wait", "w_r1", "w_bar"):
        print(f"  phase B per wave {nm:6s}: " + " ".join(f"{v:6.2f}" for v in np.median([x[nm] for x in rr], axis=0)))
    med = lambda f: float(np.median([f(x) for x in tl[3:]]))  # noqa: E731
    print("launch timeline (us from the first workgroup's start, medians):")
    print(f"  workgroup starts: reduction max {med(lambda x: x['red_start'].max()):.2f}, samples max "
          f"{med(lambda x: x['smp_start'].max()):.2f}")
    print("  sample block 0 step starts: " + " ".join(f"{med(lambda x, k=k: x['steps'][k]):.2f}" for k in range(steps)))
    print(f"  samples end max {med(lambda x: x['smp_end'].max()):.2f}, reduction end med "
          f"{med(lambda x: np.median(x['red_end'])):.2f} max {med(lambda x: x['red_end'].max()):.2f}")
    print("last step's reduction (us from that step's start; sample block 0 stored its end-of-step "
          f"arrival at {med(lambda x: x['arrive0']):.2f}):")
    for name, sl in (("conv1 WGs 0-3", slice(0, 4)), ("conv2 WGs 4-22", slice(4, 23)), ("MLP WGs 23-56", slice(23, 57))):
        print(f"  {name:15s} rows seen med/max {med(lambda x: np.median(x['red_seen'][sl])):.2f}/"
              f"{med(lambda x: x['red_seen'][sl].max()):.2f}  body done {med(lambda x: np.median(x['red_body'][sl])):.2f}/"
              f"{med(lambda x: x['red_body'][sl].max()):.2f}  ready stored {med(lambda x: np.median(x['red_ready'][sl])):.2f}/"
              f"{med(lambda x: x['red_ready'][sl].max()):.2f}")
    print("  conv1 WGs per wave (us from the step's start; medians): body done / vmcnt drained")
    for w in range(4):
        print(f"    WG {w}: " + "  ".join(f"{med(lambda x, w=w, v=v: x['c1_body'][w][v]):.2f}/"
                                         f"{med(lambda x, w=w, v=v: x['c1_drain'][w][v]):.2f}" for v in range(8)))
    w8, w64 = float(np.median(walls[steps][3:])), float(np.median(walls[64][3:]))
    print(f"launch wall (events): {steps} steps {w8:.2f} us, 64 steps {w64:.2f} us -> steady step "
          f"{(w64 - w8) / (64 - steps):.3f} us")


def main(reps: int = 50, batch: int = 64):
    tr = synthetic(4096, 0)
    eng = HipEngine(batch=batch, seed=0, use_graphs=False)
    eng.attach(tr)
    eng.begin_epoch(np.arange(4096, dtype=np.int32))
    stamps = torch.zeros(16 + 4 * 1024, dtype=torch.int64, device=eng.device)
    blocks = []
    waves_e = []
    rows = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    walls = []
    for r in range(reps):
        eng.begin_epoch(np.roll(np.arange(4096, dtype=np.int32), -64 * (r % 60)))
        ev0.record()
        e = eng
        st = dict(next_ids=e._p(e.next_ids), stage=e._p(e.stage)) if e._staged else {}
        e.ext.fused_train(e._p(e.train.images), e._p(e.train.labels), e._p(e.batch_ids), e.order_len, e.batch,
                          e._p(e.state), e._p(e.master), e._p(e.shadow), e._p(e.a0), e._p(e.h1), e._p(e.h2),
                          e._p(e.z1), e._p(e.z2), e._p(e.z3), e._p(e.slab), e._p(e.loss), e._p(e.correct),
                          e._stream(), stamps=stamps.data_ptr(), **st)
        ev1.record()
        torch.cuda.synchronize()
        walls.append(ev0.elapsed_time(ev1) * 1000)
        s = stamps.cpu().numpy()
        waves_e.append((s[3000:3008] - s[8]) * 0.01)
        nb = batch
        blocks.append(s[16:16 + 4 * nb].reshape(nb, 4).copy())
        rows.append(np.concatenate([np.diff(s[:8]), [s[8] - s[5], s[6] - s[8], s[10] - s[6],
                                                      s[7] - s[10], s[9] - s[0], s[11] - s[9],
                                                      s[1] - s[11]]]) * 0.01)  # 100 MHz ticks -> us
    med = np.median(np.array(rows[5:]), axis=0)
    for name, v in zip(PHASES, med):
        print(f"{name:20s} {v:8.2f} us")
    print(f"{'sum (block 0)':20s} {med[:7].sum():8.2f} us")
    we = np.median(np.array(waves_e[5:]), axis=0)
    print("  E2 per-wave finish (us after E1):", " ".join(f"w{i}:{v:.2f}" for i, v in enumerate(we)))
    print(f"{'kernel wall (event)':20s} {np.median(walls[5:]):8.2f} us")
    # per-block timeline (us from the earliest block start), medians over repeats
    bl = np.array(blocks[5:])  # [reps, nb, 4]
    t0 = bl[:, :, 0].min(axis=1, keepdims=True)
    rel = (bl[:, :, :3] - t0[:, :, None]) * 0.01
    med_b = np.median(rel, axis=0)
    smp = med_b[:batch]
    print("sample blocks  start min/med/max %.2f/%.2f/%.2f  rows %.2f/%.2f/%.2f  end %.2f/%.2f/%.2f us" % (
        smp[:, 0].min(), np.median(smp[:, 0]), smp[:, 0].max(), smp[:, 1].min(), np.median(smp[:, 1]),
        smp[:, 1].max(), smp[:, 2].min(), np.median(smp[:, 2]), smp[:, 2].max()))
    xcc = bl[-1, :, 3]
    for x in sorted(set(xcc[:batch].tolist())):
        m = xcc[:batch] == x
        print(f"  xcc {x}: {m.sum():2d} blocks, end med {np.median(smp[m, 2]):.2f} max {smp[m, 2].max():.2f} us")
    slow = np.argsort(-smp[:, 2])[:6]
    print("  slowest blocks:", ", ".join(f"b{i}(xcc{xcc[i]}) start {smp[i, 0]:.2f} rows {smp[i, 1]:.2f} "
                                         f"end {smp[i, 2]:.2f}" for i in slow))


if __name__ == "__main__":
    if "--pers" in sys.argv:
        pers_main()
    elif "--pipe" in sys.argv:
        pipe_main()
    else:
        main()
