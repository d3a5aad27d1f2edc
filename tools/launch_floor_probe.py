"""The fixed cost of a timed window: what one launch + synchronize costs, whatever the kernel does.

`tools/window_host_probe.py` (profiles/r6/window/) shows the bench's 20/5 window pays ~26 us over
its 20 kernel steps, and a graph of ONE trivial kernel pays the same ~25 us between launch and the
synchronize's return: the fixed cost is the runtime's launch / completion path, not the kernel.
This probe measures that floor, and the persistent 20-step window, under the HIP / HSA runtime
settings of this process (run it once per setting: they are read when the runtime starts), in
microseconds, medians:

    idle_sync      torch.cuda.synchronize() on an idle device
    eager_trivial  launch of one 1-element add + synchronize
    graph_trivial  graph replay of that kernel + synchronize (gpu: events around the replay)
    window20       graph replay of the persistent 20-step window + synchronize (bench-shaped)

    python tools/launch_floor_probe.py        # one JSON line (the runtime env it ran under included)
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import synthetic  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402

KNOBS = ("AMD_DIRECT_DISPATCH", "ROC_ACTIVE_WAIT_TIMEOUT", "ROC_SYSTEM_SCOPE_SIGNAL", "HSA_ENABLE_INTERRUPT",
         "DEBUG_CLR_GRAPH_PACKET_CAPTURE", "ROC_CPU_WAIT_FOR_SIGNAL", "DEBUG_HIP_BLOCK_SYNC",
         "GPU_FORCE_QUEUE_PROFILING", "ROC_SKIP_KERNEL_ARG_COPY", "HIP_FORCE_DEV_KERNARG", "DNN_SYNC_SPIN")


def med(v, skip=10):
    return round(float(np.median(v[skip:])), 2)


def main(reps: int = 60) -> None:
    dev = torch.device("cuda:0")
    x = torch.zeros(1, device=dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        x.add_(1)
        torch.cuda.synchronize()
        tg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(tg, stream=s):
            x.add_(1)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    idle, eager, gw, gg = [], [], [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        idle.append(1e6 * (time.perf_counter() - t0))
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        eager.append(1e6 * (time.perf_counter() - t0))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tg.replay()
        torch.cuda.synchronize()
        gw.append(1e6 * (time.perf_counter() - t0))
        ev0.record()
        tg.replay()
        ev1.record()
        torch.cuda.synchronize()
        gg.append(1e3 * ev0.elapsed_time(ev1))

    tr = synthetic(50000, 0)
    eng = HipEngine(batch=64, seed=0)
    eng.attach(tr)
    spe = 50000 // 64
    eng.begin_epoch(np.arange(50000, dtype=np.int32))
    eng.prepare_graphs(exact=(20,))
    g = eng._graph(20)
    left = spe
    win = []
    for _ in range(30):
        if left < 21:
            eng.begin_epoch(np.arange(50000, dtype=np.int32))
            left = spe
        g.replay()  # warm-up step chunk right before the window, as in the bench
        left -= 20
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        win.append(1e6 * (time.perf_counter() - t0))
        left -= 20
    print(json.dumps({"env": {k: os.environ[k] for k in KNOBS if k in os.environ},
                      "persistent": bool(eng._pers_ok()),
                      "idle_sync": med(idle), "eager_trivial": med(eager),
                      "graph_trivial": {"wall": med(gw), "gpu": med(gg)},
                      "window20": {"wall": med(win, 5), "per_step": round(med(win, 5) / 20, 3),
                                   "min": round(min(win[5:]), 2)}}))


if __name__ == "__main__":
    main()
