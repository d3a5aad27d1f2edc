"""Host-side cost of the bench's timed window (diagnostic).

The persistent launch runs a 20-step window as ONE kernel, so whatever the window measures beyond
the kernel is host work: the Python dispatch, the graph (or kernel) launch, and the wake-up of the
final synchronize.  For each way of launching the window this prints, in microseconds (medians over
repeats): ``submit`` (host time until the launch call returns), ``wall`` (launch + synchronize, as
the bench times it), ``gpu`` (events around the launch) and ``wall - gpu``.

    python tools/window_host_probe.py [steps]
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


def main(steps: int = 20, reps: int = 40) -> None:
    tr = synthetic(50000, 0)
    eng = HipEngine(batch=64, seed=0)
    eng.attach(tr)
    spe = 50000 // 64
    eng.begin_epoch(np.arange(50000, dtype=np.int32))
    eng.prepare_graphs(exact=(steps,))
    left = spe
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def graph_replay():
        eng.run_steps(steps)

    g = eng._graph(steps)

    def raw_replay():
        g.replay()

    def eager():
        with torch.cuda.device(eng.device):
            eng._launch_steps(steps)

    res = {"persistent": bool(eng._pers_ok()), "steps": steps}
    for name, fn, sync in (("run_steps", graph_replay, "device"), ("graph.replay", raw_replay, "device"),
                           ("eager", eager, "device"), ("graph.replay+event", raw_replay, "event"),
                           ("graph.replay+spin", raw_replay, "spin")):
        sub, wall, gpu = [], [], []
        for r in range(reps):
            if left < steps + 1:
                eng.begin_epoch(np.arange(50000, dtype=np.int32))
                left = spe
            torch.cuda.synchronize()
            ev0.record()
            t0 = time.perf_counter()
            fn()
            t1 = time.perf_counter()
            ev1.record()
            if sync == "device":
                torch.cuda.synchronize()
            elif sync == "event":
                ev1.synchronize()
            else:
                while not ev1.query():
                    pass
            t2 = time.perf_counter()
            left -= steps
            sub.append(1e6 * (t1 - t0))
            wall.append(1e6 * (t2 - t0))
            gpu.append(1e3 * ev0.elapsed_time(ev1))
        m = lambda v: round(float(np.median(v[5:])), 2)  # noqa: E731
        res[name] = {"submit": m(sub), "wall": m(wall), "gpu": m(gpu),
                     "wall_minus_gpu": round(m(wall) - m(gpu), 2)}

    # the floor: the same launch + synchronize around a graph of ONE trivial kernel, and an idle
    # synchronize - what any window pays whatever the kernel does
    x = torch.zeros(1, device=eng.device)
    s = torch.cuda.Stream(eng.device)
    with torch.cuda.stream(s):
        x.add_(1)
        torch.cuda.synchronize()
        tg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(tg, stream=s):
            x.add_(1)
    torch.cuda.synchronize()
    idle, fw, fg = [], [], []
    for r in range(200):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        idle.append(1e6 * (time.perf_counter() - t0))
        ev0.record()
        t0 = time.perf_counter()
        tg.replay()
        ev1.record()
        torch.cuda.synchronize()
        fw.append(1e6 * (time.perf_counter() - t0))
        fg.append(1e3 * ev0.elapsed_time(ev1))
    m = lambda v: round(float(np.median(v[20:])), 2)  # noqa: E731
    res["idle_synchronize"] = m(idle)
    res["trivial_graph"] = {"wall": m(fw), "gpu": m(fg)}

    # the persistent launch's own fixed cost: GPU time (events) and wall per window length
    sweep = {}
    for n in (1, 2, 4, 8, steps):
        eng.prepare_graphs(exact=(n,))
        gn = eng._graph(n)
        wall, gpu = [], []
        for r in range(30):
            if left < n + 1:
                eng.begin_epoch(np.arange(50000, dtype=np.int32))
                left = spe
            torch.cuda.synchronize()
            ev0.record()
            t0 = time.perf_counter()
            gn.replay()
            ev1.record()
            torch.cuda.synchronize()
            wall.append(1e6 * (time.perf_counter() - t0))
            gpu.append(1e3 * ev0.elapsed_time(ev1))
            left -= n
        sweep[n] = {"wall": round(float(np.median(wall[5:])), 2), "gpu": round(float(np.median(gpu[5:])), 2)}
    ns = sorted(sweep)
    a = np.polyfit(ns, [sweep[n]["gpu"] for n in ns], 1)
    b = np.polyfit(ns, [sweep[n]["wall"] for n in ns], 1)
    res["steps_sweep"] = {str(n): v for n, v in sweep.items()}
    res["fit_gpu_us"] = {"per_step": round(float(a[0]), 3), "fixed": round(float(a[1]), 2)}
    res["fit_wall_us"] = {"per_step": round(float(b[0]), 3), "fixed": round(float(b[1]), 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
