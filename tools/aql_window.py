"""Driver-shaped window timing of the persistent launch: graph replay vs direct AQL dispatch
(csrc/runtime/aql_dispatch.h), alternating in one process on the same engine state, plus the
bit check of the two paths.  One JSON line (us per step: medians; host-clock dispatch costs).

    python tools/aql_window.py [steps] [reps]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import synthetic  # noqa: E402
from distributed_neural_network_amd.models.network import init_arena  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402


def main(steps: int = 20, reps: int = 40) -> None:
    dev = torch.cuda.current_device()
    tr = synthetic(50000, 0)
    a = init_arena(seed=0)
    out = {"steps": steps}
    engs = {}
    for name in ("graph", "direct"):
        e = HipEngine(batch=64, arena=a)
        e.attach(tr)
        e.begin_epoch(np.arange(50000, dtype=np.int32))
        if name == "direct":
            why = e.ext.aql_status(dev)
            if why:
                print(json.dumps({"error": why}))
                return
            e.direct = True
        e.prepare_graphs(exact=(steps, 5))
        engs[name] = e
    # bits: the same 200 steps on both
    for e in engs.values():
        e.run_steps(200)
    torch.cuda.synchronize()
    out["bitwise"] = bool(torch.equal(engs["graph"].master, engs["direct"].master))
    wall = {k: [] for k in engs}
    left = 50000 // 64 - 200
    for r in range(reps):
        if left < steps + 6:
            for e in engs.values():
                e.begin_epoch(np.arange(50000, dtype=np.int32))
            left = 50000 // 64
        for name in (("graph", "direct") if r % 2 == 0 else ("direct", "graph")):
            e = engs[name]
            e.run_steps(5)  # the warmup right before the window, as in the bench
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e.run_steps(steps)
            torch.cuda.synchronize()
            wall[name].append(1e6 * (time.perf_counter() - t0) / steps)
        left -= steps + 5
    for k, v in wall.items():
        out[k] = {"median": round(float(np.median(v[4:])), 3), "min": round(float(min(v[4:])), 3)}
    out["direct_dispatch_us"] = {"doorbell_to_done": round(engs["direct"].ext.aql_last_us(dev, False), 2),
                                 "whole_call": round(engs["direct"].ext.aql_last_us(dev, True), 2)}
    out["window_fixed_us_saved"] = round((out["graph"]["median"] - out["direct"]["median"]) * steps, 2)
    # host cost of the direct branch's Python (run_steps before the dispatch), per call
    e = engs["direct"]
    for name, fn in (("direct_ok", e._direct_ok), ("direct_handle", lambda: e._direct(steps)),
                     ("current_stream", e._stream), ("idle_synchronize", torch.cuda.synchronize)):
        t0 = time.perf_counter()
        for _ in range(2000):
            fn()
        out.setdefault("host_us", {})[name] = round(1e6 * (time.perf_counter() - t0) / 2000, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:3]))
