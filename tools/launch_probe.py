"""Per-kernel cost of a chain of tiny dependent kernels, eager and inside one hipGraph.

Prints one JSON line with microseconds per kernel:
  - trivial one-workgroup kernels (torch `add_` on a 1-element tensor);
  - the same kernel on 64K elements;
  - a 1-block kernel of our own extension (`xent_kernel` via ops.layers.cross_entropy).
Runtime knobs come from the environment (e.g. HIP_FORCE_DEV_KERNARG), so run it once per
setting: python tools/launch_probe.py [label]
"""
import json
import os
import sys
import time

import torch


def per_kernel_us(fn, n, graph, reps=20):
    torch.cuda.synchronize()
    if graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(n):
                fn()
        run = g.replay
    else:
        def run():
            for _ in range(n):
                fn()
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        e0.record()
        run()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1000.0 / n)
    return round(best, 3)


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "default"
    dev = torch.device("cuda:0")
    x1 = torch.zeros(1, device=dev)
    x64k = torch.zeros(65536, device=dev)
    out = {"label": label, "env": {k: v for k, v in os.environ.items() if k.startswith(("HIP_", "DEBUG_CLR", "GPU_"))}}
    for n in (10, 100):
        out[f"tiny_graph_n{n}"] = per_kernel_us(lambda: x1.add_(1.0), n, True)
    out["tiny_eager_n100"] = per_kernel_us(lambda: x1.add_(1.0), 100, False)
    out["64k_graph_n100"] = per_kernel_us(lambda: x64k.add_(1.0), 100, True)
    try:
        sys.path.insert(0, os.getcwd())
        from distributed_neural_network_amd.ops import layers
        logits = torch.randn(64, 10, device=dev)
        labels = torch.randint(0, 10, (64,), device=dev, dtype=torch.int32)
        out["xent_graph_n100"] = per_kernel_us(lambda: layers.cross_entropy(logits, labels, None, True), 100, True)
    except Exception as e:  # the probe stays useful without the extension
        out["xent_error"] = repr(e)[:200]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    t0 = time.time()
    main()
