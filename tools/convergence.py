"""Convergence parity: the same reference CNN, initial weights, data and sample order trained by
the fused bf16 engine, the layer engine (fp32 and bf16 convolution operands) and the fp32 CPU
oracle (plain PyTorch); per-epoch training loss and validation accuracy side by side.

The synthetic data here uses maximal noise (so accuracy does not saturate in one epoch), and
the reference's optimiser settings (SGD lr 0.001, momentum 0.9, bs 64).  Prints a table and one
JSON line.  usage: python tools/convergence.py [--epochs 6] [--train 20000] [--test 5000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data.datasets import Split  # noqa: E402
from distributed_neural_network_amd.data.partition import EpochSampler  # noqa: E402
from distributed_neural_network_amd.models.network import init_arena  # noqa: E402
from distributed_neural_network_amd.ops import native  # noqa: E402
from distributed_neural_network_amd.runtime.engine import CpuEngine, HipEngine  # noqa: E402
from distributed_neural_network_amd.runtime.layer_engine import LayerEngine  # noqa: E402


def split(n, seed, which):
    im, lb = native.io().synthetic(n, seed, noise=255, split=which)
    return Split(torch.from_numpy(im), torch.from_numpy(lb), f"synthetic-noisy-{which}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--train", type=int, default=20000)
    ap.add_argument("--test", type=int, default=5000)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    tr, te = split(a.train, 3, 0), split(a.test, 3, 1)
    arena = init_arena(seed=17)
    sampler = EpochSampler(np.arange(a.train, dtype=np.int32), seed=5, stream=0)
    engines = {"fused bf16": lambda: HipEngine(batch=a.batch, arena=arena),
               "layers fp32": lambda: LayerEngine(batch=a.batch, model="lenet", arena=arena, device="cuda",
                                                  gemm_dtype="fp32"),
               "layers bf16": lambda: LayerEngine(batch=a.batch, model="lenet", arena=arena, device="cuda",
                                                  gemm_dtype="bf16")}
    if not a.no_cpu:
        engines["cpu fp32 (oracle)"] = lambda: CpuEngine(batch=a.batch, arena=arena)
    steps = (a.train + a.batch - 1) // a.batch
    res = {}
    for name, mk in engines.items():
        eng = mk()
        eng.attach(tr)
        curve = []
        t0 = time.perf_counter()
        for ep in range(a.epochs):
            eng.begin_epoch(sampler.order(ep))
            eng.run_steps(steps)
            st = eng.epoch_stats()
            loss, corr = eng.evaluate_samples(te)
            curve.append((st.loss_sum / max(st.batches, 1), 100.0 * float(corr.float().mean())))
        res[name] = {"train_loss": [round(c[0], 4) for c in curve], "val_acc": [round(c[1], 2) for c in curve],
                     "wall_s": round(time.perf_counter() - t0, 2)}
    names = list(res)
    print(f"{'epoch':>5s} " + " ".join(f"{n:>24s}" for n in names))
    for ep in range(a.epochs):
        print(f"{ep:5d} " + " ".join(f"{res[n]['train_loss'][ep]:11.4f} {res[n]['val_acc'][ep]:11.2f}%" for n in names))
    ref = res.get("cpu fp32 (oracle)", res["layers fp32"])
    dev = {n: max(abs(x - y) for x, y in zip(res[n]["val_acc"], ref["val_acc"])) for n in names}
    print(json.dumps({"metric": "convergence parity (val acc %, train loss per epoch)", "epochs": a.epochs,
                      "train": a.train, "test": a.test, "lr": 0.001, "momentum": 0.9, "batch": a.batch,
                      "max_val_acc_gap_vs_reference_pts": dev, "runs": res}))


if __name__ == "__main__":
    main()
