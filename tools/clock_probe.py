"""Does a short timed window start on a clocked-down GPU?  The bench protocol (W warmup steps,
sync, K timed steps, sync) after the device sat idle for `idle` seconds, with and without a
`busy` ms burst of training steps before the warmup.  usage: python tools/clock_probe.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import EpochSampler, synthetic  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402


def main():
    K, W = 20, 5
    dev = torch.device("cuda", 0)
    train = synthetic(50_000, 0, True)
    samp = EpochSampler.for_rank(len(train), 0, 1, seed=0, mode="shard")
    eng = HipEngine(batch=64, seed=0, device=dev, graph_chunk=64)
    eng.attach(train)
    eng.begin_epoch(samp.order(0))
    eng.prepare_graphs()
    for idle in (0.0, 0.05, 0.5, 2.0):
        for busy_steps in (0, 500):
            walls = []
            for _ in range(5):
                eng.begin_epoch(samp.order(0))
                torch.cuda.synchronize()
                time.sleep(idle)
                if busy_steps:
                    eng.run_steps(busy_steps)
                    eng.begin_epoch(samp.order(0))
                eng.run_steps(W)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                eng.run_steps(K)
                torch.cuda.synchronize()
                walls.append((time.perf_counter() - t0) * 1e6)
            print(f"idle {idle:4.2f} s, busy {busy_steps:3d} steps before warmup: K={K} wall median "
                  f"{np.median(walls):6.1f} us ({np.median(walls) / K:5.2f}/step)  all {[round(w) for w in walls]}",
                  flush=True)


if __name__ == "__main__":
    main()
