"""Where does the fixed cost of a SHORT timed run go?  (The driver times --steps 20 --warmup 5.)

Measures, on one GPU with the bench's engine and protocol:
  idle_sync     torch.cuda.synchronize() on an idle device
  cold          run(K) right after warmup (first replay of the largest chunk graph)
  warm          run(K) again (every graph replayed before)
  upload        same as cold, but every chunk graph was hipGraphUpload-ed after capture
  gpu_only      device-side time of a warm run(K) (events)
for chunk sizes given on the command line.  usage: python tools/short_run_probe.py [K] [W]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import EpochSampler, synthetic  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402


def make(chunk, upload):
    dev = torch.device("cuda", 0)
    eng = HipEngine(batch=64, seed=0, device=dev, graph_chunk=chunk)
    train = synthetic(50_000, 0, True)
    eng.attach(train)
    samp = EpochSampler.for_rank(len(train), 0, 1, seed=0, mode="shard")
    eng.begin_epoch(samp.order(0))
    eng.prepare_graphs()
    if upload:
        s = torch.cuda.current_stream(dev).cuda_stream
        for g in eng._graphs.values():
            eng.ext.graph_upload(g.raw_cuda_graph_exec(), s)
        torch.cuda.synchronize()
    return eng


def timed(eng, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run_steps(k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"idle_sync {1e6 * (time.perf_counter() - t0):.1f} us")
    for chunk in (64, 32, 16, 1):
        for upload in (False, True):
            eng = make(chunk, upload)
            eng.run_steps(W)
            cold = timed(eng, K)
            warm = [timed(eng, K) for _ in range(5)]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            eng.run_steps(K)
            b.record()
            torch.cuda.synchronize()
            gpu = a.elapsed_time(b) * 1e3
            steady = timed(eng, 2000) / 2000
            print(f"chunk {chunk:3d} upload {int(upload)}: cold {cold:7.1f} us ({cold / K:5.2f}/step)  "
                  f"warm {np.median(warm):7.1f} us ({np.median(warm) / K:5.2f}/step)  gpu {gpu:7.1f} us  "
                  f"steady {steady:5.2f} us/step", flush=True)
            del eng
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
