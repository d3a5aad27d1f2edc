"""Diagnostic: rebuild the xGMI group across communicator generations and check that the
one-shot all-reduce still equals a host all-reduce of the same random data.

    DNN_BACKEND=gloo torchrun --nproc-per-node 2 tools/xgmi_reform_check.py [--close-first]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.parallel import Communicator  # noqa: E402
from distributed_neural_network_amd.parallel import xgmi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--close-first", action="store_true", help="free the old group before building the new one")
ap.add_argument("--gens", type=int, default=3)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
torch.cuda.set_device(0)
comm = Communicator(device=torch.device("cuda", 0))
old = None
bad = 0
for gen in range(a.gens):
    if gen:
        comm.reform([])  # same members, new generation (what recovery does minus the death)
    if old is not None and a.close_first:
        old.close()
    grp = xgmi.build_group(comm, 62_400)
    assert grp is not None, "group refused"
    if old is not None and not a.close_first:
        old.close()
    old = grp
    g = torch.Generator(device="cpu").manual_seed(1234 + gen)
    for s in range(a.steps):
        x = torch.randn(62_400, generator=g) * (comm.rank + 1)
        t = x.cuda()
        grp.allreduce_(t)
        torch.cuda.synchronize()
        ref = x.clone()
        comm.allreduce_(ref, "sum")
        ref = ref * (1.0 / comm.world)
        err = float((t.cpu() - ref).abs().max())
        if err > 1e-5 or grp.failed():
            bad += 1
            print(f"rank {comm.rank} gen {gen} step {s}: max err {err} failed={grp.failed()} "
                  f"regions={[hex(r) for r in grp.regions]}", flush=True)
print(f"rank {comm.rank}: {'OK' if bad == 0 else f'{bad} BAD steps'}", flush=True)
comm.close()
sys.exit(1 if bad else 0)
