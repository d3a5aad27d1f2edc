"""Diagnostic (2 ranks on one GPU, gloo + xGMI one-launch exchange): parameters after 1, 2 and 3
steps, early-MLP in-launch vs serial, from the same start; prints per-tensor max diffs."""
import os
import pathlib
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, ROOT)
W = r'''
import os, numpy as np, torch
from distributed_neural_network_amd.data import EpochSampler, synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.parallel import Communicator, make_policy
torch.cuda.set_device(0)
comm = Communicator(device=torch.device("cuda", 0))
from distributed_neural_network_amd.runtime import HipEngine
data = synthetic(2048, 3)
eng = HipEngine(batch=64, arena=init_arena(seed=11), graph_chunk=8, use_graphs=os.environ["GRAPHS"] == "1")
eng.attach(data)
pol = make_policy("step-allreduce", comm)
pol.attach(eng)
pol.initial_broadcast(eng)
samp = EpochSampler.for_rank(len(data), comm.rank, comm.world, seed=1, mode="shard")
out = []
for ep in range(2):
    pol.epoch_start(eng, ep)
    eng.begin_epoch(samp.order(ep))
    if os.environ["SPLIT"] == "1":
        for k in range(2):
            eng.run_steps(8)
            eng.synchronize()
            out.append(eng.master.cpu().clone())
    else:
        eng.run_steps(16)
        eng.synchronize()
        out += [eng.master.cpu().clone()] * 2
    pol.epoch_end(eng, ep)
torch.save(out, os.path.join(os.environ["OUT"], f"r{comm.rank}.pt"))
comm.close()
'''
tmp = pathlib.Path(tempfile.mkdtemp())
(tmp / "w.py").write_text(W)
res = {}
for early, graphs, split, port in (("0", "1", "0", 29711), ("1", "1", "0", 29713), ("1", "0", "0", 29715),
                                  ("1", "1", "1", 29717)):
    out = tmp / (early + graphs + split)
    out.mkdir()
    env = dict(os.environ, PYTHONPATH=ROOT, DNN_BACKEND="gloo", DNN_ALLREDUCE="xgmi", OMP_NUM_THREADS="2", OUT=str(out),
               DNN_EARLY_MLP=early, DNN_XGMI_EXCHANGE="pull", GRAPHS=graphs, SPLIT=split)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(tmp / "w.py")],
                       env=env, capture_output=True, text=True, timeout=300)
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(1)
    res[early + graphs + split] = [torch.load(out / f"r{i}.pt", weights_only=True) for i in range(2)]
from distributed_neural_network_amd.models.network import LAYOUT  # noqa: E402
for key in ("110", "100", "111"):
    for k in range(4):
        d = (res[key][0][k] - res["010"][0][k]).abs()
        parts = {n: float(d[o:o + int(torch.Size(LAYOUT.shapes[n]).numel())].max()) for n, o in LAYOUT.offsets.items()}
        print("early, graphs", key[1], "split", key[2], "after", 8 * (k + 1), "steps vs serial (rank 0):", {n: v for n, v in parts.items() if v},
              "| replicas equal:", torch.equal(res[key][0][k], res[key][1][k]))
