"""4-rank (one GPU) training probe of the xGMI exchange forms: 2 epochs, per-epoch wall time,
the error word after each epoch.  Run under torch.distributed.run with DNN_BACKEND=gloo."""
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import EpochSampler, synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.parallel import Communicator, make_policy
from distributed_neural_network_amd.runtime import HipEngine
torch.cuda.set_device(0)
comm = Communicator(device=torch.device("cuda", 0))
data = synthetic(2048, 3)
eng = HipEngine(batch=64, arena=init_arena(seed=11), graph_chunk=8, use_graphs=True)
eng.attach(data)
pol = make_policy("step-allreduce", comm)
pol.attach(eng)
pol.initial_broadcast(eng)
g = eng.grad_sync.group
samp = EpochSampler.for_rank(len(data), comm.rank, comm.world, seed=1, mode="shard")
for ep in range(int(os.environ.get("EPOCHS", "4"))):
    t = time.time()
    pol.epoch_start(eng, ep)
    eng.begin_epoch(samp.order(ep))
    eng.run_steps(samp.steps(64))
    eng.synchronize()
    print(f"rank {comm.rank} ep {ep} mode={g.xp_mode} ar_mode={g.ar_mode} one={g.one_launch} "
          f"{time.time() - t:.3f}s failed={g.failed()} ctr0={int(g.xp_ctr[0])}", file=sys.stderr, flush=True)
comm.close()
