"""Worker launched (one process per rank) by tests/test_distributed_cpu.py."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import EpochSampler, synthetic  # noqa: E402
from distributed_neural_network_amd.models.network import init_arena  # noqa: E402
from distributed_neural_network_amd.parallel import Communicator, make_policy  # noqa: E402
from distributed_neural_network_amd.runtime import CpuEngine  # noqa: E402


def failvote(out: str) -> None:
    """Only rank 1's (fake) one-shot all-reduce reports a failed wait: the epoch-end vote must
    raise CommError on EVERY rank, so all of them enter recovery together."""
    from distributed_neural_network_amd.parallel import CommError

    comm = Communicator(device="cpu")

    class _Sync:
        def failed(self):
            return comm.rank == 1

    eng = CpuEngine(batch=4, arena=init_arena(seed=0))
    policy = make_policy("step-allreduce", comm)
    policy.attach(eng)
    eng.grad_sync = _Sync()
    try:
        policy.epoch_end(eng, 0)
        raised = ""
    except CommError as e:
        raised = str(e)
    with open(os.path.join(out, f"vote{comm.rank}.txt"), "w") as f:
        f.write(raised)
    comm.close()


def ab(out: str) -> None:
    """The all-reduce start-up A/B (parallel/autotune.py) over gloo with three test paths: the
    real host all-reduce, a slower copy of it, and one that fails its install on rank 1 only.
    Every rank must pick the same (fastest passing) path and get its start parameters back."""
    import time

    from distributed_neural_network_amd.parallel import StepAllReduce
    from distributed_neural_network_amd.parallel.autotune import allreduce_ab
    from distributed_neural_network_amd.parallel.comm import GradAllReduce
    from distributed_neural_network_amd.runtime.cursor import EpochCursor

    comm = Communicator(device="cpu")

    class Slow(GradAllReduce):
        def allreduce_grads(self, grad, buckets, before_last=None):
            time.sleep(0.004)
            super().allreduce_grads(grad, buckets, before_last)

    class Policy(StepAllReduce):
        def install(self, engine, name):
            if name == "slow":
                engine.grad_sync = Slow(self.comm)
                return True
            if name == "flaky":  # agreed outcome: fails everywhere because rank 1 failed
                return all(v == 1.0 for v in self.comm.gather_scalars(0.0 if self.comm.rank == 1 else 1.0))
            return super().install(engine, name)

    data = synthetic(256, 3)
    eng = CpuEngine(batch=16, lr=0.05, momentum=0.9, arena=init_arena(seed=comm.rank + 100))
    eng.attach(data)
    policy = Policy(comm)
    policy.attach(eng)
    policy.initial_broadcast(eng)
    start = eng.master.clone()
    samp = EpochSampler.for_rank(256, comm.rank, comm.world, seed=1, mode="shard")
    cur = EpochCursor(eng, samp, policy, 16)
    res = allreduce_ab(policy, eng, cur, steps=6, warmup=2, reps=2, spin=4, candidates=("torch-pg", "slow", "flaky"))
    restored = bool(torch.equal(eng.master, start))
    cur.run(3)  # the adopted path trains: replicas stay identical
    torch.save({"master": eng.master, "res": res, "restored": restored, "path": policy.path},
               os.path.join(out, f"ab{comm.rank}.pt"))
    comm.close()


def main(mode: str, out: str, n: int, batch: int, epochs: int) -> None:
    torch.set_num_threads(1)
    if mode == "failvote":
        return failvote(out)
    if mode == "ab":
        return ab(out)
    comm = Communicator(device="cpu")
    data = synthetic(n, 3)
    eng = CpuEngine(batch=batch, lr=0.05, momentum=0.9, arena=init_arena(seed=comm.rank + 100))  # differ on purpose
    eng.attach(data)
    policy = make_policy(mode, comm)
    policy.attach(eng)
    policy.initial_broadcast(eng)  # rank 0's init wins
    samp = EpochSampler.for_rank(n, comm.rank, comm.world, seed=1, mode="shard", parent=mode == "parent",
                                 shuffle=False)
    for ep in range(epochs):
        policy.epoch_start(eng, ep)
        if policy.trains():
            eng.begin_epoch(samp.order(ep))
            eng.run_steps(samp.steps(batch))
        policy.epoch_end(eng, ep)
    torch.save({"master": eng.master, "rank": comm.rank}, os.path.join(out, f"rank{comm.rank}.pt"))
    comm.close()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
