#!/usr/bin/env python3
"""Headline benchmark: whole-node training images/sec + epoch time (BASELINE.json).

Config: reference CIFAR-10 CNN (models/model.py Network, 62,006 params), batch 64
per GPU (weak scaling), synthetic CIFAR-shaped data (50,000 train / 10,000 test,
3x32x32 uint8 -> normalised in-kernel), random-init weights, bf16 MFMA operands
with fp32 master weights/accumulation, momentum SGD (lr 0.001, m 0.9) every step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--sync step-allreduce|epoch-avg]

Synchronisation defaults to a per-step gradient all-reduce inside the step hipGraph.  At N > 1
the bench first MEASURES its transport (--allreduce ab, parallel/autotune.py): in the untimed
set-up it times every candidate with the timed window's own shape (one exact-size graph of K
steps inside one epoch, W warmup steps, 3 windows, median) - the one-launch xGMI exchange in
its one-hop (xgmi-pull) and two-hop (xgmi-rsag) forms inside the batch-reduction kernel, native
ncclAllReduce of one fused bucket (rccl) and of two buckets with the MLP bucket on a side stream
(rccl-overlap) - plus the no-all-reduce step as the baseline, takes the max over ranks, and all
ranks adopt the fastest path that passed its self-test.  The JSON line reports every
candidate's us/step (allreduce_ab), the chosen path and the per-step exchange wait measured
inside the kernel (s_memrealtime around the granule wait; median / p99 over the timed steps,
max over ranks).  --sync epoch-avg runs the reference algorithm
(data_parallelism_train.py:185-254): local SGD over the rank's shard with a fresh momentum
buffer per epoch and an RCCL parameter all-reduce at every epoch end (epoch boundaries fall
inside the timed window: 50,000 / N samples per rank and epoch).

For N > 1 it runs one rank per GPU (RCCL over xGMI): under torchrun / mpiexec /
parallel/launch.py, or - plain ``python bench.py --gpus N`` - it launches its own N ranks
before anything touches the GPU (parallel/selflaunch.py) and relays rank 0's JSON line.
W untimed warmup steps, then EXACTLY K timed optimizer steps bracketed by barrier + device
sync; epoch boundaries inside the window re-shuffle and continue (no step is skipped).
The max over ranks is reported.  Rank 0 prints one JSON line; every rank prints a stamped
start-up trace to stderr (store / process group, native RCCL, xGMI IPC map, each A/B
candidate), so a stalled multi-GPU start shows where it sits.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_neural_network_amd.hsa_env import DEFAULTS as HSA_DEFAULTS, apply as _hsa_env  # noqa: E402

_hsa_env()  # HSA runtime defaults, before torch can start the runtime (hsa_env.py)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_neural_network_amd.data import EpochSampler, synthetic  # noqa: E402
from distributed_neural_network_amd.data.datasets import SYNTH_NOISE_HARD  # noqa: E402
from distributed_neural_network_amd.parallel import Communicator, detect, make_policy  # noqa: E402
from distributed_neural_network_amd.parallel import selflaunch  # noqa: E402
from distributed_neural_network_amd.parallel.autotune import (BF16_PATHS, ORDER, PERS_PATHS, ab_window,  # noqa: E402
                                                              allreduce_ab, default_candidates, launch_ab)
from distributed_neural_network_amd.runtime import HipEngine, eval_metrics, make_engine  # noqa: E402
from distributed_neural_network_amd.runtime.cursor import EpochCursor  # noqa: E402

BASELINE_IMG_S = 1261.0  # BASELINE.md headline: bs64, "4 procs", training-phase whole-node img/s
METRIC = "images/sec (whole node) + epoch time, CIFAR-10 CNN bs=64 at 1/2/4/8 MI355X"
_T0 = time.time()


def stamp(rank: int, msg: str) -> None:
    """Start-up trace line on stderr (seconds since this process started)."""
    print(f"[bench r{rank} +{time.time() - _T0:.3f}s] {msg}", file=sys.stderr, flush=True)


def _reserve_stdout() -> int:
    """Route fd 1 to stderr for the whole run and return a private handle on the real
    stdout: RCCL (and other native libraries) print banners with printf, and the driver
    expects exactly ONE line - the JSON result - on stdout."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    return real


def main():
    out_fd = _reserve_stdout()
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5000)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--batch-size", type=int, default=64, help="per-GPU batch")
    ap.add_argument("--sync", default="step-allreduce", choices=["step-allreduce", "epoch-avg"],
                    help="step-allreduce (default, the performance path) = DDP-style per-step gradient "
                         "all-reduce over RCCL; epoch-avg = the reference data_parallelism_train.py algorithm: "
                         "local momentum-SGD steps on each shard, parameters all-reduced (avg) at every epoch end")
    ap.add_argument("--graph-chunk", type=int, default=64)
    ap.add_argument("--overlap", action="store_true",
                    help="2 gradient buckets, MLP all-reduce overlapped with the conv-bucket reduction "
                         "(default: one fused bucket - the 248 KB all-reduce is latency-bound)")
    ap.add_argument("--allreduce", default="ab", choices=("ab",) + ORDER + PERS_PATHS + BF16_PATHS + ("default",),
                    help="per-step all-reduce at N > 1: ab (default) = time every candidate in the untimed "
                         "set-up and keep the fastest; a path name pins it; default = the policy's own choice")
    ap.add_argument("--launch", default="ab", choices=("ab", "direct", "graph"),
                    help="how the persistent window is launched (bf16 engine, no per-step all-reduce): ab "
                         "(default) = time the direct AQL dispatch and the graph replay in the untimed set-up "
                         "and keep the faster; direct / graph pin one")
    ap.add_argument("--grad-comm", default="fp32", choices=("fp32", "bf16"),
                    help="bf16: the A/B also times the xGMI exchanges with bf16 gradient granules (opt-in "
                         "lower-precision gradient communication; the default path becomes its -bf16 form)")
    ap.add_argument("--ab-steps", type=int, default=0,
                    help="timed steps per A/B window (0: the timed window's own --steps, capped at 256); every "
                         "candidate is timed exactly like the reported window (parallel/autotune.py)")
    ap.add_argument("--ab-reps", type=int, default=3, help="A/B windows per candidate and round (median)")
    ap.add_argument("--noise", type=int, default=SYNTH_NOISE_HARD,
                    help="synthetic data noise amplitude (255: the hard split of tools/convergence.py, so the "
                         "epoch's val_acc / val_loss carry signal; 96: the easy template set)")
    ap.add_argument("--model", default="lenet", help="lenet (headline) | lenet-bn | cifar-vgg (layer engine)")
    ap.add_argument("--engine", default="auto", choices=["auto", "fused", "layers"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="bf16: bf16 MFMA operands, fp32 accumulation / master weights (lenet_fused.hip); fp32: "
                         "fp32 operands throughout, the reference's arithmetic (lenet_f32.hip)")
    ap.add_argument("--no-epoch", action="store_true", help="skip the full-epoch timing")
    ap.add_argument("--no-graphs", action="store_true",
                    help="eager launches (needed with DNN_BACKEND=gloo, whose collectives are not capturable)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--diag-windows", type=int, default=0,
                    help="diagnostic: time this many extra K-step windows after the reported one (stderr)")
    ap.add_argument("--train-samples", type=int, default=50_000,
                    help="synthetic training-set size (CIFAR-10: 50,000); smaller = more epoch boundaries "
                         "inside the timed window (diagnostic)")
    args = ap.parse_args()

    me = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    if args.gpus > 1 and not selflaunch.launcher_present():
        # no launcher: become one (nothing has touched the GPU yet; children, never an exec); a job
        # that ends without a result is retried in fresh ranks with a conservative transport
        sys.exit(selflaunch.run(me, args.gpus, out_fd=out_fd))
    if selflaunch.supervisor_wanted():
        # a torchrun rank: supervise the real rank as a child (same retry plan, coordinated
        # through torchrun's store) - this process never touches the GPU
        sys.exit(selflaunch.supervise(me, out_fd=out_fd))
    selflaunch.die_with_parent()  # (a self-launched rank: dies with its launcher; no-op otherwise)
    # a retry attempt of the launcher (parallel/selflaunch.py ATTEMPTS): no xGMI group and no
    # A/B (level 1: native RCCL, or the process group under gloo); level 2 adds eager launches
    # (gloo host collectives cannot be captured)
    safe = int(os.environ.get("DNN_SAFE_TRANSPORT", "0") or 0)
    if safe:
        args.allreduce = "default"
        if safe >= 2:
            args.no_graphs = True
    os.environ.setdefault("DNN_STARTUP_TRACE", "1")
    env = detect()
    if env.world != args.gpus:
        stamp(env.rank, f"note: --gpus {args.gpus} but the launcher started {env.world} ranks; using {env.world}")
    dev_index = env.local_rank % torch.cuda.device_count()  # 1 GPU per rank (wraps only in tests)
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    stamp(env.rank, f"rank {env.rank}/{env.world} on cuda:{dev_index}; rendezvous {env.master_addr}:{env.master_port}")
    comm = Communicator(env, device)
    if comm.distributed:
        stamp(env.rank, f"store + process group ({comm.backend}) up")
    B = args.batch_size

    train = synthetic(args.train_samples, args.seed, True, noise=args.noise)
    test = synthetic(10_000, args.seed, False, noise=args.noise)
    sampler = EpochSampler.for_rank(len(train), comm.rank, comm.world, seed=args.seed, mode="shard")
    if args.model == "lenet" and args.engine in ("auto", "fused"):
        engine = HipEngine(batch=B, seed=args.seed, device=device, graph_chunk=args.graph_chunk,
                           overlap=args.overlap, use_graphs=not args.no_graphs, dtype=args.dtype)
    else:  # modular layer engine (other models / fp32)
        engine = make_engine(str(device), B, 0.001, 0.9, seed=args.seed, model=args.model, engine="layers",
                             dtype=args.dtype, graph_chunk=min(args.graph_chunk, 16), use_graphs=not args.no_graphs)
    engine.attach(train)
    test_dev = test.to(device)
    policy = make_policy(args.sync, comm)
    policy.lazy_check = True  # no per-epoch host sync; the xGMI error word is checked after the run
    policy.record_waits = True  # per-step exchange wait stamps (one store per wave and step)
    policy.grad_comm = args.grad_comm
    if args.allreduce in ORDER + PERS_PATHS + BF16_PATHS:
        policy.path = args.allreduce
    stamp(comm.rank, f"engine {type(engine).__name__} ready; installing the all-reduce path")
    policy.attach(engine)
    policy.initial_broadcast(engine)
    if comm.distributed:
        stamp(comm.rank, f"all-reduce path {policy.installed(engine) if hasattr(policy, 'installed') else None}; "
                         "initial broadcast done")
    cur = EpochCursor(engine, sampler, policy, B)
    # first-call costs of the eval path (kernel, D2H, host ops) - before the A/B too: a full-chip
    # kernel, after which the A/B's candidates run on the GPU state the timed window will see
    if not args.no_epoch:
        wl, wc = engine.evaluate_samples(test_dev, 0, len(test))
        wl2, wc2 = torch.zeros_like(wl), torch.zeros_like(wc, dtype=torch.float32)
        comm.allreduce_(wl2, "sum")
        eval_metrics(wl + wl2, wc.float() + wc2, B)
    ab = {}
    if comm.distributed and args.sync == "step-allreduce" and args.allreduce == "ab":
        ab_steps, ab_warm = ab_window(cur.steps_per_epoch, args.ab_steps or args.steps, args.warmup)
        ab = allreduce_ab(policy, engine, cur, steps=ab_steps, warmup=ab_warm, reps=args.ab_reps,
                          candidates=default_candidates(args.grad_comm),
                          log=lambda m: stamp(comm.rank, m) if comm.rank == 0 else None)
        stamp(comm.rank, f"all-reduce A/B (us/step, max over ranks): {ab}")
        cur.left = 0  # the timed run starts on a fresh epoch

    # the persistent window's launch path (direct AQL dispatch vs graph replay), timed like the
    # all-reduce A/B above with the run's own window shape (untimed; engines without a per-step
    # all-reduce only)
    lab = {}
    if args.launch == "ab" and isinstance(engine, HipEngine):
        ab_steps, ab_warm = ab_window(cur.steps_per_epoch, args.ab_steps or args.steps, args.warmup)
        lab = launch_ab(comm, engine, cur, steps=ab_steps, warmup=ab_warm,
                        log=lambda m: stamp(comm.rank, m) if comm.rank == 0 else None)
        if lab:
            stamp(comm.rank, f"launch A/B (us/step, max over ranks): {lab}")
            cur.left = 0
    elif args.launch == "graph" and isinstance(engine, HipEngine):
        engine.direct = False

    # untimed set-up: capture every chunk graph (or prepare the direct dispatches), then the W
    # warmup steps LAST, so the timed window starts on a busy, clocked-up GPU right behind them
    # (a host-side gap here shows up in short runs)
    cur._next_epoch()
    if isinstance(engine, HipEngine):
        # the timed window as ONE launch when it fits in the current epoch: a prepared direct AQL
        # dispatch of the persistent kernel, or one exact-size graph replay (a 20-step window: one
        # launch instead of 16 + 4; profiles/r2/window/, profiles/r6/aql/)
        engine.prepare_graphs(exact=(args.steps,) if args.steps <= min(512, cur.left - args.warmup) else ())
    else:
        engine.prepare_graphs()
    # (the eval path's first-call costs were paid before the A/Bs: a second evaluation here put
    # a different kernel between them and the warmup, 16.20 vs 16.12 us/step; profiles/r6/aql/)
    cur.run(args.warmup)
    if getattr(engine, "pipeline", False) and (engine._pipe_ok() or engine._pers_ok()):
        torch.cuda.synchronize(device)
        if engine.step_wait_failed():  # a wait timed out (never seen): fall back one level and time that
            level = engine.degrade()
            stamp(comm.rank, f"an in-launch step wait timed out in the warmup; using the {level} step")
            cur.left = 0
            cur._next_epoch()
            engine.prepare_graphs(exact=(args.steps,) if args.steps <= min(512, cur.left - args.warmup) else ())
            cur.run(args.warmup)
    xg = getattr(engine.grad_sync, "group", None)
    if xg is not None:
        xg.reset_wait_stats()
    stamp(comm.rank, selflaunch.WINDOW_MARK)  # (the launcher records failures before / after this line)
    comm.barrier()
    torch.cuda.synchronize(device)

    diag = args.diag_windows > 0
    if diag:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
    t0 = time.perf_counter()
    cur.run(args.steps)
    if diag:
        ev[1].record()
    torch.cuda.synchronize(device)
    if comm.distributed:  # (one rank: the barrier is a no-op, and so would a second synchronize be)
        comm.barrier()
        torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    stamp(comm.rank, f"timed window done: {1e6 * dt / args.steps:.3f} us/step on this rank")
    if diag:
        print(f"[bench] reported window: {1e6 * dt / args.steps:.2f} us/step wall, "
              f"{1e3 * ev[0].elapsed_time(ev[1]) / args.steps:.2f} us/step events", file=sys.stderr)
    if hasattr(engine.grad_sync, "check"):
        engine.grad_sync.check()  # raises if any xGMI wait in the timed window timed out
    if getattr(engine, "step_wait_failed", lambda: False)():  # an in-launch wait timed out: not a valid number
        raise RuntimeError("an in-launch step wait timed out inside the timed window")
    # per-step exchange wait inside the kernel over the timed steps (xGMI paths): this rank's
    # median / p99 / max, then the max over ranks
    waits = xg.wait_stats() if xg is not None else None
    if comm.distributed and args.sync == "step-allreduce":
        have = comm.gather_scalars(1.0 if waits else 0.0)
        if all(v == 1.0 for v in have):
            waits = {k: comm.reduce_scalar(float(waits[k]), "max") for k in ("median", "p99", "max")}
            waits = {k: round(v, 3) for k, v in waits.items()}
        else:
            waits = None
    for _ in range(args.diag_windows):  # diagnostic only: the reported window is the first one
        comm.barrier()
        torch.cuda.synchronize(device)
        ev[0].record()
        t1 = time.perf_counter()
        cur.run(args.steps)
        ev[1].record()
        torch.cuda.synchronize(device)
        comm.barrier()
        torch.cuda.synchronize(device)
        print(f"[bench] extra window: {1e6 * (time.perf_counter() - t1) / args.steps:.2f} us/step wall, "
              f"{1e3 * ev[0].elapsed_time(ev[1]) / args.steps:.2f} us/step events", file=sys.stderr)
    if diag and ab and comm.distributed:
        # diagnostic: the A/B's own measurement of the installed path, after the timed window
        from distributed_neural_network_amd.parallel.autotune import _measure
        us, _ = _measure(comm, engine, cur, min(args.steps, 256), args.warmup, 3, 200)
        stamp(comm.rank, f"A/B-style re-measure of {policy.installed(engine)} after the timed window: {us:.3f} us/step")
    dt = comm.reduce_scalar(dt, "max")
    ms_per_step = 1000.0 * dt / args.steps
    value = comm.world * B * args.steps / dt

    # one complete epoch from its first step: train + averaging/sync + full test-set eval
    epoch = {}
    if not args.no_epoch:
        cur.left = 0
        cur._next_epoch()
        engine.epoch_stats(reset=True)
        comm.barrier()
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        engine.run_steps(cur.steps_per_epoch)
        cur.left = 0
        policy.epoch_end(engine, cur.epoch)
        stats = engine.epoch_stats(reset=True)
        torch.cuda.synchronize(device)
        t2 = time.perf_counter()
        lo = comm.rank * len(test) // comm.world
        hi = (comm.rank + 1) * len(test) // comm.world
        loss, corr = engine.evaluate_samples(test_dev, lo, hi)
        full_l = torch.zeros(len(test), device=device)
        full_c = torch.zeros(len(test), device=device, dtype=torch.float32)
        full_l[lo:hi] = loss
        full_c[lo:hi] = corr.float()
        comm.allreduce_(full_l, "sum")
        comm.allreduce_(full_c, "sum")
        val_loss, val_acc = eval_metrics(full_l, full_c, B)
        torch.cuda.synchronize(device)
        t3 = time.perf_counter()
        epoch_s = comm.reduce_scalar(t3 - t1, "max")
        epoch = {"epoch_s": round(epoch_s, 6), "epoch_train_s": round(comm.reduce_scalar(t2 - t1, "max"), 6),
                 "eval_s": round(comm.reduce_scalar(t3 - t2, "max"), 6),
                 "epoch_images": int(len(sampler) * comm.world),
                 "train_loss": round(stats.mean_loss, 5), "val_loss": round(val_loss, 5),
                 "val_acc": round(val_acc, 3)}

    if comm.rank == 0:
        out = {"metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": comm.world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 6),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": round(value / BASELINE_IMG_S, 2),
               "dtype": args.dtype, "data": f"synthetic (CIFAR-10-shaped 3x32x32 uint8, template + noise "
                                        f"{args.noise}, {args.train_samples // 1000}k train / 10k test), "
                                        "random-init weights",
               "config": {"model": "reference CIFAR-10 CNN (models/model.py Network, 62,006 params)"
                          if args.model == "lenet" else args.model,
                          "engine": type(engine).__name__,
                          # pipelined step: step k's reduction + SGD in step k+1's launch (lenet_fused.hip PIPE)
                          "pipelined_step": bool(getattr(engine, "_pipe_ok", lambda: False)()),
                          # persistent launch: the whole timed window's steps in one launch (lenet_fused.hip PERS)
                          "persistent_launch": bool(getattr(engine, "_pers_ok", lambda: False)()),
                          # how that launch is issued: "direct-aql" (this process's own HSA queue,
                          # csrc/runtime/aql_dispatch.h) or "graph" (a captured hipGraph replay)
                          "launch": ("direct-aql" if getattr(engine, "_direct_ok", lambda: False)() else
                                     "graph" if getattr(engine, "use_graphs", False) else "eager"),
                          "global_batch": B * comm.world, "per_gpu_batch": B, "seq_len": None,
                          "image": [3, 32, 32], "parallelism": f"dp{comm.world}", "sync": args.sync,
                          "optimizer": "SGD lr=0.001 momentum=0.9, every step",
                          "allreduce": policy.installed(engine) if hasattr(policy, "installed") else None,
                          # the HSA runtime defaults this process ran with (distributed_neural_network_amd/hsa_env.py)
                          "runtime_env": {k: os.environ.get(k) for k in HSA_DEFAULTS},
                          # launcher retry level this number was measured at (0: as requested)
                          "safe_transport": safe},
               **epoch}
        if lab:
            out["launch_ab"] = lab["launch_ab"]
        if ab:
            out["allreduce_ab"] = ab["allreduce_ab"]
            out["allreduce_failed"] = ab["failed"]
            out["allreduce_failed_why"] = ab["why"]
            out["local_step_us"] = ab["local_us_per_step"]  # same steps with no all-reduce (A/B baseline)
            # the reported window's us/step next to the A/B's number for the same path (same shape)
            out["chosen_timed_us"] = round(1000.0 * ms_per_step, 3)
            out["ab_wall_s"] = ab["ab_wall_s"]
            out["allreduce_ab_variant"] = ab["variant"]
        if comm.distributed and args.sync == "step-allreduce":
            out["exchange_wait_us"] = waits
        os.write(out_fd, (json.dumps(out) + "\n").encode())
    comm.close()


if __name__ == "__main__":
    main()
