"""Synchronisation policies of data-parallel training.

* ``epoch-avg`` - the reference algorithm: every rank runs a
  full local epoch of momentum SGD with a freshly created optimizer
  (data_parallelism_train.py:187 - momentum restarts every epoch), then the models
  are averaged (data_parallelism_train.py:238-244).  Here the average is ONE
  all-reduce(avg) of the flat parameter arena instead of N-1 pickled sends + a
  rank-0 mean.
* ``parent``    - exact reference topology: rank 0 is a non-training parameter
  server (data_parallelism_train.py:101-129); the average is over ranks 1..N-1
  (rank 0 contributes zeros to a sum all-reduce, everyone divides by N-1).
* ``step-allreduce`` - DDP-style per-step gradient averaging (the report's future
  work, Project_Report.pdf p.4 §6.2), captured in the step hipGraph: on one node a
  one-shot xGMI all-reduce fused with the SGD update (parallel/xgmi.py); otherwise
  (or with --overlap / --bucket-kb) bucketed RCCL all-reduces, the MLP bucket
  overlapped with the conv-bucket reduction.
"""
from __future__ import annotations

import os

import time

import torch

from .comm import CommError, Communicator, GradAllReduce, trace

SYNC_MODES = ("step-allreduce", "epoch-avg", "parent")


class SyncPolicy:
    name = "base"
    reset_momentum_each_epoch = False

    bucket_kb = 0  # step-allreduce: gradient bucket size limit (0 = one fused bucket)

    def __init__(self, comm: Communicator, reset_momentum_each_epoch: bool | None = None) -> None:
        self.comm = comm
        if reset_momentum_each_epoch is not None:
            self.reset_momentum_each_epoch = reset_momentum_each_epoch
        self.comm_time = 0.0

    def trains(self) -> bool:
        return True

    def trainer_count(self) -> int:
        return self.comm.world

    def attach(self, engine) -> None:
        self.engine = engine

    def initial_broadcast(self, engine) -> None:
        """Rank 0's initial weights are authoritative (reference: parent sends before epoch 0)."""
        t0 = time.perf_counter()
        self.comm.broadcast_(engine.master, src=0)
        buf = getattr(engine, "buffers", None)
        if buf is not None:
            self.comm.broadcast_(buf, src=0)
        engine.params_changed()
        self.comm.wait_device()
        self.comm_time += time.perf_counter() - t0

    def epoch_start(self, engine, epoch: int) -> None:
        if self.reset_momentum_each_epoch:
            engine.reset_momentum()

    def epoch_end(self, engine, epoch: int) -> None:
        self.sync_buffers(engine)

    def sync_buffers(self, engine, trainers_only: bool = False) -> None:
        """Average non-trained state (BatchNorm running statistics of layer-engine models)
        over the training ranks, so every replica evaluates / checkpoints the same model."""
        buf = getattr(engine, "buffers", None)
        if buf is None or not self.comm.distributed:
            return
        with torch.no_grad():
            if trainers_only:
                if not self.trains():
                    buf.zero_()
                self.comm.allreduce_(buf, "sum")
                buf.div_(self.trainer_count())
            else:
                self.comm.allreduce_(buf, "avg")


def replica_checksums(engine) -> tuple[float, float]:
    """(sum, position-weighted sum) of the fp32 parameter arena in fp64: equal on two
    ranks iff (with overwhelming probability) their arenas are bit-identical.  Computed on a
    host copy: the check itself allocates no device temporaries (a GPU-side version once
    reported a mismatch between bit-identical arenas: profiles/r1_xcd_map_experiment.txt)."""
    m = engine.master.detach().to("cpu", torch.float64)
    w = torch.arange(1, m.numel() + 1, dtype=torch.float64).remainder_(9973).add_(1)
    return float(m.sum()), float((m * w).sum())


def assert_replicas_identical(comm: Communicator, engine) -> None:
    """Cross-rank parameter checksum after a synchronisation point: catches
    replica divergence and comm/compute stream races."""
    if not comm.distributed:
        return
    a, b = replica_checksums(engine)
    sa, sb = comm.gather_scalars(a), comm.gather_scalars(b)
    if len(set(sa)) != 1 or len(set(sb)) != 1:
        raise RuntimeError(f"replicas diverged: parameter checksums per rank {sa} / {sb}; "
                           f"rank {comm.rank}: {_divergence_report(comm, engine)}")


def _divergence_report(comm: Communicator, engine) -> str:
    """Where this rank's arena differs from rank 0's (collective: every rank calls it)."""
    mine = engine.master.detach().float().cpu()
    ref = mine.clone()
    try:
        comm.broadcast_(ref, 0)
    except Exception as e:  # diagnostics only
        return f"(no report: {e})"
    bad = (mine != ref).nonzero().flatten()
    if bad.numel() == 0:
        return "arena equals rank 0's"
    i = int(bad[0])
    same_multiset = bool(torch.equal(mine.sort().values, ref.sort().values))
    return (f"{bad.numel()} of {mine.numel()} elements differ from rank 0, indices {int(bad[0])}..{int(bad[-1])}, "
            f"first: {float(mine[i])} vs {float(ref[i])}, permutation of rank 0's values: {same_multiset}")


class StepAllReduce(SyncPolicy):
    """Per-step gradient all-reduce.  The transport is one of the PATHS below; ``path`` None
    means the default choice (``default_path``), a name pins it (the multi-GPU bench sets the
    winner of its start-up A/B, parallel/autotune.py).  ``attach`` re-installs the path after
    every communicator re-form (rank-drop recovery)."""

    name = "step-allreduce"
    # xgmi-pull / xgmi-rsag: the batch-reduction kernel exchanges its elements over xGMI
    # (one-hop pull / two-hop reduce-scatter + all-gather) and applies SGD in ONE launch;
    # rccl: ncclAllReduce of the fused gradient bucket + sgd_apply; rccl-overlap: the MLP bucket
    # all-reduced on a side stream while the conv bucket is reduced; local: no all-reduce (A/B
    # baseline only: replicas diverge)
    # (xgmi-pull-bf16 / xgmi-rsag-bf16: the same exchanges with bf16 gradient granules, opt-in)
    # (xgmi-pull-pers / xgmi-rsag-pers: the same exchanges inside the PERSISTENT launch's reduction
    # workgroups - the whole window one launch, no kernel boundary between steps, the exchange +
    # SGD before each step's ready hand-off; lenet_fused.hip XNR; self-tested bit for bit against
    # the serial one-launch exchange)
    PATHS = ("xgmi-pull-pers", "xgmi-rsag-pers", "xgmi-pull", "xgmi-rsag", "rccl", "rccl-overlap", "xgmi-pull-bf16",
             "xgmi-rsag-bf16")
    path: str | None = None
    grad_comm = "fp32"  # "bf16": the default xGMI path uses bf16 gradient granules (--grad-comm)
    record_waits = False  # xGMI paths: record every step's exchange wait (XgmiGroup.wait_stats)

    def attach(self, engine) -> None:
        super().attach(engine)
        if not self.comm.distributed:
            engine.grad_sync = None
            return
        name = self.path or self.default_path(engine)
        chain = [name]
        if name.endswith("-pers"):
            chain.append(name.removesuffix("-pers"))
        if name.startswith("xgmi") and "xgmi-pull" not in chain:
            chain.append("xgmi-pull")
        if name.startswith("xgmi"):
            chain.append("rccl" if self.comm.backend == "nccl" else "torch-pg")
        for i, n in enumerate(chain):
            if self.install(engine, n):
                if i and self.comm.rank == 0:
                    import sys

                    print(f"[allreduce] {name} unavailable: using {n}", file=sys.stderr, flush=True)
                return
        raise CommError(f"per-step all-reduce path {name!r} could not be installed")

    def default_path(self, engine) -> str:
        from . import xgmi

        if getattr(engine, "overlap", False) or self.bucket_kb:
            # --overlap / --bucket-kb ask for the bucketed collective path
            return ("rccl-overlap" if getattr(engine, "overlap", False) else "rccl") \
                if self.comm.backend == "nccl" else "torch-pg"
        if xgmi.wanted(self.comm) and engine.grad.numel() <= self.XGMI_MAX_ELEMS:
            mode = xgmi.exchange_mode() | (4 if self.grad_comm == "bf16" else 0)
            # the serial one-launch exchange; the exchange inside the persistent launch only with
            # DNN_AB_PERS=1 (it lost to the serial form by 32 us/step with two ranks side by side
            # on one GPU, profiles/r6/inproc/; parallel/autotune.py ORDER) and where the engine
            # has that launch (fp32 granules; falls back to the serial exchange if its self-test
            # fails): the bf16 kernel's (on top of its pipelined step) or the fp32 kernel's
            has_pers = getattr(engine, "persist", False) and (getattr(engine, "pipeline", False)
                                                               or getattr(engine, "dtype", "") == "fp32")
            pers = "-pers" if mode in (0, 2) and has_pers and os.environ.get("DNN_AB_PERS") == "1" else ""
            return "xgmi-" + xgmi.MODE_NAMES[mode] + pers
        return "rccl" if self.comm.backend == "nccl" else "torch-pg"

    def installed(self, engine) -> str | None:
        """Name of the path the engine runs now (None: one rank, no all-reduce)."""
        gs = engine.grad_sync
        if gs is None:
            return None if not self.comm.distributed else "local"
        kind = type(gs).__name__
        if kind == "XgmiGradSync":
            from .xgmi import MODE_NAMES

            form = MODE_NAMES[gs.group.xp_mode]
            pers = "-pers" if getattr(engine, "pers_exchange", False) and engine._pers_xchg() is not None else ""
            return f"xgmi-{form}{pers}" + ("" if gs.group.one_launch else "-two-launch")
        if kind == "NativeGradAllReduce":
            return "rccl-overlap" if gs.overlap else "rccl"
        return "torch-pg"

    def install(self, engine, name: str) -> bool:
        """Collective: put path ``name`` on the engine.  Returns the agreed outcome (False on
        every rank if it failed on any; the engine then has no all-reduce installed)."""
        self.install_why = ""  # why the last install returned False (the A/B's failure reason)
        if hasattr(engine, "invalidate_graphs"):
            engine.invalidate_graphs()
        if hasattr(engine, "overlap"):
            engine.overlap = name == "rccl-overlap"
        engine.grad_sync = None
        pers = name.endswith("-pers")
        if hasattr(engine, "pers_exchange"):
            engine.pers_exchange = False
        elif pers:
            self.install_why = "the persistent (-pers) exchange needs the fused engine"
            return False
        if name == "local":
            return True
        if name.startswith("xgmi"):
            from .xgmi import EXCHANGE_MODES

            mode = EXCHANGE_MODES[name[len("xgmi-"):].removesuffix("-pers")]
            if not self._install_xgmi(engine, mode):
                return False
            if pers:
                return self._install_pers(engine, mode)
            return True
        if name in ("rccl", "rccl-overlap"):
            if self.comm.backend != "nccl":
                self.install_why = f"RCCL needs the nccl backend (this run's host collectives: {self.comm.backend})"
                return False
            from .rccl import NativeGradAllReduce, RcclComm

            rc = getattr(self.comm, "native", None)
            trace("native RCCL communicator ...")
            if rc is None:
                rc = self.comm.native = RcclComm(self.comm)
            elif rc.generation != self.comm.generation:
                rc.reinit()
            trace("native RCCL communicator up")
            engine.grad_sync = NativeGradAllReduce(rc, engine.device, overlap=name == "rccl-overlap",
                                                   bucket_kb=self.bucket_kb)
            return True
        if name == "torch-pg":
            engine.grad_sync = GradAllReduce(self.comm, bucket_kb=self.bucket_kb)
            if getattr(engine, "use_graphs", False):
                # host-side (gloo) collectives cannot live inside a captured hipGraph
                engine.use_graphs = False
            return True
        raise ValueError(f"unknown all-reduce path {name!r}; expected one of {self.PATHS + ('local', 'torch-pg')}")

    def _install_xgmi(self, engine, mode: int) -> bool:
        from .xgmi import XgmiGradSync, one_launch_wanted

        xg = self._xgmi_group(engine)
        if xg is None:
            self.install_why = "no xGMI group (not one node, refused, or its self-test failed)"
            return False
        engine.grad_sync = XgmiGradSync(xg)
        xg.one_launch, xg.xp_mode = False, mode
        xg.enable_wait_stats(self.record_waits)
        if one_launch_wanted() and hasattr(engine, "selftest_exchange"):
            # batch reduction + all-reduce + SGD in ONE launch, once it has matched the
            # two-launch path bit for bit on every rank (all ranks get the same vote); results
            # are cached per form for this group
            cache = xg.__dict__.setdefault("selftested", {})
            if mode not in cache:
                cache[mode] = engine.selftest_exchange(xg, self.comm)
                if xg.broken:
                    # a pass raised / timed out on some rank: the step counters may be out of
                    # step across ranks - this group must not be used again
                    self._drop_xgmi_group()
                    engine.grad_sync = None
                    self.install_why = "the one-launch exchange self-test raised or timed out"
                    return False
            xg.one_launch = cache[mode]
            if not xg.one_launch:
                if mode != 0:
                    engine.grad_sync = None
                    self.install_why = "the one-launch exchange self-test did not match the two-launch path"
                    return False  # the two-hop form exists only as the one-launch exchange
                if self.comm.rank == 0:
                    import sys

                    print("[xgmi] one-launch exchange self-test failed: two-launch all-reduce", file=sys.stderr,
                          flush=True)
        if hasattr(engine, "invalidate_graphs"):
            engine.invalidate_graphs()
        return True

    def _install_pers(self, engine, mode: int) -> bool:
        """The "-pers" form on top of an installed one-launch exchange: self-tested once per group
        and form (HipEngine.selftest_pers_exchange: bit for bit against the serial one-launch
        exchange on every rank), then the engine runs its persistent launch with the exchange
        inside.  Collective; False (on every rank) leaves nothing installed."""
        xg = engine.grad_sync.group if engine.grad_sync is not None else None
        if xg is None or not xg.one_launch or mode not in (0, 2) or not hasattr(engine, "selftest_pers_exchange"):
            engine.grad_sync = None
            self.install_why = "the persistent exchange needs the self-tested one-launch exchange (fp32 granules)"
            return False
        cache = xg.__dict__.setdefault("selftested_pers", {})
        if mode not in cache:
            cache[mode] = engine.selftest_pers_exchange(xg, self.comm)
            if xg.broken:
                self._drop_xgmi_group()
                engine.grad_sync = None
                self.install_why = f"the persistent exchange self-test raised or timed out ({cache[mode][1]})"
                return False
        ok, why = cache[mode]
        if not ok:
            engine.grad_sync = None
            self.install_why = f"the persistent exchange self-test failed: {why or 'on a peer'}"
            return False
        engine.pers_exchange = True
        engine.invalidate_graphs()
        return True

    def _drop_xgmi_group(self) -> None:
        grp = getattr(self.comm, "xgmi", None)
        if grp is not None:
            grp.close()
        self.comm.xgmi = None

    XGMI_MAX_ELEMS = 4 << 20  # one-shot reads N x the gradient: beyond ~16 MB the RCCL ring wins

    def _xgmi_group(self, engine):
        """The one-shot xGMI group for this generation (built collectively, self-tested;
        None -> not available here)."""
        from . import xgmi

        if not xgmi.wanted(self.comm):
            return None
        n = engine.grad.numel()
        if n > self.XGMI_MAX_ELEMS:
            return None
        grp = getattr(self.comm, "xgmi", None)
        stale = None
        if grp is not None and (grp.generation != self.comm.generation or grp.capacity < n):
            stale, grp = grp, None
        if grp is None and not getattr(self.comm, "xgmi_refused", False):
            trace("xGMI group: IPC regions + self-test ...")
            grp = self.comm.xgmi = xgmi.build_group(self.comm, n)
            self.comm.xgmi_refused = grp is None
            trace(f"xGMI group {'up' if grp is not None else 'refused / failed'}")
        if stale is not None:
            stale.close()  # after the new regions exist: no address of the old ones is reused
        if hasattr(engine, "invalidate_graphs"):
            engine.invalidate_graphs()
        return grp

    lazy_check = False  # True: the caller checks the xGMI error word itself (bench: once, at the end)

    def epoch_end(self, engine, epoch: int) -> None:
        failed = getattr(engine.grad_sync, "failed", None)
        if failed is not None and not self.lazy_check:
            # a timed-out / aborted xGMI wait sets a sticky word on the rank that waited; the
            # ranks agree on it (one tiny collective per epoch), so EVERY rank raises and
            # enters recovery together - a late but live straggler included, which then
            # counts as alive and the recovery becomes a retry, not an exclusion
            votes = self.comm.gather_scalars(1.0 if failed() else 0.0)
            if any(v != 0.0 for v in votes):
                bad = [i for i, v in enumerate(votes) if v != 0.0]
                raise CommError(f"xGMI all-reduce wait failed on rank(s) {bad} in epoch {epoch}")
        super().epoch_end(engine, epoch)


class EpochAverage(SyncPolicy):
    name = "epoch-avg"
    reset_momentum_each_epoch = True

    def attach(self, engine) -> None:
        super().attach(engine)
        engine.grad_sync = None

    def epoch_end(self, engine, epoch: int) -> None:
        if not self.comm.distributed:
            return
        t0 = time.perf_counter()
        self.comm.allreduce_(engine.master, "avg")
        self.sync_buffers(engine)
        engine.params_changed()
        self.comm.wait_device()
        self.comm_time += time.perf_counter() - t0


class ParentAverage(EpochAverage):
    """Reference topology: rank 0 only averages/evaluates; ranks 1..N-1 train."""

    name = "parent"

    def __init__(self, comm: Communicator, reset_momentum_each_epoch: bool | None = None) -> None:
        super().__init__(comm, reset_momentum_each_epoch)
        if comm.world < 2:
            raise ValueError("--sync parent needs >= 2 processes: rank 0 is the parameter server")

    def trains(self) -> bool:
        return self.comm.rank != 0

    def trainer_count(self) -> int:
        return self.comm.world - 1

    def epoch_end(self, engine, epoch: int) -> None:
        t0 = time.perf_counter()
        with torch.no_grad():
            if self.comm.rank == 0:
                engine.master.zero_()
            self.comm.allreduce_(engine.master, "sum")
            engine.master.div_(self.comm.world - 1)
        self.sync_buffers(engine, trainers_only=True)
        engine.params_changed()
        self.comm.wait_device()
        self.comm_time += time.perf_counter() - t0


def make_policy(mode: str, comm: Communicator, reset_momentum_each_epoch: bool | None = None) -> SyncPolicy:
    if mode == "step-allreduce":
        return StepAllReduce(comm, reset_momentum_each_epoch)
    if mode == "epoch-avg":
        return EpochAverage(comm, reset_momentum_each_epoch)
    if mode == "parent":
        return ParentAverage(comm, reset_momentum_each_epoch)
    raise ValueError(f"unknown sync mode {mode!r}; expected one of {SYNC_MODES}")
