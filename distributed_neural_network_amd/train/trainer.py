"""Orchestrator: epochs, sync policy, evaluation, fault recovery, logs and metrics.

Capability parity with the reference orchestration:
  * ``main()`` / parent-child roles / epoch loop  (data_parallelism_train.py:56-152,
    model_replication_train.py:31-68, single_proc_train.py:16-105),
  * ``run_child``  -> engine.run_steps over this rank's epoch order (:185-213),
  * ``run_parent`` -> SyncPolicy.epoch_end (one all-reduce instead of N-1 receives
    and a rank-0 mean, :219-254) + the same stdout lines,
  * ``eval``       -> fused forward kernel over the test set, sharded over ranks,
    with the reference metric definitions (:157-183),
  * timers / log files / neptune series -> utils.timers / utils.logfiles /
    utils.metrics,
  * ``simulate_failure`` -> parallel.fault (plus real rank-drop recovery).

Stdout lines are kept verbatim so log scrapers keep working.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import numpy as np
import torch

from ..data import EpochSampler, get_splits
from ..parallel import CommError, Communicator, assert_replicas_identical, detect, make_policy
from ..parallel.fault import (DropInjector, Heartbeat, agree_survivors, announce_alive, beat_pause_injection,
                              end_skew_injection, recovery_fault_injection, simulate_failure, stall_injection,
                              stall_process)
from ..runtime import StepWaitTimeout, eval_metrics, make_engine
from ..utils import checkpoint, logfiles
from ..utils.metrics import Run
from ..utils.timers import PhaseTimers
from .config import TrainConfig


def resolve_device(spec: str, local_rank: int) -> torch.device:
    if spec == "cpu":
        return torch.device("cpu")
    if spec == "auto":
        if torch.cuda.is_available():
            return torch.device("cuda", local_rank % torch.cuda.device_count())
        return torch.device("cpu")
    if spec == "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("--device cuda requested but no ROCm GPU is visible")
        return torch.device("cuda", local_rank % torch.cuda.device_count())
    return torch.device(spec)


class Trainer:
    def __init__(self, cfg: TrainConfig) -> None:
        self.cfg = cfg
        if os.environ.get("DNN_FAULTHANDLER_S"):
            # hang forensics: every rank dumps all thread stacks to stderr every N seconds
            import faulthandler
            import sys

            faulthandler.dump_traceback_later(float(os.environ["DNN_FAULTHANDLER_S"]), repeat=True, file=sys.stderr)
        self.env = detect()
        self.device = resolve_device(cfg.device, self.env.local_rank)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        if self.device.type == "cpu" and self.env.world > 1:
            # N CPU ranks on one host: split the cores instead of oversubscribing them
            # (the reference's anti-scaling mechanism, Project_Report.pdf p.3 §5.3)
            torch.set_num_threads(max(1, (os.cpu_count() or 1) // self.env.world))
        self.comm = Communicator(self.env, self.device)
        # longest injected straggler sleep: bounded collective waits must outlast it
        self.comm.straggler_s = cfg.failure_duration if cfg.failure_probability > 0 else 0.0
        self.rank0 = self.comm.orig_rank == 0
        self.drop = DropInjector(cfg.drop_rank, cfg.drop_at_epoch, cfg.drop_at_step)
        self.hb: Optional[Heartbeat] = Heartbeat(self.comm) if self.comm.distributed else None
        self.rng = np.random.default_rng([cfg.seed, 0x57A66, self.comm.orig_rank])
        self.run_log = Run(cfg.metrics if self.rank0 else None)
        self.recoveries: list[dict] = []
        self.history: list[dict] = []
        self._resume_pending: Optional[dict] = None  # recovery record awaiting its first step
        self._paused: set[int] = set()

    # -- helpers --------------------------------------------------------------------------
    def _sampler(self) -> EpochSampler:
        c = self.cfg
        n = len(self.train)
        if c.mode in ("single", "replication"):
            return EpochSampler.for_rank(n, self.comm.rank, self.comm.world, c.seed, mode="full")
        return EpochSampler.for_rank(n, self.comm.rank, self.comm.world, c.seed, mode="shard",
                                     parent=c.sync == "parent")

    def _say(self, *a, **kw) -> None:
        if self.rank0:
            print(*a, **kw, flush=True)

    def _evaluate(self) -> tuple[float, float]:
        n = len(self.test)
        if self.cfg.eval_sharded and self.comm.distributed:
            lo, hi = self.comm.rank * n // self.comm.world, (self.comm.rank + 1) * n // self.comm.world
        else:
            lo, hi = 0, n
        loss, corr = self.engine.evaluate_samples(self.test, lo, hi)
        if self.cfg.eval_sharded and self.comm.distributed:
            dev = self.device if self.comm.backend == "nccl" else torch.device("cpu")
            full = torch.zeros(2, n, dtype=torch.float32, device=dev)
            full[0, lo:hi] = loss.to(dev)
            full[1, lo:hi] = corr.to(dev).float()
            self.comm.allreduce_(full, "sum")
            self.comm.wait_device()
            loss, corr = full[0], full[1]
        return eval_metrics(loss, corr, self.cfg.batch_size)

    def _train_epoch(self, epoch: int) -> None:
        order = self.sampler.order(epoch)
        self.engine.begin_epoch(order)
        n = self.sampler.steps(self.cfg.batch_size)
        lim = self.drop.step_limit(self.comm.orig_rank, epoch)
        if lim is not None and lim <= n:
            self.engine.run_steps(lim)
            self.comm.wait_device()
            self.drop.die(self.comm.orig_rank, epoch, lim, self.comm.store)
        if self._resume_pending is not None and n > 0:
            # first step on the re-formed group, timed on its own: the end of the recovery
            self.engine.run_steps(1)
            self.comm.wait_device()
            rec = self._resume_pending
            rec["t_resumed"] = time.time()
            rec["time_to_resume_s"] = round(rec["t_resumed"] - rec["t_error"], 6)
            rec["first_step_s"] = round(time.time() - rec["t_reformed"], 6)
            self._resume_pending = None
            self._say(f"[fault] first step on the re-formed group done {rec['time_to_resume_s']:.3f} s after the "
                      f"failure was detected")
            self.run_log.record(event="resumed", epoch=epoch, **{k: rec[k] for k in (
                "t_resumed", "time_to_resume_s", "first_step_s", "generation")})
            n -= 1
        self.engine.run_steps(n)
        self.comm.wait_device()  # interruptible: raises CommError if a peer is declared dead

    def _check_step_waits(self, epoch: int) -> None:
        """Raise StepWaitTimeout if a bounded in-launch wait timed out this epoch.  With a per-step
        all-reduce installed every rank votes (one tiny collective per epoch), so all ranks step
        down and redo the epoch together and their exchange step counters stay in step; without
        one (one rank, epoch-avg) the ranks train independently within an epoch and each decides
        alone (a rank that redoes its epoch only arrives later at the epoch-end average)."""
        failed = getattr(self.engine, "step_wait_failed", None)
        if failed is None:
            return
        bad = bool(failed())
        if self.comm.distributed and self.engine.grad_sync is not None:
            votes = self.comm.gather_scalars(1.0 if bad else 0.0)
            ranks = [i for i, v in enumerate(votes) if v != 0.0]
            if ranks:
                raise StepWaitTimeout(f"an in-launch step wait timed out on rank(s) {ranks} in epoch {epoch}")
        elif bad:
            raise StepWaitTimeout(f"an in-launch step wait timed out in epoch {epoch}")

    RECOVERY_ATTEMPTS = 3  # recoveries of one failure (a CommError inside _recover starts it over)

    def _recover(self, epoch: int, snap: tuple[torch.Tensor, torch.Tensor], err: Exception) -> None:
        """Survivor side of a failure: every stage is timed (wall clock, so the stamps compare
        across the ranks of one host) and recorded: detect (the watchdog flagged a peer, or the
        collective failed) -> abort -> agree -> reform -> restore/re-attach -> barrier, then the
        first step on the new group (``_train_epoch``).  ``recovery_s`` is reform-side only
        (error caught -> barrier passed); ``detect_s`` (tools/fault_bench.py) and
        ``time_to_resume_s`` put the detection and the first useful step around it."""
        t_err = time.time()
        t0 = time.perf_counter()
        stages = {}

        def stage(name: str) -> None:
            stages[name] = round(time.perf_counter() - t0, 6)
            if os.environ.get("DNN_FAULT_TRACE") == "1":
                print(f"[fault] rank {self.comm.orig_rank} recovery stage {name} at +{stages[name]:.3f} s",
                      flush=True)

        old = list(self.comm.members)
        assert self.hb is not None
        detected = {r: t for r, t in self.hb.detected_at.items() if r in old}
        # tear our side of the broken group down FIRST: closing its sockets/communicator
        # fails the collectives peers may still be blocked in on us (a gloo ring peer would
        # otherwise sit in recv until our reform, past the agreement deadline)
        announce_alive(self.comm)
        self.comm.abort()
        stage("abort")
        members = agree_survivors(self.comm, self.hb)
        stage("agree")
        if self.comm.orig_rank not in members:
            raise RuntimeError("this rank was excluded from the re-formed group") from err
        # the survivors are alive by agreement: a live rank whose beat was only late must not
        # stay flagged (check_alive would raise on every later replay / collective)
        self.hb.clear(members)
        dead = [r for r in old if r not in members]
        self.comm.reform(dead)
        stage("reform")
        if recovery_fault_injection(self.comm.orig_rank, self.comm.generation):
            raise CommError(f"injected recovery failure (generation {self.comm.generation})")
        if dead and self.comm.rank == 0:
            try:  # the dropped ranks will never check out of the store (parallel/store_server.py)
                self.comm.store.add("dnn/dropped", len(dead))
            except Exception:
                pass
        with torch.no_grad():
            self.engine.master.copy_(snap[0])
            self.engine.mom.copy_(snap[1])
        self.engine.params_changed()
        self.engine.epoch_stats(reset=True)
        if hasattr(self.engine, "invalidate_graphs"):
            self.engine.invalidate_graphs()  # captured collectives belong to the old communicator
        self.policy.attach(self.engine)
        self.sampler = self._sampler()
        stage("reattach")
        self.comm.barrier()
        stage("barrier")
        dt = time.perf_counter() - t0
        rec = {"epoch": epoch, "dead": dead, "survivors": members, "generation": self.comm.generation,
               "recovery_s": dt, "stages_s": stages, "t_error": t_err,
               "t_detected": min(detected.values()) if detected else None,
               "error": str(err).splitlines()[0][:200] if str(err) else type(err).__name__}
        self._resume_pending = dict(rec, t_reformed=time.time())
        self.recoveries.append(rec)
        self.rank0 = self.comm.rank == 0
        if self.comm.rank == 0:
            if dead:
                print(f"[fault] rank(s) {dead} dropped in epoch {epoch}; communicator re-formed "
                      f"(generation {self.comm.generation}, {self.comm.world} ranks) in {dt:.3f} s; "
                      f"data re-partitioned, epoch restarted from the last consistent parameters", flush=True)
            else:
                # every member is alive (e.g. an xGMI wait timed out behind a straggler):
                # a retry - fresh communicator generation, same members, epoch redone
                print(f"[fault] collective failure in epoch {epoch} with every rank alive; communicator "
                      f"re-created (generation {self.comm.generation}) in {dt:.3f} s, epoch retried", flush=True)
        self.run_log.record(event="recovery", **rec)

    # -- main ------------------------------------------------------------------------------
    def run(self) -> dict:
        c = self.cfg
        eng_kw = {}
        if self.device.type == "cuda":
            eng_kw = dict(graph_chunk=c.graph_chunk, overlap=c.overlap, use_graphs=c.use_graphs)
        self.timers = PhaseTimers()
        with self.timers.phase(PhaseTimers.DATA, sync=False):
            self.train, self.test = get_splits(c.data, c.data_root, c.train_samples, c.test_samples, c.seed)
            self.engine = make_engine(str(self.device) if self.device.type == "cuda" else "cpu", c.batch_size,
                                      c.lr, c.momentum, seed=c.seed, model=c.model, engine=c.engine,
                                      dtype=c.dtype, **eng_kw)
            self.engine.attach(self.train)
            self.test = self.test.to(self.device)
            self.engine.synchronize()
        self.timers._sync = self.comm.wait_device if self.comm.distributed else self.engine.synchronize
        self.policy = make_policy(c.sync if self.comm.distributed else "step-allreduce", self.comm,
                                  c.momentum_reset)
        if c.mode == "single":
            self.policy.reset_momentum_each_epoch = bool(c.momentum_reset)
        self.policy.bucket_kb = c.bucket_kb
        self.policy.grad_comm = getattr(c, "grad_comm", "fp32")
        if c.allreduce not in ("default", "ab") and hasattr(self.policy, "PATHS"):
            self.policy.path = c.allreduce
        self.policy.attach(self.engine)
        if self.comm.distributed and hasattr(self.policy, "installed"):
            self._say(f"[allreduce] per-step all-reduce path: {self.policy.installed(self.engine)}")
        self.sampler = self._sampler()
        self.allreduce_ab = None
        if c.allreduce == "ab" and self.comm.distributed and hasattr(self.policy, "PATHS"):
            # start-up A/B of the per-step all-reduce on this node (parameters restored after)
            from ..parallel.autotune import ab_window, allreduce_ab, default_candidates
            from ..runtime.cursor import EpochCursor

            cur = EpochCursor(self.engine, self.sampler, self.policy, c.batch_size)
            cands = default_candidates(self.policy.grad_comm)
            steps, warmup = ab_window(cur.steps_per_epoch)
            self.allreduce_ab = allreduce_ab(self.policy, self.engine, cur, steps=steps, warmup=warmup,
                                             candidates=cands)
            self._say(f"[allreduce] start-up A/B (us/step, max over ranks): {self.allreduce_ab['allreduce_ab']}; "
                      f"using {self.allreduce_ab['allreduce']}")
            self.run_log.record(event="allreduce_ab", **self.allreduce_ab)
        if self.hb is not None:
            self.engine.poll = self.comm.check_alive  # between graph replays (main thread)
            self.engine.device_wait = self.comm.wait_device  # graph capture, buffer resizes

        start_epoch = 0
        if c.resume:
            sd, side = checkpoint.load(c.resume, getattr(self.engine, "checkpoint_keys", lambda: None)())
            self.engine.load_state_dict(sd)
            if "momentum" in side:
                self.engine.mom.copy_(side["momentum"].to(self.engine.mom.device))
            start_epoch = int(side.get("epoch", -1)) + 1
            self._say(f"(Resumed from {c.resume} at epoch {start_epoch})")
        self.policy.initial_broadcast(self.engine)
        self.comm_time_children = 0.0

        if self.rank0:
            self.run_log["parameters"] = {"learning_rate": c.lr, "momentum": c.momentum, "optimizer": "SGD",
                                          "model_name": {"single": "nodistmodel"}.get(c.mode, "distmodel"),
                                          "epochs": c.epochs, "batch_size": c.batch_size, "sync": c.sync,
                                          "world_size": self.comm.world, "device": str(self.device)}
        if c.mode == "single":
            print(self.device, flush=True)
            print(len(self.train), flush=True)
            print(len(self.test), flush=True)
        elif self.policy.trains():
            print("(Loaded Train Dataset for worker {0} of length {1})".format(self.comm.orig_rank, len(self.sampler)),
                  flush=True)

        epoch = start_epoch
        while epoch < c.epochs:
            t_epoch = time.perf_counter()
            if c.mode != "single":
                self._say("Starting epoch ", epoch)
            simulate_failure(self.comm.orig_rank, c.failure_probability, c.failure_duration, self.rng)
            kind, stall = stall_injection(self.comm.orig_rank, epoch)
            if stall and ("stall", epoch) not in self._paused:
                self._paused.add(("stall", epoch))
                stall_process(kind, stall)
            pause = beat_pause_injection(self.comm.orig_rank, epoch)
            if pause and self.hb is not None and epoch not in self._paused:
                self._paused.add(epoch)
                self.hb.paused_until = time.time() + pause
                print(f"[fault] injected heartbeat pause: rank {self.comm.orig_rank} stops beating for {pause} s "
                      f"(epoch {epoch}) while it keeps training", flush=True)
            snap = (self.engine.master.detach().clone(), self.engine.mom.detach().clone())
            try:
                self.policy.epoch_start(self.engine, epoch)
                if self.policy.trains():
                    with self.timers.phase(PhaseTimers.TRAIN):
                        self._train_epoch(epoch)
                self._check_step_waits(epoch)
                stats = self.engine.epoch_stats(reset=True)
                t0 = time.perf_counter()
                self.policy.epoch_end(self.engine, epoch)
                if c.check_sync:
                    assert_replicas_identical(self.comm, self.engine)
                tot = torch.tensor([stats.loss_sum, stats.batches, stats.correct, stats.samples],
                                   dtype=torch.float64)
                if self.comm.distributed:
                    dev = self.device if self.comm.backend == "nccl" else torch.device("cpu")
                    tt = tot.to(dev)
                    self.comm.allreduce_(tt, "sum")
                    self.comm.wait_device()
                    tot = tt.cpu()
                self.timers.add(PhaseTimers.COMM_PARENT if self.rank0 else PhaseTimers.COMM_CHILDREN,
                                time.perf_counter() - t0)
                # evaluated inside the recovery scope (its metric all-reduce can meet a dead
                # peer too); the lines are printed below in the reference's order
                with self.timers.phase(PhaseTimers.EVAL):
                    val_loss, val_acc = self._evaluate()
                if epoch == c.epochs - 1 and self.comm.distributed:
                    skew = end_skew_injection(self.comm.orig_rank)
                    if skew:
                        print(f"[fault] injected end skew: rank {self.comm.orig_rank} idles {skew} s after the last "
                              f"collective", flush=True)
                        time.sleep(skew)
                    # nobody leaves before every rank is done with the last collective (a fast rank's
                    # exit must not reach a slow peer's watchdog while that peer still waits on it);
                    # inside the recovery scope: a real death here still re-forms and redoes the epoch
                    self.comm.barrier()
            except StepWaitTimeout as e:
                # an in-launch wait of the pipelined / persistent step timed out (e.g. the grid
                # lost co-residency to other work on the device): restore the epoch's snapshot,
                # step the engine down one level and redo the epoch - the job goes on
                level = self.engine.degrade() if hasattr(self.engine, "degrade") else None
                if level is None:
                    raise
                print(f"[engine] rank {self.comm.orig_rank}: {e}; stepping down to the {level} step and redoing "
                      f"epoch {epoch} from its start", flush=True)
                self.run_log.record(event="step_degraded", epoch=epoch, level=level, rank=self.comm.orig_rank)
                grp = getattr(getattr(self.engine, "grad_sync", None), "group", None)
                if grp is not None and self.comm.distributed and hasattr(grp, "clear_error"):
                    # (voted: every rank is here) a ready wait long enough to time out also times
                    # out the peers' in-launch exchange waits, which set the group's sticky error
                    # word: every rank drains its device, then all clear it - else the redo would
                    # run with the word set and end in a CommError recovery that drops nobody
                    self.comm.wait_device()
                    self.comm.barrier()
                    grp.clear_error()
                with torch.no_grad():
                    self.engine.master.copy_(snap[0])
                    self.engine.mom.copy_(snap[1])
                self.engine.params_changed()
                self.engine.epoch_stats(reset=True)
                continue
            except CommError as e:
                if not self.comm.distributed or self.hb is None:
                    raise
                # a failure DURING the recovery (e.g. a survivor flagged stale under load while
                # the re-formed group's barrier runs) starts the recovery over: agree, re-form
                err: Exception = e
                for _ in range(self.RECOVERY_ATTEMPTS):
                    try:
                        self._recover(epoch, snap, err)
                        break
                    except CommError as e2:
                        print(f"[fault] rank {self.comm.orig_rank}: recovery interrupted ({e2}); recovering again",
                              flush=True)
                        err = e2
                else:
                    raise err
                continue
            loss_sum, batches, correct, samples = [float(x) for x in tot.tolist()]
            trainers = self.policy.trainer_count()
            if c.mode == "single":
                avg = loss_sum / max(batches, 1)
                print(f"Epoch {epoch + 1}, Average Training Loss: {avg:.3f}", flush=True)
            else:
                for p in range(trainers):
                    self._say("(Received a trained model from process {0} of {1} workers...)".format(p + 1, trainers))
                self._say("* Averaging models...")
                # reference quirk (§2.7 #1): it divides by 10 (state_dict keys) per worker
                avg = loss_sum / (10.0 * trainers) if c.compat else loss_sum / max(batches, 1)
                self._say(f"Global Average Training Loss: {avg}")
                self._say("evaluating model")
            if c.mode == "single":
                print("Validation Accuracy: %.2f %%" % val_acc, flush=True)
                print("Validation Loss: %.3f" % val_loss, flush=True)
            else:
                self._say("Validation loss of updated master model: ", val_loss)
            dt = time.perf_counter() - t_epoch
            rec = {"epoch": epoch, "train_loss": avg, "train_acc": 100.0 * correct / max(samples, 1),
                   "val_loss": val_loss, "val_acc": val_acc, "epoch_s": dt, "samples": samples,
                   "img_per_s": samples / dt if dt > 0 else 0.0, "world": self.comm.world,
                   "phases": self.timers.as_dict() if c.profile else None}
            self.history.append(rec)
            if self.recoveries and self.recoveries[-1]["epoch"] == epoch and self.rank0:
                # recovery latency is printed by _recover; this is the
                # throughput of the first epoch on the re-formed group
                print(f"[fault] post-recovery epoch {epoch}: {rec['img_per_s']:.1f} img/s on "
                      f"{self.comm.world} ranks", flush=True)
            if self.rank0:
                self.run_log["train/loss"].append(avg)
                self.run_log["val/loss"].append(val_loss)
                self.run_log["val/acc"].append(val_acc)
                self.run_log.record(**rec)
                if c.save:
                    checkpoint.save(c.save, self.engine.state_dict(), self.engine.mom, epoch=epoch,
                                    seed=c.seed, world=self.comm.world, sync=c.sync, mode=c.mode)
            epoch += 1

        # recoveries with every member alive: heartbeat false positives / transient collective
        # failures (each cost one epoch redo, never a rank)
        retries = sum(1 for r in self.recoveries if not r["dead"])
        if self.rank0:
            self.run_log.record(event="summary", recoveries=len(self.recoveries), retries_all_alive=retries,
                                heartbeat_timeout_s=round(self.hb.timeout, 3) if self.hb is not None else None)
        self._finish()
        return {"history": self.history, "recoveries": self.recoveries, "timers": self.timers.as_dict(),
                "world": self.comm.world, "rank": self.comm.rank, "retries_all_alive": retries}

    def _finish(self) -> None:
        c = self.cfg
        T = self.timers
        if c.mode == "data-parallel":
            if self.rank0:
                print("Eval data loading time: {0}".format(T[PhaseTimers.DATA]), flush=True)
                print("Time spent on evaluation: {0}".format(T[PhaseTimers.EVAL]), flush=True)
                print("Time spent on parent communication and param sync: {0}".format(T[PhaseTimers.COMM_PARENT]),
                      flush=True)
                if c.write_logs:
                    logfiles.write_log(c.log_dir, logfiles.log_name(c.batch_size, c.epochs, c.nb_proc, "parent"),
                                       logfiles.parent_lines(T[PhaseTimers.DATA], T[PhaseTimers.EVAL],
                                                             T[PhaseTimers.COMM_PARENT]))
            # reference: rank 2 only (a 2-process job never wrote it); default: the
            # lowest training rank other than 0 that exists
            child = 2 if c.compat else min(2, self.comm.world - 1)
            if self.comm.rank == child and (child != 0 or not c.compat) and self.policy.trains():
                comm_c = T[PhaseTimers.COMM_CHILDREN] if child != 0 else T[PhaseTimers.COMM_PARENT]
                print("Training data loading time: {0}".format(T[PhaseTimers.DATA]), flush=True)
                print("Time spent on training: {0}".format(T[PhaseTimers.TRAIN]), flush=True)
                print("Time spent on children communication: {0}".format(comm_c), flush=True)
                if c.write_logs:
                    logfiles.write_log(c.log_dir, logfiles.log_name(c.batch_size, c.epochs, c.nb_proc, "children"),
                                       logfiles.children_lines(T[PhaseTimers.DATA], T[PhaseTimers.TRAIN], comm_c))
        skew = end_skew_injection(self.comm.orig_rank, "after") if self.comm.distributed else 0.0
        if skew:
            print(f"[fault] injected end skew: rank {self.comm.orig_rank} idles {skew} s after the final barrier",
                  flush=True)
            time.sleep(skew)
        if self.hb is not None:
            # check out before the beat stops and the process exits: peers never flag this exit
            try:
                self.hb.check_out()
            except Exception:
                pass
            self.hb.stop()
        self.run_log.stop()
        self.comm.close()


def run(cfg: TrainConfig) -> dict:
    return Trainer(cfg).run()
