"""Communicator: one process per GPU, collectives over RCCL (xGMI) or gloo (CPU).

Capability parity: replaces the reference's pickled point-to-point mpi4py traffic
(data_parallelism_train.py:118,135,210,227):

  reference                                   here
  [comm.send(state_dict, k) for k]  (:118)    broadcast_(arena) once at start-up
  child send / parent recv + mean  (:210-240) allreduce_(arena, "avg")  (epoch-avg)
  (future work in the report)                 bucketed per-step gradient all-reduce

On MI355X the backend is torch.distributed "nccl", which IS RCCL: a flat fp32
arena means one (or two bucketed) collectives per sync instead of 10 pickled
tensors per child; the per-step gradient all-reduce is issued on RCCL's stream
and overlapped with the conv-bucket reduction kernel (see GradAllReduce).

Fault tolerance: the process group is created over our own TCPStore under a
generation prefix, so survivors of a dropped rank can abort the old
communicator and rendezvous a fresh one (generation + 1) with re-numbered ranks
(ncclCommAbort + new ncclCommInitRank; torch's bundled RCCL 2.26 has no
ncclCommShrink).  See fault.py for detection and recovery.
"""
from __future__ import annotations

import datetime as _dt
import os
import threading
import time
from typing import Callable, Optional, Sequence

import torch
import torch.distributed as dist

from .env import DistEnv, detect


class CommError(RuntimeError):
    """A collective failed (peer died, communicator aborted, timeout)."""


_TRACE_T0 = time.time()


def trace(msg: str) -> None:
    """Stamped start-up trace on stderr (``DNN_STARTUP_TRACE=1``; bench.py sets it): process
    group, native RCCL init, xGMI IPC map - so a stalled multi-GPU start shows where it sits."""
    if os.environ.get("DNN_STARTUP_TRACE") == "1":
        import sys

        print(f"[trace r{os.environ.get('RANK', '0')} +{time.time() - _TRACE_T0:.3f}s] {msg}", file=sys.stderr,
              flush=True)


class Communicator:
    def __init__(self, env: DistEnv | None = None, device: torch.device | str = "cpu",
                 backend: str | None = None, timeout_s: float = 300.0) -> None:
        self.env = env or detect()
        self.device = torch.device(device)
        # DNN_BACKEND=gloo forces host collectives (multi-rank tests on a single GPU, where
        # RCCL refuses two ranks on one device)
        self.backend = backend or os.environ.get("DNN_BACKEND") or ("nccl" if self.device.type == "cuda" else "gloo")
        self.timeout = _dt.timedelta(seconds=timeout_s)
        self.generation = 0
        self.members: list[int] = list(range(self.env.world))  # original ranks of the live group
        self.orig_rank = self.env.rank
        self.store: dist.Store | None = None
        self.aborted = False
        self.watch: Optional[Callable[[], Sequence[int]]] = None  # liveness watch (fault.Heartbeat)
        self.rccl_error = False  # set by the watchdog when ncclCommGetAsyncError reports an error
        # set by the watchdog when other members started a recovery of this generation (their
        # announce_alive): a rank blocked in a collective those peers have left learns it here
        self.peer_recovery = -1
        # DNN_FORCE_COLLECTIVES=1: build a real process group and issue every collective
        # even at world size 1 (exercises the RCCL + hipGraph-capture path on one GPU)
        self.force = os.environ.get("DNN_FORCE_COLLECTIVES", "0") == "1"
        if self.env.world > 1 or self.force:
            trace(f"store {self.env.master_addr}:{self.env.master_port} ...")
            self._init_store()
            trace(f"store connected; process group ({self.backend}, generation {self.generation}) ...")
            self._init_group()
            trace("process group up")

    # -- identity ----------------------------------------------------------------------
    @property
    def rank(self) -> int:
        return self.members.index(self.orig_rank) if self.orig_rank in self.members else 0

    @property
    def world(self) -> int:
        return len(self.members)

    @property
    def distributed(self) -> bool:
        return self.world > 1 or (self.force and dist.is_initialized() and not self.aborted)

    # -- setup ---------------------------------------------------------------------------
    def _init_store(self) -> None:
        agent = (os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
                 or os.environ.get("DNN_STORE_EXTERNAL", "") == "1")
        if agent:
            # torchrun's agent (or parallel/launch.py) already serves a TCPStore on
            # MASTER_ADDR:MASTER_PORT; every rank is a client, so any rank may die.
            self.store = dist.TCPStore(self.env.master_addr, self.env.master_port, self.env.world,
                                       is_master=False, timeout=self.timeout)
        elif self.env.world > 1 and os.environ.get("DNN_STORE_IN_RANK0", "0") != "1":
            # no agent (mpiexec / plain env launch): rank 0 starts a stand-alone store process and
            # every rank is a client, so the store survives rank 0 (parallel/store_server.py)
            token = None
            if self.env.rank == 0:
                token = f"{os.getpid()}-{os.urandom(6).hex()}"
                self._store_proc = _spawn_store_server(self.env.master_port, self.env.world, token)
            self.store = dist.TCPStore(self.env.master_addr, self.env.master_port, self.env.world,
                                       is_master=False, timeout=self.timeout)
            self._check_fresh_store(token)
        else:
            self.store = dist.TCPStore(self.env.master_addr, self.env.master_port, self.env.world,
                                       is_master=self.env.rank == 0, timeout=self.timeout,
                                       wait_for_workers=False)
        # process identity (host:pid): the stand-alone store stays up while a rank of this host is
        # alive and exits once they are all gone (parallel/store_server.py); the heartbeat
        # watchdog reads it too (a gone local pid is a dead rank, fault.Heartbeat)
        try:
            import socket

            self.store.set(f"dnn/pid/{self.orig_rank}", f"{socket.gethostname()}:{os.getpid()}")
        except Exception:
            pass

    STALE_BEAT_S = 30.0

    def _check_fresh_store(self, token: str | None) -> None:
        """Fail loudly if the store on MASTER_PORT is a server left over from an earlier job
        (ADVICE r3): its keys - recovery leaders, member lists, RCCL ids, closed counters -
        would steer this job.  Rank 0 checks that the server answering is the child it just
        started (job token, and the child is still running: a second server on a taken port
        exits at once); every rank checks that nothing has checked out of this store yet and
        that no rank's heartbeat in it is older than ``STALE_BEAT_S`` (a left-over server exits
        on its own after that long without beats, parallel/store_server.py)."""
        st = self.store
        assert st is not None
        where = f"{self.env.master_addr}:{self.env.master_port}"
        if token is not None:
            st.wait(["dnn/store_server"])
            got = st.get("dnn/store_server").decode()
            proc = getattr(self, "_store_proc", None)
            if got != token or (proc is not None and proc.poll() is not None):
                raise CommError(f"the rendezvous store on {where} is not this job's (token {got!r}, expected "
                                f"{token!r}; store child exit code {proc.poll() if proc is not None else None}): "
                                "a server from an earlier job still holds the port - wait for it to exit "
                                f"(<= {self.STALE_BEAT_S:.0f} s after its job's last heartbeat) or use another MASTER_PORT")
        if st.add("dnn/closed", 0) != 0 or st.add("dnn/dropped", 0) != 0:
            raise CommError(f"the rendezvous store on {where} belongs to a finished job (ranks have checked out)")
        now = time.time()
        for r in range(self.env.world):
            k = f"dnn/hb/{r}"
            if st.check([k]):
                try:
                    age = now - float(st.get(k).decode())
                except ValueError:
                    continue
                if age > self.STALE_BEAT_S:
                    raise CommError(f"the rendezvous store on {where} holds a {age:.0f} s old heartbeat of rank {r}: "
                                    "it belongs to an earlier job")

    def _init_group(self) -> None:
        assert self.store is not None
        prefix = dist.PrefixStore(f"dnn/g{self.generation}", self.store)
        # The default group's store keys carry torch's group counter, which only
        # destroy_process_group resets - and only when it completes.  After a recovery whose
        # teardown raised part-way, survivors could name the new group differently and wait
        # for each other's gloo rendezvous keys until the group timeout: every generation
        # starts from the same name.
        dc = dist.distributed_c10d
        if not dist.is_initialized() and hasattr(dc, "_world"):
            dc._world.group_count = 0
        kwargs = {}
        if self.backend == "nccl":
            kwargs["device_id"] = self.device
        dist.init_process_group(self.backend, store=prefix, rank=self.rank, world_size=self.world,
                                timeout=self.timeout, **kwargs)
        self.aborted = False

    # -- liveness (fault.Heartbeat installs ``watch``) -------------------------------------
    def lost(self) -> list[int]:
        """Members the heartbeat watchdog has declared dead (original rank ids)."""
        watch = self.watch
        if watch is None:
            return []
        return sorted(set(watch()) & set(self.members))

    def check_alive(self) -> None:
        """Raise ``CommError`` on the calling (main) thread if a member was declared dead.

        The watchdog thread only FLAGS a dead peer (and releases xGMI flag waits through the
        host-mapped abort word); every teardown - ncclCommAbort, process-group destruction -
        happens on the main thread in ``Trainer._recover``, never concurrently with a graph
        replay or a collective the main thread is issuing."""
        lost = self.lost()
        if lost:
            raise CommError(f"peer rank(s) {lost} lost (heartbeat stale / process exited)")
        if self.rccl_error:
            raise CommError("RCCL communicator reported an asynchronous error (ncclCommGetAsyncError)")
        if self.peer_recovery == self.generation:
            raise CommError(f"peers entered recovery of generation {self.generation}")

    def wait_device(self, poll_s: float = 50e-6) -> None:
        """Wait for this rank's queued GPU work without blocking uninterruptibly.

        A collective whose peer died spins on the GPU until its communicator is aborted, so
        ``torch.cuda.synchronize`` could block the main thread forever.  With a liveness
        watch installed, the wait polls an event and raises ``CommError`` as soon as a member
        is declared dead; the caller then aborts on this thread (``Trainer._recover``)."""
        if self.device.type != "cuda":
            return
        if self.watch is None or not self.distributed:
            torch.cuda.synchronize(self.device)
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        while not ev.query():
            self.check_alive()
            time.sleep(poll_s)

    def signal_lost(self) -> None:
        """Watchdog-thread side of a peer loss: only thread-safe, non-blocking actions.  The
        xGMI abort word is a host-mapped word that in-flight kernels poll - setting it
        releases their bounded flag waits, so the GPU drains and the main thread's
        ``wait_device`` returns or raises."""
        xg = getattr(self, "xgmi", None)
        if xg is not None:
            try:
                xg.abort()
            except Exception:
                pass
        nat = getattr(self, "native", None)
        if nat is not None and os.environ.get("HIP_LAUNCH_BLOCKING") == "1":
            # --debug-sync: launches block the main thread until the kernel finishes, so an
            # ncclAllReduce on a dead peer holds it INSIDE the launch, where no interruptible wait
            # runs - only ncclCommAbort from this thread releases it (NCCL's watchdog pattern)
            try:
                nat.abort()
            except Exception:
                pass

    # -- collectives ---------------------------------------------------------------------
    def _avg_op(self):
        return dist.ReduceOp.AVG if self.backend == "nccl" else None

    def _wait(self, w) -> None:
        """Wait for a host-blocking (gloo) collective, interruptibly.

        A gloo ring peer of a dead rank can sit in recv on a LIVE rank that has already
        left the collective, until that rank tears its group down.  With a liveness
        watch installed (fault.Heartbeat), the wait polls and raises as soon as a
        member is declared dead instead of blocking to the group timeout."""
        watch = self.watch
        if watch is None or self.backend == "nccl":
            w.wait()
            return
        members = set(self.members)
        while not w.is_completed():
            lost = set(watch()) & members
            if lost:
                raise CommError(f"peer rank(s) {sorted(lost)} lost during a collective")
            if self.peer_recovery == self.generation:
                raise CommError(f"peers entered recovery of generation {self.generation} during a collective")
            time.sleep(0.0005)
        w.wait()  # re-raises the collective's own error, if any

    def allreduce_(self, t: torch.Tensor, op: str = "avg", async_op: bool = False):
        """In-place all-reduce; ``op`` in {avg, sum, max, min}."""
        if not self.distributed:
            return None
        try:
            if op == "avg":
                aop = self._avg_op()
                if aop is not None:
                    return dist.all_reduce(t, op=aop, async_op=async_op)
                self._wait(dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True))
                t.div_(self.world)
                return None if not async_op else _Done()
            rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
            if async_op or self.backend == "nccl":
                return dist.all_reduce(t, op=rop, async_op=async_op)
            self._wait(dist.all_reduce(t, op=rop, async_op=True))
            return None
        except CommError:
            raise
        except Exception as e:  # gloo raises on a dead peer; nccl after abort/timeout
            raise CommError(str(e)) from e

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> None:
        if not self.distributed:
            return
        try:
            if self.backend == "nccl":
                dist.broadcast(t, src=src)
            else:
                self._wait(dist.broadcast(t, src=src, async_op=True))
        except CommError:
            raise
        except Exception as e:
            raise CommError(str(e)) from e

    def barrier(self) -> None:
        if not self.distributed:
            return
        try:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                self._wait(dist.barrier(async_op=True))
        except CommError:
            raise
        except Exception as e:
            raise CommError(str(e)) from e

    def reduce_scalar(self, x: float, op: str = "max") -> float:
        if not self.distributed:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64,
                         device=self.device if self.backend == "nccl" else "cpu")
        self.allreduce_(t, op)
        if self.backend == "nccl":
            self.wait_device()  # interruptible: the D2H read below would block on a dead peer
        return float(t.item())

    def gather_scalars(self, x: float) -> list[float]:
        """All ranks' values of a scalar (rank order of the current group)."""
        if not self.distributed:
            return [float(x)]
        dev = self.device if self.backend == "nccl" else "cpu"
        t = torch.zeros(self.world, dtype=torch.float64, device=dev)
        t[self.rank] = float(x)
        self.allreduce_(t, "sum")
        if self.backend == "nccl":
            self.wait_device()
        return [float(v) for v in t.cpu().tolist()]

    # -- fault handling --------------------------------------------------------------------
    def abort(self) -> None:
        """Tear down the current communicator without waiting for peers.  Main thread only
        (the watchdog thread calls ``signal_lost``): it aborts the native RCCL communicator
        that captured step graphs use and destroys the process group, so nothing may be
        replaying or issuing collectives concurrently."""
        xg = getattr(self, "xgmi", None)
        if xg is not None:
            try:
                xg.abort()  # releases xGMI flag waits spinning on a dead peer
            except Exception:
                pass
        nat = getattr(self, "native", None)
        if nat is not None:
            try:
                nat.abort()
            except Exception:
                pass
        if self.aborted or not dist.is_initialized():
            self.aborted = True
            return
        self.aborted = True
        pg = None
        try:
            pg = dist.distributed_c10d._get_default_group()
            if self.backend == "nccl":
                be = pg._get_backend(self.device)
                if be is not None and hasattr(be, "abort"):
                    be.abort()
            elif hasattr(pg, "abort"):
                # gloo: close the pairs so a collective still pending on the dead peer (or on
                # a survivor blocked the same way) fails now - destroy_process_group would
                # otherwise wait for it up to the group timeout, and two survivors can each
                # wait on the other's pending ring step
                pg.abort()
        except Exception:
            pass
        if self.backend != "nccl" and pg is not None:
            # the aborted gloo group's destructor joins its work threads, and one of them can
            # sit in a collective on the dead peer until the group timeout: it must not run on
            # this thread (it did, when this frame released ``pg``: an intermittent hang of the
            # rank-drop test).  Unregister it, then let a daemon thread drop the last reference.
            box = [pg]
            del pg
            if _forget_default_group():
                t = threading.Thread(target=box.clear, daemon=True, name="dnn-pg-reaper")
                t.start()
                _REAPERS.append(t)
                return
            pg = box.pop()
        try:
            dist.destroy_process_group()
        except Exception:
            pass

    def reform(self, dead: Sequence[int]) -> None:
        """Re-create the group over the survivors (original rank ids not in ``dead``)."""
        if self.orig_rank in dead:
            raise CommError("a dropped rank cannot join the re-formed group")
        self.abort()
        self.rccl_error = False
        self.members = [r for r in self.members if r not in set(dead)]
        self.generation += 1
        if self.world > 1 or self.force:
            self._init_group()

    def close(self) -> None:
        if self.store is not None:
            try:
                self.store.add("dnn/closed", 1)  # check out (the stand-alone store exits after the last)
            except Exception:
                pass
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


_REAPERS: list[threading.Thread] = []


def _spawn_store_server(port: int, world: int, token: str):
    """Start parallel/store_server.py as a child in its own session (a signal to this rank's
    process group does not reach it) and return the Popen.  A child process, never an exec of
    this one; it imports no GPU runtime.  ``token`` identifies this job's server."""
    import subprocess
    import sys

    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    return subprocess.Popen([sys.executable, "-m", "distributed_neural_network_amd.parallel.store_server",
                             "--port", str(port), "--world", str(world), "--token", token], env=env,
                            start_new_session=True,
                            stdin=subprocess.DEVNULL, cwd=os.path.dirname(os.path.dirname(os.path.dirname(
                                os.path.abspath(__file__)))))


def exit_now_if_reaping(code: int = 0) -> None:
    """End the process at once when an aborted gloo group is still being torn down.

    A reaper thread (``Communicator.abort``) can still be inside the aborted group's
    destructor, waiting for a work thread stuck on the dead peer; a normal interpreter exit
    would then terminate in C++ teardown (SIGABRT) or wait out the group timeout.  The
    entrypoints call this after a finished run: output is flushed, nothing else runs."""
    if any(t.is_alive() for t in _REAPERS):
        import sys

        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(code)


def _forget_default_group() -> bool:
    """Drop torch's registry of the (aborted) default gloo group without ``shutdown()``.

    ``destroy_process_group`` shuts the group down, and a gloo shutdown waits for the work
    threads - one of them can sit in a collective on the dead peer until the group timeout
    (300 s), long after the other survivors wait in the next generation's rendezvous (seen
    as an intermittent hang of the rank-drop test under load).  The aborted group's threads
    end on their own; this clears what destroy_process_group clears, counter included.
    Returns False (caller falls back to destroy_process_group) if torch's internals differ."""
    dc = dist.distributed_c10d
    w = getattr(dc, "_world", None)
    need = ("pg_map", "pg_names", "pg_group_ranks", "pg_backend_config", "pg_to_tag", "tags_to_pg",
            "pg_coalesce_state")
    if w is None or not hasattr(dc, "_update_default_pg") or not all(hasattr(w, n) for n in need):
        return False
    try:
        dc._update_default_pg(None)
        for n in need:
            getattr(w, n).clear()
        if hasattr(dc, "_unregister_all_process_groups"):
            dc._unregister_all_process_groups()
        w.group_count = 0
    except Exception:
        return False
    return not dist.is_initialized()


class _Done:
    def wait(self) -> None:
        return None


class GradAllReduce:
    """Per-step gradient averaging with bucket fusion and comm/compute overlap.

    The engine hands over the flat gradient arena and the bucket ranges in the order
    their gradients become ready.  Each bucket's all-reduce is issued asynchronously
    (RCCL runs it on its own stream); ``before_last`` is the compute that produces
    the last bucket, so it runs on the compute stream concurrently with the earlier
    buckets' all-reduces.  All waits are stream-level (no host sync), so the whole
    sequence can be captured into the step's hipGraph.
    """

    def __init__(self, comm: Communicator, bucket_kb: int = 0) -> None:
        self.comm = comm
        self.bucket_elems = max(0, int(bucket_kb)) * 256  # fp32 elements per bucket (0: no split)

    def allreduce_grads(self, grad: torch.Tensor, buckets: list[tuple[int, int]],
                        before_last: Optional[Callable[[], None]] = None) -> None:
        buckets = split_buckets(buckets, self.bucket_elems)
        works = []
        for i, (lo, hi) in enumerate(buckets):
            if i == len(buckets) - 1 and before_last is not None:
                before_last()
            w = self.comm.allreduce_(grad[lo:hi], "avg", async_op=True)
            if w is not None:
                works.append(w)
        for w in works:
            w.wait()


def split_buckets(buckets: list[tuple[int, int]], max_elems: int) -> list[tuple[int, int]]:
    """``--bucket-kb``: cut each [lo, hi) range into pieces of at most ``max_elems``
    (0 = keep the ranges).  At this model size one fused bucket is latency-optimal; for
    layer-engine models with MB-scale gradients, smaller buckets pipeline the ring."""
    if max_elems <= 0:
        return list(buckets)
    out = []
    for lo, hi in buckets:
        for a in range(lo, hi, max_elems):
            out.append((a, min(hi, a + max_elems)))
    return out


def wait_for_store_key(store: dist.Store, key: str, timeout_s: float) -> bool:
    deadline = time.time() + timeout_s
    while time.time() < deadline:
        try:
            if store.check([key]):
                return True
        except Exception:
            return False
        time.sleep(0.05)
    return False
