"""Failure injection, detection and recovery.

Capability parity:
  * ``simulate_failure`` (data_parallelism_train.py:41-46, flags :266-269): with
    probability p a rank prints ``Process {rank} failed! Sleeping for {d} seconds.``,
    sleeps d seconds, prints ``Process {rank} woke up!`` - once per epoch, called by
    the parent before the broadcast (:117) and by every child before training (:141).
    A straggler, not a crash; reproduced verbatim (but seeded, so runs are repeatable).
  * The reference has no detection and no recovery: a dead rank would
    leave the parent blocked in ``comm.recv()`` forever.  Here:
      - ``DropInjector``: ``--drop-rank R --drop-at-epoch E [--drop-at-step S]`` makes
        rank R die hard (``os._exit``, no cleanup) at that point;
      - ``Heartbeat``: every rank stamps ``hb/<rank>`` in the rendezvous TCPStore from
        a background thread every 0.1 s; a watchdog marks a rank dead when its stamp is
        older than ``DNN_HEARTBEAT_TIMEOUT`` (1 s), when the launcher reports the rank's
        process gone (``dead/<rank>``, parallel/launch.py - detection within ~0.1 s), or
        when the native RCCL communicator reports an asynchronous error
        (``ncclCommGetAsyncError``).
        The thread only flags it (and sets the xGMI abort word, which in-flight kernels
        poll); the main thread notices between graph replays and in its interruptible
        waits (``Communicator.check_alive`` / ``wait_device``), raises ``CommError`` and
        aborts RCCL / the process group itself, so no teardown ever races a replay or a
        collective (gloo collectives also fail fast on a closed peer socket);
      - ``agree_survivors``: the survivors agree on the new member list through the
        store (first survivor to win a compare_set is the leader and publishes it);
      - the trainer then re-forms the communicator over the survivors
        (Communicator.reform: abort + new generation group), restores the last
        consistent parameters (start-of-epoch snapshot), re-partitions the data over
        the new world size and re-runs the epoch, reporting recovery latency.
"""
from __future__ import annotations

import os
import socket
import threading
import time
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .comm import Communicator

DROP_EXIT_CODE = 17


def simulate_failure(rank: int, probability: float, duration: float, rng: np.random.Generator) -> bool:
    """Reference straggler injection; returns True if this rank slept."""
    if probability > 0 and rng.random() < probability:
        print(f"Process {rank} failed! Sleeping for {duration} seconds.", flush=True)
        time.sleep(float(duration))
        print(f"Process {rank} woke up!", flush=True)
        return True
    return False


@dataclass
class DropInjector:
    rank: Optional[int] = None
    at_epoch: int = 0
    at_step: int = 0

    def active(self) -> bool:
        return self.rank is not None and self.rank >= 0

    def step_limit(self, orig_rank: int, epoch: int) -> Optional[int]:
        """Steps this rank may run in ``epoch`` before it must die (None: no limit)."""
        if self.active() and orig_rank == self.rank and epoch == self.at_epoch:
            return self.at_step
        return None

    def die(self, orig_rank: int, epoch: int, step: int, store=None) -> None:
        t = time.time()
        if store is not None:
            try:  # the kill time, for the survivors' detection latency (tools/fault_bench.py)
                store.set(f"dnn/drop_time/{orig_rank}", repr(t))
            except Exception:
                pass
        print(f"[fault] injected drop: rank {orig_rank} exits at epoch {epoch} step {step} (t={t:.6f})", flush=True)
        os._exit(DROP_EXIT_CODE)


class Heartbeat:
    """Background heartbeat + watchdog over the rendezvous TCPStore."""

    def __init__(self, comm: Communicator, period_s: float = 0.1, timeout_s: float | None = None) -> None:
        import torch.distributed as dist

        self.comm = comm
        self.period = period_s
        # DNN_HEARTBEAT_TIMEOUT: seconds without a beat before a peer is flagged (default
        # 1 s + 0.1 s per rank: more ranks on one host, more beat-thread contention).  The
        # effective timeout also follows the beat jitter actually observed: at least 4x the p99
        # gap between a peer's consecutive beats (``timeout``).  A flag only starts a recovery;
        # a live rank whose beat was late still announces itself alive in the agreement and
        # keeps its place (an all-alive retry; ``clear`` drops the flag).  Launcher-reported
        # deaths (dnn/dead/<r>) bypass all of this and are flagged within one period.
        env_t = os.environ.get("DNN_HEARTBEAT_TIMEOUT")
        self.base_timeout = (float(env_t) if env_t else 1.0 + 0.1 * comm.world) if timeout_s is None else timeout_s
        self._gaps: list[float] = []  # recent gaps between a peer's consecutive beat stamps (s)
        self._last_val: dict[int, float] = {}
        self.dead: set[int] = set()
        self.done: set[int] = set()  # peers that checked out (finished normally; never flagged)
        self.detected_at: dict[int, float] = {}  # rank -> time.time() when the watchdog flagged it
        # rank -> time its flag was cleared by a recovery agreement: staleness counts from here,
        # so a rank that was only late gets a full timeout to beat again before a new flag
        self.grace: dict[int, float] = {}
        self.paused_until = 0.0  # fault injection (DNN_INJECT_BEAT_PAUSE): this rank's beats stop
        self._stop = threading.Event()
        env = comm.env
        # a private client connection for the thread
        self.store = dist.TCPStore(env.master_addr, env.master_port, env.world, is_master=False,
                                   timeout=comm.timeout)
        # process identity: a peer on the same host whose process is gone is dead at once, even
        # with no launcher to report it (mpiexec / plain env launches) - a stale beat alone only
        # starts the (patient) agreement
        self.host = socket.gethostname()
        self.store.set(f"dnn/pid/{comm.orig_rank}", f"{self.host}:{os.getpid()}")
        self._pids: dict[int, Optional[int]] = {}
        self._beat()
        comm.watch = lambda: tuple(self.dead)  # makes host-blocking collectives interruptible
        self._thread = threading.Thread(target=self._run, name="dnn-heartbeat", daemon=True)
        self._thread.start()

    JITTER_FACTOR = 4.0

    @property
    def timeout(self) -> float:
        """Base timeout, raised to JITTER_FACTOR x the p99 observed beat gap (last 256 gaps)."""
        g = sorted(self._gaps)
        p99 = g[min(len(g) - 1, int(0.99 * len(g)))] if g else 0.0
        return max(self.base_timeout, self.JITTER_FACTOR * p99)

    def _observe(self, rank: int, stamp: float) -> None:
        prev = self._last_val.get(rank)
        if prev is not None and stamp > prev:
            self._gaps.append(stamp - prev)
            if len(self._gaps) > 256:
                del self._gaps[:-256]
        self._last_val[rank] = stamp

    def _beat(self) -> None:
        if time.time() < self.paused_until:
            return
        self.store.set(f"dnn/hb/{self.comm.orig_rank}", repr(time.time()))

    def last_seen(self, rank: int) -> float:
        try:
            if not self.store.check([f"dnn/hb/{rank}"]):
                return 0.0
            return float(self.store.get(f"dnn/hb/{rank}").decode())
        except Exception:
            return 0.0

    def stale(self, rank: int) -> bool:
        seen = self.last_seen(rank)
        if seen and rank not in self.dead:
            self._observe(rank, seen)
        return time.time() - max(seen, self.grace.get(rank, 0.0)) > self.timeout

    def reported_dead(self, rank: int) -> bool:
        """The rank's process is known to be gone: the launcher saw it exit (parallel/launch.py,
        selflaunch.py, torchrun's agent publish ``dnn/dead/<r>``), or it ran on this host and its
        pid no longer names a live process."""
        try:
            if self.store.check([f"dnn/dead/{rank}"]):
                return True
        except Exception:
            return False
        return self._local_pid_gone(rank)

    def check_out(self) -> None:
        """This rank finished its run normally (``Trainer._finish``, after the final barrier):
        peers must never take its exit for a death.  Written BEFORE the process exits, so a peer
        that sees the pid gone (or the launcher's notice) and THEN reads this key always finds it
        (``_run`` tests in that order)."""
        self.store.set(f"dnn/done/{self.comm.orig_rank}", repr(time.time()))

    def checked_out(self, rank: int) -> bool:
        if rank in self.done:
            return True
        try:
            if self.store.check([f"dnn/done/{rank}"]):
                self.done.add(rank)
                return True
        except Exception:
            pass
        return False

    def _local_pid_gone(self, rank: int) -> bool:
        if rank not in self._pids:
            pid = None
            try:
                if self.store.check([f"dnn/pid/{rank}"]):
                    host, _, p = self.store.get(f"dnn/pid/{rank}").decode().rpartition(":")
                    pid = int(p) if host == self.host else None
                else:
                    return False  # not registered yet: ask again later
            except Exception:
                return False
            self._pids[rank] = pid
        pid = self._pids[rank]
        return pid is not None and not pid_alive(pid)

    def _flag(self, r: int, why: str) -> None:
        self.dead.add(r)
        self.detected_at.setdefault(r, time.time())
        print(f"[fault] watchdog: rank {r} {why}", flush=True)
        # flag only: the main thread sees ``comm.lost()`` between graph replays / in its
        # interruptible waits and does every teardown (ncclCommAbort, group destruction)
        # itself in Trainer._recover
        self.comm.signal_lost()

    def clear(self, members) -> None:
        """Members of the re-formed group are alive by agreement: drop their flags."""
        now = time.time()
        for r in members:
            self.dead.discard(r)
            self.detected_at.pop(r, None)
            self.grace[r] = now

    def _run(self) -> None:
        while not self._stop.wait(self.period):
            try:
                self._beat()
                for r in list(self.comm.members):
                    if r == self.comm.orig_rank or r in self.dead or r in self.done:
                        continue
                    # order matters: liveness first, then the check-out - a rank writes its
                    # check-out before it exits, so a gone process whose key is not there yet
                    # cannot be a normal exit
                    gone = self.reported_dead(r)
                    if self.checked_out(r):
                        continue  # finished its run: its exit and its silence are not a death
                    if gone:
                        self._flag(r, "process exited (reported by the launcher)")
                    elif self.stale(r):
                        self._flag(r, f"heartbeat stale > {self.timeout}s")
                # peers started a recovery of this generation (a live rank they flagged, or a
                # failed collective on their side): join it instead of waiting in a collective
                # they have left
                gen = self.comm.generation
                if self.comm.peer_recovery != gen and self.store.check([f"dnn/recover/{gen}/begun"]):
                    self.comm.peer_recovery = gen
                    self.comm.signal_lost()
                # native RCCL: an asynchronous error (e.g. ncclRemoteError after a peer died)
                # flags the communicator itself; check_alive raises on the main thread
                nat = getattr(self.comm, "native", None)
                if nat is not None and not self.comm.rccl_error and not nat.healthy():
                    self.comm.rccl_error = True
                    print("[fault] watchdog: RCCL communicator reports an asynchronous error", flush=True)
                    self.comm.signal_lost()
            except Exception:
                pass

    def stop(self) -> None:
        self.comm.watch = None
        self._stop.set()
        self._thread.join(timeout=2.0)


def pid_alive(pid: int) -> bool:
    """Does ``pid`` name a live (not zombie) process on this host?"""
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except OSError:
        return True  # no /proc: kill(0) said it exists


def announce_alive(comm: Communicator) -> None:
    """Mark this rank alive for generation g's agreement.  Called BEFORE tearing the broken
    group down: destroying a gloo group can block until a collective pending on the dead
    peer times out (~30 s), and a survivor that announced itself only afterwards used to
    miss the agreement deadline and get excluded."""
    assert comm.store is not None
    comm.store.set(f"dnn/recover/{comm.generation}/alive/{comm.orig_rank}", "1")
    comm.store.set(f"dnn/recover/{comm.generation}/begun", str(comm.orig_rank))


def exclusion_grace(hb: Heartbeat) -> float:
    """Seconds a heartbeat-only-stale rank gets to announce itself before it is excluded
    (``DNN_EXCLUDE_GRACE_S``, default max(10 s, 2 heartbeat timeouts)).  Separate from the
    flagging timeout: a whole-process stall of a few seconds (swap, a long GIL hold, SIGSTOP,
    host contention) costs an all-alive retry, never the rank's place."""
    env = os.environ.get("DNN_EXCLUDE_GRACE_S")
    return float(env) if env else max(10.0, 2.0 * hb.timeout)


def agree_survivors(comm: Communicator, hb: Heartbeat, wait_s: float = 30.0, grace_s: float | None = None) -> list[int]:
    """Survivors of generation g agree on the member list of generation g+1.

    A member is alive once it announced itself (``announce_alive``).  It is dead at once if the
    launcher reported its process gone, and dead after ``grace_s`` (``exclusion_grace``) if its
    heartbeat is stale - a live rank whose beat was only late reaches its own recovery (its next
    collective fails once the others tore their group down, or its watchdog sees the recovery
    begin) and announces itself within that grace, so it stays in the group: the recovery is an
    all-alive retry.  Ranks neither stale nor announced are waited for up to ``wait_s``."""
    assert comm.store is not None
    st = comm.store
    p = f"dnn/recover/{comm.generation}/"
    st.set(f"{p}alive/{comm.orig_rank}", "1")
    grace = exclusion_grace(hb) if grace_s is None else grace_s
    wait_s = max(wait_s, grace + 5.0)
    t0 = time.time()
    deadline = t0 + wait_s
    while True:
        alive, undecided = [], []
        for r in comm.members:
            if st.check([f"{p}alive/{r}"]):
                alive.append(r)
            elif hb.reported_dead(r) or (hb.stale(r) and time.time() - t0 > grace):
                pass  # dead
            else:
                undecided.append(r)
        if not undecided or time.time() > deadline:
            break
        time.sleep(0.02)
    # first survivor to win the compare_set publishes the member list
    won = st.compare_set(f"{p}leader", "", str(comm.orig_rank)).decode() == str(comm.orig_rank)
    if won:
        st.set(f"{p}members", ",".join(str(r) for r in sorted(alive)))
    st.wait([f"{p}members"])
    members = [int(x) for x in st.get(f"{p}members").decode().split(",") if x]
    return members


def stall_injection(orig_rank: int, epoch: int) -> tuple[str, float]:
    """Fault injection for tests: a WHOLE-process stall of a live rank at the start of an epoch.
    ``DNN_INJECT_STALL=rank:epoch:seconds[:kind]``, kind ``sigstop`` (default: the process is
    stopped, every thread included, and a helper process continues it) or ``gil`` (the main
    thread holds the GIL - a long C call - so the heartbeat thread cannot beat).  Returns
    (kind, seconds); seconds 0: none."""
    spec = os.environ.get("DNN_INJECT_STALL", "")
    if not spec:
        return "", 0.0
    parts = spec.split(":")
    r, e, d = int(parts[0]), int(parts[1]), float(parts[2])
    kind = parts[3] if len(parts) > 3 else "sigstop"
    return (kind, d) if r == orig_rank and e == epoch else ("", 0.0)


def stall_process(kind: str, seconds: float) -> None:
    """Carry out a ``stall_injection``."""
    import signal
    import subprocess
    import sys

    print(f"[fault] injected {kind} stall: this process stops for {seconds} s", flush=True)
    if kind == "gil":
        old = sys.getswitchinterval()
        sys.setswitchinterval(seconds + 1.0)  # no other thread gets the GIL while this one spins
        t_end = time.time() + seconds
        try:
            while time.time() < t_end:
                pass
        finally:
            sys.setswitchinterval(old)
        return
    subprocess.Popen(["/bin/sh", "-c", f"sleep {seconds}; kill -CONT {os.getpid()}"], start_new_session=True)
    os.kill(os.getpid(), signal.SIGSTOP)


def end_skew_injection(orig_rank: int, where: str = "before") -> float:
    """Fault injection for tests (``DNN_INJECT_END_SKEW=rank:seconds[:after]``): that rank idles
    this long after the last epoch's last collective - before the final barrier (default: its
    peers wait in the barrier), or ``after`` it (its peers check out and exit first, while its
    watchdog still runs).  Returns the delay for the point ``where`` (0: none)."""
    spec = os.environ.get("DNN_INJECT_END_SKEW", "")
    if not spec:
        return 0.0
    parts = spec.split(":")
    at = parts[2] if len(parts) > 2 else "before"
    return float(parts[1]) if int(parts[0]) == orig_rank and at == where else 0.0


_RECOVERY_FAULTS_DONE: set = set()


def recovery_fault_injection(orig_rank: int, generation: int) -> bool:
    """Fault injection for tests (``DNN_INJECT_RECOVERY_FAIL=rank:generation``): that rank's
    recovery fails ONCE right after it re-formed the group into that generation, before the new
    group's barrier (as if a survivor were flagged mid-recovery) - the trainer must start the
    recovery over instead of dying.  Returns whether to fail now."""
    spec = os.environ.get("DNN_INJECT_RECOVERY_FAIL", "")
    if not spec:
        return False
    r, g = (int(x) for x in spec.split(":"))
    if r != orig_rank or g != generation or (r, g) in _RECOVERY_FAULTS_DONE:
        return False
    _RECOVERY_FAULTS_DONE.add((r, g))
    return True


def beat_pause_injection(orig_rank: int, epoch: int) -> float:
    """Fault injection for tests (``DNN_INJECT_BEAT_PAUSE=rank:epoch:seconds``): this rank's
    heartbeat thread stops beating for that long at the start of that epoch while the rank itself
    keeps training - a live rank that LOOKS dead.  Returns the pause (0: none)."""
    spec = os.environ.get("DNN_INJECT_BEAT_PAUSE", "")
    if not spec:
        return 0.0
    r, e, d = spec.split(":")
    return float(d) if int(r) == orig_rank and int(e) == epoch else 0.0


def setup_crash_injection(site: str, orig_rank: int) -> None:
    """Fault injection for tests: the process dies (exit code 134, as a GPU fault's abort) at a
    set-up site of the FIRST launch attempt only, so the launcher's retry in fresh ranks
    (parallel/selflaunch.py) can be exercised.  ``DNN_INJECT_XGMI_SETUP_FAIL=rank`` hits the xGMI
    group set-up (parallel/xgmi.py, before any IPC mapping is made); ``DNN_INJECT_CRASH=site:rank``
    any named site."""
    import sys

    if os.environ.get("DNN_LAUNCH_ATTEMPT", "1") != "1":
        return
    want = []
    v = os.environ.get("DNN_INJECT_XGMI_SETUP_FAIL", "")
    if v != "":
        want.append(("xgmi-setup", int(v)))
    spec = os.environ.get("DNN_INJECT_CRASH", "")
    if spec:
        s, r = spec.rsplit(":", 1)
        want.append((s, int(r)))
    if (site, orig_rank) in want:
        print(f"[fault] injected crash at {site} on rank {orig_rank} (launch attempt 1)", file=sys.stderr, flush=True)
        os._exit(134)
