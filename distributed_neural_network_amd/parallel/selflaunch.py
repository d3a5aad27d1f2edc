"""Self-launch: a script run as plain ``python script.py --gpus N`` spawns its own N ranks.

Capability parity: the reference's headline experiment is a process-count sweep launched by
``mpiexec -n {N} python data_parallelism_train.py --nb-proc {N}`` (README.md:28,
run_training.sh:1-3).  ``bench.py --gpus N`` must produce its number whether a launcher
(torchrun, mpiexec, parallel/launch.py) started the ranks or not, so when it finds no launcher
environment it becomes its own launcher:

* it runs BEFORE anything touches the GPU (no HIP call, no ``torch.cuda.is_available()``): the
  parent only counts devices (KFD topology in sysfs + the visibility variables, never a HIP
  call), hosts the rendezvous TCPStore (so any rank may die and the others
  still see it: ``dnn/dead/<rank>`` is published the moment a child fails, as in
  parallel/launch.py) and starts N children with ``subprocess`` - never an exec;
* every child gets RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1 / MASTER_PORT and
  ``DNN_STORE_EXTERNAL=1``; when N exceeds the visible GPUs (a one-GPU rehearsal) the ranks
  share devices, RCCL refuses that, so the host collectives default to gloo
  (``DNN_BACKEND=gloo``);
* the children's stderr is relayed line by line with a ``[rK]`` prefix, their stdout is kept;
  the parent writes rank 0's last JSON line to its own stdout and exits 0 - or, if any rank
  failed (or rank 0 printed no JSON), prints every failed rank's stderr tail and exits with the
  first failing rank's code.  Once one rank has failed, the others get ``grace_s`` to finish
  before their process groups are terminated, so a rank stuck on a dead peer cannot hold the
  job forever;
* a job that ends without rank 0's result line is RETRIED in fresh children with a more
  conservative transport (``ATTEMPTS``: as requested -> RCCL without any xGMI group -> gloo host
  collectives), within a wall budget; the result line then carries ``launch_attempts``,
  ``launch_transport`` and ``launch_failures`` (first failing rank, exit code, phase, stderr tail);
* under torchrun (which launched the ranks itself) every rank process becomes a supervisor of
  one child and the supervisors run the same attempt plan together (``supervise``).
"""
from __future__ import annotations

import collections
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import IO, Optional, Sequence

from .. import hsa_env


def launcher_present(env: Optional[dict] = None) -> bool:
    """True if a launcher already set up this process as one rank of a job."""
    e = os.environ if env is None else env
    return any(e.get(k) not in (None, "") for k in ("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE",
                                                      "SLURM_NTASKS"))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _kfd_gpu_nodes(root: str = "/sys/class/kfd/kfd/topology/nodes", dri: str = "/dev/dri") -> int:
    """GPU nodes of the KFD topology that this process can open (sysfs: a node with a non-zero
    ``gfx_target_version`` is a GPU; it counts only if its render node ``/dev/dri/renderD<minor>``
    is accessible - a container sees every GPU of the host in the topology but gets only its own
    render nodes, which is the filter the ROCm runtime applies).  -1 if the topology cannot be read."""
    try:
        names = os.listdir(root)
    except OSError:
        return -1
    n = 0
    for d in names:
        props = {}
        try:
            with open(os.path.join(root, d, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    props[k] = v.strip()
        except OSError:
            continue
        try:
            if int(props.get("gfx_target_version", "0") or 0) == 0:
                continue
        except ValueError:
            continue
        minor = props.get("drm_render_minor")
        if minor is not None and os.path.isdir(dri):
            if not os.access(os.path.join(dri, f"renderD{minor}"), os.R_OK | os.W_OK):
                continue
        n += 1
    return n


def _visible_list(n_nodes: int) -> int:
    """Apply the runtime's visibility masks (ROCR_, then HIP_ / CUDA_VISIBLE_DEVICES) to n_nodes."""
    n = n_nodes
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(k)
        if v is None:
            continue
        ids = [x for x in v.split(",") if x.strip() != ""]
        n = min(n, len(ids)) if n >= 0 else len(ids)
    return n


def visible_devices() -> int:
    """GPUs this process could use, counted WITHOUT any HIP call in this process (the launcher
    must not initialise the GPU runtime: its children are started from it).  Reads the KFD
    topology in sysfs and the visibility variables; if sysfs is unreadable, a short-lived child
    process asks torch (whatever that initialises dies with the child)."""
    n = _kfd_gpu_nodes()
    if n >= 0:
        return max(0, _visible_list(n))
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=300)
        return int(r.stdout.strip().splitlines()[-1])
    except Exception:
        return 0


def die_with_parent() -> None:
    """Called by a self-launched rank (``DNN_SELF_LAUNCHED=1``) at its start: SIGKILL it when the
    launcher dies (a driver timeout that kills the launcher must not leave ranks holding GPUs in
    their own sessions).  The rank sets this itself - the launcher passes no preexec_fn, which
    would force fork + exec in a copy of a multi-threaded parent.  If the launcher is already gone
    (it died before this call), the rank exits at once."""
    if os.environ.get("DNN_SELF_LAUNCHED") != "1":
        return
    try:
        import ctypes

        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)  # PR_SET_PDEATHSIG
    except Exception:
        return
    want = os.environ.get("DNN_LAUNCHER_PID")
    if want and os.getppid() != int(want):
        os._exit(1)


class _Child:
    def __init__(self, rank: int, proc: subprocess.Popen, tail: int) -> None:
        self.rank, self.proc = rank, proc
        self.err_tail: collections.deque[str] = collections.deque(maxlen=tail)
        self.out: list[str] = []
        self.threads: list[threading.Thread] = []
        self.saw_window = False  # this rank printed WINDOW_MARK (its timed window started)

    def keep_err(self, line: str) -> None:
        self.err_tail.append(line)
        if WINDOW_MARK in line:
            self.saw_window = True

    def result(self) -> str | None:
        """The last JSON object line this rank printed on stdout."""
        found = None
        for line in self.out:
            s = line.strip()
            if s.startswith("{"):
                try:
                    json.loads(s)
                    found = s
                except ValueError:
                    pass
        return found


def _pump(stream: IO[str], sink, keep) -> None:
    for line in stream:
        keep(line)
        if sink is not None:
            try:
                sink.write(line)
                sink.flush()
            except Exception:
                pass


def _prefixed(rank: int, out: IO[str], attempt: int = 1):
    tag = f"[r{rank}] " if attempt == 1 else f"[r{rank} a{attempt}] "

    class _W:
        def write(self, s: str) -> None:
            out.write(tag + s if s.strip() else s)

        def flush(self) -> None:
            out.flush()

    return _W()


# ---- bounded retry in fresh children with a conservative transport -------------------------------
#
# The first multi-GPU run on a node is the first time cross-device IPC of uncached memory, RCCL with
# more than one rank and N co-resident persistent grids polling remote granules execute.  A fault
# there (a GPU page fault aborts the process; one rank gone takes the job with it) must not leave the
# job without a number.  The launcher has never touched the GPU, so it can start a FRESH set of
# ranks with a more conservative transport - and says so in the result line (``launch_attempts``,
# ``launch_failures``: the failing rank, its exit code, the phase and its stderr tail), so the fault
# is reported, not hidden.  The reference had no such path: a dead MPI rank hung or aborted the
# whole job (data_parallelism_train.py:118,210).
ATTEMPTS: tuple[tuple[str, dict], ...] = (
    ("as requested", {}),
    # no xGMI group at all (no IPC mapping, no in-launch exchange, no persistent grid polling a
    # peer): the per-step all-reduce is native RCCL (nccl process group) - or the process group
    # itself when the ranks already use host collectives (gloo: shared-GPU rehearsals)
    ("rccl: no xGMI group, no in-launch exchange", {"DNN_SAFE_TRANSPORT": "1", "DNN_ALLREDUCE": "rccl"}),
    # no RCCL either: gloo host collectives, eager launches (slow, but it yields a number)
    ("gloo host collectives: no RCCL, no xGMI, eager launches",
     {"DNN_SAFE_TRANSPORT": "2", "DNN_ALLREDUCE": "rccl", "DNN_BACKEND": "gloo"}),
)
# printed on stderr by bench.py right before its timed window (the launcher records whether the
# first failure came before it)
WINDOW_MARK = "timed window start"


def attempt_plan(env: Optional[dict] = None) -> list[tuple[str, dict]]:
    """The attempts a launch may use: ``DNN_LAUNCH_ATTEMPTS`` (default all of ATTEMPTS; 1 = no
    retry)."""
    e = os.environ if env is None else env
    n = int(e.get("DNN_LAUNCH_ATTEMPTS", str(len(ATTEMPTS))) or len(ATTEMPTS))
    return list(ATTEMPTS[:max(1, min(n, len(ATTEMPTS)))])


def _pre_window_grace(grace_s: float) -> float:
    """Grace after a failure for ranks that have not started their timed window: they cannot
    produce a result any more (every collective before the window needs the dead rank), so they
    are stopped sooner - ``DNN_PREWINDOW_GRACE_S`` (10 s), at most ``grace_s``."""
    return min(grace_s, float(os.environ.get("DNN_PREWINDOW_GRACE_S", "10")))


def _budget(env: Optional[dict] = None) -> tuple[float, float]:
    """(job wall budget: no new attempt starts after it, one attempt's wall limit) in seconds:
    ``DNN_LAUNCH_BUDGET_S`` (1500), ``DNN_ATTEMPT_TIMEOUT_S`` (900; 0 = none)."""
    e = os.environ if env is None else env
    return float(e.get("DNN_LAUNCH_BUDGET_S", "1500")), float(e.get("DNN_ATTEMPT_TIMEOUT_S", "900"))


class _Attempt:
    """Outcome of one attempt: rank 0's result line, every rank's exit code, the order ranks
    failed in (the first is the root cause), stderr tails, whether the timed window started."""

    def __init__(self, number: int, transport: str) -> None:
        self.number, self.transport = number, transport
        self.result: str | None = None
        self.codes: dict[int, int | None] = {}
        self.fail_order: list[int] = []
        self.tails: dict[int, list[str]] = {}
        self.saw_window = False
        self.timed_out = False
        self.wall_s = 0.0

    def failure(self) -> dict:
        r = self.fail_order[0] if self.fail_order else 0
        if self.timed_out:
            why = "attempt wall limit reached"
        elif self.fail_order:
            why = f"rank {r} exited with code {self.codes.get(r)}"
        else:
            why = "rank 0 printed no result line"
        return {"attempt": self.number, "transport": self.transport, "rank": r, "exit_code": self.codes.get(r),
                "reason": why, "phase": "after the timed window started" if self.saw_window
                else "before the timed window", "wall_s": round(self.wall_s, 3),
                "stderr_tail": [ln.rstrip() for ln in self.tails.get(r, [])][-12:]}

    def first_code(self) -> int:
        for r in self.fail_order:
            c = self.codes.get(r)
            if c:
                return c
        return 1


def annotate(result: str, attempts: Sequence[_Attempt]) -> str:
    """Rank 0's JSON line plus the launch record: ``launch_attempts`` always; after a retry also
    ``launch_transport`` (the attempt that produced the number) and ``launch_failures``."""
    out = json.loads(result)
    out["launch_attempts"] = len(attempts)
    if len(attempts) > 1:
        out["launch_transport"] = attempts[-1].transport
        out["launch_failures"] = [a.failure() for a in attempts[:-1]]
    return json.dumps(out)


def _stop(children: Sequence[_Child], codes: dict, sig: int) -> None:
    for c in children:
        if c.rank not in codes:
            _kill_group(c.proc, sig)


def _attempt_local(cmd: Sequence[str], nproc: int, number: int, transport: str, base: dict, grace_s: float,
                   tail_lines: int, err: IO[str], timeout_s: float, t_launch: float) -> _Attempt:
    """One attempt of ``run``: a fresh store and N fresh children; returns when all have exited."""
    import torch.distributed as dist

    att = _Attempt(number, transport)
    port = _free_port()
    t0 = time.time()
    store = dist.TCPStore("127.0.0.1", port, nproc + 1, is_master=True, wait_for_workers=False)
    children: list[_Child] = []
    for r in range(nproc):
        env = dict(base)
        env.update(RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(nproc),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DNN_STORE_EXTERNAL="1",
                   DNN_SELF_LAUNCHED="1", DNN_LAUNCHER_PID=str(os.getpid()), PYTHONUNBUFFERED="1",
                   DNN_LAUNCH_ATTEMPT=str(number))
        p = subprocess.Popen(list(cmd), env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             bufsize=1, start_new_session=True, stdin=subprocess.DEVNULL)
        children.append(_Child(r, p, tail_lines))
    # the relay threads start only once every child exists (no child is spawned while they run)
    for c in children:
        r, p = c.rank, c.proc
        c.threads = [threading.Thread(target=_pump, args=(p.stderr, _prefixed(r, err, number), c.keep_err), daemon=True),
                     threading.Thread(target=_pump, args=(p.stdout, None if r == 0 else _prefixed(r, err, number),
                                                          c.out.append), daemon=True)]
        for t in c.threads:
            t.start()
    print(f"[launch +{time.time() - t_launch:.3f}s] attempt {number} ({transport}): store on 127.0.0.1:{port}, "
          f"{nproc} ranks started", file=err, flush=True)

    def _forward(signum, frame):  # the launcher is being stopped: stop the ranks first
        for c in children:
            _kill_group(c.proc, signal.SIGTERM)
        time.sleep(2.0)
        for c in children:
            _kill_group(c.proc, signal.SIGKILL)
        raise SystemExit(128 + signum)

    prev = {sig: signal.signal(sig, _forward) for sig in (signal.SIGTERM, signal.SIGINT)} \
        if threading.current_thread() is threading.main_thread() else {}

    codes: dict[int, int] = {}
    first_fail: float | None = None
    terminated = False
    try:
        while len(codes) < nproc:
            for c in children:
                if c.rank in codes:
                    continue
                rc = c.proc.poll()
                if rc is None:
                    continue
                codes[c.rank] = rc
                if rc != 0:
                    att.fail_order.append(c.rank)
                    try:
                        store.set(f"dnn/dead/{c.rank}", repr(time.time()))
                    except Exception:
                        pass
                    print(f"[launch +{time.time() - t_launch:.3f}s] rank {c.rank} exited with code {rc}", file=err,
                          flush=True)
                    if first_fail is None:
                        first_fail = time.time()
            now = time.time()
            # (no rank past its window mark: nothing left to wait for, the shorter grace applies)
            grace = grace_s if any(c.saw_window for c in children) else _pre_window_grace(grace_s)
            if timeout_s > 0 and now - t0 > timeout_s and first_fail is None:
                print(f"[launch] attempt {number} still running after its wall limit ({timeout_s:.0f} s): "
                      "terminating its ranks", file=err, flush=True)
                att.timed_out = True
                first_fail = now - grace  # (terminate now, kill 10 s later)
            if first_fail is not None and now - first_fail > grace and not terminated:
                for c in children:
                    if c.rank not in codes:
                        print(f"[launch] rank {c.rank} still running {grace:.0f} s after a failure: terminating it",
                              file=err, flush=True)
                _stop(children, codes, signal.SIGTERM)
                terminated = True
            if first_fail is not None and now - first_fail > grace + 10:
                _stop(children, codes, signal.SIGKILL)
            time.sleep(0.02)
    finally:
        for sig, h in prev.items():
            signal.signal(sig, h)
    for c in children:
        for t in c.threads:
            t.join(timeout=5.0)
    del store
    att.codes = dict(codes)
    att.tails = {c.rank: list(c.err_tail) for c in children}
    att.saw_window = any(c.saw_window for c in children)
    att.result = children[0].result()
    att.wall_s = time.time() - t0
    if att.timed_out and 0 not in att.fail_order:
        att.fail_order = att.fail_order or [0]
    return att


def run(cmd: Sequence[str], nproc: int, out_fd: int | None = None, extra_env: Optional[dict] = None,
        grace_s: float = 60.0, tail_lines: int = 40, err: IO[str] | None = None) -> int:
    """Run ``cmd`` as ``nproc`` ranks of one job (see the module docstring), retrying a failed job
    in fresh children with the next transport of ``attempt_plan()``; returns the exit code.
    ``out_fd``: where rank 0's (annotated) JSON line goes (default: fd 1)."""
    err = err or sys.stderr
    t_launch = time.time()
    base = hsa_env.strip(dict(os.environ))  # (ranks of a multi-rank job keep the runtime's defaults)
    base.update(extra_env or {})
    ndev = visible_devices()
    print(f"[launch] {ndev} GPU(s) visible to this job (KFD topology + visibility variables)", file=err, flush=True)
    if nproc > max(ndev, 1) and not base.get("DNN_BACKEND"):
        base["DNN_BACKEND"] = "gloo"
        print(f"[launch] {nproc} ranks on {ndev} visible GPU(s): ranks share devices, host collectives over gloo",
              file=err, flush=True)
    plan = attempt_plan(base)
    budget, timeout_s = _budget(base)
    done: list[_Attempt] = []
    for number, (transport, aenv) in enumerate(plan, 1):
        env = dict(base)
        env.update(aenv)
        att = _attempt_local(cmd, nproc, number, transport, env, grace_s, tail_lines, err, timeout_s, t_launch)
        done.append(att)
        if att.result is not None:
            if att.fail_order:
                print(f"[launch] rank(s) {att.fail_order} failed after rank 0 printed its result: the result stands",
                      file=err, flush=True)
            os.write(1 if out_fd is None else out_fd, (annotate(att.result, done) + "\n").encode())
            return 0
        for r in att.fail_order or [0]:
            print(f"[launch] ---- attempt {number}: rank {r} (exit code {att.codes.get(r)}) stderr tail ----",
                  file=err)
            for ln in att.tails.get(r, []):
                print(f"[launch]   {ln.rstrip()}", file=err)
        f = att.failure()
        print(f"[launch] attempt {number} ({transport}) failed {f['phase']}: {f['reason']}", file=err, flush=True)
        if number < len(plan):
            if time.time() - t_launch > budget:
                print(f"[launch] no retry: the launch wall budget ({budget:.0f} s) is spent", file=err, flush=True)
                break
            print(f"[launch] retrying in fresh ranks: attempt {number + 1} ({plan[number][0]})", file=err, flush=True)
    if done and done[-1].result is None:
        print("[launch] rank 0 printed no JSON result line", file=err, flush=True)
    return done[-1].first_code() if done else 1


# ---- per-rank supervisor under an external launcher (torchrun) --------------------------------
#
# Under torchrun the ranks are torchrun's processes, and a dead rank ends the whole job.  Each
# rank process of bench.py therefore becomes a SUPERVISOR that never touches the GPU: it starts the
# real rank as its child and the supervisors run the same attempt plan together.  They coordinate
# through torchrun's agent store (MASTER_ADDR:MASTER_PORT; every supervisor is a client): rank 0's
# supervisor serves a fresh rendezvous store per attempt and publishes its port there, a
# supervisor whose child failed publishes the death notice in the attempt's store (the peers'
# fault watchdogs see it within a beat) and in the agent store (the other supervisors stop their
# children after ``grace_s``), every supervisor reports its child's exit code and stderr tail,
# and rank 0's supervisor decides: done, retry, or give up.


def supervisor_wanted(env: Optional[dict] = None) -> bool:
    """True for a rank process of a torchrun job (agent store) that is not itself a supervised
    child (``DNN_SUPERVISE=0`` turns supervision off)."""
    e = os.environ if env is None else env
    try:
        world = int(e.get("WORLD_SIZE", "1") or 1)
    except ValueError:
        return False
    return (e.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true" and world > 1
            and e.get("DNN_SUPERVISED") != "1" and e.get("DNN_SELF_LAUNCHED") != "1"
            and e.get("DNN_SUPERVISE", "1") != "0")


def _wait_key(store, key: str, deadline: float, poll_s: float = 0.05) -> bool:
    while time.time() < deadline:
        try:
            if store.check([key]):
                return True
        except Exception:
            pass
        time.sleep(poll_s)
    return False


def supervise(cmd: Sequence[str], out_fd: int | None = None, grace_s: float = 60.0, tail_lines: int = 40,
              err: IO[str] | None = None, report_wait_s: float = 120.0) -> int:
    """Run ``cmd`` as this torchrun rank's child under the shared attempt plan (see above).
    Returns this supervisor's exit code (0 once an attempt produced rank 0's result line)."""
    import datetime

    import torch.distributed as dist

    err = err or sys.stderr
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    addr, port = os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"])
    t_launch = time.time()
    agent = dist.TCPStore(addr, port, world, is_master=False, timeout=datetime.timedelta(seconds=600))
    ns = (f"dnn/sup/{os.environ.get('TORCHELASTIC_RUN_ID', 'run')}/"
          f"{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}")
    plan = attempt_plan()
    budget, timeout_s = _budget()
    done: list[_Attempt] = []
    for number, (transport, aenv) in enumerate(plan, 1):
        k = f"{ns}/a{number}"
        srv = None
        if rank == 0:
            aport = _free_port()
            srv = dist.TCPStore("127.0.0.1", aport, world + 1, is_master=True, wait_for_workers=False)
            agent.set(f"{k}/port", str(aport))
        if not _wait_key(agent, f"{k}/port", time.time() + 600):
            print(f"[supervise r{rank}] no attempt-{number} store from rank 0's supervisor", file=err, flush=True)
            return 1
        aport = int(agent.get(f"{k}/port").decode())
        st = srv if srv is not None else dist.TCPStore(addr, aport, world + 1, is_master=False,
                                                       timeout=datetime.timedelta(seconds=600))
        env = hsa_env.strip(dict(os.environ))
        env.update(aenv)
        env.update(MASTER_PORT=str(aport), DNN_STORE_EXTERNAL="1", TORCHELASTIC_USE_AGENT_STORE="False",
                   DNN_SUPERVISED="1", DNN_SELF_LAUNCHED="1", DNN_LAUNCHER_PID=str(os.getpid()),
                   DNN_LAUNCH_ATTEMPT=str(number), PYTHONUNBUFFERED="1")
        t0 = time.time()
        p = subprocess.Popen(list(cmd), env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             bufsize=1, start_new_session=True, stdin=subprocess.DEVNULL)
        c = _Child(rank, p, tail_lines)
        sink = err if number == 1 else _prefixed(rank, err, number)
        c.threads = [threading.Thread(target=_pump, args=(p.stderr, sink, c.keep_err), daemon=True),
                     threading.Thread(target=_pump, args=(p.stdout, None if rank == 0 else sink, c.out.append),
                                      daemon=True)]
        for t in c.threads:
            t.start()
        if rank == 0:
            print(f"[supervise +{time.time() - t_launch:.3f}s] attempt {number} ({transport}): store on port {aport}, "
                  f"{world} ranks", file=err, flush=True)

        def _forward(signum, frame):
            _kill_group(p, signal.SIGTERM)
            time.sleep(2.0)
            _kill_group(p, signal.SIGKILL)
            raise SystemExit(128 + signum)

        prev = {sig: signal.signal(sig, _forward) for sig in (signal.SIGTERM, signal.SIGINT)} \
            if threading.current_thread() is threading.main_thread() else {}
        failed_at: float | None = None
        terminated = timed_out = False
        try:
            while True:
                rc = p.poll()
                if rc is not None:
                    break
                now = time.time()
                grace = grace_s if c.saw_window else _pre_window_grace(grace_s)
                if failed_at is None:
                    try:
                        if agent.add(f"{k}/nfail", 0) > 0:
                            failed_at = now
                    except Exception:
                        failed_at = now  # the agent store is gone: torchrun is tearing the job down
                if timeout_s > 0 and now - t0 > timeout_s and not timed_out:
                    print(f"[supervise r{rank}] attempt {number} still running after its wall limit "
                          f"({timeout_s:.0f} s): terminating", file=err, flush=True)
                    timed_out = True
                    agent.add(f"{k}/nfail", 1)
                    failed_at = now - grace
                if failed_at is not None and now - failed_at > grace and not terminated:
                    _kill_group(p, signal.SIGTERM)
                    terminated = True
                if failed_at is not None and now - failed_at > grace + 10:
                    _kill_group(p, signal.SIGKILL)
                time.sleep(0.05)
        finally:
            for sig, h in prev.items():
                signal.signal(sig, h)
        if rc != 0:
            try:
                st.set(f"dnn/dead/{rank}", repr(time.time()))
            except Exception:
                pass
            agent.add(f"{k}/nfail", 1)
            print(f"[supervise r{rank} +{time.time() - t_launch:.3f}s] rank {rank} exited with code {rc}", file=err,
                  flush=True)
        for t in c.threads:
            t.join(timeout=5.0)
        agent.set(f"{k}/rc/{rank}", json.dumps({"rc": rc, "t": time.time(), "saw": c.saw_window,
                                                 "timed_out": timed_out, "tail": list(c.err_tail)[-12:]}))
        if rank == 0:
            att = _Attempt(number, transport)
            att.result = c.result()
            att.wall_s = time.time() - t0
            reports = {}
            for r in range(world):
                if _wait_key(agent, f"{k}/rc/{r}", time.time() + report_wait_s):
                    reports[r] = json.loads(agent.get(f"{k}/rc/{r}").decode())
            for r in range(world):
                rep = reports.get(r, {"rc": None, "t": float("inf"), "saw": False, "timed_out": False,
                                      "tail": ["(no report from this rank's supervisor)"]})
                att.codes[r] = rep["rc"]
                att.tails[r] = rep["tail"]
                att.saw_window = att.saw_window or bool(rep["saw"])
                att.timed_out = att.timed_out or bool(rep["timed_out"])
            att.fail_order = sorted((r for r in range(world) if att.codes[r] != 0),
                                    key=lambda r: reports.get(r, {}).get("t", float("inf")))
            done.append(att)
            if att.result is not None:
                decision = "done"
            elif number < len(plan) and time.time() - t_launch <= budget:
                decision = "retry"
            else:
                decision = "fail"
            if att.result is None:
                f = att.failure()
                print(f"[supervise] attempt {number} ({transport}) failed {f['phase']}: {f['reason']}", file=err)
                for ln in f["stderr_tail"]:
                    print(f"[supervise]   {ln}", file=err)
                if decision == "retry":
                    print(f"[supervise] retrying in fresh ranks: attempt {number + 1} ({plan[number][0]})", file=err,
                          flush=True)
            agent.set(f"{k}/decision", decision)
        else:
            if not _wait_key(agent, f"{k}/decision", time.time() + report_wait_s + 600):
                return rc or 1
            decision = agent.get(f"{k}/decision").decode()
        del st, srv
        if decision == "done":
            if rank == 0:
                os.write(1 if out_fd is None else out_fd, (annotate(done[-1].result, done) + "\n").encode())
            return 0
        if decision == "fail":
            return (done[-1].first_code() if rank == 0 else rc) or 1
    return 1


def _kill_group(p: subprocess.Popen, sig: int) -> None:
    try:
        os.killpg(p.pid, sig)  # the child runs in its own session: its pid is its group id
    except Exception:
        try:
            p.send_signal(sig)
        except Exception:
            pass


__all__ = ["ATTEMPTS", "WINDOW_MARK", "annotate", "attempt_plan", "die_with_parent", "launcher_present", "run",
           "supervise", "supervisor_wanted", "visible_devices"]
