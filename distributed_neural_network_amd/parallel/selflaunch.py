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
  job forever.
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


def _pump(stream: IO[str], sink, keep) -> None:
    for line in stream:
        keep(line)
        if sink is not None:
            try:
                sink.write(line)
                sink.flush()
            except Exception:
                pass


def _prefixed(rank: int, out: IO[str]):
    class _W:
        def write(self, s: str) -> None:
            out.write(f"[r{rank}] {s}" if s.strip() else s)

        def flush(self) -> None:
            out.flush()

    return _W()


def run(cmd: Sequence[str], nproc: int, out_fd: int | None = None, extra_env: Optional[dict] = None,
        grace_s: float = 60.0, tail_lines: int = 40, err: IO[str] | None = None) -> int:
    """Run ``cmd`` as ``nproc`` ranks of one job (see the module docstring); returns the exit code.
    ``out_fd``: where rank 0's JSON line goes (default: fd 1)."""
    import torch.distributed as dist

    err = err or sys.stderr
    port = _free_port()
    t0 = time.time()
    store = dist.TCPStore("127.0.0.1", port, nproc + 1, is_master=True, wait_for_workers=False)
    base = dict(os.environ)
    base.update(extra_env or {})
    ndev = visible_devices()
    print(f"[launch] {ndev} GPU(s) visible to this job (KFD topology + visibility variables)", file=err, flush=True)
    if nproc > max(ndev, 1) and not base.get("DNN_BACKEND"):
        base["DNN_BACKEND"] = "gloo"
        print(f"[launch] {nproc} ranks on {ndev} visible GPU(s): ranks share devices, host collectives over gloo",
              file=err, flush=True)
    children: list[_Child] = []
    for r in range(nproc):
        env = dict(base)
        env.update(RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(nproc),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DNN_STORE_EXTERNAL="1",
                   DNN_SELF_LAUNCHED="1", DNN_LAUNCHER_PID=str(os.getpid()), PYTHONUNBUFFERED="1")
        p = subprocess.Popen(list(cmd), env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             bufsize=1, start_new_session=True, stdin=subprocess.DEVNULL)
        children.append(_Child(r, p, tail_lines))
    # the relay threads start only once every child exists (no child is spawned while they run)
    for c in children:
        r, p = c.rank, c.proc
        c.threads = [threading.Thread(target=_pump, args=(p.stderr, _prefixed(r, err), c.err_tail.append), daemon=True),
                     threading.Thread(target=_pump, args=(p.stdout, None if r == 0 else _prefixed(r, err),
                                                          c.out.append), daemon=True)]
        for t in c.threads:
            t.start()
    print(f"[launch +{time.time() - t0:.3f}s] store on 127.0.0.1:{port}, {nproc} ranks started", file=err, flush=True)

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
    fail_order: list[int] = []  # ranks in the order they failed: the first is the root cause
    first_fail: float | None = None
    killed: set[int] = set()
    while len(codes) < nproc:
        for c in children:
            if c.rank in codes:
                continue
            rc = c.proc.poll()
            if rc is None:
                continue
            codes[c.rank] = rc
            if rc != 0:
                fail_order.append(c.rank)
                try:
                    store.set(f"dnn/dead/{c.rank}", repr(time.time()))
                except Exception:
                    pass
                print(f"[launch +{time.time() - t0:.3f}s] rank {c.rank} exited with code {rc}", file=err, flush=True)
                if first_fail is None:
                    first_fail = time.time()
        if first_fail is not None and time.time() - first_fail > grace_s:
            for c in children:
                if c.rank not in codes and c.rank not in killed:
                    print(f"[launch] rank {c.rank} still running {grace_s:.0f} s after a failure: terminating it",
                          file=err, flush=True)
                    _kill_group(c.proc, signal.SIGTERM)
                    killed.add(c.rank)
            if time.time() - first_fail > grace_s + 10:
                for c in children:
                    if c.rank not in codes:
                        _kill_group(c.proc, signal.SIGKILL)
        time.sleep(0.02)
    for sig, h in prev.items():
        signal.signal(sig, h)
    for c in children:
        for t in c.threads:
            t.join(timeout=5.0)
    del store

    result = None
    for line in children[0].out:
        s = line.strip()
        if s.startswith("{"):
            try:
                json.loads(s)
                result = s
            except ValueError:
                pass
    bad = [children[r] for r in fail_order]
    if bad or result is None:
        for c in bad or children[:1]:
            print(f"[launch] ---- rank {c.rank} (exit code {codes[c.rank]}) stderr tail ----", file=err)
            for ln in c.err_tail:
                print(f"[launch]   {ln.rstrip()}", file=err)
        if result is None:
            print("[launch] rank 0 printed no JSON result line", file=err, flush=True)
        return next((codes[c.rank] for c in bad), 1) or 1
    os.write(1 if out_fd is None else out_fd, (result + "\n").encode())
    return 0


def _kill_group(p: subprocess.Popen, sig: int) -> None:
    try:
        os.killpg(p.pid, sig)  # the child runs in its own session: its pid is its group id
    except Exception:
        try:
            p.send_signal(sig)
        except Exception:
            pass


__all__ = ["die_with_parent", "launcher_present", "run", "visible_devices"]
