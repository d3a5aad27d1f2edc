"""Stand-alone rendezvous store for launches without an agent (mpiexec, a plain env launch).

Under ``torchrun`` the agent serves the TCPStore and under ``parallel/launch.py`` the launcher
does, so any rank may die and the survivors still rendezvous.  Under ``mpiexec -n N``
(the reference launcher, README.md:28) nobody does: if rank 0 hosted the store, its death would
take the store - and with it every survivor's recovery - down.  Rank 0 therefore starts THIS
small process first (a child in its own session, so a signal to rank 0's process group does
not reach it), every rank including rank 0 connects as a client, and the store outlives any
single rank.

It exits when every rank of the job has checked out (``dnn/closed`` counter, incremented by
``Communicator.close``; a rank the recovery dropped counts through ``dnn/dropped``), when every
heartbeat it has seen is older than ``--stale`` seconds (the ranks are gone without checking
out: a crash, Ctrl-C, SIGKILL), when every rank process registered on this host
(``dnn/pid/<r>`` = host:pid, written by every rank at connect) is gone and no rank of another
host is registered (those may still need the store to recover), or when nothing at all
has changed for ``--idle`` seconds - the idle exit only while no registered rank of this host
is alive: a live job that makes no store writes for a while (a bench without a heartbeat) keeps
its store.  It
publishes ``dnn/store_server`` = ``--token`` (rank 0's job token), so rank 0 can tell its own
server from one an earlier job left on the port (Communicator._check_fresh_store).

usage (started by Communicator; not by hand):
    python -m distributed_neural_network_amd.parallel.store_server --port P --world N
"""
from __future__ import annotations

import argparse
import os
import socket
import sys
import time


def _pid_alive(pid: int) -> bool:
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
        return True


def decide(world: int, closed: int, dropped: int, beats: list, stale: float, pids: dict, alive: list,
           idle_for: float, idle: float, now: float) -> str | None:
    """Why the server should exit now (None: keep serving).  ``beats``: each rank's last heartbeat
    stamp (None: none seen); ``pids``: registered ranks -> pid on this host (-1: another host);
    ``alive``: the registered local pids still running; ``idle_for``: seconds since anything in
    the store last changed."""
    if closed + dropped >= world:
        return "every rank checked out"
    seen = [t for t in beats if t is not None]
    if seen and now - max(seen) > stale:
        return f"no heartbeat for {stale:.0f} s: the job is gone"
    local = [p for p in pids.values() if p > 0]
    # ranks on other hosts (pid -1) may outlive every rank of this one - and need the store for
    # their recovery (agree_survivors, reform): with any of them registered, only the check-out
    # and heartbeat-staleness rules above apply
    remote = any(p <= 0 for p in pids.values())
    if local and not alive and len(pids) == world and not remote:
        return "every rank process of this host is gone"
    if idle_for > idle and not alive and not remote:
        return f"no activity for {idle:.0f} s"
    return None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--idle", type=float, default=300.0)
    ap.add_argument("--stale", type=float, default=30.0)
    ap.add_argument("--token", default="up")
    a = ap.parse_args(argv)

    import torch.distributed as dist

    store = dist.TCPStore(a.host, a.port, a.world + 1, is_master=True, wait_for_workers=False,
                          timeout=__import__("datetime").timedelta(seconds=30))
    store.set("dnn/store_server", a.token)
    last_change, last_sig = time.time(), None
    host = socket.gethostname()
    pids: dict[int, int] = {}  # registered ranks of this host
    while True:
        time.sleep(0.2)
        try:
            closed = store.add("dnn/closed", 0)
            dropped = store.add("dnn/dropped", 0)
            beats = []
            for r in range(a.world):
                k = f"dnn/hb/{r}"
                beats.append(store.get(k) if store.check([k]) else b"")
            sig = (closed, dropped, store.num_keys(), tuple(beats))
        except Exception:
            return 1
        stamps = []
        for v in beats:
            try:
                stamps.append(float(v.decode()) if v else None)
            except ValueError:
                stamps.append(None)
        for r in range(a.world):
            if r not in pids:
                try:
                    k = f"dnn/pid/{r}"
                    if store.check([k]):
                        h, _, p = store.get(k).decode().rpartition(":")
                        pids[r] = int(p) if h == host else -1
                except Exception:
                    pass
        alive = [p for p in pids.values() if p > 0 and _pid_alive(p)]
        if sig != last_sig:
            last_sig, last_change = sig, time.time()
        why = decide(a.world, closed, dropped, stamps, a.stale, pids, alive, time.time() - last_change, a.idle,
                     time.time())
        if why is not None:
            if closed + dropped >= a.world:
                time.sleep(1.0)  # let the last clients finish their final reads
            else:
                print(f"[store] {why}: exiting", file=sys.stderr, flush=True)
            return 0


if __name__ == "__main__":
    sys.exit(main())
