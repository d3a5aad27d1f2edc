"""Multi-process launcher: one process per GPU (or per CPU rank for gloo).

Capability parity: ``mpiexec -n N python data_parallelism_train.py --nb-proc N``
(README.md:28, run_training.sh:3).  Usage::

    python -m distributed_neural_network_amd.parallel.launch -n 4 data_parallelism_train.py --batch-size 64

The launcher hosts the rendezvous TCPStore itself (like torchrun's agent), so any
rank - rank 0 included - may die and the survivors can still re-form.  Unlike
torchrun it does NOT tear the job down when one rank exits: a rank that exits with
the injected-drop code is reported as dropped and the rest keep running.  The moment a
rank's process exits with a failure code the launcher publishes ``dnn/dead/<rank>`` in the
store, which the survivors' fault watchdogs read within one beat period (~0.1 s) - far
sooner than a heartbeat going stale.
``torchrun`` and ``mpiexec`` launches work too (parallel/env.py reads their env).
"""
from __future__ import annotations

import argparse
import os
import socket
import subprocess
import sys
import time

from .fault import DROP_EXIT_CODE


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-n", "--nproc", type=int, required=True)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("--cpu", action="store_true", help="hide GPUs from the ranks (gloo backend)")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)

    import torch.distributed as dist

    port = a.master_port or _free_port()
    store = dist.TCPStore(a.master_addr, port, a.nproc + 1, is_master=True, wait_for_workers=False)
    procs = []
    for r in range(a.nproc):
        env = dict(os.environ)
        env.update(RANK=str(r), WORLD_SIZE=str(a.nproc), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(a.nproc),
                   MASTER_ADDR=a.master_addr, MASTER_PORT=str(port), DNN_STORE_EXTERNAL="1")
        if a.cpu:
            env["CUDA_VISIBLE_DEVICES"] = ""
            env["HIP_VISIBLE_DEVICES"] = ""
        procs.append(subprocess.Popen([sys.executable, a.script] + a.args, env=env))
    codes: dict[int, int] = {}
    while len(codes) < len(procs):
        for r, p in enumerate(procs):
            if r not in codes and p.poll() is not None:
                codes[r] = p.returncode
                if p.returncode != 0:
                    try:
                        store.set(f"dnn/dead/{r}", repr(time.time()))
                    except Exception:
                        pass
                if p.returncode == DROP_EXIT_CODE:
                    print(f"[launch] rank {r} dropped (injected failure)", flush=True)
                elif p.returncode != 0:
                    print(f"[launch] rank {r} exited with code {p.returncode}", flush=True)
        time.sleep(0.02)
    del store
    bad = [c for c in codes.values() if c not in (0, DROP_EXIT_CODE)]
    return bad[0] if bad else 0


if __name__ == "__main__":
    sys.exit(main())
