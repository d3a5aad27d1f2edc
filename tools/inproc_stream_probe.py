#!/usr/bin/env python3
"""Diagnostic: does the in-process two-engine exchange harness (tests/test_inproc_pair_gpu.py)
depend on how many HIP streams the process created before it?  PyTorch hands out pool streams
round-robin and HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES), so the
streams created earlier decide whether the two ranks' streams share a hardware queue.

    python tools/inproc_stream_probe.py [--dtype fp32] [--graphs 0] [--max-skip 7]

For each k in 0..max-skip a fresh process creates k pool streams first and then runs the
harness check; one JSON line: {k: "ok" | first line of the failure}.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = """
import sys, torch
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
keep = [torch.cuda.Stream() for _ in range({k})]
import test_inproc_pair_gpu as t
t._check({dtype!r}, {graphs})
print("ok")
"""


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--graphs", type=int, default=0)
    ap.add_argument("--max-skip", type=int, default=7)
    ap.add_argument("--min-skip", type=int, default=0)
    a = ap.parse_args()
    out = {}
    for k in range(a.min_skip, a.max_skip + 1):
        code = CHILD.format(root=ROOT, tests=os.path.join(ROOT, "tests"), k=k, dtype=a.dtype, graphs=bool(a.graphs))
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                           env=dict(os.environ, PYTHONPATH=ROOT))
        if r.returncode == 0:
            out[k] = "ok"
        else:
            err = [ln for ln in r.stderr.splitlines() if "Error" in ln or "assert" in ln]
            out[k] = (err[-1] if err else r.stderr.strip().splitlines()[-1:])[:300] if r.stderr else f"rc {r.returncode}"
            if "detail" not in out:
                out["detail"] = {"k": k, "stdout": r.stdout[-4000:], "stderr": r.stderr[-6000:]}
        print(f"[probe] skip {k}: {out[k]}", file=sys.stderr, flush=True)
    print(json.dumps({"dtype": a.dtype, "graphs": a.graphs, "results": out}))


if __name__ == "__main__":
    main()
