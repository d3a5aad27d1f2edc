#!/usr/bin/env python3
"""Per-dispatch table of a rocprofv3 kernel trace, grouped by (kernel, grid): median duration
and calls per step.  The layer engine launches one kernel per layer op, so the grid size
tells the layers apart.   usage: python tools/layer_dispatch_table.py OUT/run_results.db STEPS"""
import sqlite3
import sys
from collections import defaultdict

import numpy as np

db = sqlite3.connect(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = db.execute("select name, grid_x, grid_y, grid_z, workgroup_x, lds_size, duration from kernels").fetchall()
g = defaultdict(list)
for name, gx, gy, gz, wx, lds, dur in rows:
    short = name.replace("dnn::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
    g[(short, gx // max(wx, 1), gy, gz, lds)].append(dur / 1000.0)
tot = sum(sum(v) for v in g.values())
print(f"{'kernel':60s} {'grid':>16s} {'lds':>6s} {'calls/step':>10s} {'med_us':>8s} {'us/step':>8s}")
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    cps = len(v) / steps
    if cps < 0.5:
        continue
    print(f"{k[0]:60s} {f'{k[1]}x{k[2]}x{k[3]}':>16s} {k[4]:6d} {cps:10.1f} {np.median(v):8.2f} {sum(v) / steps:8.2f}")
print(f"total GPU time per step: {tot / steps:.1f} us")
