"""Diagnostic: 2 ranks on one GPU, early-MLP in-launch vs serial one-launch exchange - where do
the parameters differ (per tensor of the arena), and are the replicas identical?"""
import os
import sys
import tempfile
import pathlib

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_xgmi_gpu as T  # noqa: E402
import torch  # noqa: E402
from distributed_neural_network_amd.models.network import LAYOUT  # noqa: E402

tmp = pathlib.Path(tempfile.mkdtemp())
ref, _ = T._two_ranks(tmp, "xgmi", "1", 29701, exchange="pull")
for graphs, port in (("1", 29703), ("0", 29705)):
    res, r = T._two_ranks(tmp, "xgmi", graphs, port, exchange="pull", early="1")
    print("graphs", graphs, "replicas equal:", torch.equal(res[0]["master"], res[1]["master"]))
    for i in range(2):
        d = (res[i]["master"] - ref[i]["master"]).abs()
        parts = {k: float(d[o:o + n].max()) for k, (o, n) in
                 ((k, (LAYOUT.offsets[k], int(torch.Size(LAYOUT.shapes[k]).numel()))) for k in LAYOUT.offsets) if n}
        print("  rank", i, "max diff", float(d.max()), {k: v for k, v in parts.items() if v})
    print(r.stderr[-1500:])
