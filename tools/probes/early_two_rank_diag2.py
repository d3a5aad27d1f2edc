"""Diagnostic: the 2-rank test worker (tests/test_xgmi_gpu.py _TWO_RANK), early-MLP vs serial,
with cwd = tmp (as the test) and cwd = repo root."""
import os
import pathlib
import subprocess
import sys
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import test_xgmi_gpu as T  # noqa: E402

tmp = pathlib.Path(tempfile.mkdtemp())
(tmp / "w.py").write_text(T._TWO_RANK)
res = {}
port = 29721
for early in ("0", "1"):
    for cwd in ("tmp", "root"):
        out = tmp / f"{early}{cwd}"
        out.mkdir()
        env = dict(os.environ, PYTHONPATH=ROOT, DNN_BACKEND="gloo", DNN_ALLREDUCE="xgmi", OMP_NUM_THREADS="2",
                   OUT=str(out), GRAPHS="1", DNN_XGMI_ONE_LAUNCH="1", DNN_XGMI_EXCHANGE="pull", ENGINE="fused",
                   DNN_EARLY_MLP=early)
        r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                            "--master-addr", "127.0.0.1", "--master-port", str(port), str(tmp / "w.py")],
                           cwd=tmp if cwd == "tmp" else ROOT, env=env, capture_output=True, text=True, timeout=300)
        port += 2
        if r.returncode:
            print(r.stderr[-3000:])
            sys.exit(1)
        res[early + cwd] = [torch.load(out / f"r{i}.pt", weights_only=True)["master"] for i in range(2)]
for k, v in res.items():
    print(k, "vs 0tmp:", [float((v[i] - res["0tmp"][i]).abs().max()) for i in range(2)])
