"""A timed-out in-launch wait degrades the step instead of killing the job.

The persistent step's reduction and sample workgroups wait on each other with bounded waits; a
wait past its bound sets a sticky error word and the launch drains.  The trainer then restores
the epoch's snapshot, steps the engine down (persistent -> pipelined -> serial, each bit-identical
to the next) and redoes the epoch.  Here a timeout is FORCED: a tiny wait bound
(DNN_PIPE_TIMEOUT_S) plus an injected delay of sample workgroup 0 in step 1 of a persistent
launch (DNN_PIPE_FLAGS=256, lenet_fused.hip pers_arrive_kind).  The run must finish and its
parameters must equal a run on the serial step bit for bit.
"""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _train(tmp_path, name, env_extra, dtype="bf16"):
    d = tmp_path / name
    d.mkdir()
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "2",
                        "--batch-size", "64", "--train-samples", "1024", "--test-samples", "256", "--lr", "0.01",
                        "--seed", "3", "--save", "ck.pt", "--device", "cuda", "--dtype", dtype], cwd=d, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return torch.load(d / "ck.pt", weights_only=True), r


@pytest.mark.parametrize("dtype,level", [("bf16", "pipelined"), ("fp32", "serial")])
def test_forced_persistent_timeout_steps_down_and_matches_serial(tmp_path, dtype, level):
    # (fp32: lenet_f32.hip's persistent launch, same injected delay; it steps down to the serial step)
    forced = {"DNN_PIPE_FLAGS": "256", "DNN_PIPE_TIMEOUT_S": "0.002", "DNN_PERSIST_F32": "1"}  # (fp32's is opt-in)
    sd, r = _train(tmp_path, "forced", forced, dtype)
    assert f"stepping down to the {level} step" in r.stdout, r.stdout[-3000:]
    assert r.stdout.count("Validation loss of updated master model:") == 2
    ref, _ = _train(tmp_path, "serial", {"DNN_PERSIST": "0", "DNN_PIPELINE": "0"}, dtype)
    for k in ref:
        assert torch.equal(sd[k], ref[k]), k
