"""Multi-process (gloo, CPU) correctness of the sync policies, the CLI and fault recovery.

Every policy is checked against a single-process computation of the same math:
  * step-allreduce, 2 ranks x batch b  == 1 process x batch 2b (gradient of the mean)
  * epoch-avg                          == arithmetic mean of the locally trained models
                                          (reference data_parallelism_train.py:238-240)
  * parent                             == mean over workers 1..N-1 only
"""
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import torch

from distributed_neural_network_amd.data import EpochSampler, synthetic
from distributed_neural_network_amd.models.network import LAYOUT, init_arena
from distributed_neural_network_amd.runtime import CpuEngine
from distributed_neural_network_amd.utils import checkpoint, logfiles

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(n, args, cwd, timeout=240):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "distributed_neural_network_amd.parallel.launch", "-n", str(n), "--cpu"] + args
    return subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)


def _launch_env(n, args, cwd, env_extra, timeout=300):
    """Run a launched job; on a timeout, kill it and fail WITH its output so far (every rank dumps
    its thread stacks every 30 s: DNN_FAULTHANDLER_S) - a hang must name where it sits."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", **env_extra)
    env.setdefault("DNN_FAULTHANDLER_S", "30")
    cmd = [sys.executable, "-m", "distributed_neural_network_amd.parallel.launch", "-n", str(n), "--cpu"] + args
    p = subprocess.Popen(cmd, cwd=cwd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        import signal
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        raise AssertionError(f"job timed out after {timeout} s\n--- stdout ---\n{out[-6000:]}\n--- stderr ---\n"
                             f"{err[-12000:]}")
    return subprocess.CompletedProcess(cmd, p.returncode, out, err)


def _run_worker(tmp_path, mode, world, n=192, batch=16, epochs=2):
    r = _launch(world, [os.path.join(ROOT, "tests", "dist_worker.py"), mode, str(tmp_path), str(n), str(batch),
                        str(epochs)], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    return [torch.load(tmp_path / f"rank{i}.pt", weights_only=True)["master"] for i in range(world)]


def _local(arena, data, idx, batch, epochs_orders, lr=0.05, momentum=0.9, reset=False):
    eng = CpuEngine(batch=batch, lr=lr, momentum=momentum, arena=arena)
    eng.attach(data)
    for order in epochs_orders:
        if reset:
            eng.reset_momentum()
        eng.begin_epoch(order)
        eng.run_steps((len(order) + batch - 1) // batch)
    return eng


@pytest.mark.parametrize("world,per_rank", [(2, 48), (4, 48), (8, 48), (4, 40)])
def test_step_allreduce_equals_big_batch(tmp_path, world, per_rank):
    n = per_rank * world  # 48: 3 full batches of 16 per rank; 40: 2 full + a tail of 8
    got = _run_worker(tmp_path, "step-allreduce", world, n=n, batch=16, epochs=1)
    for r in range(1, world):
        assert torch.allclose(got[0], got[r], atol=0, rtol=0)  # replicas stay bitwise identical
    data = synthetic(n, 3)
    # single process, batch 16 * world: step t takes shard_r[16t:16t+16] of every rank r (the
    # tail step: the tails of every rank - the mean of per-rank means of equal tails)
    shard = n // world
    order = np.concatenate([np.concatenate([shard * r + np.arange(16 * t, min(16 * t + 16, shard))
                                            for r in range(world)])
                            for t in range((shard + 15) // 16)]).astype(np.int32)
    ref = _local(init_arena(seed=100), data, None, 16 * world, [order])
    assert torch.allclose(got[0], ref.master, atol=2e-6), float((got[0] - ref.master).abs().max())


def test_epoch_average_equals_mean_of_local_models(tmp_path):
    got = _run_worker(tmp_path, "epoch-avg", 2, n=192, batch=16, epochs=2)
    assert torch.equal(got[0], got[1])
    data = synthetic(192, 3)
    a = init_arena(seed=100)
    for ep in range(2):
        ms = []
        for r in range(2):
            e = _local(a, data, None, 16, [np.arange(96 * r, 96 * r + 96, dtype=np.int32)], reset=True)
            ms.append(e.master)
        a = (ms[0] + ms[1]) / 2
    assert torch.allclose(got[0], a, atol=1e-6)


def test_parent_topology_averages_workers_only(tmp_path):
    got = _run_worker(tmp_path, "parent", 3, n=192, batch=16, epochs=1)
    assert torch.allclose(got[0], got[1]) and torch.allclose(got[1], got[2])
    data = synthetic(192, 3)
    a = init_arena(seed=100)
    ms = [_local(a, data, None, 16, [np.arange(96 * r, 96 * r + 96, dtype=np.int32)], reset=True).master
          for r in range(2)]
    assert torch.allclose(got[0], (ms[0] + ms[1]) / 2, atol=1e-6)


SMALL = ["--train-samples", "384", "--test-samples", "128", "--lr", "0.01", "--device", "cpu"]


def test_cli_data_parallel_stdout_and_logs(tmp_path):
    r = _launch(3, [os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "2", "--batch-size", "32",
                    "--nb-proc", "3", "--compat", "--metrics", "m.jsonl"] + SMALL, tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    assert out.count("Starting epoch  ") == 2
    assert "(Received a trained model from process 3 of 3 workers...)" in out
    assert "* Averaging models..." in out and "evaluating model" in out
    assert re.search(r"Global Average Training Loss: [0-9.]+", out)
    assert re.search(r"Validation loss of updated master model:  [0-9.]+", out)
    assert "(Loaded Train Dataset for worker 2 of length 128)" in out
    par = logfiles.read_log(str(tmp_path / "log" / "bs32_log_epochs2_proc3_parent.txt"))
    chi = logfiles.read_log(str(tmp_path / "log" / "bs32_log_epochs2_proc3_children.txt"))
    assert set(par) == {"Eval data loading time", "Time spent on evaluation",
                        "Time spent on parent communication and param sync"}
    assert set(chi) == {"Train data loading time", "Time spent on training", "Time spent on children communication"}
    assert (tmp_path / "m.jsonl").exists()


def test_cli_single_and_replication(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "single_proc_train.py"), "--epochs", "2"] + SMALL,
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "cpu" and lines[1] == "384" and lines[2] == "128"
    assert re.match(r"Epoch 1, Average Training Loss: \d+\.\d{3}$", lines[3])
    assert re.match(r"Validation Accuracy: \d+\.\d{2} %$", lines[4])
    assert re.match(r"Validation Loss: \d+\.\d{3}$", lines[5])
    r = _launch(2, [os.path.join(ROOT, "model_replication_train.py"), "--epochs", "1", "--batch-size", "64"] + SMALL,
                tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "(Loaded Train Dataset for worker 1 of length 384)" in r.stdout  # full set on every worker


def test_typed_cli_overrides_work():
    from distributed_neural_network_amd.train import parse
    c = parse("data-parallel", ["--lr", "0.05", "--momentum", "0.5", "--batch-size", "8", "--epochs", "3",
                                "--failure-probability", "0.25", "--failure-duration", "0.1"])
    assert (c.lr, c.momentum, c.batch_size, c.epochs) == (0.05, 0.5, 8, 3)
    assert c.failure_probability == 0.25 and c.nb_proc == 4
    d = parse("replication", [])
    assert (d.batch_size, d.epochs, d.sync) == (16, 10, "epoch-avg")
    s = parse("single", [])
    assert (s.batch_size, s.epochs) == (4, 15)


def test_debug_sync_flag(monkeypatch):
    """--debug-sync: serialised launches via the HIP environment (set before the runtime starts),
    eager steps, RCCL debug output and the cross-rank checksum after every sync."""
    from distributed_neural_network_amd.train import parse
    from distributed_neural_network_amd.train.config import DEBUG_SYNC_ENV
    env = {k: v for k, v in os.environ.items() if k not in DEBUG_SYNC_ENV}
    monkeypatch.setattr(os, "environ", env)  # restored after the test
    c = parse("single", ["--debug-sync"])
    assert c.check_sync and not c.use_graphs
    for k, v in DEBUG_SYNC_ENV.items():
        assert os.environ[k] == v
    assert parse("single", []).use_graphs


def test_straggler_prints(capsys):
    from distributed_neural_network_amd.parallel.fault import simulate_failure
    rng = np.random.default_rng(0)
    assert simulate_failure(3, 1.0, 0.01, rng)
    out = capsys.readouterr().out
    assert "Process 3 failed! Sleeping for 0.01 seconds." in out and "Process 3 woke up!" in out
    assert not simulate_failure(3, 0.0, 1.0, rng)


@pytest.mark.parametrize("sync", ["step-allreduce", "epoch-avg"])
def test_rank_drop_reforms_and_finishes(tmp_path, sync):
    r = _launch(3, [os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "3", "--batch-size", "32",
                    "--sync", sync, "--drop-rank", "1", "--drop-at-epoch", "1", "--drop-at-step", "2",
                    "--save", "ck.pt", "--nb-proc", "3"] + SMALL, tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "rank 1 dropped (injected failure)" in r.stdout
    m = re.search(r"\[fault\] rank\(s\) \[1\] dropped in epoch 1; communicator re-formed \(generation 1, 2 ranks\)",
                  r.stdout)
    assert m, r.stdout
    assert r.stdout.count("Validation loss of updated master model:") == 3
    assert "[fault] post-recovery epoch 1:" in r.stdout
    sd, side = checkpoint.load(str(tmp_path / "ck.pt"))
    assert side["epoch"] == 2 and side["world"] == 2


def test_failure_during_recovery_recovers_again(tmp_path):
    """A CommError INSIDE a recovery (DNN_INJECT_RECOVERY_FAIL: rank 0 fails once right after it
    re-formed generation 1, before the new group's barrier) starts the recovery over - rank 2's
    barrier fails with it and both agree again - instead of escaping the recovery scope: the run
    finishes on the two survivors."""
    r = _launch_env(3, [os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "3", "--batch-size", "32",
                        "--sync", "step-allreduce", "--drop-rank", "1", "--drop-at-epoch", "1", "--drop-at-step", "2",
                        "--save", "ck.pt", "--nb-proc", "3"] + SMALL, tmp_path, {"DNN_INJECT_RECOVERY_FAIL": "0:1"})
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "recovery interrupted (injected recovery failure (generation 1))" in r.stdout, r.stdout[-4000:]
    assert r.stdout.count("Validation loss of updated master model:") == 3
    sd, side = checkpoint.load(str(tmp_path / "ck.pt"))
    assert side["epoch"] == 2 and side["world"] == 2


def test_survivor_agreement_counts_early_announcements():
    """A survivor that announced itself before tearing its group down (announce_alive) is in
    the next generation even if it has not reached agree_survivors yet; a stale rank is not."""
    import time
    from types import SimpleNamespace

    import torch.distributed as dist

    from distributed_neural_network_amd.parallel.fault import agree_survivors, announce_alive

    store = dist.TCPStore("127.0.0.1", 0, 1, is_master=True, wait_for_workers=False)
    mk = lambda r: SimpleNamespace(store=store, generation=3, orig_rank=r, members=[0, 1, 2])
    hb = SimpleNamespace(stale=lambda r: r == 2, reported_dead=lambda r: r == 2, timeout=1.0)
    announce_alive(mk(1))  # rank 1 is still blocked in its group teardown
    t0 = time.time()
    assert agree_survivors(mk(0), hb, wait_s=5.0) == [0, 1]
    assert time.time() - t0 < 2.0  # nobody undecided: no waiting for the deadline
    assert agree_survivors(mk(1), hb, wait_s=5.0) == [0, 1]  # the late survivor reads the same list


def test_live_rank_with_stale_heartbeat_is_retried_not_dropped(tmp_path):
    """A live rank whose heartbeat stops for longer than the timeout (DNN_INJECT_BEAT_PAUSE) is
    flagged by its peers; the recovery agreement keeps it (it announces itself within the
    grace), the flag is cleared, and the run finishes after ONE all-alive retry - no exclusion,
    no endless retries (the flag used to stay set forever)."""
    env_extra = {"DNN_INJECT_BEAT_PAUSE": "2:1:1.6", "DNN_HEARTBEAT_TIMEOUT": "1.0"}
    r = _launch_env(3, [os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "12", "--batch-size", "32",
                        "--sync", "step-allreduce", "--nb-proc", "3", "--train-samples", "3072", "--test-samples",
                        "128", "--lr", "0.01", "--device", "cpu"], tmp_path, env_extra)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "injected heartbeat pause: rank 2" in r.stdout
    assert r.stdout.count("with every rank alive; communicator re-created") == 1, r.stdout
    assert "dropped in epoch" not in r.stdout
    assert r.stdout.count("Validation loss of updated master model:") == 12


def test_straggler_longer_than_heartbeat_timeout_is_not_excluded(tmp_path):
    """Reference straggler injection (--failure-probability / --failure-duration) sleeps the
    MAIN thread longer than the 1 s heartbeat timeout: the beat thread keeps beating, so nobody
    is flagged, nothing is re-formed, every epoch completes."""
    r = _launch_env(3, [os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "2", "--batch-size", "32",
                        "--nb-proc", "3", "--failure-probability", "1.0", "--failure-duration", "1.5"] + SMALL,
                    tmp_path, {"DNN_HEARTBEAT_TIMEOUT": "1.0"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("failed! Sleeping for 1.5 seconds.") == 6
    assert "[fault]" not in r.stdout, r.stdout
    assert r.stdout.count("Validation loss of updated master model:") == 2


def test_rank0_drop_under_env_launch(tmp_path):
    """mpiexec-style launch (RANK / WORLD_SIZE / MASTER_* only, no launcher-hosted store): rank 0
    starts the stand-alone store process, so when rank 0 itself dies the survivors still agree,
    re-form and finish (the new rank 0 prints the parent lines)."""
    import socket

    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    procs = []
    for rank in range(3):
        env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", RANK=str(rank), WORLD_SIZE="3",
                   LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="",
                   HIP_VISIBLE_DEVICES="")
        for k in ("DNN_STORE_EXTERNAL", "TORCHELASTIC_USE_AGENT_STORE", "LOCAL_WORLD_SIZE"):
            env.pop(k, None)
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "3", "--batch-size", "32",
             "--sync", "step-allreduce", "--drop-rank", "0", "--drop-at-epoch", "1", "--drop-at-step", "2",
             "--nb-proc", "3"] + SMALL, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
            text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    codes = [p.returncode for p in procs]
    assert codes[0] == 17 and codes[1] == 0 and codes[2] == 0, (codes, outs)
    out1 = outs[1][0]
    assert "[fault] rank(s) [0] dropped in epoch 1; communicator re-formed (generation 1, 2 ranks)" in out1, outs
    assert out1.count("Validation loss of updated master model:") == 2  # epochs 1 and 2 as the new rank 0
