"""Fault-detection hardening for a loaded multi-GPU host:

* a WHOLE-process stall of a live rank (SIGSTOP for 3 s; a 1.5 s GIL hold on one of 8 ranks)
  costs at most one all-alive retry, never the rank's place - the exclusion grace for a
  heartbeat-only-stale rank is separate from (and much longer than) the flag timeout;
* a rank whose process is gone on this host is dead at once even without a launcher
  (pid liveness), so the longer grace does not slow real drops down;
* the heartbeat timeout follows the observed beat jitter;
* the stand-alone rendezvous store of agentless launches refuses to serve a new job when it is
  a left-over from an earlier one (job token, stale heartbeats, checked-out counters), and
  exits by itself once its job's heartbeats go stale.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest
import torch.distributed as dist

from distributed_neural_network_amd.parallel import CommError, Communicator, DistEnv
from distributed_neural_network_amd.parallel.fault import Heartbeat, exclusion_grace, pid_alive

from test_distributed_cpu import ROOT, _launch_env

SMALL = ["--train-samples", "1536", "--test-samples", "128", "--device", "cpu", "--lr", "0.01"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _summary(path):
    for line in open(path):
        rec = json.loads(line).get("record", {})
        if rec.get("event") == "summary":
            return rec
    raise AssertionError("no summary record")


def test_sigstop_stall_is_a_retry_not_an_exclusion(tmp_path):
    env = {"DNN_INJECT_STALL": "1:1:3.0:sigstop", "DNN_HEARTBEAT_TIMEOUT": "1.0"}
    r = _launch_env(3, [os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "4", "--batch-size", "32",
                        "--sync", "step-allreduce", "--nb-proc", "3", "--metrics", "m.jsonl"] + SMALL, tmp_path, env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "injected sigstop stall" in r.stdout
    assert "dropped in epoch" not in r.stdout and "excluded" not in r.stdout + r.stderr, r.stdout
    assert r.stdout.count("with every rank alive; communicator re-created") <= 1, r.stdout
    assert r.stdout.count("Validation loss of updated master model:") == 4
    s = _summary(tmp_path / "m.jsonl")
    assert s["retries_all_alive"] <= 1 and s["recoveries"] == s["retries_all_alive"], s


@pytest.mark.timeout(600)
def test_eight_ranks_gil_hold_no_exclusion(tmp_path):
    """8 gloo ranks on one loaded host; rank 3's main thread holds the GIL for 1.5 s (its beat
    thread cannot run): with the default timeout (1 s + 0.1 s per rank) nobody is excluded and
    there is at most one all-alive retry."""
    env = {"DNN_INJECT_STALL": "3:1:1.5:gil"}
    env.pop("DNN_HEARTBEAT_TIMEOUT", None)
    r = _launch_env(8, [os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "3", "--batch-size", "16",
                        "--sync", "step-allreduce", "--nb-proc", "8", "--metrics", "m.jsonl"] + SMALL, tmp_path, env,
                    timeout=540)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "injected gil stall" in r.stdout
    assert "dropped in epoch" not in r.stdout, r.stdout
    assert r.stdout.count("with every rank alive; communicator re-created") <= 1, r.stdout
    assert r.stdout.count("Validation loss of updated master model:") == 3
    s = _summary(tmp_path / "m.jsonl")
    assert s["retries_all_alive"] <= 1 and s["heartbeat_timeout_s"] >= 1.8, s


def test_dead_local_pid_is_dead_at_once(monkeypatch):
    store = dist.TCPStore("127.0.0.1", 0, 1, is_master=True, wait_for_workers=False)
    c = Communicator(DistEnv(0, 1, 0, "127.0.0.1", store.port), "cpu")
    c.members = [0, 1, 2]
    p = subprocess.Popen([sys.executable, "-c", "pass"])
    p.wait()
    store.set("dnn/pid/1", f"{socket.gethostname()}:{p.pid}")         # exited, reaped
    store.set("dnn/pid/2", f"some-other-host:{os.getpid()}")          # remote: unknown
    store.set("dnn/hb/2", repr(time.time() + 60.0))                   # ...and beating
    hb = Heartbeat(c, period_s=0.05, timeout_s=30.0)
    try:
        assert hb.reported_dead(1) and not hb.reported_dead(2)
        assert not hb.reported_dead(0)
        t0 = time.time()
        while 1 not in hb.dead and time.time() - t0 < 5:
            time.sleep(0.02)
        assert 1 in hb.dead and 2 not in hb.dead
    finally:
        hb.stop()
    assert pid_alive(os.getpid()) and not pid_alive(p.pid)


def test_timeout_follows_observed_jitter():
    store = dist.TCPStore("127.0.0.1", 0, 1, is_master=True, wait_for_workers=False)
    c = Communicator(DistEnv(0, 1, 0, "127.0.0.1", store.port), "cpu")
    hb = Heartbeat(c, period_s=10.0, timeout_s=1.0)
    try:
        assert hb.timeout == 1.0
        t = 1000.0
        for gap in [0.1] * 50 + [0.6] * 5:
            t += gap
            hb._observe(1, t)
        assert hb.timeout == pytest.approx(4 * 0.6)
        assert exclusion_grace(hb) >= 10.0
    finally:
        hb.stop()


def _env_for(rank, world, port):
    env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for k in ("DNN_STORE_EXTERNAL", "TORCHELASTIC_USE_AGENT_STORE"):
        env.pop(k, None)
    return env


def _server(port, world, token, *extra):
    return subprocess.Popen([sys.executable, "-m", "distributed_neural_network_amd.parallel.store_server", "--port",
                             str(port), "--world", str(world), "--token", token, *extra], cwd=ROOT,
                            env=dict(os.environ, PYTHONPATH=ROOT))


def _wait_up(port, token):
    t0 = time.time()
    while time.time() - t0 < 30:
        try:
            c = dist.TCPStore("127.0.0.1", port, 1, is_master=False, timeout=__import__("datetime").timedelta(seconds=2))
            if c.check(["dnn/store_server"]) and c.get("dnn/store_server").decode() == token:
                return c
        except Exception:
            pass
        time.sleep(0.1)
    raise AssertionError("store server did not come up")


def test_left_over_store_is_refused(monkeypatch):
    port = _free_port()
    old = _server(port, 2, "old-job")
    try:
        st = _wait_up(port, "old-job")
        st.set("dnn/hb/1", repr(time.time() - 120.0))  # the earlier job's last beat
        # rank 0 of a new job: its own server cannot bind the taken port, the token differs
        for k, v in _env_for(0, 2, port).items():
            monkeypatch.setenv(k, v)
        monkeypatch.delenv("DNN_STORE_EXTERNAL", raising=False)
        with pytest.raises(CommError, match="not this job's"):
            Communicator(device="cpu", timeout_s=20)
        # rank 1 of the new job cannot check a token; the stale heartbeat gives the store away
        for k, v in _env_for(1, 2, port).items():
            monkeypatch.setenv(k, v)
        with pytest.raises(CommError, match="old heartbeat"):
            Communicator(device="cpu", timeout_s=20)
        st.set("dnn/hb/1", repr(time.time()))
        st.add("dnn/closed", 1)
        with pytest.raises(CommError, match="finished job"):
            Communicator(device="cpu", timeout_s=20)
    finally:
        old.kill()
        old.wait()


def test_store_server_exits_when_heartbeats_go_stale():
    port = _free_port()
    srv = _server(port, 2, "tok", "--stale", "1.0")
    try:
        st = _wait_up(port, "tok")
        st.set("dnn/hb/0", repr(time.time()))
        assert srv.wait(timeout=20) == 0
    finally:
        if srv.poll() is None:
            srv.kill()


def test_checked_out_peer_is_never_flagged():
    """A peer that finished its run (``dnn/done/<r>``, written before it exits) is not dead when
    its pid is gone or its heartbeat goes stale (a fast rank's normal exit
    was taken for a death and the last epoch was redone without it)."""
    store = dist.TCPStore("127.0.0.1", 0, 1, is_master=True, wait_for_workers=False)
    c = Communicator(DistEnv(0, 1, 0, "127.0.0.1", store.port), "cpu")
    c.members = [0, 1]
    p = subprocess.Popen([sys.executable, "-c", "pass"])
    p.wait()
    store.set("dnn/pid/1", f"{socket.gethostname()}:{p.pid}")  # exited
    store.set("dnn/hb/1", repr(time.time() - 60.0))             # and silent
    store.set("dnn/done/1", repr(time.time()))                  # but checked out first
    hb = Heartbeat(c, period_s=0.02, timeout_s=0.1)
    try:
        time.sleep(0.5)
        assert 1 not in hb.dead and hb.checked_out(1) and c.lost() == []
    finally:
        hb.stop()


@pytest.mark.parametrize("where", ["before", "after"])
def test_normal_exit_of_fast_rank_is_not_a_drop(tmp_path, where):
    """Rank 0 idles 0.5 s after the last epoch's last collective (``before``: the final barrier
    holds its peers; ``after``: its peers pass the barrier, check out and EXIT while rank 0's
    watchdog still runs): no flag, no recovery, every epoch reported once."""
    env = {"DNN_INJECT_END_SKEW": f"0:0.5:{where}", "DNN_HEARTBEAT_TIMEOUT": "1.0"}
    r = _launch_env(3, [os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "2", "--batch-size", "32",
                        "--sync", "step-allreduce", "--nb-proc", "3"] + SMALL, tmp_path, env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "injected end skew: rank 0" in r.stdout
    assert "[fault] watchdog" not in r.stdout and "dropped in epoch" not in r.stdout, r.stdout
    assert "re-created" not in r.stdout, r.stdout
    assert r.stdout.count("Validation loss of updated master model:") == 2


def test_store_server_outlives_idle_while_a_local_rank_lives():
    """No heartbeat, no store writes (a bench rank): the idle exit waits while a registered rank
    process of this host is alive, and the server exits once every registered rank is gone
    (the idle exit could pull the store from under a live job)."""
    from distributed_neural_network_amd.parallel.store_server import decide

    kw = dict(world=2, closed=0, dropped=0, beats=[None, None], stale=30.0, idle=5.0, now=1000.0)
    assert decide(pids={0: 11, 1: 12}, alive=[11], idle_for=1e4, **kw) is None  # a live rank: stay
    assert "gone" in decide(pids={0: 11, 1: 12}, alive=[], idle_for=0.0, **kw)  # all local ranks gone
    assert decide(pids={0: 11}, alive=[], idle_for=1.0, **kw) is None  # rank 1 not registered yet
    assert "no activity" in decide(pids={}, alive=[], idle_for=6.0, **kw)  # nothing known: idle exit
    assert "checked out" in decide(pids={0: 11}, alive=[11], idle_for=0.0, **dict(kw, closed=2))
    assert "heartbeat" in decide(pids={0: 11}, alive=[11], idle_for=0.0, **dict(kw, beats=[900.0, None]))
    # rank 1 runs on another host (pid -1): rank 0's host losing its only rank must not
    # pull the store from under the survivor; only stale heartbeats (or check-outs) end it then
    assert decide(pids={0: 11, 1: -1}, alive=[], idle_for=0.0, **kw) is None
    assert decide(pids={0: 11, 1: -1}, alive=[], idle_for=1e4, **kw) is None
    assert "heartbeat" in decide(pids={0: 11, 1: -1}, alive=[], idle_for=0.0, **dict(kw, beats=[900.0, 960.0]))
    # the running server applies it: a registered live rank keeps it up past the idle bound
    port = _free_port()
    srv = _server(port, 2, "tok2", "--idle", "5")
    live = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    try:
        st = _wait_up(port, "tok2")
        st.set("dnn/pid/0", f"{socket.gethostname()}:{live.pid}")
        st.set("dnn/pid/1", f"{socket.gethostname()}:{os.getpid() + 10 ** 7}")  # never a live pid
        time.sleep(6.5)
        assert srv.poll() is None, "store exited under a live rank"
        live.kill()
        live.wait()
        assert srv.wait(timeout=20) == 0
    finally:
        for p in (srv, live):
            if p.poll() is None:
                p.kill()
