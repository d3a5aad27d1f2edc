"""CPU tests of the N>1 bench plumbing (VERDICT r3 "make the N>1 bench unkillable"):

* parallel/selflaunch.py - ``python bench.py --gpus N`` without a launcher spawns its own N
  ranks (children, never an exec), relays rank 0's JSON line and, when a rank fails, returns
  non-zero with that rank's stderr tail and terminates the ranks still waiting on it;
* parallel/autotune.py - the start-up A/B is fault-contained: an RCCL communicator whose init
  raises (monkeypatched ``RcclComm``) is listed as failed with its reason and the A/B still picks
  the fastest xGMI path; an xGMI wait failure across an epoch boundary fails only its candidate;
  every candidate is timed inside one epoch with the window's shape.
"""
import io
import json
import os
import sys
import textwrap
import time

import pytest
import torch

from distributed_neural_network_amd.parallel import autotune, selflaunch
from distributed_neural_network_amd.parallel.comm import CommError
from distributed_neural_network_amd.parallel.sync import StepAllReduce
from distributed_neural_network_amd.runtime.cursor import EpochCursor

STUB = textwrap.dedent("""
    import json, os, sys, time
    r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and os.environ["DNN_STORE_EXTERNAL"] == "1"
    mode = sys.argv[1]
    print(f"rank {r} of {n} starting", file=sys.stderr, flush=True)
    if mode == "fail" and r == 1:
        print("boom: rank 1 fails", file=sys.stderr, flush=True)
        sys.exit(3)
    if mode == "fail":
        time.sleep(120)  # stuck on the dead peer: the launcher must end it
    if r == 0:
        print("banner that is not json")
        print(json.dumps({"metric": "m", "value": 1.5, "n_gpus": n}))
""")


def _stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return str(p)


def test_launcher_present():
    assert not selflaunch.launcher_present({})
    assert selflaunch.launcher_present({"WORLD_SIZE": "4"})
    assert selflaunch.launcher_present({"OMPI_COMM_WORLD_SIZE": "2"})
    assert not selflaunch.launcher_present({"WORLD_SIZE": ""})


def test_spawn_and_relay(tmp_path, monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    r, w = os.pipe()
    err = io.StringIO()
    rc = selflaunch.run([sys.executable, _stub(tmp_path), "ok"], 3, out_fd=w, err=err)
    os.close(w)
    out = os.read(r, 1 << 16).decode()
    os.close(r)
    assert rc == 0, err.getvalue()
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1 and json.loads(lines[0]) == {"metric": "m", "value": 1.5, "n_gpus": 3, "launch_attempts": 1}
    log = err.getvalue()
    assert "[r1] rank 1 of 3 starting" in log and "[r2] rank 2 of 3 starting" in log
    assert "banner that is not json" not in out


def test_failed_rank_reports_and_ends_the_job(tmp_path, monkeypatch):
    monkeypatch.setenv("DNN_LAUNCH_ATTEMPTS", "1")  # (the retry is tested below)
    r, w = os.pipe()
    err = io.StringIO()
    t0 = time.time()
    rc = selflaunch.run([sys.executable, _stub(tmp_path), "fail"], 2, out_fd=w, err=err, grace_s=1.0)
    os.close(w)
    out = os.read(r, 1 << 16).decode()
    os.close(r)
    assert rc == 3, err.getvalue()
    assert out == ""
    log = err.getvalue()
    assert "attempt 1: rank 1 (exit code 3) stderr tail" in log and "boom: rank 1 fails" in log
    assert "terminating" in log
    assert time.time() - t0 < 60  # rank 0 (sleeping 120 s) was terminated after the grace


# ---- A/B fault containment ------------------------------------------------------------------


class _Comm:
    backend, distributed, rank, world, generation = "nccl", True, 0, 1, 0
    native = None

    def gather_scalars(self, x):
        return [float(x)]

    def reduce_scalar(self, x, op="max"):
        return float(x)

    def barrier(self):
        pass


class _Group:
    def __init__(self, mode):
        self.xp_mode, self.one_launch = mode, True


class XgmiGradSync:  # (named like the real one: StepAllReduce.installed reads the class name)
    fuses_sgd = True

    def __init__(self, mode, cost_s, fail=False):
        self.group, self.cost, self.fail = _Group(mode), cost_s, fail

    def failed(self):
        return self.fail


class _Engine:
    device = torch.device("cpu")

    def __init__(self):
        self.master = torch.arange(8, dtype=torch.float32)
        self.mom = torch.zeros(8)
        self.grad_sync = None
        self.windows = []  # (steps left in the epoch when a window of run_steps started)
        self.epochs = 0
        self.exact = set()

    def params_changed(self):
        pass

    def epoch_stats(self, reset=True):
        return None

    def begin_epoch(self, order):
        self.epochs += 1

    def prepare_graphs(self, exact=()):
        self.exact = set(exact)

    def run_steps(self, n):
        gs = self.grad_sync
        time.sleep(n * (0.0002 + (gs.cost if gs is not None else 0.0)))
        self.master.add_(1.0)  # training moves the parameters: the A/B must restore them


class _Sampler:
    def __init__(self, steps):
        self.n = steps

    def steps(self, batch):
        return self.n

    def order(self, epoch):
        return list(range(self.n))


class _Policy(StepAllReduce):
    """The real install() (RCCL paths included); only the xGMI group build is faked."""
    COST = {0: 0.0003, 2: 0.0006}
    FAIL = ()

    def _install_xgmi(self, engine, mode):
        engine.grad_sync = XgmiGradSync(mode, self.COST[mode], fail=mode in self.FAIL)
        return True


def _ab(policy, engine, spe=40, **kw):
    cur = EpochCursor(engine, _Sampler(spe), policy, 16)
    return autotune.allreduce_ab(policy, engine, cur, steps=8, warmup=2, reps=2, spin=3, **kw), cur


def test_ab_contains_an_rccl_init_failure(monkeypatch):
    from distributed_neural_network_amd.parallel import rccl

    class Boom:
        def __init__(self, comm):
            raise CommError("ncclCommInitRankConfig did not finish within 60 s")

    monkeypatch.setattr(rccl, "RcclComm", Boom)
    eng, pol = _Engine(), _Policy(_Comm())
    start = eng.master.clone()
    res, _ = _ab(pol, eng, candidates=autotune.ORDER)
    assert res["allreduce"] == "xgmi-pull" and pol.path == "xgmi-pull", res
    assert "rccl" in res["failed"] and "rccl-overlap" in res["failed"], res
    assert "CommError" in res["why"]["rccl"] and "60 s" in res["why"]["rccl"], res
    assert res["allreduce_ab"]["xgmi-pull"] < res["allreduce_ab"]["xgmi-rsag"], res
    assert res["allreduce_ab"]["rccl"] is None
    assert torch.equal(eng.master, start), "parameters not restored"
    assert pol.comm.native is None


def test_ab_wait_failure_across_epoch_boundaries_fails_only_its_candidate():
    """a failing candidate's error vote at an epoch end must not escape the A/B."""
    eng, pol = _Engine(), _Policy(_Comm())
    pol.FAIL = (2,)  # the two-hop exchange's waits fail
    pol.lazy_check = False
    res, cur = _ab(pol, eng, spe=11, candidates=("xgmi-pull", "xgmi-rsag"))  # 11 < 2 + 8 + 2: boundaries
    assert res["failed"] == ["xgmi-rsag"] and "wait failed" in res["why"]["xgmi-rsag"], res
    assert res["allreduce"] == "xgmi-pull"
    assert pol.lazy_check is False  # restored
    assert cur.epoch > 1


def test_ab_times_inside_one_epoch_with_an_exact_graph():
    eng, pol = _Engine(), _Policy(_Comm())
    seen = []
    orig = EpochCursor.run

    def run(self, k):
        if k == 8:
            seen.append((self.left, set(eng.exact)))
        return orig(self, k)

    EpochCursor.run = run
    try:
        res, _ = _ab(pol, eng, spe=40, candidates=("xgmi-pull",))
    finally:
        EpochCursor.run = orig
    assert res["allreduce"] == "xgmi-pull"
    assert seen and all(left >= 8 and 8 in exact for left, exact in seen), seen


def test_ab_no_path_at_all_falls_back_to_the_policy_default(monkeypatch):
    """Every candidate failing is not fatal to the A/B itself: the policy's own attach runs."""
    eng = _Engine()

    class P(_Policy):
        def install(self, engine, name):
            if name == "local":
                return super().install(engine, name)
            raise RuntimeError(f"{name} broken")

        def attach(self, engine):
            engine.grad_sync = None
            self.attached = True

    pol = P(_Comm())
    res, _ = _ab(pol, eng, candidates=("xgmi-pull", "rccl"))
    assert res["failed"] == ["rccl", "xgmi-pull"] and getattr(pol, "attached", False), res
    assert "broken" in res["why"]["rccl"]


@pytest.mark.parametrize("n", [2])
def test_bench_refuses_nothing_without_launcher(n):
    """bench.py no longer exits at --gpus N>1 without torchrun: it self-launches (source check;
    the GPU run itself is tools/gpu_run.sh rehearse2)."""
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")).read()
    assert "needs torchrun" not in src
    i_launch = src.index("selflaunch.run(")
    i_gpu = src.index("torch.cuda.set_device")
    assert i_launch < i_gpu  # children are spawned before the first GPU call


def test_device_count_reads_sysfs_not_hip(tmp_path, monkeypatch):
    """The launcher counts GPUs from the KFD topology + visibility variables (a
    torch.cuda.device_count() fallback could initialise HIP in the launcher)."""
    topo, dri = tmp_path / "nodes", tmp_path / "dri"
    topo.mkdir()
    dri.mkdir()
    for i, gfx in enumerate([0, 90500, 90500, 0, 90500]):  # 2 CPU nodes, 3 GPU nodes
        d = topo / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 4\ngfx_target_version {gfx}\nsimd_count 1024\n"
                                      f"drm_render_minor {128 + i}\n")
    for i in (1, 2):  # this "container" may open the render nodes of two of the three GPUs
        (dri / f"renderD{128 + i}").write_text("")
    assert selflaunch._kfd_gpu_nodes(str(topo), str(dri)) == 2
    assert selflaunch._kfd_gpu_nodes(str(topo), str(tmp_path / "no-dri")) == 3  # no /dev/dri to check
    assert selflaunch._kfd_gpu_nodes(str(tmp_path / "missing")) == -1
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    assert selflaunch._visible_list(3) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")
    assert selflaunch._visible_list(3) == 2
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")
    assert selflaunch._visible_list(3) == 0
    # the module never imports the GPU runtime's device query at launch time
    src = open(selflaunch.__file__).read()
    body = src[src.index("def visible_devices"):src.index("def die_with_parent")]
    assert "torch.cuda" not in body.split("subprocess.run")[0]


def test_ab_wall_budget_bounds_the_start_up(monkeypatch):
    """a candidate whose set-up sleeps past the A/B's wall budget is marked
    failed, the candidates after it are skipped, RCCL's init timeout is capped by the budget left
    (and after an xGMI pass), and the JSON carries ab_wall_s + the step variant per path."""
    from distributed_neural_network_amd.parallel import rccl

    seen_tmo = []

    class Slow:
        def __init__(self, comm):
            seen_tmo.append(float(os.environ["DNN_RCCL_INIT_TIMEOUT_S"]))
            time.sleep(1.6)  # ignores every deadline
            raise CommError("init too slow")

    monkeypatch.setattr(rccl, "RcclComm", Slow)
    eng, pol = _Engine(), _Policy(_Comm())
    t0 = time.perf_counter()
    res, _ = _ab(pol, eng, candidates=("xgmi-pull", "rccl", "rccl-overlap", "xgmi-rsag"), budget_s=1.0,
                 rounds=1)
    wall = time.perf_counter() - t0
    assert res["allreduce"] == "xgmi-pull", res
    assert "rccl" in res["failed"] and "rccl-overlap" in res["failed"] and "xgmi-rsag" in res["failed"], res
    assert "skipped" in res["why"]["xgmi-rsag"] and "budget" in res["why"]["xgmi-rsag"], res
    assert seen_tmo and seen_tmo[0] <= 15.0, seen_tmo  # capped after the xGMI pass
    assert wall < 1.0 + 1.6 + 1.0 and res["ab_wall_s"] <= wall + 0.01, (wall, res)
    assert res["variant"]["xgmi-pull"] in ("persistent", "pipelined", "serial")
    assert pol.ab_deadline is None


def test_ab_default_candidates(monkeypatch):
    c = autotune.default_candidates()
    assert c == autotune.ORDER and not set(autotune.BF16_PATHS) & set(c)
    assert set(autotune.BF16_PATHS) <= set(autotune.default_candidates("bf16"))
    assert not any(p.endswith("-ovl") for p in StepAllReduce.PATHS)  # (removed in round 6: they lost 3x)


# ---- bounded retry in fresh ranks -----------------------------------------

RETRY_STUB = textwrap.dedent("""
    import json, os, sys, time
    import torch.distributed as dist
    from distributed_neural_network_amd.parallel.fault import setup_crash_injection
    r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    print(f"rank {r} attempt {os.environ.get('DNN_LAUNCH_ATTEMPT')} starting", file=sys.stderr, flush=True)
    st = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), n, is_master=False)
    setup_crash_injection("xgmi-setup", r)   # the xGMI group set-up of parallel/xgmi.py
    # a "collective": every rank arrives; a rank whose peer died sees the launcher's death notice
    st.add("arrive", 1)
    while st.add("arrive", 0) < n:
        if any(st.check([f"dnn/dead/{p}"]) for p in range(n)):
            print("peer died: collective failed", file=sys.stderr, flush=True)
            sys.exit(5)
        time.sleep(0.01)
    print("timed window start", file=sys.stderr, flush=True)
    if r == 0:
        print(json.dumps({"metric": "m", "value": 2.0, "n_gpus": n,
                          "safe": os.environ.get("DNN_SAFE_TRANSPORT", "0"),
                          "allreduce_env": os.environ.get("DNN_ALLREDUCE", "")}))
""")


def _retry_stub(tmp_path):
    p = tmp_path / "retry_stub.py"
    p.write_text(RETRY_STUB)
    return str(p)


def _env_for_stub(monkeypatch):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    monkeypatch.setenv("PYTHONPATH", root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "DNN_SAFE_TRANSPORT", "DNN_LAUNCH_ATTEMPT",
              "DNN_LAUNCH_ATTEMPTS", "DNN_INJECT_CRASH", "TORCHELASTIC_USE_AGENT_STORE"):
        monkeypatch.delenv(k, raising=False)


def test_retry_after_an_injected_xgmi_setup_crash(tmp_path, monkeypatch):
    """Attempt 1 loses rank 1 in the xGMI set-up (exit 134, like a GPU fault's abort); the launcher
    starts attempt 2 in fresh ranks with the conservative transport and prints exactly ONE result
    line, from attempt 2, carrying launch_attempts and the first failure (rank, code, phase, tail)."""
    _env_for_stub(monkeypatch)
    monkeypatch.setenv("DNN_INJECT_XGMI_SETUP_FAIL", "1")
    r, w = os.pipe()
    err = io.StringIO()
    rc = selflaunch.run([sys.executable, _retry_stub(tmp_path)], 2, out_fd=w, err=err, grace_s=2.0)
    os.close(w)
    out = os.read(r, 1 << 16).decode()
    os.close(r)
    assert rc == 0, err.getvalue()
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out
    res = json.loads(lines[0])
    assert res["launch_attempts"] == 2 and res["safe"] == "1" and res["allreduce_env"] == "rccl", res
    assert res["launch_transport"].startswith("rccl"), res
    (f,) = res["launch_failures"]
    assert f["attempt"] == 1 and f["rank"] == 1 and f["exit_code"] == 134, f
    assert f["phase"] == "before the timed window", f
    assert any("injected crash at xgmi-setup on rank 1" in ln for ln in f["stderr_tail"]), f
    log = err.getvalue()
    assert "retrying in fresh ranks: attempt 2" in log and "[r0 a2] rank 0 attempt 2 starting" in log, log


def test_no_retry_when_one_attempt_is_allowed(tmp_path, monkeypatch):
    _env_for_stub(monkeypatch)
    monkeypatch.setenv("DNN_INJECT_XGMI_SETUP_FAIL", "1")
    monkeypatch.setenv("DNN_LAUNCH_ATTEMPTS", "1")
    r, w = os.pipe()
    err = io.StringIO()
    rc = selflaunch.run([sys.executable, _retry_stub(tmp_path)], 2, out_fd=w, err=err, grace_s=2.0)
    os.close(w)
    out = os.read(r, 1 << 16).decode()
    os.close(r)
    assert rc == 134 and out == "", (rc, out, err.getvalue())
    assert "no JSON result line" in err.getvalue()


def test_attempt_plan_and_annotation():
    assert [t for t, _ in selflaunch.attempt_plan({})] == [t for t, _ in selflaunch.ATTEMPTS]
    assert len(selflaunch.attempt_plan({"DNN_LAUNCH_ATTEMPTS": "2"})) == 2
    assert selflaunch.attempt_plan({"DNN_LAUNCH_ATTEMPTS": "0"}) == list(selflaunch.ATTEMPTS[:1])
    # every retry level drops the xGMI group; the last one drops RCCL as well
    assert all(env.get("DNN_ALLREDUCE") == "rccl" for _, env in selflaunch.ATTEMPTS[1:])
    assert selflaunch.ATTEMPTS[-1][1]["DNN_BACKEND"] == "gloo"
    one = selflaunch._Attempt(1, "as requested")
    assert json.loads(selflaunch.annotate('{"value": 1}', [one])) == {"value": 1, "launch_attempts": 1}


def test_supervisors_under_torchrun_retry_together(tmp_path, monkeypatch):
    """torchrun launched the ranks (agent store on MASTER_PORT): every rank process supervises its
    real rank as a child; after rank 1's injected set-up crash both supervisors start attempt 2,
    rank 0's supervisor prints the one annotated result line, both exit 0."""
    import subprocess

    import torch.distributed as dist

    _env_for_stub(monkeypatch)
    port = selflaunch._free_port()
    agent = dist.TCPStore("127.0.0.1", port, 3, is_master=True, wait_for_workers=False)
    stub = _retry_stub(tmp_path)
    code = ("import sys; from distributed_neural_network_amd.parallel import selflaunch as s; "
            f"assert s.supervisor_wanted(); sys.exit(s.supervise([sys.executable, {stub!r}], grace_s=2.0))")
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True", TORCHELASTIC_RUN_ID="t1",
                   DNN_INJECT_XGMI_SETUP_FAIL="1")
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    del agent
    assert [p.returncode for p in procs] == [0, 0], outs
    lines = [ln for ln in outs[0][0].splitlines() if ln.strip()]
    assert len(lines) == 1 and outs[1][0].strip() == "", outs
    res = json.loads(lines[0])
    assert res["launch_attempts"] == 2 and res["launch_failures"][0]["rank"] == 1, res
    assert res["launch_failures"][0]["exit_code"] == 134 and res["safe"] == "1", res
    assert not selflaunch.supervisor_wanted({"TORCHELASTIC_USE_AGENT_STORE": "True", "WORLD_SIZE": "2",
                                             "DNN_SUPERVISED": "1"})
    assert not selflaunch.supervisor_wanted({"WORLD_SIZE": "2"})  # mpiexec / plain env: no supervisor


def test_bench_supervises_before_touching_the_gpu():
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")).read()
    assert src.index("selflaunch.supervise(") < src.index("torch.cuda.set_device")
    assert "DNN_SAFE_TRANSPORT" in src and "selflaunch.WINDOW_MARK" in src


def test_trainer_and_bench_share_the_ab_window_rule():
    """one A/B window rule for bench.py and the trainer."""
    assert autotune.ab_window(782, 20, 5) == (20, 5)  # the bench's driver window
    assert autotune.ab_window(782, 5000, 500) == (autotune.AB_MAX_STEPS, 500)
    steps, warm = autotune.ab_window(782)  # a trainer: as much of an epoch as fits
    assert steps == autotune.AB_MAX_STEPS and 1 <= warm <= 64 and steps + warm <= 782
    steps, warm = autotune.ab_window(11)
    assert steps + warm <= 11 and steps >= 1 and warm >= 1
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "distributed_neural_network_amd", "train", "trainer.py")).read()
    assert "ab_window(cur.steps_per_epoch)" in src and "steps=64, warmup=16" not in src
