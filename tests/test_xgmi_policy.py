"""CPU tests of the per-step all-reduce choice: the xGMI exchange form (parallel/xgmi.py
``exchange_mode``) and the start-up A/B that the multi-GPU bench runs (parallel/autotune.py):
its selection rule and, over 2 gloo ranks, its collective behaviour (every rank adopts the same
winner, a path that fails on one rank is excluded everywhere, parameters are restored)."""
import math
import os
import subprocess
import sys

import pytest
import torch

from distributed_neural_network_amd.parallel import autotune, xgmi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_auto_mode_is_pull(monkeypatch):
    monkeypatch.delenv("DNN_XGMI_EXCHANGE", raising=False)
    assert xgmi.exchange_mode() == 0


def test_explicit_modes(monkeypatch):
    for name, want in (("pull", 0), ("rsag", 2), ("pull-bf16", 4), ("rsag-bf16", 6)):
        monkeypatch.setenv("DNN_XGMI_EXCHANGE", name)
        assert xgmi.exchange_mode() == want
    for bad in ("push", "ring"):
        monkeypatch.setenv("DNN_XGMI_EXCHANGE", bad)
        with pytest.raises(ValueError):
            xgmi.exchange_mode()


def test_path_names_map_to_exchange_modes(monkeypatch):
    """Every xGMI path name of the policy maps to its exchange form and back; --grad-comm bf16
    turns the default xGMI path into its bf16-granule form; the bf16 forms are A/B candidates only
    when asked for."""
    from distributed_neural_network_amd.parallel.sync import StepAllReduce

    for name in StepAllReduce.PATHS:
        if name.startswith("xgmi-"):
            # (-pers: the same exchange inside the persistent launch)
            base = name.removesuffix("-pers")
            mode = xgmi.EXCHANGE_MODES[base[len("xgmi-"):]]
            assert "xgmi-" + xgmi.MODE_NAMES[mode] == base
    assert set(autotune.BF16_PATHS) <= set(StepAllReduce.PATHS)
    assert not set(autotune.BF16_PATHS) & set(autotune.ORDER)

    class _Comm:
        backend, distributed = "nccl", True

    class _Eng:
        overlap = False
        grad = torch.zeros(62006)

    class _PersEng(_Eng):
        persist = True
        pipeline = True

    class _PersF32Eng(_Eng):  # (the fp32 persistent launch has no in-launch exchange)
        persist = True
        pipeline = False

    pol = StepAllReduce.__new__(StepAllReduce)
    pol.comm, pol.bucket_kb = _Comm(), 0
    monkeypatch.setattr(xgmi, "wanted", lambda comm: True)
    monkeypatch.delenv("DNN_XGMI_EXCHANGE", raising=False)
    assert pol.default_path(_Eng()) == "xgmi-pull"
    # the exchange inside the persistent launch is opt-in (DNN_AB_PERS=1; fp32 granules only)
    monkeypatch.delenv("DNN_AB_PERS", raising=False)
    assert pol.default_path(_PersEng()) == "xgmi-pull"
    monkeypatch.setenv("DNN_AB_PERS", "1")
    assert pol.default_path(_PersEng()) == "xgmi-pull-pers"
    assert pol.default_path(_PersF32Eng()) == "xgmi-pull"
    pol.grad_comm = "bf16"
    assert pol.default_path(_PersEng()) == "xgmi-pull-bf16"
    assert pol.default_path(_Eng()) == "xgmi-pull-bf16"
    monkeypatch.setenv("DNN_XGMI_EXCHANGE", "rsag")
    assert pol.default_path(_Eng()) == "xgmi-rsag-bf16"


def test_choose_bf16_tie_prefers_fp32():
    res = {"xgmi-pull-bf16": _r(20.0), "xgmi-pull": _r(20.0)}
    assert autotune.choose(res) == "xgmi-pull"
    res["xgmi-pull-bf16"] = _r(19.0)
    assert autotune.choose(res) == "xgmi-pull-bf16"


def _r(us, ok=True):
    return {"us_per_step": us, "ok": ok}


def test_choose_fastest_passing():
    res = {"local": _r(10.0), "xgmi-pull": _r(30.0), "xgmi-rsag": _r(25.0), "rccl": _r(40.0),
           "rccl-overlap": _r(None, False)}
    assert autotune.choose(res) == "xgmi-rsag"


def test_pers_forms_are_opt_in_candidates(monkeypatch):
    """Round 6: the exchange inside the persistent launch lost to the serial
    one-launch exchange by tens of us/step in the in-process harness (profiles/r6/inproc/), so it
    is an A/B candidate only with DNN_AB_PERS=1 (and then ranked first)."""
    monkeypatch.delenv("DNN_AB_PERS", raising=False)
    c = autotune.default_candidates()
    assert not any(k.endswith("-pers") for k in c) and c[0] == "xgmi-pull"
    monkeypatch.setenv("DNN_AB_PERS", "1")
    c = autotune.default_candidates("bf16")
    assert c[:2] == autotune.PERS_PATHS and set(autotune.BF16_PATHS) <= set(c)


def test_choose_never_local_and_skips_failed():
    res = {"local": _r(1.0), "xgmi-pull": _r(5.0, False), "rccl": _r(50.0)}
    assert autotune.choose(res) == "rccl"
    assert autotune.choose({"local": _r(1.0)}) is None
    assert autotune.choose({"rccl": _r(math.inf)}) is None


def test_choose_tie_prefers_order():
    res = {"rccl": _r(30.0), "xgmi-rsag": _r(20.0), "xgmi-pull": _r(20.0)}
    assert autotune.choose(res) == "xgmi-pull"
    res["xgmi-pull-pers"] = _r(20.0)  # the persistent form is ranked first
    assert autotune.choose(res) == "xgmi-pull-pers"


def test_choose_prefers_rccl_within_noise(monkeypatch):
    """VERDICT r5 weak #7 / SURVEY §5.8: the custom xGMI exchange is chosen only when it beats RCCL
    by more than the A/B's noise margin (DNN_AB_RCCL_MARGIN, 3 %)."""
    monkeypatch.delenv("DNN_AB_RCCL_MARGIN", raising=False)
    res = {"rccl": _r(20.5), "rccl-overlap": _r(21.0), "xgmi-pull": _r(20.0), "xgmi-pull-pers": _r(20.2)}
    assert autotune.choose(res) == "rccl"  # 2.5 % slower: within noise
    res["rccl"] = _r(21.0)
    assert autotune.choose(res) == "xgmi-pull"  # 5 % slower: the xGMI exchange wins
    assert autotune.choose(res, margin=0.1) == "rccl"
    monkeypatch.setenv("DNN_AB_RCCL_MARGIN", "0")
    assert autotune.choose({"rccl": _r(20.0), "xgmi-pull": _r(20.0)}) == "rccl"  # (a tie is no win)
    assert autotune.choose({"rccl": _r(20.0), "xgmi-pull": _r(19.9)}) == "xgmi-pull"


def test_ab_two_ranks_agree(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "distributed_neural_network_amd.parallel.launch", "-n", "2", "--cpu",
           os.path.join(ROOT, "tests", "dist_worker.py"), "ab", str(tmp_path), "0", "0", "0"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    got = [torch.load(tmp_path / f"ab{i}.pt", weights_only=True) for i in range(2)]
    for g in got:
        res = g["res"]
        assert res["allreduce"] == "torch-pg" and g["path"] == "torch-pg", res
        assert res["failed"] == ["flaky"], res
        assert res["allreduce_ab"]["slow"] > res["allreduce_ab"]["torch-pg"], res
        assert res["local_us_per_step"] is not None
        assert g["restored"], "parameters not restored after the A/B"
    assert got[0]["res"] == got[1]["res"]  # one decision, from all-reduced numbers only
    assert torch.equal(got[0]["master"], got[1]["master"])


def test_pers_install_and_fallback(monkeypatch):
    """The "-pers" paths: installed on top of the one-launch exchange only after the persistent-
    exchange self-test passed on every rank (cached per group and form); a failing self-test makes
    the default chain fall back to the serial one-launch exchange of the same form."""
    from distributed_neural_network_amd.parallel import sync

    class _Grp:
        one_launch, xp_mode, broken = True, 0, False

    class _Sync:
        fuses_sgd = True

        def __init__(self, grp):
            self.group = grp

    class _Comm:
        backend, distributed, rank, world = "nccl", True, 0, 2

    class _Eng:
        overlap = False
        persist = pipeline = True
        grad = torch.zeros(62006)

        def __init__(self, ok):
            self.ok, self.calls, self.grad_sync, self.pers_exchange = ok, 0, None, False

        def invalidate_graphs(self):
            pass

        def selftest_pers_exchange(self, grp, comm):
            self.calls += 1
            return (self.ok, "" if self.ok else "mismatch in ['master']")

    grp = _Grp()

    def fake_install_xgmi(self, engine, mode):
        grp.xp_mode = mode
        engine.grad_sync = _Sync(grp)
        return True

    monkeypatch.setattr(sync.StepAllReduce, "_install_xgmi", fake_install_xgmi)
    monkeypatch.setattr(xgmi, "wanted", lambda comm: True)
    monkeypatch.delenv("DNN_XGMI_EXCHANGE", raising=False)
    pol = sync.StepAllReduce(_Comm())
    eng = _Eng(True)
    assert pol.install(eng, "xgmi-rsag-pers") and eng.pers_exchange and grp.xp_mode == 2
    assert pol.install(eng, "xgmi-rsag-pers") and eng.calls == 1  # cached per group and form
    assert pol.install(eng, "xgmi-pull") and not eng.pers_exchange  # a plain path clears it
    bad = _Eng(False)
    grp.__dict__.pop("selftested_pers", None)
    assert not pol.install(bad, "xgmi-pull-pers") and "self-test failed" in pol.install_why
    assert bad.grad_sync is None and not bad.pers_exchange
    pol.attach(bad)  # default path xgmi-pull-pers -> its self-test fails (cached) -> xgmi-pull
    assert bad.grad_sync is not None and not bad.pers_exchange and grp.xp_mode == 0


class _LaunchEngine:
    """Stands in for a HipEngine with an AQL queue: records which launch path each window ran."""

    def __init__(self, ok=True):
        self.direct, self.ok, self.seen = True, ok, []

    def _direct_ok(self):
        return self.direct and self.ok


def _fake_measure(times):
    def measure(comm, engine, cur, steps, warmup, reps, spin):
        p = "direct-aql" if engine.direct else "graph"
        engine.seen.append((p, spin))
        return times[p], True
    return measure


@pytest.mark.parametrize("direct_us, graph_us, winner", [(16.2, 16.5, "direct-aql"), (16.54, 16.5, "direct-aql"),
                                                          (16.9, 16.5, "graph")])
def test_launch_ab_keeps_direct_within_margin(monkeypatch, direct_us, graph_us, winner):
    """The launch A/B times both paths alternately (spin steps only before the first window) and
    keeps the direct dispatch unless the graph replay wins by more than launch_margin()."""
    from distributed_neural_network_amd.parallel import autotune

    monkeypatch.setattr(autotune, "_measure", _fake_measure({"direct-aql": direct_us, "graph": graph_us}))
    eng = _LaunchEngine()
    out = autotune.launch_ab(None, eng, None, steps=20, warmup=5, rounds=4, spin=500)
    assert out["launch"] == winner and eng.direct == (winner == "direct-aql")
    assert out["launch_ab"] == {"direct-aql": direct_us, "graph": graph_us}
    assert [p for p, _ in eng.seen] == ["direct-aql", "graph", "graph", "direct-aql"] * 2
    assert [s for _, s in eng.seen] == [500] + [0] * 7


def test_launch_ab_without_a_direct_path_is_a_no_op(monkeypatch):
    from distributed_neural_network_amd.parallel import autotune

    monkeypatch.setattr(autotune, "_measure", _fake_measure({"direct-aql": 1.0, "graph": 2.0}))
    eng = _LaunchEngine(ok=False)
    assert autotune.launch_ab(None, eng, None) == {} and not eng.seen
