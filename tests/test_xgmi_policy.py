"""CPU tests of the xGMI exchange-form choice (parallel/xgmi.py ``exchange_mode``).

The kernels themselves are covered by tests/test_xgmi_gpu.py; this pins the policy: the
one-hop pull form by default, the two-hop and push forms only on request (push only over
uncached regions), and every rank voting on the region kind."""
import types

import pytest

from distributed_neural_network_amd.parallel import xgmi


def _grp(world, devices, kinds):
    calls = []

    def gather_scalars(v):
        calls.append(v)
        return [1.0 if k == "uncached" else 0.0 for k in kinds]

    comm = types.SimpleNamespace(gather_scalars=gather_scalars)
    return types.SimpleNamespace(comm=comm, world=world, devices=devices, kind=kinds[0]), calls


@pytest.mark.parametrize("world,devices,want", [(1, 1, 0), (2, 2, 0), (4, 4, 0), (8, 8, 0), (4, 1, 0), (8, 1, 0)])
def test_auto_mode(monkeypatch, world, devices, want):
    monkeypatch.delenv("DNN_XGMI_EXCHANGE", raising=False)
    g, calls = _grp(world, devices, ["uncached"] * world)
    assert xgmi.exchange_mode(g) == want
    assert len(calls) == 1  # collective: every rank takes part in the vote


def test_explicit_modes(monkeypatch):
    for name, want in (("pull", 0), ("push", 1), ("rsag", 2)):
        monkeypatch.setenv("DNN_XGMI_EXCHANGE", name)
        g, _ = _grp(8, 8, ["uncached"] * 8)
        assert xgmi.exchange_mode(g) == want
    # push needs uncached regions on EVERY rank
    monkeypatch.setenv("DNN_XGMI_EXCHANGE", "push")
    g, _ = _grp(4, 4, ["uncached", "device", "uncached", "uncached"])
    assert xgmi.exchange_mode(g) == 0 and not xgmi.push_wanted(g)
    monkeypatch.setenv("DNN_XGMI_EXCHANGE", "ring")
    with pytest.raises(ValueError):
        xgmi.exchange_mode(g)
