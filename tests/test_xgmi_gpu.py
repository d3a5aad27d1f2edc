"""GPU tests of the one-shot xGMI gradient all-reduce (csrc/comm/xgmi_allreduce.hip).

The box has one GPU, so the multi-rank cases run 2 processes on the same device (IPC
regions of another process on the same GPU go through the same hipIpc path as peers on
other GPUs); host collectives use gloo there (RCCL refuses two ranks on one device).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _py(code, env_extra, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=timeout)


def test_xgmi_one_rank_matches_local_sgd():
    """World size 1 with forced collectives: the one-launch exchange (grad_reduce publishes,
    flags, gathers, applies SGD + bf16 images) and the two-launch path (batch reduce -> xGMI
    kernel) must both reproduce the fused local-SGD step bitwise."""
    code = r'''
import numpy as np, torch
from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.parallel import Communicator, make_policy
from distributed_neural_network_amd.parallel.xgmi import XgmiGradSync
from distributed_neural_network_amd.runtime import HipEngine
torch.cuda.set_device(0)
comm = Communicator(device=torch.device("cuda", 0))
data = synthetic(1000, 5)
a = init_arena(seed=9)
res = []
import os
for sync_on, graphs, one, xch in [(False, True, "1", "pull"), (True, True, "1", "pull"), (True, False, "1", "pull"),
                                  (True, True, "0", "pull"), (True, True, "1", "rsag")]:
    os.environ["DNN_XGMI_ONE_LAUNCH"] = one
    os.environ["DNN_XGMI_EXCHANGE"] = xch
    eng = HipEngine(batch=64, arena=a, graph_chunk=4, use_graphs=graphs)
    pol = make_policy("step-allreduce", comm)
    pol.attach(eng)
    if not sync_on:
        eng.grad_sync = None
    else:
        assert isinstance(eng.grad_sync, XgmiGradSync), type(eng.grad_sync)
        assert eng.grad_sync.group.one_launch == (one == "1"), "exchange self-test failed"
        assert eng.grad_sync.group.xp_mode == (2 if xch == "rsag" else 0)
    eng.attach(data); eng.begin_epoch(np.arange(1000, dtype=np.int32)); eng.run_steps(16)
    torch.cuda.synchronize()
    if sync_on:
        pol.epoch_end(eng, 0)  # raises if a wait timed out
    res.append((eng.master.cpu(), eng.mom.cpu(), eng.shadow.cpu(), eng.epoch_stats()))
for m, mo, sh, st in res[1:]:
    assert torch.equal(res[0][0], m) and torch.equal(res[0][1], mo) and torch.equal(res[0][2], sh)
    assert st.samples == 1000 and st.loss_sum == res[0][3].loss_sum
print("kind", comm.xgmi.kind)
comm.close()
print("OK")
'''
    r = _py(code, {"DNN_FORCE_COLLECTIVES": "1", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29631"})
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_xgmi_one_rank_layer_engine_matches_local_sgd():
    """The layer engine on a 1-rank xGMI group (all-reduce fused with SGD) must equal its local
    SGD tail bitwise, and still advance the step cursor and the epoch statistics (the fused
    path once skipped the bookkeeping: every step re-ran the first batch)."""
    code = r'''
import numpy as np, torch
from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.parallel import Communicator, make_policy
from distributed_neural_network_amd.parallel.xgmi import XgmiGradSync
from distributed_neural_network_amd.runtime.layer_engine import LayerEngine
torch.cuda.set_device(0)
comm = Communicator(device=torch.device("cuda", 0))
data = synthetic(1000, 5)
res = []
for sync_on, graphs in [(False, True), (True, True), (True, False)]:
    eng = LayerEngine(batch=64, model="lenet", seed=4, device="cuda", graph_chunk=4, use_graphs=graphs)
    pol = make_policy("step-allreduce", comm)
    pol.attach(eng)
    if not sync_on:
        eng.grad_sync = None
    else:
        assert isinstance(eng.grad_sync, XgmiGradSync), type(eng.grad_sync)
    eng.attach(data); eng.begin_epoch(np.arange(1000, dtype=np.int32)); eng.run_steps(16)
    torch.cuda.synchronize()
    if sync_on:
        pol.epoch_end(eng, 0)
    res.append((eng.master.cpu(), eng.mom.cpu(), eng.epoch_stats(), int(eng.state[0])))
for m, mo, st, cur in res:
    assert st.samples == 1000 and st.batches == 16 and cur == 16, (st, cur)
for m, mo, st, cur in res[1:]:
    assert torch.equal(res[0][0], m) and torch.equal(res[0][1], mo)
    assert st.loss_sum == res[0][2].loss_sum
comm.close()
print("OK")
'''
    r = _py(code, {"DNN_FORCE_COLLECTIVES": "1", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29633"})
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


_TWO_RANK = r'''
import os, sys, numpy as np, torch
from distributed_neural_network_amd.data import EpochSampler, synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.parallel import Communicator, make_policy, replica_checksums
torch.cuda.set_device(0)
comm = Communicator(device=torch.device("cuda", 0))
from distributed_neural_network_amd.runtime import HipEngine
data = synthetic(2048, 3)
if os.environ.get("ENGINE", "fused") == "layers":
    from distributed_neural_network_amd.runtime.layer_engine import LayerEngine
    eng = LayerEngine(batch=64, model="lenet-bn", seed=11, device="cuda", graph_chunk=8,
                      use_graphs=os.environ["GRAPHS"] == "1")
else:
    eng = HipEngine(batch=int(os.environ.get("BATCH", "64")), arena=init_arena(seed=11), graph_chunk=8,
                    use_graphs=os.environ["GRAPHS"] == "1", dtype=os.environ.get("DTYPE", "bf16"))
eng.attach(data)
pol = make_policy("step-allreduce", comm)
pol.attach(eng)
pol.initial_broadcast(eng)
samp = EpochSampler.for_rank(len(data), comm.rank, comm.world, seed=1, mode="shard")
for ep in range(2):
    pol.epoch_start(eng, ep)
    eng.begin_epoch(samp.order(ep))
    eng.run_steps(samp.steps(eng.batch))
    eng.synchronize()
    pol.epoch_end(eng, ep)
kind = type(eng.grad_sync).__name__
one = bool(getattr(getattr(eng.grad_sync, "group", None), "one_launch", False))
xp_mode = int(getattr(getattr(eng.grad_sync, "group", None), "xp_mode", -1))
ar_mode = int(getattr(getattr(eng.grad_sync, "group", None), "ar_mode", -1))
path = pol.installed(eng)
torch.save({"master": eng.master.cpu(), "kind": kind, "one_launch": one, "xp_mode": xp_mode, "ar_mode": ar_mode,
            "path": path, "pers": bool(getattr(eng, "_pers_ok", lambda: False)())},
           os.path.join(os.environ["OUT"], f"r{comm.rank}.pt"))
comm.close()
'''


def _two_ranks(tmp_path, allreduce, graphs, port, one_launch="1", nproc=2, exchange="auto", engine="fused",
               persist="0", batch=64, dtype="bf16"):
    out = tmp_path / f"{allreduce}{one_launch}{nproc}{exchange}{engine}{persist}{batch}{graphs}{dtype}"
    out.mkdir()
    env = dict(os.environ, PYTHONPATH=ROOT, DNN_BACKEND="gloo", DNN_ALLREDUCE=allreduce, OMP_NUM_THREADS="2",
               OUT=str(out), GRAPHS=graphs, DNN_XGMI_ONE_LAUNCH=one_launch, DNN_XGMI_EXCHANGE=exchange, ENGINE=engine,
               DNN_PERSIST=persist, DNN_AB_PERS=persist, BATCH=str(batch), DTYPE=dtype)
    script = tmp_path / "w.py"
    script.write_text(_TWO_RANK)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    import torch
    return [torch.load(out / f"r{i}.pt", weights_only=True) for i in range(nproc)], r


def test_xgmi_two_ranks_match_host_allreduce(tmp_path):
    """2 ranks on the box's GPU: the one-launch exchange (reduce + xGMI all-reduce + SGD in
    grad_reduce) keeps the replicas bit-identical, equals the two-launch path bit for bit and
    matches the gloo all-reduce + sgd_apply path."""
    import torch

    xg, r = _two_ranks(tmp_path, "xgmi", "1", 29641)
    assert xg[0]["kind"] == "XgmiGradSync", r.stderr[-2000:]
    assert xg[0]["one_launch"] and xg[1]["one_launch"], r.stderr[-2000:]  # exchange self-test passed
    assert torch.equal(xg[0]["master"], xg[1]["master"])
    # the two-launch path (reduce -> slot, all-reduce kernel) gives the same bits
    two, r2 = _two_ranks(tmp_path, "xgmi", "1", 29645, one_launch="0")
    assert two[0]["kind"] == "XgmiGradSync" and not two[0]["one_launch"], r2.stderr[-2000:]
    assert torch.equal(two[0]["master"], xg[0]["master"]) and torch.equal(two[1]["master"], xg[1]["master"])
    host, _ = _two_ranks(tmp_path, "rccl", "0", 29643)  # DNN_BACKEND=gloo: host all-reduce, eager
    assert host[0]["kind"] == "GradAllReduce"
    assert torch.equal(host[0]["master"], host[1]["master"])
    # same math up to fma contraction: sgd_apply rounds grad * grad_scale separately
    assert torch.allclose(xg[0]["master"], host[0]["master"], rtol=0, atol=1e-6), \
        float((xg[0]["master"] - host[0]["master"]).abs().max())


def test_xgmi_rsag_exchange_two_ranks(tmp_path):
    """2 ranks on the box's GPU: the two-hop pull exchange (owner reads its elements from the
    peers' pull slots, publishes the rank-order sum in its own region, the others read it; the
    default from 4 ranks on distinct GPUs) passes its self-test and gives the one-hop pull
    form's parameters bit for bit, identical on both ranks."""
    import torch

    rs, r = _two_ranks(tmp_path, "xgmi", "1", 29671, exchange="rsag")
    assert all(x["one_launch"] and x["xp_mode"] == 2 and x["ar_mode"] == 2 for x in rs), r.stderr[-2000:]
    pull, r2 = _two_ranks(tmp_path, "xgmi", "1", 29673, exchange="pull")
    assert all(x["one_launch"] and x["xp_mode"] == 0 and x["ar_mode"] == 0 for x in pull), r2.stderr[-2000:]
    # the two-launch path with the all-reduce kernel in its two-hop form
    two, r3 = _two_ranks(tmp_path, "xgmi", "1", 29675, one_launch="0", exchange="rsag")
    assert all(not x["one_launch"] and x["ar_mode"] == 2 for x in two), r3.stderr[-2000:]
    for i in range(2):
        assert torch.equal(rs[i]["master"], rs[0]["master"])
        assert torch.equal(rs[i]["master"], pull[i]["master"])
        assert torch.equal(two[i]["master"], pull[i]["master"])


def test_xgmi_rsag_allreduce_layer_engine_two_ranks(tmp_path):
    """2 ranks of the layer engine (lenet-bn, fp32): the all-reduce kernel's two-hop form keeps
    the replicas identical and equals its one-hop pull form bit for bit."""
    import torch

    rs, r = _two_ranks(tmp_path, "xgmi", "1", 29677, exchange="rsag", engine="layers")
    assert all(x["kind"] == "XgmiGradSync" and x["ar_mode"] == 2 for x in rs), r.stderr[-2000:]
    pull, r2 = _two_ranks(tmp_path, "xgmi", "1", 29679, exchange="pull", engine="layers")
    assert all(x["ar_mode"] == 0 for x in pull), r2.stderr[-2000:]
    for i in range(2):
        assert torch.equal(rs[i]["master"], rs[0]["master"])
        assert torch.equal(rs[i]["master"], pull[i]["master"])


def test_bench_two_ranks_xgmi(tmp_path):
    """bench.py with 2 ranks sharing the GPU: the start-up all-reduce A/B (RCCL refuses two ranks
    on one device, so over gloo the xGMI forms compete), the graph-captured exchange of the winner
    and the in-kernel exchange-wait statistics in the JSON line."""
    env = dict(os.environ, PYTHONPATH=ROOT, DNN_BACKEND="gloo", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29657", os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "200", "--warmup", "20"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    assert out["n_gpus"] == 2 and out["config"]["allreduce"] in ("xgmi-pull", "xgmi-rsag"), out
    ab = out["allreduce_ab"]
    # (the -pers forms are candidates only with DNN_AB_PERS=1: parallel/autotune.py ORDER)
    assert set(ab) == {"xgmi-pull", "xgmi-rsag", "rccl", "rccl-overlap"}, out
    assert out["ab_wall_s"] > 0, out
    assert ab["xgmi-pull"] is not None and ab["rccl"] is None and "rccl" in out["allreduce_failed"], out
    assert out["local_step_us"] > 0, out
    w = out["exchange_wait_us"]
    assert w is not None and 0 <= w["median"] <= w["p99"] <= w["max"], out


def test_xgmi_bf16_granule_exchanges_two_ranks(tmp_path):
    """2 ranks on the box's GPU: the bf16-granule forms of the one-launch exchange (pairs of
    bf16 gradients per {value, step} word, --grad-comm bf16) pass their self-test against the
    all-reduce kernel's bf16 form (a separate implementation with different element pairs) bit
    for bit, keep the replicas identical, and stay within bf16 rounding of the fp32 exchange."""
    import torch

    fp, r0 = _two_ranks(tmp_path, "xgmi", "1", 29681, exchange="pull")
    for port, xch, mode in ((29683, "pull-bf16", 4), (29685, "rsag-bf16", 6)):
        res, r = _two_ranks(tmp_path, "xgmi", "1", port, exchange=xch)
        assert all(x["kind"] == "XgmiGradSync" and x["one_launch"] and x["xp_mode"] == mode for x in res), \
            r.stderr[-2000:]
        assert torch.equal(res[0]["master"], res[1]["master"])
        d = (res[0]["master"] - fp[0]["master"]).abs().max().item()
        assert 0 < d < 1e-4, (xch, d)  # rounded (not the fp32 bits), but only by bf16 gradient rounding


# (fp32 at batch 32: two ranks' fp32 grids, 2 x (63 + B) workgroups, must fit the GPU they share)
@pytest.mark.parametrize("batch,dtype", [(16, "bf16"), (64, "bf16"), (32, "fp32")])
def test_xgmi_exchange_inside_persistent_launch_two_ranks(tmp_path, batch, dtype):
    """2 ranks on the box's GPU, the per-step exchange INSIDE the persistent
    launch (xgmi-pull-pers / xgmi-rsag-pers: the reduction workgroups exchange their elements
    over xGMI after each step's batch reduction, sum in rank order, apply SGD and only then signal
    the samples) - installed after its self-test, engaged, and bit-identical on both ranks to the
    serial one-launch exchange, over 2 epochs with graph replays and eager launches.  fp32 (VERDICT
    r5 next #5): the fp32 kernel's persistent launch with the exchange inside."""
    import torch

    port = 29701 + (batch // 16) * 10 + (40 if dtype == "fp32" else 0)
    ref, r0 = _two_ranks(tmp_path, "xgmi", "1", port, exchange="pull", batch=batch, dtype=dtype)
    assert all(not x["pers"] and x["path"] == "xgmi-pull" for x in ref), r0.stderr[-2000:]
    for k, (xch, graphs) in enumerate((("pull", "1"), ("rsag", "1"), ("pull", "0"))):
        res, r = _two_ranks(tmp_path, "xgmi", graphs, port + 2 + 2 * k, exchange=xch, persist="1", batch=batch,
                            dtype=dtype)
        assert all(x["pers"] and x["path"] == f"xgmi-{xch}-pers" for x in res), (
            [(x["path"], x["pers"]) for x in res], r.stdout[-2000:] + r.stderr[-3000:])
        for i in range(2):
            assert torch.equal(res[i]["master"], ref[i]["master"]), (xch, graphs, i)


def test_xgmi_pers_one_rank_matches_local_sgd():
    """World size 1 with forced collectives: the persistent launch with the exchange inside
    (a 1-rank group: every wait is on this rank's own granules) equals the persistent local step."""
    code = r'''
import numpy as np, torch
from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.parallel import Communicator, make_policy
torch.cuda.set_device(0)
comm = Communicator(device=torch.device("cuda", 0))
data = synthetic(1000, 5)
a = init_arena(seed=9)
res = []
for path in (None, "xgmi-pull-pers", "xgmi-rsag-pers"):
    eng = HipEngine(batch=64, arena=a, graph_chunk=8)
    eng.attach(data)
    pol = make_policy("step-allreduce", comm)
    pol.path = path
    pol.attach(eng)
    if path is None:
        eng.grad_sync = None
    else:
        assert pol.installed(eng) == path, pol.installed(eng)
    eng.begin_epoch(np.arange(1000, dtype=np.int32))
    assert eng._pers_ok()
    eng.run_steps(16)
    torch.cuda.synchronize()
    if path is not None:
        pol.epoch_end(eng, 0)
    res.append((eng.master.cpu(), eng.mom.cpu(), eng.shadow.cpu(), eng.epoch_stats()))
for m, mo, sh, st in res[1:]:
    assert torch.equal(res[0][0], m) and torch.equal(res[0][1], mo) and torch.equal(res[0][2], sh)
    assert st.samples == 1000 and st.loss_sum == res[0][3].loss_sum
comm.close()
print("OK")
'''.replace("torch.cuda.set_device(0)", "from distributed_neural_network_amd.runtime import HipEngine\ntorch.cuda.set_device(0)")
    r = _py(code, {"DNN_FORCE_COLLECTIVES": "1", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29727"})
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
