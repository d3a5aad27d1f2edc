"""GPU tests of the engine/trainer paths: graphs, RCCL-captured gradient all-reduce, trainer."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.runtime import HipEngine

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _train(eng, data, steps):
    eng.attach(data)
    eng.begin_epoch(np.arange(len(data), dtype=np.int32))
    eng.run_steps(steps)
    torch.cuda.synchronize()
    return eng.master.clone(), eng.epoch_stats()


def test_graphs_are_bitwise_identical_to_eager():
    data = synthetic(1000, 1)  # 16 steps incl. a 40-sample tail batch
    a = init_arena(seed=3)
    m1, s1 = _train(HipEngine(batch=64, arena=a, use_graphs=False), data, 16)
    m2, s2 = _train(HipEngine(batch=64, arena=a, use_graphs=True, graph_chunk=8), data, 16)
    assert torch.equal(m1, m2)
    assert s1.samples == s2.samples == 1000 and s1.batches == 16


@pytest.mark.parametrize("graphs", [True, False])
def test_staged_images_match_batch_id_path(graphs):
    """Image staging (the fused kernel of step c stores step c + 1's images; epoch_begin
    stages step 0) must give the same bits as loading every image through its batch id:
    shuffled epochs, a tail batch, steps past the end of an epoch, a new epoch mid-chunk."""
    data = synthetic(1000, 9)
    a = init_arena(seed=8)
    rng = np.random.default_rng(0)
    orders = [rng.permutation(1000).astype(np.int32) for _ in range(3)]
    res = []
    for stage in (False, True):
        eng = HipEngine(batch=64, arena=a, graph_chunk=8, use_graphs=graphs, stage_images=stage)
        eng.attach(data)
        stats = []
        for ep, order in enumerate(orders):
            eng.begin_epoch(order)
            eng.run_steps(16 + (ep == 1) * 3)  # epoch 1 runs 3 steps past its end (no-ops)
            stats.append(eng.epoch_stats())
        torch.cuda.synchronize()
        assert (eng.stage is not None) == stage
        res.append((eng.master.cpu(), eng.mom.cpu(), stats))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    for s0, s1 in zip(res[0][2], res[1][2]):
        assert s0.loss_sum == s1.loss_sum and s0.correct == s1.correct and s0.samples == s1.samples == 1000


def test_deterministic_run_to_run():
    data = synthetic(512, 2)
    a = init_arena(seed=4)
    m1, _ = _train(HipEngine(batch=64, arena=a), data, 8)
    m2, _ = _train(HipEngine(batch=64, arena=a), data, 8)
    assert torch.equal(m1, m2)  # slab reductions, no float atomics


def _run_py(code, env_extra):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)


def test_rccl_captured_bucketed_allreduce_path():
    """1-rank RCCL group with forced collectives: the graph-captured, overlapped bucket
    all-reduce (+ separate SGD kernel) must reproduce the fused local-SGD step."""
    code = r'''
import numpy as np, torch, os
from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.parallel import Communicator, make_policy
from distributed_neural_network_amd.runtime import HipEngine
torch.cuda.set_device(0)
comm = Communicator(device=torch.device("cuda", 0))
assert comm.distributed
data = synthetic(1000, 5)
a = init_arena(seed=9)
res = []
for sync_on, overlap in [(False, True), (True, True), (True, False)]:
    eng = HipEngine(batch=64, arena=a, graph_chunk=4, overlap=overlap)
    pol = make_policy("step-allreduce", comm)
    pol.attach(eng)
    if not sync_on:
        eng.grad_sync = None
    eng.attach(data); eng.begin_epoch(np.arange(1000, dtype=np.int32)); eng.run_steps(16)
    torch.cuda.synchronize()
    res.append(eng.master.cpu())
print("maxdiff", [float((res[0]-r).abs().max()) for r in res[1:]])
assert all(torch.allclose(res[0], r, atol=1e-6) for r in res[1:])
comm.close()
print("OK")
'''
    r = _run_py(code, {"DNN_FORCE_COLLECTIVES": "1", "DNN_ALLREDUCE": "rccl", "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": "29611"})
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


def test_trainer_data_parallel_on_gpu(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "2",
                        "--batch-size", "64", "--train-samples", "4096", "--test-samples", "1000", "--lr", "0.01",
                        "--save", "ck.pt", "--device", "cuda"], cwd=tmp_path, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Validation loss of updated master model:") == 2
    assert (tmp_path / "log" / "bs64_log_epochs2_proc4_parent.txt").exists()
    from distributed_neural_network_amd.models.network import Network
    net = Network()
    net.load_state_dict(torch.load(tmp_path / "ck.pt", weights_only=True))


@pytest.mark.parametrize("model,dtype", [("lenet", "fp32"), ("lenet-bn", "fp32"), ("cifar-vgg", "bf16")])
def test_trainer_layer_engine_on_gpu(tmp_path, model, dtype):
    """Entry point -> trainer -> LayerEngine on the GPU (zoo models, fp32 / bf16 GEMMs),
    checkpoint loadable by the torch module of the same spec."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "2",
                        "--batch-size", "32", "--train-samples", "1024", "--test-samples", "256", "--lr", "0.01",
                        "--model", model, "--dtype", dtype, "--engine", "layers", "--save", "ck.pt", "--device", "cuda"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Validation loss of updated master model:") == 2
    from distributed_neural_network_amd.models import zoo
    zoo.SpecNet(model).load_state_dict(torch.load(tmp_path / "ck.pt", weights_only=True))


def test_bench_two_ranks_one_gpu_gloo(tmp_path):
    """Multi-rank bench.py plumbing (torchrun, barriers, max over ranks, eval sharding,
    rank-0-only JSON) with 2 ranks sharing the one GPU of the test box over gloo."""
    env = dict(os.environ, PYTHONPATH=ROOT, DNN_BACKEND="gloo", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29677", os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "20", "--warmup", "4", "--no-graphs"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    import json
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 128
    assert out["value"] > 0 and out["steps"] == 20 and 0 <= out["val_acc"] <= 100


@pytest.mark.parametrize("sync", ["step-allreduce", "epoch-avg"])
def test_rank_drop_recovery_on_gpu_engine(tmp_path, sync):
    """Fault recovery with the fused GPU engine: 3 ranks share the box's GPU over gloo,
    rank 1 dies mid-epoch; survivors re-form, restore, re-partition and finish."""
    env = dict(os.environ, PYTHONPATH=ROOT, DNN_BACKEND="gloo", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "distributed_neural_network_amd.parallel.launch", "-n", "3",
                        os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "3", "--batch-size", "32",
                        "--sync", sync, "--drop-rank", "1", "--drop-at-epoch", "1", "--drop-at-step", "2",
                        "--train-samples", "768", "--test-samples", "256", "--device", "cuda", "--save", "ck.pt",
                        "--nb-proc", "3", "--check-sync"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "communicator re-formed (generation 1, 2 ranks)" in r.stdout
    assert r.stdout.count("Validation loss of updated master model:") == 3


@pytest.mark.parametrize("graphs,chunk", [(True, 8), (True, 1), (False, 4), (True, 64)])
def test_pipelined_step_matches_serial_step(graphs, chunk):
    """The pipelined step (launch i = step i - 1's reduction + step i's samples, the samples
    waiting on in-launch ready counters for the weights the reduction writes through) gives the
    serial step's parameters, momentum, bf16 images and epoch statistics BIT FOR BIT: shuffled
    epochs with a tail batch, steps past an epoch's end, chunk graphs of 1 / 8 / 64 steps (odd
    and even launch counts) and eager launches; 3 epochs x 17 steps re-read every weight after
    every hand-off (a stale L1 / L2 line would show as a mismatch), and no wait times out."""
    data = synthetic(1000, 11)  # 15 full batches + a tail of 40
    a = init_arena(seed=5)
    rng = np.random.default_rng(3)
    orders = [rng.permutation(1000).astype(np.int32) for _ in range(3)]
    res = []
    # serial, pipelined (one launch per step), persistent (one launch per chunk, graph replays)
    for pipe, pers in ((False, False), (True, False), (True, True)):
        eng = HipEngine(batch=64, arena=a, graph_chunk=chunk, use_graphs=graphs, pipeline=pipe, persist=pers)
        eng.attach(data)
        stats = []
        for ep, order in enumerate(orders):
            eng.begin_epoch(order)
            if ep == 0:
                assert eng._pipe_ok() == pipe and eng._pers_ok() == pers
            eng.run_steps(5)
            eng.run_steps(12 if ep != 1 else 13)  # epoch 1 runs a step past its end (a no-op)
            stats.append(eng.epoch_stats())
        torch.cuda.synchronize()
        assert not (pipe and eng.pipe_failed()), f"variant pipe={pipe} persist={pers}: a wait timed out"
        res.append((eng.master.cpu(), eng.mom.cpu(), eng.shadow.cpu(), stats, (pipe, pers)))
    m0, mo0, sh0, st0, _ = res[0]
    for m1, mo1, sh1, st1, var in res[1:]:
        assert torch.equal(m0, m1), f"variant {var}: master differs at {int((m0 != m1).sum())} elements"
        assert torch.equal(mo0, mo1) and torch.equal(sh0, sh1), f"variant {var}: momentum / images differ"
        assert [(x.loss_sum, x.samples, x.correct, x.batches) for x in st0] == \
            [(x.loss_sum, x.samples, x.correct, x.batches) for x in st1], f"variant {var}: statistics differ"
        assert all(x.samples == 1000 and x.batches == 16 for x in st1), f"variant {var}: sample counts"


@pytest.mark.parametrize("flags", [1, 2])
def test_persistent_fc1_stream_forms_match_serial(flags):
    """The persistent step's three fc1-stream placements give the same bits: by default wave 0
    streams fc1 during the conv1 wait once the MLP group is ready; DNN_PIPE_FLAGS=2 streams it
    mid-phase B (every wave its part, after the conv2-group poll); =1 after phase B (the late
    path, with the conv2 fragments consumed first)."""
    data = synthetic(1000, 11)
    a = init_arena(seed=5)
    order = np.random.default_rng(3).permutation(1000).astype(np.int32)
    res = []
    for pers, fl in ((False, 0), (True, 0), (True, flags)):
        eng = HipEngine(batch=64, arena=a, graph_chunk=8, pipeline=pers, persist=pers)
        eng.pipe_flags = fl
        eng.attach(data)
        for _ in range(2):
            eng.begin_epoch(order)
            eng.run_steps(16)
        st = eng.epoch_stats()
        torch.cuda.synchronize()
        assert not eng.pipe_failed()
        res.append((eng.master.cpu(), eng.mom.cpu(), eng.shadow.cpu(), st.loss_sum))
    for r in res[1:]:
        assert all(torch.equal(x, y) for x, y in zip(res[0][:3], r[:3])) and res[0][3] == r[3]


@pytest.mark.parametrize("graphs,chunk", [(True, 8), (True, 1), (False, 4), (True, 64)])
def test_fp32_persistent_matches_serial_step(graphs, chunk):
    """The fp32 kernel's persistent launch (lenet_f32.hip PERS: 4 reduction blocks per 1024-thread
    workgroup, write-through fp32 master, sc1 weight loads, rows of two parities) gives the serial
    fp32 step's parameters, momentum, bf16 images and epoch statistics BIT FOR BIT - shuffled
    epochs with a tail batch, a step past an epoch's end, chunk graphs of 1 / 8 / 64 steps and
    eager launches - and no wait times out."""
    data = synthetic(1000, 11)  # 15 full batches + a tail of 40
    a = init_arena(seed=5)
    rng = np.random.default_rng(3)
    orders = [rng.permutation(1000).astype(np.int32) for _ in range(3)]
    res = []
    for pers in (False, True):
        eng = HipEngine(batch=64, arena=a, graph_chunk=chunk, use_graphs=graphs, dtype="fp32", persist=pers)
        assert eng.persist == pers
        eng.attach(data)
        stats = []
        for ep, order in enumerate(orders):
            eng.begin_epoch(order)
            if ep == 0:
                assert eng._pers_ok() == pers
            eng.run_steps(5)
            eng.run_steps(12 if ep != 1 else 13)
            stats.append(eng.epoch_stats())
        torch.cuda.synchronize()
        assert not eng.pipe_failed(), f"persist={pers}: a wait timed out"
        res.append((eng.master.cpu(), eng.mom.cpu(), eng.shadow.cpu(), stats))
    (m0, mo0, sh0, st0), (m1, mo1, sh1, st1) = res
    assert torch.equal(m0, m1), f"master differs at {int((m0 != m1).sum())} elements"
    assert torch.equal(mo0, mo1) and torch.equal(sh0, sh1), "momentum / images differ"
    assert [(x.loss_sum, x.samples, x.correct, x.batches) for x in st0] == \
        [(x.loss_sum, x.samples, x.correct, x.batches) for x in st1], "statistics differ"
    assert all(x.samples == 1000 and x.batches == 16 for x in st1)


def test_pipelined_long_run_under_load():
    """600 pipelined steps next to a second stream of GPU work (uneven load on the CUs the
    hand-off crosses) against the serial step, bit for bit."""
    data = synthetic(4096, 12)
    a = init_arena(seed=6)
    order = np.random.default_rng(4).permutation(4096).astype(np.int32)
    res = []
    for pipe, pers, dt in ((False, False, "bf16"), (True, False, "bf16"), (True, True, "bf16"), (False, False, "fp32"),
                           (False, True, "fp32")):
        eng = HipEngine(batch=64, arena=a, graph_chunk=32, pipeline=pipe, persist=pers, dtype=dt)
        assert eng.persist == pers
        eng.attach(data)
        side = torch.cuda.Stream()
        x = torch.randn(2048, 2048, device="cuda")
        for ep in range(10):
            eng.begin_epoch(order)
            with torch.cuda.stream(side):
                for _ in range(4):
                    x = torch.tanh(x @ x * 1e-3)
            eng.run_steps(60)
        torch.cuda.synchronize()
        assert not eng.pipe_failed()
        res.append((eng.master.cpu(), eng.mom.cpu(), eng.epoch_stats()))
    names = ("bf16 serial", "bf16 pipelined", "bf16 persistent", "fp32 serial", "fp32 persistent")
    for i in (1, 2, 4):  # (bf16 variants against bf16 serial, fp32 persistent against fp32 serial)
        r, r0 = res[i], res[0] if i < 3 else res[3]
        bad = (r0[0] != r[0]).nonzero().flatten()
        assert torch.equal(r0[0], r[0]) and torch.equal(r0[1], r[1]), \
            f"{names[i]}: {bad.numel()} master values differ, first at {bad[:8].tolist()}"
        assert r0[2].loss_sum == r[2].loss_sum, names[i]


def test_fp32_persistent_back_to_back_launches_race_regression():
    """Round 5's fp32 persistent race (profiles/r5/fp32_pers_race): the launch-start bookkeeping
    overwrote the batch ids that late-starting sample workgroups still had to read as their step-0
    ids, so ~1 in 3 back-to-back chunk sequences (run_steps(60) = graphs of 32 + 16 + 8 + 4 steps)
    next to a side stream trained on wrong samples.  15 such runs, each bit for bit against the
    serial fp32 step (before the fix: P(no mismatch) ~ 0.65^15 < 0.2 %)."""
    data = synthetic(4096, 12)
    order = np.random.default_rng(4).permutation(4096).astype(np.int32)

    def run(pers, seed):
        eng = HipEngine(batch=64, arena=init_arena(seed=6), graph_chunk=32, pipeline=False, persist=pers, dtype="fp32")
        assert eng.persist == pers
        eng.attach(data)
        side = torch.cuda.Stream()
        x = torch.randn(2048, 2048, device="cuda", generator=torch.Generator(device="cuda").manual_seed(seed))
        for _ in range(10):
            eng.begin_epoch(order)
            with torch.cuda.stream(side):
                for _ in range(4):
                    x = torch.tanh(x @ x * 1e-3)
            eng.run_steps(60)
        torch.cuda.synchronize()
        assert not eng.pipe_failed()
        return eng.master.cpu(), eng.mom.cpu(), eng.epoch_stats().loss_sum

    ref = run(False, 0)
    for r in range(15):
        got = run(True, r + 1)
        assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1]) and ref[2] == got[2], f"run {r}"
