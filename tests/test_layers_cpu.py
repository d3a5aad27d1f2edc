"""Modular (layer) engine on the CPU: zoo models vs plain PyTorch training.

The CPU implementations of ops/layers.py are the semantics the HIP kernels are tested
against on the GPU (tests/test_layers_gpu.py); here they are pinned to torch.nn modules
(nn.Conv2d / nn.BatchNorm2d in train mode / nn.Linear + CrossEntropyLoss + SGD) and to
the reference-model oracle engine.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.models import zoo
from distributed_neural_network_amd.models.network import Network, init_arena
from distributed_neural_network_amd.runtime import CpuEngine, LayerEngine, make_engine
from distributed_neural_network_amd.utils import checkpoint

from test_distributed_cpu import ROOT, _launch


def _torch_train(net, data, order, batch, steps, lr=0.001, momentum=0.9):
    opt = torch.optim.SGD(net.parameters(), lr=lr, momentum=momentum)
    net.train()
    for s in range(steps):
        idx = torch.from_numpy(order[s * batch:(s + 1) * batch].astype(np.int64))
        x = (data.images[idx].float() / 255 - 0.5) / 0.5
        opt.zero_grad()
        F.cross_entropy(net(x), data.labels[idx].long()).backward()
        opt.step()


def test_layer_engine_lenet_matches_reference_oracle():
    data = synthetic(200, 1)  # 16-sample batches: 12 full + a tail of 8
    a = init_arena(seed=3)
    ref, eng = CpuEngine(batch=16, arena=a), LayerEngine(batch=16, arena=a, model="lenet")
    for e in (ref, eng):
        e.attach(data)
        e.begin_epoch(np.arange(200, dtype=np.int32))
        e.run_steps(13)
    assert float((ref.master - eng.master).abs().max()) < 1e-6
    s1, s2 = ref.epoch_stats(), eng.epoch_stats()
    assert s1.samples == s2.samples == 200 and s1.correct == s2.correct
    assert abs(s1.loss_sum - s2.loss_sum) < 1e-5


@pytest.mark.parametrize("model", ["lenet-bn", "cifar-vgg"])
def test_layer_engine_bn_models_match_torch_modules(model):
    data = synthetic(72, 2)  # batch 16: tail batch of 8 exercises the masked statistics
    torch.manual_seed(0)
    net = zoo.SpecNet(model)
    eng = LayerEngine(batch=16, model=model)
    eng.load_state_dict(net.state_dict())
    order = np.random.default_rng(0).permutation(72).astype(np.int32)
    eng.attach(data)
    eng.begin_epoch(order)
    eng.run_steps(5)
    _torch_train(net, data, order, 16, 5)
    sd, ref = eng.state_dict(), net.state_dict()
    for k, v in ref.items():
        if v.is_floating_point():
            err = float((sd[k] - v).abs().max() / (v.abs().max() + 1e-12))
            assert err < 1e-4, f"{model} {k}: rel err {err:.2e}"
    # eval mode (running statistics) matches too
    net.eval()
    loss, corr = eng.evaluate_samples(data, 0, 40)
    with torch.no_grad():
        logits = net((data.images[:40].float() / 255 - 0.5) / 0.5)
    assert torch.allclose(loss, F.cross_entropy(logits, data.labels[:40].long(), reduction="none"), atol=1e-4)


def test_zoo_checkpoint_round_trip(tmp_path):
    eng = LayerEngine(batch=8, model="lenet-bn", seed=1)
    eng.attach(synthetic(32, 0))
    eng.begin_epoch(np.arange(32, dtype=np.int32))
    eng.run_steps(4)
    p = str(tmp_path / "bn.pt")
    checkpoint.save(p, eng.state_dict(), eng.mom, epoch=0)
    sd, side = checkpoint.load(p, zoo.checkpoint_keys("lenet-bn"))
    net = zoo.SpecNet("lenet-bn")
    net.load_state_dict(sd)  # strict: exactly the torch key set (incl. num_batches_tracked)
    assert int(sd["bn1.num_batches_tracked"]) == 4
    eng2 = LayerEngine(batch=8, model="lenet-bn")
    eng2.load_state_dict(sd)
    assert torch.equal(eng2.master, eng.master) and torch.equal(eng2.buffers, eng.buffers)
    # the lenet layer-engine checkpoint is the reference Network format
    e3 = LayerEngine(batch=8, model="lenet", seed=2)
    Network().load_state_dict(e3.state_dict())


def test_make_engine_selection():
    assert isinstance(make_engine("cpu", 4, 0.001, 0.9), CpuEngine)
    assert isinstance(make_engine("cpu", 4, 0.001, 0.9, model="lenet-bn"), LayerEngine)
    assert isinstance(make_engine("cpu", 4, 0.001, 0.9, engine="layers", dtype="fp32"), LayerEngine)
    with pytest.raises(ValueError):
        make_engine("cpu", 4, 0.001, 0.9, model="lenet-bn", engine="fused")


@pytest.mark.parametrize("sync", ["step-allreduce", "epoch-avg"])
def test_bn_model_data_parallel_check_sync(tmp_path, sync):
    """2 gloo ranks, BatchNorm model, --check-sync: replicas bit-identical after every sync
    (running statistics averaged), checkpoint loads into the torch module."""
    r = _launch(2, [os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "2", "--batch-size", "16",
                    "--model", "lenet-bn", "--sync", sync, "--check-sync", "--train-samples", "96",
                    "--test-samples", "48", "--save", "ck.pt", "--nb-proc", "2"], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Validation loss of updated master model:") == 2
    sd, _ = checkpoint.load(str(tmp_path / "ck.pt"), zoo.checkpoint_keys("lenet-bn"))
    zoo.SpecNet("lenet-bn").load_state_dict(sd)


def test_bucketed_step_allreduce_matches_fused_bucket(tmp_path):
    """--bucket-kb splits the gradient into several all-reduces; with 2 ranks every
    element is still a + b, so the result must equal the single fused bucket bitwise."""
    outs = []
    for bk in ("0", "16"):
        d = tmp_path / f"b{bk}"
        d.mkdir()
        r = _launch(2, [os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", "1", "--batch-size", "16",
                        "--sync", "step-allreduce", "--bucket-kb", bk, "--train-samples", "128",
                        "--test-samples", "32", "--save", "ck.pt", "--nb-proc", "2", "--check-sync"], d)
        assert r.returncode == 0, r.stdout + r.stderr
        outs.append(checkpoint.load(str(d / "ck.pt"))[0])
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k


def test_split_buckets():
    from distributed_neural_network_amd.parallel.comm import split_buckets
    assert split_buckets([(0, 10)], 0) == [(0, 10)]
    assert split_buckets([(0, 10), (10, 13)], 4) == [(0, 4), (4, 8), (8, 10), (10, 13)]


@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("arena", [False, True])
def test_linear_fn_cpu_matches_nn_linear(relu, arena):
    """LinearFn's CPU path (the oracle of linear.hip) with and without the fused ReLU, with
    gradients into arena views or returned, equals nn.Linear (+ F.relu) under autograd."""
    from distributed_neural_network_amd.ops import layers as L

    torch.manual_seed(3)
    lin = torch.nn.Linear(37, 11)
    x = torch.randn(5, 37, requires_grad=True)
    g = torch.randn(5, 11)
    y_ref = lin(x)
    if relu:
        y_ref = F.relu(y_ref)
    y_ref.backward(g)
    x2 = x.detach().clone().requires_grad_(True)
    w2, b2 = lin.weight.detach().clone().requires_grad_(True), lin.bias.detach().clone().requires_grad_(True)
    gw = torch.zeros_like(w2) if arena else None
    gb = torch.zeros_like(b2) if arena else None
    y = L.LinearFn.apply(x2, w2, b2, torch.float32, gw, gb, relu)
    y.backward(g)
    assert torch.allclose(y, y_ref, atol=1e-6)
    assert torch.allclose(x2.grad, x.grad, atol=1e-6)
    assert torch.allclose(gw if arena else w2.grad, lin.weight.grad, atol=1e-6)
    assert torch.allclose(gb if arena else b2.grad, lin.bias.grad, atol=1e-6)
