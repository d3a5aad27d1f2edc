"""Model layout / checkpoint format / data partitioning (CPU)."""
import numpy as np
import pytest
import torch

from distributed_neural_network_amd.data import EpochSampler, shard_bounds, synthetic, write_cifar_bin
from distributed_neural_network_amd.data.datasets import load_cifar10
from distributed_neural_network_amd.models.network import (LAYOUT, PARAM_SHAPES, Network, arena_state_dict,
                                                           init_arena, load_state_dict_into)
from distributed_neural_network_amd.utils import checkpoint


def test_state_dict_keys_shapes_order_match_reference():
    sd = Network().state_dict()
    assert list(sd.keys()) == [k for k, _ in PARAM_SHAPES]
    for k, shape in PARAM_SHAPES:
        assert tuple(sd[k].shape) == shape and sd[k].dtype == torch.float32
    assert LAYOUT.num_params == 62006 == sum(v.numel() for v in sd.values())


def test_arena_layout_alignment_and_buckets():
    for k, off in LAYOUT.offsets.items():
        assert off % 64 == 0
    lo, hi = LAYOUT.conv_range
    assert lo == 0 and hi == LAYOUT.offsets["fc1.weight"]
    assert LAYOUT.mlp_range == (LAYOUT.offsets["fc1.weight"], LAYOUT.total)
    assert int(LAYOUT.pad_mask().sum()) == 62006


def test_arena_roundtrip_and_views_alias():
    a = init_arena(seed=3)
    sd = arena_state_dict(a)
    b = torch.zeros(LAYOUT.total)
    load_state_dict_into(b, sd)
    assert torch.equal(a, b)
    v = LAYOUT.views(a)
    v["fc2.bias"][0] = 123.0
    assert a[LAYOUT.offsets["fc2.bias"]] == 123.0
    # padding stays zero
    assert float(a[~LAYOUT.pad_mask()].abs().sum()) == 0.0


def test_init_arena_is_seeded_and_pytorch_default():
    a, b = init_arena(seed=11), init_arena(seed=11)
    assert torch.equal(a, b)
    w = LAYOUT.views(a)["fc1.weight"]
    bound = 1.0 / np.sqrt(400)  # kaiming_uniform(a=sqrt(5)) bound == 1/sqrt(fan_in)
    assert float(w.abs().max()) <= bound + 1e-6


def test_checkpoint_is_reference_state_dict(tmp_path):
    a = init_arena(seed=5)
    mom = torch.randn(LAYOUT.total)
    p = str(tmp_path / "ck.pt")
    checkpoint.save(p, arena_state_dict(a), mom, epoch=4, seed=5)
    raw = torch.load(p, weights_only=True)           # plain state_dict, nothing else
    assert list(raw.keys()) == [k for k, _ in PARAM_SHAPES]
    net = Network()
    net.load_state_dict(raw)                           # loads into the reference module unmodified
    sd, side = checkpoint.load(p)
    assert side["epoch"] == 4 and torch.equal(side["momentum"], mom)
    assert torch.equal(net.fc1.weight, LAYOUT.views(a)["fc1.weight"])


def test_reference_partition_semantics():
    # data_parallelism_train.py:49-53: ps = len // (size-1); worker r gets [(r-1)ps, r*ps)
    assert shard_bounds(50000, 1, 4, parent=True) == (0, 16666)
    assert shard_bounds(50000, 3, 4, parent=True) == (33332, 49998)
    assert shard_bounds(50000, 0, 4, parent=True) == (0, 0)
    assert shard_bounds(50000, 3, 4) == (37500, 50000)
    with pytest.raises(ValueError):
        shard_bounds(10, 0, 1, parent=True)


def test_epoch_sampler_deterministic_and_reshuffles():
    s = EpochSampler.for_rank(1000, 1, 4, seed=7)
    o0, o0b, o1 = s.order(0), s.order(0), s.order(1)
    assert np.array_equal(o0, o0b) and not np.array_equal(o0, o1)
    assert sorted(o0.tolist()) == list(range(250, 500))
    assert s.steps(64) == 4
    full = EpochSampler.for_rank(100, 2, 4, seed=7, mode="full")
    other = EpochSampler.for_rank(100, 3, 4, seed=7, mode="full")
    assert len(full) == 100 and not np.array_equal(full.order(0), other.order(0))


def test_synthetic_splits_share_classes_but_not_samples():
    tr, te = synthetic(200, 1, True), synthetic(200, 1, False)
    assert tr.images.shape == (200, 3, 32, 32) and tr.images.dtype == torch.uint8
    assert tr.labels.dtype == torch.int32 and int(tr.labels.max()) <= 9
    assert not torch.equal(tr.images, te.images)
    # same class templates: per-class mean images correlate strongly across splits
    k = int(tr.labels[0])
    mt = tr.images[tr.labels == k].float().mean(0)
    me = te.images[te.labels == k].float().mean(0)
    assert torch.corrcoef(torch.stack([mt.flatten(), me.flatten()]))[0, 1] > 0.8


def test_cifar_binary_reader_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    d = tmp_path / "cifar-10-batches-bin"
    imgs = {}
    for i in range(1, 6):
        x = rng.integers(0, 256, (7, 3, 32, 32), dtype=np.uint8)
        y = rng.integers(0, 10, 7)
        write_cifar_bin(d / f"data_batch_{i}.bin", x, y)
        imgs[i] = (x, y)
    xt = rng.integers(0, 256, (5, 3, 32, 32), dtype=np.uint8)
    write_cifar_bin(d / "test_batch.bin", xt, np.arange(5))
    tr = load_cifar10(tmp_path, True)
    te = load_cifar10(tmp_path, False)
    assert len(tr) == 35 and len(te) == 5
    assert np.array_equal(tr.images[7:14].numpy(), imgs[2][0])
    assert np.array_equal(tr.labels[:7].numpy(), imgs[1][1])
    assert np.array_equal(te.images.numpy(), xt)


def test_cli_aliases_from_survey_flag_list():
    from distributed_neural_network_amd.train.config import parse
    assert parse("data-parallel", []).overlap is False
    assert parse("data-parallel", ["--overlap"]).overlap is True
    assert parse("data-parallel", ["--overlap", "--no-overlap"]).overlap is False
    assert parse("data-parallel", ["--emulate-parent"]).sync == "parent"
    c = parse("data-parallel", ["--dtype", "fp32", "--model", "lenet-bn", "--bucket-kb", "64", "--check-sync"])
    assert (c.dtype, c.model, c.bucket_kb, c.check_sync) == ("fp32", "lenet-bn", 64, True)
