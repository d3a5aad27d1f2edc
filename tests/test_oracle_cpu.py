"""The fp32 oracle and the CPU engine against plain PyTorch (nn.Module + optim.SGD)."""
import numpy as np
import torch
import torch.nn.functional as F

from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.models.network import LAYOUT, Network, arena_state_dict, init_arena
from distributed_neural_network_amd.ops import reference
from distributed_neural_network_amd.runtime import CpuEngine, eval_metrics


def test_per_sample_rows_consistent_with_batch_gradient():
    s = synthetic(16, 2)
    a = init_arena(seed=2)
    out = reference.per_sample_outputs(a, s.images[:6], s.labels[:6])
    g, _ = reference.batch_grad(a, s.images[:6], s.labels[:6])
    v = LAYOUT.views(g)
    conv = torch.cat([v[k].flatten() for k in ["conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias"]])
    assert torch.allclose(out["slab"].sum(0), conv, atol=1e-6)
    # fc weight grads from the (z, x) rows
    assert torch.allclose(out["z1"].T @ out["a0"], v["fc1.weight"], atol=1e-6)
    assert torch.allclose(out["z3"][:, :10].T @ out["h2"], v["fc3.weight"], atol=1e-6)
    assert torch.allclose(out["z2"].sum(0), v["fc2.bias"], atol=1e-6)


def test_bf16_emulation_close_to_fp32():
    s = synthetic(8, 4)
    a = init_arena(seed=4)
    r = reference.per_sample_outputs(a, s.images[:4], s.labels[:4])
    e = reference.per_sample_outputs_bf16(a, a, s.images[:4], s.labels[:4])
    assert torch.allclose(r["loss"], e["loss"], rtol=1e-2)


def test_cpu_engine_matches_torch_sgd():
    s = synthetic(256, 6)
    a = init_arena(seed=6)
    net = Network()
    net.load_state_dict(arena_state_dict(a))
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
    eng = CpuEngine(batch=32, lr=0.01, momentum=0.9, arena=a)
    eng.attach(s)
    order = np.arange(256, dtype=np.int32)[::-1].copy()
    eng.begin_epoch(order)
    eng.run_steps(8)
    for i in range(8):
        idx = torch.from_numpy(order[i * 32:(i + 1) * 32].astype(np.int64))
        x = reference.normalize_u8(s.images[idx])
        opt.zero_grad()
        F.cross_entropy(net(x), s.labels[idx].long()).backward()
        opt.step()
    ref = torch.cat([p.detach().flatten() for p in net.state_dict().values()])
    got = torch.cat([v.flatten() for v in eng.state_dict().values()])
    assert torch.allclose(got, ref, atol=1e-6)
    st = eng.epoch_stats()
    assert st.batches == 8 and st.samples == 256


def test_eval_metric_definitions():
    loss = torch.tensor([1.0, 2.0, 3.0, 4.0, 10.0])
    corr = torch.tensor([1, 0, 1, 1, 0])
    vl, acc = eval_metrics(loss, corr, batch_size=2)
    # batches: [1,2] [3,4] [10] -> means 1.5, 3.5, 10 -> mean 5.0 (np.mean of batch means)
    assert abs(vl - 5.0) < 1e-12 and abs(acc - 60.0) < 1e-12


def test_fma_normalisation_matches_totensor_normalize_in_bf16():
    """The fused kernel normalises u8 pixels with ONE fma, fmaf(u, 2/255, -1), instead of
    ToTensor+Normalize ((u/255 - 0.5)/0.5, data_parallelism_train.py:24-27).  The fp32
    values differ in the last bits, but the bf16 MFMA operand must be identical for all
    256 codes (fma = exact product + single rounding, emulated in float64)."""
    import numpy as np
    u = np.arange(256, dtype=np.float32)
    exact = (u / np.float32(255) - np.float32(0.5)) / np.float32(0.5)
    fma = (u.astype(np.float64) * np.float64(np.float32(2.0 / 255.0)) - 1.0).astype(np.float32)
    assert torch.equal(torch.from_numpy(exact).bfloat16(), torch.from_numpy(fma).bfloat16())


def test_masked_oracle_reproduces_fp32_oracle_with_its_own_decisions():
    """ops/reference.per_sample_outputs_masked (the bf16 kernel's mask-aware fp32 oracle) fed
    with the pool argmax codes / ReLU masks of an exact fp32 pass equals per_sample_outputs."""
    import torch.nn.functional as F

    from distributed_neural_network_amd.data import synthetic
    from distributed_neural_network_amd.models.network import init_arena
    from distributed_neural_network_amd.ops import reference as R

    d = synthetic(16, 3)
    a = init_arena(seed=1)
    x, y = R.normalize_u8(d.images[:8]), d.labels[:8]
    p = R.LAYOUT.views(a)

    def codes_of(c, h):
        B, C = c.shape[:2]
        win = F.relu(c).reshape(B, C, h, 2, h, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, h * h, 4)
        mx, idx = win.max(-1)
        return torch.where(mx > 0, idx, torch.full_like(idx, 4)).to(torch.uint8)

    c1 = F.conv2d(x, p["conv1.weight"], p["conv1.bias"])
    c2 = F.conv2d(F.max_pool2d(F.relu(c1), 2, 2), p["conv2.weight"], p["conv2.bias"])
    codes = torch.cat([codes_of(c1, 14).reshape(8, -1), codes_of(c2, 5).reshape(8, -1)], 1)
    assert codes.shape[1] == R.CODES_PER_SAMPLE
    ref = R.per_sample_outputs(a, d.images[:8], y, 8)
    got = R.per_sample_outputs_masked(a, a, d.images[:8], y, codes, ref["h1"] > 0, ref["h2"] > 0, 8)
    for k in ["a0", "h1", "h2", "z1", "z2", "z3", "slab", "loss"]:
        assert float((got[k] - ref[k]).norm() / (ref[k].norm() + 1e-30)) < 1e-5, k
