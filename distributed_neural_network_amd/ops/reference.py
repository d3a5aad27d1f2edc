"""fp32 PyTorch oracle of every quantity the HIP kernels produce.

Used (1) by the numerics tests, which compare each kernel output against the same
quantity computed here in fp32, and (2) by the CPU engine (``CpuEngine``), the
explicit CPU-only execution path ("a pure-PyTorch CPU path
used only as the test oracle and for config #1").

All functions address parameters through views of the flat arena, so the oracle and
the kernels share one parameter layout.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from ..models.network import LAYOUT

SLAB = 2872


def normalize_u8(x: torch.Tensor) -> torch.Tensor:
    """ToTensor + Normalize((.5,.5,.5),(.5,.5,.5)) of data_parallelism_train.py:24-27."""
    return (x.float() / 255.0 - 0.5) / 0.5


def forward(arena: torch.Tensor, x: torch.Tensor, return_acts: bool = False):
    p = LAYOUT.views(arena)
    c1 = F.conv2d(x, p["conv1.weight"], p["conv1.bias"])
    p1 = F.max_pool2d(F.relu(c1), 2, 2)
    c2 = F.conv2d(p1, p["conv2.weight"], p["conv2.bias"])
    p2 = F.max_pool2d(F.relu(c2), 2, 2)
    a0 = p2.flatten(1)
    h1 = F.relu(F.linear(a0, p["fc1.weight"], p["fc1.bias"]))
    h2 = F.relu(F.linear(h1, p["fc2.weight"], p["fc2.bias"]))
    logits = F.linear(h2, p["fc3.weight"], p["fc3.bias"])
    if return_acts:
        return logits, {"a0": a0, "h1": h1, "h2": h2}
    return logits


def per_sample_outputs(arena: torch.Tensor, images_u8: torch.Tensor, labels: torch.Tensor,
                       bvalid: int | None = None) -> Dict[str, torch.Tensor]:
    """Exactly the rows the fused kernel writes for a batch (fp32, CPU).

    ``z3`` includes the 1/bvalid of CrossEntropy(reduction='mean');  ``slab`` is the
    per-sample conv weight/bias gradient [dW1 450 | db1 6 | dW2 2400 | db2 16].
    """
    arena = arena.detach().float().cpu()
    x = normalize_u8(images_u8.cpu())
    y = labels.cpu().long()
    B = x.shape[0]
    bvalid = B if bvalid is None else bvalid
    logits, acts = forward(arena, x, return_acts=True)
    loss = F.cross_entropy(logits, y, reduction="none")
    correct = (logits.argmax(1) == y).int()
    p = LAYOUT.views(arena)
    z3 = (torch.softmax(logits, 1) - F.one_hot(y, 10).float()) / bvalid
    z2 = (z3 @ p["fc3.weight"]) * (acts["h2"] > 0).float()
    z1 = (z2 @ p["fc2.weight"]) * (acts["h1"] > 0).float()
    slabs = torch.zeros(B, SLAB)
    conv_keys = ["conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias"]
    for b in range(B):
        a = arena.clone().requires_grad_(True)
        out = forward(a, x[b:b + 1])
        (F.cross_entropy(out, y[b:b + 1]) / bvalid).backward()
        g = LAYOUT.views(a.grad)
        slabs[b] = torch.cat([g[k].flatten() for k in conv_keys])
    z3p = torch.zeros(B, 16)
    z3p[:, :10] = z3
    return {"a0": acts["a0"], "h1": acts["h1"], "h2": acts["h2"], "z1": z1, "z2": z2, "z3": z3p,
            "slab": slabs, "loss": loss, "correct": correct, "logits": logits}


def batch_grad(arena: torch.Tensor, images_u8: torch.Tensor, labels: torch.Tensor,
               return_correct: bool = False):
    """Flat-arena gradient of mean CrossEntropy over the batch (zeros in padding)."""
    a = arena.detach().float().cpu().clone().requires_grad_(True)
    y = labels.cpu().long()
    logits = forward(a, normalize_u8(images_u8.cpu()))
    loss = F.cross_entropy(logits, y)
    loss.backward()
    if return_correct:
        return a.grad.detach(), float(loss.detach()), int((logits.detach().argmax(1) == y).sum())
    return a.grad.detach(), float(loss.detach())


def sgd_momentum_(params: torch.Tensor, grad: torch.Tensor, mom: torch.Tensor, lr: float, momentum: float) -> None:
    """torch.optim.SGD(lr, momentum, dampening=0) on flat tensors; zero buffer == fresh optimizer."""
    mom.mul_(momentum).add_(grad)
    params.sub_(lr * mom)


def _bf(t: torch.Tensor) -> torch.Tensor:
    return t.bfloat16().float()


def per_sample_outputs_bf16(shadow: torch.Tensor, master: torch.Tensor, images_u8: torch.Tensor,
                            labels: torch.Tensor, bvalid: int | None = None) -> Dict[str, torch.Tensor]:
    """The fused kernel's math with bf16 rounding at exactly the kernel's rounding points.

    Weights come from the bf16 shadow, biases from the fp32 master; every MFMA
    operand is rounded to bf16 (the image, the pooled conv1 output, the MLP inputs
    a0/h1/h2 and deltas dz3/dz2/dz1, dY2 and dY1); accumulators, losses and bias
    gradients are fp32.
    A correct kernel matches this to accumulation-order noise.
    """
    w = LAYOUT.views(shadow.detach().float().cpu())
    bm = LAYOUT.views(master.detach().float().cpu())
    x = _bf(normalize_u8(images_u8.cpu()))
    y = labels.cpu().long()
    B = x.shape[0]
    bvalid = B if bvalid is None else bvalid
    W1, W2 = w["conv1.weight"], w["conv2.weight"]
    c1 = F.conv2d(x, W1, bm["conv1.bias"])
    p1, i1 = F.max_pool2d_with_indices(F.relu(c1), 2, 2)
    p1b = _bf(p1)
    c2 = F.conv2d(p1b, W2, bm["conv2.bias"])
    p2, i2 = F.max_pool2d_with_indices(F.relu(c2), 2, 2)
    a0 = p2.flatten(1)
    # MLP: activations / deltas are bf16 MFMA operands, accumulation fp32
    h1 = F.relu(F.linear(_bf(a0), w["fc1.weight"], bm["fc1.bias"]))
    h2 = F.relu(F.linear(_bf(h1), w["fc2.weight"], bm["fc2.bias"]))
    logits = F.linear(_bf(h2), w["fc3.weight"], bm["fc3.bias"])
    loss = F.cross_entropy(logits, y, reduction="none")
    correct = (logits.argmax(1) == y).int()
    z3 = (torch.softmax(logits, 1) - F.one_hot(y, 10).float()) / bvalid
    z2 = (_bf(z3) @ w["fc3.weight"]) * (h2 > 0).float()
    z1 = (_bf(z2) @ w["fc2.weight"]) * (h1 > 0).float()
    da0 = _bf(z1) @ w["fc1.weight"]
    dp2 = da0.view(B, 16, 5, 5) * (p2 > 0).float()
    dy2 = F.max_unpool2d(dp2, i2, 2, 2, output_size=c2.shape[-2:])
    db2 = dy2.sum((2, 3))
    dy2b = _bf(dy2)
    dW2 = torch.stack([torch.nn.grad.conv2d_weight(p1b[b:b + 1], W2.shape, dy2b[b:b + 1]) for b in range(B)])
    dp1 = torch.nn.grad.conv2d_input(p1.shape, W2, dy2b) * (p1 > 0).float()
    dy1 = F.max_unpool2d(dp1, i1, 2, 2, output_size=c1.shape[-2:])
    db1 = dy1.sum((2, 3))
    dy1b = _bf(dy1)
    dW1 = torch.stack([torch.nn.grad.conv2d_weight(x[b:b + 1], W1.shape, dy1b[b:b + 1]) for b in range(B)])
    slab = torch.cat([dW1.flatten(1), db1, dW2.flatten(1), db2], 1)
    z3p = torch.zeros(B, 16)
    z3p[:, :10] = z3
    codes = torch.cat([_codes_from_pool(p1, i1, 28), _codes_from_pool(p2, i2, 10)], 1)
    return {"a0": a0, "h1": h1, "h2": h2, "z1": z1, "z2": z2, "z3": z3p, "slab": slab, "loss": loss,
            "correct": correct, "logits": logits, "codes": codes}


def _codes_from_pool(pooled: torch.Tensor, idx: torch.Tensor, w: int) -> torch.Tensor:
    """The fused kernel's 2-bit max-pool code of a ReLU + 2x2 max-pool: the pixel dy * 2 + dx the
    max came from, 4 where the pooled value is 0 (every input <= 0: no gradient)."""
    B, C = pooled.shape[:2]
    y, x = idx // w, idx % w
    code = (y % 2) * 2 + (x % 2)
    code = torch.where(pooled > 0, code, torch.full_like(code, 4))
    return code.reshape(B, -1).to(torch.uint8)


CODES_PER_SAMPLE = 6 * 196 + 400  # lenet_fused.hip: CODE1 [6][14*14] | CODE2 [16][5*5]


def _pool_by_code(c: torch.Tensor, code: torch.Tensor, h: int) -> torch.Tensor:
    """ReLU + 2x2 max-pool of ``c`` [B, C, 2h, 2h] with the window decisions ``code`` [B, C, h*h]
    (the pixel index dy * 2 + dx the kernel picked, 4 = max <= 0: output 0, no gradient)."""
    B, C = c.shape[:2]
    win = c.reshape(B, C, h, 2, h, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, h * h, 4)
    idx = code.long().clamp(max=3).unsqueeze(-1)
    return torch.where(code < 4, win.gather(3, idx).squeeze(-1), torch.zeros(()))


def _unpool_by_code(d: torch.Tensor, code: torch.Tensor, h: int) -> torch.Tensor:
    """Route the pooled gradient ``d`` [B, C, h*h] to the chosen pixel of each window."""
    B, C = d.shape[:2]
    out = torch.zeros(B, C, h * h, 4)
    out.scatter_(3, code.long().clamp(max=3).unsqueeze(-1), (d * (code < 4).float()).unsqueeze(-1))
    return out.reshape(B, C, h, h, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, 2 * h, 2 * h)


def per_sample_outputs_masked(weights: torch.Tensor, master: torch.Tensor, images_u8: torch.Tensor,
                              labels: torch.Tensor, codes: torch.Tensor, h1_mask: torch.Tensor,
                              h2_mask: torch.Tensor, bvalid: int | None = None) -> Dict[str, torch.Tensor]:
    """The fp32 oracle (every operand and accumulator fp32, no rounding) evaluated with the
    KERNEL'S OWN decisions: its ReLU + max-pool argmax codes (``codes``, written by the fused
    kernel's diagnostic output) and its fc ReLU masks (h1 > 0, h2 > 0 of its rows).  A near-tie
    that bf16 operands flip then cannot turn a 1e-3 difference into a 15 % one, so the bf16
    kernel can be held to ~1e-2 of fp32 per tensor.  ``weights``: the arena the
    kernel multiplies by (the bf16 shadow as fp32); biases come from ``master``, as in the kernel."""
    w = LAYOUT.views(weights.detach().float().cpu())
    bm = LAYOUT.views(master.detach().float().cpu())
    x = normalize_u8(images_u8.cpu())
    y = labels.cpu().long()
    B = x.shape[0]
    bvalid = B if bvalid is None else bvalid
    codes = codes.cpu()
    code1 = codes[:, :6 * 196].reshape(B, 6, 196)
    code2 = codes[:, 6 * 196:].reshape(B, 16, 25)
    m1, m2 = h1_mask.cpu().float(), h2_mask.cpu().float()
    W1, W2 = w["conv1.weight"], w["conv2.weight"]
    c1 = F.conv2d(x, W1, bm["conv1.bias"])
    p1 = _pool_by_code(c1, code1, 14).reshape(B, 6, 14, 14)
    c2 = F.conv2d(p1, W2, bm["conv2.bias"])
    a0 = _pool_by_code(c2, code2, 5).reshape(B, 400)
    h1 = F.linear(a0, w["fc1.weight"], bm["fc1.bias"]) * m1
    h2 = F.linear(h1, w["fc2.weight"], bm["fc2.bias"]) * m2
    logits = F.linear(h2, w["fc3.weight"], bm["fc3.bias"])
    loss = F.cross_entropy(logits, y, reduction="none")
    z3 = (torch.softmax(logits, 1) - F.one_hot(y, 10).float()) / bvalid
    z2 = (z3 @ w["fc3.weight"]) * m2
    z1 = (z2 @ w["fc2.weight"]) * m1
    da0 = z1 @ w["fc1.weight"]
    dy2 = _unpool_by_code(da0.reshape(B, 16, 25), code2, 5)
    db2 = dy2.sum((2, 3))
    dW2 = torch.stack([torch.nn.grad.conv2d_weight(p1[b:b + 1], W2.shape, dy2[b:b + 1]) for b in range(B)])
    dp1 = torch.nn.grad.conv2d_input(p1.shape, W2, dy2)
    dy1 = _unpool_by_code(dp1.reshape(B, 6, 196), code1, 14)
    db1 = dy1.sum((2, 3))
    dW1 = torch.stack([torch.nn.grad.conv2d_weight(x[b:b + 1], W1.shape, dy1[b:b + 1]) for b in range(B)])
    slab = torch.cat([dW1.flatten(1), db1, dW2.flatten(1), db2], 1)
    z3p = torch.zeros(B, 16)
    z3p[:, :10] = z3
    return {"a0": a0, "h1": h1, "h2": h2, "z1": z1, "z2": z2, "z3": z3p, "slab": slab, "loss": loss,
            "logits": logits}


def reduce_rows(rows: Dict[str, torch.Tensor]) -> torch.Tensor:
    """The batch reduction of per-sample rows into the flat gradient arena (fp64 sums, the kernel's
    grad_reduce contract: fc wgrad = z^T x over the batch, biases and conv slabs = column sums)."""
    g = torch.zeros(LAYOUT.total, dtype=torch.float64)
    v = LAYOUT.views(g)
    r = {k: rows[k].double() for k in ("a0", "h1", "h2", "z1", "z2", "z3", "slab")}
    v["fc1.weight"].copy_(r["z1"].T @ r["a0"])
    v["fc1.bias"].copy_(r["z1"].sum(0))
    v["fc2.weight"].copy_(r["z2"].T @ r["h1"])
    v["fc2.bias"].copy_(r["z2"].sum(0))
    v["fc3.weight"].copy_(r["z3"][:, :10].T @ r["h2"])
    v["fc3.bias"].copy_(r["z3"][:, :10].sum(0))
    sl = r["slab"].sum(0)
    v["conv1.weight"].copy_(sl[0:450].view(6, 3, 5, 5))
    v["conv1.bias"].copy_(sl[450:456])
    v["conv2.weight"].copy_(sl[456:2856].view(16, 6, 5, 5))
    v["conv2.bias"].copy_(sl[2856:2872])
    return g.float()


def train_steps_bf16(master: torch.Tensor, images_u8: torch.Tensor, labels: torch.Tensor, order, batch: int,
                     steps: int, lr: float, momentum: float, mom: torch.Tensor | None = None):
    """``steps`` training steps of the bf16 fused engine, emulated on the CPU: every step runs
    ``per_sample_outputs_bf16`` on the bf16 images of the current fp32 master (the shadow the
    optimizer packs), reduces the rows over the batch, and applies momentum SGD in fp32 exactly as
    the kernel does (m = fma(momentum, m, g); p = fma(-lr, m, p)).  Returns (master, momentum,
    per-step mean losses).  The kernel matches it to accumulation-order noise, step after step."""
    p = master.detach().float().cpu().clone()
    m = torch.zeros_like(p) if mom is None else mom.detach().float().cpu().clone()
    order = torch.as_tensor(order, dtype=torch.int64)
    losses = []
    mask = LAYOUT.pad_mask().float()
    for s in range(steps):
        idx = order[s * batch:(s + 1) * batch]
        if idx.numel() == 0:
            break
        n = int(idx.numel())
        rows = per_sample_outputs_bf16(p.bfloat16(), p, images_u8[idx], labels[idx], n)
        g = reduce_rows(rows) * mask
        # fp32 fma, as sgd_update: rounding once per operation pair like the kernel's fmaf
        m = (momentum * m.double() + g.double()).float()
        p = (-lr * m.double() + p.double()).float()
        losses.append(float(rows["loss"].double().mean()))
    return p, m, losses


def decisions_fp32(weights: torch.Tensor, master: torch.Tensor, images_u8: torch.Tensor) -> Dict[str, torch.Tensor]:
    """The plain fp32 forward's OWN decisions (no rounding anywhere): the ReLU + max-pool codes of
    both convolutions (``_codes_from_pool``, the kernel's code format) and the fc ReLU masks."""
    w = LAYOUT.views(weights.detach().float().cpu())
    bm = LAYOUT.views(master.detach().float().cpu())
    x = normalize_u8(images_u8.cpu())
    c1 = F.conv2d(x, w["conv1.weight"], bm["conv1.bias"])
    p1, i1 = F.max_pool2d_with_indices(F.relu(c1), 2, 2)
    c2 = F.conv2d(p1, w["conv2.weight"], bm["conv2.bias"])
    p2, i2 = F.max_pool2d_with_indices(F.relu(c2), 2, 2)
    h1 = F.relu(F.linear(p2.flatten(1), w["fc1.weight"], bm["fc1.bias"]))
    h2 = F.relu(F.linear(h1, w["fc2.weight"], bm["fc2.bias"]))
    return {"codes": torch.cat([_codes_from_pool(p1, i1, 28), _codes_from_pool(p2, i2, 10)], 1),
            "h1": h1 > 0, "h2": h2 > 0}


def decision_flips(a: Dict[str, torch.Tensor], b: Dict[str, torch.Tensor]) -> tuple[int, int, torch.Tensor]:
    """(decisions that differ, decisions compared, per-sample count of differing decisions) between
    two decision sets (``decisions_fp32`` / the bf16 emulation's codes + fc masks)."""
    per = ((a["codes"] != b["codes"]).sum(1) + (a["h1"] != b["h1"]).sum(1) + (a["h2"] != b["h2"]).sum(1))
    total = a["codes"].shape[1] + a["h1"].shape[1] + a["h2"].shape[1]
    return int(per.sum()), total * int(per.numel()), per


def train_steps_fp32_masked(master: torch.Tensor, images_u8: torch.Tensor, labels: torch.Tensor, order, batch: int,
                            steps: int, lr: float, momentum: float, flips: list | None = None):
    """The fp32 reference arithmetic over ``steps`` steps, MASK-AWARE: every step's ReLU / max-pool
    decisions are those of the bf16 trajectory (``train_steps_bf16``, run alongside from the same
    start), every operand and accumulator stays fp32 (``per_sample_outputs_masked`` on the fp32
    master).  A near-tie that bf16 operands flip then cannot turn rounding noise into an O(1)
    change of one sample's gradient, so the bf16 kernel's trajectory can be held to bf16 precision
    of fp32 (~1e-2).  Returns (fp32 master, momentum, per-step mean losses).

    ``flips`` (optional list): per step, how often the plain fp32 forward's OWN decisions on this
    trajectory's parameters differ from the bf16 trajectory's (the kernel's) - (decisions flipped,
    decisions compared, samples with a flip, samples): the steps' mask-aware gradients equal the
    plain fp32 ones on every sample without a flip, so the pair (flip counts, mask-aware error)
    bounds the plain fp32 comparison."""
    pe = master.detach().float().cpu().clone()
    p32 = pe.clone()
    me, m32 = torch.zeros_like(pe), torch.zeros_like(pe)
    order = torch.as_tensor(order, dtype=torch.int64)
    mask = LAYOUT.pad_mask().float()
    losses = []
    for s in range(steps):
        idx = order[s * batch:(s + 1) * batch]
        if idx.numel() == 0:
            break
        n = int(idx.numel())
        emu = per_sample_outputs_bf16(pe.bfloat16(), pe, images_u8[idx], labels[idx], n)
        f32 = per_sample_outputs_masked(p32, p32, images_u8[idx], labels[idx], emu["codes"], emu["h1"] > 0,
                                        emu["h2"] > 0, n)
        if flips is not None:
            own = decisions_fp32(p32, p32, images_u8[idx])
            d, tot, per = decision_flips(own, {"codes": emu["codes"], "h1": emu["h1"] > 0, "h2": emu["h2"] > 0})
            flips.append((d, tot, int((per > 0).sum()), n))
        for p, m, rows in ((pe, me, emu), (p32, m32, f32)):
            g = reduce_rows(rows) * mask
            m.copy_((momentum * m.double() + g.double()).float())
            p.copy_((-lr * m.double() + p.double()).float())
        losses.append(float(f32["loss"].double().mean()))
    return p32, m32, losses
