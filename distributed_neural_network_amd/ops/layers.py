"""Autograd layer ops of the modular engine, backed by csrc/kernels/layers.hip on MI355X.

Every op has two implementations with the SAME semantics:

* on a ROCm device: the hand-written gfx950 kernels (``_dnn_hip``) - Conv2d as
  implicit-GEMM MFMA kernels (conv_igemm.hip), ReLU / pool / BatchNorm / loss / SGD in
  layers.hip - and the library GEMMs (hipBLASLt via ``torch.matmul``) for Linear only;
* on the CPU: plain PyTorch ops - the test double / CPU-only path (never used on a GPU:
  a missing extension there raises instead of silently falling back).

Masking: a captured training step always runs the full batch shape; ``state`` (device
int32, word ST_BVALID) holds how many samples of it are real.  BatchNorm statistics and
the cross-entropy mean exclude the padded tail, exactly like the reference's smaller
last batch (drop_last=False, data_parallelism_train.py:74-79).

Capability parity: the ATen ops of SURVEY.md §2.5 (K1-K20) - conv (fwd, dgrad, wgrad),
ReLU, max-pool (with first-max tie-break), BatchNorm2d (north star), linear,
CrossEntropyLoss (mean), SGD-momentum.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import native

ST_BVALID = 1
# data gradient of a conv with a fused ReLU + max-pool straight from the pooled gradient
# (conv_fwd_packed_unpool); DNN_UNPOOL_DGRAD=0 restores relu_pool_bwd + the plain dgrad
_UNPOOL_DGRAD = os.environ.get("DNN_UNPOOL_DGRAD", "1") != "0"


def _is_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


def _ext():
    return native.hip()


def _s(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t: torch.Tensor) -> int:
    return t.data_ptr()


def _bvalid_cpu(state: torch.Tensor | None, batch: int) -> int:
    return batch if state is None else min(int(state[ST_BVALID]), batch)


def _partials(t: torch.Tensor, B: int, C: int, L: int) -> torch.Tensor:
    """fp64 workspace of the two-stage per-channel reductions (layers.hip)."""
    return torch.empty(C * _ext().chan_parts(B, L) * 2, device=t.device, dtype=torch.float64)


def _workspace(t: torch.Tensor, nbytes: int) -> torch.Tensor:
    """Scratch bytes for a native launch (stream-ordered caching allocator: capture-safe)."""
    return torch.empty(max(int(nbytes), 16), device=t.device, dtype=torch.uint8)


def _gemm(a: torch.Tensor, b: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Library GEMM with optional bf16 operands (fp32 accumulate / result)."""
    if dtype == torch.float32:
        return torch.matmul(a, b)
    return torch.matmul(a.to(dtype), b.to(dtype)).float()


# ---- Conv2d (stride 1, square kernel, zero padding) -------------------------------------------
class Conv2dFn(torch.autograd.Function):
    """On MI355X: implicit-GEMM MFMA kernels (csrc/kernels/conv_igemm.hip) - forward with the
    bias in the epilogue (LDS-patch kernel with packed weights), dgrad as the same kernel
    over dY with flipped weights, wgrad (+ the bias gradient as an all-ones im2col row)
    split over workgroup slices + a fixed-order slice sum; fp32 or bf16 operands
    (converted while staging to LDS).  On the CPU: unfold + matmul (the oracle).

    ``packed``: (forward image, dgrad image) from the engine's once-per-step
    ``conv_pack_all`` launch (either may be None: packed per call).
    ``gw`` / ``gb``: when given, the weight / bias gradients are written straight into
    them (views of the engine's flat gradient arena) and autograd gets None for the
    parameters - no per-parameter accumulation kernels, no arena zeroing.
    ``slice_sink``: a list (GPU, with ``gw``): the backward leaves the weight gradient as split-K
    slice partials and appends (partials, S, Cout, C K^2, gw, gb) for the engine's SGD tail
    launch to sum (one launch fewer per layer); the list keeps the partials alive until then.
    ``pool``: the following ReLU + 2x2 max-pool runs in the forward kernel's epilogue (GPU, packed
    forward image): the op returns the pooled output, and its backward starts with the pool's.
    ``stats``: a ``BnStats`` (GPU, packed forward image): the epilogue also writes the following
    BatchNorm's batch-statistics partials, which ``BatchNormActFn`` then uses instead of its own
    statistics pass."""

    @staticmethod
    def forward(ctx, x, w, b, pad: int, gemm_dtype: torch.dtype, gw=None, gb=None, packed=None, slice_sink=None,
                pool: bool = False, stats: "BnStats | None" = None, bnbwd: "BnBwdStats | None" = None,
                ingest: "IngestSrc | None" = None):
        B, C, H, W = x.shape
        Cout, _, K, _ = w.shape
        OH, OW = H + 2 * pad - K + 1, W + 2 * pad - K + 1
        x = x.contiguous()
        bf = int(gemm_dtype == torch.bfloat16)
        ctx.code = None
        if _is_gpu(x) and ingest is not None:
            # the step's ingest folded into this (first) conv: x is OUTPUT here - the kernel reads
            # the u8 images of the batch ids, stores the normalised input into x and the labels
            assert packed is not None and packed[0] is not None, "ingest conv needs the packed forward image"
            ext = _ext()
            code = part = 0
            if pool:
                y = torch.empty(B, Cout, OH // 2, OW // 2, device=x.device, dtype=torch.float32)
                ctx.code = torch.empty(B, Cout, OH // 2, OW // 2, device=x.device, dtype=torch.uint8)
                code = _p(ctx.code)
            else:
                y = torch.empty(B, Cout, OH, OW, device=x.device, dtype=torch.float32)
                if stats is not None:
                    stats.nparts = ext.conv_fwd_stat_parts(B, C, H, W, Cout, K, pad, bf)
                    stats.part = torch.empty(Cout * stats.nparts * 2, device=x.device, dtype=torch.float64)
                    part = _p(stats.part)
            st = stats.state if stats is not None else None
            ext.conv_fwd_packed_ingest(_p(ingest.images), _p(ingest.ids), _p(ingest.labels), _p(x), _p(ingest.lab_out),
                                       _p(packed[0]), _p(b), _p(y), code, part, _p(st) if st is not None else 0,
                                       B, C, H, W, Cout, K, pad, bf, _s(x))
        elif _is_gpu(x) and pool:
            assert packed is not None and packed[0] is not None, "pooled conv needs the packed forward image"
            y = torch.empty(B, Cout, OH // 2, OW // 2, device=x.device, dtype=torch.float32)
            ctx.code = torch.empty(B, Cout, OH // 2, OW // 2, device=x.device, dtype=torch.uint8)
            _ext().conv_fwd_packed_pool(_p(x), _p(packed[0]), _p(b), _p(y), _p(ctx.code), B, C, H, W, Cout, K, pad, bf,
                                        _s(x))
        elif _is_gpu(x) and stats is not None:
            assert packed is not None and packed[0] is not None, "conv statistics epilogue needs the packed image"
            y = torch.empty(B, Cout, OH, OW, device=x.device, dtype=torch.float32)
            ext = _ext()
            stats.nparts = ext.conv_fwd_stat_parts(B, C, H, W, Cout, K, pad, bf)
            stats.part = torch.empty(Cout * stats.nparts * 2, device=x.device, dtype=torch.float64)
            ext.conv_fwd_packed_stats(_p(x), _p(packed[0]), _p(b), _p(y), _p(stats.part),
                                      _p(stats.state) if stats.state is not None else 0, B, C, H, W, Cout, K, pad, bf,
                                      _s(x))
        elif _is_gpu(x):
            ext = _ext()
            y = torch.empty(B, Cout, OH, OW, device=x.device, dtype=torch.float32)
            if packed is not None and packed[0] is not None:  # image packed by the engine's conv_pack_all
                ext.conv_fwd_packed(_p(x), _p(packed[0]), _p(b), _p(y), B, C, H, W, Cout, K, pad, bf, _s(x))
            else:
                ws = _workspace(x, ext.conv_fwd_workspace(B, C, H, W, Cout, K, pad, bf, 0))
                ext.conv_fwd(_p(x), _p(w), _p(b), _p(y), _p(ws), B, C, H, W, Cout, K, pad, bf, 0, _s(x))
        else:
            cols = F.unfold(x, K, padding=pad)
            y = (_gemm(w.reshape(Cout, -1), cols, gemm_dtype) + b.view(1, Cout, 1)).view(B, Cout, OH, OW)
        ctx.save_for_backward(x, w)
        ctx.shape = (B, C, H, W, K, pad, OH, OW)
        ctx.gemm_dtype = gemm_dtype
        ctx.gw, ctx.gb = gw, gb
        ctx.packed = packed
        ctx.slice_sink = slice_sink if gw is not None else None
        ctx.bnbwd = bnbwd
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        B, C, H, W, K, pad, OH, OW = ctx.shape
        Cout = w.shape[0]
        dy = dy.contiguous()
        pool_code = 0
        bf = int(ctx.gemm_dtype == torch.bfloat16)
        # the fused pool's backward: both gradient kernels unpool dy on their loads when the
        # data gradient runs on the packed LDS-patch path (EPI_UNPOOL); otherwise dy is
        # scattered to the argmax positions once and the dgrad reads the full-size tensor
        unpool_dgrad = (ctx.code is not None and ctx.needs_input_grad[0] and _is_gpu(dy) and _UNPOOL_DGRAD
                        and ctx.packed is not None
                        and ctx.packed[1] is not None and (ctx.bnbwd is None or ctx.bnbwd.z is None)
                        and bool(_ext().conv_fwd_unpool_ok(B, Cout, OH, OW, C, K, K - 1 - pad, bf)))
        if ctx.code is not None and ctx.needs_input_grad[0] and not unpool_dgrad:
            full = torch.empty(B, Cout, OH, OW, device=dy.device, dtype=torch.float32)
            _ext().relu_pool_bwd(_p(dy), _p(ctx.code), B * Cout, OH, OW, _p(full), _s(dy))
            dy = full
        elif ctx.code is not None:  # the weight gradient unpools dy on its loads
            pool_code = _p(ctx.code)
        dw = ctx.gw if ctx.gw is not None else torch.empty_like(w)
        db = ctx.gb if ctx.gb is not None else torch.empty(Cout, device=dy.device, dtype=torch.float32)
        dx = None
        if _is_gpu(dy):
            ext, st = _ext(), _s(dy)
            S = ext.conv_wgrad_slices(B, C, H, W, Cout, K, pad)
            part = torch.empty(S * Cout * (C * K * K + 1), device=dy.device, dtype=torch.float32)
            if ctx.slice_sink is not None:  # partials only: summed by the engine's SGD tail
                ext.conv_wgrad(_p(x), _p(dy), _p(part), 0, 0, B, C, H, W, Cout, K, pad, bf, st, pool_code)
                ctx.slice_sink.append((part, S, Cout, C * K * K, dw, db))
            else:  # dW, db
                ext.conv_wgrad(_p(x), _p(dy), _p(part), _p(dw), _p(db), B, C, H, W, Cout, K, pad, bf, st, pool_code)
            if ctx.needs_input_grad[0]:
                # dgrad: the forward kernel over dY with the flipped, transposed weights
                # (flip=1: packed from w inside the launch), pad' = K - 1 - pad
                dx = torch.empty(B, C, H, W, device=dy.device, dtype=torch.float32)
                h = ctx.bnbwd
                if ctx.packed is not None and ctx.packed[1] is not None and h is not None and h.z is not None:
                    # + the backward statistics of the BatchNorm + ReLU whose output this is
                    h.nparts = ext.conv_fwd_stat_parts(B, Cout, OH, OW, C, K, K - 1 - pad, bf)
                    h.part = torch.empty(C * h.nparts * 2, device=dy.device, dtype=torch.float64)
                    ext.conv_fwd_packed_bnbwd(_p(dy), _p(ctx.packed[1]), _p(dx), _p(h.part),
                                              _p(h.state) if h.state is not None else 0, _p(h.z), _p(h.mean),
                                              _p(h.invstd), _p(h.gamma), _p(h.beta),
                                              _p(h.code) if h.code is not None else 0, h.z.shape[2], h.z.shape[3],
                                              B, Cout, OH, OW, C, K, K - 1 - pad, bf, st)
                elif unpool_dgrad:
                    ext.conv_fwd_packed_unpool(_p(dy), _p(ctx.code), _p(ctx.packed[1]), _p(dx), B, Cout, OH, OW, C, K,
                                               K - 1 - pad, bf, st)
                elif ctx.packed is not None and ctx.packed[1] is not None:
                    ext.conv_fwd_packed(_p(dy), _p(ctx.packed[1]), 0, _p(dx), B, Cout, OH, OW, C, K, K - 1 - pad, bf,
                                        st)
                else:
                    ws = _workspace(dy, ext.conv_fwd_workspace(B, Cout, OH, OW, C, K, K - 1 - pad, bf, 1))
                    ext.conv_fwd(_p(dy), _p(w), 0, _p(dx), _p(ws), B, Cout, OH, OW, C, K, K - 1 - pad, bf, 1, st)
        else:
            cols = F.unfold(x, K, padding=pad)
            dy2 = dy.view(B, Cout, OH * OW)
            torch.sum(_gemm(dy2, cols.transpose(1, 2), ctx.gemm_dtype), 0, out=dw.view(Cout, -1))
            db.copy_(dy2.sum((0, 2)))
            if ctx.needs_input_grad[0]:
                dcols = _gemm(w.reshape(Cout, -1).t(), dy2, ctx.gemm_dtype).contiguous()  # [B, CKK, L]
                dx = F.fold(dcols, (H, W), K, padding=pad)
        if ctx.gw is not None:
            return dx, None, None, None, None, None, None, None, None, None, None, None, None
        return dx, dw, db, None, None, None, None, None, None, None, None, None, None


class IngestSrc:
    """The training step's ingest for the first conv (``Conv2dFn(..., ingest=)``): u8 dataset
    images / labels, the batch's sample ids, and where the labels go."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, ids: torch.Tensor, lab_out: torch.Tensor) -> None:
        self.images, self.labels, self.ids, self.lab_out = images, labels, ids, lab_out


class BnBwdStats:
    """Hand-off of a BatchNorm (+ ReLU) layer's backward statistics (sum dz, sum dz * xhat) from the
    data-gradient epilogue of the conv that consumed its output: ``BatchNormActFn`` fills the
    forward tensors the epilogue needs, ``Conv2dFn.backward`` fills ``part`` / ``nparts``, and the
    BatchNorm backward then skips its own statistics pass."""

    def __init__(self, state: torch.Tensor | None) -> None:
        self.state = state
        self.z = self.mean = self.invstd = self.gamma = self.beta = None
        self.code: torch.Tensor | None = None  # ReLU + max-pool: the pool's argmax codes
        self.part: torch.Tensor | None = None
        self.nparts = 0


class BnStats:
    """Hand-off of a BatchNorm's batch-statistics partials from the conv forward epilogue that
    produced its input (``part``: fp64 [C][nparts][2], filled by the conv) to BatchNormActFn."""

    def __init__(self, state: torch.Tensor | None) -> None:
        self.state = state
        self.part: torch.Tensor | None = None
        self.nparts = 0


# ---- fused ReLU + 2x2 max-pool ---------------------------------------------------------------
class ReluPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        B, C, H, W = x.shape
        OH, OW = H // 2, W // 2
        x = x.contiguous()
        if _is_gpu(x):
            y = torch.empty(B, C, OH, OW, device=x.device, dtype=torch.float32)
            code = torch.empty(B, C, OH, OW, device=x.device, dtype=torch.uint8)
            _ext().relu_pool_fwd(_p(x), B * C, H, W, _p(y), _p(code), _s(x))
        else:
            win = x[:, :, :2 * OH, :2 * OW].reshape(B, C, OH, 2, OW, 2).permute(0, 1, 2, 4, 3, 5)
            win = win.reshape(B, C, OH, OW, 4)
            best, arg = win.max(-1)  # first maximal index (torch tie rule)
            y = best.clamp_min(0.0)
            code = torch.where(best > 0, arg, torch.full_like(arg, 4)).to(torch.uint8)
        ctx.save_for_backward(code)
        ctx.shape = (B, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        (code,) = ctx.saved_tensors
        B, C, H, W = ctx.shape
        dy = dy.contiguous()
        if _is_gpu(dy):
            dx = torch.empty(B, C, H, W, device=dy.device, dtype=torch.float32)
            _ext().relu_pool_bwd(_p(dy), _p(code), B * C, H, W, _p(dx), _s(dy))
            return dx
        OH, OW = H // 2, W // 2
        pos = torch.arange(4).view(1, 1, 1, 1, 4)
        g = torch.where(code.long().unsqueeze(-1) == pos, dy.unsqueeze(-1), torch.zeros(()))
        g = g.view(B, C, OH, OW, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, 2 * OH, 2 * OW)
        dx = torch.zeros(B, C, H, W)
        dx[:, :, :2 * OH, :2 * OW] = g
        return dx


# ---- ReLU -----------------------------------------------------------------------------------
class ReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        if _is_gpu(x):
            y = torch.empty_like(x)
            _ext().relu_fwd(_p(x), x.numel(), _p(y), _s(x))
        else:
            y = x.clamp_min(0.0)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        if _is_gpu(dy):
            dx = torch.empty_like(dy)
            _ext().relu_bwd(_p(dy), _p(y), dy.numel(), _p(dx), _s(dy))
            return dx
        return torch.where(y > 0, dy, torch.zeros(()))


# ---- Linear ---------------------------------------------------------------------------------
# GEMMs up to this many multiply-adds run on the hand-written MFMA kernels (linear.hip); the
# library GEMM only wins on the large ones (cifar-vgg fc1, 64 x 4096 x 256: 7 us vs 17-31 us),
# while it runs the small ones as single-workgroup tiles (lenet fc1 forward: 19 us vs 5-9 us;
# profiles/r2/linear/).  DNN_LINEAR_MFMA_MAX overrides (0: library everywhere).
LINEAR_MFMA_MAX_MACS = int(os.environ.get("DNN_LINEAR_MFMA_MAX", 16 << 20))
# forwards past that size with a long reduction (cifar-vgg's fc1: K = 4096) run as split-K MFMA
# GEMMs + a fixed-order combine (linear.hip) instead of the library GEMM (DNN_LINEAR_SPLITK=0: off)
LINEAR_SPLITK_MIN_K = 2048
LINEAR_SPLITK = os.environ.get("DNN_LINEAR_SPLITK", "1") != "0"


class XentFusion:
    """Request + result of a softmax cross-entropy fused into the last Linear's forward (GPU,
    no ReLU, at most 16 classes, MFMA path): set ``labels`` / ``state`` before the forward;
    afterwards ``out`` is (per-sample loss, per-sample correct, dlogits) exactly as
    ``cross_entropy`` returns them, or None when the layer could not fuse it."""

    def __init__(self, labels: torch.Tensor, state: torch.Tensor | None) -> None:
        self.labels, self.state = labels, state
        self.out = None


class LinearFn(torch.autograd.Function):
    """y = act(x W^T + b), act = ReLU when ``relu`` (the following zoo ReLU fused in).

    GPU: hand-written MFMA kernels (csrc/kernels/linear.hip) for every GEMM of at most
    ``LINEAR_MFMA_MAX_MACS`` multiply-adds: forward with bias + ReLU in the epilogue; backward
    as ONE launch for the data and weight gradients (grid z picks the GEMM), the bias gradient coming out of the
    weight-gradient MFMAs (an all-ones column) and the ReLU mask applied on the operand loads
    (no relu / threshold_backward / sum kernels).  Larger GEMMs use the library GEMM.  fp32
    operands and accumulation in both dtype modes (``gemm_dtype`` only affects the CPU
    oracle path).  CPU: addmm / mm (+ relu).  ``gw`` / ``gb``: gradient arena views written
    in place (see Conv2dFn)."""

    @staticmethod
    def forward(ctx, x, w, b, gemm_dtype: torch.dtype, gw=None, gb=None, relu: bool = False,
                xent: XentFusion | None = None):
        ctx.gemm_dtype = gemm_dtype
        ctx.gw, ctx.gb, ctx.relu = gw, gb, relu
        if _is_gpu(x):
            x = x.contiguous()
            B, K = x.shape
            N = w.shape[0]
            if xent is not None and not relu and N <= 16 and B * K * N <= LINEAR_MFMA_MAX_MACS:
                # logits + softmax cross-entropy (loss, accuracy, dlogits) in one launch
                y = torch.empty(B, N, device=x.device, dtype=torch.float32)
                loss = torch.empty(B, device=x.device, dtype=torch.float32)
                corr = torch.empty(B, device=x.device, dtype=torch.int32)
                dl = torch.empty(B, N, device=x.device, dtype=torch.float32)
                st = _p(xent.state) if xent.state is not None else 0
                _ext().linear_fwd_xent(_p(x), _p(w), _p(b), _p(y), _p(xent.labels), st, _p(loss), _p(corr), _p(dl),
                                       B, K, N, _s(x))
                xent.out = (loss, corr, dl)
            elif B * K * N <= LINEAR_MFMA_MAX_MACS:
                y = torch.empty(B, N, device=x.device, dtype=torch.float32)
                _ext().linear_fwd(_p(x), _p(w), _p(b), _p(y), B, K, N, int(relu), _s(x))
            elif LINEAR_SPLITK and K >= LINEAR_SPLITK_MIN_K:
                ext = _ext()
                S = ext.linear_splitk_splits(B, K, N)
                y = torch.empty(B, N, device=x.device, dtype=torch.float32)
                part = torch.empty(S * B * N, device=x.device, dtype=torch.float32)
                ext.linear_fwd_splitk(_p(x), _p(w), _p(b), _p(y), _p(part), S, B, K, N, int(relu), _s(x))
            else:
                y = torch.addmm(b, x, w.t())
                if relu:
                    y.relu_()
            ctx.save_for_backward(x, w, y if relu else None)
            return y
        if gemm_dtype == torch.float32:
            y = torch.addmm(b, x, w.t())
        else:
            y = _gemm(x, w.t(), gemm_dtype) + b
        if relu:
            y = torch.relu(y)
        ctx.save_for_backward(x, w, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        if _is_gpu(dy):
            dy = dy.contiguous()
            B, K = x.shape
            N = w.shape[0]
            ext, st = _ext(), _s(dy)
            small = B * K * N <= LINEAR_MFMA_MAX_MACS
            gw = ctx.gw if ctx.gw is not None else torch.empty_like(w)
            gb = ctx.gb if ctx.gb is not None else torch.empty(N, device=dy.device, dtype=torch.float32)
            dx = None
            if small:  # data + weight (+ bias) gradients in ONE launch
                ym = _p(y) if y is not None else 0
                if ctx.needs_input_grad[0]:
                    dx = torch.empty(B, K, device=dy.device, dtype=torch.float32)
                ext.linear_bwd(_p(dy), ym, _p(w), _p(x), _p(dx) if dx is not None else 0, _p(gw), _p(gb), B, K, N,
                               st)
            else:
                dz = dy
                if y is not None:  # ReLU mask: one relu_bwd launch (not torch's compare + multiply)
                    dz = torch.empty_like(dy)
                    ext.relu_bwd(_p(dy), _p(y), dy.numel(), _p(dz), st)
                if ctx.needs_input_grad[0]:
                    dx = torch.mm(dz, w)
                torch.mm(dz.t(), x, out=gw)
                torch.sum(dz, 0, out=gb)
            if ctx.gw is not None:
                return dx, None, None, None, None, None, None, None
            return dx, gw, gb, None, None, None, None, None
        if y is not None:
            dy = dy * (y > 0)
        dx = _gemm(dy, w, ctx.gemm_dtype) if ctx.needs_input_grad[0] else None
        if ctx.gw is not None:
            if ctx.gemm_dtype == torch.float32:
                torch.mm(dy.t(), x, out=ctx.gw)
            else:
                ctx.gw.copy_(_gemm(dy.t(), x, ctx.gemm_dtype))
            torch.sum(dy, 0, out=ctx.gb)
            return dx, None, None, None, None, None, None, None
        return dx, _gemm(dy.t(), x, ctx.gemm_dtype), dy.sum(0), None, None, None, None, None


# ---- BatchNorm2d (train: masked batch statistics; eval: running statistics) -----------------
class BatchNorm2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, state, training: bool, eps: float, momentum: float,
                ggamma=None, gbeta=None):
        B, C, H, W = x.shape
        L = H * W
        x = x.contiguous()
        if not training:
            if _is_gpu(x):
                y = torch.empty_like(x)
                _ext().bn_fwd_eval(_p(x), B, C, L, _p(gamma), _p(beta), eps, _p(running_mean), _p(running_var),
                                   _p(y), _s(x))
            else:
                y = (x - running_mean.view(1, C, 1, 1)) * torch.rsqrt(running_var.view(1, C, 1, 1) + eps) \
                    * gamma.view(1, C, 1, 1) + beta.view(1, C, 1, 1)
            ctx.training = False
            return y
        mean = torch.empty(C, device=x.device, dtype=torch.float32)
        invstd = torch.empty(C, device=x.device, dtype=torch.float32)
        if _is_gpu(x):
            y = torch.empty_like(x)
            part = _partials(x, B, C, L)
            _ext().bn_fwd_train(_p(x), B, C, L, _p(state) if state is not None else 0, _p(gamma), _p(beta), eps,
                                momentum, _p(running_mean), _p(running_var), _p(y), _p(mean), _p(invstd), _p(part),
                                _s(x))
        else:
            bv = _bvalid_cpu(state, B)
            xv = x[:bv]
            n = bv * L
            mu = xv.mean((0, 2, 3)) if bv else torch.zeros(C)
            var = ((xv - mu.view(1, C, 1, 1)) ** 2).mean((0, 2, 3)) if bv else torch.zeros(C)
            mean.copy_(mu)
            invstd.copy_(torch.rsqrt(var + eps))
            y = torch.zeros_like(x)
            y[:bv] = (xv - mu.view(1, C, 1, 1)) * invstd.view(1, C, 1, 1) * gamma.view(1, C, 1, 1) \
                + beta.view(1, C, 1, 1)
            if n > 0:
                unb = var * n / (n - 1) if n > 1 else var
                running_mean.mul_(1 - momentum).add_(momentum * mu)
                running_var.mul_(1 - momentum).add_(momentum * unb)
        ctx.training = True
        ctx.gg, ctx.gb = ggamma, gbeta
        ctx.save_for_backward(x, gamma, mean, invstd, state if state is not None else torch.zeros(0))
        return y

    @staticmethod
    def backward(ctx, dy):
        assert ctx.training, "BatchNorm2d backward in eval mode is not supported"
        x, gamma, mean, invstd, state = ctx.saved_tensors
        state = state if state.numel() else None
        B, C, H, W = x.shape
        L = H * W
        dy = dy.contiguous()
        inplace = ctx.gg is not None
        none9 = (None,) * 8
        if _is_gpu(dy):
            dx = torch.empty_like(x)
            dgamma = ctx.gg if inplace else torch.empty(C, device=x.device, dtype=torch.float32)
            dbeta = ctx.gb if inplace else torch.empty(C, device=x.device, dtype=torch.float32)
            _ext().bn_bwd(_p(dy), _p(x), B, C, L, _p(state) if state is not None else 0, _p(gamma), _p(mean),
                          _p(invstd), _p(dx), _p(dgamma), _p(dbeta), _p(_partials(dy, B, C, L)), _s(dy))
            if inplace:
                return (dx, None, None) + none9
            return (dx, dgamma, dbeta) + none9
        bv = _bvalid_cpu(state, B)
        n = bv * L
        xhat = (x[:bv] - mean.view(1, C, 1, 1)) * invstd.view(1, C, 1, 1)
        d = dy[:bv]
        dbeta = d.sum((0, 2, 3))
        dgamma = (d * xhat).sum((0, 2, 3))
        dx = torch.zeros_like(x)
        if n:
            dx[:bv] = gamma.view(1, C, 1, 1) * invstd.view(1, C, 1, 1) * (
                d - dbeta.view(1, C, 1, 1) / n - xhat * dgamma.view(1, C, 1, 1) / n)
        if inplace:
            ctx.gg.copy_(dgamma)
            ctx.gb.copy_(dbeta)
            return (dx, None, None) + none9
        return (dx, dgamma, dbeta) + none9


class BatchNormActFn(torch.autograd.Function):
    """BatchNorm2d (training statistics, tail-masked) fused with the activation after it -
    act 1: ReLU, act 2: ReLU + 2x2 max-pool (2-bit argmax code) - MI355X only.  Forward: the
    statistics pass, then one kernel that normalises AND activates (and pools); backward:
    the ReLU mask is re-derived from x (bit-exact affine recompute) or the pooled gradient
    is routed through the code inside the two BN backward kernels.  Saves the activation
    kernels and one full read + write of the activation per direction (the separate
    ReluFn / ReluPoolFn path is the CPU oracle and the eval path)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, state, eps: float, momentum: float, act: int,
                ggamma=None, gbeta=None, stats: BnStats | None = None, bwd: BnBwdStats | None = None):
        B, C, H, W = x.shape
        x = x.contiguous()
        ext = _ext()
        mean = torch.empty(C, device=x.device, dtype=torch.float32)
        invstd = torch.empty(C, device=x.device, dtype=torch.float32)
        if act == 2:
            y = torch.empty(B, C, H // 2, W // 2, device=x.device, dtype=torch.float32)
            code = torch.empty(B, C, H // 2, W // 2, device=x.device, dtype=torch.uint8)
        else:
            y = torch.empty_like(x)
            code = torch.zeros(0, device=x.device, dtype=torch.uint8)
        if stats is not None and stats.part is not None:  # partials from the conv epilogue
            part, ext_parts = stats.part, stats.nparts
        else:
            part, ext_parts = _partials(x, B, C, H * W), 0
        ext.bn_act_fwd_train(_p(x), B, C, H, W, _p(state) if state is not None else 0, _p(gamma), _p(beta), eps,
                             momentum, _p(running_mean), _p(running_var), _p(y), _p(code) if act == 2 else 0,
                             _p(mean), _p(invstd), _p(part), act, _s(x), ext_parts)
        ctx.act = act
        ctx.gg, ctx.gb = ggamma, gbeta
        ctx.bwd = bwd if act in (1, 2) else None
        if ctx.bwd is not None:  # what the next conv's data-gradient epilogue needs
            bwd.z, bwd.mean, bwd.invstd, bwd.gamma, bwd.beta = x, mean, invstd, gamma, beta
            bwd.code = code if act == 2 else None
        ctx.save_for_backward(x, gamma, beta, mean, invstd, code, state if state is not None else torch.zeros(0))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, mean, invstd, code, state = ctx.saved_tensors
        state = state if state.numel() else None
        B, C, H, W = x.shape
        dy = dy.contiguous()
        inplace = ctx.gg is not None
        dx = torch.empty_like(x)
        dgamma = ctx.gg if inplace else torch.empty(C, device=x.device, dtype=torch.float32)
        dbeta = ctx.gb if inplace else torch.empty(C, device=x.device, dtype=torch.float32)
        h = ctx.bwd
        if h is not None and h.part is not None:  # statistics from the consuming conv's dgrad epilogue
            part, ext_parts = h.part, h.nparts
        else:
            part, ext_parts = _partials(dy, B, C, H * W), 0
        _ext().bn_act_bwd(_p(dy), _p(x), B, C, H, W, _p(state) if state is not None else 0, _p(gamma), _p(beta),
                          _p(mean), _p(invstd), _p(code) if ctx.act == 2 else 0, _p(dx), _p(dgamma), _p(dbeta),
                          _p(part), ctx.act, _s(dy), ext_parts)
        none10 = (None,) * 10
        if inplace:
            return (dx, None, None) + none10
        return (dx, dgamma, dbeta) + none10


# ---- softmax cross-entropy (mean over the valid batch) + accuracy ----------------------------
def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, state: torch.Tensor | None, want_grad: bool = True):
    """Returns (per-sample loss [B], per-sample correct [B] int32, dlogits [B, NC] or None)."""
    B, NC = logits.shape
    logits = logits.contiguous()
    if _is_gpu(logits):
        loss = torch.empty(B, device=logits.device, dtype=torch.float32)
        corr = torch.empty(B, device=logits.device, dtype=torch.int32)
        dl = torch.empty_like(logits) if want_grad else None
        _ext().xent(_p(logits), _p(labels), B, NC, _p(state) if state is not None else 0, _p(loss), _p(corr),
                    _p(dl) if dl is not None else 0, _s(logits))
        return loss, corr, dl
    bv = _bvalid_cpu(state, B)
    lab = labels.long()
    loss = torch.zeros(B)
    corr = torch.zeros(B, dtype=torch.int32)
    z = logits.detach()
    loss[:bv] = F.cross_entropy(z[:bv], lab[:bv], reduction="none")
    corr[:bv] = (z[:bv].argmax(1) == lab[:bv]).int()
    dl = None
    if want_grad:
        dl = torch.zeros_like(z)
        if bv:
            dl[:bv] = (torch.softmax(z[:bv], 1) - F.one_hot(lab[:bv], NC).float()) / bv
    return loss, corr, dl
