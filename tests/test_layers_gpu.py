"""Generic layer kernels (csrc/kernels/layers.hip) vs the fp32 PyTorch implementations of
the same ops (ops/layers.py CPU path, itself pinned to torch.nn in test_layers_cpu.py),
and the layer engine on the GPU vs the CPU."""
import numpy as np
import pytest
import torch

from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.ops import layers as L
from distributed_neural_network_amd.runtime import CpuEngine, LayerEngine

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, tol=1e-5):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    err = float((a - b).abs().max() / (b.abs().max() + 1e-12))
    assert err <= tol, f"rel err {err:.2e}"


def _both(fn, *tensors):
    """Run fn on CPU copies and on GPU copies (leaf, requires_grad where floating)."""
    outs = []
    for dev in ("cpu", DEV):
        args = [t.detach().to(dev).requires_grad_(t.is_floating_point() and t.requires_grad) if torch.is_tensor(t)
                else t for t in tensors]
        outs.append((fn(*args), args))
    return outs


@pytest.mark.parametrize("B,C,H,K,pad,Cout", [(3, 3, 32, 5, 0, 6), (4, 6, 14, 5, 0, 16), (2, 8, 9, 3, 1, 5),
                                               (16, 32, 16, 3, 1, 64), (33, 3, 32, 5, 0, 6), (5, 40, 8, 3, 1, 24),
                                               (2, 20, 12, 7, 3, 40)])
def test_conv2d_fwd_bwd(B, C, H, K, pad, Cout):
    """Implicit-GEMM conv (conv_igemm.hip) vs unfold + matmul; the larger shapes run the
    wgrad with many slices (fixed-order slice sum) and partial M / N / K tiles; the 7x7
    layer does not fit the LDS-patch kernel and runs the general gather kernel."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, C, H, H, generator=g).requires_grad_()
    w = torch.randn(Cout, C, K, K, generator=g).requires_grad_()
    b = torch.randn(Cout, generator=g).requires_grad_()
    (yc, ac), (yg, ag) = _both(lambda x, w, b: L.Conv2dFn.apply(x, w, b, pad, torch.float32), x, w, b)
    _close(yg, yc)
    dy = torch.randn(yc.shape, generator=g)
    yc.backward(dy)
    yg.backward(dy.to(DEV))
    for tc, tg in zip(ac, ag):
        _close(tg.grad, tc.grad)


def test_conv_fast_path_covers_zoo_layers():
    """Every zoo conv layer (forward and dgrad, fp32 and bf16) runs on the LDS-patch kernel;
    the 7x7 test layer above does not (it exercises the general kernel)."""
    ext = L._ext()
    for (C, H, K, pad, M) in [(3, 32, 5, 0, 6), (6, 14, 5, 0, 16), (3, 32, 3, 1, 32), (32, 32, 3, 1, 32),
                              (32, 16, 3, 1, 64), (64, 16, 3, 1, 64)]:
        OH = H + 2 * pad - K + 1
        for bf in (0, 1):
            assert ext.conv_fwd_fast(64, C, H, H, M, K, pad, bf) == 1
            assert ext.conv_fwd_fast(64, M, OH, OH, C, K, K - 1 - pad, bf) == 1
    assert ext.conv_fwd_fast(2, 20, 12, 12, 40, 7, 3, 0) == 0


@pytest.mark.parametrize("B,C,H,K,pad,Cout", [(8, 32, 16, 3, 1, 64), (6, 3, 32, 5, 0, 6)])
def test_conv2d_bf16_operands_track_fp32(B, C, H, K, pad, Cout):
    """bf16 MFMA operands (fp32 accumulate): within bf16 rounding of the fp32 oracle."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, C, H, H, generator=g).requires_grad_()
    w = torch.randn(Cout, C, K, K, generator=g).requires_grad_()
    b = torch.randn(Cout, generator=g).requires_grad_()
    yc = L.Conv2dFn.apply(x, w, b, pad, torch.float32)
    xg, wg, bg = (t.detach().to(DEV).requires_grad_() for t in (x, w, b))
    yg = L.Conv2dFn.apply(xg, wg, bg, pad, torch.bfloat16)
    _close(yg, yc, 2e-2)
    dy = torch.randn(yc.shape, generator=g)
    yc.backward(dy)
    yg.backward(dy.to(DEV))
    for tc, tg in zip((x, w, b), (xg, wg, bg)):
        _close(tg.grad, tc.grad, 2e-2)


@pytest.mark.parametrize("B,K,N", [(64, 400, 120), (64, 120, 84), (3, 84, 10), (64, 4096, 256), (17, 130, 33),
                                   (1, 5, 1), (17, 2180, 33)])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("arena", [False, True])
@pytest.mark.parametrize("mfma_max", [None, 0])
def test_linear_mfma_fwd_bwd(B, K, N, relu, arena, mfma_max, monkeypatch):
    """linear.hip (forward + bias + fused ReLU, data gradient, weight gradient with the bias
    gradient from the all-ones column, ReLU mask on the operand loads) vs the fp32 CPU path;
    arena=True writes the parameter gradients into preallocated views (the engine's mode)."""
    if mfma_max is not None:  # 0: past the small-GEMM kernels - split-K forward for K >= 2048, else library
        monkeypatch.setattr(L, "LINEAR_MFMA_MAX_MACS", mfma_max)
    else:  # the MFMA kernels for every size
        monkeypatch.setattr(L, "LINEAR_MFMA_MAX_MACS", 1 << 40)
    torch.manual_seed(B * 131 + K + N)
    x = torch.randn(B, K, requires_grad=True)
    w = torch.randn(N, K, requires_grad=True) / K ** 0.5
    b = torch.randn(N, requires_grad=True)
    g = torch.randn(B, N)
    res = []
    for dev in ("cpu", DEV):
        xx, ww, bb = (t.detach().to(dev).requires_grad_(True) for t in (x, w, b))
        gw = torch.full((N, K), float("nan"), device=dev) if arena else None
        gb = torch.full((N,), float("nan"), device=dev) if arena else None
        y = L.LinearFn.apply(xx, ww, bb, torch.float32, gw, gb, relu)
        y.backward(g.to(dev))
        res.append((y, xx.grad, gw if arena else ww.grad, gb if arena else bb.grad))
    for c, d in zip(res[0], res[1]):
        _close(d, c, 2e-5)


@pytest.mark.parametrize("shape", [(2, 6, 28, 28), (3, 4, 7, 9)])
def test_relu_pool_fwd_bwd(shape):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(shape, generator=g)
    x[0, 0, :2, :2] = 0.5  # ties: first max wins (torch order)
    x = x.requires_grad_()
    (yc, ac), (yg, ag) = _both(L.ReluPoolFn.apply, x)
    _close(yg, yc, 0)
    dy = torch.randn(yc.shape, generator=g)
    yc.backward(dy)
    yg.backward(dy.to(DEV))
    _close(ag[0].grad, ac[0].grad, 0)


def test_relu_fwd_bwd():
    x = torch.randn(5, 37).requires_grad_()
    (yc, ac), (yg, ag) = _both(L.ReluFn.apply, x)
    _close(yg, yc, 0)
    dy = torch.randn(5, 37)
    yc.backward(dy)
    yg.backward(dy.to(DEV))
    _close(ag[0].grad, ac[0].grad, 0)


@pytest.mark.parametrize("bvalid", [6, 4])
def test_batchnorm_train_masked_and_eval(bvalid):
    g = torch.Generator().manual_seed(2)
    B, C = 6, 5
    x = torch.randn(B, C, 7, 7, generator=g).requires_grad_()
    gamma = (torch.rand(C, generator=g) + 0.5).requires_grad_()
    beta = torch.randn(C, generator=g).requires_grad_()
    rm0, rv0 = torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
    outs = []
    for dev in ("cpu", DEV):
        xs, gs, bs = (t.detach().to(dev).requires_grad_() for t in (x, gamma, beta))
        rm, rv = rm0.clone().to(dev), rv0.clone().to(dev)
        st = torch.tensor([0, bvalid, 0, 0], dtype=torch.int32, device=dev)
        y = L.BatchNorm2dFn.apply(xs, gs, bs, rm, rv, st, True, 1e-5, 0.1)
        dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(3)).to(dev)
        y.backward(dy)
        ye = L.BatchNorm2dFn.apply(xs.detach(), gs.detach(), bs.detach(), rm, rv, None, False, 1e-5, 0.1)
        outs.append((y, xs.grad, gs.grad, bs.grad, rm, rv, ye))
    for c, gg in zip(*outs):
        _close(gg, c, 2e-5)
    assert float(outs[1][0][bvalid:].abs().sum()) == 0.0  # padded tail masked out


@pytest.mark.parametrize("act,bvalid,hw", [(1, 6, 7), (2, 6, 8), (2, 4, 7), (1, 3, 6)])
def test_batchnorm_act_fused_matches_composition(act, bvalid, hw):
    """BatchNormActFn (BN + ReLU / ReLU-pool in the BN kernels) == BatchNorm2dFn followed by
    ReluFn / ReluPoolFn (CPU oracle composition), tail-masked, odd sizes (pool floor)."""
    g = torch.Generator().manual_seed(7)
    B, C = 6, 5
    x = torch.randn(B, C, hw, hw, generator=g)
    gamma, beta = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.5
    rm0, rv0 = torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
    outs = []
    for dev in ("cpu", DEV):
        xs, gs, bs = (t.detach().to(dev).requires_grad_() for t in (x, gamma, beta))
        rm, rv = rm0.clone().to(dev), rv0.clone().to(dev)
        st = torch.tensor([0, bvalid, 0, 0], dtype=torch.int32, device=dev)
        if dev == "cpu":
            y = L.BatchNorm2dFn.apply(xs, gs, bs, rm, rv, st, True, 1e-5, 0.1)
            y = L.ReluPoolFn.apply(y) if act == 2 else L.ReluFn.apply(y)
        else:
            y = L.BatchNormActFn.apply(xs, gs, bs, rm, rv, st, 1e-5, 0.1, act)
        dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(3)).to(dev)
        y.backward(dy)
        outs.append((y, xs.grad, gs.grad, bs.grad, rm, rv))
    for c, gg in zip(*outs):
        _close(gg, c, 2e-5)
    assert float(outs[1][0][bvalid:].abs().sum()) == 0.0  # padded tail masked out


def test_cross_entropy_masked():
    g = torch.Generator().manual_seed(4)
    z = torch.randn(9, 10, generator=g)
    y = torch.randint(0, 10, (9,), generator=g, dtype=torch.int32)
    st = torch.tensor([0, 7, 0, 0], dtype=torch.int32)
    c = L.cross_entropy(z, y, st)
    gg = L.cross_entropy(z.to(DEV), y.to(DEV), st.to(DEV))
    for a, b in zip(gg, c):
        _close(a.float(), b.float(), 1e-5)


@pytest.mark.parametrize("B,K,N,bvalid", [(64, 84, 10, 64), (64, 84, 10, 40), (9, 256, 10, 7), (33, 17, 16, 33),
                                          (5, 3, 1, 5)])
def test_linear_fused_cross_entropy(B, K, N, bvalid):
    """linear_fwd_xent (logits + softmax CE + accuracy + dlogits in one launch) vs the CPU
    Linear + cross_entropy oracle; the padded tail (>= bvalid) must come out as zeros, and the
    backward through the same LinearFn must still give the parameter gradients."""
    torch.manual_seed(B * 7 + K + N + bvalid)
    x = torch.randn(B, K)
    w = torch.randn(N, K) / K ** 0.5
    b = torch.randn(N)
    lab = torch.randint(0, N, (B,), dtype=torch.int32)
    x[1] = x[0]  # a repeated row: equal logits
    st = torch.tensor([0, bvalid, 0, 0], dtype=torch.int32)
    zc = L.LinearFn.apply(x, w, b, torch.float32)
    ref = L.cross_entropy(zc, lab, st)
    xg, wg, bg = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    fx = L.XentFusion(lab.to(DEV), st.to(DEV))
    gw, gb = torch.full((N, K), float("nan"), device=DEV), torch.full((N,), float("nan"), device=DEV)
    zg = L.LinearFn.apply(xg, wg, bg, torch.float32, gw, gb, False, fx)
    assert fx.out is not None
    _close(zg, zc, 2e-5)
    loss, corr, dl = fx.out
    _close(loss, ref[0], 2e-5)
    _close(dl, ref[2], 2e-6)
    assert torch.equal(corr.cpu(), ref[1])
    assert float(loss[bvalid:].abs().sum()) == 0.0 and float(dl[bvalid:].abs().sum()) == 0.0
    zg.backward(dl)
    zc2 = L.LinearFn.apply(x.requires_grad_(True), w.requires_grad_(True), b.requires_grad_(True), torch.float32)
    zc2.backward(ref[2])
    _close(xg.grad, x.grad, 2e-5)
    _close(gw, w.grad, 2e-5)
    _close(gb, b.grad, 2e-5)


@pytest.mark.parametrize("model,dtype", [("lenet", "fp32"), ("cifar-vgg", "bf16"), ("lenet-bn", "fp32")])
def test_sgd_tail_refreshes_packed_conv_images(model, dtype):
    """After steps whose conv-weight images come from the SGD tail (no pack launch), the images
    must equal a fresh conv_pack_all of the updated arena bit for bit."""
    data = synthetic(300, 2).to(DEV)
    eng = LayerEngine(batch=32, model=model, device=DEV, gemm_dtype=dtype, use_graphs=True, graph_chunk=4, seed=3)
    eng.attach(data)
    eng.begin_epoch(np.arange(300, dtype=np.int32))
    eng.run_steps(7)
    torch.cuda.synchronize()
    imgs = [(v[0].clone() if v[0] is not None else None, v[1].clone() if v[1] is not None else None)
            for v in eng._packed.values()]
    assert eng._pack_jobs
    eng.ext.conv_pack_all(eng._pack_jobs, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for (f0, d0), (f1, d1) in zip(imgs, eng._packed.values()):
        for a, b in ((f0, f1), (d0, d1)):
            if a is not None:
                assert torch.equal(a, b)
    st = eng.epoch_stats()
    assert st.batches == 7 and st.samples == 7 * 32


@pytest.mark.parametrize("model,dtype", [("lenet", "fp32"), ("cifar-vgg", "bf16")])
def test_deferred_slice_sums_bitwise(model, dtype):
    """Conv weight-gradient slice sums inside the SGD tail launch == slice_sum_kernel + SGD, bit
    for bit (same summation order), over several steps."""
    data = synthetic(200, 6).to(DEV)
    res = []
    for defer in (True, False):
        eng = LayerEngine(batch=32, model=model, device=DEV, gemm_dtype=dtype, graph_chunk=4, seed=8)
        eng.defer_slice_sums = defer
        eng.attach(data)
        eng.begin_epoch(np.arange(200, dtype=np.int32))
        eng.run_steps(6)
        torch.cuda.synchronize()
        res.append((eng.master.cpu(), eng.mom.cpu(), eng.grad.cpu()))
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("model,dtype", [("lenet", "fp32"), ("lenet", "bf16"), ("cifar-vgg", "bf16"),
                                         ("cifar-vgg", "fp32")])
def test_ingest_folded_into_first_conv_bitwise(model, dtype):
    """The first conv reading the u8 images of the batch ids itself (normalising on the load,
    storing the input for its weight gradient, copying the labels) == the ingest kernel + the
    conv on its output, bit for bit over steps with a shuffled order and a tail batch.  (lenet-bn
    has no plan: its 28-wide statistics tiles are not row-aligned.)"""
    data = synthetic(150, 4).to(DEV)
    order = np.random.default_rng(2).permutation(150).astype(np.int32)
    res = []
    for fuse in (True, False):
        eng = LayerEngine(batch=32, model=model, device=DEV, gemm_dtype=dtype, graph_chunk=4, seed=9)
        if fuse:
            assert eng.fuse_ingest, "expected an ingest plan for the first conv"
        eng.fuse_ingest = fuse
        eng.attach(data)
        eng.begin_epoch(order)
        eng.run_steps(5)  # 4 full batches + a 22-sample tail
        torch.cuda.synchronize()
        st = eng.epoch_stats()
        res.append((eng.master.cpu(), eng.mom.cpu(), eng.x.cpu(), eng.labels.cpu(), st.loss_sum, st.correct))
    for a, b in zip(*res):
        assert (a == b) if not isinstance(a, torch.Tensor) else torch.equal(a, b)


@pytest.mark.parametrize("B,C,H,M,K,pad,dtype", [(8, 3, 32, 6, 5, 0, torch.float32), (8, 6, 14, 16, 5, 0, torch.float32),
                                                  (4, 32, 16, 64, 3, 1, torch.bfloat16), (3, 5, 11, 7, 3, 1, torch.float32)])
@pytest.mark.parametrize("xgrad", [True, False])
def test_conv_pooled_epilogue_matches_conv_then_relu_pool(B, C, H, M, K, pad, dtype, xgrad):
    """conv_fwd_packed_pool (ReLU + 2x2 max-pool in the conv epilogue, row-aligned tiles) must equal
    the plain conv kernel followed by relu_pool_fwd bit for bit (same MFMA order per output), codes
    included; the backward through the fused op equals the two-op backward (xgrad=False: the
    weight gradient unpools the pooled dy on its loads, no relu_pool_bwd launch)."""
    ext = L._ext()
    bf = int(dtype == torch.bfloat16)
    OH = H + 2 * pad - K + 1
    if not (ext.conv_fwd_fast(B, C, H, H, M, K, pad, bf) and ext.conv_fwd_pool_ok(B, C, H, H, M, K, pad, bf)):
        pytest.skip("no pooled plan for this shape")
    torch.manual_seed(B + C + H + M)
    x = torch.randn(B, C, H, H, device=DEV)
    w = (torch.randn(M, C, K, K) / (C * K * K) ** 0.5).to(DEV)
    b = torch.randn(M, device=DEV)
    img = torch.empty(ext.conv_fwd_workspace(B, C, H, H, M, K, pad, bf, 0), device=DEV, dtype=torch.uint8)
    ext.conv_pack_all([(w.data_ptr(), img.data_ptr(), B, C, H, H, M, K, pad, bf, 0)], torch.cuda.current_stream().cuda_stream)
    packed = (img, None)
    outs = []
    for fused in (True, False):
        xx = x.clone().requires_grad_(xgrad)
        gw, gb = torch.zeros(M, C, K, K, device=DEV), torch.zeros(M, device=DEV)
        ww = w.clone().requires_grad_(not xgrad)  # autograd needs one input that requires grad
        y = L.Conv2dFn.apply(xx, ww, b, pad, dtype, gw, gb, packed, None, fused)
        if not fused:
            y = L.ReluPoolFn.apply(y)
        dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(5)).to(DEV)
        y.backward(dy)
        outs.append((y.detach(), xx.grad, gw, gb))
    assert outs[0][0].shape == (B, M, OH // 2, OH // 2)
    for a, c in zip(*outs):
        assert (a is None and c is None) or torch.equal(a, c)


@pytest.mark.parametrize("B,Co,OH,Ci,K,pad,dtype", [(8, 16, 10, 6, 5, 0, torch.float32),
                                                   (4, 7, 11, 5, 3, 1, torch.float32),
                                                   (3, 6, 28, 3, 5, 0, torch.float32),
                                                   (4, 16, 10, 6, 5, 0, torch.bfloat16)])
def test_conv_unpool_dgrad_matches_relu_pool_bwd_then_dgrad(B, Co, OH, Ci, K, pad, dtype):
    """The data gradient of a pooled conv read straight from the pooled gradient and its argmax
    codes (EPI_UNPOOL: the patch loads unpool) must equal relu_pool_bwd followed by the plain
    packed dgrad bit for bit - codes 0-3 and 4 (max <= 0), odd sizes (the last row / column of
    an odd map gets no gradient)."""
    ext = L._ext()
    bf = int(dtype == torch.bfloat16)
    pd = K - 1 - pad
    if not ext.conv_fwd_unpool_ok(B, Co, OH, OH, Ci, K, pd, bf):
        pytest.skip("no unpooling plan for this shape")
    torch.manual_seed(B + Co + OH)
    w = (torch.randn(Co, Ci, K, K) / (Ci * K * K) ** 0.5).to(DEV)  # the forward layer's weight
    img = torch.empty(ext.conv_fwd_workspace(B, Co, OH, OH, Ci, K, pd, bf, 1), device=DEV, dtype=torch.uint8)
    st = torch.cuda.current_stream().cuda_stream
    ext.conv_pack_all([(w.data_ptr(), img.data_ptr(), B, Co, OH, OH, Ci, K, pd, bf, 1)], st)
    P = OH // 2
    dp = torch.randn(B, Co, P, P, device=DEV)
    code = torch.randint(0, 5, (B, Co, P, P), device=DEV, dtype=torch.uint8)
    full = torch.empty(B, Co, OH, OH, device=DEV)
    ext.relu_pool_bwd(dp.data_ptr(), code.data_ptr(), B * Co, OH, OH, full.data_ptr(), st)
    H = OH + 2 * pd - K + 1
    ref = torch.full((B, Ci, H, H), float("nan"), device=DEV)
    got = torch.full((B, Ci, H, H), float("nan"), device=DEV)
    ext.conv_fwd_packed(full.data_ptr(), img.data_ptr(), 0, ref.data_ptr(), B, Co, OH, OH, Ci, K, pd, bf, st)
    ext.conv_fwd_packed_unpool(dp.data_ptr(), code.data_ptr(), img.data_ptr(), got.data_ptr(), B, Co, OH, OH, Ci, K,
                               pd, bf, st)
    torch.cuda.synchronize()
    assert torch.equal(ref, got)


def test_pooled_conv_backward_with_unpool_dgrad():
    """Conv2dFn with the fused pool and the packed flipped image (the layer engine's setup):
    backward through the unpooling dgrad + unpooling wgrad equals conv -> ReluPoolFn -> backward
    on the plain packed path, bitwise (dx, dW, db)."""
    ext = L._ext()
    B, C, H, M, K, pad = 8, 6, 14, 16, 5, 0
    OH = H - K + 1
    torch.manual_seed(3)
    x = torch.randn(B, C, H, H, device=DEV)
    w = (torch.randn(M, C, K, K) / (C * K * K) ** 0.5).to(DEV)
    b = torch.randn(M, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    img = torch.empty(ext.conv_fwd_workspace(B, C, H, H, M, K, pad, 0, 0), device=DEV, dtype=torch.uint8)
    imgf = torch.empty(ext.conv_fwd_workspace(B, M, OH, OH, C, K, K - 1 - pad, 0, 1), device=DEV, dtype=torch.uint8)
    ext.conv_pack_all([(w.data_ptr(), img.data_ptr(), B, C, H, H, M, K, pad, 0, 0),
                       (w.data_ptr(), imgf.data_ptr(), B, M, OH, OH, C, K, K - 1 - pad, 0, 1)], st)
    assert ext.conv_fwd_unpool_ok(B, M, OH, OH, C, K, K - 1 - pad, 0)
    outs = []
    for fused in (True, False):
        xx = x.clone().requires_grad_(True)
        gw, gb = torch.zeros(M, C, K, K, device=DEV), torch.zeros(M, device=DEV)
        y = L.Conv2dFn.apply(xx, w, b, pad, torch.float32, gw, gb, (img, imgf), None, fused)
        if not fused:
            y = L.ReluPoolFn.apply(y)
        dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(7)).to(DEV)
        y.backward(dy)
        outs.append((y.detach(), xx.grad, gw, gb))
    for a, c in zip(*outs):
        assert torch.equal(a, c)


@pytest.mark.parametrize("B,C,H,M,K,pad,dtype,act,bvalid", [(8, 3, 32, 16, 3, 1, torch.bfloat16, 1, 8),
                                                          (8, 6, 14, 16, 5, 0, torch.float32, 2, 5),
                                                          (6, 32, 16, 64, 3, 1, torch.bfloat16, 2, 6)])
def test_conv_epilogue_batchnorm_statistics(B, C, H, M, K, pad, dtype, act, bvalid):
    """BatchNorm statistics computed in the conv forward epilogue (fp64 per-tile partials, padded
    tail masked) vs BatchNorm's own statistics pass: same normalised output, running stats and
    backward (different fp64 summation order: close, not bitwise)."""
    ext = L._ext()
    bf = int(dtype == torch.bfloat16)
    if not ext.conv_fwd_fast(B, C, H, H, M, K, pad, bf):
        pytest.skip("not on the LDS-patch path")
    torch.manual_seed(B * 3 + C + M)
    x = torch.randn(B, C, H, H, device=DEV)
    w = (torch.randn(M, C, K, K) / (C * K * K) ** 0.5).to(DEV)
    b = torch.randn(M, device=DEV)
    gamma, beta = torch.rand(M, device=DEV) + 0.5, torch.randn(M, device=DEV)
    st = torch.tensor([0, bvalid, 0, 0], dtype=torch.int32, device=DEV)
    img = torch.empty(ext.conv_fwd_workspace(B, C, H, H, M, K, pad, bf, 0), device=DEV, dtype=torch.uint8)
    ext.conv_pack_all([(w.data_ptr(), img.data_ptr(), B, C, H, H, M, K, pad, bf, 0)], torch.cuda.current_stream().cuda_stream)
    outs = []
    for fused in (True, False):
        xx = x.clone().requires_grad_(True)
        rm, rv = torch.zeros(M, device=DEV), torch.ones(M, device=DEV)
        gw, gb = torch.zeros(M, C, K, K, device=DEV), torch.zeros(M, device=DEV)
        gg, gbb = torch.zeros(M, device=DEV), torch.zeros(M, device=DEV)
        stats = L.BnStats(st) if fused else None
        y = L.Conv2dFn.apply(xx, w, b, pad, dtype, gw, gb, (img, None), None, False, stats)
        if fused:
            assert stats.part is not None and stats.nparts > 0
        z = L.BatchNormActFn.apply(y, gamma, beta, rm, rv, st, 1e-5, 0.1, act, gg, gbb, stats)
        dz = torch.randn(z.shape, generator=torch.Generator().manual_seed(9)).to(DEV)
        z.backward(dz)
        outs.append((z.detach(), rm, rv, xx.grad, gw, gb, gg, gbb))
    for a, c in zip(*outs):
        _close(a, c, 1e-5)


@pytest.mark.parametrize("model,dtype", [("lenet", "fp32"), ("cifar-vgg", "bf16")])
def test_tail_capacity_fallback_bitwise(model, dtype):
    """Past the tail launch's capacities the engine packs every step and keeps the slice-sum
    kernels: same parameters bit for bit as the one-launch tail."""
    data = synthetic(200, 7).to(DEV)
    res = []
    for fallback in (False, True):
        eng = LayerEngine(batch=32, model=model, device=DEV, gemm_dtype=dtype, graph_chunk=4, seed=2)
        if fallback:
            eng._tail_packs = False
        eng.attach(data)
        eng.begin_epoch(np.arange(200, dtype=np.int32))
        eng.run_steps(6)
        torch.cuda.synchronize()
        res.append((eng.master.cpu(), eng.mom.cpu(), eng.epoch_stats().samples))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1]) and res[0][2] == res[1][2]


@pytest.mark.parametrize("dtype,bvalid,act", [(torch.bfloat16, 6, 1), (torch.float32, 4, 1), (torch.bfloat16, 5, 2),
                                             (torch.float32, 6, 2)])
def test_conv_dgrad_epilogue_batchnorm_backward_statistics(dtype, bvalid, act):
    """BatchNorm + ReLU -> conv: the conv's data-gradient epilogue computes the BatchNorm's backward
    statistics (sum dz, sum dz * xhat); the BatchNorm backward with them equals the one with its
    own statistics pass (close: another fp64 summation order)."""
    ext = L._ext()
    B, C, H, M = 6, 32, 16, 64  # BN over C channels (+ ReLU, + 2x2 pool if act 2), then conv C -> M (3x3, pad 1)
    Hc = H // 2 if act == 2 else H  # the conv's input size
    bf = int(dtype == torch.bfloat16)
    torch.manual_seed(11)
    z = torch.randn(B, C, H, H, device=DEV)
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3
    w = (torch.randn(M, C, 3, 3) / (9 * C) ** 0.5).to(DEV)
    b = torch.randn(M, device=DEV)
    st = torch.tensor([0, bvalid, 0, 0], dtype=torch.int32, device=DEV)
    fwd = torch.empty(ext.conv_fwd_workspace(B, C, Hc, Hc, M, 3, 1, bf, 0), device=DEV, dtype=torch.uint8)
    dgr = torch.empty(ext.conv_fwd_workspace(B, M, Hc, Hc, C, 3, 1, bf, 1), device=DEV, dtype=torch.uint8)
    s0 = torch.cuda.current_stream().cuda_stream
    ext.conv_pack_all([(w.data_ptr(), fwd.data_ptr(), B, C, Hc, Hc, M, 3, 1, bf, 0),
                       (w.data_ptr(), dgr.data_ptr(), B, M, Hc, Hc, C, 3, 1, bf, 1)], s0)
    outs = []
    for fused in (True, False):
        zz = z.clone().requires_grad_(True)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        gg, gbb = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        gw, gb = torch.zeros(M, C, 3, 3, device=DEV), torch.zeros(M, device=DEV)
        h = L.BnBwdStats(st) if fused else None
        a = L.BatchNormActFn.apply(zz, gamma, beta, rm, rv, st, 1e-5, 0.1, act, gg, gbb, None, h)
        y = L.Conv2dFn.apply(a, w, b, 1, dtype, gw, gb, (fwd, dgr), None, False, None, h)
        y.backward(torch.randn(y.shape, generator=torch.Generator().manual_seed(3)).to(DEV))
        if fused:
            assert h.part is not None and h.nparts > 0
        outs.append((zz.grad, gg, gbb, gw, gb))
    for x1, x2 in zip(*outs):
        _close(x1, x2, 1e-5)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_bn_backward_statistics_fusion_engine(dtype):
    """cifar-vgg steps with and without the BatchNorm backward statistics in the conv dgrad
    epilogue stay together (close, not bitwise: a different fp64 summation order)."""
    data = synthetic(200, 5).to(DEV)
    res = []
    for fuse in (True, False):
        eng = LayerEngine(batch=32, model="cifar-vgg", device=DEV, gemm_dtype=dtype, graph_chunk=4, seed=6)
        eng.fuse_bn_bwd = fuse
        eng.attach(data)
        eng.begin_epoch(np.arange(200, dtype=np.int32))
        eng.run_steps(5)
        torch.cuda.synchronize()
        res.append(eng.master.cpu())
    _close(res[0], res[1], 1e-4)


def test_ingest_and_sgd_flat():
    data = synthetic(50, 5).to(DEV)
    eng = LayerEngine(batch=8, model="lenet", device=DEV, use_graphs=False)
    eng.attach(data)
    eng.begin_epoch(np.arange(50, dtype=np.int32)[::-1].copy())
    eng._ingest()
    ids = eng.batch_ids.long().cpu()
    # CPU torch = IEEE division, as torchvision's ToTensor on the reference's CPU workers
    # (torch's CUDA scalar division multiplies by the reciprocal instead)
    ref = (data.images.cpu()[ids].float() / 255.0 - 0.5) / 0.5
    assert torch.equal(eng.x.cpu(), ref) and torch.equal(eng.labels.cpu(), data.labels.cpu()[ids].int())
    p, gr, m = torch.randn(1000, device=DEV), torch.randn(1000, device=DEV), torch.randn(1000, device=DEV)
    p0, m0 = p.clone(), m.clone()
    eng.ext.sgd_flat(p.data_ptr(), gr.data_ptr(), m.data_ptr(), 1000, 0.01, 0.9, 1.0,
                     torch.cuda.current_stream().cuda_stream)
    m_ref = 0.9 * m0 + gr
    _close(m, m_ref, 1e-6)
    _close(p, p0 - 0.01 * m_ref, 1e-6)


def _run(eng, data, steps):
    eng.attach(data)
    eng.begin_epoch(np.arange(len(data), dtype=np.int32))
    eng.run_steps(steps)
    return eng


def test_layer_engine_gpu_fp32_matches_cpu_oracle():
    data = synthetic(200, 1)
    a = init_arena(seed=3)
    ref = _run(CpuEngine(batch=16, arena=a), data, 13)
    gpu = _run(LayerEngine(batch=16, arena=a, model="lenet", device=DEV, graph_chunk=4), data, 13)
    _close(gpu.master - a.to(DEV), ref.master - a, 1e-4)
    s1, s2 = ref.epoch_stats(), gpu.epoch_stats()
    assert s1.samples == s2.samples == 200 and abs(s1.loss_sum - s2.loss_sum) < 1e-4


def test_layer_engine_bn_gpu_graphs_match_eager_and_cpu():
    data = synthetic(72, 2)
    e_cpu = _run(LayerEngine(batch=16, model="lenet-bn", seed=5), data, 5)
    e_eag = _run(LayerEngine(batch=16, model="lenet-bn", seed=5, device=DEV, use_graphs=False), data, 5)
    e_gr = _run(LayerEngine(batch=16, model="lenet-bn", seed=5, device=DEV, graph_chunk=2), data, 5)
    assert torch.equal(e_eag.master, e_gr.master) and torch.equal(e_eag.buffers, e_gr.buffers)
    _close(e_gr.master - e_cpu.master.to(DEV) + e_cpu.master.to(DEV), e_cpu.master, 1e-5)
    _close(e_gr.buffers, e_cpu.buffers, 1e-5)
    l1, c1 = e_cpu.evaluate_samples(data, 0, 72)
    l2, c2 = e_gr.evaluate_samples(data, 0, 72)
    _close(l2, l1, 1e-4)


def test_layer_engine_bf16_gemms_track_fp32():
    data = synthetic(256, 6)
    e32 = _run(LayerEngine(batch=32, model="cifar-vgg", seed=7, device=DEV), data, 8)
    e16 = _run(LayerEngine(batch=32, model="cifar-vgg", seed=7, device=DEV, gemm_dtype="bf16"), data, 8)
    s32, s16 = e32.epoch_stats(), e16.epoch_stats()
    assert abs(s32.mean_loss - s16.mean_loss) < 0.05 * abs(s32.mean_loss)
