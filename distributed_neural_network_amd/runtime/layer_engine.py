"""Modular engine: any zoo model (models/zoo.py) on the generic layer kernels.

Same interface as ``HipEngine`` (attach / begin_epoch / run_steps / epoch_stats /
evaluate_samples / master / grad / mom / grad_sync), so the trainer, every sync policy,
fault recovery and checkpointing work unchanged.  Where the fused engine is one
hand-scheduled kernel for the reference LeNet in bf16, this engine runs a layer stack
(csrc/kernels/conv_igemm.hip, linear.hip, layers.hip; the library GEMM only for Linears
above 16M multiply-adds) in fp32 - the reference's arithmetic class - or with bf16
convolution operands, and supports BatchNorm.

The step is launch-bound (a dependent kernel boundary costs ~1.65 us), so producers absorb
their consumers where the data allows: ReLU + max-pool and BatchNorm statistics in the conv
forward epilogue, the loss in the last Linear, both Linear gradients in one launch, and one
tail launch for the conv slice sums, SGD, the next step's packed conv weights and the
bookkeeping (profiles/r2/layer_fusion/).

MI355X design points kept from the fused engine:
  * flat fp32 parameter / gradient / momentum arenas; every layer op writes its parameter
    gradients straight into views of the gradient arena (no per-parameter accumulation
    kernels), so a per-step all-reduce is one collective on one buffer and SGD is one
    kernel;
  * BatchNorm running statistics live in a second flat arena (averaged across ranks at
    the epoch sync);
  * the step cursor, tail-batch size, next batch ids and epoch loss/accuracy live on the
    device (the fused engine's bookkeeping kernel), so a whole step - ingest, forward,
    loss, backward, all-reduce, SGD - is captured in a hipGraph and replays with no host
    work; the tail batch runs at full shape with the padding masked out of BatchNorm
    statistics and the loss mean.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..data.datasets import Split
from ..models import zoo
from ..ops import layers as L
from ..ops import native
from .engine import Engine, StepStats


TAIL_MAX_PACKS = 16   # PackScatter::kMax
TAIL_MAX_SLICES = 8   # SliceSet::kMax


class LayerEngine(Engine):
    def __init__(self, batch: int, lr: float = 0.001, momentum: float = 0.9, model: str = "lenet",
                 arena: torch.Tensor | None = None, seed: int | None = None, device: str | torch.device = "cpu",
                 gemm_dtype: str = "fp32", use_graphs: bool = True, graph_chunk: int = 8,
                 buffers: torch.Tensor | None = None) -> None:
        self.model = model
        self.spec = zoo.spec(model)
        p0, b0 = zoo.init_arenas(model, seed)
        super().__init__(batch, lr, momentum, arena if arena is not None else p0, seed)
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.gpu = self.device.type == "cuda"
        if self.gpu:
            self.ext = native.hip()  # fails loudly if the extension is missing on a GPU host
        self.gemm_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[gemm_dtype]
        self.play, self.blay = zoo.layouts(model)
        dev = self.device
        self.master = self._init_arena.to(dev, torch.float32).clone()
        self.grad = torch.zeros_like(self.master)
        self.mom = torch.zeros_like(self.master)
        self.buffers = (buffers if buffers is not None else b0).to(dev, torch.float32).clone()
        self.num_batches_tracked = 0
        self.P = self.play.views(self.master)
        self.G = self.play.views(self.grad)
        self.Bf = self.blay.views(self.buffers)
        for v in self.P.values():
            v.requires_grad_(True)  # builds the autograd graph; gradients land in G directly
        B = self.batch
        self.state = torch.zeros(4, device=dev, dtype=torch.int32)
        self.stats = torch.zeros(4, device=dev, dtype=torch.float64)
        self.batch_ids = torch.zeros(B, device=dev, dtype=torch.int32)
        self.order = torch.zeros(0, device=dev, dtype=torch.int32)
        self.x = torch.zeros(B, 3, 32, 32, device=dev)
        self.labels = torch.zeros(B, device=dev, dtype=torch.int32)
        self.use_graphs = use_graphs and self.gpu
        self.graph_chunk = 1 << max(0, int(graph_chunk).bit_length() - 1)
        self._graphs: dict[tuple, torch.cuda.CUDAGraph] = {}
        self._warm = False
        self._packed: dict[str, tuple] = {}
        self._pack_jobs: list[tuple] = []
        self._pool_ok: set[str] = set()  # conv layers with a pooled-epilogue plan
        self.defer_slice_sums = True  # conv wgrad slice sums inside the SGD tail (single GPU)
        self._tail_packs = True       # the SGD tail refreshes the packed conv-weight images
        self.fuse_bn_bwd = True       # BatchNorm + ReLU backward statistics in the next conv's dgrad
        # the step's ingest folded into the first conv's loads (DNN_FUSE_INGEST=0: ingest kernel)
        self.fuse_ingest = False
        if self.gpu:
            self._plan_weight_packing()
        # capacities of the one-launch step tail (csrc/kernels/launchers.h PackScatter / SliceSet):
        # past them the tail leaves that part to the separate kernels
        n_conv = sum(isinstance(layer, zoo.Conv) for layer in self.spec)
        self._tail_packs = len(self._pack_jobs) <= TAIL_MAX_PACKS
        self.defer_slice_sums = n_conv <= TAIL_MAX_SLICES

    def _plan_weight_packing(self) -> None:
        """Persistent packed weight images of every LDS-patch convolution (forward and, except
        for the input layer, dgrad), refreshed by ONE conv_pack_all launch per forward instead
        of a pack kernel inside each convolution (7 launches per cifar-vgg step).  The images
        do not depend on the batch size, so the eval forward uses them too."""
        ext, B = self.ext, self.batch
        bf = int(self.gemm_dtype == torch.bfloat16)
        H = W = 32
        first = True
        for layer in self.spec:
            if isinstance(layer, zoo.Conv):
                n, C, M, K, pad = layer.name, layer.cin, layer.cout, layer.k, layer.pad
                OH, OW = H + 2 * pad - K + 1, W + 2 * pad - K + 1
                w = self.P[f"{n}.weight"].data_ptr()
                fwd = dgr = None
                if ext.conv_fwd_fast(B, C, H, W, M, K, pad, bf):
                    fwd = torch.empty(ext.conv_fwd_workspace(B, C, H, W, M, K, pad, bf, 0), device=self.device,
                                      dtype=torch.uint8)
                    self._pack_jobs.append((w, fwd.data_ptr(), B, C, H, W, M, K, pad, bf, 0))
                if not first and ext.conv_fwd_fast(B, M, OH, OW, C, K, K - 1 - pad, bf):
                    dgr = torch.empty(ext.conv_fwd_workspace(B, M, OH, OW, C, K, K - 1 - pad, bf, 1),
                                      device=self.device, dtype=torch.uint8)
                    self._pack_jobs.append((w, dgr.data_ptr(), B, M, OH, OW, C, K, K - 1 - pad, bf, 1))
                self._packed[n] = (fwd, dgr)
                if fwd is not None and ext.conv_fwd_pool_ok(B, C, H, W, M, K, pad, bf):
                    self._pool_ok.add(n)
                if first and fwd is not None and self.spec[0] is layer:
                    # the epilogue forward() will pick for this layer in training
                    i = self.spec.index(layer)
                    nxt = self.spec[i + 1] if i + 1 < len(self.spec) else None
                    nn2 = self.spec[i + 2] if i + 2 < len(self.spec) else None
                    epi = (1 if isinstance(nxt, zoo.ReluPool) and n in self._pool_ok else
                           2 if isinstance(nxt, zoo.BN) and isinstance(nn2, (zoo.Relu, zoo.ReluPool)) else 0)
                    self.fuse_ingest = (os.environ.get("DNN_FUSE_INGEST", "1") != "0" and C == 3 and H == W == 32
                                        and bool(ext.conv_fwd_ingest_ok(B, C, H, W, M, K, pad, bf, epi)))
                first = False
                H, W = OH, OW
            elif isinstance(layer, zoo.ReluPool):
                H, W = H // 2, W // 2

    # -- parameters / checkpoints ------------------------------------------------------------
    def state_dict(self):
        return zoo.state_dict_from_arenas(self.model, self.master, self.buffers, self.num_batches_tracked)

    def load_state_dict(self, sd) -> None:
        p, b = zoo.arenas_from_state_dict(self.model, sd)
        with torch.no_grad():
            self.master.copy_(p.to(self.device))
            self.buffers.copy_(b.to(self.device))
        k = next((key for key in sd if key.endswith("num_batches_tracked")), None)
        if k is not None:
            self.num_batches_tracked = int(sd[k])

    def checkpoint_keys(self):
        return zoo.checkpoint_keys(self.model)

    def synchronize(self) -> None:
        if self.gpu:
            torch.cuda.synchronize(self.device)

    def invalidate_graphs(self) -> None:
        self._graphs.clear()

    # -- data -------------------------------------------------------------------------------------
    def attach(self, train: Split) -> None:
        self.train = train.to(self.device)
        self.invalidate_graphs()

    def begin_epoch(self, order: np.ndarray) -> None:
        order = np.ascontiguousarray(order, dtype=np.int32)
        n = int(order.shape[0])
        if self.order.numel() < n:
            self.order = torch.zeros(n, device=self.device, dtype=torch.int32)
            self.invalidate_graphs()
        if n != self.order_len:
            self.invalidate_graphs()
        self.order_len = n
        if n:
            self.order[:n].copy_(torch.from_numpy(order))
        first = min(self.batch, n)
        self.state[0] = 0
        self.state[1] = first
        self.batch_ids.zero_()
        if first:
            self.batch_ids[:first].copy_(self.order[:first])

    # -- model ------------------------------------------------------------------------------------
    def forward(self, x: torch.Tensor, training: bool, state: torch.Tensor | None, pack: bool = True,
                xent: L.XentFusion | None = None, slice_sink: list | None = None,
                ingest: L.IngestSrc | None = None) -> torch.Tensor:
        """Layer stack.  Training: every op writes its parameter gradients straight into the
        flat gradient arena (views ``G``), so backward leaves ``grad`` complete with no
        accumulation or zeroing kernels.  ``pack``: refresh the packed conv-weight images
        from the arena first (False: the previous step's SGD tail already stored them).
        ``xent``: offered to the last layer, which may fuse the loss (``xent.out``).
        ``slice_sink``: conv layers defer their weight-gradient slice sums to the SGD tail.
        ``ingest``: the first conv reads the batch's u8 images itself and fills ``x``."""
        P, G, Bf, dt = self.P, self.G, self.Bf, self.gemm_dtype
        if pack and self._pack_jobs:
            self.ext.conv_pack_all(self._pack_jobs, torch.cuda.current_stream(self.device).cuda_stream)
        fuse_act = training and self.gpu  # BN + following ReLU / ReLU-pool in one op (MI355X training)
        skip = False
        bn_stats = None  # statistics partials a conv epilogue produced for the BatchNorm after it
        bn_bwd = None    # a BatchNorm + ReLU whose backward statistics the next conv's dgrad computes
        for i, layer in enumerate(self.spec):
            if skip:  # activation already applied by the fused BatchNorm
                skip = False
                continue
            n = getattr(layer, "name", "")
            gw, gb = (G[f"{n}.weight"], G[f"{n}.bias"]) if (training and n) else (None, None)
            nxt = self.spec[i + 1] if i + 1 < len(self.spec) else None
            if fuse_act and isinstance(layer, zoo.BN) and isinstance(nxt, (zoo.Relu, zoo.ReluPool)):
                act = 2 if isinstance(nxt, zoo.ReluPool) else 1
                # BatchNorm + ReLU (+ pool) -> conv: that conv's data gradient also produces this
                # layer's backward statistics (no statistics pass in the BatchNorm backward)
                nn2 = self.spec[i + 2] if i + 2 < len(self.spec) else None
                nxt_packed = self._packed.get(getattr(nn2, "name", "")) if isinstance(nn2, zoo.Conv) else None
                if self.fuse_bn_bwd and nxt_packed is not None and nxt_packed[1] is not None:
                    bn_bwd = L.BnBwdStats(state)
                x = L.BatchNormActFn.apply(x, P[f"{n}.weight"], P[f"{n}.bias"], Bf[f"{n}.running_mean"],
                                           Bf[f"{n}.running_var"], state, layer.eps, layer.momentum, act, gw, gb,
                                           bn_stats, bn_bwd)
                bn_stats = None
                skip = True
            elif isinstance(layer, zoo.Conv):
                packed = self._packed.get(n)
                # conv -> ReLU + max-pool: the pool in the conv kernel's epilogue (one launch)
                pool = (self.gpu and isinstance(nxt, zoo.ReluPool) and packed is not None and packed[0] is not None
                        and n in self._pool_ok)
                # conv -> BatchNorm (+ activation) in training: the conv epilogue computes the
                # BatchNorm's batch statistics (no statistics pass over the conv output)
                nn2 = self.spec[i + 2] if i + 2 < len(self.spec) else None
                if (fuse_act and isinstance(nxt, zoo.BN) and isinstance(nn2, (zoo.Relu, zoo.ReluPool))
                        and packed is not None and packed[0] is not None):
                    bn_stats = L.BnStats(state)
                x = L.Conv2dFn.apply(x, P[f"{n}.weight"], P[f"{n}.bias"], layer.pad, dt, gw, gb, packed, slice_sink,
                                     pool, bn_stats, bn_bwd, ingest if i == 0 else None)
                bn_bwd = None
                skip = pool
            elif isinstance(layer, zoo.BN):
                x = L.BatchNorm2dFn.apply(x, P[f"{n}.weight"], P[f"{n}.bias"], Bf[f"{n}.running_mean"],
                                          Bf[f"{n}.running_var"], state, training, layer.eps, layer.momentum, gw, gb)
            elif isinstance(layer, zoo.ReluPool):
                x = L.ReluPoolFn.apply(x)
            elif isinstance(layer, zoo.Relu):
                x = L.ReluFn.apply(x)
            elif isinstance(layer, zoo.Flatten):
                x = x.reshape(x.shape[0], -1)
            elif isinstance(layer, zoo.FC):
                # Linear stays fp32 in both modes: the fc GEMMs are < 0.3 GFLOP per step (fp32
                # MFMA, linear.hip); on the GPU a following ReLU is fused into it
                relu = self.gpu and isinstance(nxt, zoo.Relu)
                last = nxt is None
                x = L.LinearFn.apply(x, P[f"{n}.weight"], P[f"{n}.bias"], torch.float32, gw, gb, relu,
                                     xent if last else None)
                skip = relu
        return x

    def _ingest(self) -> None:
        tr = self.train
        if self.gpu:
            self.ext.ingest(tr.images.data_ptr(), tr.labels.data_ptr(), self.batch_ids.data_ptr(), self.batch,
                            3 * 32 * 32, self.x.data_ptr(), self.labels.data_ptr(),
                            torch.cuda.current_stream(self.device).cuda_stream)
        else:
            ids = self.batch_ids.long()
            self.x.copy_((tr.images[ids].float() / 255.0 - 0.5) / 0.5)
            self.labels.copy_(tr.labels[ids])

    def _bookkeeping(self, loss: torch.Tensor, corr: torch.Tensor) -> None:
        if self.gpu:
            self.ext.layer_bookkeeping(loss.data_ptr(), corr.data_ptr(), self.batch, self.state.data_ptr(),
                                       self.stats.data_ptr(), self.order.data_ptr(), self.order_len,
                                       self.batch_ids.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream)
            return
        bv = int(self.state[1])
        if bv > 0:
            self.stats[0] += float(loss[:bv].double().sum()) / bv
            self.stats[1] += 1
            self.stats[2] += int(corr[:bv].sum())
            self.stats[3] += bv
        nxt = int(self.state[0]) + 1
        base = nxt * self.batch
        for b in range(self.batch):
            g = base + b
            self.batch_ids[b] = self.order[g] if g < self.order_len else 0
        self.state[0] = nxt
        self.state[1] = max(0, min(self.batch, self.order_len - base))

    def _fused_sgd(self) -> bool:
        return self.grad_sync is not None and getattr(self.grad_sync, "fuses_sgd", False)

    def _launch_step(self, first: bool = True) -> None:
        """One training step.  ``first``: the first step of a launch sequence (graph chunk or
        eager call) - it packs the conv-weight images from the arena, which may have changed
        since the last step (epoch averaging, checkpoint load, recovery); later steps find
        them refreshed by the previous step's SGD tail."""
        assert self.train is not None
        ingest = None
        if self.fuse_ingest:
            ingest = L.IngestSrc(self.train.images, self.train.labels, self.batch_ids, self.labels)
        else:
            self._ingest()
        tail = self.gpu and not self._fused_sgd() and self._tail_packs
        xent = L.XentFusion(self.labels, self.state) if self.gpu else None
        # single GPU: the conv weight-gradient slice sums run inside the SGD tail launch (with a
        # gradient all-reduce the gradients must be complete before it)
        sink = [] if (tail and self.grad_sync is None and self.defer_slice_sums) else None
        logits = self.forward(self.x, True, self.state, pack=first or not tail, xent=xent, slice_sink=sink,
                              ingest=ingest)
        if xent is not None and xent.out is not None:
            loss, corr, dl = xent.out  # fused into the last Linear's launch
        else:
            loss, corr, dl = L.cross_entropy(logits, self.labels, self.state)
        logits.backward(dl)  # writes every parameter gradient into self.grad (no zeroing needed)
        if self._fused_sgd():
            # one-shot xGMI all-reduce with the momentum-SGD update in the same launch (the next
            # step packs its conv weights itself: pack=True above)
            self.grad_sync.allreduce_sgd(self.grad, self.master, self.mom, None, self.lr, self.momentum,
                                         self.play.total)
        elif self.gpu:
            if self.grad_sync is not None:
                self.grad_sync.allreduce_grads(self.grad, [(0, self.play.total)])
            packs = self._pack_jobs if self._tail_packs else []
            # conv slice sums + SGD + the next step's packed conv weights + bookkeeping: one launch
            g0 = self.grad.data_ptr()
            slices = [(part.data_ptr(), S, M, Kd, (dw.data_ptr() - g0) // 4, (db.data_ptr() - g0) // 4)
                      for part, S, M, Kd, dw, db in (sink or [])]
            self.ext.sgd_tail(self.master.data_ptr(), g0, self.mom.data_ptr(), self.play.total, self.lr,
                              self.momentum, 1.0, packs, self.master.data_ptr(), slices, loss.data_ptr(),
                              corr.data_ptr(), self.batch, self.state.data_ptr(), self.stats.data_ptr(),
                              self.order.data_ptr(), self.order_len, self.batch_ids.data_ptr(),
                              torch.cuda.current_stream(self.device).cuda_stream)
            return
        else:
            if self.grad_sync is not None:
                self.grad_sync.allreduce_grads(self.grad, [(0, self.play.total)])
            with torch.no_grad():
                self.mom.mul_(self.momentum).add_(self.grad)
                self.master.sub_(self.lr * self.mom)
        self._bookkeeping(loss, corr)

    def _graph(self, nsteps: int) -> torch.cuda.CUDAGraph:
        key = (nsteps, id(self.grad_sync), self.order_len)
        g = self._graphs.get(key)
        if g is None:
            if not self._warm:
                self._warmup()
            self._wait()  # interruptible (queued replays may hold collectives on a dead peer)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(nsteps):
                    self._launch_step(first=i == 0)
            torch.cuda.synchronize(self.device)
            self._graphs[key] = g
        return g

    def _warmup(self) -> None:
        """Run two eager steps on a side stream (library/allocator lazy init happens outside
        any capture), then restore every piece of state they touched."""
        saved = [t.clone() for t in (self.master, self.mom, self.buffers, self.state, self.stats, self.batch_ids)]
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for i in range(2):
                self._launch_step(first=i == 0)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        for t, v in zip((self.master, self.mom, self.buffers, self.state, self.stats, self.batch_ids), saved):
            t.copy_(v)
        self._warm = True

    def prepare_graphs(self) -> None:
        if self.use_graphs:
            k = 1
            while k <= self.graph_chunk:
                self._graph(k)
                k *= 2

    def run_steps(self, n: int) -> None:
        if n <= 0:
            return
        poll = self.poll
        if not self.use_graphs:
            ctx = torch.cuda.device(self.device) if self.gpu else _Null()
            with ctx:
                for i in range(n):
                    if poll is not None:
                        poll()
                    self._launch_step(first=i == 0)
            self.num_batches_tracked += n
            return
        k = self.graph_chunk
        total = n
        while k >= 1:
            reps, n = divmod(n, k)
            if reps:
                g = self._graph(k)
                for _ in range(reps):
                    if poll is not None:
                        poll()
                    g.replay()
            k //= 2
        self.num_batches_tracked += total

    def epoch_stats(self, reset: bool = True) -> StepStats:
        v = self.stats.cpu().tolist()
        if reset:
            self.stats.zero_()
        return StepStats(v[0], int(round(v[1])), int(round(v[2])), int(round(v[3])))

    # -- evaluation -------------------------------------------------------------------------------
    def evaluate_samples(self, split: Split, lo: int = 0, hi: int | None = None, chunk: int = 1000):
        split = split.to(self.device)
        hi = len(split) if hi is None else hi
        losses, corrs = [], []
        with torch.no_grad():
            for s in range(lo, hi, chunk):
                e = min(hi, s + chunk)
                if self.gpu:  # same ingest kernel as training (IEEE division, like ToTensor)
                    ids = torch.arange(s, e, device=self.device, dtype=torch.int32)
                    x = torch.empty(e - s, 3, 32, 32, device=self.device)
                    lab = torch.empty(e - s, device=self.device, dtype=torch.int32)
                    self.ext.ingest(split.images.data_ptr(), split.labels.data_ptr(), ids.data_ptr(), e - s,
                                    3 * 32 * 32, x.data_ptr(), lab.data_ptr(),
                                    torch.cuda.current_stream(self.device).cuda_stream)
                else:
                    x = (split.images[s:e].float() / 255.0 - 0.5) / 0.5
                    lab = split.labels[s:e].to(torch.int32).contiguous()
                logits = self.forward(x, False, None)
                loss, corr, _ = L.cross_entropy(logits, lab, None, want_grad=False)
                losses.append(loss)
                corrs.append(corr)
        if not losses:
            return (torch.zeros(0, device=self.device), torch.zeros(0, device=self.device, dtype=torch.int32))
        return torch.cat(losses), torch.cat(corrs)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
