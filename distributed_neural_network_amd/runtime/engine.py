"""Training engines: the MI355X HIP engine and the CPU oracle engine.

Both expose one interface used by the trainer / sync policies:

* ``attach(train_split)`` - make the training split resident on the device,
* ``begin_epoch(order)``  - this rank's sample order for the epoch (cursor <- 0),
* ``run_steps(n)``        - n optimizer steps (fwd + bwd + [grad sync] + SGD),
* ``epoch_stats()``       - device-accumulated loss/accuracy of the epoch,
* ``evaluate(split, bs)`` - per-sample test loss/correct (reference eval semantics),
* ``master`` / ``mom``    - flat fp32 parameter / momentum arenas (state_dict views).

Capability parity: ``run_child``'s hot loop (data_parallelism_train.py:185-213,
model_replication_train.py:96-114, single_proc_train.py:61-74) and ``eval``
(data_parallelism_train.py:157-183).

HipEngine design (MI355X): a step is 2 kernels (fused per-sample fwd/bwd, batch
reduce + SGD) or, with a per-step gradient all-reduce, 3 kernels (fused, batch reduce,
one-shot xGMI all-reduce + SGD; parallel/xgmi.py) - or 2 + 1 kernels around bucketed
RCCL all-reduces when the xGMI path is unavailable.  Steps are captured into hipGraphs (through
torch.cuda.CUDAGraph) in chunks of ``graph_chunk`` steps; the step cursor, the
tail-batch size and the epoch loss/accuracy accumulators live on the device, so a
chunk replays with zero host work per step and no host<->device sync until the
epoch ends.
"""
from __future__ import annotations

import os
import sys
import time
from dataclasses import dataclass
from typing import Callable, Optional, Protocol

import numpy as np
import torch
import torch.nn.functional as F

from ..data.datasets import Split
from ..models.network import LAYOUT, arena_state_dict, init_arena, load_state_dict_into
from ..ops import native, reference


class StepWaitTimeout(RuntimeError):
    """A bounded in-launch wait of the pipelined / persistent step timed out: the epoch's parameters are not trustworthy.  ``Trainer.run`` restores the epoch's
    snapshot, steps the engine down (``HipEngine.degrade``: persistent -> pipelined -> serial)
    and redoes the epoch; nothing else is lost."""


class GradSync(Protocol):
    """Per-step gradient synchronisation (the step-allreduce policy implements it)."""

    def allreduce_grads(self, grad: torch.Tensor, buckets: list[tuple[int, int]],
                        before_last: Optional[Callable[[], None]] = None) -> None: ...


@dataclass
class StepStats:
    loss_sum: float      # sum over batches of the batch-mean loss
    batches: int
    correct: int
    samples: int

    @property
    def mean_loss(self) -> float:
        return self.loss_sum / max(self.batches, 1)

    @property
    def accuracy(self) -> float:
        return 100.0 * self.correct / max(self.samples, 1)


def eval_metrics(loss: torch.Tensor, correct: torch.Tensor, batch_size: int) -> tuple[float, float]:
    """Reference eval metrics from per-sample values.

    val loss = mean over test batches of the batch-mean loss (np.mean(losses),
    data_parallelism_train.py:176); accuracy = 100 * correct / total (:177).
    """
    loss = loss.double().cpu()
    n = loss.numel()
    nb = (n + batch_size - 1) // batch_size
    sums = torch.zeros(nb, dtype=torch.float64).index_add_(0, torch.arange(n) // batch_size, loss)
    counts = torch.full((nb,), float(batch_size), dtype=torch.float64)
    counts[-1] = n - (nb - 1) * batch_size
    return float((sums / counts).mean()), 100.0 * float(correct.sum()) / max(n, 1)


def ranks_per_gpu() -> int:
    """Ranks of this job per visible GPU on this host (1 unless ranks time-share a device: the
    one-GPU rehearsals).  The local rank count comes from the launcher's environment (torchrun,
    OpenMPI, MPICH / Intel MPI, Slurm); without one, the world size is taken as local."""
    n = None
    for k in ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "SLURM_NTASKS_PER_NODE"):
        v = os.environ.get(k)
        if v:
            try:
                n = int(v.split("(")[0])
                break
            except ValueError:
                pass
    if n is None:
        n = int(os.environ.get("WORLD_SIZE", os.environ.get("OMPI_COMM_WORLD_SIZE", "1")) or 1)
    d = max(1, torch.cuda.device_count())
    return max(1, -(-n // d))


def gpu_shared_by_ranks() -> bool:
    """Do other ranks of this job run on this process's GPU (the one-GPU rehearsals)?"""
    return ranks_per_gpu() > 1


class Engine:
    device: torch.device
    batch: int

    def __init__(self, batch: int, lr: float, momentum: float, arena: torch.Tensor | None, seed: int | None) -> None:
        self.batch = int(batch)
        self.lr = float(lr)
        self.momentum = float(momentum)
        self._init_arena = arena if arena is not None else init_arena(seed)
        self.grad_sync: GradSync | None = None
        self.train: Split | None = None
        self.order_len = 0
        # liveness check between graph replays / steps (Trainer installs
        # Communicator.check_alive): raises CommError on the main thread when the heartbeat
        # watchdog has flagged a dead peer, instead of queueing more work behind a
        # collective that can no longer complete
        self.poll: Optional[Callable[[], None]] = None
        # interruptible device wait (Trainer installs Communicator.wait_device): every host wait
        # on this rank's queued work - graph capture, buffer resizes - polls instead of blocking
        # in torch.cuda.synchronize, which a collective spinning on a dead peer (native RCCL: no
        # bounded wait) would never release
        self.device_wait: Optional[Callable[[], None]] = None

    # -- parameters --------------------------------------------------------------------
    def state_dict(self):
        return arena_state_dict(self.master)

    def load_state_dict(self, sd) -> None:
        with torch.no_grad():
            host = torch.zeros(LAYOUT.total)
            load_state_dict_into(host, sd)
            self.master.copy_(host.to(self.master.device))
        self.params_changed()

    def params_changed(self) -> None:
        """Call after writing ``master`` from outside (all-reduce, load)."""

    def reset_momentum(self) -> None:
        self.mom.zero_()

    def steps_per_epoch(self) -> int:
        return (self.order_len + self.batch - 1) // self.batch

    def synchronize(self) -> None:
        pass

    def _wait(self) -> None:
        """Wait for this rank's queued device work (interruptibly when a watch is installed)."""
        if self.device_wait is not None:
            self.device_wait()
        else:
            self.synchronize()

    def _wait_event(self, ev) -> None:
        if self.device_wait is None or self.poll is None:
            ev.synchronize()
            return
        while not ev.query():
            self.poll()
            time.sleep(50e-6)


class CpuEngine(Engine):
    """fp32 PyTorch execution on the CPU (oracle / CPU-only hosts), same arena layout."""

    def __init__(self, batch: int, lr: float = 0.001, momentum: float = 0.9, arena: torch.Tensor | None = None,
                 seed: int | None = None) -> None:
        super().__init__(batch, lr, momentum, arena, seed)
        self.device = torch.device("cpu")
        self.master = self._init_arena.clone().float()
        self.grad = torch.zeros_like(self.master)
        self.mom = torch.zeros_like(self.master)
        self._stats = [0.0, 0, 0, 0]
        self._order = np.zeros(0, dtype=np.int32)
        self._cursor = 0

    def attach(self, train: Split) -> None:
        self.train = train.to("cpu")

    def begin_epoch(self, order: np.ndarray) -> None:
        self._order = np.asarray(order, dtype=np.int32)
        self.order_len = int(self._order.shape[0])
        self._cursor = 0

    def run_steps(self, n: int) -> None:
        assert self.train is not None
        for _ in range(n):
            if self.poll is not None:
                self.poll()
            lo = self._cursor * self.batch
            idx = torch.from_numpy(self._order[lo:lo + self.batch].astype(np.int64))
            self._cursor += 1
            if idx.numel() == 0:
                continue
            x = self.train.images[idx]
            y = self.train.labels[idx]
            g, loss, correct = reference.batch_grad(self.master, x, y, return_correct=True)
            self.grad.copy_(g)
            if self.grad_sync is not None:
                self.grad_sync.allreduce_grads(self.grad, [(0, LAYOUT.total)])
            reference.sgd_momentum_(self.master, self.grad, self.mom, self.lr, self.momentum)
            self._stats[0] += loss
            self._stats[1] += 1
            self._stats[2] += correct
            self._stats[3] += int(idx.numel())

    def epoch_stats(self, reset: bool = True) -> StepStats:
        s = StepStats(float(self._stats[0]), int(self._stats[1]), int(self._stats[2]), int(self._stats[3]))
        if reset:
            self._stats = [0.0, 0, 0, 0]
        return s

    def evaluate_samples(self, split: Split, lo: int = 0, hi: int | None = None, chunk: int = 1000):
        hi = len(split) if hi is None else hi
        losses, corrects = [], []
        with torch.no_grad():
            for s in range(lo, hi, chunk):
                e = min(hi, s + chunk)
                x = reference.normalize_u8(split.images[s:e])
                y = split.labels[s:e].long()
                logits = reference.forward(self.master, x)
                losses.append(F.cross_entropy(logits, y, reduction="none"))
                corrects.append((logits.argmax(1) == y).int())
        if not losses:
            return torch.zeros(0), torch.zeros(0, dtype=torch.int32)
        return torch.cat(losses), torch.cat(corrects)


class HipEngine(Engine):
    """MI355X engine: hand-written gfx950 kernels + hipGraph-captured step chunks."""

    def __init__(self, batch: int, lr: float = 0.001, momentum: float = 0.9, arena: torch.Tensor | None = None,
                 seed: int | None = None, device: str | torch.device = "cuda", graph_chunk: int = 32,
                 use_graphs: bool = True, overlap: bool = False, stage_images: bool | None = None,
                 dtype: str = "bf16", pipeline: bool | None = None, persist: bool | None = None) -> None:
        super().__init__(batch, lr, momentum, arena, seed)
        if dtype not in ("bf16", "fp32"):
            raise ValueError(f"HipEngine dtype must be bf16 or fp32, not {dtype!r}")
        # bf16: lenet_fused.hip (bf16 MFMA operands from the optimizer-packed shadow, fp32
        # accumulation); fp32: lenet_f32.hip (fp32 operands straight from the master arena -
        # the reference's arithmetic).  Both write the same per-sample rows for grad_reduce.
        self.dtype = dtype
        if not torch.cuda.is_available():
            raise RuntimeError("HipEngine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.ext = native.hip()
        self.ext.init()
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        dev = self.device
        B = self.batch
        f32 = dict(device=dev, dtype=torch.float32)
        self.master = self._init_arena.to(**f32).contiguous()
        self.grad = torch.zeros(LAYOUT.total, **f32)
        self.mom = torch.zeros(LAYOUT.total, **f32)
        # bf16 [plain arena copy | kernel-ready weight images] (csrc/kernels/common.h SH_*)
        self.shadow = torch.zeros(self.ext.layout()["shadow_total"], device=dev, dtype=torch.bfloat16)
        self.state = torch.zeros(4, device=dev, dtype=torch.int32)
        self.stats = torch.zeros(4, device=dev, dtype=torch.float64)
        self.a0 = torch.zeros(B, 400, **f32)
        self.h1 = torch.zeros(B, 120, **f32)
        self.h2 = torch.zeros(B, 84, **f32)
        self.z1 = torch.zeros(B, 120, **f32)
        self.z2 = torch.zeros(B, 84, **f32)
        self.z3 = torch.zeros(B, 16, **f32)
        self.slab = torch.zeros(B, native.SLAB, **f32)
        self.loss = torch.zeros(B, **f32)
        self.correct = torch.zeros(B, device=dev, dtype=torch.int32)
        self.order = torch.zeros(0, device=dev, dtype=torch.int32)
        self.staged = torch.zeros(0, device=dev, dtype=torch.int32)  # epoch order upload target
        self._pin = [torch.empty(0, dtype=torch.int32), torch.empty(0, dtype=torch.int32)]
        self._pin_ev = [torch.cuda.Event(), torch.cuda.Event()]
        self._pin_i = 0
        self.batch_ids = torch.zeros(B, device=dev, dtype=torch.int32)  # sample ids of the next step
        # next step's images + labels, staged by the fused kernel of the current step
        # ([B][3072] u8 | [B] int32; lenet_fused.hip), so a step's image load has no
        # dependency on its sample ids (stage_images=False / DNN_STAGE_IMAGES=0 turns it off)
        if stage_images is None:
            stage_images = os.environ.get("DNN_STAGE_IMAGES", "1") != "0" and dtype == "bf16"
        if stage_images and dtype != "bf16":
            raise ValueError("image staging is a feature of the bf16 kernel")
        self.stage = torch.zeros(B * (3072 + 4), device=dev, dtype=torch.uint8) if stage_images else None
        self.next_ids = torch.full((B,), -1, device=dev, dtype=torch.int32)  # ids two steps ahead
        self._staged = False  # stage holds this epoch's step-0 batch (set by begin_epoch)
        self._ahead = False  # (fp32 persistent) next_ids holds this epoch's step-1 ids (set by begin_epoch)
        self.graph_chunk = 1 << max(0, int(graph_chunk).bit_length() - 1)  # power of two
        self.use_graphs = use_graphs
        self.overlap = overlap
        # Pipelined step (lenet_fused.hip PIPE; bf16, staged images, local step): launch i of a
        # step chunk runs step i - 1's batch reduction + SGD in its first workgroups and step i's
        # samples in the rest, which wait (in-launch ready counters) for the new weights before
        # they load them - the reduction hides under the samples' image ingest, and a chunk of n
        # steps is n + 1 launches instead of 2 n.  Bit-identical to the serial step (the same
        # kernels' arithmetic).  On by default: 18.5 vs 18.9 us per step over 2000 steps, 19.9
        # vs 20.4 in the 20-step window (profiles/r4/pipe_v2, pipe_v3); DNN_PIPELINE=0 turns it off.
        if pipeline is None:
            pipeline = os.environ.get("DNN_PIPELINE", "1") != "0"
        self.pipeline = bool(pipeline) and dtype == "bf16" and stage_images
        # Persistent launch (lenet_fused.hip PERS; on top of the pipelined step - or, fp32,
        # lenet_f32.hip PERS on its own: the fp32 kernel has no pipelined form): a chunk of n steps
        # is ONE launch - the reduction and sample workgroups loop over the steps and hand off
        # through in-launch arrival / ready flags, so no kernel boundary sits between two steps.
        # Its reduction and sample workgroups wait on each other, so the whole grid must be
        # co-resident: batch <= persist_max_batch() (one workgroup per CU), and no other rank's
        # persistent grid on the same GPU (ranks time-sharing a device would each hold part of
        # the CUs); DNN_PERSIST=0 turns it off.
        if persist is None:
            # (fp32: DNN_PERSIST_F32=0 turns it off - with one conv reduction block per workgroup
            # it matches the serial fp32 step over 5000 steps, 26.46 vs 26.43 us, and beats it in
            # the 20/5 window, 27.61 vs 28.07 us: profiles/r5/fp32_pers)
            persist = (os.environ.get("DNN_PERSIST", "1") != "0" if dtype == "bf16"
                       else os.environ.get("DNN_PERSIST_F32", "1") != "0" and os.environ.get("DNN_PERSIST", "1") != "0")
        # ranks time-sharing this GPU (one-GPU rehearsals): every rank's grid must be resident at
        # once - ranks x (reduction + sample workgroups) within the occupancy-derived count
        share = ranks_per_gpu()
        if dtype == "fp32":
            fits = B <= self.ext.persist_max_batch_f32() and (
                share == 1 or share * (self.ext.persist_wg_f32() + B)
                <= self.ext.persist_resident_workgroups_f32() - 8)
        else:
            fits = B <= self.ext.persist_max_batch() and (
                share == 1 or share * (self.ext.pipe_reduce_blocks() // 2 + 1 + B)
                <= self.ext.persist_resident_workgroups() - 8)
        self.persist = bool(persist) and (self.pipeline or dtype == "fp32") and fits
        if self.pipeline or self.persist:
            # the second parity's per-sample rows (the first is a0 .. correct above) - each row
            # kind as ONE [2][B][...] buffer, parity 1 right after parity 0 (the persistent
            # launch addresses both from one pointer) -, the second {bvalid, next_ids}
            # bookkeeping slot (bvalid in state[2]) and the sticky wait-timeout word
            self._rows2 = {}
            for k in ("a0", "h1", "h2", "z1", "z2", "z3", "slab", "loss", "correct"):
                t = getattr(self, k)
                both = torch.zeros((2,) + tuple(t.shape), device=dev, dtype=t.dtype)
                setattr(self, k, both[0])
                self._rows2[k] = both[1]
            self.next_ids2 = torch.full((B,), -1, device=dev, dtype=torch.int32)
            self.pipe_err = torch.zeros(1, device=dev, dtype=torch.int32)
        if self.pipeline:
            # arrival counters [parity][group] and ready flags [parity][group][sample], a 128-B line
            # each, in uncached memory: every poll reads memory (lenet_fused.hip pipe_wait)
            ng = self.ext.pipe_groups()
            self._pipe_ctr_ptr = self.ext.uncached_alloc(2 * ng * 128)
            self._pipe_flg_ptr = self.ext.uncached_alloc(2 * ng * B * 128)
        # the per-step xGMI all-reduce inside the persistent launch (installed by the
        # step-allreduce policy's "-pers" paths after their self-test; lenet_fused.hip XNR)
        self.pers_exchange = False
        # control words of the persistent launch (generation, ready and arrival words): uncached
        # (fine-grained) memory, or (DNN_PERS_CTL=coarse, measurement) an ordinary device buffer -
        # every access to them is an sc1 load / store either way
        self._pers_ctl_t = None
        if self.persist and os.environ.get("DNN_PERS_CTL", "uncached") == "coarse":
            self._pers_ctl_t = torch.zeros(max(self.ext.persist_ctl_bytes(B), self.ext.persist_ctl_bytes_f32(B)) // 4 + 64,
                                           device=dev, dtype=torch.int32)
            self._pers_ctl = self._pers_ctl_t.data_ptr()
        else:
            ctl_bytes = self.ext.persist_ctl_bytes_f32(B) if dtype == "fp32" else self.ext.persist_ctl_bytes(B)
            self._pers_ctl = self.ext.uncached_alloc(ctl_bytes) if self.persist else 0
        self.stream = torch.cuda.Stream(dev)
        self._graphs: dict[tuple, torch.cuda.CUDAGraph] = {}
        # Direct AQL dispatch of the persistent launch (csrc/runtime/aql_dispatch.h; default
        # on, DNN_AQL=0 turns it off): the kernel the graphs replay, dispatched through this
        # process's own HSA queue with its arguments in device memory, and waited for by spinning
        # on its completion signal - no stream, graph or interrupt in the launch + completion path
        # (a graph of one trivial kernel costs ~20 us from replay to the synchronize's return;
        # 20/5 windows 16.75 vs 16.95 us/step: profiles/r6/aql/).  run_steps then returns once the
        # steps are done (synchronous), after the stream's earlier work.  Only without a per-step
        # all-reduce: the in-launch exchange needs every rank's launch in flight together.
        self._direct_h: dict[tuple, int] = {}
        self.direct = False
        self.direct_why = "off (DNN_AQL=0)"
        if os.environ.get("DNN_AQL", "1") != "0":
            # (the queue is created by the first prepared dispatch; if that fails - no HSA agent
            # for the device, a refused queue - run_steps falls back to graph replays, loudly)
            self.direct, self.direct_why = (True, "on") if self.persist else (False, "the persistent launch is off")
        self.params_changed()
        torch.cuda.synchronize(dev)

    # -- helpers ------------------------------------------------------------------------
    @staticmethod
    def _p(t: torch.Tensor) -> int:
        return t.data_ptr()

    # the current stream's raw handle: torch's accessor for it costs ~0.2 us, a Stream object ~2 us
    # (a direct window's whole Python path was ~3 us: profiles/r6/aql/)
    _RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)

    def _stream(self) -> int:
        if self._RAW_STREAM is not None:
            return self._RAW_STREAM(self.device.index)
        return torch.cuda.current_stream(self.device).cuda_stream

    def synchronize(self) -> None:
        torch.cuda.synchronize(self.device)

    def params_changed(self) -> None:
        with torch.cuda.device(self.device):
            self.ext.sgd_apply(self._p(self.master), self._p(self.grad), self._p(self.mom), self._p(self.shadow),
                               LAYOUT.total, 0.0, 0.0, 1.0, 1, self._stream())

    def invalidate_graphs(self) -> None:
        self._graphs.clear()
        self._direct_h.clear()

    # -- data ---------------------------------------------------------------------------
    def attach(self, train: Split) -> None:
        self.train = train.to(self.device)
        self._staged = False  # the stage holds images of the previous split until begin_epoch
        self.invalidate_graphs()

    def begin_epoch(self, order: np.ndarray) -> None:
        """Queue the epoch start without a host<->device synchronisation: the order goes
        through a pinned staging buffer with a stream-ordered async copy, then ONE
        ``epoch_begin`` launch sets the order, the first step's sample ids and the cursor.
        (Measured at 100 steps per epoch: 0.15 us/step of boundary cost vs 0.5-0.8 for a
        blocking upload + separate fill/copy ops; an upload on a side stream with a
        cross-stream event wait was slower still, 1.4 us/step, even in steady state.)"""
        order = np.ascontiguousarray(order, dtype=np.int32)
        n = int(order.shape[0])
        if self.order.numel() < n:
            self._wait()
            self.order = torch.zeros(n, device=self.device, dtype=torch.int32)
            self.staged = torch.zeros(n, device=self.device, dtype=torch.int32)
            self.invalidate_graphs()
        if n != self.order_len:
            self.invalidate_graphs()  # order_len is a baked kernel argument
        self.order_len = n
        main = torch.cuda.current_stream(self.device)
        if n:
            i = self._pin_i = self._pin_i ^ 1
            if self._pin[i].numel() < n:
                self._pin[i] = torch.empty(n, dtype=torch.int32, pin_memory=True)
            self._wait_event(self._pin_ev[i])  # this staging buffer's previous upload is done
            self._pin[i][:n].numpy()[:] = order
            self.staged[:n].copy_(self._pin[i][:n], non_blocking=True)
            self._pin_ev[i].record(main)
        staged = self.stage is not None and self.train is not None and n > 0
        if staged != self._staged:
            self.invalidate_graphs()  # the stage pointer is a baked kernel argument
        self._staged = staged
        # the fp32 persistent launch reads the next step's ids from the bookkeeping slots (no stage)
        ahead = self.dtype == "fp32" and self.persist and self.train is not None and n > 0
        if ahead != self._ahead:
            self.invalidate_graphs()  # next_ids is a baked reduction argument
        self._ahead = ahead
        st = dict(images=self._p(self.train.images), labels=self._p(self.train.labels),
                  next_ids=self._p(self.next_ids), stage=self._p(self.stage)) if staged else {}
        if ahead:
            st = dict(next_ids=self._p(self.next_ids))
        with torch.cuda.device(self.device):
            self.ext.epoch_begin(self._p(self.staged), self._p(self.order), n, self._p(self.state),
                                 self._p(self.batch_ids), self.batch, main.cuda_stream, **st)

    # -- one step (launch sequence; also what graphs capture) ---------------------------
    def _reduce(self, fuse_sgd: int, lo: int, hi: int, bookkeeping: int, s: int, **xg) -> None:
        self.ext.grad_reduce(self._p(self.a0), self._p(self.h1), self._p(self.h2), self._p(self.z1),
                             self._p(self.z2), self._p(self.z3), self._p(self.slab), self._p(self.loss),
                             self._p(self.correct), self.batch, self._p(self.master), self._p(self.grad),
                             self._p(self.mom), self._p(self.shadow), self._p(self.state), self._p(self.stats),
                             self.lr, self.momentum, 1.0, fuse_sgd, lo, hi, bookkeeping, self._p(self.order),
                             self.order_len, self._p(self.batch_ids), s,
                             next_ids=self._p(self.next_ids) if self._staged or self._ahead else 0, **xg)

    def pipe_failed(self) -> bool:
        return hasattr(self, "pipe_err") and int(self.pipe_err.item()) != 0

    def _pipe_ok(self) -> bool:
        """The pipelined step runs: bf16 with staged images, no all-reduce installed (one rank)."""
        return self.pipeline and self.grad_sync is None and self._staged

    def _pers_xchg(self):
        """The xGMI group whose one-launch exchange runs inside the persistent launch, or None:
        installed by a "-pers" path (pers_exchange), self-tested one-launch exchange, fp32
        granules (pull or two-hop)."""
        if not self.pers_exchange or self.grad_sync is None or not getattr(self.grad_sync, "fuses_sgd", False):
            return None
        grp = getattr(self.grad_sync, "group", None)
        if grp is None or not grp.one_launch or grp.xp_mode not in (0, 2):
            return None
        return grp

    # bound of one ready wait (then a sticky error word, raised at epoch_stats); DNN_PIPE_TIMEOUT_S
    # overrides it (tests force a timeout with a tiny bound + an injected delay, DNN_PIPE_FLAGS=256)
    PIPE_TIMEOUT_S = float(os.environ.get("DNN_PIPE_TIMEOUT_S", "10.0"))
    _pipe_stamps = 0  # diagnostic (tools/phase_trace.py --pipe): stamp buffer of the merged launches
    # lenet_fused.hip PipeCtl.flags (measurement switches): & 1 no mid-phase-B fc1 stream
    pipe_flags = int(os.environ.get("DNN_PIPE_FLAGS", "0"))

    def _rows(self, par: int) -> dict:
        if par == 0:
            return dict(a0=self.a0, h1=self.h1, h2=self.h2, z1=self.z1, z2=self.z2, z3=self.z3, slab=self.slab,
                        loss=self.loss, correct=self.correct)
        return self._rows2

    def _launch_steps_pipe(self, n: int) -> None:
        """n steps as n + 1 launches: launch i (< n) = [step i - 1's reduction] + [step i's
        samples]; launch n = step n - 1's reduction alone (grad_reduce), which also re-publishes
        the bookkeeping slot the next chunk's first launch reads (slot 0).  Bookkeeping slots:
        slot 0 = (state[ST_BVALID], next_ids) - the serial layout epoch_begin writes -, slot 1 =
        (state[2], next_ids2); launch i's samples read slot i & 1 and its bookkeeping publishes
        slot (i + 1) & 1 one launch ahead."""
        s = self._stream()
        sp = self._p(self.state)
        slot_bv = (sp + 4, sp + 8)
        slot_nid = (self._p(self.next_ids), self._p(self.next_ids2))
        f1w = LAYOUT.offsets["fc1.weight"]
        for i in range(n + 1):
            par = i & 1
            prev = self._rows((i - 1) & 1)
            red = dict(a0=self._p(prev["a0"]), h1=self._p(prev["h1"]), h2=self._p(prev["h2"]), z1=self._p(prev["z1"]),
                       z2=self._p(prev["z2"]), z3=self._p(prev["z3"]), slab=self._p(prev["slab"]),
                       loss=self._p(prev["loss"]), correct=self._p(prev["correct"]), batch=self.batch,
                       master=self._p(self.master), grad=self._p(self.grad), mom=self._p(self.mom),
                       shadow=self._p(self.shadow), state=sp, stats=self._p(self.stats), lr=self.lr,
                       momentum=self.momentum, grad_scale=1.0, fuse_sgd=1, bookkeeping=1, order=self._p(self.order),
                       order_len=self.order_len, batch_ids=self._p(self.batch_ids), stream=s)
            if i == n:  # the chunk's last reduction: its own launch, re-publishing slot 0
                self.ext.grad_reduce(lo=0, hi=LAYOUT.total, next_ids=slot_nid[0], bk_bv_in=slot_bv[(i - 1) & 1],
                                     bk_bv_out=slot_bv[0], bk_adv=0, **red)
                break
            first = i == 0
            self.ext.grad_reduce(lo=f1w if first else 0, hi=f1w if first else LAYOUT.total, defer=2,
                                 next_ids=slot_nid[par ^ 1], bk_bv_in=slot_bv[(i - 1) & 1],
                                 bk_bv_out=slot_bv[par ^ 1], bk_adv=1, bk_stats=0 if first else 1, **red)
            rows = self._rows(par)
            self.ext.fused_train_pipe(self._p(self.train.images), self._p(self.train.labels), self.order_len,
                                      self.batch, self._p(self.master), self._p(self.shadow), self._p(rows["a0"]),
                                      self._p(rows["h1"]), self._p(rows["h2"]), self._p(rows["z1"]),
                                      self._p(rows["z2"]), self._p(rows["z3"]), self._p(rows["slab"]),
                                      self._p(rows["loss"]), self._p(rows["correct"]), slot_nid[par],
                                      self._p(self.stage), self._pipe_ctr_ptr, par, 0 if first else 1,
                                      1 if first else self.ext.pipe_reduce_blocks(), slot_bv[par],
                                      self._p(self.pipe_err), self.PIPE_TIMEOUT_S, s,
                                      stamps=0 if first else self._pipe_stamps, flags=self.pipe_flags,
                                      flg=self._pipe_flg_ptr)

    def _pers_ok(self) -> bool:
        """The persistent launch runs: the pipelined step's conditions and persist - or, with a
        per-step all-reduce, its "-pers" form (the exchange inside the launch's reduction).
        fp32: lenet_f32.hip's persistent launch (its "-pers" exchange too: round 6)."""
        if self.dtype == "fp32":
            return self.persist and self._ahead and (self.grad_sync is None or self._pers_xchg() is not None)
        if not (self.persist and self.pipeline and self._staged):
            return False
        return self.grad_sync is None or self._pers_xchg() is not None

    def _launch_steps_pers(self, n: int, direct: bool = False) -> int:
        """n steps as ONE launch (lenet_fused.hip PERS): the same reduction, bookkeeping slots and
        publication sequence as _launch_steps_pipe's n + 1 launches, with the reduction of step
        n - 1 inside the launch too (it re-publishes slot 0 for the next chunk)."""
        s = self._stream()
        sp = self._p(self.state)
        r = self._rows(0)
        grp = self._pers_xchg()
        xg = grp.exchange() if grp is not None else {}
        if self.dtype == "fp32":
            self.ext.grad_reduce(self._p(r["a0"]), self._p(r["h1"]), self._p(r["h2"]), self._p(r["z1"]),
                                 self._p(r["z2"]), self._p(r["z3"]), self._p(r["slab"]), self._p(r["loss"]),
                                 self._p(r["correct"]), self.batch, self._p(self.master), self._p(self.grad),
                                 self._p(self.mom), self._p(self.shadow), sp, self._p(self.stats), self.lr,
                                 self.momentum, 1.0, 1, 0, LAYOUT.total, 1, self._p(self.order), self.order_len,
                                 self._p(self.batch_ids), s, defer=2, next_ids=self._p(self.next_ids), **xg)
            return self.ext.fused_train_persist_f32(
                self._p(self.train.images), self._p(self.train.labels), self.order_len, self.batch,
                self._p(self.master), self._p(r["a0"]), self._p(r["h1"]), self._p(r["h2"]), self._p(r["z1"]),
                self._p(r["z2"]), self._p(r["z3"]), self._p(r["slab"]), self._p(r["loss"]), self._p(r["correct"]),
                self._pers_ctl, n, sp + 4, sp + 8, self._p(self.next_ids), self._p(self.next_ids2),
                self._p(self.pipe_err), self.PIPE_TIMEOUT_S, s, flags=self.pipe_flags, stamps=self._pipe_stamps,
                direct=direct)
        self.ext.grad_reduce(self._p(r["a0"]), self._p(r["h1"]), self._p(r["h2"]), self._p(r["z1"]),
                             self._p(r["z2"]), self._p(r["z3"]), self._p(r["slab"]), self._p(r["loss"]),
                             self._p(r["correct"]), self.batch, self._p(self.master), self._p(self.grad),
                             self._p(self.mom), self._p(self.shadow), sp, self._p(self.stats), self.lr,
                             self.momentum, 1.0, 1, 0, LAYOUT.total, 1, self._p(self.order), self.order_len,
                             self._p(self.batch_ids), s, defer=2, next_ids=self._p(self.next_ids), **xg)
        return self.ext.fused_train_persist(self._p(self.train.images), self._p(self.train.labels), self.order_len,
                                            self.batch, self._p(self.master), self._p(self.shadow), self._p(r["a0"]),
                                            self._p(r["h1"]), self._p(r["h2"]), self._p(r["z1"]), self._p(r["z2"]),
                                            self._p(r["z3"]), self._p(r["slab"]), self._p(r["loss"]),
                                            self._p(r["correct"]), self._p(self.stage), self._pers_ctl, n, sp + 4,
                                            sp + 8, self._p(self.next_ids), self._p(self.next_ids2),
                                            self._p(self.pipe_err), self.PIPE_TIMEOUT_S, s,
                                            stamps=self._pipe_stamps, flags=self.pipe_flags, direct=direct)

    def _launch_steps(self, n: int) -> None:
        """n training steps' launches (what a chunk graph captures)."""
        if self._pers_ok():
            self._launch_steps_pers(n)
            return
        if self._pipe_ok():
            self._launch_steps_pipe(n)
            return
        for _ in range(n):
            self._launch_step()

    def __del__(self) -> None:
        """Give the uncached control buffers back to the extension's pool (never to the driver:
        csrc/comm/xgmi_allreduce.hip uncached_alloc) once this engine's queued work is done."""
        bufs = [getattr(self, "_pipe_ctr_ptr", 0), getattr(self, "_pipe_flg_ptr", 0),
                getattr(self, "_pers_ctl", 0) if getattr(self, "_pers_ctl_t", None) is None else 0]
        if not any(bufs):
            return
        try:
            torch.cuda.synchronize(self.device)
        except Exception:
            return  # (the device is gone: nothing can be handed back safely)
        for p in bufs:  # each on its own: one failing free must not leak the others
            if p:
                try:
                    self.ext.uncached_free(p)
                except Exception:
                    pass

    def _launch_step(self) -> None:
        assert self.train is not None
        s = self._stream()
        if self.dtype == "fp32":
            self.ext.fused_train_f32(self._p(self.train.images), self._p(self.train.labels), self._p(self.batch_ids),
                                     self.order_len, self.batch, self._p(self.state), self._p(self.master),
                                     self._p(self.a0), self._p(self.h1), self._p(self.h2), self._p(self.z1),
                                     self._p(self.z2), self._p(self.z3), self._p(self.slab), self._p(self.loss),
                                     self._p(self.correct), s)
        else:
            self.ext.fused_train(self._p(self.train.images), self._p(self.train.labels), self._p(self.batch_ids),
                                 self.order_len, self.batch, self._p(self.state), self._p(self.master),
                                 self._p(self.shadow), self._p(self.a0), self._p(self.h1), self._p(self.h2),
                                 self._p(self.z1), self._p(self.z2), self._p(self.z3), self._p(self.slab),
                                 self._p(self.loss), self._p(self.correct), s,
                                 next_ids=self._p(self.next_ids) if self._staged else 0,
                                 stage=self._p(self.stage) if self._staged else 0)
        if self.grad_sync is None:
            self._reduce(1, 0, LAYOUT.total, 1, s)
            return
        if getattr(self.grad_sync, "fuses_sgd", False):
            grp = self.grad_sync.group
            if grp.one_launch:
                # one-launch all-reduce: each reduction block reduces its elements over the
                # batch, exchanges them with the same block of every peer over xGMI (1 hop)
                # and applies the averaged momentum-SGD update + bf16 images itself
                self._reduce(1, 0, LAYOUT.total, 1, s, **grp.exchange())
                return
            # two launches: batch reduction -> grad; one-shot xGMI all-reduce kernel [publish,
            # 1 hop, rank-order sum, momentum SGD, bf16 weight images] (parallel/xgmi.py)
            self._reduce(0, 0, LAYOUT.total, 1, s)
            grp.allreduce_sgd(self.grad, self.master, self.mom, self.shadow, self.lr, self.momentum, LAYOUT.total)
            return
        mlp, conv = LAYOUT.mlp_range, LAYOUT.conv_range
        if self.overlap:
            # MLP bucket (95% of the bytes) is reduced first; its all-reduce runs on the
            # comm stream while the conv bucket is being reduced on the compute stream.
            self._reduce(0, mlp[0], mlp[1], 1, s)
            self.grad_sync.allreduce_grads(self.grad, [mlp, conv],
                                           before_last=lambda: self._reduce(0, conv[0], conv[1], 0, self._stream()))
        else:
            self._reduce(0, 0, LAYOUT.total, 1, s)
            self.grad_sync.allreduce_grads(self.grad, [(0, LAYOUT.total)])
        self.ext.sgd_apply(self._p(self.master), self._p(self.grad), self._p(self.mom), self._p(self.shadow),
                           LAYOUT.total, self.lr, self.momentum, 1.0, 0, self._stream())

    def selftest_exchange(self, grp, comm, steps: int = 2) -> bool:
        """Collective: does the one-launch all-reduce (``grp.exchange()``) reproduce the
        two-launch path (batch reduce, then the xGMI all-reduce kernel) BIT FOR BIT on every
        rank?  Random per-rank reduction inputs, both parity slots; the engine's parameters,
        optimizer state and buffers are restored afterwards.  Every rank returns the same vote.
        The ranks vote after EACH pass and stop together at the first failure; a pass that
        raised or timed out anywhere marks the group ``broken`` (its step counters may differ
        across ranks from then on)."""
        dev = self.device
        bufs = [self.a0, self.h1, self.h2, self.z1, self.z2, self.z3, self.slab]
        saved = [t.clone() for t in bufs + [self.master, self.mom, self.shadow]]
        gen = torch.Generator().manual_seed(1009 + 7 * comm.rank)
        with torch.no_grad():
            for t in bufs:
                t.copy_(torch.randn(t.shape, generator=gen))
            # arena padding stays zero, as in training (the two-launch kernel updates every
            # element of its slices, the exchange only the real parameters)
            real = LAYOUT.pad_mask().float()
            p0 = (torch.randn(self.master.shape, generator=torch.Generator().manual_seed(3)) * 0.1 * real).to(dev)
            m0 = (torch.randn(self.master.shape, generator=torch.Generator().manual_seed(4)) * 0.01 * real).to(dev)
        results, why = [], ""
        timeout, grp.timeout_s = grp.timeout_s, min(grp.timeout_s, 10.0)
        # bf16 granules: the two-launch kernel's form of the same exchange is the reference
        # (its own code: element pairs (e, e + 256) instead of the reduce lanes' tile rows)
        ar_mode = grp.ar_mode
        if grp.xp_mode & 4:
            grp.ar_mode = grp.xp_mode
        ok = True
        for one_launch in (False, True):
            err = False
            try:
                with torch.cuda.device(dev):
                    self.master.copy_(p0)
                    self.mom.copy_(m0)
                    self.params_changed()
                    s = self._stream()
                    for _ in range(steps):
                        if one_launch:
                            self._reduce(1, 0, LAYOUT.total, 0, s, **grp.exchange())
                        else:
                            self._reduce(0, 0, LAYOUT.total, 0, s)
                            grp.allreduce_sgd(self.grad, self.master, self.mom, self.shadow, self.lr,
                                              self.momentum, LAYOUT.total)
                    torch.cuda.synchronize(dev)
                    err = grp.failed()
                    why = "wait failed" if err else why
                    results.append((self.master.cpu(), self.mom.cpu(), self.shadow.cpu()))
            except Exception as e:
                err = True
                why = f"{type(e).__name__}: {e}"
            # (every rank) done with these slots before they are reused; stop together
            if any(v != 0.0 for v in comm.gather_scalars(1.0 if err else 0.0)):
                grp.broken = True
                ok = False
                break
        grp.timeout_s = timeout
        grp.ar_mode = ar_mode
        if ok:
            same = all(torch.equal(x, y) for x, y in zip(*results))
            why = "" if same else "mismatch in " + str(
                [name for name, (x, y) in zip(("master", "mom", "shadow"), zip(*results)) if not torch.equal(x, y)])
            ok = same
        if not ok and os.environ.get("DNN_DEBUG_XGMI") == "1":
            print(f"[xgmi] rank {comm.rank}: exchange self-test: {why}", file=sys.stderr, flush=True)
        votes = comm.gather_scalars(1.0 if ok else 0.0)
        with torch.no_grad():
            for t, v in zip(bufs + [self.master, self.mom, self.shadow], saved):
                t.copy_(v)
        torch.cuda.synchronize(dev)
        return all(v == 1.0 for v in votes)

    def selftest_pers_exchange(self, grp, comm, steps: int = 3) -> tuple[bool, str]:
        """Collective: do ``steps`` training steps with the exchange INSIDE the persistent launch
        give the serial one-launch exchange's parameters, momentum and bf16 images BIT FOR BIT on
        every rank?  Both runs start from the same parameters and the same sample order (this
        rank's first ``steps`` batches of the attached split), launched eagerly.  Everything the
        runs touch - parameters, optimizer state, epoch cursor and order, bookkeeping slots, the
        image stage, epoch statistics - is restored afterwards, so it can run mid-epoch (the
        start-up A/B).  Returns (every rank passed, this rank's reason if not)."""
        avail = self.train is not None and self.persist and (
            self.dtype == "fp32" or (self.pipeline and self.stage is not None))
        if not all(v == 1.0 for v in comm.gather_scalars(1.0 if avail else 0.0)):  # (same collectives everywhere)
            return False, "the persistent launch is not available on " + ("this rank" if not avail else "a peer")
        dev = self.device
        keep = [t for t in (self.master, self.mom, self.shadow, self.state, self.stats, self.batch_ids, self.next_ids,
                            self.next_ids2, self.stage) if t is not None]
        saved = [t.clone() for t in keep]
        saved_attrs = (self.order_len, self._staged, self._ahead, self.pers_exchange)
        saved_order = self.order[:self.order_len].clone()
        n = min(len(self.train), steps * self.batch)
        order = np.arange(n, dtype=np.int32)
        results, why, ok = [], "", True
        timeout, grp.timeout_s = grp.timeout_s, min(grp.timeout_s, 10.0)
        for pers in (False, True):
            err = False
            try:
                with torch.cuda.device(dev), torch.no_grad():
                    self.master.copy_(saved[0])
                    self.mom.copy_(saved[1])
                    self.params_changed()
                    self.pers_exchange = pers
                    self.invalidate_graphs()
                    self.begin_epoch(order)
                    if pers != self._pers_ok():
                        raise RuntimeError("the persistent exchange form did not engage")
                    self._launch_steps(steps)
                    torch.cuda.synchronize(dev)
                    err = grp.failed() or self.pipe_failed()
                    why = "a wait failed" if err else why
                    results.append((self.master.cpu(), self.mom.cpu(), self.shadow.cpu()))
            except Exception as e:
                err, why = True, f"{type(e).__name__}: {e}"
            if any(v != 0.0 for v in comm.gather_scalars(1.0 if err else 0.0)):
                grp.broken = True
                ok = False
                break
        grp.timeout_s = timeout
        if ok:
            same = all(torch.equal(x, y) for x, y in zip(*results))
            why = "" if same else "mismatch in " + str(
                [k for k, (x, y) in zip(("master", "mom", "shadow"), zip(*results)) if not torch.equal(x, y)])
            ok = same
        votes = comm.gather_scalars(1.0 if ok else 0.0)
        with torch.no_grad():
            self.order_len, self._staged, self._ahead, self.pers_exchange = saved_attrs
            if self.order_len:
                self.order[:self.order_len].copy_(saved_order)
            for t, v in zip(keep, saved):
                t.copy_(v)
            if hasattr(self, "pipe_err"):
                self.pipe_err.zero_()
        self.invalidate_graphs()
        torch.cuda.synchronize(dev)
        return all(v == 1.0 for v in votes), why

    def _launch_key(self, nsteps: int) -> tuple:
        return (nsteps, id(self.grad_sync), self.overlap, self.order_len,
                getattr(getattr(self.grad_sync, "group", None), "one_launch", None),
                getattr(getattr(self.grad_sync, "group", None), "xp_mode", None), self._staged, self._pipe_ok(),
                self._pers_ok(), self.pers_exchange)

    _direct_checked: dict = {}  # device index -> the direct path passed its self-test in this process

    def _direct_ok(self) -> bool:
        return self.direct and self.grad_sync is None and self._pers_ok()

    def _direct(self, nsteps: int) -> int:
        """The prepared direct dispatch of an nsteps persistent launch (the graph's counterpart:
        the same launch, arguments fixed once)."""
        key = (self._launch_key(nsteps), self._stream())
        h = self._direct_h.get(key)
        if h is None:
            with torch.cuda.device(self.device):
                if not HipEngine._direct_checked.get(self.device.index, False):
                    # the path end to end on a trivial kernel first (bounded: 5 s), once per device
                    why = self.ext.aql_selftest()
                    if why:
                        raise RuntimeError(why)
                    HipEngine._direct_checked[self.device.index] = True
                h = self._launch_steps_pers(nsteps, direct=True)
            if h is None or h < 0:
                raise RuntimeError("the persistent launcher did not prepare a direct dispatch")
            self._direct_h[key] = h
        return h

    def _direct_or_off(self, nsteps: int) -> int | None:
        """_direct, or None after turning the direct path off if preparing it failed (nothing was
        dispatched: the graph replays take over, and the reason is printed and kept in direct_why)."""
        try:
            return self._direct(nsteps)
        except RuntimeError as e:
            self.direct, self.direct_why = False, f"preparing a direct dispatch failed: {e}"
            print(f"[engine] {self.direct_why}; using graph replays", file=sys.stderr, flush=True)
            return None

    def _graph(self, nsteps: int) -> torch.cuda.CUDAGraph:
        key = self._launch_key(nsteps)
        g = self._graphs.get(key)
        if g is None:
            # Capture advances nothing: kernels are recorded, not run.  The wait before it is
            # interruptible: queued replays may hold collectives on a dead peer
            self._wait()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=self.stream):
                self._launch_steps(nsteps)
            torch.cuda.synchronize(self.device)
            self._graphs[key] = g
        return g

    def _chunk_sizes(self) -> list[int]:
        sizes, k = [], 1
        while k <= self.graph_chunk:
            sizes.append(k)
            k *= 2
        return sizes[::-1]

    def prepare_graphs(self, exact: tuple[int, ...] = ()) -> None:
        """Capture every chunk graph up front (capture is not free: keep it out of timed loops).
        ``exact``: step counts that also get a graph of their own, so ``run_steps(n)`` for such
        an n is ONE replay instead of its power-of-two decomposition (a 20-step window: one
        graph instead of 16 + 4, ~6 us less per window; profiles/r2/window/)."""
        if self._direct_ok():  # direct dispatches replace the graphs (run_steps takes them first)
            if all(self._direct_or_off(k) is not None
                   for k in sorted(set(self._chunk_sizes()) | {int(k) for k in exact if 0 < int(k)})):
                return
        if self.use_graphs:
            for k in self._chunk_sizes():
                self._graph(k)
            self._exact = {int(k) for k in exact if 0 < int(k)}
            for k in self._exact:
                self._graph(k)

    def run_steps(self, n: int, host_work=None) -> None:
        """Queue n training steps.  host_work: a host-only callable to run while they run (the
        next epoch's shuffle): with the direct dispatch, which returns only when its steps are
        done, it overlaps the kernel instead of following it."""
        if n <= 0:
            if host_work is not None:
                host_work()
            return
        poll = self.poll
        if self._direct_ok():  # ONE direct dispatch, returning when the n steps are done
            h = self._direct_or_off(n)
            if h is not None:
                if poll is not None:
                    poll()
                if host_work is None:
                    self.ext.persist_direct_run(h)
                    return
                self.ext.persist_direct_launch(h)
                try:
                    host_work()
                finally:
                    self.ext.persist_direct_wait(h)
                return
        self._run_steps_graphs(n, poll)
        if host_work is not None:
            host_work()

    def _run_steps_graphs(self, n: int, poll) -> None:
        if not self.use_graphs:
            with torch.cuda.device(self.device):
                if self._pipe_ok() or self._pers_ok():
                    if poll is not None:
                        poll()
                    self._launch_steps(n)
                    return
                for _ in range(n):
                    if poll is not None:
                        poll()
                    self._launch_step()
            return
        if n in getattr(self, "_exact", ()):
            if poll is not None:
                poll()
            self._graph(n).replay()
            return
        # binary decomposition over power-of-two chunk graphs: <= log2(chunk)+n/chunk replays
        for k in self._chunk_sizes():
            reps, n = divmod(n, k)
            if reps:
                g = self._graph(k)
                for _ in range(reps):
                    if poll is not None:
                        poll()
                    g.replay()

    def step_wait_failed(self) -> bool:
        """Did an in-launch wait of this engine's step time out (sticky error word)?"""
        return self.pipe_failed()

    def degrade(self) -> str | None:
        """Step down one level after a StepWaitTimeout, from the step form that actually ran
        (ADVICE r5): persistent -> pipelined -> serial (each bit-identical to the next).  With a
        per-step all-reduce the persistent form is the "-pers" exchange; it steps down to the
        serial one-launch exchange (the pipelined step has no all-reduce form).  Clears the sticky
        error word and the cached graphs; returns the new level, or None if the engine already
        runs the serial step (nothing to step down to: the caller re-raises)."""
        if self._pers_ok():
            self.persist = False
            self.pers_exchange = False
            level = ("pipelined" if self._pipe_ok() else
                     "serial (one-launch exchange)" if self.grad_sync is not None else "serial")
        elif self._pipe_ok():
            self.pipeline = False
            level = "serial"
        else:
            return None
        if hasattr(self, "pipe_err"):
            self.pipe_err.zero_()
        self.invalidate_graphs()
        return level

    def epoch_stats(self, reset: bool = True) -> StepStats:
        v = self.stats.cpu().tolist()
        if self.pipe_failed():
            raise StepWaitTimeout("pipelined / persistent step: a ready or arrival wait timed out (a reduction or "
                                  "sample workgroup did not see its hand-off in time)")
        if reset:
            self.stats.zero_()
        return StepStats(v[0], int(round(v[1])), int(round(v[2])), int(round(v[3])))

    # -- evaluation -----------------------------------------------------------------------
    def evaluate_samples(self, split: Split, lo: int = 0, hi: int | None = None):
        """Per-sample test loss/correct for samples [lo, hi) of ``split`` (one launch)."""
        split = split.to(self.device)
        hi = len(split) if hi is None else hi
        n = max(0, hi - lo)
        loss = torch.zeros(n, device=self.device, dtype=torch.float32)
        corr = torch.zeros(n, device=self.device, dtype=torch.int32)
        if n:
            with torch.cuda.device(self.device):
                if self.dtype == "fp32":
                    self.ext.fused_eval_f32(self._p(split.images), self._p(split.labels), hi, lo, n,
                                            self._p(self.master), self._p(loss), self._p(corr), self._stream())
                else:
                    self.ext.fused_eval(self._p(split.images), self._p(split.labels), 0, hi, lo, n,
                                        self._p(self.master), self._p(self.shadow), self._p(loss), self._p(corr),
                                        self._stream())
        return loss, corr


ENGINES = ("auto", "fused", "layers")


def make_engine(device: str, batch: int, lr: float, momentum: float, arena: torch.Tensor | None = None,
                seed: int | None = None, model: str = "lenet", engine: str = "auto", dtype: str = "bf16",
                **kw) -> Engine:
    """Pick the engine for (model, device, dtype).

    * ``fused``  - the reference LeNet as ONE hand-scheduled gfx950 kernel per step (+ the
      batch reduction): bf16 MFMA operands / fp32 accumulation (lenet_fused.hip, the
      performance path) or fp32 throughout (lenet_f32.hip, the reference's arithmetic); GPU only.
    * ``layers`` - any zoo model on the generic layer kernels (runtime/layer_engine.py),
      fp32 or bf16 GEMM operands, BatchNorm support; CPU or GPU.
    * ``auto``   - fused for lenet on a GPU, the CPU oracle engine for lenet on the CPU,
      layers otherwise.
    """
    if engine not in ENGINES:
        raise ValueError(f"unknown engine {engine!r}; expected one of {ENGINES}")
    if engine == "auto":
        if model == "lenet" and device == "cpu":
            return CpuEngine(batch, lr, momentum, arena, seed)
        engine = "fused" if model == "lenet" else "layers"
    if engine == "fused":
        if model != "lenet":
            raise ValueError(f"the fused engine implements the reference lenet only, not {model!r}")
        if device == "cpu":
            return CpuEngine(batch, lr, momentum, arena, seed)
        return HipEngine(batch, lr, momentum, arena, seed, device=device, dtype=dtype, **kw)
    from .layer_engine import LayerEngine
    lkw = {k: v for k, v in kw.items() if k in ("use_graphs", "graph_chunk")}
    return LayerEngine(batch, lr, momentum, model=model, arena=arena, seed=seed, device=device,
                       gemm_dtype=dtype, **lkw)
