"""One-hop xGMI all-reduce for the per-step gradient (csrc/comm/xgmi_allreduce.hip and the
one-launch exchange in csrc/kernels/reduce_sgd.hip).

Why a second collective path next to RCCL: the step-allreduce gradient is 248 KB, so the
collective is pure latency.  RCCL's ring (or tree) walks 2 (N-1) dependent hops over
single links; an 8x MI355X node is a full xGMI mesh, so one hop suffices: every rank
publishes its gradient in an IPC-shared region as {value, step} granules (one 64-bit word
per element) and reads the same elements from all N regions over the 7 links at once,
until every tag shows the current step.  The sum runs in rank order (replicas stay
bit-identical), is scaled by 1/N and feeds the momentum-SGD update in the same launch - it
replaces ``ncclAllReduce`` + ``sgd_apply`` inside the captured step graph.  With the fused
engine the exchange runs inside the batch-reduction kernel itself (``exchange()``): one
launch for reduce + all-reduce + SGD.

Scope: one node (all ranks share the xGMI mesh), 1..8 ranks, a GPU engine.  At set-up the
group runs a self-test (random data, both parity slots, exact against a host rank-order
sum) and every rank votes through the process group; if any rank fails (IPC refused,
wrong sums, timeout), every rank falls back to the native RCCL path together.  The engine
then checks the one-launch exchange against the two-launch path (``HipEngine.
selftest_exchange``).  RCCL stays the transport for everything else (broadcast, epoch
averaging, eval metrics).

Fault tolerance: every granule wait is bounded (timeout, plus a host-mapped abort word the
fault watchdog sets through ``Communicator.signal_lost``); a failed wait sets a sticky
device error word instead of hanging, and ``check()`` raises ``CommError`` at the next
epoch boundary, which the trainer's recovery path handles like any other comm failure.
After ``Communicator.reform`` the group is rebuilt over the survivors.
"""
from __future__ import annotations

import itertools
import os
import socket
import sys

import torch

from ..ops import native
from .comm import CommError, Communicator

MAX_RANKS = 8
MAX_SHARED = 2  # ranks that may time-share one GPU and still use the exchange (rehearsals / tests)
_ids = itertools.count()


def _local_world() -> int | None:
    """Ranks on this node according to the launcher (torchrun, OpenMPI, MPICH/Intel MPI,
    Slurm); None when no launcher says.  Only a hint: ``build_group`` decides single-node
    from a hostname all-gather through the store, which every launcher supports."""
    for name in ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS"):
        v = os.environ.get(name)
        if v:
            return int(v)
    v = os.environ.get("SLURM_NTASKS_PER_NODE", "")
    if v.isdigit():
        return int(v)
    return None


def wanted(comm: Communicator) -> bool:
    """xGMI path requested and applicable (DNN_ALLREDUCE=rccl forces RCCL)."""
    choice = os.environ.get("DNN_ALLREDUCE", "xgmi")
    if choice not in ("xgmi", "rccl"):
        raise ValueError(f"DNN_ALLREDUCE must be xgmi or rccl, not {choice!r}")
    if choice != "xgmi" or comm.device.type != "cuda" or not comm.distributed:
        return False
    if comm.world > MAX_RANKS:
        return False
    local = _local_world()
    return local is None or local >= comm.env.world  # launcher says multi-node: RCCL


def one_launch_wanted() -> bool:
    """The fused engine's one-launch exchange (DNN_XGMI_ONE_LAUNCH=0 keeps two launches)."""
    v = os.environ.get("DNN_XGMI_ONE_LAUNCH", "1")
    if v not in ("0", "1"):
        raise ValueError(f"DNN_XGMI_ONE_LAUNCH must be 0 or 1, not {v!r}")
    return v == "1"


# xp_mode / all-reduce kernel form: bit 2 = two-hop, bit 4 = bf16 granules (a lane's elements
# travel in pairs as {bf16 | bf16, step} words: half the link bytes; every rank sums the same
# bf16-rounded gradients in fp32, rank order - opt-in lower-precision communication, like a
# bf16 compression hook, never chosen unless asked for: ``--grad-comm bf16``)
EXCHANGE_MODES = {"pull": 0, "rsag": 2, "pull-bf16": 4, "rsag-bf16": 6}
MODE_NAMES = {v: k for k, v in EXCHANGE_MODES.items()}


def exchange_mode(grp: "XgmiGroup | None" = None) -> int:
    """``xp_mode`` of the one-launch exchange from ``DNN_XGMI_EXCHANGE``: pull (0: one hop, E
    granules per link) or rsag (2: two-hop pull - reduce-scatter + all-gather where every rank
    writes only its own region, 2 E / N granules per link, one more dependent remote read).
    auto (default) = pull; the multi-GPU bench measures both (parallel/autotune.py) and keeps
    the faster.  With several ranks time-sharing ONE GPU the two-hop form's two-level wait (the
    owner's sum needs every peer's block to have run first) stalls for seconds when the GPU
    time-slices the processes (profiles/r2/push/); the pull form has no failure seen in any
    setup."""
    choice = os.environ.get("DNN_XGMI_EXCHANGE", "auto")
    if choice != "auto" and choice not in EXCHANGE_MODES:
        raise ValueError(f"DNN_XGMI_EXCHANGE must be auto or one of {sorted(EXCHANGE_MODES)}, not {choice!r}")
    return 0 if choice == "auto" else EXCHANGE_MODES[choice]


def wait_timeout(comm: Communicator) -> float:
    """Bound of one granule wait.  A live straggler (``--failure-duration`` sleeps before its
    epoch) must not be mistaken for a dead peer: the bound covers the longest injected
    sleep twice over, plus the base minute."""
    base = float(os.environ.get("DNN_XGMI_TIMEOUT_S", "60"))
    return base + 2.0 * float(getattr(comm, "straggler_s", 0.0) or 0.0)


class XgmiGroup:
    """IPC-mapped regions of every rank + the per-rank launch state."""

    def __init__(self, comm: Communicator, capacity: int, timeout_s: float | None = None,
                 device_ids: list[str] | None = None) -> None:
        assert comm.store is not None
        self.comm = comm
        self.ext = native.hip()
        self.capacity = int(capacity)
        self.timeout_s = wait_timeout(comm) if timeout_s is None else float(timeout_s)
        self.rank, self.world = comm.rank, comm.world
        self.generation = comm.generation
        self.opened: list[int] = []
        self.local = 0
        self.abort_host = 0
        try:
            self._setup(comm, device_ids)
        except BaseException:
            self.close()  # a half-built group must not leak peer mappings, its region or the abort word
            raise

    def _setup(self, comm: Communicator, device_ids: list[str] | None) -> None:
        from .fault import setup_crash_injection

        setup_crash_injection("xgmi-setup", comm.orig_rank)  # (tests: the launcher's retry path)
        dev = comm.device
        self.abort_host, self.abort_dev = self.ext.xgmi_abort_word()
        nb = self.ext.xgmi_max_blocks(self.capacity)
        self.ctr = torch.zeros(nb + 1, device=dev, dtype=torch.int32)  # [per-slice steps | error word]
        # per-block step counters of the one-launch exchange inside grad_reduce (flag table B)
        self.xp_ctr = torch.zeros(self.ext.xgmi_xp_max_blocks(), device=dev, dtype=torch.int32)
        # set once the exchange matched the two-launch path bit for bit on every rank
        # (HipEngine.selftest_exchange, run by the step-allreduce policy)
        self.one_launch = False
        # set when a self-test pass raised or timed out on some rank: the per-block step counters
        # may then be out of step across ranks, so the group must be rebuilt before any use
        self.broken = False
        self.xp_mode = 0  # one-launch exchange form (EXCHANGE_MODES, self-tested): 0 pull, 2 rsag, + 4 bf16
        self.ar_mode = 0  # form of the all-reduce kernel (build_group: exchange_mode + self-test)
        # per-step exchange-wait records (ReduceArgs::xp_wait): [ring][block][wave] words of
        # {step << 32 | ticks}; None = not recorded (enable_wait_stats)
        self.wait: torch.Tensor | None = None
        key = f"dnn/xgmi/g{comm.generation}/i{next(_ids)}"
        # every rank publishes SOMETHING (an empty handle on failure), so no peer blocks
        # on a key that never comes
        handle, err = b"", None
        try:
            with torch.cuda.device(dev):
                self.local, handle, self.kind = self.ext.xgmi_alloc(self.capacity)
        except Exception as e:
            err = e
        comm.store.set(f"{key}/h{self.rank}", handle)
        handles = [comm.store.get(f"{key}/h{r}") for r in range(self.world)]
        if err is not None:
            raise err
        bad = [r for r, h in enumerate(handles) if not h]
        if bad:
            raise CommError(f"rank(s) {bad} could not export an xGMI region")
        regions = []
        with torch.cuda.device(dev):
            for r in range(self.world):
                if r == self.rank:
                    regions.append(self.local)
                    continue
                p = self.ext.xgmi_open(handles[r])
                self.opened.append(p)
                regions.append(p)
        self.regions = regions
        # Every shared byte moves as part of a {value, step} granule written and read with
        # single 64-bit system-scope atomics (csrc/comm/xgmi_layout.h): a reader that sees the
        # step sees the value, so the hand-off needs no flag and no fence on any topology.
        self.devices = len(set(device_ids)) if device_ids else 1

    # -- launches --------------------------------------------------------------------------
    def exchange(self) -> dict:
        """grad_reduce kwargs of the one-launch all-reduce: every reduction lane publishes its
        reduced elements as {value, step} granules, reads the same elements' granules from
        every peer and applies the averaged update itself (no separate all-reduce launch, no
        hand-off inside the GPU, no flag: the step tag travels in the value's atomic word)."""
        err = self.ctr.data_ptr() + 4 * (self.ctr.numel() - 1)  # the same sticky error word
        return dict(xp_regions=list(self.regions), xp_rank=self.rank, xp_capacity=self.capacity,
                    xp_ctr=self.xp_ctr.data_ptr(), xp_err=err, xp_abort=self.abort_dev,
                    xp_timeout_s=self.timeout_s, xp_scale=1.0 / self.world, xp_mode=self.xp_mode,
                    xp_wait=self._wait_ptr())

    # -- exchange-wait accounting ---------------------------------------------------------------
    def _wait_ptr(self) -> int:
        return 0 if self.wait is None else self.wait.data_ptr()

    def enable_wait_stats(self, on: bool = True) -> None:
        """Record every step's exchange wait (per wave: the longest lane wait, s_memrealtime
        ticks) in a device ring.  One plain store per wave and step; launches captured into
        graphs before this call do not record (re-capture after toggling)."""
        if on and self.wait is None:
            ring, blocks, waves = self.ext.xgmi_wait_ring()
            self.wait = torch.zeros(ring * blocks * waves, device=self.comm.device, dtype=torch.int64)
        elif not on:
            self.wait = None

    def reset_wait_stats(self) -> None:
        if self.wait is not None:
            self.wait.zero_()

    def wait_stats(self) -> dict | None:
        """Per-step exchange wait over the recorded steps (max over this rank's blocks and
        waves), in microseconds: {steps, median, p99, max}.  None when nothing was recorded."""
        if self.wait is None:
            return None
        ring, blocks, waves = self.ext.xgmi_wait_ring()
        w = self.wait.view(ring, blocks * waves).cpu()
        steps = (w >> 32) & 0xffffffff
        ticks = (w & 0xffffffff).double()
        valid = steps.max(dim=1).values > 0
        if not bool(valid.any()):
            return None
        # per ring entry: the longest wait among the words of the entry's newest step
        newest = steps.max(dim=1, keepdim=True).values
        per_step = torch.where(steps == newest, ticks, torch.zeros_like(ticks)).max(dim=1).values[valid]
        us = per_step / 100.0  # 100 MHz ticks -> us
        q = torch.quantile(us, torch.tensor([0.5, 0.99], dtype=torch.float64))
        return {"steps": int(us.numel()), "median": round(float(q[0]), 3), "p99": round(float(q[1]), 3),
                "max": round(float(us.max()), 3)}

    def clear_error(self) -> None:
        """Reset the sticky error word (only after every rank's kernels have drained)."""
        self.ctr[-1].zero_()

    def allreduce_sgd(self, grad: torch.Tensor, master: torch.Tensor, mom: torch.Tensor, shadow: torch.Tensor | None,
                      lr: float, momentum: float, n: int | None = None) -> None:
        """grad <- avg over ranks; momentum SGD on master/mom (+ bf16 shadow images)."""
        n = grad.numel() if n is None else n
        s = torch.cuda.current_stream(grad.device).cuda_stream
        mode = 1 if shadow is not None else 2
        self.ext.xgmi_allreduce(self.regions, self.rank, self.capacity, n, grad.data_ptr(), grad.data_ptr(),
                                master.data_ptr(), mom.data_ptr(), shadow.data_ptr() if shadow is not None else 0,
                                lr, momentum, 1.0 / self.world, mode, self.ctr.data_ptr(), self.abort_dev,
                                self.timeout_s, s, self.ar_mode, self._wait_ptr())

    def allreduce_(self, t: torch.Tensor) -> None:
        """In-place average of a flat fp32 tensor."""
        assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() <= self.capacity
        s = torch.cuda.current_stream(t.device).cuda_stream
        self.ext.xgmi_allreduce(self.regions, self.rank, self.capacity, t.numel(), t.data_ptr(), t.data_ptr(),
                                0, 0, 0, 0.0, 0.0, 1.0 / self.world, 0, self.ctr.data_ptr(), self.abort_dev,
                                self.timeout_s, s, self.ar_mode, 0)

    # -- health ------------------------------------------------------------------------------
    def failed(self) -> bool:
        if self.comm.watch is not None:
            self.comm.wait_device()  # the D2H read below must not block on a stuck peer
        return bool(self.ctr[-1].item())

    def check(self) -> None:
        if self.failed():
            raise CommError("xGMI all-reduce: a peer did not publish within the timeout (or the group was aborted)")

    def abort(self) -> None:
        """Release every spinning wait (called from the fault watchdog thread)."""
        if self.abort_host:
            self.ext.xgmi_set_abort(self.abort_host, 1)

    def preflight(self, timeout_s: float = 5.0) -> tuple[bool, str]:
        """A tiny bounded round trip over every peer mapping before anything larger uses them:
        rank r publishes 2**r in 64 granules and reads every peer's, so the rank-order sum must be
        exactly 2**N - 1 (times fp32(1/N)).  A mapping that faults aborts this process HERE, in
        set-up (the launcher then retries without xGMI, parallel/selflaunch.py); one that returns
        stale or foreign data times out within ``timeout_s`` or sums wrong, and the caller turns
        that into a voted refusal.  Returns (ok, why) - why names the peers whose contribution is
        missing."""
        dev = self.comm.device
        timeout, self.timeout_s = self.timeout_s, min(self.timeout_s, timeout_s)
        try:
            with torch.cuda.device(dev):
                t = torch.full((64,), float(1 << self.rank), device=dev, dtype=torch.float32)
                self.allreduce_(t)
                got = t.cpu()
                err = self.failed()
        finally:
            self.timeout_s = timeout
        inv = torch.tensor(1.0 / self.world, dtype=torch.float32)
        want = torch.tensor(float((1 << self.world) - 1), dtype=torch.float32) * inv
        if not err and bool((got == want).all()):
            return True, ""
        v = float(got[0])
        seen = int(round(v * self.world)) if v == v and abs(v) < 1e6 else -1
        missing = [r for r in range(self.world) if seen < 0 or not (seen >> r) & 1]
        return False, ("a granule wait timed out; " if err else "") + f"missing / wrong peer contributions: {missing}"

    def selftest(self, steps: int = 4) -> bool:
        """``steps`` all-reduces of random per-rank data (both parity slots, fresh flags),
        checked EXACTLY against the rank-order fp32 sum every rank recomputes on the host
        from the shared seeds (the kernel adds in rank order, then scales by fp32(1/N))."""
        dev = self.comm.device
        n = min(self.capacity, 62_400)
        ok = True
        timeout, self.timeout_s = self.timeout_s, min(self.timeout_s, 10.0)
        inv = torch.tensor(1.0 / self.world, dtype=torch.float32)
        with torch.cuda.device(dev):
            for it in range(steps):
                xs = [torch.randn(n, generator=torch.Generator().manual_seed(7919 * it + r)) * (r + 1)
                      for r in range(self.world)]
                t = xs[self.rank].to(dev)
                self.allreduce_(t)
                want = xs[0].clone()
                for x in xs[1:]:
                    want += x
                want *= inv
                ok = ok and bool(torch.equal(t.cpu(), want)) and not self.failed()
        self.timeout_s = timeout
        return ok

    def close(self) -> None:
        for p in self.opened:
            try:
                self.ext.xgmi_close(p)
            except Exception:
                pass
        self.opened = []
        if self.local:
            self.ext.xgmi_free(self.local)
            self.local = 0
        if self.abort_host:
            self.ext.xgmi_free_abort_word(self.abort_host)
            self.abort_host = 0


def _topology(comm: Communicator) -> tuple[bool, list[str]]:
    """Collective: (all ranks on this host?, physical device id per rank).  Every rank reads
    every rank's entry, so all reach the same decision (no launcher variable needed)."""
    assert comm.store is not None
    key = f"dnn/xgmi/g{comm.generation}/topo{next(_ids)}"
    try:
        with torch.cuda.device(comm.device):
            dev_id = native.hip().xgmi_device_id()
    except Exception:
        dev_id = f"?{comm.rank}"
    comm.store.set(f"{key}/{comm.rank}", f"{socket.gethostname()}|{dev_id}")
    entries = [comm.store.get(f"{key}/{r}").decode() for r in range(comm.world)]
    hosts = {e.split("|", 1)[0] for e in entries}
    return len(hosts) == 1, [e for e in entries]


def build_group(comm: Communicator, capacity: int) -> XgmiGroup | None:
    """Collective: every rank builds + self-tests the group, and all agree on the outcome."""
    single_node, device_ids = _topology(comm)
    if not single_node:
        if comm.rank == 0:
            print("[xgmi] ranks span several hosts: per-step all-reduce over RCCL", file=sys.stderr, flush=True)
        return None
    per_dev = max(device_ids.count(d) for d in device_ids)
    if per_dev > MAX_SHARED and os.environ.get("DNN_XGMI_SHARED_OK") != "1":
        # The exchange's waits assume every rank's kernels make progress.  Ranks time-sharing
        # one GPU compete for its CUs: with >2 of them, the blocks spinning in their exchange
        # can hold enough CUs that a peer's fused kernel (1 workgroup per CU, whole register
        # file) cannot be dispatched - a stall until the wait bound (profiles/r3/fault_bench/).
        # One process per GPU (the product setup) never shares.
        if comm.rank == 0:
            print(f"[xgmi] {per_dev} ranks share one GPU: exchange progress is not guaranteed there; "
                  f"per-step all-reduce over the process group", file=sys.stderr, flush=True)
        return None
    grp, ok, why = None, True, ""
    try:
        grp = XgmiGroup(comm, capacity, device_ids=device_ids)
    except Exception as e:  # IPC export/import refused, etc.
        ok, why = False, f"{type(e).__name__}: {e}"
    # agree that every rank mapped every region BEFORE any rank launches a kernel that waits for
    # peers; then a tiny bounded round trip over every mapping (pre-flight), agreed on too, before
    # the full self-test - and long before any engine kernel polls the regions
    mapped = all(v == 1.0 for v in comm.gather_scalars(1.0 if ok else 0.0))
    if ok and not mapped:
        ok, why = False, "a peer could not map the regions"
    if mapped:
        pre, pre_why = False, ""
        try:
            pre, pre_why = grp.preflight()
        except Exception as e:
            pre_why = f"{type(e).__name__}: {e}"
        if not all(v == 1.0 for v in comm.gather_scalars(1.0 if pre else 0.0)):
            ok, why = False, f"pre-flight round trip failed ({pre_why or 'on a peer'})"
        else:
            try:
                ok = grp.selftest()
                why = "" if ok else "self-test mismatch"
            except Exception as e:
                ok, why = False, f"{type(e).__name__}: {e}"
    votes = comm.gather_scalars(1.0 if ok else 0.0)
    if os.environ.get("DNN_DEBUG_XGMI") == "1":
        print(f"[xgmi] gen {comm.generation} rank {comm.rank}/{comm.world} ok={ok} {why} votes={votes} "
              f"regions={[hex(r) for r in grp.regions] if grp is not None and ok else None} "
              f"kind={getattr(grp, 'kind', None)} devices={getattr(grp, 'devices', None)}", file=sys.stderr, flush=True)
    if all(v == 1.0 for v in votes):
        # the all-reduce kernel's two-hop form where it is wanted, kept only if its own exact
        # self-test passes on every rank
        mode = exchange_mode(grp) & 2  # (bf16 granules: only with their one-launch exchange)
        if mode != 0:
            grp.ar_mode = mode
            try:
                ok = grp.selftest()
            except Exception:
                ok = False
            if not all(v == 1.0 for v in comm.gather_scalars(1.0 if ok else 0.0)):
                grp.ar_mode = 0
                if comm.rank == 0:
                    print(f"[xgmi] all-reduce form {mode} failed its self-test: pull form", file=sys.stderr, flush=True)
        return grp
    if grp is not None:
        grp.close()
    if comm.rank == 0 or not ok:
        print(f"[xgmi] one-shot all-reduce unavailable on rank(s) "
              f"{[i for i, v in enumerate(votes) if v != 1.0]} ({why or 'peer failed'}); using RCCL",
              file=sys.stderr, flush=True)
    return None


class XgmiGradSync:
    """GradSync whose all-reduce also applies the optimizer (``fuses_sgd``)."""

    fuses_sgd = True

    def __init__(self, group: XgmiGroup) -> None:
        self.group = group

    def allreduce_sgd(self, grad, master, mom, shadow, lr, momentum, n=None) -> None:
        self.group.allreduce_sgd(grad, master, mom, shadow, lr, momentum, n)

    def allreduce_grads(self, grad: torch.Tensor, buckets, before_last=None) -> None:
        if before_last is not None:
            before_last()
        self.group.allreduce_(grad)

    def check(self) -> None:
        self.group.check()

    def failed(self) -> bool:
        return self.group.failed()


__all__ = ["XgmiGroup", "XgmiGradSync", "build_group", "exchange_mode", "one_launch_wanted", "wanted"]
