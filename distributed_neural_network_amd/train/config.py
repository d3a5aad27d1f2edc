"""Typed configuration + argparse for the three reference entrypoints.

Capability parity (reference flags and defaults):

  entrypoint                  bs  epochs  lr     momentum  other
  single_proc_train.py         4  15      0.001  0.9       (hard-coded in the reference)
  model_replication_train.py  16  10      0.001  0.9       --lr --momentum --batch-size --epochs
  data_parallelism_train.py   16  25      0.001  0.9       + --nb-proc 4 --failure-probability 0.0
                                                             --failure-duration 0.0

Every reference flag keeps its name and default, but is TYPED (the reference's untyped
argparse crashes on ``--lr 0.01`` / ``--batch-size 8`` from the CLI; quirk §2.7 #7).
New flags: --sync, --device, --data, --data-root, --seed, --save, --resume,
--drop-rank/--drop-at-epoch/--drop-at-step, --overlap, --compat, --profile,
--metrics, --log-dir, --graph-chunk, --train-samples/--test-samples, --eval-sharded,
--model, --engine, --dtype, --check-sync, --allreduce.
"""
from __future__ import annotations

import argparse
import os
from dataclasses import dataclass, field
from typing import Optional

from ..models.zoo import MODELS
from ..parallel.sync import SYNC_MODES
from ..runtime.engine import ENGINES

DEFAULTS = {
    "single": dict(batch_size=4, epochs=15, sync="step-allreduce"),
    "replication": dict(batch_size=16, epochs=10, sync="epoch-avg"),
    "data-parallel": dict(batch_size=16, epochs=25, sync="epoch-avg"),
}


@dataclass
class TrainConfig:
    mode: str = "data-parallel"          # single | replication | data-parallel
    lr: float = 0.001
    momentum: float = 0.9
    batch_size: int = 16
    epochs: int = 25
    nb_proc: int = 4                     # file-name only, as in the reference
    failure_probability: float = 0.0
    failure_duration: float = 0.0
    sync: str = "epoch-avg"
    device: str = "auto"                 # auto | cpu | cuda | cuda:N
    data: str = "synthetic"              # synthetic | cifar10
    data_root: str = "./data"
    train_samples: Optional[int] = None
    test_samples: Optional[int] = None
    seed: int = 0
    save: Optional[str] = None
    resume: Optional[str] = None
    drop_rank: Optional[int] = None
    drop_at_epoch: int = 0
    drop_at_step: int = 0
    overlap: bool = False
    compat: bool = False
    profile: bool = False
    metrics: Optional[str] = None
    log_dir: str = "log"
    write_logs: bool = True
    graph_chunk: int = 32
    eval_sharded: bool = True
    momentum_reset: Optional[bool] = None  # default: per policy (epoch-avg resets, like the reference)
    model: str = "lenet"
    engine: str = "auto"
    dtype: str = "bf16"
    check_sync: bool = False
    debug_sync: bool = False
    use_graphs: bool = True
    bucket_kb: int = 0
    allreduce: str = "default"           # step-allreduce transport: default | ab | a StepAllReduce.PATHS name
    grad_comm: str = "fp32"              # step-allreduce gradient communication precision: fp32 | bf16
    extra: dict = field(default_factory=dict)


def _common(ap: argparse.ArgumentParser, mode: str) -> None:
    d = DEFAULTS[mode]
    ap.add_argument("--lr", dest="lr", type=float, default=0.001)
    ap.add_argument("--momentum", dest="momentum", type=float, default=0.9)
    ap.add_argument("--batch-size", dest="batch_size", type=int, default=d["batch_size"])
    ap.add_argument("--epochs", dest="epochs", type=int, default=d["epochs"])
    g = ap.add_argument_group("MI355X framework options")
    g.add_argument("--sync", choices=SYNC_MODES, default=d["sync"],
                   help="epoch-avg: reference per-epoch model averaging (all ranks train); parent: exact "
                        "reference topology (rank 0 = non-training parameter server); step-allreduce: "
                        "per-step bucketed gradient all-reduce")
    g.add_argument("--device", default="auto", help="auto | cpu | cuda | cuda:N (auto: this rank's GPU if any)")
    g.add_argument("--data", choices=["synthetic", "synthetic-hard", "cifar10"], default="synthetic",
                   help="synthetic: learnable template + noise CIFAR-shaped set; synthetic-hard: maximal noise "
                        "(accuracy climbs over several epochs); cifar10: the binary batches under --data-root")
    g.add_argument("--data-root", default="./data", help="directory holding cifar-10-batches-bin/")
    g.add_argument("--train-samples", type=int, default=None, help="use only the first N training samples")
    g.add_argument("--test-samples", type=int, default=None, help="use only the first N test samples")
    g.add_argument("--seed", type=int, default=0)
    g.add_argument("--save", default=None, help="write a reference-format state_dict checkpoint here")
    g.add_argument("--resume", default=None, help="resume from a checkpoint written by --save")
    g.add_argument("--drop-rank", type=int, default=None, help="fault injection: this rank dies hard")
    g.add_argument("--drop-at-epoch", type=int, default=0)
    g.add_argument("--drop-at-step", type=int, default=0)
    g.add_argument("--no-overlap", dest="overlap", action="store_false", default=False,
                   help="one fused gradient bucket on the compute stream (the default)")
    g.add_argument("--emulate-parent", dest="sync", action="store_const", const="parent",
                   help="alias of --sync parent: rank 0 is the reference's non-training parameter server")
    g.add_argument("--overlap", dest="overlap", action="store_true",
                   help="step-allreduce: 2 gradient buckets, the MLP all-reduce overlapped with the conv-bucket "
                        "reduction on a side stream (default: one fused bucket, latency-optimal at 248 KB)")
    g.add_argument("--compat", action="store_true",
                   help="reproduce reference quirks (loss denominator 10*(N-1), rank-2-only children log)")
    g.add_argument("--profile", action="store_true", help="roctx ranges + per-epoch phase breakdown")
    g.add_argument("--metrics", default=None, help="JSONL metrics file (neptune-series replacement)")
    g.add_argument("--log-dir", default="log")
    g.add_argument("--graph-chunk", type=int, default=32, help="optimizer steps per captured hipGraph")
    g.add_argument("--no-eval-sharding", dest="eval_sharded", action="store_false")
    g.add_argument("--model", default="lenet", choices=sorted(MODELS),
                   help="lenet = the reference Network (models/model.py); lenet-bn / cifar-vgg: zoo models "
                        "with BatchNorm (layer engine)")
    g.add_argument("--engine", default="auto", choices=ENGINES,
                   help="fused: one gfx950 kernel per step (lenet, bf16); layers: generic layer kernels "
                        "(any model, fp32 or bf16); auto picks")
    g.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                   help="operand precision (fp32 accumulation always): bf16 MFMA operands, or fp32 throughout = "
                        "the reference's arithmetic (fused fp32 kernel for lenet, fp32 GEMMs in the layer engine)")
    g.add_argument("--bucket-kb", type=int, default=0,
                   help="step-allreduce: split the flat gradient into all-reduce buckets of at most this many "
                        "KB (0 = one fused bucket, latency-optimal for the 248 KB reference gradient)")
    g.add_argument("--allreduce", default="default",
                   choices=("default", "ab", "xgmi-pull-pers", "xgmi-rsag-pers", "xgmi-pull", "xgmi-rsag", "rccl",
                            "rccl-overlap", "xgmi-pull-bf16", "xgmi-rsag-bf16"),
                   help="step-allreduce transport: default (one-launch xGMI exchange on one node, else RCCL), "
                        "ab (time every candidate at start-up and keep the fastest; parallel/autotune.py) or a "
                        "path name")
    g.add_argument("--grad-comm", default="fp32", choices=["fp32", "bf16"],
                   help="step-allreduce gradient communication precision: fp32 (default) or bf16 = the xGMI "
                        "exchange carries bf16 gradient pairs per granule (half the link bytes; every rank sums "
                        "the same rounded values in fp32) - the default path becomes its -bf16 form and --allreduce "
                        "ab also times the -bf16 forms")
    g.add_argument("--check-sync", action="store_true",
                   help="after every synchronisation assert that all ranks hold bit-identical parameters "
                        "(cross-rank checksum)")
    g.add_argument("--debug-sync", action="store_true",
                   help="race / fault hunting: serialised kernel launches (AMD_SERIALIZE_KERNEL=3, "
                        "HIP_LAUNCH_BLOCKING=1), no hipGraphs, NCCL_DEBUG=INFO and --check-sync")


def parser(mode: str) -> argparse.ArgumentParser:
    desc = {"single": "single-process CNN training (reference single_proc_train.py)",
            "replication": "model replication: every rank trains on the full set, models averaged per epoch "
                           "(reference model_replication_train.py)",
            "data-parallel": "data parallelism: sharded data, models averaged per epoch or gradients per step "
                             "(reference data_parallelism_train.py)"}[mode]
    ap = argparse.ArgumentParser(description=desc)
    _common(ap, mode)
    if mode == "data-parallel":
        ap.add_argument("--nb-proc", dest="nb_proc", type=int, default=4)
        ap.add_argument("--failure-probability", dest="failure_probability", type=float, default=0.0,
                        help="Probability of simulated process failure at each epoch")
        ap.add_argument("--failure-duration", dest="failure_duration", type=float, default=0.0,
                        help="Duration of simulated process failure in seconds")
    return ap


def parse(mode: str, argv=None) -> TrainConfig:
    ns = parser(mode).parse_args(argv)
    cfg = TrainConfig(mode=mode)
    for k, v in vars(ns).items():
        setattr(cfg, k, v)
    if cfg.debug_sync:
        apply_debug_sync(cfg)
    return cfg


DEBUG_SYNC_ENV = {"AMD_SERIALIZE_KERNEL": "3", "HIP_LAUNCH_BLOCKING": "1", "NCCL_DEBUG": "INFO"}


def apply_debug_sync(cfg: TrainConfig) -> None:
    """--debug-sync: every kernel runs alone and the host waits for it, so a
    faulting or racing kernel is reported at its own launch; replicas are checksummed after every
    sync.  The HIP variables only act before the runtime initialises, which parse() precedes."""
    for k, v in DEBUG_SYNC_ENV.items():
        os.environ.setdefault(k, v)
    cfg.check_sync = True
    cfg.use_graphs = False
