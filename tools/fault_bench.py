"""Rank-drop recovery benchmark (BASELINE.json config 5: "8x MI355X with 1-rank fault-tolerance
drop + communicator re-form").

It launches ``data_parallelism_train.py`` on N ranks (one per GPU; ``--share-gpu`` puts every rank
on GPU 0 over gloo, a one-GPU rehearsal). One rank is killed hard mid-epoch (``--drop-rank``).
The survivors detect the failure, agree on the new group, re-form the communicator, restore the
last consistent parameters, re-partition the data and redo the epoch. Every rank's output is
streamed as it happens, each line stamped with the seconds since launch, to stderr and to
``--log`` (a hang shows where it sits; ``DNN_FAULTHANDLER_S`` makes every rank dump its thread
stacks periodically). The tool then reads the run's JSONL metrics and prints ONE JSON line:

  detect_s            kill (the victim's own clock stamp, just before os._exit) -> the first
                      survivor's watchdog flag (launcher death notice / stale heartbeat / RCCL
                      async error) or failed collective
  recovery_s          survivor side, error caught -> re-formed group passed its barrier
                      (stages_s: abort / agree / reform / reattach / barrier)
  time_to_resume_s    kill -> the first optimizer step on the re-formed group completed
  img_per_s_before / _after, epoch_s_before / _after, world_before / _after, total_wall_s

usage: python tools/fault_bench.py [-n 8] [--share-gpu] [--epochs 3] [--drop-rank 1]
       [--drop-at-epoch 1] [--drop-at-step 2] [--train-samples 50000] [--batch-size 64]
       [--allreduce default|ab|xgmi-pull|rccl] [--log gpurun_out/fault.log]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", type=int, default=8)
    ap.add_argument("--share-gpu", action="store_true", help="every rank on GPU 0, gloo host collectives")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--drop-rank", type=int, default=1)
    ap.add_argument("--drop-at-epoch", type=int, default=1)
    ap.add_argument("--drop-at-step", type=int, default=2)
    ap.add_argument("--train-samples", type=int, default=50_000)
    ap.add_argument("--test-samples", type=int, default=10_000)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--sync", default="step-allreduce")
    ap.add_argument("--allreduce", default="default",
                    help="step-allreduce transport of the run: default | ab | xgmi-pull | xgmi-rsag | rccl | "
                         "rccl-overlap (rccl exercises ncclCommAbort + re-init with a real dead peer)")
    ap.add_argument("--device", default="cuda", help="cuda (default) | cpu (plumbing check without a GPU)")
    ap.add_argument("--timeout", type=int, default=900)
    ap.add_argument("--log", default=None, help="also write the stamped per-rank output here")
    ap.add_argument("--no-check-sync", dest="check_sync", action="store_false",
                    help="skip the cross-rank parameter checksum after every sync (default: on, so the survivors' "
                         "parameters are asserted bit-identical after the re-form)")
    a = ap.parse_args()
    env = dict(os.environ, PYTHONPATH=ROOT, DNN_FAULT_TRACE="1")
    env.setdefault("DNN_FAULTHANDLER_S", "60")
    if a.device == "cpu":
        env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    elif a.share_gpu:  # every rank maps to GPU 0 (local rank mod the visible devices); RCCL refuses that
        env.update(DNN_BACKEND="gloo", HIP_VISIBLE_DEVICES="0", OMP_NUM_THREADS="2")
    logf = open(a.log, "w") if a.log else None
    lines: list[str] = []
    with tempfile.TemporaryDirectory() as tmp:
        metrics = os.path.join(tmp, "m.jsonl")
        cmd = [sys.executable, "-u", "-m", "distributed_neural_network_amd.parallel.launch", "-n", str(a.n),
               os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", str(a.epochs), "--batch-size",
               str(a.batch_size), "--sync", a.sync, "--drop-rank", str(a.drop_rank), "--drop-at-epoch",
               str(a.drop_at_epoch), "--drop-at-step", str(a.drop_at_step), "--train-samples", str(a.train_samples),
               "--test-samples", str(a.test_samples), "--device", a.device, "--nb-proc", str(a.n), "--metrics",
               metrics, "--allreduce", a.allreduce] + (["--check-sync"] if a.check_sync else [])
        t0 = time.perf_counter()
        p = subprocess.Popen(cmd, cwd=tmp, env=dict(env, PYTHONUNBUFFERED="1"), stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, text=True, bufsize=1)

        def pump() -> None:
            for ln in p.stdout:
                stamped = f"[{time.perf_counter() - t0:8.3f}] {ln.rstrip()}"
                lines.append(ln)
                print(stamped, file=sys.stderr, flush=True)
                if logf:
                    logf.write(stamped + "\n")
                    logf.flush()

        th = threading.Thread(target=pump, daemon=True)
        th.start()
        try:
            rc = p.wait(timeout=a.timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            rc = -9
        th.join(timeout=5)
        wall = time.perf_counter() - t0
        if rc != 0:
            return rc if rc > 0 else 1
        recs = [json.loads(ln)["record"] for ln in open(metrics) if '"record"' in ln]
    recov = [x for x in recs if x.get("event") == "recovery"]
    resumed = [x for x in recs if x.get("event") == "resumed"]
    epochs = [x for x in recs if "img_per_s" in x]
    if not recov or not epochs:
        sys.stderr.write("no recovery / epoch records in the metrics file\n")
        return 1
    drop = [x for x in recov if x["dead"]]
    rv = drop[0] if drop else recov[0]
    kill = None
    for ln in lines:
        m = re.search(r"injected drop: rank \d+ exits at epoch \d+ step \d+ \(t=([0-9.]+)\)", ln)
        if m:
            kill = float(m.group(1))
    t_det = rv.get("t_detected") or rv.get("t_error")
    res = next((x for x in resumed if x.get("generation") == rv["generation"]), None)
    before = [e for e in epochs if e["epoch"] < rv["epoch"]]
    after = [e for e in epochs if e["epoch"] >= rv["epoch"]]
    out = {"metric": "rank-drop recovery: detection, re-form and resume latency + throughput before/after "
                     "(BASELINE config 5)",
           "n_ranks": a.n, "share_gpu": a.share_gpu, "allreduce": a.allreduce, "dropped": rv["dead"],
           "generation": rv["generation"], "all_alive_retries": len([x for x in recov if not x["dead"]]),
           "check_sync": a.check_sync,
           "detect_s": round(t_det - kill, 4) if kill and t_det else None,
           "recovery_s": round(rv["recovery_s"], 4), "stages_s": rv.get("stages_s"),
           "time_to_resume_s": round(res["t_resumed"] - kill, 4) if kill and res else None,
           "world_before": before[-1]["world"] if before else None, "world_after": after[0]["world"] if after else None,
           "img_per_s_before": round(before[-1]["img_per_s"], 1) if before else None,
           "img_per_s_after": round(after[0]["img_per_s"], 1) if after else None,
           "epoch_s_before": round(before[-1]["epoch_s"], 4) if before else None,
           "epoch_s_after": round(after[0]["epoch_s"], 4) if after else None,
           "epochs_completed": len(epochs), "total_wall_s": round(wall, 2),
           "config": {"sync": a.sync, "per_gpu_batch": a.batch_size, "train_samples": a.train_samples,
                      "drop_at": [a.drop_at_epoch, a.drop_at_step]}}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
