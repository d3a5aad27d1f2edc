"""Rank-drop recovery benchmark (BASELINE.json config 5: "8x MI355X with 1-rank fault-tolerance
drop + communicator re-form").

It launches ``data_parallelism_train.py`` on N ranks (one per GPU; ``--share-gpu`` puts every rank
on GPU 0 over gloo, a one-GPU rehearsal). One rank is killed hard mid-epoch (``--drop-rank``).
The survivors then detect the failure, agree on the new group, re-form the communicator,
restore the last consistent parameters, re-partition the data and redo the epoch. The tool
reads the run's JSONL metrics and prints ONE JSON line:

  recovery_s                    detection is NOT included: from the failed collective to the
                                re-formed group (the trainer's own clock)
  img_per_s_before / _after     training throughput of the last clean epoch / the first epoch
                                on the re-formed group, whole job
  epoch_s_before / _after, world_before / _after, total_wall_s

usage: python tools/fault_bench.py [-n 8] [--share-gpu] [--epochs 3] [--drop-rank 1]
       [--drop-at-epoch 1] [--drop-at-step 2] [--train-samples 50000] [--batch-size 64]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
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
    ap.add_argument("--timeout", type=int, default=900)
    a = ap.parse_args()
    env = dict(os.environ, PYTHONPATH=ROOT)
    if a.share_gpu:  # every rank maps to GPU 0 (local rank mod the visible devices); RCCL refuses that
        env.update(DNN_BACKEND="gloo", HIP_VISIBLE_DEVICES="0", OMP_NUM_THREADS="2")
    with tempfile.TemporaryDirectory() as tmp:
        metrics = os.path.join(tmp, "m.jsonl")
        cmd = [sys.executable, "-m", "distributed_neural_network_amd.parallel.launch", "-n", str(a.n),
               os.path.join(ROOT, "data_parallelism_train.py"), "--epochs", str(a.epochs), "--batch-size",
               str(a.batch_size), "--sync", a.sync, "--drop-rank", str(a.drop_rank), "--drop-at-epoch",
               str(a.drop_at_epoch), "--drop-at-step", str(a.drop_at_step), "--train-samples", str(a.train_samples),
               "--test-samples", str(a.test_samples), "--device", "cuda", "--nb-proc", str(a.n), "--metrics",
               metrics]
        t0 = time.perf_counter()
        r = subprocess.run(cmd, cwd=tmp, env=env, capture_output=True, text=True, timeout=a.timeout)
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
            return r.returncode
        recs = [json.loads(ln)["record"] for ln in open(metrics) if '"record"' in ln]
    recov = [x for x in recs if x.get("event") == "recovery"]
    epochs = [x for x in recs if "img_per_s" in x]
    if not recov or not epochs:
        sys.stderr.write("no recovery / epoch records in the metrics file\n" + r.stdout[-3000:])
        return 1
    rv = recov[0]
    before = [e for e in epochs if e["epoch"] < rv["epoch"]]
    after = [e for e in epochs if e["epoch"] >= rv["epoch"]]
    out = {"metric": "rank-drop recovery: re-form latency + throughput before/after (BASELINE config 5)",
           "n_ranks": a.n, "share_gpu": a.share_gpu, "dropped": rv["dead"], "generation": rv["generation"],
           "recovery_s": round(rv["recovery_s"], 4),
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
