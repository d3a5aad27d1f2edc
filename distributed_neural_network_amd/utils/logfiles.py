"""Reference-format timing logs (``log/*.txt``).

Capability parity: data_parallelism_train.py:103-104,123-129 (parent) and
:143-152 (children).  File names and line formats are kept byte-for-byte so log
scrapers and the report's tables keep working:

  log/bs{bs}_log_epochs{E}_proc{nb_proc}_parent.txt
      Eval data loading time: {s}
      Time spent on evaluation: {s}
      Time spent on parent communication and param sync: {s}
  log/bs{bs}_log_epochs{E}_proc{nb_proc}_children.txt
      Train data loading time: {s}
      Time spent on training: {s}
      Time spent on children communication: {s}

Unlike the reference, the ``log/`` directory is created if missing.
"""
from __future__ import annotations

import os


def log_name(bs: int, epochs: int, nb_proc: int, role: str) -> str:
    return f"bs{bs}_log_epochs{epochs}_proc{nb_proc}_{role}.txt"


def parent_lines(data_loading: float, evaluation: float, comm: float) -> list[str]:
    return [f"Eval data loading time: {data_loading}",
            f"Time spent on evaluation: {evaluation}",
            f"Time spent on parent communication and param sync: {comm}"]


def children_lines(data_loading: float, training: float, comm: float) -> list[str]:
    return [f"Train data loading time: {data_loading}",
            f"Time spent on training: {training}",
            f"Time spent on children communication: {comm}"]


def write_log(log_dir: str, name: str, lines: list[str]) -> str:
    os.makedirs(log_dir, exist_ok=True)
    path = os.path.join(log_dir, name)
    with open(path, "w") as f:
        for line in lines:
            f.write(line + "\n")
    return path


def read_log(path: str) -> dict[str, float]:
    out = {}
    with open(path) as f:
        for line in f:
            if ":" in line:
                k, v = line.rsplit(":", 1)
                out[k.strip()] = float(v)
    return out
