"""Experiment tracking: a local run object with neptune-like series, written as JSONL.

Capability parity: the reference logs ``run["parameters"]`` and the series
``train/loss``, ``val/loss``, ``val/acc`` to neptune.ai (single_proc_train.py:20-26,
78, 100-101; data_parallelism_train.py:106-112, 180-181, 250).  There is no network
or credential on the target machines (and the reference leaks a hard-coded token
that must never be copied), so the same API writes to a local JSONL file instead:

    run = Run("metrics.jsonl"); run["parameters"] = {...}; run["train/loss"].append(x)

Every record carries a wall-clock timestamp; ``Run.record`` adds free-form per-epoch
records (throughput, phase breakdown, world size, recovery events).
"""
from __future__ import annotations

import json
import os
import time
from typing import Any


class _Series:
    def __init__(self, run: "Run", name: str) -> None:
        self.run, self.name, self.values = run, name, []

    def append(self, value: Any) -> None:
        v = float(value) if isinstance(value, (int, float)) or hasattr(value, "__float__") else value
        self.values.append(v)
        self.run._emit({"series": self.name, "step": len(self.values) - 1, "value": v})


class Run:
    def __init__(self, path: str | None = None, enabled: bool = True) -> None:
        self.path = path
        self.enabled = enabled and path is not None
        self._series: dict[str, _Series] = {}
        self._fields: dict[str, Any] = {}
        if self.enabled:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
            self._fh = open(path, "a")

    def _emit(self, rec: dict) -> None:
        if self.enabled:
            rec = {"t": time.time(), **rec}
            self._fh.write(json.dumps(rec) + "\n")
            self._fh.flush()

    def __getitem__(self, name: str) -> _Series:
        if name not in self._series:
            self._series[name] = _Series(self, name)
        return self._series[name]

    def __setitem__(self, name: str, value: Any) -> None:
        self._fields[name] = value
        self._emit({"field": name, "value": value})

    def record(self, **kw: Any) -> None:
        self._emit({"record": kw})

    def stop(self) -> None:
        if self.enabled:
            self._fh.close()
            self.enabled = False
