#!/usr/bin/env python3
"""Reference-compatible entrypoint `data_parallelism_train.py` (mode: data-parallel).

Same flags and defaults as the reference script (typed), plus the framework options
(--sync, --device, --data, --save/--resume, fault injection, ...); see
`python data_parallelism_train.py --help` and distributed_neural_network_amd/train/config.py.
Multi-process: `python -m distributed_neural_network_amd.parallel.launch -n N data_parallelism_train.py ...`,
torchrun, or mpiexec (one process per GPU).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_neural_network_amd.parallel.comm import exit_now_if_reaping  # noqa: E402
from distributed_neural_network_amd.train import main  # noqa: E402

if __name__ == "__main__":
    main("data-parallel")
    exit_now_if_reaping()  # a recovered run may still be tearing an aborted group down
