#!/usr/bin/env bash
# Batch-size sweep of the reference (run_training.sh: `mpiexec -n 4 python
# data_parallelism_train.py --nb-proc 4 --batch-size $bs` for bs in 1..64).
# One process per GPU; set NPROC to the number of GPUs (default 4).
set -euo pipefail
NPROC=${NPROC:-4}
for bs in 1 2 4 8 16 32 64
do
  python -m distributed_neural_network_amd.parallel.launch -n "$NPROC" data_parallelism_train.py \
      --nb-proc "$NPROC" --batch-size "$bs" "$@"
done
