from .comm import CommError, Communicator, GradAllReduce
from .env import DistEnv, detect
from .sync import (SYNC_MODES, EpochAverage, ParentAverage, StepAllReduce, SyncPolicy, assert_replicas_identical,
                   make_policy, replica_checksums)

__all__ = ["CommError", "Communicator", "GradAllReduce", "DistEnv", "detect", "SYNC_MODES", "EpochAverage",
           "ParentAverage", "StepAllReduce", "SyncPolicy", "assert_replicas_identical", "make_policy",
           "replica_checksums"]
