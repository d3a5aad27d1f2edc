from .comm import CommError, Communicator, GradAllReduce
from .env import DistEnv, detect
from .sync import SYNC_MODES, EpochAverage, ParentAverage, StepAllReduce, SyncPolicy, make_policy

__all__ = ["CommError", "Communicator", "GradAllReduce", "DistEnv", "detect", "SYNC_MODES", "EpochAverage",
           "ParentAverage", "StepAllReduce", "SyncPolicy", "make_policy"]
