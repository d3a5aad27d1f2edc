from . import checkpoint, logfiles, metrics, roctx, timers

__all__ = ["checkpoint", "logfiles", "metrics", "roctx", "timers"]
