from .engine import CpuEngine, Engine, HipEngine, StepStats, eval_metrics, make_engine

__all__ = ["CpuEngine", "Engine", "HipEngine", "StepStats", "eval_metrics", "make_engine"]
