from .engine import ENGINES, CpuEngine, Engine, HipEngine, StepStats, StepWaitTimeout, eval_metrics, make_engine
from .layer_engine import LayerEngine

__all__ = ["ENGINES", "CpuEngine", "Engine", "HipEngine", "LayerEngine", "StepStats", "StepWaitTimeout", "eval_metrics",
           "make_engine"]
