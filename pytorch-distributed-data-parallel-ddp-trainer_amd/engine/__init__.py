from .fused_step import FusedSimpleCNNEngine, EngineOptions

__all__ = ["FusedSimpleCNNEngine", "EngineOptions"]
