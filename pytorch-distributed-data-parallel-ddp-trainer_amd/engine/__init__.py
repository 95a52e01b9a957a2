from .fused_step import FusedSimpleCNNEngine, EngineOptions
from .graph_step import GraphedStep

__all__ = ["FusedSimpleCNNEngine", "EngineOptions", "GraphedStep"]
