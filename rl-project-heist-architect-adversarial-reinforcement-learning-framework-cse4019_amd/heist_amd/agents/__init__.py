from .architect import ArchitectAgent
from .solver import Rollout, SolverAgent

__all__ = ["ArchitectAgent", "SolverAgent", "Rollout"]
