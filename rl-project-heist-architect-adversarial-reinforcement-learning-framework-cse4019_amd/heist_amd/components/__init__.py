from .security import Wall, Camera, Guard
from .visibility import DynamicVisibilityMap
from .budget import BudgetManager, BUDGET_COSTS

__all__ = ["Wall", "Camera", "Guard", "DynamicVisibilityMap", "BudgetManager", "BUDGET_COSTS"]
