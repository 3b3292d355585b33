"""Asset costs and the Architect's budget (reference: components/budget.py).

Host bookkeeping only; the per-env purchase gate of set_layout runs inside the
heist_set_layout kernel with the same rules.
"""
from dataclasses import dataclass
from typing import Dict

BUDGET_COSTS: Dict[str, int] = {"wall": 1, "camera": 3, "guard": 5}  # budget.py:13-17


@dataclass
class BudgetManager:  # budget.py:23-78
    total_budget: int = 15
    spent: int = 0

    @property
    def remaining(self) -> int:
        return self.total_budget - self.spent

    def can_afford(self, asset_type: str) -> bool:
        return self.remaining >= BUDGET_COSTS.get(asset_type, 0)

    def purchase(self, asset_type: str) -> bool:
        cost = BUDGET_COSTS.get(asset_type, 0)
        if cost == 0:
            return False
        if self.remaining >= cost:
            self.spent += cost
            return True
        return False

    def reset(self):
        self.spent = 0

    def scale_budget(self, new_budget: int):
        self.total_budget = new_budget
        self.spent = 0

    def get_affordable_assets(self) -> Dict[str, bool]:
        return {a: self.can_afford(a) for a in BUDGET_COSTS}

    def __repr__(self):
        return "Budget(remaining=%d/%d, affordable=%s)" % (self.remaining, self.total_budget, self.get_affordable_assets())
