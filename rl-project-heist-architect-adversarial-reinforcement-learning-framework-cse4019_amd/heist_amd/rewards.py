"""Architect/Solver episode rewards (reference: heist_architect/rewards.py)."""
from typing import Dict


class RewardCalculator:  # rewards.py:10-111
    def __init__(self, config=None):
        self.config = config or {}
        c = self.config
        self.architect_detect = c.get("architect_detect", 1.0)
        self.architect_invalid = c.get("architect_invalid", -1.0)
        self.architect_vault_fail = c.get("architect_vault_fail", -0.5)
        self.architect_difficulty_bonus = c.get("architect_difficulty_bonus", 0.2)
        self.solver_vault = c.get("solver_vault", 10.0)
        self.solver_detected = c.get("solver_detected", -1.0)
        self.solver_step = c.get("solver_step", -0.01)
        self.solver_timeout = c.get("solver_timeout", -0.5)

    def architect_reward_from_rate(self, level_valid: bool, solve_rate: float) -> float:
        """calculate_architect_reward (rewards.py:43-73) given the validity bit."""
        if not level_valid:
            return self.architect_invalid
        reward = 0.0
        reward += (1.0 - solve_rate) * self.architect_detect
        if solve_rate > 0.8:
            reward += self.architect_vault_fail
        if 0.2 <= solve_rate <= 0.6:
            reward += self.architect_difficulty_bonus
        return reward

    def calculate_architect_reward(self, env, solve_rate: float = 0.0) -> float:
        return self.architect_reward_from_rate(env.is_level_valid(), solve_rate)

    def calculate_solver_episode_reward(self, env) -> float:  # rewards.py:75-98
        reward = 0.0
        if env.vault_reached:
            reward += self.solver_vault
        if env.solver_detected:
            reward += self.solver_detected
        if env.tick >= env.config.max_steps and not env.vault_reached:
            reward += self.solver_timeout
        return reward

    def get_reward_summary(self) -> Dict[str, float]:
        return {k: getattr(self, k) for k in ("architect_detect", "architect_invalid", "architect_vault_fail",
                                              "architect_difficulty_bonus", "solver_vault", "solver_detected",
                                              "solver_step", "solver_timeout")}
