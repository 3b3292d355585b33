"""EnvironmentConfig and the single-env HeistEnvironment (reference: environment.py).

HeistEnvironment keeps the reference's class API name for name (set_layout, reset,
step, get_state_tensor, is_level_valid, get_architect_reward,
get_environment_state, render_text and the attributes callers read), but every
tick runs on the GPU through a one-env HeistEnv; the Python side only mirrors the
state the reference exposes as attributes.  Batched training uses HeistEnv directly.
"""
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .components.budget import BUDGET_COSTS, BudgetManager
from .components.security import Camera, Guard, Wall
from .components.visibility import DynamicVisibilityMap
from .utils import TileType, create_empty_grid, grid_to_text, manhattan_distance
from .vec_env import STATUS_NAMES, HeistEnv


@dataclass
class EnvironmentConfig:  # environment.py:18-37
    grid_rows: int = 20
    grid_cols: int = 20
    max_steps: int = 200
    start_pos: Tuple[int, int] = (1, 1)
    vault_pos: Tuple[int, int] = None
    architect_budget: int = 15
    reward_vault: float = 10.0
    reward_detection: float = -1.0
    reward_step: float = -0.01
    reward_architect_detect: float = 1.0
    reward_architect_invalid: float = -1.0

    def __post_init__(self):
        if self.vault_pos is None:
            self.vault_pos = (self.grid_rows - 2, self.grid_cols - 2)


def accept_layout(walls, cameras, guards, cfg: EnvironmentConfig, budget: int):
    """The placements set_layout accepts (environment.py:102-152: walls and cameras on
    interior EMPTY tiles, guards unchecked at patrol_path[0], each while the budget
    lasts) as the reference's Wall / Camera / Guard objects, plus the resulting grid.
    Host bookkeeping for frames and attributes; heist_set_layout does the same on the GPU."""
    R, C = cfg.grid_rows, cfg.grid_cols
    g = create_empty_grid(R, C)
    g[cfg.start_pos] = TileType.START
    g[cfg.vault_pos] = TileType.VAULT
    b = BudgetManager(total_budget=budget)
    ok = lambda r, c: 0 < r < R - 1 and 0 < c < C - 1 and g[r, c] == TileType.EMPTY  # noqa: E731
    ws, cs, gs = [], [], []
    for r, c in walls:
        if ok(r, c) and b.purchase("wall"):
            g[r, c] = TileType.WALL
            ws.append(Wall(r, c))
    for cd in cameras:
        r, c = cd["row"], cd["col"]
        if ok(r, c) and b.purchase("camera"):
            g[r, c] = TileType.CAMERA
            cs.append(Camera(row=r, col=c, fov_angle=cd.get("fov_angle", 60.0), heading=cd.get("heading", 0.0),
                             rotation_speed=cd.get("rotation_speed", 15.0), vision_range=cd.get("vision_range", 6)))
    for gd in guards:
        path = gd["patrol_path"]
        if path and b.purchase("guard"):
            gu = Guard(patrol_path=list(path), speed=gd.get("speed", 1), vision_range=gd.get("vision_range", 4),
                       fov_angle=gd.get("fov_angle", 90.0))
            g[gu.row, gu.col] = TileType.GUARD
            gs.append(gu)
    return ws, cs, gs, g


class HeistEnvironment:
    """The reference's single-environment API backed by the GPU kernels."""

    ACTIONS = {0: (0, 0), 1: (-1, 0), 2: (1, 0), 3: (0, -1), 4: (0, 1)}  # environment.py:52-58
    ACTION_NAMES = {0: "WAIT", 1: "UP", 2: "DOWN", 3: "LEFT", 4: "RIGHT"}
    NUM_SOLVER_ACTIONS = 5

    def __init__(self, config: Optional[EnvironmentConfig] = None, device=None, max_cams: int = 16,
                 max_guards: int = 8, max_path: int = 64):
        self.config = config or EnvironmentConfig()
        cfg = self.config
        self._vec = HeistEnv(1, cfg, max_cams=max_cams, max_guards=max_guards, max_path=max_path, device=device,
                             auto_reset=False)
        self.grid = create_empty_grid(cfg.grid_rows, cfg.grid_cols)
        self.grid[cfg.start_pos] = TileType.START
        self.grid[cfg.vault_pos] = TileType.VAULT
        self.walls: List[Wall] = []
        self.cameras: List[Camera] = []
        self.guards: List[Guard] = []
        self.visibility_map = DynamicVisibilityMap(cfg.grid_rows, cfg.grid_cols)
        self.budget = BudgetManager(total_budget=cfg.architect_budget)
        self.solver_pos = cfg.start_pos
        self.tick = 0
        self.done = False
        self.solver_detected = False
        self.vault_reached = False
        self._prev_dist = manhattan_distance(cfg.start_pos, cfg.vault_pos)
        self._initial_dist = self._prev_dist
        self.solver_path: List[Tuple[int, int]] = [self.solver_pos]
        self.detection_events: List[Dict] = []
        self._state = None

    # -- Architect phase ---------------------------------------------------------
    def set_layout(self, walls: List[Tuple[int, int]], cameras: List[Dict], guards: List[Dict]) -> bool:
        """environment.py:102-152; placement and budget run in heist_set_layout."""
        valid = bool(self._vec.set_layouts([(list(walls), list(cameras), list(guards))],
                                           budget=self.budget.total_budget)[0].item())
        st = self._vec.export(grid=True)
        self.grid = st["grid"][0].cpu().numpy().astype(np.int32)
        self._mirror_layout(walls, cameras, guards)
        self.budget.spent = int(st["spent"][0].item())
        if (len(self.walls), len(self.cameras), len(self.guards)) != (int(st["n_walls"][0]), int(st["n_cams"][0]),
                                                                     int(st["n_guards"][0])):
            raise RuntimeError("host layout mirror disagrees with the device placement")
        return valid

    def _mirror_layout(self, walls, cameras, guards):
        """Rebuild the reference's Wall/Camera/Guard lists with its acceptance rules."""
        self.walls, self.cameras, self.guards, _ = accept_layout(walls, cameras, guards, self.config,
                                                                 self.budget.total_budget)

    def is_level_valid(self) -> bool:  # environment.py:154-158
        from .utils import bfs_path_exists
        return bfs_path_exists(self.grid, self.config.start_pos, self.config.vault_pos)

    # -- Solver phase ---------------------------------------------------------------
    def _pull(self):
        st = self._vec.export()
        s = {k: int(v[0].item()) for k, v in st.items() if v.dim() == 1}
        self.solver_pos = (s["pos_r"], s["pos_c"])
        self.tick = s["tick"]
        self.done = bool(s["done"])
        self.solver_detected = bool(s["detected"])
        self.vault_reached = bool(s["vault_reached"])
        self._prev_dist = s["prev_dist"]
        self._initial_dist = s["initial_dist"]
        ch = st["cam_heading"][0].cpu().numpy()
        for k, cam in enumerate(self.cameras):
            cam.heading = float(ch[k])
        gi = st["guard_idx"][0].cpu().numpy()
        gh = st["guard_heading"][0].cpu().numpy()
        for k, g in enumerate(self.guards):
            g.current_idx = int(gi[k])
            g.heading = float(gh[k])
        self._state = self._vec.obs[0].cpu().numpy()
        self.visibility_map._record(self._state[1])

    def reset(self) -> Dict[str, np.ndarray]:  # environment.py:183-214
        self.visibility_map.reset()
        self._vec.reset()
        self._pull()
        self.solver_path = [self.solver_pos]
        self.detection_events = []
        return self._get_observation()

    def step(self, action: int):  # environment.py:216-299
        if self.done:
            return self._get_observation(), 0.0, True, {"status": "already_done"}
        info = {"status": "running", "tick": self.tick}
        self._vec.step(torch.tensor([int(action)]), auto_reset=False)
        reward = float(self._vec.reward64[0].item())
        info["status"] = STATUS_NAMES[int(self._vec.status[0].item())]
        tick_before = self.tick
        self._pull()
        self.solver_path.append(self.solver_pos)
        if self.solver_detected:  # only this tick can set it: a done env never gets here
            self.detection_events.append({"tick": tick_before, "position": self.solver_pos})
        return self._get_observation(), reward, self.done, info

    # -- observations ---------------------------------------------------------------
    def _get_observation(self) -> Dict[str, np.ndarray]:  # environment.py:305-345
        cfg = self.config
        rows, cols = cfg.grid_rows, cfg.grid_cols
        occupancy = self.grid.astype(np.float32) / max(TileType.GUARD, 1)
        return {
            "occupancy_grid": occupancy,
            "visibility_map": self.visibility_map.visibility.copy(),
            "solver_position": np.array([self.solver_pos[0] / rows, self.solver_pos[1] / cols], dtype=np.float32),
            "vault_direction": np.array([(cfg.vault_pos[0] - self.solver_pos[0]) / rows,
                                         (cfg.vault_pos[1] - self.solver_pos[1]) / cols], dtype=np.float32),
            "time_feature": np.array([self.tick / cfg.max_steps], dtype=np.float32),
        }

    def get_state_tensor(self) -> np.ndarray:  # environment.py:347-374
        """The [3, R, C] float32 state the GPU wrote for the current tick."""
        if self._state is None:
            self._vec.reset()
            self._pull()
        return self._state.copy()

    # -- info & rendering -------------------------------------------------------------
    def get_architect_reward(self) -> float:  # environment.py:380-386
        if not self.is_level_valid():
            return self.config.reward_architect_invalid
        if self.solver_detected:
            return self.config.reward_architect_detect
        return 0.0

    def get_environment_state(self) -> Dict[str, Any]:  # environment.py:388-417
        return {
            "grid": self.grid.tolist(),
            "visibility": self.visibility_map.visibility.tolist(),
            "solver_pos": self.solver_pos,
            "solver_path": self.solver_path,
            "vault_pos": self.config.vault_pos,
            "start_pos": self.config.start_pos,
            "tick": self.tick,
            "done": self.done,
            "cameras": [{"row": c.row, "col": c.col, "heading": c.heading, "fov_angle": c.fov_angle,
                         "vision_range": c.vision_range} for c in self.cameras],
            "guards": [{"row": g.row, "col": g.col, "heading": g.heading, "patrol_path": g.patrol_path,
                        "current_idx": g.current_idx} for g in self.guards],
            "detection_events": self.detection_events,
        }

    def render_text(self) -> str:  # environment.py:419-421
        return grid_to_text(self.grid, self.solver_pos)

    def __repr__(self):
        return "HeistEnvironment(grid=%dx%d, cameras=%d, guards=%d, walls=%d, tick=%d)" % (
            self.config.grid_rows, self.config.grid_cols, len(self.cameras), len(self.guards), len(self.walls),
            self.tick)
