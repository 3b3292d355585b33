"""Walls, rotating cameras and patrol guards (reference: components/security.py).

These are the reference's data classes.  Their vision cones are computed by the
GPU raycaster (heist_cones), which reproduces security.py:53-101 / :161-192 bit
for bit; update() keeps the reference's pose arithmetic for standalone use (the
batched environment updates poses on the GPU).
"""
import math
from dataclasses import dataclass, field
from typing import List, Tuple

import numpy as np


@dataclass
class Wall:  # security.py:16-23
    row: int
    col: int

    def __repr__(self):
        return "Wall(%d, %d)" % (self.row, self.col)


def _cone_tiles(kind, row, col, fov, heading, rng, grid_rows, grid_cols, walls) -> List[Tuple[int, int]]:
    """The visible tiles in the reference's list order (first visit by ray index, then by
    distance along the ray), from heist_cone_order's first-visit keys."""
    import torch
    from .. import _native as nat
    dev = nat.require_gpu()
    w = torch.as_tensor(np.ascontiguousarray(np.asarray(walls, dtype=np.uint8).reshape(1, grid_rows, grid_cols)), device=dev)
    meta = torch.tensor([[kind, row, col, rng]], dtype=torch.int32, device=dev)
    par = torch.tensor([[float(fov), float(heading)]], dtype=torch.float64, device=dev)
    keys = torch.empty((1, grid_rows, grid_cols), dtype=torch.int32, device=dev)  # uint32 bits
    nat.check(nat.lib().heist_cone_order(1, grid_rows, grid_cols, nat.ptr(w), nat.ptr(meta), nat.ptr(par),
                                         nat.ptr(keys), nat.stream(dev)), "heist_cone_order")
    k = keys[0].cpu().numpy().view(np.uint32).reshape(-1)
    hit = np.nonzero(k != 0xFFFFFFFF)[0]
    hit = hit[np.argsort(k[hit], kind="stable")]
    return [(int(i // grid_cols), int(i % grid_cols)) for i in hit]


@dataclass
class Camera:  # security.py:30-106
    row: int
    col: int
    fov_angle: float = 60.0
    heading: float = 0.0
    rotation_speed: float = 15.0
    vision_range: int = 6

    def update(self, tick: int = 1):
        self.heading = (self.heading + self.rotation_speed * tick) % 360.0

    def get_vision_cone_tiles(self, grid_rows: int, grid_cols: int, walls: np.ndarray) -> List[Tuple[int, int]]:
        """Visible tiles in the reference's order (security.py:53-101)."""
        return _cone_tiles(0, self.row, self.col, self.fov_angle, self.heading, self.vision_range, grid_rows,
                           grid_cols, walls)

    def __repr__(self):
        return "Camera(pos=(%d,%d), heading=%.0f°, fov=%.0f°, speed=%.0f°/tick, range=%d)" % (
            self.row, self.col, self.heading, self.fov_angle, self.rotation_speed, self.vision_range)


@dataclass
class Guard:  # security.py:113-197
    patrol_path: List[Tuple[int, int]] = field(default_factory=list)
    speed: int = 1
    current_idx: int = 0
    vision_range: int = 4
    fov_angle: float = 90.0
    heading: float = 0.0

    @property
    def row(self) -> int:
        return self.patrol_path[self.current_idx][0] if self.patrol_path else 0

    @property
    def col(self) -> int:
        return self.patrol_path[self.current_idx][1] if self.patrol_path else 0

    @property
    def position(self) -> Tuple[int, int]:
        return (self.row, self.col)

    def update(self, tick: int = 1):
        if not self.patrol_path or len(self.patrol_path) < 2:
            return
        old = self.current_idx
        self.current_idx = (self.current_idx + self.speed * tick) % len(self.patrol_path)
        dr = self.patrol_path[self.current_idx][0] - self.patrol_path[old][0]
        dc = self.patrol_path[self.current_idx][1] - self.patrol_path[old][1]
        if dr != 0 or dc != 0:
            self.heading = math.degrees(math.atan2(-dr, dc)) % 360.0

    def get_visible_tiles(self, grid_rows: int, grid_cols: int, walls: np.ndarray) -> List[Tuple[int, int]]:
        return _cone_tiles(1, self.row, self.col, self.fov_angle, self.heading, self.vision_range, grid_rows,
                           grid_cols, walls)

    def __repr__(self):
        return "Guard(pos=(%d,%d), path_len=%d, heading=%.0f°, range=%d)" % (
            self.row, self.col, len(self.patrol_path), self.heading, self.vision_range)
