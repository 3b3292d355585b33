"""Tile types, grid helpers and the layout-validity BFS (reference: heist_architect/utils.py).

bfs_path_exists runs the wave-level bitboard flood fill on the GPU
(heist_bfs_valid); there is no CPU fallback.
"""
from typing import List, Optional, Tuple

import numpy as np
import torch


def get_device() -> torch.device:
    """utils.py:15-23: the compute device (HIP if present)."""
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


DEVICE = get_device()


class TileType:  # utils.py:31-37
    EMPTY = 0
    WALL = 1
    START = 2
    VAULT = 3
    CAMERA = 4
    GUARD = 5


TILE_NAMES = {TileType.EMPTY: "Empty", TileType.WALL: "Wall", TileType.START: "Start",
              TileType.VAULT: "Vault", TileType.CAMERA: "Camera", TileType.GUARD: "Guard"}


def manhattan_distance(a: Tuple[int, int], b: Tuple[int, int]) -> int:  # utils.py:122-124
    return abs(a[0] - b[0]) + abs(a[1] - b[1])


def create_empty_grid(rows: int, cols: int) -> np.ndarray:  # utils.py:131-139
    grid = np.full((rows, cols), TileType.EMPTY, dtype=np.int32)
    grid[0, :] = TileType.WALL
    grid[-1, :] = TileType.WALL
    grid[:, 0] = TileType.WALL
    grid[:, -1] = TileType.WALL
    return grid


_SYMBOLS = {TileType.EMPTY: ".", TileType.WALL: "#", TileType.START: "S", TileType.VAULT: "V",
            TileType.CAMERA: "C", TileType.GUARD: "G"}


def grid_to_text(grid: np.ndarray, solver_pos: Optional[Tuple[int, int]] = None) -> str:  # utils.py:142-165
    rows, cols = grid.shape
    lines = []
    for r in range(rows):
        lines.append("".join("@" if solver_pos and (r, c) == tuple(solver_pos) else _SYMBOLS.get(int(grid[r, c]), "?")
                             for c in range(cols)))
    return "\n".join(lines)


def bfs_valid_batch(grids: torch.Tensor, start: Tuple[int, int], goal: Tuple[int, int]) -> torch.Tensor:
    """bfs_path_exists over a batch of device grids [N, R, C] (int32) -> bool [N]."""
    from . import _native as nat
    g = grids.to(torch.int32).contiguous()
    n, R, C = g.shape
    out = torch.empty(n, dtype=torch.uint8, device=g.device)
    nat.check(nat.lib().heist_bfs_valid(nat.ptr(g), n, R, C, start[0], start[1], goal[0], goal[1], nat.ptr(out),
                                        nat.stream(g.device)), "heist_bfs_valid")
    return out.bool()


def bfs_path_exists(grid: np.ndarray, start: Tuple[int, int], goal: Tuple[int, int]) -> bool:  # utils.py:52-85
    from . import _native as nat
    dev = nat.require_gpu()
    g = torch.as_tensor(np.ascontiguousarray(grid, dtype=np.int32), device=dev)[None]
    return bool(bfs_valid_batch(g, tuple(start), tuple(goal)).item())
