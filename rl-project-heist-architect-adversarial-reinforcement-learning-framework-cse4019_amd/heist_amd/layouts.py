"""Synthetic layout generator in the reference's list/dict format.

Walls are uniform over interior empty cells; cameras draw fov ~ U[30,120],
heading ~ U[0,360), speed ~ U[5,35] rounded to float32 like the Architect's
sigmoid heads (networks.py:233-237), range 6; guards use the Architect's 8-point
rectangular patrol (networks.py:324-335) with speed 1, range 4, fov 90.
"""
from typing import List, Optional, Tuple

import numpy as np


def architect_patrol(row: int, col: int, grid_h: int, grid_w: int) -> List[Tuple[int, int]]:
    """ArchitectNetwork._generate_patrol (networks.py:324-335)."""
    offsets = [(0, 0), (0, 1), (0, 2), (1, 2), (2, 2), (2, 1), (2, 0), (1, 0)]
    return [(max(1, min(grid_h - 2, row + dr - 1)), max(1, min(grid_w - 2, col + dc - 1))) for dr, dc in offsets]


def synthetic_layout(rng: np.random.Generator, R: int, C: int, budget: int, n_cams: Optional[int] = None,
                     n_guards: Optional[int] = None, start=(1, 1), vault=None):
    vault = vault if vault is not None else (R - 2, C - 2)
    interior = np.array([(r, c) for r in range(1, R - 1) for c in range(1, C - 1)
                         if (r, c) != tuple(start) and (r, c) != tuple(vault)], np.int64)
    if n_cams is None:
        n_cams = int(rng.integers(0, budget // 3 + 1))
    if n_guards is None:
        n_guards = int(rng.integers(0, max(0, budget - 3 * n_cams) // 5 + 1))
    n_walls = max(0, budget - 3 * n_cams - 5 * n_guards)
    k = n_walls + n_cams + n_guards
    pick = interior[rng.permutation(len(interior))[:k]]
    walls = [(int(r), int(c)) for r, c in pick[:n_walls]]
    cams = []
    for r, c in pick[n_walls:n_walls + n_cams]:
        cams.append({"row": int(r), "col": int(c), "fov_angle": float(np.float32(rng.uniform(30, 120))),
                     "heading": float(np.float32(rng.uniform(0, 360))),
                     "rotation_speed": float(np.float32(rng.uniform(5, 35))), "vision_range": 6})
    guards = []
    for r, c in pick[n_walls + n_cams:]:
        guards.append({"patrol_path": architect_patrol(int(r), int(c), R, C), "speed": 1, "vision_range": 4,
                       "fov_angle": 90.0})
    return walls, cams, guards


def synthetic_layouts(n: int, R: int, C: int, budget: int, seed: int, **kw):
    rng = np.random.Generator(np.random.PCG64(seed))
    return [synthetic_layout(rng, R, C, budget, **kw) for _ in range(n)]


def valid_synthetic_layouts(env, budget: int, seed: int, max_rounds: int = 20, **kw):
    """Layouts for every env of a HeistEnv, resampling until bfs_path_exists holds."""
    rng = np.random.Generator(np.random.PCG64(seed))
    R, C = env.rows, env.cols
    lays = [synthetic_layout(rng, R, C, budget, **kw) for _ in range(env.n_envs)]
    for _ in range(max_rounds):
        valid = env.set_layouts(lays, budget=budget).cpu().numpy()
        bad = np.nonzero(~valid)[0]
        if len(bad) == 0:
            return lays
        for i in bad:
            lays[i] = synthetic_layout(rng, R, C, budget, **kw)
    env.set_layouts(lays, budget=budget)
    return lays


def architect_checkpoint_layouts(env, budget: int, seed: int, ckpt: str, max_rounds: int = 20):
    """BASELINE config 2's layouts for every env of a HeistEnv: the fixed Architect
    checkpoint `ckpt` (reference dict format, agents/architect.py:157-170) sampled at T = 1.0
    with `budget`, cameras and guards allowed (networks.py:241-335 decoded on the GPU), every
    env resampled until its layout is BFS-valid.  Returns (LayoutBatch, all_valid); the
    layouts are set on env."""
    import torch
    from .agents import ArchitectAgent
    from .training import _scatter_layout
    ag = ArchitectAgent(grid_rows=env.rows, grid_cols=env.cols, budget=budget, device=env.device)
    ag.load(ckpt)
    gen = torch.Generator(device=env.device)
    gen.manual_seed(seed)
    n = env.n_envs
    lb, _, _ = ag.generate_layouts(n, 1.0, True, True, env=env, generator=gen, record=False)
    valid = env.set_layout_batch(lb).clone()
    for _ in range(max_rounds):
        bad = (~valid).nonzero().reshape(-1)
        if bad.numel() == 0:
            break
        lbk, _, _ = ag.generate_layouts(int(bad.numel()), 1.0, True, True, env=env, generator=gen, record=False)
        full = _scatter_layout(lbk, bad.cpu().numpy(), env)
        m = torch.zeros(n, dtype=torch.uint8, device=env.device)
        m[bad] = 1
        v = env.set_layout_batch(full, m)
        for k in lb.__dataclass_fields__:
            getattr(lb, k)[bad] = getattr(lbk, k)
        valid[bad] = v[bad]
    return lb, bool(valid.all())
