"""Batched Architect layout decode on the GPU (heist_architect_decode).

networks.py:283-335 turns one sampled asset map into wall / camera / guard lists with
a greedy row-major budget scan; here N maps are decoded in one launch directly into
the LayoutBatch arrays heist_set_layout consumes.
"""
from typing import Optional, Union

import torch

from . import _native as nat
from .vec_env import LayoutBatch


def capacities(budget: int):
    """Largest list lengths a budget can buy (wall 1, camera 3, guard 5)."""
    return max(1, budget), max(1, budget // 3), max(1, budget // 5)


def decode_layouts(asset_map: torch.Tensor, cam_params, budget: Union[int, torch.Tensor], allow_cams: bool = True,
                   allow_guards: bool = True, max_walls: Optional[int] = None, max_cams: Optional[int] = None,
                   max_guards: Optional[int] = None, max_path: int = 8) -> LayoutBatch:
    """asset_map [N,R,C] classes; cam_params = the network's dict of [1,1] or [N,1] tensors
    (or a [3] / [N,3] float tensor of fov, speed, heading); budget int or [N]."""
    am = asset_map.to(torch.int64).contiguous()
    dev = am.device
    n, R, C = am.shape
    if isinstance(cam_params, dict):
        cp = torch.cat([cam_params[k].reshape(-1, 1) for k in ("fov", "speed", "heading")], dim=1)
    else:
        cp = cam_params.reshape(-1, 3)
    cp = cp.to(device=dev, dtype=torch.float32).contiguous()
    stride = 0 if cp.shape[0] == 1 else 3
    if isinstance(budget, torch.Tensor):
        bud = budget.to(device=dev, dtype=torch.int32).reshape(n).contiguous()
        bmax = int(bud.max().item()) if n else 0
    else:
        bud = torch.full((n,), int(budget), dtype=torch.int32, device=dev)
        bmax = int(budget)
    cw, cc, cg = capacities(bmax)
    mw, mc, mg = max_walls or cw, max_cams or cc, max_guards or cg
    kw = dict(device=dev)
    lb = LayoutBatch(
        wall_rc=torch.zeros((n, mw, 2), dtype=torch.int32, **kw), n_walls=torch.zeros(n, dtype=torch.int32, **kw),
        cam_params=torch.zeros((n, mc, 6), dtype=torch.float64, **kw), n_cams=torch.zeros(n, dtype=torch.int32, **kw),
        guard_paths=torch.zeros((n, mg, max_path, 2), dtype=torch.int32, **kw),
        guard_meta=torch.zeros((n, mg, 3), dtype=torch.int32, **kw),
        guard_fov=torch.zeros((n, mg), dtype=torch.float64, **kw), n_guards=torch.zeros(n, dtype=torch.int32, **kw),
        budget=bud)
    nat.check(nat.lib().heist_architect_decode(
        nat.ptr(am), n, R, C, nat.ptr(cp), stride, nat.ptr(bud), int(bool(allow_cams)), int(bool(allow_guards)),
        mw, mc, mg, max_path, nat.ptr(lb.wall_rc), nat.ptr(lb.n_walls), nat.ptr(lb.cam_params), nat.ptr(lb.n_cams),
        nat.ptr(lb.guard_paths), nat.ptr(lb.guard_meta), nat.ptr(lb.guard_fov), nat.ptr(lb.n_guards),
        nat.stream(dev)), "heist_architect_decode")
    return lb
