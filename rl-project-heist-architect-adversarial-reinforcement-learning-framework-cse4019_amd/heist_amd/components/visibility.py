"""Surveillance map (reference: components/visibility.py).

update() raycasts every camera and guard in ONE heist_cones launch and ORs the
cones on the device; the heat map is host bookkeeping (not on the training path).
"""
from typing import List, Tuple

import numpy as np


class DynamicVisibilityMap:  # visibility.py:11-90
    def __init__(self, rows: int, cols: int):
        self.rows = rows
        self.cols = cols
        self.visibility = np.zeros((rows, cols), dtype=np.float32)
        self.heat_map = np.zeros((rows, cols), dtype=np.float32)
        self._total_updates = 0

    def _record(self, vis: np.ndarray):
        self.visibility = vis.astype(np.float32)
        self._total_updates += 1
        self.heat_map += self.visibility

    def update(self, cameras, guards, walls: np.ndarray) -> np.ndarray:
        import torch
        from .. import _native as nat
        emit = [(0, c.row, c.col, c.vision_range, c.fov_angle, c.heading) for c in cameras]
        emit += [(1, g.row, g.col, g.vision_range, g.fov_angle, g.heading) for g in guards]
        vis = np.zeros((self.rows, self.cols), dtype=bool)
        if emit:
            dev = nat.require_gpu()
            n = len(emit)
            w = np.ascontiguousarray(np.broadcast_to(np.asarray(walls, dtype=np.uint8), (n, self.rows, self.cols)))
            wt = torch.as_tensor(w, device=dev)
            meta = torch.tensor([e[:4] for e in emit], dtype=torch.int32, device=dev)
            par = torch.tensor([e[4:] for e in emit], dtype=torch.float64, device=dev)
            out = torch.empty((n, self.rows, self.cols), dtype=torch.uint8, device=dev)
            nat.check(nat.lib().heist_cones(n, self.rows, self.cols, nat.ptr(wt), nat.ptr(meta), nat.ptr(par),
                                            nat.ptr(out), nat.stream(dev)), "heist_cones")
            vis = out.amax(0).bool().cpu().numpy()
        for g in guards:  # visibility.py:59
            vis[g.row, g.col] = True
        self._record(vis)
        return self.visibility

    def is_visible(self, row: int, col: int) -> bool:
        return self.visibility[row, col] > 0.5

    def get_safe_tiles(self) -> List[Tuple[int, int]]:
        rr, cc = np.nonzero(self.visibility < 0.5)
        return [(int(r), int(c)) for r, c in zip(rr, cc)]

    def get_normalized_heat_map(self) -> np.ndarray:
        if self._total_updates == 0:
            return self.heat_map.copy()
        return self.heat_map / self._total_updates

    def reset(self):
        self.visibility = np.zeros((self.rows, self.cols), dtype=np.float32)
        self.heat_map = np.zeros((self.rows, self.cols), dtype=np.float32)
        self._total_updates = 0
