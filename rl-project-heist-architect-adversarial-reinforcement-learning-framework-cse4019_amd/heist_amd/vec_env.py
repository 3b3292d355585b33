"""HeistEnv -- N independent Heist environments stepped by one HIP launch.

This is the batched form of the reference's HeistEnvironment (environment.py:40-426):
set_layout / reset / step have the same semantics per env, the observation is the
reference's get_state_tensor() stacked as [N, 3, R, C] float32, and all state stays
in HBM.  Layout lists in the reference's dict format are packed by LayoutBatch.
"""
import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import _native as nat

STATUS_NAMES = {0: "running", 1: "detected", 2: "vault_reached", 3: "timeout", 4: "already_done"}
STATUS_CODES = {v: k for k, v in STATUS_NAMES.items()}

Layout = Tuple[Sequence[Tuple[int, int]], Sequence[dict], Sequence[dict]]


@dataclass
class LayoutBatch:
    """Padded device arrays for heist_set_layout (see include/heist.h)."""
    wall_rc: torch.Tensor      # [N, max_walls, 2] int32
    n_walls: torch.Tensor      # [N] int32
    cam_params: torch.Tensor   # [N, max_cams, 6] float64
    n_cams: torch.Tensor       # [N] int32
    guard_paths: torch.Tensor  # [N, max_guards, max_path, 2] int32
    guard_meta: torch.Tensor   # [N, max_guards, 3] int32
    guard_fov: torch.Tensor    # [N, max_guards] float64
    n_guards: torch.Tensor     # [N] int32
    budget: torch.Tensor       # [N] int32

    @property
    def max_walls(self) -> int:
        return int(self.wall_rc.shape[1])

    @staticmethod
    def from_lists(layouts: Sequence[Layout], budget: Union[int, Sequence[int]], max_cams: int, max_guards: int,
                   max_path: int, device, rows: int = 64, cols: int = 64) -> "LayoutBatch":
        n = len(layouts)
        mw = max(1, max((len(w) for w, _, _ in layouts), default=0))
        W = np.zeros((n, mw, 2), np.int32)
        nw = np.zeros(n, np.int32)
        CP = np.zeros((n, max(1, max_cams), 6), np.float64)
        nc = np.zeros(n, np.int32)
        GP = np.zeros((n, max(1, max_guards), max_path, 2), np.int32)
        GM = np.zeros((n, max(1, max_guards), 3), np.int32)
        GF = np.zeros((n, max(1, max_guards)), np.float64)
        ng = np.zeros(n, np.int32)
        for e, (walls, cams, guards) in enumerate(layouts):
            if len(cams) > max_cams or len(guards) > max_guards:
                raise ValueError("env %d: %d cameras / %d guards exceed capacity %d / %d"
                                 % (e, len(cams), len(guards), max_cams, max_guards))
            nw[e] = len(walls)
            for i, (r, c) in enumerate(walls):
                W[e, i] = (r, c)
            nc[e] = len(cams)
            for i, cd in enumerate(cams):  # environment.py:127-133 defaults
                CP[e, i] = (cd["row"], cd["col"], cd.get("fov_angle", 60.0), cd.get("heading", 0.0),
                            cd.get("rotation_speed", 15.0), cd.get("vision_range", 6))
            ng[e] = len(guards)
            for i, gd in enumerate(guards):  # environment.py:141-146 defaults
                path = list(gd["patrol_path"])
                if len(path) > max_path:
                    raise ValueError("env %d guard %d: patrol path of %d points exceeds max_path %d"
                                     % (e, i, len(path), max_path))
                for k, (r, c) in enumerate(path):
                    if not (0 <= r < rows and 0 <= c < cols):
                        raise ValueError("env %d guard %d: patrol point %s outside the %dx%d grid"
                                         % (e, i, (r, c), rows, cols))
                    GP[e, i, k] = (r, c)
                GM[e, i] = (len(path), gd.get("speed", 1), gd.get("vision_range", 4))
                GF[e, i] = gd.get("fov_angle", 90.0)
        b = np.broadcast_to(np.asarray(budget, np.int32), (n,)).copy()
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        return LayoutBatch(t(W), t(nw), t(CP), t(nc), t(GP), t(GM), t(GF), t(ng), t(b))


def _layout_to_lists(lb: "LayoutBatch"):
    W, nw, CP, nc, GP, GM, GF, ng = (t.cpu().numpy() for t in (lb.wall_rc, lb.n_walls, lb.cam_params, lb.n_cams,
                                                              lb.guard_paths, lb.guard_meta, lb.guard_fov, lb.n_guards))
    out = []
    for e in range(len(nw)):
        walls = [(int(r), int(c)) for r, c in W[e, :nw[e]]]
        cams = [{"row": int(c[0]), "col": int(c[1]), "fov_angle": float(c[2]), "rotation_speed": float(c[4]),
                 "heading": float(c[3]), "vision_range": int(c[5])} for c in CP[e, :nc[e]]]
        guards = [{"patrol_path": [(int(r), int(c)) for r, c in GP[e, i, :GM[e, i, 0]]], "speed": int(GM[e, i, 1]),
                   "vision_range": int(GM[e, i, 2]), "fov_angle": float(GF[e, i])} for i in range(ng[e])]
        out.append((walls, cams, guards))
    return out


LayoutBatch.to_lists = _layout_to_lists


class HeistEnv:
    """Batched HeistEnvironment on one HIP device.

    step(actions) returns (obs, reward, done, status) as device tensors: obs [N,3,R,C]
    float32 (get_state_tensor, environment.py:347-374), reward [N] float32, done [N]
    bool, status [N] int8 (STATUS_NAMES).  With auto_reset=True an env that finishes is
    reset in the same launch (headings carry over, environment.py:204-208) and its obs
    row is the next attempt's first observation.
    """

    def __init__(self, n_envs: int, config=None, max_cams: int = 8, max_guards: int = 4, max_path: int = 16,
                 device=None, auto_reset: bool = True):
        from .environment import EnvironmentConfig
        self.config = config or EnvironmentConfig()
        cfg = self.config
        self.device = nat.require_gpu(device)
        self.n_envs = int(n_envs)
        self.rows, self.cols = cfg.grid_rows, cfg.grid_cols
        self.max_cams, self.max_guards, self.max_path = max_cams, max_guards, max_path
        self.auto_reset = auto_reset
        consts = (ctypes.c_double * 3)(cfg.reward_step, cfg.reward_detection, cfg.reward_vault)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            nat.check(nat.lib().heist_create(cfg.grid_rows, cfg.grid_cols, cfg.max_steps, cfg.start_pos[0],
                                             cfg.start_pos[1], cfg.vault_pos[0], cfg.vault_pos[1], consts, self.n_envs,
                                             max_cams, max_guards, max_path, ctypes.byref(h)), "heist_create")
        self._h = h
        kw = dict(device=self.device)
        self.obs = torch.zeros((self.n_envs, 3, self.rows, self.cols), dtype=torch.float32, **kw)
        self.reward = torch.zeros(self.n_envs, dtype=torch.float32, **kw)
        self.reward64 = torch.zeros(self.n_envs, dtype=torch.float64, **kw)
        self.done = torch.zeros(self.n_envs, dtype=torch.uint8, **kw)
        self.status = torch.zeros(self.n_envs, dtype=torch.int8, **kw)
        self._done_bool = self.done.view(torch.bool)
        self._bufs = tuple(t.data_ptr() for t in (self.obs, self.reward, self.reward64, self.done, self.status))
        self.valid = torch.zeros(self.n_envs, dtype=torch.uint8, **kw)

    # -- lifecycle ---------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            with torch.cuda.device(self.device):
                torch.cuda.synchronize(self.device)
                nat.lib().heist_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return nat.stream(self.device)

    # -- layout ------------------------------------------------------------------
    def set_layout_batch(self, lb: LayoutBatch, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """heist_set_layout on pre-packed device arrays (only envs in mask if given);
        returns valid [N] bool."""
        n, mc, mg, mp = self.n_envs, max(1, self.max_cams), max(1, self.max_guards), self.max_path
        want = {"wall_rc": (n, lb.max_walls, 2), "n_walls": (n,), "cam_params": (n, mc, 6), "n_cams": (n,),
                "guard_paths": (n, mg, mp, 2), "guard_meta": (n, mg, 3), "guard_fov": (n, mg), "n_guards": (n,),
                "budget": (n,)}
        dtypes = {"cam_params": torch.float64, "guard_fov": torch.float64}
        for k, shp in want.items():  # the kernel indexes with this handle's capacities
            t = getattr(lb, k)
            if tuple(t.shape) != shp or t.dtype != dtypes.get(k, torch.int32) or t.device != self.device \
                    or not t.is_contiguous():
                raise ValueError("LayoutBatch.%s: expected contiguous %s %s on %s, got %s %s on %s"
                                 % (k, dtypes.get(k, torch.int32), shp, self.device, t.dtype, tuple(t.shape), t.device))
        m = None if mask is None else mask.to(device=self.device, dtype=torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            nat.check(nat.lib().heist_set_layout(
                self._h, lb.max_walls, nat.ptr(lb.wall_rc), nat.ptr(lb.n_walls), nat.ptr(lb.cam_params),
                nat.ptr(lb.n_cams), nat.ptr(lb.guard_paths), nat.ptr(lb.guard_meta), nat.ptr(lb.guard_fov),
                nat.ptr(lb.n_guards), nat.ptr(lb.budget), nat.ptr(m), nat.ptr(self.valid), self._stream()),
                "heist_set_layout")
        return self.valid.view(torch.bool)

    def set_layouts(self, layouts: Sequence[Layout], budget: Union[int, Sequence[int]] = None,
                    env_ids: Optional[Sequence[int]] = None) -> torch.Tensor:
        """HeistEnvironment.set_layout (environment.py:102-152) for every env, or only for
        env_ids (then layouts[i] goes to env env_ids[i])."""
        if budget is None:
            budget = self.config.architect_budget
        mask = None
        if env_ids is not None:
            if len(layouts) != len(env_ids):
                raise ValueError("expected one layout per env id")
            full = [([], [], [])] * self.n_envs
            b = np.broadcast_to(np.asarray(budget, np.int32), (len(env_ids),))
            bud = np.zeros(self.n_envs, np.int32)
            for i, e in enumerate(env_ids):
                full[int(e)] = layouts[i]
                bud[int(e)] = b[i]
            m = np.zeros(self.n_envs, np.uint8)
            m[np.asarray(env_ids, np.int64)] = 1
            mask = torch.from_numpy(m).to(self.device)
            layouts, budget = full, bud
        elif len(layouts) != self.n_envs:
            raise ValueError("expected %d layouts, got %d" % (self.n_envs, len(layouts)))
        lb = LayoutBatch.from_lists(layouts, budget, self.max_cams, self.max_guards, self.max_path, self.device,
                                    self.rows, self.cols)
        return self.set_layout_batch(lb, mask)

    # -- episode -----------------------------------------------------------------
    def reset(self, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """HeistEnvironment.reset + get_state_tensor for envs with mask (None: all)."""
        m = None if mask is None else mask.to(device=self.device, dtype=torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            nat.check(nat.lib().heist_reset(self._h, nat.ptr(m), nat.ptr(self.obs), self._stream()), "heist_reset")
        return self.obs

    def step(self, actions: torch.Tensor, auto_reset: Optional[bool] = None, obs_out: torch.Tensor = None):
        """HeistEnvironment.step + get_state_tensor for all envs (environment.py:216-299).

        The per-call host path is kept short (cached buffer addresses, no device switch
        when the handle's device is current) so that back-to-back steps stay GPU-bound."""
        a = actions
        if a.device != self.device or a.dtype != torch.int64 or not a.is_contiguous():
            a = a.to(device=self.device, dtype=torch.int64).contiguous()
        if a.numel() != self.n_envs:
            raise ValueError("step: %d actions for %d envs" % (a.numel(), self.n_envs))
        ar = self.auto_reset if auto_reset is None else auto_reset
        if obs_out is None:
            obs, optr = self.obs, self._bufs[0]
        else:
            if (obs_out.shape != self.obs.shape or obs_out.dtype != torch.float32 or obs_out.device != self.device
                    or not obs_out.is_contiguous()):
                raise ValueError("step: obs_out must be a contiguous float32 %s tensor on %s"
                                 % (tuple(self.obs.shape), self.device))
            obs, optr = obs_out, obs_out.data_ptr()
        L = nat.lib()
        if torch.cuda.current_device() == self.device.index:
            rc = L.heist_step(self._h, a.data_ptr(), optr, *self._bufs[1:], 1 if ar else 0,
                              torch.cuda.current_stream(self.device).cuda_stream)
        else:
            with torch.cuda.device(self.device):
                rc = L.heist_step(self._h, a.data_ptr(), optr, *self._bufs[1:], 1 if ar else 0,
                                  torch.cuda.current_stream(self.device).cuda_stream)
        nat.check(rc, "heist_step")
        return obs, self.reward, self._done_bool, self.status

    def step_multi(self, actions: torch.Tensor, obs_out: Optional[torch.Tensor] = None,
                   auto_reset: Optional[bool] = None, reward64: bool = False):
        """K steps in one launch (heist_step_multi) for actions [K, N] known in advance:
        tick k's observation, reward, done and status land in obs[k], reward[k], ... exactly
        as K step() calls would produce them.  Returns (obs [K,N,3,R,C], reward [K,N] f32,
        done [K,N] bool, status [K,N] int8, reward64 [K,N] f64 or None).  The per-env state
        is on chip between the ticks; env.obs is not updated (obs[K-1] is the latest)."""
        a = actions
        if a.device != self.device or a.dtype != torch.int64 or not a.is_contiguous():
            a = a.to(device=self.device, dtype=torch.int64).contiguous()
        if a.dim() != 2 or a.shape[1] != self.n_envs:
            raise ValueError("step_multi: actions must be [K, %d]" % self.n_envs)
        K = int(a.shape[0])
        kw = dict(device=self.device)
        shape = (K, self.n_envs, 3, self.rows, self.cols)
        if obs_out is None:
            obs_out = torch.empty(shape, dtype=torch.float32, **kw)
        elif (tuple(obs_out.shape) != shape or obs_out.dtype != torch.float32 or obs_out.device != self.device
              or not obs_out.is_contiguous()):
            raise ValueError("step_multi: obs_out must be a contiguous float32 %s tensor on %s" % (shape, self.device))
        rew = torch.empty((K, self.n_envs), dtype=torch.float32, **kw)
        r64 = torch.empty((K, self.n_envs), dtype=torch.float64, **kw) if reward64 else None
        done = torch.empty((K, self.n_envs), dtype=torch.uint8, **kw)
        status = torch.empty((K, self.n_envs), dtype=torch.int8, **kw)
        ar = self.auto_reset if auto_reset is None else auto_reset
        with torch.cuda.device(self.device):
            nat.check(nat.lib().heist_step_multi(self._h, K, nat.ptr(a), nat.ptr(obs_out), nat.ptr(rew), nat.ptr(r64),
                                                 nat.ptr(done), nat.ptr(status), 1 if ar else 0, self._stream()),
                      "heist_step_multi")
        return obs_out, rew, done.view(torch.bool), status, r64

    def step_multi_raw(self, K: int, actions: torch.Tensor, obs_out: torch.Tensor, reward: torch.Tensor,
                       done: torch.Tensor, status: torch.Tensor, auto_reset: bool = True) -> None:
        """heist_step_multi on caller-owned buffers with no checks or allocation (the
        benchmark's timed loop; shapes as step_multi's)."""
        rc = nat.lib().heist_step_multi(self._h, K, actions.data_ptr(), obs_out.data_ptr(), reward.data_ptr(), None,
                                        done.data_ptr(), status.data_ptr(), 1 if auto_reset else 0,
                                        torch.cuda.current_stream(self.device).cuda_stream)
        nat.check(rc, "heist_step_multi")

    def step_multi_launcher(self, K: int, actions: torch.Tensor, obs_out: torch.Tensor, reward: torch.Tensor,
                            done: torch.Tensor, status: torch.Tensor, auto_reset: bool = True):
        """step_multi_raw with every argument resolved now (device pointers, the stream, the
        bound C function): returns a zero-argument callable that only issues the launch, so
        a timed region around it holds no Python argument handling.  The tensors must stay
        alive while the callable is used."""
        fn = nat.lib().heist_step_multi
        args = (self._h, K, actions.data_ptr(), obs_out.data_ptr(), reward.data_ptr(), None, done.data_ptr(),
                status.data_ptr(), 1 if auto_reset else 0, torch.cuda.current_stream(self.device).cuda_stream)

        def launch():
            rc = fn(*args)
            if rc:
                nat.check(rc, "heist_step_multi")
        return launch

    # -- introspection -------------------------------------------------------------
    def export(self, grid: bool = False) -> dict:
        """Per-env state (get_environment_state source) as device tensors."""
        kw = dict(device=self.device)
        sc = torch.empty((self.n_envs, 12), dtype=torch.int32, **kw)
        ch = torch.empty((self.n_envs, max(1, self.max_cams)), dtype=torch.float64, **kw)
        gi = torch.empty((self.n_envs, max(1, self.max_guards)), dtype=torch.int32, **kw)
        gh = torch.empty((self.n_envs, max(1, self.max_guards)), dtype=torch.float64, **kw)
        gr = torch.empty((self.n_envs, self.rows, self.cols), dtype=torch.int8, **kw) if grid else None
        with torch.cuda.device(self.device):
            nat.check(nat.lib().heist_export(self._h, nat.ptr(sc), nat.ptr(gr), nat.ptr(ch), nat.ptr(gi), nat.ptr(gh),
                                             self._stream()), "heist_export")
        keys = ("pos_r", "pos_c", "tick", "done", "detected", "vault_reached", "prev_dist", "initial_dist",
                "n_cams", "n_guards", "n_walls", "spent")
        out = {k: sc[:, i] for i, k in enumerate(keys)}
        out.update(cam_heading=ch, guard_idx=gi, guard_heading=gh)
        if grid:
            out["grid"] = gr
        return out

    def count_samples(self, counter: Optional[torch.Tensor]) -> None:
        """Instrumentation (no reference counterpart): later step/reset calls add the number of
        ray samples env e evaluates to ``counter[e]`` (int64 [n_envs] on this device, zeroed by
        the caller) -- the ALU work figure of SURVEY 8(d).  ``None`` switches counting off."""
        if counter is not None and (counter.dtype != torch.int64 or counter.numel() != self.n_envs
                                    or counter.device != self.device or not counter.is_contiguous()):
            raise ValueError("count_samples: need a contiguous int64 [%d] tensor on %s" % (self.n_envs, self.device))
        nat.check(nat.lib().heist_count_samples(self._h, nat.ptr(counter)), "heist_count_samples")
        self._counter = counter  # keep the buffer alive while the library holds its pointer

    def count_exact_rays(self, counter: Optional[torch.Tensor]) -> None:
        """Instrumentation: later step/reset calls add to ``counter[e]`` the number of env e's
        rays cast on the exact fp64 path (near-tie re-casts of the fp32 fast path, or every
        ray with ``set_ray_mode(1)``).  ``None`` switches counting off."""
        if counter is not None and (counter.dtype != torch.int64 or counter.numel() != self.n_envs
                                    or counter.device != self.device or not counter.is_contiguous()):
            raise ValueError("count_exact_rays: need a contiguous int64 [%d] tensor on %s" % (self.n_envs, self.device))
        nat.check(nat.lib().heist_count_redo(self._h, nat.ptr(counter)), "heist_count_redo")
        self._redo_counter = counter

    def set_ray_mode(self, mode: int) -> None:
        """0 (default): fp32 fast raycast with exact fp64 re-cast of near-tie rays; 1: exact
        fp64 raycast for every ray.  Results are bit-identical; 1 is for parity tests and A/B
        timing."""
        nat.check(nat.lib().heist_set_ray_mode(self._h, int(mode)), "heist_set_ray_mode")

    def set_guard_cones(self, on: bool) -> None:
        """True (default): the next set_layout precomputes every guard's vision cone per
        (patrol point, heading) on the exact path and step/reset OR the cached cone instead
        of raycasting the guard; False: every guard is raycast every tick.  Results are
        bit-identical; takes effect at the next set_layout."""
        nat.check(nat.lib().heist_set_guard_cones(self._h, 1 if on else 0), "heist_set_guard_cones")

    CONFIG_KEYS = ("step_waves", "ray_chunk", "step_occ", "vis_gap", "obs_store", "ray_mode", "probe_mode",
                   "dispatch_order", "split_obs", "guard_cones", "multi_waves", "fan_on", "lean", "interval_fans",
                   "step_lean", "lean_waves")

    def kernel_config(self) -> dict:
        """The handle's effective kernel configuration (heist_get_config): the HEIST_* knobs as
        heist_create resolved them plus later set_* calls.  probe_mode != 0 means the
        profiling step kernel, whose results are wrong by design."""
        out = (ctypes.c_int32 * len(self.CONFIG_KEYS))()
        nat.check(nat.lib().heist_get_config(self._h, ctypes.cast(out, ctypes.c_void_p), len(self.CONFIG_KEYS)),
                  "heist_get_config")
        return dict(zip(self.CONFIG_KEYS, (int(v) for v in out)))

    @property
    def visibility(self) -> torch.Tensor:
        """Current visibility plane [N, R, C] (obs channel 1)."""
        return self.obs[:, 1]
