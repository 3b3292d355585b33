"""ctypes wrapper of liboracle.so -- the CPU restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / baseline, never as the
product path.  Each method cites the reference code it restates (paths relative
to the reference repository root).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_f64p = ctypes.POINTER(ctypes.c_double)
_f32p = ctypes.POINTER(ctypes.c_float)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_i8p = ctypes.POINTER(ctypes.c_int8)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_env_create.restype = ctypes.c_void_p
        L.oracle_env_create.argtypes = [ctypes.c_int] * 7 + [ctypes.c_double] * 3 + [ctypes.c_int]
        L.oracle_env_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_env_set_budget.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_env_set_layout.restype = ctypes.c_int
        L.oracle_env_set_layout.argtypes = [ctypes.c_void_p, ctypes.c_int, _i32p, ctypes.c_int, _f64p,
                                            ctypes.c_int, _i64p, _f64p, _i32p]
        L.oracle_env_reset.argtypes = [ctypes.c_void_p]
        L.oracle_env_step.restype = ctypes.c_double
        L.oracle_env_step.argtypes = [ctypes.c_void_p, ctypes.c_int, _i32p, _i32p]
        L.oracle_env_state_tensor.argtypes = [ctypes.c_void_p, _f32p]
        L.oracle_env_info.argtypes = [ctypes.c_void_p, _i32p]
        L.oracle_env_vis.argtypes = [ctypes.c_void_p, _u8p]
        L.oracle_env_grid.argtypes = [ctypes.c_void_p, _i8p]
        L.oracle_env_headings.argtypes = [ctypes.c_void_p, _f64p, _i32p, _f64p]
        L.oracle_cone.argtypes = [ctypes.c_int] * 3 + [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                                       ctypes.c_double, ctypes.c_int, _u8p]
        L.oracle_bfs.restype = ctypes.c_int
        L.oracle_bfs.argtypes = [_i8p] + [ctypes.c_int] * 6
        L.oracle_gae.argtypes = [_f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_double, ctypes.c_double, _f32p]
        L.oracle_ppo_loss.argtypes = [ctypes.c_int, ctypes.c_int, _f32p, _f32p, _i64p, _f32p, _f32p, _f32p,
                                      ctypes.c_double, ctypes.c_double, ctypes.c_double, _f32p, _f32p, _f32p]
        L.oracle_run_random.restype = ctypes.c_int64
        L.oracle_run_random.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int,
                                        ctypes.c_uint64, ctypes.c_int]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


STATUS_NAMES = {0: "running", 1: "detected", 2: "vault_reached", 3: "timeout", 4: "already_done"}


class OracleEnv:
    """One HeistEnvironment (environment.py:40-426) restated in C."""

    def __init__(self, R=20, C=20, max_steps=200, start=(1, 1), vault=None, budget=15,
                 r_step=-0.01, r_detect=-1.0, r_vault=10.0):
        vault = vault if vault is not None else (R - 2, C - 2)
        self.R, self.C = R, C
        self._h = lib().oracle_env_create(R, C, max_steps, start[0], start[1], vault[0], vault[1],
                                          r_step, r_detect, r_vault, budget)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.oracle_env_destroy(self._h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def set_budget(self, total):
        lib().oracle_env_set_budget(self._h, total)

    def set_layout(self, walls, cameras, guards):
        """walls [(r,c)], cameras [dict], guards [dict] -- reference dict formats."""
        w = np.ascontiguousarray(np.array(walls, np.int32).reshape(-1, 2))
        cm = np.ascontiguousarray(np.array(
            [(c["row"], c["col"], c.get("fov_angle", 60.0), c.get("heading", 0.0), c.get("rotation_speed", 15.0),
              c.get("vision_range", 6)) for c in cameras], np.float64).reshape(-1, 6))
        gi, gf, pts = [], [], []
        for g in guards:
            path = list(g["patrol_path"])
            gi.append((len(pts), len(path), g.get("speed", 1), g.get("vision_range", 4)))
            gf.append(g.get("fov_angle", 90.0))
            pts.extend(path)
        gi = np.ascontiguousarray(np.array(gi, np.int64).reshape(-1, 4))
        gf = np.ascontiguousarray(np.array(gf, np.float64))
        pts = np.ascontiguousarray(np.array(pts, np.int32).reshape(-1, 2))
        return bool(lib().oracle_env_set_layout(self._h, len(w), _p(w, _i32p), len(cm), _p(cm, _f64p), len(gi),
                                                _p(gi, _i64p), _p(gf, _f64p), _p(pts, _i32p)))

    def reset(self):
        lib().oracle_env_reset(self._h)

    def step(self, action):
        d = ctypes.c_int32()
        s = ctypes.c_int32()
        r = lib().oracle_env_step(self._h, int(action), ctypes.byref(d), ctypes.byref(s))
        return r, bool(d.value), int(s.value)

    def state_tensor(self):
        out = np.empty((3, self.R, self.C), np.float32)
        lib().oracle_env_state_tensor(self._h, _p(out, _f32p))
        return out

    def info(self):
        out = np.empty(10, np.int32)
        lib().oracle_env_info(self._h, _p(out, _i32p))
        keys = ("pos_r", "pos_c", "tick", "done", "detected", "vault_reached", "n_walls", "n_cams", "n_guards", "spent")
        return dict(zip(keys, (int(x) for x in out)))

    def visibility(self):
        out = np.empty(self.R * self.C, np.uint8)
        lib().oracle_env_vis(self._h, _p(out, _u8p))
        return out.reshape(self.R, self.C)

    def grid(self):
        out = np.empty(self.R * self.C, np.int8)
        lib().oracle_env_grid(self._h, _p(out, _i8p))
        return out.reshape(self.R, self.C)

    def headings(self):
        inf = self.info()
        ch = np.zeros(max(1, inf["n_cams"]), np.float64)
        gi = np.zeros(max(1, inf["n_guards"]), np.int32)
        gh = np.zeros(max(1, inf["n_guards"]), np.float64)
        lib().oracle_env_headings(self._h, _p(ch, _f64p), _p(gi, _i32p), _p(gh, _f64p))
        return ch[:inf["n_cams"]], gi[:inf["n_guards"]], gh[:inf["n_guards"]]


def cone(kind, walls, row, col, fov, heading, rng):
    """kind 0 = Camera.get_vision_cone_tiles, 1 = Guard.get_visible_tiles; returns bool [R,C]."""
    walls = np.ascontiguousarray(walls.astype(np.uint8))
    R, C = walls.shape
    out = np.zeros(R * C, np.uint8)
    lib().oracle_cone(kind, R, C, _p(walls, _u8p), row, col, fov, heading, rng, _p(out, _u8p))
    return out.reshape(R, C).astype(bool)


def bfs(grid, start, goal):
    g = np.ascontiguousarray(grid.astype(np.int8))
    R, C = g.shape
    return bool(lib().oracle_bfs(_p(g, _i8p), R, C, start[0], start[1], goal[0], goal[1]))


def gae(r, v, d, gamma=0.99, lam=0.95):
    r, v, d = (np.ascontiguousarray(np.asarray(x, np.float32)) for x in (r, v, d))
    out = np.empty_like(r)
    lib().oracle_gae(_p(r, _f32p), _p(v, _f32p), _p(d, _f32p), len(r), gamma, lam, _p(out, _f32p))
    return out


def ppo_loss(logits, values, actions, old_logp, adv, ret, clip=0.2, vcoef=0.5, ecoef=0.05):
    logits = np.ascontiguousarray(logits, np.float32)
    M, A = logits.shape
    vals = [np.ascontiguousarray(x, np.float32) for x in (values, old_logp, adv, ret)]
    acts = np.ascontiguousarray(actions, np.int64)
    parts = np.empty(4, np.float32)
    dl = np.empty_like(logits)
    dv = np.empty(M, np.float32)
    lib().oracle_ppo_loss(M, A, _p(logits, _f32p), _p(vals[0], _f32p), _p(acts, _i64p), _p(vals[1], _f32p),
                          _p(vals[2], _f32p), _p(vals[3], _f32p), clip, vcoef, ecoef, _p(parts, _f32p),
                          _p(dl, _f32p), _p(dv, _f32p))
    return parts, dl, dv


def run_random(envs, n_steps, seed=0, n_threads=1):
    arr = (ctypes.c_void_p * len(envs))(*[e.handle for e in envs])
    return int(lib().oracle_run_random(arr, len(envs), n_steps, seed, n_threads))
