"""Generate the golden parity fixtures by running the Python reference.

Runs ONLY in the build container (it imports /root/reference, which never
travels to the GPU box).  Everything it writes under tests/golden/ is data:
layouts, action sequences and the reference's outputs for them.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Fixture files (all numpy .npz, loaded with allow_pickle=False):
  env_traces.npz  layouts + action/reset sequences replayed through
                  HeistEnvironment.set_layout/reset/step/get_state_tensor
                  (environment.py:102-374): per-op reward (f64), done, status,
                  position, tick, camera headings, guard idx/headings,
                  visibility bits, state tensors for the first ops.
  cones.npz       Camera.get_vision_cone_tiles / Guard.get_visible_tiles
                  sweeps (security.py:53-101, :161-192).
  cone_order.npz  the same methods' LIST order (first visit by ray index, then
                  distance) on 600 more cases: ordered flat tile indices.
  bfs.npz         bfs_path_exists on random grids (utils.py:52-85).
  ppo.npz         SolverAgent._compute_gae (agents/solver.py:228-244) and the
                  clipped-PPO loss + d(loss)/d(logits, values) of
                  SolverAgent.update (agents/solver.py:112-204), captured
                  through a stub network.
  nets.npz        seeded SolverNetwork / ArchitectNetwork weights and forward
                  outputs (networks.py:13-239) + ArchitectNetwork
                  .generate_layout decode cases (networks.py:241-335).
  kat.json        the numbers test_sanity.py / test_fixes.py print.
  arch_update.npz ArchitectAgent.update (agents/architect.py:91-155) from the
                  nets.npz seed-32 ArchitectNetwork: per case the buffered
                  (log_prob, value, reward) transitions in, the returned losses,
                  and per parameter tensor the gradient left after the update
                  (clipped) and the parameter change, as L2 norms plus 4 fixed
                  random projections (proj_vectors(): data, not weights).
"""
import json
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)

import torch  # noqa: E402

from heist_architect.environment import HeistEnvironment, EnvironmentConfig  # noqa: E402
from heist_architect.components.security import Camera, Guard  # noqa: E402
from heist_architect.utils import bfs_path_exists, create_empty_grid, TileType  # noqa: E402
from heist_architect.agents.solver import SolverAgent  # noqa: E402
from heist_architect.agents.architect import ArchitectAgent  # noqa: E402
from heist_architect.networks import SolverNetwork, ArchitectNetwork  # noqa: E402
from heist_architect.rewards import RewardCalculator  # noqa: E402

STATUS = {"running": 0, "detected": 1, "vault_reached": 2, "timeout": 3, "already_done": 4, "reset": 5}


# ---------------------------------------------------------------------------
# layouts
# ---------------------------------------------------------------------------

def f32(x):
    return float(np.float32(x))


def synth_layout(rng, R, C, budget, n_cams=None, n_guards=None, int_params=False):
    """Direct synthetic generator."""
    walls, cams, guards = [], [], []
    interior = [(r, c) for r in range(1, R - 1) for c in range(1, C - 1)
                if (r, c) not in ((1, 1), (R - 2, C - 2))]
    if n_cams is None:
        n_cams = int(rng.integers(0, budget // 3 + 1))
    if n_guards is None:
        n_guards = int(rng.integers(0, budget // 5 + 1))
    left = budget - 3 * n_cams - 5 * n_guards
    n_walls = max(0, left + int(rng.integers(-1, 3)))
    picks = rng.permutation(len(interior))
    k = 0
    for _ in range(n_walls):
        walls.append(interior[picks[k]]); k += 1
    for _ in range(n_cams):
        r, c = interior[picks[k % len(interior)]]; k += 1
        if int_params:
            fov, head, spd = float(rng.choice([30, 45, 60, 75, 90, 120])), float(rng.integers(0, 24) * 15), float(rng.choice([5, 10, 15, 20, 30, -15]))
        else:
            fov, head, spd = f32(rng.uniform(30, 120)), f32(rng.uniform(0, 360)), f32(rng.uniform(5, 35))
        cams.append({"row": r, "col": c, "fov_angle": fov, "heading": head,
                     "rotation_speed": spd, "vision_range": int(rng.choice([6, 6, 6, 4, 8]))})
    for _ in range(n_guards):
        r, c = interior[picks[k % len(interior)]]; k += 1
        guards.append({"patrol_path": ArchitectNetwork._generate_patrol(None, r, c, R, C),
                       "speed": 1, "vision_range": 4, "fov_angle": 90.0})
    return walls, cams, guards


def hand_layouts():
    """(R, C, max_steps, budget, walls, cams, guards, name) quirk layouts."""
    L = []
    # test_sanity.py:20-29
    L.append((10, 10, 200, 15, [(3, 3), (3, 4), (3, 5)],
              [{"row": 5, "col": 5, "fov_angle": 60, "heading": 0, "rotation_speed": 15, "vision_range": 4}],
              [{"patrol_path": [(7, 2), (7, 3), (7, 4), (7, 5)], "speed": 1, "vision_range": 3, "fov_angle": 90}],
              "sanity"))
    # test_fixes.py: empty 10x10
    L.append((10, 10, 200, 15, [], [], [], "empty10"))
    # guard start on a wall, on START, on VAULT, on a camera (environment.py:138-149)
    L.append((12, 12, 60, 40, [(4, 4), (4, 5), (2, 6)],
              [{"row": 6, "col": 6, "fov_angle": 90.0, "heading": 45.0, "rotation_speed": 10.0, "vision_range": 5}],
              [{"patrol_path": [(4, 4), (4, 5), (5, 5), (5, 4)], "speed": 1},
               {"patrol_path": [(1, 1), (1, 2)], "speed": 1},
               {"patrol_path": [(6, 6), (7, 6), (7, 7)], "speed": 2, "vision_range": 3, "fov_angle": 120.0}],
              "guard_overwrites"))
    # duplicates, out-of-interior placements and over budget (budget.py:48-58)
    L.append((10, 10, 50, 9, [(2, 2), (2, 2), (0, 3), (9, 9), (1, 1), (3, 3), (8, 8)],
              [{"row": 2, "col": 2, "fov_angle": 60.0}, {"row": 5, "col": 3, "fov_angle": 33.3, "heading": 359.5, "rotation_speed": -7.25},
               {"row": 6, "col": 6}],
              [{"patrol_path": [(7, 7), (7, 8)]}],
              "placement_rules"))
    # vault reachable exactly on the last tick (status overwritten by timeout)
    L.append((6, 6, 6, 0, [], [], [], "vault_last_tick"))
    # single-point patrol, empty patrol, speed 3 wrap, negative speed
    L.append((14, 14, 120, 40, [(5, 5), (5, 6), (5, 7)], [],
              [{"patrol_path": [(8, 8)]}, {"patrol_path": []},
               {"patrol_path": [(2, 9), (2, 10), (2, 11), (3, 11), (4, 11)], "speed": 3, "vision_range": 5, "fov_angle": 70.0},
               {"patrol_path": [(10, 2), (10, 3), (11, 3), (11, 2)], "speed": -1, "vision_range": 4, "fov_angle": 90.0}],
              "patrol_variants"))
    # wide and narrow cameras near walls, integer headings, range 8
    L.append((16, 16, 150, 40, [(7, 7), (7, 8), (8, 7), (3, 10), (10, 3)],
              [{"row": 8, "col": 8, "fov_angle": 120.0, "heading": 0.0, "rotation_speed": 15.0, "vision_range": 8},
               {"row": 3, "col": 3, "fov_angle": 30.0, "heading": 270.0, "rotation_speed": 30.0, "vision_range": 6},
               {"row": 12, "col": 12, "fov_angle": 75.0, "heading": 135.0, "rotation_speed": 22.5, "vision_range": 6}],
              [], "cameras_integer"))
    # blocked level (BFS false)
    L.append((10, 10, 50, 40, [(2, 1), (2, 2), (1, 2)], [], [], "blocked"))
    return L


def architect_layouts(n, R, C, budget, seed, allow_cams=True, allow_guards=True, temps=(1.0, 1.5, 0.5, 2.0)):
    torch.manual_seed(seed)
    arch = ArchitectAgent(grid_rows=R, grid_cols=C, budget=budget)
    out = []
    for i in range(n):
        w, c, g = arch.generate_layout(temps[i % len(temps)])
        if not allow_cams:
            c = []
        if not allow_guards:
            g = []
        out.append((w, c, g))
    return out


# ---------------------------------------------------------------------------
# env traces
# ---------------------------------------------------------------------------

def gen_ops(rng, n_ops, R, C):
    """Action sequence (0-4) with -1 = reset().  Biased toward the vault."""
    ops = [-1]
    for _ in range(n_ops):
        u = rng.random()
        if u < 0.35:
            ops.append(int(rng.choice([2, 4])))
        else:
            ops.append(int(rng.integers(0, 5)))
    return ops


def run_trace(cfg, layout, ops, n_state, budget):
    env = HeistEnvironment(cfg)
    env.budget.scale_budget(budget)
    walls, cams, guards = layout
    valid = env.set_layout(walls, cams, guards)
    rec = {"valid": valid, "grid": env.grid.copy(), "n_walls": len(env.walls),
           "n_cams": len(env.cameras), "n_guards": len(env.guards), "spent": env.budget.spent,
           "reward": [], "done": [], "status": [], "pos": [], "tick": [], "cam_h": [],
           "g_idx": [], "g_h": [], "vis": [], "state": []}
    done = False
    for k, op in enumerate(ops):
        if op == -1:
            env.reset()
            r, d, st = 0.0, env.done, STATUS["reset"]
        else:
            _, r, d, info = env.step(op)
            st = STATUS[info["status"]]
        rec["reward"].append(float(r)); rec["done"].append(bool(d)); rec["status"].append(st)
        rec["pos"].append(env.solver_pos); rec["tick"].append(env.tick)
        rec["cam_h"].extend(cm.heading for cm in env.cameras)
        rec["g_idx"].extend(g.current_idx for g in env.guards)
        rec["g_h"].extend(g.heading for g in env.guards)
        rec["vis"].append(env.visibility_map.visibility > 0.5)
        if k < n_state:
            rec["state"].append(env.get_state_tensor())
    return rec


def pack_layouts(items):
    """Flatten (walls, cams, guards) lists into padded arrays + offsets."""
    W, Wo, Cm, Co, Gp, Gi, Gf, Go, Pp = [], [0], [], [0], [], [], [], [0], []
    for walls, cams, guards in items:
        for r, c in walls:
            W.append((r, c))
        Wo.append(len(W))
        for cd in cams:
            Cm.append((cd["row"], cd["col"], cd.get("fov_angle", 60.0), cd.get("heading", 0.0),
                       cd.get("rotation_speed", 15.0), cd.get("vision_range", 6)))
        Co.append(len(Cm))
        for gd in guards:
            path = gd["patrol_path"]
            Gi.append((len(Pp), len(path), gd.get("speed", 1), gd.get("vision_range", 4)))
            Gf.append(gd.get("fov_angle", 90.0))
            Pp.extend(path)
        Go.append(len(Gi))
    return dict(walls=np.array(W, np.int32).reshape(-1, 2), walls_off=np.array(Wo, np.int64),
                cams=np.array(Cm, np.float64).reshape(-1, 6), cams_off=np.array(Co, np.int64),
                guards_i=np.array(Gi, np.int64).reshape(-1, 4), guards_fov=np.array(Gf, np.float64),
                guards_off=np.array(Go, np.int64), paths=np.array(Pp, np.int32).reshape(-1, 2))


def make_env_traces():
    rng = np.random.default_rng(20260215)
    cases = []  # (name, R, C, max_steps, budget, layout, n_ops)
    for (R, C, ms, b, w, c, g, name) in hand_layouts():
        cases.append((name, R, C, ms, b, (w, c, g), 400))
    for i, lay in enumerate(architect_layouts(6, 20, 20, 15, 101)):
        cases.append(("arch20_b15_%d" % i, 20, 20, 200, 15, lay, 420))
    for i, lay in enumerate(architect_layouts(3, 20, 20, 40, 102)):
        cases.append(("arch20_b40_%d" % i, 20, 20, 200, 40, lay, 300))
    for i, lay in enumerate(architect_layouts(3, 20, 20, 8, 103, allow_guards=False)):
        cases.append(("arch20_b8_cams_%d" % i, 20, 20, 200, 8, lay, 300))
    for i, lay in enumerate(architect_layouts(2, 20, 20, 5, 104, allow_cams=False, allow_guards=False)):
        cases.append(("arch20_walls_%d" % i, 20, 20, 200, 5, lay, 300))
    for i, lay in enumerate(architect_layouts(2, 10, 10, 5, 105)):
        cases.append(("arch10_b5_%d" % i, 10, 10, 200, 5, lay, 300))
    for i, lay in enumerate(architect_layouts(2, 32, 32, 27, 106)):
        cases.append(("arch32_b27_%d" % i, 32, 32, 200, 27, lay, 250))
    for i in range(6):
        R = C = 20
        lay = synth_layout(rng, R, C, 15, int_params=(i % 2 == 0))
        cases.append(("synth20_%d" % i, R, C, 200, 15, lay, 400))
    for i in range(2):
        lay = synth_layout(rng, 32, 32, 40, n_cams=4, n_guards=3)
        cases.append(("synth32_%d" % i, 32, 32, 200, 40, lay, 250))
    lay = synth_layout(rng, 24, 17, 25, n_cams=3, n_guards=2)
    cases.append(("synth24x17", 24, 17, 80, 25, lay, 300))

    names, cfgs, valid, layouts, grids, nacc = [], [], [], [], [], []
    ops_all, ops_off = [], [0]
    out = {k: [] for k in ("reward", "done", "status", "pos", "tick", "cam_h", "g_idx", "g_h")}
    vis_bits, state = [], []
    n_state = 24
    for (name, R, C, ms, b, lay, n_ops) in cases:
        cfg = EnvironmentConfig(grid_rows=R, grid_cols=C, max_steps=ms, architect_budget=b)
        ops = gen_ops(rng, n_ops, R, C)
        if name == "vault_last_tick":
            ops = [-1, 2, 2, 4, 4, 0, 4, 0]  # vault on tick 6 == max_steps
        if name == "sanity":
            ops = [-1, 4, 4, 4, 4, 4, 4, -1] + ops[1:]
        if name == "empty10":
            ops = [-1] + [2] * 7 + [4] * 7 + [3, -1] + ops[1:]
        rec = run_trace(cfg, lay, ops, n_state, b)
        names.append(name)
        cfgs.append((R, C, ms, cfg.start_pos[0], cfg.start_pos[1], cfg.vault_pos[0], cfg.vault_pos[1], b))
        valid.append(rec["valid"]); layouts.append(lay); grids.append(rec["grid"].reshape(-1).astype(np.int8))
        nacc.append((rec["n_walls"], rec["n_cams"], rec["n_guards"], rec["spent"]))
        ops_all.extend(ops); ops_off.append(len(ops_all))
        for k in out:
            out[k].extend(rec[k])
        vis_bits.append(np.packbits(np.array(rec["vis"]).reshape(len(ops), -1), axis=1).reshape(-1))
        state.append(np.array(rec["state"], np.float32).reshape(-1))
        print("trace %-20s %dx%d valid=%s cams=%d guards=%d ops=%d" % (name, R, C, rec["valid"], rec["n_cams"], rec["n_guards"], len(ops)), flush=True)
    arrs = pack_layouts(layouts)
    arrs.update(
        names=np.array(names), cfg=np.array(cfgs, np.int64), valid=np.array(valid, bool),
        grid=np.concatenate(grids), accepted=np.array(nacc, np.int64),
        ops=np.array(ops_all, np.int8), ops_off=np.array(ops_off, np.int64),
        reward=np.array(out["reward"], np.float64), done=np.array(out["done"], bool),
        status=np.array(out["status"], np.int8), pos=np.array(out["pos"], np.int16).reshape(-1, 2),
        tick=np.array(out["tick"], np.int32), cam_h=np.array(out["cam_h"], np.float64),
        g_idx=np.array(out["g_idx"], np.int32), g_h=np.array(out["g_h"], np.float64),
        vis_bits=np.concatenate(vis_bits), state=np.concatenate(state), n_state=np.int64(n_state))
    np.savez_compressed(os.path.join(OUT, "env_traces.npz"), **arrs)


# ---------------------------------------------------------------------------
# cone sweeps and BFS
# ---------------------------------------------------------------------------

def make_cones():
    rng = np.random.default_rng(7)
    rows = []  # kind, R, C, r, c, fov, heading, range, wall_density, seed
    vis = []
    walls_all = []
    for i in range(1500):
        R, C = [(20, 20), (32, 32), (10, 10), (13, 21)][i % 4]
        dens = [0.0, 0.1, 0.25][i % 3]
        wm = rng.random((R, C)) < dens
        wm[0, :] = wm[-1, :] = wm[:, 0] = wm[:, -1] = True
        r, c = int(rng.integers(1, R - 1)), int(rng.integers(1, C - 1))
        wm[r, c] = False
        kind = i % 3  # 0 camera f32 params, 1 camera integer params, 2 guard
        if kind == 0:
            fov, head = f32(rng.uniform(30, 120)), f32(rng.uniform(0, 360))
            rngv = int(rng.choice([4, 6, 8]))
        elif kind == 1:
            fov = float(rng.choice([30, 45, 60, 75, 90, 120]))
            head = float(rng.integers(0, 72) * 5) - (360.0 if rng.random() < 0.1 else 0.0)
            rngv = int(rng.choice([4, 6, 8]))
        else:
            fov = float(rng.choice([90.0, 60.0, 120.0, 45.0]))
            head = float(rng.choice([0.0, 90.0, 180.0, 270.0, 135.0, 26.565051177077994]))
            rngv = int(rng.choice([3, 4, 5]))
        if kind < 2:
            tiles = Camera(row=r, col=c, fov_angle=fov, heading=head, vision_range=rngv).get_vision_cone_tiles(R, C, wm)
        else:
            tiles = Guard(patrol_path=[(r, c)], vision_range=rngv, fov_angle=fov, heading=head).get_visible_tiles(R, C, wm)
        v = np.zeros((R, C), bool)
        for (tr, tc) in tiles:
            v[tr, tc] = True
        rows.append((kind, R, C, r, c, rngv))
        vis.append((fov, head))
        walls_all.append(np.packbits(wm.reshape(-1)))
        walls_all[-1] = (walls_all[-1], np.packbits(v.reshape(-1)))
    np.savez_compressed(os.path.join(OUT, "cones.npz"), meta=np.array(rows, np.int64), params=np.array(vis, np.float64),
                        walls=np.concatenate([w for w, _ in walls_all]), tiles=np.concatenate([t for _, t in walls_all]))


def make_cone_order():
    """The LIST order of get_vision_cone_tiles / get_visible_tiles (first visit by ray, then
    by distance): per case the ordered flat tile indices r * C + c."""
    rng = np.random.default_rng(17)
    rows, vis, walls, order, lens = [], [], [], [], []
    for i in range(600):
        R, C = [(20, 20), (32, 32), (10, 10), (13, 21)][i % 4]
        dens = [0.0, 0.1, 0.25][i % 3]
        wm = rng.random((R, C)) < dens
        wm[0, :] = wm[-1, :] = wm[:, 0] = wm[:, -1] = True
        r, c = int(rng.integers(1, R - 1)), int(rng.integers(1, C - 1))
        wm[r, c] = False
        kind = i % 3  # 0 camera f32 params, 1 camera integer params, 2 guard
        if kind == 0:
            fov, head = f32(rng.uniform(30, 120)), f32(rng.uniform(0, 360))
            rngv = int(rng.choice([4, 6, 8]))
        elif kind == 1:
            fov = float(rng.choice([30, 45, 60, 75, 90, 120]))
            head = float(rng.integers(0, 72) * 5)
            rngv = int(rng.choice([4, 6]))
        else:
            fov = float(rng.choice([90.0, 60.0, 120.0]))
            head = float(rng.choice([0.0, 90.0, 180.0, 270.0, 135.0]))
            rngv = int(rng.choice([3, 4, 5]))
        if kind < 2:
            tiles = Camera(row=r, col=c, fov_angle=fov, heading=head, vision_range=rngv).get_vision_cone_tiles(R, C, wm)
        else:
            tiles = Guard(patrol_path=[(r, c)], vision_range=rngv, fov_angle=fov, heading=head).get_visible_tiles(R, C, wm)
        rows.append((1 if kind == 2 else 0, R, C, r, c, rngv))
        vis.append((fov, head))
        walls.append(np.packbits(wm.reshape(-1)))
        order.extend(tr * C + tc for tr, tc in tiles)
        lens.append(len(tiles))
    np.savez_compressed(os.path.join(OUT, "cone_order.npz"), meta=np.array(rows, np.int64),
                        params=np.array(vis, np.float64), walls=np.concatenate(walls),
                        order=np.array(order, np.int32), lens=np.array(lens, np.int32))


def make_bfs():
    rng = np.random.default_rng(11)
    meta, grids, res = [], [], []
    for i in range(3000):
        R, C = [(20, 20), (10, 10), (32, 32), (7, 19)][i % 4]
        g = create_empty_grid(R, C)
        dens = rng.uniform(0.05, 0.55)
        m = rng.random((R, C)) < dens
        g[m] = TileType.WALL
        g[0, :] = g[-1, :] = g[:, 0] = g[:, -1] = TileType.WALL
        start, goal = (1, 1), (R - 2, C - 2)
        if i % 10 == 0:
            start = goal
        if i % 7 == 0:
            g[rng.integers(1, R - 1), rng.integers(1, C - 1)] = TileType.GUARD
        g[start] = TileType.START if i % 5 else TileType.WALL  # start tile itself never checked
        g[goal] = TileType.VAULT
        meta.append((R, C, start[0], start[1], goal[0], goal[1]))
        grids.append(g.reshape(-1).astype(np.int8))
        res.append(bfs_path_exists(g, start, goal))
    np.savez_compressed(os.path.join(OUT, "bfs.npz"), meta=np.array(meta, np.int64), grids=np.concatenate(grids), valid=np.array(res, bool))


# ---------------------------------------------------------------------------
# GAE and PPO loss
# ---------------------------------------------------------------------------

class _StubNet(torch.nn.Module):
    """Returns fixed per-sample logits/values; state[:,0,0,0] is the sample id."""

    def __init__(self, logits, values):
        super().__init__()
        self.L = torch.nn.Parameter(torch.tensor(logits))
        self.V = torch.nn.Parameter(torch.tensor(values).reshape(-1, 1))

    def forward(self, states, hidden=None):
        idx = states[:, 0, 0, 0].long()
        return self.L[idx], self.V[idx], hidden


def make_ppo():
    rng = np.random.default_rng(5)
    agent = SolverAgent(grid_rows=4, grid_cols=4)
    gae_cases = []
    for T in (1, 2, 7, 64, 200, 513):
        r = rng.normal(0, 1, T).astype(np.float32)
        r[rng.random(T) < 0.05] += 10.0
        v = rng.normal(0, 1, T).astype(np.float32)
        d = (rng.random(T) < 0.08).astype(np.float32)
        d[-1] = 1.0 if T % 2 else 0.0
        adv = agent._compute_gae(torch.tensor(r), torch.tensor(v), torch.tensor(d)).numpy()
        ret = adv + v
        an = torch.tensor(adv)
        norm = ((an - an.mean()) / (an.std() + 1e-8)).numpy() if T > 1 else adv
        gae_cases.append((r, v, d, adv, ret, norm))
    loss_cases = []
    for M, scale, clipmix in ((64, 1.0, 0.0), (64, 3.0, 0.5), (17, 0.1, 0.9), (1, 1.0, 0.0), (200, 8.0, 0.3)):
        logits = (rng.normal(0, scale, (M, 5))).astype(np.float32)
        if M > 20:
            logits[0] = [60.0, -60.0, 0.0, 1.0, -1.0]  # forces the probability clamp
        values = rng.normal(0, 1, M).astype(np.float32)
        actions = rng.integers(0, 5, M)
        p = torch.softmax(torch.tensor(logits), -1)
        logp = torch.log(torch.clamp(p.gather(1, torch.tensor(actions)[:, None])[:, 0], 1.1920929e-07, 1 - 1.1920929e-07)).numpy()
        old = (logp + rng.normal(0, 0.3, M) * (rng.random(M) < clipmix + 0.5)).astype(np.float32)
        rewards = rng.normal(0, 1, M).astype(np.float32)
        dones = (rng.random(M) < 0.1)
        dones[-1] = True
        vals_roll = rng.normal(0, 1, M).astype(np.float32)
        # Drive the reference update() with a stub network: one epoch, one minibatch
        # of everything, lr 0 and no clipping so .grad holds d(loss)/d(logits, values).
        ag = SolverAgent(grid_rows=1, grid_cols=1, lr=0.0, max_grad_norm=1e30, ppo_epochs=1, batch_size=10 ** 6)
        ag.network = _StubNet(logits, values)
        ag.optimizer = torch.optim.SGD(ag.network.parameters(), lr=0.0)
        for i in range(M):
            ag.states.append(np.full((1, 1, 1), float(i), np.float32))
            ag.actions.append(int(actions[i])); ag.log_probs.append(float(old[i]))
            ag.values.append(float(vals_roll[i])); ag.rewards.append(float(rewards[i])); ag.dones.append(bool(dones[i]))
        np.random.seed(0)
        m = ag.update()
        adv = ag._compute_gae(torch.tensor(rewards), torch.tensor(vals_roll), torch.tensor(dones.astype(np.float32)))
        ret = (adv + torch.tensor(vals_roll)).numpy()
        adv_n = ((adv - adv.mean()) / (adv.std() + 1e-8)).numpy() if M > 1 else adv.numpy()
        loss_cases.append(dict(logits=logits, values=values, actions=actions.astype(np.int64), old=old,
                               rewards=rewards, dones=dones, vals_roll=vals_roll, adv=adv_n.astype(np.float32),
                               ret=ret.astype(np.float32), pg=m["solver_policy_loss"], vl=m["solver_value_loss"],
                               ent=m["solver_entropy"], dlogits=ag.network.L.grad.numpy().copy(),
                               dvalues=ag.network.V.grad.numpy().reshape(-1).copy()))
    arrs = {}
    for i, (r, v, d, adv, ret, norm) in enumerate(gae_cases):
        arrs.update({"gae%d_r" % i: r, "gae%d_v" % i: v, "gae%d_d" % i: d, "gae%d_adv" % i: adv,
                     "gae%d_ret" % i: ret, "gae%d_norm" % i: norm})
    for i, c in enumerate(loss_cases):
        for k, val in c.items():
            arrs["loss%d_%s" % (i, k)] = np.asarray(val)
    arrs["n_gae"] = np.int64(len(gae_cases)); arrs["n_loss"] = np.int64(len(loss_cases))
    np.savez_compressed(os.path.join(OUT, "ppo.npz"), **arrs)


# ---------------------------------------------------------------------------
# networks and architect decode
# ---------------------------------------------------------------------------

def make_nets():
    arrs = {}
    torch.manual_seed(31)
    sn = SolverNetwork(grid_rows=20, grid_cols=20)
    for k, v in sn.state_dict().items():
        arrs["solver/" + k] = v.numpy()
    x = torch.randn(6, 3, 20, 20)
    h = (torch.randn(1, 6, 128) * 0.5, torch.randn(1, 6, 128) * 0.5)
    with torch.no_grad():
        lg, val, (h1, c1) = sn(x, h)
        lg0, val0, (h0, c0) = sn(x)
    arrs.update({"solver_in": x.numpy(), "solver_h": h[0].numpy(), "solver_c": h[1].numpy(),
                 "solver_logits": lg.numpy(), "solver_value": val.numpy(), "solver_h1": h1.numpy(), "solver_c1": c1.numpy(),
                 "solver_logits0": lg0.numpy(), "solver_value0": val0.numpy()})
    torch.manual_seed(32)
    an = ArchitectNetwork(grid_rows=20, grid_cols=20)
    for k, v in an.state_dict().items():
        arrs["architect/" + k] = v.numpy()
    gs = np.zeros((1, 1, 20, 20), np.float32)
    gs[0, 0, 1, 1] = TileType.START / 5.0
    gs[0, 0, 18, 18] = TileType.VAULT / 5.0
    with torch.no_grad():
        pl, av, cp = an(torch.tensor(gs))
    arrs.update({"arch_in": gs, "arch_logits": pl.numpy(), "arch_value": av.numpy(),
                 "arch_fov": cp["fov"].numpy(), "arch_speed": cp["speed"].numpy(), "arch_heading": cp["heading"].numpy()})
    # decode cases: record the sampled class map by re-running the sampler with the same seed
    dec_meta, dec_maps, dec_out = [], [], []
    rng = np.random.default_rng(3)
    for i in range(40):
        R = C = [20, 10, 32, 20][i % 4]
        budget = int([5, 8, 15, 22, 40, 27][i % 6])
        temp = float([1.0, 0.5, 2.0, 1.3][i % 4])
        net = ArchitectNetwork(grid_rows=R, grid_cols=C)
        with torch.no_grad():
            for p in net.parameters():
                p.add_(torch.randn_like(p) * 0.3)
        g = np.zeros((1, 1, R, C), np.float32)
        seed = 1000 + i
        torch.manual_seed(seed)
        with torch.no_grad():
            walls, cams, guards, tlp, val = net.generate_layout(torch.tensor(g), budget, temp)
        torch.manual_seed(seed)
        with torch.no_grad():
            pl, _, cp = net(torch.tensor(g))
            probs = torch.softmax(pl / temp, dim=1)
            flat = probs.view(1, 4, -1).permute(0, 2, 1)
            sampled = torch.distributions.Categorical(flat).sample()
        amap = sampled.view(R, C).numpy().astype(np.int8)
        dec_meta.append((R, C, budget, len(walls), len(cams), len(guards)))
        dec_maps.append(amap.reshape(-1))
        cam_p = (float(cp["fov"].item()), float(cp["speed"].item()), float(cp["heading"].item()))
        lay = [list(w) for w in walls], [(c["row"], c["col"]) for c in cams], [g_["patrol_path"] for g_ in guards]
        dec_out.append({"cam_params": cam_p, "walls": lay[0], "cams": lay[1], "guards": lay[2],
                        "total_log_prob": float(tlp.item()), "temperature": temp})
    arrs["dec_meta"] = np.array(dec_meta, np.int64)
    arrs["dec_maps"] = np.concatenate(dec_maps)
    np.savez_compressed(os.path.join(OUT, "nets.npz"), **arrs)
    with open(os.path.join(OUT, "architect_decode.json"), "w") as f:
        json.dump(dec_out, f)


def make_kat():
    kat = {}
    cfg = EnvironmentConfig(grid_rows=10, grid_cols=10, start_pos=(1, 1), vault_pos=(8, 8))
    env = HeistEnvironment(cfg)
    valid = env.set_layout([(3, 3), (3, 4), (3, 5)],
                           [{"row": 5, "col": 5, "fov_angle": 60, "heading": 0, "rotation_speed": 15, "vision_range": 4}],
                           [{"patrol_path": [(7, 2), (7, 3), (7, 4), (7, 5)], "speed": 1, "vision_range": 3, "fov_angle": 90}])
    env.reset()
    rews = []
    for _ in range(5):
        _, r, d, info = env.step(4)
        rews.append(r)
        if d:
            break
    kat["sanity"] = {"valid": bool(valid), "pos": list(env.solver_pos), "tick": env.tick, "status": info["status"],
                     "rewards": rews, "surveilled": int(np.sum(env.visibility_map.visibility > 0.5)),
                     "render": env.render_text()}
    env = HeistEnvironment(EnvironmentConfig(grid_rows=10, grid_cols=10))
    env.set_layout([], [], [])
    env.reset()
    tot = 0.0
    for _ in range(7):
        _, r, d, info = env.step(2)
        tot += r
    kat["fixes_down"] = tot
    for _ in range(7):
        _, r, d, info = env.step(4)
        tot += r
        if d:
            break
    kat["fixes_right"] = tot
    kat["fixes_status"] = info["status"]
    env2 = HeistEnvironment(EnvironmentConfig(grid_rows=10, grid_cols=10))
    env2.set_layout([], [], [])
    env2.reset()
    st = env2.get_state_tensor()
    kat["pos_channel_min"] = float(st[2].min())
    kat["pos_channel_max"] = float(st[2].max())
    kat["params"] = {"architect": sum(p.numel() for p in ArchitectNetwork(10, 10).parameters()),
                     "solver": sum(p.numel() for p in SolverNetwork(10, 10).parameters())}
    kat["architect_reward"] = {str(s): RewardCalculator().calculate_architect_reward(env2, s)
                               for s in (0.0, 0.1, 0.2, 0.5, 0.6, 0.7, 0.8, 0.81, 1.0)}
    with open(os.path.join(OUT, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)


def proj_vectors(i, n, k=4):
    """The fixed projection vectors of parameter tensor i (also used by the tests)."""
    return np.random.default_rng(7000 + i).standard_normal((k, n))


ARCH_CASES = [  # (log_probs, values, rewards) per update; consecutive updates of one agent
    [([-52.5], [0.02], [1.0])],
    [([-61.25], [-0.013], [-1.0])],
    [([-50.0, -55.5, -48.25, -60.0, -51.0], [0.01, 0.01, 0.01, 0.01, 0.01], [1.0, -1.0, 0.7, 0.2, -0.5])],
    [([-53.0], [0.015], [0.6]), ([-58.0], [0.011], [-0.5]), ([-49.5, -50.5], [0.012, 0.012], [1.2, 0.3])],
]


def make_arch_update():
    from heist_architect.agents.architect import ArchitectAgent
    z = np.load(os.path.join(OUT, "nets.npz"), allow_pickle=False)
    sd = {k[len("architect/"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("architect/")}
    arrs = {"n_cases": np.int64(len(ARCH_CASES))}
    for ci, case in enumerate(ARCH_CASES):
        ag = ArchitectAgent(grid_rows=20, grid_cols=20, budget=15)
        ag.network.load_state_dict(sd)
        for ui, (lps, vals, rews) in enumerate(case):
            p0 = [p.detach().clone() for p in ag.network.parameters()]
            ag.log_probs = [torch.tensor(x) for x in lps]
            ag.values = [torch.tensor([[x]]) for x in vals]
            ag.rewards = []
            for r in rews:
                ag.store_reward(r)
            m = ag.update()
            key = "c%d_u%d_" % (ci, ui)
            arrs[key + "lp"] = np.array(lps, np.float32)
            arrs[key + "v"] = np.array(vals, np.float32)
            arrs[key + "r"] = np.array(rews, np.float64)
            arrs[key + "loss"] = np.array([m["architect_policy_loss"], m["architect_value_loss"],
                                           m["architect_total_loss"]], np.float64)
            gn, gp, dn, dp = [], [], [], []
            for i, (p, q) in enumerate(zip(ag.network.parameters(), p0)):
                g = (p.grad if p.grad is not None else torch.zeros_like(p)).detach().double().reshape(-1).numpy()
                d = (p.detach() - q).double().reshape(-1).numpy()
                P = proj_vectors(i, g.size)
                gn.append(np.linalg.norm(g))
                dn.append(np.linalg.norm(d))
                gp.append(P @ g)
                dp.append(P @ d)
            arrs[key + "gnorm"] = np.array(gn)
            arrs[key + "gproj"] = np.array(gp)
            arrs[key + "dnorm"] = np.array(dn)
            arrs[key + "dproj"] = np.array(dp)
        arrs["c%d_n" % ci] = np.int64(len(case))
    np.savez_compressed(os.path.join(OUT, "arch_update.npz"), **arrs)


if __name__ == "__main__":
    which = sys.argv[1:] or ["kat", "bfs", "cones", "ppo", "nets", "env", "arch", "order"]
    for w in which:
        print("==", w, flush=True)
        {"kat": make_kat, "bfs": make_bfs, "cones": make_cones, "ppo": make_ppo,
         "nets": make_nets, "env": make_env_traces, "arch": make_arch_update, "order": make_cone_order}[w]()
