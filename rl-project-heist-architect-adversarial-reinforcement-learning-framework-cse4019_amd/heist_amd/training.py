"""Adversarial training loop (reference: heist_architect/training.py), batched.

The reference plays one layout at a time: Architect samples a layout, the Solver makes
`solver_episodes_per_layout` sequential attempts on it (camera headings carry over),
then both agents update (training.py:418-600).  Here N environments run at once on one
GPU (and N per rank across GPUs):

  * every env holds its own Architect layout and counts its attempts; after an env's
    A-th attempt its layout is scored (solve/detect/timeout rates -> RewardCalculator)
    and replaced by a fresh Architect sample (masked heist_set_layout + heist_reset);
  * the Solver steps all envs for `rollout_len` ticks (batched policy forward, heist_step
    with in-kernel auto-reset writing each tick's observation straight into the rollout
    buffer, per-env LSTM state zeroed when an attempt ends), then does one PPO update on
    the [T, N] rollout: heist_gae per env column, bootstrapping V(s_T) where the rollout
    cuts an attempt (the reference's buffer always ends on done, so its 0 bootstrap is
    this with no cut), global advantage normalisation, heist_ppo_loss;
  * the Architect takes one reference-style single-reward step per layout scored during
    the rollout, in episode order (architect_update="per_layout", the default: the
    reference calls update() after every layout, training.py:479-480, :558-559, so its
    value target is the raw reward); architect_update="batched" instead runs the
    reference's update formula once over all of them, which normalises k > 1 rewards and so
    trains the value towards 0 -- faster, but not the reference's Architect learning.
Data parallel (one process per GPU, torch.distributed): every collective is called the
same number of times on every rank -- the Solver's minibatch count is agreed by a max
all-reduce, the Architect's statistics are all-reduced, episode numbers are handed out
in rank order from a global counter, so the curriculum phase, checkpoint cadence and the
end of train() are the same decision on every rank (dist_utils).
Episode numbering, the curriculum, GameLogEntry / TrainingMetrics JSON and checkpoint
file names follow the reference, so its dashboard and resume logic read our logs.
A layout may see a few extra attempts beyond A before the rollout ends; those train
the Solver but do not enter the layout's statistics.
"""
import glob
import json
import os
import re
import time
from collections import deque
from datetime import datetime
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import dist_utils
from .agents.architect import ArchitectAgent
from .agents.solver import Rollout, SolverAgent
from .environment import EnvironmentConfig, HeistEnvironment, accept_layout
from .rewards import RewardCalculator
from .utils import DEVICE
from .vec_env import STATUS_CODES, HeistEnv


class GameLogEntry:  # training.py:35-68
    def __init__(self, episode: int, phase: str, budget: int, walls: int, cameras: int, guards: int,
                 solve_rate: float, detection_rate: float, timeout_rate: float, architect_reward: float,
                 solver_reward: float, avg_steps: float, level_valid: bool, is_interactive: bool = False,
                 freeze_architect: bool = False, freeze_solver: bool = False, temperature: float = 1.0,
                 timestamp: str = ""):
        self.data = {
            "episode": episode, "phase": phase, "budget": budget, "walls": walls, "cameras": cameras,
            "guards": guards, "solve_rate": round(solve_rate, 3), "detection_rate": round(detection_rate, 3),
            "timeout_rate": round(timeout_rate, 3), "architect_reward": round(architect_reward, 3),
            "solver_reward": round(solver_reward, 3), "avg_steps": round(avg_steps, 1), "level_valid": level_valid,
            "is_interactive": is_interactive, "freeze_architect": freeze_architect, "freeze_solver": freeze_solver,
            "temperature": round(temperature, 2), "timestamp": timestamp or datetime.now().strftime("%H:%M:%S"),
        }

    def to_dict(self):
        return self.data

    @classmethod
    def batch(cls, cols: Dict[str, Sequence]) -> List["GameLogEntry"]:
        """Entries from per-field columns whose float fields are already rounded as
        __init__ rounds them (np.round on an array equals round() on each of its numpy
        scalars, value and type); the per-entry dict build is all that is left per row."""
        keys = list(cols)
        out = []
        # list() first: zipping ndarrays row by row is ~15x slower (numpy scalars made
        # one at a time); list() of an ndarray holds the same numpy scalars
        for row in zip(*(list(cols[k]) for k in keys)):
            e = cls.__new__(cls)
            e.data = dict(zip(keys, row))
            out.append(e)
        return out


class TrainingMetrics:  # training.py:71-112
    KEYS = ("episode", "solve_rate", "detection_rate", "timeout_rate", "architect_reward", "solver_reward",
            "architect_loss", "solver_loss", "avg_steps", "budget", "phase")

    def __init__(self):
        self.history = {k: [] for k in self.KEYS}
        self.recent_solve_rates = deque(maxlen=50)

    def log(self, episode: int, metrics: Dict):
        for key in self.history:
            if key in metrics:
                self.history[key].append(metrics[key])
        self.history["episode"].append(episode)

    def save(self, path: str):
        with open(path, "w") as f:
            json.dump(self.history, f, indent=2)

    def load(self, path: str):
        if os.path.exists(path):
            with open(path) as f:
                self.history = json.load(f)

    def records(self) -> List[Dict]:
        """Per-episode rows (the inverse of log); keys missing for an episode are absent."""
        eps = self.history.get("episode", [])
        cols = {k: v for k, v in self.history.items() if k != "episode"}
        # the reference logs only the keys an episode's metrics carry (invalid layouts have
        # no losses), so per-key lists can be shorter than "episode": align them from the end
        return [{"episode": e} for e in eps] if not cols else _rows(eps, cols)

    @classmethod
    def from_records(cls, rows: List[Dict]) -> "TrainingMetrics":
        m = cls()
        for r in sorted(rows, key=lambda r: r["episode"]):
            m.log(r["episode"], {k: v for k, v in r.items() if k != "episode"})
        return m

    def get_summary(self, last_n: int = 10) -> str:
        lines = []
        for key in ("solve_rate", "detection_rate", "architect_reward", "solver_reward"):
            vals = self.history.get(key, [])
            if vals:
                lines.append("  %s: %.3f" % (key, float(np.mean(vals[-last_n:]))))
        return "\n".join(lines)


CURRICULA = {
    # (episode_threshold, budget, allow_cameras, allow_guards, description)
    "reference": [(0, 5, False, False, "Walls Only"),  # training.py:128-133
                  (80, 8, True, False, "Walls + Cameras"),
                  (200, 15, True, True, "Full Security"),
                  (400, 22, True, True, "Expert")],
    # BASELINE config 4: the full adversarial curriculum over budgets 10 -> 40
    "c4": [(0, 10, False, False, "Walls Only"),
           (80, 20, True, False, "Walls + Cameras"),
           (200, 30, True, True, "Full Security"),
           (400, 40, True, True, "Expert")],
}


class AdversarialTrainer:  # training.py:115-790
    CURRICULUM = CURRICULA["reference"]
    WARMUP_EPISODES = 30

    def __init__(self, config: Optional[EnvironmentConfig] = None, solver_episodes_per_layout: int = 20,
                 total_episodes: int = 500, save_dir: str = "checkpoints", log_dir: str = "logs",
                 architect_lr: float = 3e-4, solver_lr: float = 1e-3, n_envs: int = 256,
                 rollout_len: Optional[int] = None, minibatch: int = 4096, device=None, max_budget: Optional[int] = None,
                 seed: Optional[int] = None, update_precision: str = "fp32", rollout_precision: str = "fp32",
                 curriculum: Union[str, Sequence[Tuple], None] = None, architect_update: str = "per_layout",
                 solver_cadence: str = "rollout"):
        self.config = config or EnvironmentConfig()
        self.solver_episodes = solver_episodes_per_layout
        self.total_episodes = total_episodes
        self.save_dir = save_dir
        self.log_dir = log_dir
        self.device = torch.device(device) if device is not None else DEVICE
        self.n_envs = n_envs
        self.rollout_len = rollout_len or self.config.max_steps
        self.minibatch = minibatch
        if isinstance(curriculum, str):
            if curriculum not in CURRICULA:
                raise ValueError("unknown curriculum %r (presets: %s)" % (curriculum, ", ".join(CURRICULA)))
            curriculum = CURRICULA[curriculum]
        if curriculum is not None:
            self.CURRICULUM = [tuple(p) for p in curriculum]
        if architect_update not in ("batched", "per_layout"):
            raise ValueError("architect_update must be 'batched' or 'per_layout'")
        self.architect_update = architect_update
        # "rollout": one Solver update per rollout_len-tick window (V(s_T) bootstrap where the
        # window cuts an attempt); "layout_batch": the reference's cadence (training.py:515-565)
        # for all envs at once -- every env plays its layout's A attempts to done, then one
        # update on exactly those transitions, GAE bootstrapping 0 at each env's buffer end and
        # advantages normalised per layout buffer (agents/solver.py:142-147)
        if solver_cadence not in ("rollout", "layout_batch"):
            raise ValueError("solver_cadence must be 'rollout' or 'layout_batch'")
        self.solver_cadence = solver_cadence
        if seed is not None:  # one stream per rank: ranks must not replay each other's layouts and actions
            torch.manual_seed(seed + dist_utils.rank())
            np.random.seed(seed + dist_utils.rank())
        mb = max_budget or max(b for _, b, _, _, _ in self.CURRICULUM)
        mb = max(mb, self.config.architect_budget)
        self.env = HeistEnv(n_envs, self.config, max_cams=max(1, mb // 3), max_guards=max(1, mb // 5), max_path=8,
                            device=self.device, auto_reset=True)
        R, C = self.config.grid_rows, self.config.grid_cols
        self.architect = ArchitectAgent(grid_rows=R, grid_cols=C, budget=self.config.architect_budget,
                                        lr=architect_lr, device=self.device)
        self.solver = SolverAgent(grid_rows=R, grid_cols=C, lr=solver_lr, device=self.device,
                                  update_precision=update_precision, rollout_precision=rollout_precision)
        if dist_utils.is_multi():  # replicas start equal: rank 0's initial weights everywhere
            ts = [t for net in (self.architect.network, self.solver.network)
                  for t in list(net.parameters()) + list(net.buffers())]
            flat = torch.cat([t.detach().reshape(-1).float() for t in ts])
            torch.distributed.broadcast(flat, 0)
            o = 0
            for t in ts:
                t.data.copy_(flat[o:o + t.numel()].view(t.shape))
                o += t.numel()
        self.reward_calc = RewardCalculator()
        self.metrics = TrainingMetrics()
        self.game_log: List[GameLogEntry] = []
        self.global_episode = 0
        self.current_state = None
        self.training_active = False
        self._single_env = None
        self._callback = None
        self._trace = None  # list: _rollout appends (actions, reward64, done, status) per tick
        self._arch_eps: List[int] = []  # episode number of each Architect buffer transition
        os.makedirs(save_dir, exist_ok=True)
        os.makedirs(log_dir, exist_ok=True)
        self._init_batch_state()

    # -- per-env bookkeeping (device tensors) ----------------------------------------
    def _init_batch_state(self):
        n, d = self.n_envs, self.device
        z = lambda dt=torch.int32: torch.zeros(n, dtype=dt, device=d)  # noqa: E731
        self.b_attempts, self.b_solve, self.b_detect, self.b_timeout, self.b_steps = z(), z(), z(), z(), z()
        self.b_reward = z(torch.float64)
        self.b_valid = torch.zeros(n, dtype=torch.bool, device=d)
        self.b_logp = z(torch.float32)   # the layout's Architect log-prob and value (agents/architect.py:75-81)
        self.b_value = z(torch.float32)
        self.b_episode = np.zeros(n, np.int64)
        self.b_meta = [None] * n  # (phase, budget, walls, cameras, guards, temperature)
        self.b_layout = [None] * n  # (LayoutBatch sized n, row) of the env's current layout; None: empty
        self.b_scored = torch.zeros(n, dtype=torch.bool, device=d)
        self.h = torch.zeros(1, n, self.solver.network.lstm_hidden, device=d)
        self.c = torch.zeros_like(self.h)
        self.warmup = False

    def get_curriculum_phase(self, episode: int):  # training.py:265-271
        phase = self.CURRICULUM[0]
        for threshold, budget, cams, guards, desc in self.CURRICULUM:
            if episode >= threshold:
                phase = (threshold, budget, cams, guards, desc)
        return phase

    def _temperature(self, episode: int) -> float:  # training.py:451
        return max(0.5, 2.0 - episode / max(self.total_episodes, 1) * 1.5)

    def _assign_layouts(self, env_ids, overrides: Optional[dict] = None, empty: bool = False):
        """New Architect layouts for env_ids (one episode number each); invalid layouts are
        scored -1 and resampled, as the reference skips their solver phase.  Collective:
        every rank calls it once per iteration (with any number of env ids, also none);
        episode numbers come from the global counter in rank order, and the curriculum
        phase of a round is that of its first global episode, the same on every rank."""
        ov = overrides or {}
        pending = np.asarray(env_ids, np.int64)
        rk = dist_utils.rank()
        for tries in range(8):
            counts = dist_utils.allgather_counts(len(pending), self.device).numpy()
            total = int(counts.sum())
            if total == 0:
                break
            ep_first = self.global_episode + 1
            ep0 = self.global_episode + int(counts[:rk].sum()) + 1
            self.global_episode += total
            if len(pending) == 0:
                continue
            eps = np.arange(ep0, ep0 + len(pending))
            _, budget, cams, guards, desc = self.get_curriculum_phase(ep_first)
            budget = ov.get("budget", budget)
            cams = ov.get("allow_cameras", cams)
            guards = ov.get("allow_guards", guards)
            temp = ov.get("temperature", self._temperature(ep_first))
            phase = ov.get("phase", desc)
            pidx = torch.as_tensor(pending, device=self.device)
            if empty:
                layouts = [([], [], [])] * len(pending)
                valid = self.env.set_layouts(layouts, budget=budget, env_ids=pending)[pidx]
                counts_l = np.zeros((len(pending), 3), np.int64)
                lb = None
            else:
                self.architect.budget = budget
                lbk, logp, value = self.architect.generate_layouts(len(pending), temp, cams, guards, env=self.env,
                                                                   record=False)
                lb = _scatter_layout(lbk, pending, self.env)
                valid = self.env.set_layout_batch(lb, _mask(pending, self.env))[pidx]
                counts_l = torch.stack([lbk.n_walls, lbk.n_cams, lbk.n_guards], 1).cpu().numpy()
                self.b_logp[pidx] = logp.float()
                self.b_value[pidx] = value.reshape(-1)[0].float()
            v = valid.cpu().numpy()
            for i, e in enumerate(pending):
                self.b_episode[e] = eps[i]
                self.b_meta[e] = (phase, budget, int(counts_l[i, 0]), int(counts_l[i, 1]), int(counts_l[i, 2]), temp)
                self.b_layout[e] = None if lb is None else (lb, int(e))
            bad = pending[~v]
            if len(bad) and not empty and not ov.get("freeze_architect", False):  # training.py:476-504
                bi = torch.as_tensor(bad, device=self.device)
                self.architect.store_transitions(self.b_logp[bi], self.b_value[bi],
                                                 [self.reward_calc.architect_invalid] * len(bad))
                self._arch_eps.extend(int(x) for x in eps[~v])
            for i in np.nonzero(~v)[0]:
                r = self.reward_calc.architect_invalid
                m = {"solve_rate": 0.0, "detection_rate": 0.0, "timeout_rate": 1.0, "architect_reward": r,
                     "solver_reward": 0.0, "avg_steps": 0, "budget": budget, "phase": phase}
                self._log_episode(int(eps[i]), m, counts_l[i], False, temp, ov, env_id=int(pending[i]))
            good = pending[v]
            if len(good):
                m = _mask(good, self.env)
                self.env.reset(m)
                mb = m.bool()
                for t in (self.b_attempts, self.b_solve, self.b_detect, self.b_timeout, self.b_steps):
                    t.masked_fill_(mb, 0)
                self.b_reward.masked_fill_(mb, 0.0)
                self.h[:, mb] = 0.0
                self.c[:, mb] = 0.0
                self.b_valid[mb] = True
                self.b_scored[mb] = False
            pending = bad if tries < 7 else np.zeros(0, np.int64)
            if len(bad) and tries >= 7:
                self.b_valid[torch.as_tensor(bad, device=self.device)] = False

    # -- rollout / scoring ------------------------------------------------------------------
    @torch.no_grad()
    def _tally(self, done, status, A, vault, det):
        """One tick's attempt bookkeeping (training.py:515-544 per env: steps and reward of the
        running attempt, its outcome when it ends) and the fresh LSTM state of the next attempt
        (solver.reset(), :517): one heist_rollout_tally launch on a HIP device (the torch
        expressions below, bit for bit, elsewhere)."""
        n = self.n_envs
        if self.device.type == "cuda" and self.h.is_contiguous() and self.c.is_contiguous():
            from . import _native as nat
            P = nat.ptr
            nat.check(nat.lib().heist_rollout_tally(
                P(self.b_valid), P(self.b_attempts), A, P(done), P(status), P(self.env.reward64), P(self.b_steps),
                P(self.b_reward), P(self.b_solve), P(self.b_detect), P(self.b_timeout), P(self.h), P(self.c),
                int(self.h.shape[-1]), n, nat.stream(self.device)), "heist_rollout_tally")
            return
        counting = self.b_valid & (self.b_attempts < A)
        self.b_steps += counting.int()
        self.b_reward += torch.where(counting, self.env.reward64, torch.zeros_like(self.b_reward))
        fin = counting & done
        st = status.to(torch.int32)
        self.b_solve += (fin & (st == vault)).int()
        self.b_detect += (fin & (st == det)).int()
        self.b_timeout += (fin & (st != vault) & (st != det)).int()
        self.b_attempts += fin.int()
        keep = (~done).to(self.h.dtype).reshape(1, n, 1)  # a new attempt starts with a fresh LSTM state
        self.h = self.h * keep
        self.c = self.c * keep

    def _rollout(self, T: int) -> Rollout:
        """T ticks of all envs.  The observation each tick's action is chosen from is
        obs[t]; heist_step writes the next one straight into obs[t + 1] (the last into
        env.obs), so no per-tick copy.  last_value = V(s_T) under the carried LSTM state
        (zeroed where an attempt just ended; those columns are masked by done anyway)."""
        env, n, d = self.env, self.n_envs, self.device
        obs_buf = torch.empty((T, n) + tuple(env.obs.shape[1:]), dtype=torch.float32, device=d)
        act_buf = torch.empty((T, n), dtype=torch.int64, device=d)
        lp_buf = torch.empty((T, n), dtype=torch.float32, device=d)
        v_buf = torch.empty((T, n), dtype=torch.float32, device=d)
        r_buf = torch.empty((T, n), dtype=torch.float32, device=d)
        d_buf = torch.empty((T, n), dtype=torch.uint8, device=d)
        A = self.solver_episodes
        vault, det = STATUS_CODES["vault_reached"], STATUS_CODES["detected"]
        obs_buf[0].copy_(env.obs)
        for t in range(T):
            a, lp, v, (self.h, self.c) = self.solver.act(obs_buf[t], (self.h, self.c))
            act_buf[t], lp_buf[t], v_buf[t] = a, lp, v
            _, rew, done, status = env.step(a, obs_out=obs_buf[t + 1] if t + 1 < T else None)
            r_buf[t] = rew
            d_buf[t] = done.to(torch.uint8)
            if self._trace is not None:
                self._trace.append((a.clone(), env.reward64.clone(), done.clone(), status.clone()))
            self._tally(done, status, A, vault, det)
        last_value = self.solver.value(env.obs, (self.h, self.c))
        return Rollout(obs_buf, act_buf, lp_buf, v_buf, r_buf, d_buf, mask=self.b_valid.clone(),
                       last_value=last_value)

    @torch.no_grad()
    def _rollout_layout_batch(self) -> Tuple[Rollout, torch.Tensor]:
        """Play until every valid env has finished its layout's A attempts (at most
        A * max_steps ticks; the loop checks every 16 ticks).  Returns the [T, N] rollout and
        sel [T, N] bool: the transitions of each env's A attempts -- the reference's per-layout
        buffer (training.py:515-544) -- in time order; later ticks (an env waiting for the
        others, auto-reset into attempt A + 1) are not selected."""
        env, n, d = self.env, self.n_envs, self.device
        A = self.solver_episodes
        T_max = A * self.config.max_steps
        vault, det = STATUS_CODES["vault_reached"], STATUS_CODES["detected"]
        bufs = {k: [] for k in ("obs", "act", "lp", "v", "r", "d", "sel")}
        obs = env.obs.clone()
        t = 0
        while t < T_max:
            counting = self.b_valid & (self.b_attempts < A)
            if t % 16 == 0 and not bool(counting.any()):
                break
            a, lp, v, (self.h, self.c) = self.solver.act(obs, (self.h, self.c))
            nxt, rew, done, status = env.step(a)
            for k, x in (("obs", obs), ("act", a), ("lp", lp), ("v", v), ("r", rew.clone()),
                         ("d", done.to(torch.uint8)), ("sel", counting)):
                bufs[k].append(x)
            if self._trace is not None:
                self._trace.append((a.clone(), env.reward64.clone(), done.clone(), status.clone()))
            self._tally(done, status, A, vault, det)  # (counting as above; solver.reset() per attempt)
            obs = nxt.clone()
            t += 1
        st = {k: torch.stack(v) for k, v in bufs.items()}
        ro = Rollout(st["obs"], st["act"], st["lp"], st["v"], st["r"], st["d"], mask=self.b_valid.clone(),
                     last_value=None)
        return ro, st["sel"]

    def _score_finished(self, overrides: Optional[dict] = None) -> np.ndarray:
        """Score every env whose layout has had its A attempts; returns those env ids.  The
        Architect's transition buffers are left as plain per-element lists (torch.stack on
        them sees every entry); train_iteration's own path keeps the batches whole."""
        ids = self._score_commit(self._score_prepare(), overrides)
        self._materialize_transitions()
        return ids

    def _materialize_transitions(self):
        for buf in (self.architect.log_probs, self.architect.values):
            if hasattr(buf, "materialize"):
                buf.materialize()

    def _score_prepare(self):
        """The device half of scoring: which envs finished their A attempts, their statistics
        copied to the host, and their layouts' log-prob / value gathered on the device."""
        A = self.solver_episodes
        fin = (self.b_valid & (self.b_attempts >= A) & ~self.b_scored).nonzero().reshape(-1)
        if fin.numel() == 0:
            return None
        stats = torch.stack([self.b_solve[fin], self.b_detect[fin], self.b_timeout[fin], self.b_steps[fin]], 1)
        stats = stats.cpu().numpy().astype(np.float64)
        rews = self.b_reward[fin].cpu().numpy()
        return fin, stats, rews, fin.cpu().numpy(), self.b_logp[fin], self.b_value[fin]

    def _score_commit(self, prep, overrides: Optional[dict] = None, defer_log: bool = False):
        """The host half of scoring (rewards, logs, the Architect's transitions); no GPU wait.
        defer_log=True (no callback set) returns (ids, log): the metrics history / game log
        entries are written when log() is called -- train_iteration calls it once both agents'
        updates are queued, so that host work runs beside them."""
        log = (lambda: None)
        if prep is None:
            ids = np.zeros(0, np.int64)
            return (ids, log) if defer_log else ids
        A = self.solver_episodes
        fin, stats, rews, ids, lp_fin, v_fin = prep
        ov = overrides or {}
        if self._callback is None and not self.warmup:
            ars, log = self._score_log_batch(stats, rews, ids, ov, defer=True)
            if not defer_log:
                log()
            ids_done = True
        else:
            ars, ids_done = [], False
        for i, e in enumerate([] if ids_done else ids):
            s, dt, to, steps = stats[i]
            solve_rate, det_rate, to_rate = s / A, dt / A, to / A
            ar = self.reward_calc.architect_reward_from_rate(True, solve_rate)  # rewards.py:43-73
            ars.append(ar)
            phase, budget, nw, nc, ng, temp = self.b_meta[e]
            m = {"solve_rate": solve_rate, "detection_rate": det_rate, "timeout_rate": to_rate, "architect_reward": ar,
                 "solver_reward": rews[i] / A, "architect_loss": 0, "solver_loss": 0, "avg_steps": steps / A,
                 "budget": budget, "phase": phase}
            self._log_episode(int(self.b_episode[e]), m, (nw, nc, ng), True, temp, ov, env_id=int(e))
        if not ov.get("freeze_architect", False) and not self.warmup:
            self.architect.store_transitions(lp_fin, v_fin, ars)
            self._arch_eps.extend(int(self.b_episode[e]) for e in ids)
            if self._callback is not None:  # user code may read the buffers
                self._materialize_transitions()
        self.b_scored[fin] = True
        return (ids, log) if defer_log else ids

    def _score_log_batch(self, stats, rews, ids, ov, defer: bool = False):
        """_score_commit's per-episode loop for a batch with no callback: the same rewards,
        metrics history, recent solve rates and game-log entries in the same order (element
        types included), built column-wise; the entries share one timestamp.  Returns the
        Architect rewards, or with defer=True (rewards, log): log() writes the history and
        the game log (everything it reads is captured here)."""
        A = self.solver_episodes
        solve, det, to, steps = (stats[:, j] / A for j in range(4))
        srew = rews / A
        rc = self.reward_calc
        ars = [rc.architect_reward_from_rate(True, x) for x in solve]
        metas = [self.b_meta[e] for e in ids]
        eps = [int(x) for x in self.b_episode[ids]]
        ov = dict(ov)
        if defer:
            return ars, (lambda: self._score_log_write(solve, det, to, steps, srew, ars, metas, eps, ov))
        self._score_log_write(solve, det, to, steps, srew, ars, metas, eps, ov)
        return ars

    def _score_log_write(self, solve, det, to, steps, srew, ars, metas, eps, ov):
        h = self.metrics.history
        n = len(eps)
        cols = {"solve_rate": list(solve), "detection_rate": list(det), "timeout_rate": list(to),
                "architect_reward": ars, "solver_reward": list(srew), "architect_loss": [0] * n,
                "solver_loss": [0] * n, "avg_steps": list(steps), "budget": [m[1] for m in metas],
                "phase": [m[0] for m in metas]}
        for key in h:
            if key in cols:
                h[key].extend(cols[key])
        h["episode"].extend(eps)
        self.metrics.recent_solve_rates.extend(cols["solve_rate"])
        stamp = datetime.now().strftime("%H:%M:%S")
        inter, fa, fs = (bool(ov.get(x, False)) for x in ("interactive", "freeze_architect", "freeze_solver"))
        # GameLogEntry's rounding, column-wise (its per-entry round() of numpy scalars was
        # most of the scoring's host time at ~3,800 layouts per iteration)
        ar_col = np.asarray(ars) if all(type(x) is np.float64 for x in ars) else ars
        rnd = (lambda c, d: np.round(c, d) if isinstance(c, np.ndarray) else [round(x, d) for x in c])
        self.game_log.extend(GameLogEntry.batch({
            "episode": eps, "phase": [m[0] for m in metas], "budget": [m[1] for m in metas],
            "walls": [int(m[2]) for m in metas], "cameras": [int(m[3]) for m in metas],
            "guards": [int(m[4]) for m in metas], "solve_rate": rnd(solve, 3), "detection_rate": rnd(det, 3),
            "timeout_rate": rnd(to, 3), "architect_reward": rnd(ar_col, 3), "solver_reward": rnd(srew, 3),
            "avg_steps": rnd(steps, 1), "level_valid": [True] * n, "is_interactive": [inter] * n,
            "freeze_architect": [fa] * n, "freeze_solver": [fs] * n,
            "temperature": [round(m[5], 2) for m in metas], "timestamp": [stamp] * n}))

    def _log_episode(self, episode, m, counts, valid, temp, ov, env_id=None):
        if self.warmup:
            return
        self.metrics.log(episode, m)
        self.metrics.recent_solve_rates.append(m["solve_rate"])
        entry = GameLogEntry(episode=episode, phase=m["phase"], budget=m["budget"], walls=int(counts[0]),
                             cameras=int(counts[1]), guards=int(counts[2]), solve_rate=m["solve_rate"],
                             detection_rate=m["detection_rate"], timeout_rate=m["timeout_rate"],
                             architect_reward=m["architect_reward"], solver_reward=m["solver_reward"],
                             avg_steps=m["avg_steps"], level_valid=valid,
                             is_interactive=bool(ov.get("interactive", False)),
                             freeze_architect=bool(ov.get("freeze_architect", False)),
                             freeze_solver=bool(ov.get("freeze_solver", False)), temperature=temp)
        self.game_log.append(entry)
        if self._callback is not None:  # training.py:383-384: (episode, ep_metrics, env_state)
            self.current_state = self.environment_state(env_id) if env_id is not None else None
            self._callback(episode, m, self.current_state)

    def _architect_step(self, defer: bool = False, join=None):
        """The Architect's update on the transitions scored this iteration; defer=True returns
        a callable giving its metrics (ArchitectAgent.update_sequence(defer=True, join))."""
        if self.architect_update == "batched":
            m = self.architect.update()
            if defer and join is not None:
                join.wait_stream(torch.cuda.current_stream(self.device))
            return (lambda: m) if defer else m
        # per_layout: the reference's cadence, one single-reward update per layout in episode
        # order (agents/architect.py:91-155 with len(rewards) == 1); every rank replays the
        # union of all ranks' layouts, so no gradient crosses the wire and replicas stay equal
        A = self.architect
        k = min(len(A.rewards), len(A.log_probs), len(A.values))
        rows = torch.zeros((k, 4), dtype=torch.float64, device=self.device)
        if k:
            for j, buf in ((0, A.log_probs), (1, A.values)):
                col = buf.stacked(k) if hasattr(buf, "stacked") else torch.stack([x.squeeze() for x in buf[:k]])
                rows[:, j] = col.double().reshape(-1)
            # host columns through pinned memory: a pageable host->device copy would block
            # until the device is idle, i.e. behind the Solver's update running beside this
            host = torch.tensor(np.stack([np.asarray(A.rewards[:k], np.float64),
                                          np.asarray(self._arch_eps[:k], np.float64)], 1))
            if self.device.type == "cuda":
                host = host.pin_memory()
            rows[:, 2:] = host.to(self.device, non_blocking=True)
        allrows, _ = dist_utils.allgather_rows(rows, self.device)
        A._clear()
        allrows = allrows[torch.argsort(allrows[:, 3], stable=True)]
        # one update per layout, in one persistent kernel launch (ArchitectAgent.update_sequence)
        return A.update_sequence(allrows[:, 0], allrows[:, 1], allrows[:, 2], defer=defer, join=join)

    def train_iteration(self, overrides: Optional[dict] = None, reassign: bool = True) -> Dict[str, float]:
        """One rollout of rollout_len ticks over all envs + the agents' updates.
        Collective inside a process group (every rank calls it with the same overrides)."""
        ov = overrides or {}
        out = {}
        if self.solver_cadence == "layout_batch":
            ro, sel = self._rollout_layout_batch()
            if self._trace is not None:  # kept for parity tests
                self._last_layout_batch = (ro, sel)
            out["rollout_ticks"] = int(ro.rewards.shape[0])
        else:
            ro = self._rollout(self.rollout_len)
        # Scoring reads the rollout only and the two agents' updates share no tensor, so the
        # Architect's per-layout sequence (one persistent kernel on its side stream) goes out
        # first, while the GPU is idle, and the Solver's PPO update then runs beside it on the
        # remaining CUs (the kernel holds 64 whole CUs; launched behind the Solver's queued
        # kernels it would wait for them to drain).  The next layouts are drawn only after
        # both (the joins below).
        done_ids, score_log = self._score_commit(self._score_prepare(), ov, defer_log=True)
        main = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        side = self.architect.side_stream()
        pending = None
        if not self.warmup and not ov.get("freeze_architect", False):
            if side is None:
                pending = self._architect_step(defer=True)
            else:
                side.wait_stream(main)
                # the buffered transitions (views of tensors made on the main stream) are read
                # on the side stream: keep their memory from being reused before that
                for buf in (self.architect.log_probs, self.architect.values):
                    ts = buf.tensors() if hasattr(buf, "tensors") else [x for x in buf if torch.is_tensor(x)]
                    for t_ in ts:
                        if t_.is_cuda:
                            t_.record_stream(side)
                with torch.cuda.stream(side):
                    pending = self._architect_step(defer=True, join=main)
        solver_done = None
        if not ov.get("freeze_solver", False):
            if self.solver_cadence == "layout_batch":
                solver_done = self.solver.update_layout_batch(ro, sel, minibatch=self.minibatch, defer=True)
            else:
                solver_done = self.solver.update_rollout(ro, minibatch=self.minibatch, defer=True)
        score_log()  # host bookkeeping while both updates run on the device
        if solver_done is not None:
            out.update(solver_done())
        if pending is not None:
            out.update(pending())
            self._arch_eps = []
        if reassign:
            self._assign_layouts(done_ids, ov, empty=self.warmup)
        out["layouts_scored"] = len(done_ids)
        return out

    # -- public API (training.py:336-416, :606-663) -------------------------------------------
    def _run_warmup(self, rollouts: int = 2):
        """Warmup on empty layouts (training.py:277-330)."""
        self.warmup = True
        saved = self.global_episode
        self._assign_layouts(np.arange(self.n_envs), empty=True)
        for _ in range(rollouts):
            self.train_iteration()
        self.global_episode = saved
        self.warmup = False

    def train(self, callback=None, resume: bool = False, warmup_rollouts: int = 2):
        """training.py:336-416.  callback(episode, ep_metrics, env_state) runs for every
        scored or invalid layout, as the reference's does per episode."""
        self.training_active = True
        start_episode = self.resume_from_checkpoint() if resume else 0
        self.global_episode = start_episode
        if start_episode == 0:
            self._run_warmup(warmup_rollouts)
        self._init_batch_state()
        self._callback = callback
        try:
            self._assign_layouts(np.arange(self.n_envs))
            t0 = time.time()
            next_ckpt = start_episode + 50
            while self.global_episode < start_episode + self.total_episodes:  # a global count: same on every rank
                self.train_iteration()
                if self.global_episode >= next_ckpt:  # every 50 episodes at most (training.py:397-399)
                    self._save_checkpoint(self.global_episode)
                    next_ckpt = (self.global_episode // 50 + 1) * 50
            self._save_checkpoint(self.global_episode)
        finally:
            self._callback = None
            self.training_active = False
        return time.time() - t0

    def run_interactive_episodes(self, num_episodes: int = 1, budget: int = 15, freeze_architect: bool = False,
                                 freeze_solver: bool = False, temperature: float = 1.0, solver_attempts: int = 20,
                                 allow_cameras: bool = True, allow_guards: bool = True, callback=None) -> List[Dict]:
        """training.py:606-663: num_episodes layouts under the given overrides (spread over
        ranks), played while every other env sits out (masked: not trained, not scored);
        afterwards the interactive envs get fresh curriculum layouts and the others resume.
        Returns the episodes' ep_metrics dicts, in episode order."""
        ov = dict(budget=budget, freeze_architect=freeze_architect, freeze_solver=freeze_solver,
                  temperature=temperature, allow_cameras=allow_cameras, allow_guards=allow_guards, interactive=True,
                  phase="Interactive (budget=%d)" % budget)
        w, rk = dist_utils.world_size(), dist_utils.rank()
        saved_a = self.solver_episodes
        saved_valid = self.b_valid.clone()
        self.solver_episodes = solver_attempts
        # blocks of at most n_envs layouts per rank, so that any num_episodes is played
        first = min(num_episodes, self.n_envs * w)
        ids = np.arange(first // w + (1 if rk < first % w else 0))
        others = torch.ones(self.n_envs, dtype=torch.bool, device=self.device)
        others[torch.as_tensor(ids, device=self.device)] = False
        n0 = len(self.game_log)
        self._callback = callback
        try:
            done_eps = 0
            while done_eps < num_episodes:
                block = min(num_episodes - done_eps, self.n_envs * w)
                bids = np.arange(block // w + (1 if rk < block % w else 0))
                self.b_valid &= ~others
                self._assign_layouts(bids, ov)
                for _ in range(1000):
                    cnt = dist_utils.allreduce_(torch.tensor([len(self.game_log) - n0], device=self.device))
                    if int(cnt.item()) >= done_eps + block:
                        break
                    self.train_iteration(ov, reassign=False)
                    self.b_valid &= ~self.b_scored  # a scored interactive layout sits out until its block ends
                done_eps = int(dist_utils.allreduce_(torch.tensor([len(self.game_log) - n0],
                                                                  device=self.device)).item())
        finally:
            self._callback = None
            self.solver_episodes = saved_a
        mine_log = [e.to_dict() for e in self.game_log[n0:]]
        allm = self._gather_objects(mine_log)
        self.b_valid = saved_valid & others
        self._assign_layouts(ids)
        results = sorted(allm, key=lambda r: r["episode"])[:num_episodes]
        keys = ("solve_rate", "detection_rate", "timeout_rate", "architect_reward", "solver_reward", "avg_steps",
                "budget", "phase")
        self._save_checkpoint(self.global_episode)
        return [{k: r[k] for k in keys} for r in results]

    def environment_state(self, env_id: int) -> Dict:
        """get_environment_state (environment.py:388-417) of batched env env_id: grid,
        visibility, solver, cameras and guards from the device; solver_path and
        detection_events are not tracked by the batched env (single-point path, none)."""
        cfg = self.config
        st = self.env.export(grid=True)
        e = int(env_id)
        lay = self.b_layout[e]
        walls, cams, guards = ([], [], []) if lay is None else _lb_rows(lay[0], [lay[1]]).to_lists()[0]
        budget = self.b_meta[e][1] if self.b_meta[e] else cfg.architect_budget
        _, cameras, gds, _ = accept_layout(walls, cams, guards, cfg, budget)
        ch = st["cam_heading"][e].cpu().numpy()
        gi = st["guard_idx"][e].cpu().numpy()
        gh = st["guard_heading"][e].cpu().numpy()
        for k, cam in enumerate(cameras):
            cam.heading = float(ch[k])
        for k, g in enumerate(gds):
            g.current_idx, g.heading = int(gi[k]), float(gh[k])
        pos = (int(st["pos_r"][e]), int(st["pos_c"][e]))
        return {"grid": st["grid"][e].cpu().numpy().astype(np.int32).tolist(),
                "visibility": self.env.obs[e, 1].cpu().numpy().tolist(), "solver_pos": pos, "solver_path": [pos],
                "vault_pos": cfg.vault_pos, "start_pos": cfg.start_pos, "tick": int(st["tick"][e]),
                "done": bool(st["done"][e]),
                "cameras": [{"row": c.row, "col": c.col, "heading": c.heading, "fov_angle": c.fov_angle,
                             "vision_range": c.vision_range} for c in cameras],
                "guards": [{"row": g.row, "col": g.col, "heading": g.heading, "patrol_path": g.patrol_path,
                            "current_idx": g.current_idx} for g in gds],
                "detection_events": []}

    def layout_lists(self, env_ids) -> List:
        """The (walls, cameras, guards) lists last assigned to env_ids, in the reference's
        set_layout format (for replay through the CPU oracle and for frames)."""
        out = []
        for e in env_ids:
            lay = self.b_layout[int(e)]
            out.append(([], [], []) if lay is None else _lb_rows(lay[0], [lay[1]]).to_lists()[0])
        return out

    def simulate_episode(self, budget: int = 15, solver_attempts: int = 1) -> Dict:  # training.py:713-790
        if self._single_env is None:
            self._single_env = HeistEnvironment(self.config, device=self.device)
        env = self._single_env
        saved = self.architect.budget
        self.architect.budget = budget
        walls, cameras, guards = self.architect.generate_layout(temperature=0.5)
        self.architect.log_probs.clear()
        self.architect.values.clear()
        env.budget.scale_budget(budget)
        env.set_layout(walls, cameras, guards)
        self.architect.budget = saved
        best_outcome, best_frames, max_reward = "timeout", [], -float("inf")
        for i in range(solver_attempts):
            env.reset()
            self.solver.reset()
            frames, ep_reward, outcome = [], 0.0, "timeout"
            state = env.get_state_tensor()
            for _ in range(self.config.max_steps):
                frames.append(env.get_environment_state())
                action = self.solver.select_action(state)
                _, reward, done, info = env.step(action)
                state = env.get_state_tensor()
                ep_reward += reward
                if done:
                    frames.append(env.get_environment_state())
                    outcome = info.get("status", "timeout")
                    break
            self.solver._clear_buffers()
            better = i == 0
            if not better:
                if outcome == "vault_reached":
                    better = best_outcome != "vault_reached" or ep_reward > max_reward
                elif outcome == "detected":
                    better = best_outcome == "timeout" or (best_outcome == "detected" and ep_reward > max_reward)
                else:
                    better = best_outcome == "timeout" and ep_reward > max_reward
            if better:
                best_outcome, max_reward, best_frames = outcome, ep_reward, frames
        return {"frames": best_frames, "outcome": best_outcome, "total_steps": len(best_frames) - 1,
                "reward": max_reward}

    # -- checkpoints and logs (training.py:192-259, :673-711) -------------------------------------
    def find_latest_checkpoint(self) -> Optional[int]:
        eps = [int(m.group(1)) for f in glob.glob(os.path.join(self.save_dir, "architect_ep*.pt"))
               for m in [re.search(r"architect_ep(\d+)\.pt", f)] if m]
        return max(eps) if eps else None

    def list_checkpoints(self) -> List[int]:
        return sorted(int(m.group(1)) for f in glob.glob(os.path.join(self.save_dir, "solver_ep*.pt"))
                      for m in [re.search(r"solver_ep(\d+).pt", f)] if m)

    def load_checkpoint(self, episode: int) -> bool:
        arch = os.path.join(self.save_dir, "architect_ep%d.pt" % episode)
        sol = os.path.join(self.save_dir, "solver_ep%d.pt" % episode)
        if not (os.path.exists(arch) and os.path.exists(sol)):
            return False
        self.architect.load(arch)
        self.solver.load(sol)
        if dist_utils.rank() == 0:  # the files hold every rank's episodes; one copy is enough
            mp = os.path.join(self.log_dir, "training_metrics.json")
            if os.path.exists(mp):
                self.metrics.load(mp)
            lp = os.path.join(self.log_dir, "game_log.json")
            if os.path.exists(lp):
                with open(lp) as f:
                    self.game_log = [GameLogEntry(**e) for e in json.load(f)]
        self.global_episode = episode
        return True

    def resume_from_checkpoint(self) -> int:
        ep = self.find_latest_checkpoint()
        if not ep:
            return 0
        return ep if self.load_checkpoint(ep) else 0

    def get_game_log(self) -> List[Dict]:
        return [e.to_dict() for e in self.game_log]

    def _gather_objects(self, items: List) -> List:
        """Concatenate every rank's list (all_gather_object); the local list on one rank."""
        if not dist_utils.is_multi():
            return list(items)
        out = [None] * dist_utils.world_size()
        torch.distributed.all_gather_object(out, list(items))
        return [x for part in out for x in part]

    def _save_game_log(self):
        entries = sorted(self._gather_objects(self.get_game_log()), key=lambda e: e["episode"])
        if dist_utils.rank() == 0:
            with open(os.path.join(self.log_dir, "game_log.json"), "w") as f:
                json.dump(entries, f, indent=2)

    def _save_metrics(self):
        if dist_utils.is_multi():
            m = TrainingMetrics.from_records(self._gather_objects(self.metrics.records()))
        else:
            m = self.metrics
        if dist_utils.rank() == 0:
            m.save(os.path.join(self.log_dir, "training_metrics.json"))

    def _save_checkpoint(self, episode: int):
        """training.py:700-711 + the JSON logs.  Collective: the logs of all ranks are
        merged by episode and rank 0 writes them (the replicas' weights are equal)."""
        if dist_utils.rank() == 0:
            self.architect.save(os.path.join(self.save_dir, "architect_ep%d.pt" % episode))
            self.solver.save(os.path.join(self.save_dir, "solver_ep%d.pt" % episode))
        self._save_metrics()
        self._save_game_log()


def _rows(eps, cols):
    rows = [{"episode": e} for e in eps]
    for k, v in cols.items():
        off = len(eps) - len(v)
        for i, x in enumerate(v):
            rows[off + i][k] = x
    return rows


def _mask(ids, env) -> torch.Tensor:
    m = torch.zeros(env.n_envs, dtype=torch.uint8, device=env.device)
    m[torch.as_tensor(np.asarray(ids, np.int64), device=env.device)] = 1
    return m


_LB_KEYS = ("wall_rc", "n_walls", "cam_params", "n_cams", "guard_paths", "guard_meta", "guard_fov", "n_guards",
            "budget")


def _lb_rows(lb, ids):
    """Rows `ids` of a LayoutBatch."""
    from .vec_env import LayoutBatch
    idx = torch.as_tensor(np.asarray(ids, np.int64), device=lb.n_walls.device)
    return LayoutBatch(**{k: getattr(lb, k)[idx] for k in _LB_KEYS})


def _scatter_layout(lb, ids, env):
    """Place a LayoutBatch of len(ids) layouts at rows `ids` of an env-sized batch."""
    from .vec_env import LayoutBatch
    n = env.n_envs
    idx = torch.as_tensor(np.asarray(ids, np.int64), device=env.device)
    out = {}
    for k in _LB_KEYS:
        src = getattr(lb, k)
        full = torch.zeros((n,) + tuple(src.shape[1:]), dtype=src.dtype, device=env.device)
        full[idx] = src
        out[k] = full.contiguous()
    return LayoutBatch(**out)
