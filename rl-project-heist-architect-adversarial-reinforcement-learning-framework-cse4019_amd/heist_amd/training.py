"""Adversarial training loop (reference: heist_architect/training.py), batched.

The reference plays one layout at a time: Architect samples a layout, the Solver makes
`solver_episodes_per_layout` sequential attempts on it (camera headings carry over),
then both agents update (training.py:418-600).  Here N environments run at once on one
GPU (and N per rank across GPUs):

  * every env holds its own Architect layout and counts its attempts; after an env's
    A-th attempt its layout is scored (solve/detect/timeout rates -> RewardCalculator)
    and replaced by a fresh Architect sample (masked heist_set_layout + heist_reset);
  * the Solver steps all envs for `rollout_len` ticks (batched policy forward on
    PyTorch-ROCm, heist_step with in-kernel auto-reset, per-env LSTM state zeroed when
    an attempt ends), then does one PPO update on the [T, N] rollout (heist_gae,
    global advantage normalisation, heist_ppo_loss; one flat gradient all-reduce per
    optimizer step across ranks);
  * the Architect updates once per rollout on the layouts scored during it.
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
from typing import Dict, List, Optional

import numpy as np
import torch

from .agents.architect import ArchitectAgent
from .agents.solver import Rollout, SolverAgent
from .environment import EnvironmentConfig, HeistEnvironment
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

    def get_summary(self, last_n: int = 10) -> str:
        lines = []
        for key in ("solve_rate", "detection_rate", "architect_reward", "solver_reward"):
            vals = self.history.get(key, [])
            if vals:
                lines.append("  %s: %.3f" % (key, float(np.mean(vals[-last_n:]))))
        return "\n".join(lines)


class AdversarialTrainer:  # training.py:115-790
    CURRICULUM = [  # (episode_threshold, budget, allow_cameras, allow_guards, description)
        (0, 5, False, False, "Walls Only"),
        (80, 8, True, False, "Walls + Cameras"),
        (200, 15, True, True, "Full Security"),
        (400, 22, True, True, "Expert"),
    ]
    WARMUP_EPISODES = 30

    def __init__(self, config: Optional[EnvironmentConfig] = None, solver_episodes_per_layout: int = 20,
                 total_episodes: int = 500, save_dir: str = "checkpoints", log_dir: str = "logs",
                 architect_lr: float = 3e-4, solver_lr: float = 1e-3, n_envs: int = 256,
                 rollout_len: Optional[int] = None, minibatch: int = 4096, device=None, max_budget: Optional[int] = None,
                 seed: Optional[int] = None, update_precision: str = "fp32"):
        self.config = config or EnvironmentConfig()
        self.solver_episodes = solver_episodes_per_layout
        self.total_episodes = total_episodes
        self.save_dir = save_dir
        self.log_dir = log_dir
        self.device = torch.device(device) if device is not None else DEVICE
        self.n_envs = n_envs
        self.rollout_len = rollout_len or self.config.max_steps
        self.minibatch = minibatch
        if seed is not None:
            torch.manual_seed(seed)
            np.random.seed(seed)
        mb = max_budget or max(b for _, b, _, _, _ in self.CURRICULUM)
        mb = max(mb, self.config.architect_budget)
        self.env = HeistEnv(n_envs, self.config, max_cams=max(1, mb // 3), max_guards=max(1, mb // 5), max_path=8,
                            device=self.device, auto_reset=True)
        R, C = self.config.grid_rows, self.config.grid_cols
        self.architect = ArchitectAgent(grid_rows=R, grid_cols=C, budget=self.config.architect_budget,
                                        lr=architect_lr, device=self.device)
        self.solver = SolverAgent(grid_rows=R, grid_cols=C, lr=solver_lr, device=self.device,
                                  update_precision=update_precision)
        self.reward_calc = RewardCalculator()
        self.metrics = TrainingMetrics()
        self.game_log: List[GameLogEntry] = []
        self.global_episode = 0
        self.current_state = None
        self.training_active = False
        self._single_env = None
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
        self.b_episode = np.zeros(n, np.int64)
        self.b_meta = [None] * n  # (phase, budget, walls, cameras, guards, temperature)
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

    def _assign_layouts(self, env_ids: np.ndarray, overrides: Optional[dict] = None, empty: bool = False):
        """New Architect layouts for env_ids (one episode number each); invalid layouts are
        scored -1 and resampled, as the reference skips their solver phase."""
        ov = overrides or {}
        pending = np.asarray(env_ids, np.int64)
        tries = 0
        while len(pending):
            ep0 = self.global_episode + 1
            eps = np.arange(ep0, ep0 + len(pending))
            self.global_episode += len(pending)
            _, budget, cams, guards, desc = self.get_curriculum_phase(int(eps[0]))
            budget = ov.get("budget", budget)
            cams = ov.get("allow_cameras", cams)
            guards = ov.get("allow_guards", guards)
            temp = ov.get("temperature", self._temperature(int(eps[0])))
            phase = ov.get("phase", desc)
            if empty:
                layouts = [([], [], [])] * len(pending)
                valid = self.env.set_layouts(layouts, budget=budget, env_ids=pending)[torch.as_tensor(pending)]
                counts = np.zeros((len(pending), 3), np.int64)
            else:
                self.architect.budget = budget
                lb, _, _ = self.architect.generate_layouts(len(pending), temp, cams, guards, env=self.env,
                                                           record=not ov.get("freeze_architect", False))
                lb = _scatter_layout(lb, pending, self.env)
                valid = self.env.set_layout_batch(lb, _mask(pending, self.env))[torch.as_tensor(pending)]
                counts = torch.stack([lb.n_walls, lb.n_cams, lb.n_guards], 1)[torch.as_tensor(pending)].cpu().numpy()
            v = valid.cpu().numpy()
            for i, e in enumerate(pending):
                self.b_episode[e] = eps[i]
                self.b_meta[e] = (phase, budget, int(counts[i, 0]), int(counts[i, 1]), int(counts[i, 2]), temp)
            bad = pending[~v]
            for i in np.nonzero(~v)[0]:  # training.py:476-504
                r = self.reward_calc.architect_invalid
                if not empty and not ov.get("freeze_architect", False):
                    self.architect.store_reward(r)
                self._log_episode(int(eps[i]), phase, budget, counts[i], 0.0, 0.0, 1.0, r, 0.0, 0.0, False, temp, ov)
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
            tries += 1
            pending = bad if tries < 8 else np.zeros(0, np.int64)
            if len(bad) and tries >= 8:
                self.b_valid[torch.as_tensor(bad, device=self.device)] = False

    # -- rollout / scoring ------------------------------------------------------------------
    @torch.no_grad()
    def _rollout(self, T: int) -> Rollout:
        env, n, d = self.env, self.n_envs, self.device
        obs_buf = torch.empty((T, n) + tuple(env.obs.shape[1:]), dtype=torch.float32, device=d)
        act_buf = torch.empty((T, n), dtype=torch.int64, device=d)
        lp_buf = torch.empty((T, n), dtype=torch.float32, device=d)
        v_buf = torch.empty((T, n), dtype=torch.float32, device=d)
        r_buf = torch.empty((T, n), dtype=torch.float32, device=d)
        d_buf = torch.empty((T, n), dtype=torch.uint8, device=d)
        A = self.solver_episodes
        vault, det, tmo = STATUS_CODES["vault_reached"], STATUS_CODES["detected"], STATUS_CODES["timeout"]
        for t in range(T):
            obs_buf[t].copy_(env.obs)
            a, lp, v, (self.h, self.c) = self.solver.act(env.obs, (self.h, self.c))
            act_buf[t], lp_buf[t], v_buf[t] = a, lp, v
            _, rew, done, status = env.step(a)
            r_buf[t] = rew
            d_buf[t] = done.to(torch.uint8)
            counting = self.b_valid & (self.b_attempts < A)
            self.b_steps += counting.int()
            self.b_reward += torch.where(counting, rew.double(), torch.zeros_like(self.b_reward))
            fin = counting & done
            st = status.to(torch.int32)
            self.b_solve += (fin & (st == vault)).int()
            self.b_detect += (fin & (st == det)).int()
            self.b_timeout += (fin & (st != vault) & (st != det)).int()
            self.b_attempts += fin.int()
            keep = (~done).to(self.h.dtype).reshape(1, n, 1)  # a new attempt starts with a fresh LSTM state
            self.h = self.h * keep
            self.c = self.c * keep
        return Rollout(obs_buf, act_buf, lp_buf, v_buf, r_buf, d_buf, mask=self.b_valid.clone())

    def _score_finished(self, overrides: Optional[dict] = None) -> np.ndarray:
        """Score every env whose layout has had its A attempts; returns those env ids."""
        A = self.solver_episodes
        fin = (self.b_valid & (self.b_attempts >= A) & ~self.b_scored).nonzero().reshape(-1)
        if fin.numel() == 0:
            return np.zeros(0, np.int64)
        stats = torch.stack([self.b_solve[fin], self.b_detect[fin], self.b_timeout[fin], self.b_steps[fin]], 1)
        stats = stats.cpu().numpy().astype(np.float64)
        rews = self.b_reward[fin].cpu().numpy()
        ov = overrides or {}
        ids = fin.cpu().numpy()
        for i, e in enumerate(ids):
            s, dt, to, steps = stats[i]
            solve_rate, det_rate, to_rate = s / A, dt / A, to / A
            ar = self.reward_calc.architect_reward_from_rate(True, solve_rate)  # rewards.py:43-73
            if not ov.get("freeze_architect", False) and not self.warmup:
                self.architect.store_reward(ar)
            phase, budget, nw, nc, ng, temp = self.b_meta[e]
            self._log_episode(int(self.b_episode[e]), phase, budget, (nw, nc, ng), solve_rate, det_rate, to_rate, ar,
                              rews[i] / A, steps / A, True, temp, ov)
        self.b_scored[fin] = True
        return ids

    def _log_episode(self, episode, phase, budget, counts, solve, detect, timeout, arch_r, solver_r, avg_steps,
                     valid, temp, ov):
        if self.warmup:
            return
        m = {"solve_rate": solve, "detection_rate": detect, "timeout_rate": timeout, "architect_reward": arch_r,
             "solver_reward": solver_r, "architect_loss": 0, "solver_loss": 0, "avg_steps": avg_steps,
             "budget": budget, "phase": phase}
        self.metrics.log(episode, m)
        self.metrics.recent_solve_rates.append(solve)
        self.game_log.append(GameLogEntry(episode=episode, phase=phase, budget=budget, walls=int(counts[0]),
                                          cameras=int(counts[1]), guards=int(counts[2]), solve_rate=solve,
                                          detection_rate=detect, timeout_rate=timeout, architect_reward=arch_r,
                                          solver_reward=solver_r, avg_steps=avg_steps, level_valid=valid,
                                          is_interactive=bool(ov.get("interactive", False)),
                                          freeze_architect=bool(ov.get("freeze_architect", False)),
                                          freeze_solver=bool(ov.get("freeze_solver", False)), temperature=temp))

    def train_iteration(self, overrides: Optional[dict] = None) -> Dict[str, float]:
        """One rollout of rollout_len ticks over all envs + the agents' updates."""
        ov = overrides or {}
        ro = self._rollout(self.rollout_len)
        out = {}
        if not ov.get("freeze_solver", False):
            out.update(self.solver.update_rollout(ro, minibatch=self.minibatch))
        done_ids = self._score_finished(ov)
        if len(done_ids) and not self.warmup and not ov.get("freeze_architect", False) and self.architect.rewards:
            out.update(self.architect.update())
        if len(done_ids):
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
        self.training_active = True
        start_episode = self.resume_from_checkpoint() if resume else 0
        self.global_episode = start_episode
        if start_episode == 0:
            self._run_warmup(warmup_rollouts)
        self._init_batch_state()
        self._assign_layouts(np.arange(self.n_envs))
        t0 = time.time()
        next_ckpt = start_episode + 50
        while self.global_episode < start_episode + self.total_episodes:
            m = self.train_iteration()
            if callback:
                callback(self.global_episode, m, None)
            if self.global_episode >= next_ckpt:
                self._save_checkpoint(self.global_episode)
                next_ckpt += 50
        self._save_checkpoint(self.global_episode)
        self._save_game_log()
        self.metrics.save(os.path.join(self.log_dir, "training_metrics.json"))
        self.training_active = False
        return time.time() - t0

    def run_interactive_episodes(self, num_episodes: int = 1, budget: int = 15, freeze_architect: bool = False,
                                 freeze_solver: bool = False, temperature: float = 1.0, solver_attempts: int = 20,
                                 allow_cameras: bool = True, allow_guards: bool = True, callback=None) -> List[Dict]:
        ov = dict(budget=budget, freeze_architect=freeze_architect, freeze_solver=freeze_solver,
                  temperature=temperature, allow_cameras=allow_cameras, allow_guards=allow_guards, interactive=True,
                  phase="Interactive (budget=%d)" % budget)
        saved_a = self.solver_episodes
        self.solver_episodes = solver_attempts
        n0 = len(self.game_log)
        self._assign_layouts(np.arange(min(num_episodes, self.n_envs)), ov)
        while len(self.game_log) - n0 < num_episodes:
            self.train_iteration(ov)
        self.solver_episodes = saved_a
        results = [e.to_dict() for e in self.game_log[n0:n0 + num_episodes]]
        if callback:
            for r in results:
                callback(r["episode"], r, None)
        self._save_checkpoint(self.global_episode)
        self._save_game_log()
        self.metrics.save(os.path.join(self.log_dir, "training_metrics.json"))
        return results

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

    def _save_game_log(self):
        with open(os.path.join(self.log_dir, "game_log.json"), "w") as f:
            json.dump([e.to_dict() for e in self.game_log], f, indent=2)

    def _save_checkpoint(self, episode: int):
        dist = torch.distributed
        if dist.is_available() and dist.is_initialized() and dist.get_rank() != 0:
            return
        self.architect.save(os.path.join(self.save_dir, "architect_ep%d.pt" % episode))
        self.solver.save(os.path.join(self.save_dir, "solver_ep%d.pt" % episode))
        self.metrics.save(os.path.join(self.log_dir, "training_metrics.json"))
        self._save_game_log()


def _mask(ids, env) -> torch.Tensor:
    m = torch.zeros(env.n_envs, dtype=torch.uint8, device=env.device)
    m[torch.as_tensor(np.asarray(ids, np.int64), device=env.device)] = 1
    return m


def _scatter_layout(lb, ids, env):
    """Place a LayoutBatch of len(ids) layouts at rows `ids` of an env-sized batch."""
    from .vec_env import LayoutBatch
    n = env.n_envs
    idx = torch.as_tensor(np.asarray(ids, np.int64), device=env.device)
    out = {}
    for k in ("wall_rc", "n_walls", "cam_params", "n_cams", "guard_paths", "guard_meta", "guard_fov", "n_guards",
              "budget"):
        src = getattr(lb, k)
        full = torch.zeros((n,) + tuple(src.shape[1:]), dtype=src.dtype, device=env.device)
        full[idx] = src
        out[k] = full.contiguous()
    return LayoutBatch(**out)
