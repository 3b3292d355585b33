"""Solver agent: PPO with GAE on the HIP kernels (reference: agents/solver.py).

The reference API (select_action / store_transition / end_episode / update /
_compute_gae / save / load) is kept for single-env use.  Batched training uses
act() on [N,3,R,C] observations and update_rollout() on [T,N] rollouts; both paths
compute GAE (heist_gae), advantage normalisation (heist_adv_*) and the clipped loss
and its gradient (heist_ppo_loss) on the GPU.  With torch.distributed initialised the
gradients of every optimizer step are averaged with ONE flat all-reduce.
"""
from collections import deque
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..networks import SolverNetwork
from .. import dist_utils
from ..dist_utils import allreduce_grads  # noqa: F401  (re-exported: the reference-facing name)
from ..ppo import compute_gae, normalize_advantages, ppo_loss
from ..utils import DEVICE


@dataclass
class Rollout:
    """[T, N] time-major rollout of the batched environment."""
    obs: torch.Tensor       # [T, N, 3, R, C] float32
    actions: torch.Tensor   # [T, N] int64
    logp: torch.Tensor      # [T, N] float32
    values: torch.Tensor    # [T, N] float32
    rewards: torch.Tensor   # [T, N] float32
    dones: torch.Tensor     # [T, N] uint8
    mask: Optional[torch.Tensor] = None        # [N] bool: envs whose samples train (valid layouts)
    last_value: Optional[torch.Tensor] = None  # [N] bootstrap (None: the reference's buffer-end 0)


class SolverAgent:  # agents/solver.py:18-259
    """rollout_precision selects the batched act() path:
      * "fp32" (default): the reference's fp32 forward (networks.py:76-131) on PyTorch-ROCm,
        so rollout log-probs and values are the reference's to fp32 rounding and the PPO
        ratio at epoch 0 is exactly 1 (the parity mode);
      * "bf16": the fused HIP kernels (heist_solver_features + heist_solver_head, bf16
        MFMA operands, fp32 accumulation), ~15x faster; log-probs differ from fp32 by ~1e-3
        (opt-in, labelled as such by bench.py).
    ``fused_inference=True`` is the round-1 spelling of rollout_precision="bf16"."""

    def __init__(self, grid_rows: int = 20, grid_cols: int = 20, num_actions: int = 5, lr: float = 3e-4,
                 gamma: float = 0.99, gae_lambda: float = 0.95, clip_epsilon: float = 0.2,
                 entropy_coeff: float = 0.05, value_coeff: float = 0.5, max_grad_norm: float = 0.5,
                 ppo_epochs: int = 3, batch_size: int = 64, device=None, fused_inference: Optional[bool] = None,
                 update_precision: str = "fp32", rollout_precision: Optional[str] = None):
        self.grid_rows = grid_rows
        self.grid_cols = grid_cols
        self.num_actions = num_actions
        self.gamma = gamma
        self.gae_lambda = gae_lambda
        self.clip_epsilon = clip_epsilon
        self.entropy_coeff = entropy_coeff
        self.value_coeff = value_coeff
        self.max_grad_norm = max_grad_norm
        self.ppo_epochs = ppo_epochs
        self.batch_size = batch_size
        if rollout_precision is None:
            rollout_precision = "bf16" if fused_inference else "fp32"
        if rollout_precision not in ("fp32", "bf16"):
            raise ValueError("rollout_precision must be 'fp32' or 'bf16'")
        self.rollout_precision = rollout_precision
        self._act_seed = int(torch.initial_seed()) ^ 0x5EED
        self._act_counter = 0
        self.device = torch.device(device) if device is not None else DEVICE
        self.network = SolverNetwork(grid_rows=grid_rows, grid_cols=grid_cols, num_actions=num_actions).to(self.device)
        if self.device.type == "cuda":  # NHWC convolutions: MIOpen's faster layout (same values, same state_dict)
            self.network = self.network.to(memory_format=torch.channels_last)
        if update_precision not in ("fp32", "bf16"):
            raise ValueError("update_precision must be 'fp32' or 'bf16'")
        # "fp32": the reference's arithmetic; "bf16": autocast forward/backward in the PPO update
        self.update_precision = update_precision
        self.optimizer = torch.optim.Adam(self.network.parameters(), lr=lr)
        self.hidden = None
        self.states, self.actions, self.log_probs, self.values, self.rewards, self.dones = [], [], [], [], [], []
        self.episode_count = 0
        self.total_reward = 0.0
        self.recent_rewards = deque(maxlen=100)

    @property
    def fused_inference(self) -> bool:
        return self.rollout_precision == "bf16"

    @fused_inference.setter
    def fused_inference(self, v: bool):
        self.rollout_precision = "bf16" if v else "fp32"

    # -- single-env API ------------------------------------------------------------
    def reset(self):
        self.hidden = None

    def select_action(self, state: np.ndarray) -> int:  # agents/solver.py:75-99
        self.network.eval()
        st = torch.as_tensor(np.asarray(state, np.float32)).unsqueeze(0).to(self.device)
        with torch.no_grad():
            action, log_prob, value, self.hidden = self.network.get_action(st, self.hidden)
        self.states.append(state)
        self.actions.append(int(action.item()))
        self.log_probs.append(float(log_prob.item()))
        self.values.append(float(value.item()))
        return int(action.item())

    def store_transition(self, reward: float, done: bool):
        self.rewards.append(reward)
        self.dones.append(done)

    def end_episode(self, final_reward: float):
        self.total_reward += final_reward
        self.recent_rewards.append(final_reward)
        self.episode_count += 1

    def _compute_gae(self, rewards: torch.Tensor, values: torch.Tensor, dones: torch.Tensor) -> torch.Tensor:
        """agents/solver.py:228-244 on one flat buffer (bootstrap 0 at the end)."""
        adv, _ = compute_gae(rewards, values, dones, gamma=self.gamma, lam=self.gae_lambda)
        return adv

    def _clear_buffers(self):
        for b in (self.states, self.actions, self.log_probs, self.values, self.rewards, self.dones):
            b.clear()

    def update(self) -> Dict[str, float]:  # agents/solver.py:112-217
        if len(self.states) == 0:
            return {"solver_loss": 0.0}
        n = min(len(self.states), len(self.actions), len(self.log_probs), len(self.values), len(self.rewards),
                len(self.dones))
        if n == 0:
            self._clear_buffers()
            return {"solver_loss": 0.0}
        d = self.device
        states = torch.as_tensor(np.array(self.states[:n], np.float32)).to(d)
        actions = torch.as_tensor(self.actions[:n], dtype=torch.int64).to(d)
        old_logp = torch.as_tensor(self.log_probs[:n], dtype=torch.float32).to(d)
        values = torch.as_tensor(self.values[:n], dtype=torch.float32).to(d)
        rewards = torch.as_tensor(self.rewards[:n], dtype=torch.float32).to(d)
        dones = torch.as_tensor(self.dones[:n], dtype=torch.float32).to(d)
        adv, ret = compute_gae(rewards, values, dones, gamma=self.gamma, lam=self.gae_lambda)
        if n > 1:
            adv = normalize_advantages(adv, group=_LOCAL)
        m = self._ppo_epochs(states, actions, old_logp, adv, ret, n, np.random.permutation, collective=False)
        m["solver_avg_reward"] = float(np.mean(self.recent_rewards)) if self.recent_rewards else 0.0
        m["solver_episodes"] = self.episode_count
        self._clear_buffers()
        return m

    def _ppo_epochs(self, states, actions, old_logp, adv, ret, n, perm_fn, minibatch=None,
                    collective: bool = True, defer: bool = False):
        """agents/solver.py:157-204: epochs x shuffled minibatches, zero-hidden re-forward.

        collective (batched data-parallel training): every rank runs the same number of
        optimizer steps, max over ranks of ceil(n / minibatch) per epoch.  A rank that has
        run out of samples takes part with an empty minibatch (zero gradient, weight 0);
        the one flat all-reduce per step forms the sample-weighted mean gradient, so all
        ranks clip and step identically and their parameters stay equal.

        defer=True returns a callable that produces the metrics: the steps are only enqueued
        (nothing in the loop waits for the GPU), so the host can do other work meanwhile."""
        self.network.train()
        bs = minibatch or self.batch_size
        tot = torch.zeros(3, device=self.device)
        updates = 0
        params = list(self.network.parameters())
        n_mb = (n + bs - 1) // bs
        multi = collective and dist_utils.is_multi()
        if multi:
            n_mb = int(dist_utils.allreduce_(torch.tensor([n_mb], dtype=torch.int64, device=self.device), "max").item())
        for _ in range(self.ppo_epochs):
            idx = torch.as_tensor(perm_fn(n), device=self.device) if n else None
            for k in range(n_mb):
                start = k * bs
                # grads written by the backward, not accumulated into zeros: every parameter is in
                # the loss graph, so this only saves a fill and an add per parameter and step
                self.optimizer.zero_grad(set_to_none=True)
                w = 0
                if start < n:
                    b = idx[start:start + bs]
                    w = int(b.numel())
                    x = states[b]
                    # MIOpen's convolutions want channels-last; the fp32-MFMA backbone reads the
                    # gathered rows with their own strides (one pass to NHWC4 either way)
                    if x.is_cuda and not (self.update_precision == "fp32" and self.network._train_conv_ok(x)):
                        x = x.contiguous(memory_format=torch.channels_last)
                    with torch.autocast("cuda", dtype=torch.bfloat16,
                                        enabled=self.update_precision == "bf16" and x.is_cuda):
                        logits, new_values, _ = self.network(x)
                    logits, new_values = logits.float(), new_values.float()
                    loss, parts = ppo_loss(logits, new_values.reshape(-1), actions[b], old_logp[b], adv[b], ret[b],
                                           self.clip_epsilon, self.value_coeff, self.entropy_coeff)
                    loss.backward()
                    tot += parts[1:].detach()
                    updates += 1
                if multi:
                    if dist_utils.allreduce_grads(params, weight=w) <= 0:
                        continue
                elif w == 0:
                    continue
                nn.utils.clip_grad_norm_(params, self.max_grad_norm)
                self.optimizer.step()
        def metrics():
            t = (tot / max(updates, 1)).cpu().numpy()
            return {"solver_policy_loss": float(t[0]), "solver_value_loss": float(t[1]), "solver_entropy": float(t[2]),
                    "solver_updates": n_mb * self.ppo_epochs}
        return metrics if defer else metrics()

    # -- batched API ------------------------------------------------------------------
    @torch.no_grad()
    def act(self, obs: torch.Tensor, hidden=None, generator: Optional[torch.Generator] = None,
            fused: Optional[bool] = None):
        """Batched select_action: (action [N], log_prob [N], value [N], hidden).

        fused (default: rollout_precision == "bf16") runs select_action on the fused
        bf16-MFMA HIP kernels where the grid is supported; False keeps the reference fp32
        forward."""
        self.network.eval()
        use = self.fused_inference if fused is None else fused
        if use and self.network.fused_supported(obs) and self.network.head_supported():
            # whole select_action on the fused kernels; the sample comes from a counter-based
            # hash of (seed, call counter, env), so no generator state is consumed per call
            if generator is not None:
                seed = int(torch.randint(0, 2 ** 62, (1,), generator=generator, device=generator.device).item())
            else:
                seed = self._act_seed
            self._act_counter += 1
            action, logp, value, hidden, _ = self.network.act_fused(obs, hidden, seed, self._act_counter)
            return action, logp, value, hidden
        if use and self.network.fused_supported(obs):
            logits, value, hidden = self.network.forward_fused(obs, hidden)
        else:
            logits, value, hidden = self.network(obs, hidden)
        logp_all = F.log_softmax(logits.float(), dim=-1)
        probs = logp_all.exp()
        action = torch.multinomial(probs, 1, generator=generator).reshape(-1)
        # Categorical(probs).log_prob = log(clamp(p / sum p, eps, 1 - eps))
        p = probs / probs.sum(-1, keepdim=True)
        eps = torch.finfo(p.dtype).eps
        logp = torch.log(p.gather(1, action[:, None]).clamp(eps, 1 - eps)).reshape(-1)
        return action, logp, value.reshape(-1).float(), hidden

    @torch.no_grad()
    def value(self, obs: torch.Tensor, hidden=None) -> torch.Tensor:
        """V(s) [N] on the rollout path's precision (the GAE bootstrap at a rollout cut)."""
        self.network.eval()
        if self.fused_inference and self.network.fused_supported(obs) and self.network.head_supported():
            self._act_counter += 1
            return self.network.act_fused(obs, hidden, self._act_seed, self._act_counter)[2]
        if self.fused_inference and self.network.fused_supported(obs):
            return self.network.forward_fused(obs, hidden)[1].reshape(-1).float()
        return self.network(obs, hidden)[1].reshape(-1).float()

    def rollout_advantages(self, ro: Rollout):
        """GAE per env column of a [T, N] rollout (heist_gae): (adv, ret), both [T, N].
        A column cut mid-episode bootstraps from ro.last_value (V(s_T)); a column whose
        last tick ended an episode masks it (done), as the reference's buffer-end 0 does."""
        return compute_gae(ro.rewards, ro.values, ro.dones, ro.last_value, self.gamma, self.gae_lambda)

    @staticmethod
    def _finish(m, n, defer):
        if not defer:
            m["solver_samples"] = n
            return m

        def done():
            out = m()
            out["solver_samples"] = n
            return out
        return done

    def update_rollout(self, ro: Rollout, minibatch: int = 4096, defer: bool = False):
        """One PPO update on a [T, N] rollout (GAE per env column, global advantage norm).
        Collective-safe: with torch.distributed initialised every rank enters the
        normalisation and the same number of optimizer steps, whatever its sample count.
        defer=True: enqueue only, return a callable giving the metrics (_ppo_epochs)."""
        T, N = ro.rewards.shape
        adv, ret = self.rollout_advantages(ro)
        sel = None if ro.mask is None else ro.mask.reshape(1, N).expand(T, N).reshape(-1)
        flat = lambda x: x.reshape(T * N, *x.shape[2:])  # noqa: E731
        states, actions, old_logp, adv, ret = flat(ro.obs), flat(ro.actions), flat(ro.logp), flat(adv), flat(ret)
        if sel is not None:
            states, actions, old_logp, adv, ret = (x[sel] for x in (states, actions, old_logp, adv, ret))
        n = adv.shape[0]
        if n == 0 and not dist_utils.is_multi():
            m0 = {"solver_loss": 0.0}
            return (lambda: m0) if defer else m0
        adv = normalize_advantages(adv)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(int(torch.randint(0, 2 ** 31, (1,)).item()))
        perm = lambda k: torch.randperm(k, device=self.device, generator=gen)  # noqa: E731
        m = self._ppo_epochs(states, actions, old_logp, adv, ret, n, perm, minibatch=minibatch, defer=defer)
        return self._finish(m, n, defer)

    def layout_batch_advantages(self, ro: Rollout, sel: torch.Tensor):
        """The reference's per-layout buffer statistics for a layout-batch rollout
        (agents/solver.py:142-147 for every env at once): GAE per env column with bootstrap 0
        (each env's selected ticks end with its A-th done, so its buffer's GAE is the
        column's up to there), returns = adv + values, then the advantages normalised over
        each env's selected samples with the unbiased std (+ 1e-8), a buffer of one sample
        left as is.  Returns (adv_norm, ret, env_index, tick_index) of the selected samples,
        env-major, in time order within an env."""
        T, N = ro.rewards.shape
        adv, ret = compute_gae(ro.rewards, ro.values, ro.dones, None, self.gamma, self.gae_lambda)
        m = sel.clone()
        if ro.mask is not None:
            m &= ro.mask.reshape(1, N)
        idx = m.t().nonzero()  # [n, 2] (env, tick), env-major
        e_i, t_i = idx[:, 0], idx[:, 1]
        a = adv[t_i, e_i]
        cnt = torch.zeros(N, dtype=torch.float64, device=a.device).index_add_(0, e_i, torch.ones_like(a, dtype=torch.float64))
        s1 = torch.zeros(N, dtype=torch.float64, device=a.device).index_add_(0, e_i, a.double())
        mean = s1 / cnt.clamp(min=1)
        dev2 = (a.double() - mean[e_i]) ** 2
        s2 = torch.zeros(N, dtype=torch.float64, device=a.device).index_add_(0, e_i, dev2)
        std = (s2 / (cnt - 1).clamp(min=1)).sqrt()
        an = ((a.double() - mean[e_i]) / (std[e_i] + 1e-8)).float()
        an = torch.where(cnt[e_i] > 1, an, a)
        return an, ret[t_i, e_i], e_i, t_i

    def update_layout_batch(self, ro: Rollout, sel: torch.Tensor, minibatch: int = 4096, defer: bool = False):
        """One PPO update on a layout-batch rollout (AdversarialTrainer solver_cadence=
        "layout_batch"): the selected transitions of every env's A attempts, per-layout GAE
        and advantage normalisation (layout_batch_advantages), then the clipped update of
        _ppo_epochs (collective inside a process group, as update_rollout)."""
        an, ret, e_i, t_i = self.layout_batch_advantages(ro, sel)
        self.last_layout_batch = (an, ret, e_i, t_i)
        n = int(an.shape[0])
        if n == 0 and not dist_utils.is_multi():
            m0 = {"solver_loss": 0.0}
            return (lambda: m0) if defer else m0
        states = ro.obs[t_i, e_i]
        gen = torch.Generator(device=self.device)
        gen.manual_seed(int(torch.randint(0, 2 ** 31, (1,)).item()))
        perm = lambda k: torch.randperm(k, device=self.device, generator=gen)  # noqa: E731
        m = self._ppo_epochs(states, ro.actions[t_i, e_i], ro.logp[t_i, e_i], an, ret, n, perm, minibatch=minibatch,
                             defer=defer)
        return self._finish(m, n, defer)

    # -- checkpoints ---------------------------------------------------------------------
    def save(self, path: str):  # agents/solver.py:246-252 dict format
        torch.save({"network": self.network.state_dict(), "optimizer": self.optimizer.state_dict(),
                    "episode_count": self.episode_count}, path)

    def load(self, path: str):
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.network.load_state_dict(ck["network"])
        self.optimizer.load_state_dict(ck["optimizer"])
        self.episode_count = ck.get("episode_count", 0)


# normalize_advantages over one rank's buffer even inside a process group (the
# reference-API update() is per-agent, not data-parallel)
_LOCAL = "local"
