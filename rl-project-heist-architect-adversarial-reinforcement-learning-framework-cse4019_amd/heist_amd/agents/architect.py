"""Architect agent (reference: agents/architect.py).

generate_layout / store_reward / update / save / load keep the reference semantics,
including its "simplified PPO": the log-probabilities are recorded under no_grad, so
the policy term carries no gradient and only the encoder, fc_global and value head
train (agents/architect.py:75-81, :105, :133).  generate_layouts() draws N layouts
from one forward of the (constant-input) network and decodes them on the GPU.

Batched training records each layout's (log_prob, value, reward) as one transition
(store_transitions) when the layout is scored, so rewards can never pair with another
layout's log-prob.  update() is the reference's formula over whatever the buffer holds;
inside a process group it is global: the buffer statistics are all-reduced (one float64
vector), every rank forms the same value target and takes the same step.
"""
import os
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..architect_decode import decode_layouts
from ..networks import ArchitectNetwork
from ..utils import DEVICE, TileType
from .. import dist_utils


class TensorSeq(list):
    """The Architect's per-transition buffers (log_probs, values): a list of 0-d tensors, as
    the reference keeps them, that can also take a whole batch of transitions (a 1-D tensor)
    without splitting it.  A batch is cut into per-element views only when the list is read
    element-wise; stacked(k) gives the first k entries as one tensor without that cut (the
    training loop's path: 3,800 views per iteration cost ~40 ms of host time).  torch's C++
    argument parser reads a list's storage directly (torch.stack(buf) sees only the entries
    already cut), so every path that hands the buffers out materializes them first
    (materialize(); AdversarialTrainer._score_finished, callbacks); only train_iteration,
    which consumes them itself through stacked(k), keeps batches whole."""

    def __init__(self, *a):
        super().__init__(*a)
        self._pending: List[torch.Tensor] = []

    def add_batch(self, t: torch.Tensor):
        self._pending.append(t.reshape(-1))

    def _flush(self):
        if self._pending:
            pend, self._pending = self._pending, []
            for t in pend:
                list.extend(self, t.unbind(0))

    def materialize(self):
        """Cut pending batches into per-element entries (the list then holds everything)."""
        self._flush()

    def __len__(self):
        return list.__len__(self) + sum(int(t.shape[0]) for t in self._pending)

    def __getitem__(self, i):
        self._flush()
        return list.__getitem__(self, i)

    def __iter__(self):
        self._flush()
        return list.__iter__(self)

    def append(self, x):
        self._flush()
        list.append(self, x)

    def extend(self, xs):
        self._flush()
        list.extend(self, xs)

    def clear(self):
        self._pending = []
        list.clear(self)

    def stacked(self, k: int) -> torch.Tensor:
        """The first k entries as one 1-D tensor (each entry squeezed to a scalar)."""
        if list.__len__(self) == 0 and self._pending:
            return torch.cat(self._pending)[:k]
        return torch.stack([x.reshape(()) for x in self[:k]])

    def tensors(self) -> List[torch.Tensor]:
        """The distinct tensors behind the entries (batches whole; element views by storage)."""
        out, seen = list(self._pending), set()
        for x in list.__iter__(self):
            if torch.is_tensor(x) and x.untyped_storage().data_ptr() not in seen:
                seen.add(x.untyped_storage().data_ptr())
                out.append(x)
        return out


class ArchitectAgent:  # agents/architect.py:16-170
    def __init__(self, grid_rows: int = 20, grid_cols: int = 20, budget: int = 15, lr: float = 3e-4,
                 gamma: float = 0.99, clip_epsilon: float = 0.2, entropy_coeff: float = 0.01,
                 value_coeff: float = 0.5, device=None):
        self.grid_rows = grid_rows
        self.grid_cols = grid_cols
        self.budget = budget
        self.gamma = gamma
        self.clip_epsilon = clip_epsilon
        self.entropy_coeff = entropy_coeff
        self.value_coeff = value_coeff
        self.device = torch.device(device) if device is not None else DEVICE
        self.network = ArchitectNetwork(grid_rows=grid_rows, grid_cols=grid_cols).to(self.device)
        self.optimizer = torch.optim.Adam(self.network.parameters(), lr=lr)
        self.log_probs: List[torch.Tensor] = TensorSeq()
        self.values: List[torch.Tensor] = TensorSeq()
        self.rewards: List[float] = []
        self.episode_count = 0
        self.total_reward = 0.0

    def grid_state(self) -> torch.Tensor:
        """The constant Architect input: start and vault markers (agents/architect.py:67-71)."""
        g = torch.zeros((1, 1, self.grid_rows, self.grid_cols), dtype=torch.float32)
        g[0, 0, 1, 1] = TileType.START / 5.0
        g[0, 0, self.grid_rows - 2, self.grid_cols - 2] = TileType.VAULT / 5.0
        return g.to(self.device)

    def generate_layout(self, temperature: float = 1.0):  # agents/architect.py:53-83
        self.network.eval()
        with torch.no_grad():
            walls, cams, guards, log_prob, value = self.network.generate_layout(self.grid_state(), self.budget,
                                                                                 temperature)
        self.log_probs.append(log_prob)
        self.values.append(value)
        return walls, cams, guards

    @torch.no_grad()
    def generate_layouts(self, n: int, temperature: float = 1.0, allow_cameras: bool = True,
                         allow_guards: bool = True, env=None, generator: Optional[torch.Generator] = None,
                         record: bool = True):
        """n layouts as a device LayoutBatch sized for `env` (a HeistEnv), plus per-layout
        log-probs [n] and the (shared) value."""
        self.network.eval()
        amap, total_logp, value, cam = self.network.sample_assets(self.grid_state(), n, temperature, generator)
        kw = {}
        if env is not None:
            kw = dict(max_cams=env.max_cams, max_guards=env.max_guards, max_path=env.max_path)
        lb = decode_layouts(amap, cam, self.budget, allow_cameras, allow_guards, **kw)
        if record:
            self.log_probs.extend(total_logp.unbind(0))
            self.values.extend([value] * n)
        return lb, total_logp, value

    def store_reward(self, reward: float):  # agents/architect.py:85-89
        self.rewards.append(reward)
        self.total_reward += reward
        self.episode_count += 1

    def store_rewards(self, rewards):
        for r in (rewards.tolist() if torch.is_tensor(rewards) else list(rewards)):
            self.store_reward(float(r))

    def store_transitions(self, log_probs: torch.Tensor, values: torch.Tensor, rewards):
        """Batched training: k scored layouts as (log_prob [k], value [k], reward [k]) triples."""
        rw = rewards.tolist() if torch.is_tensor(rewards) else list(rewards)
        if len(rw) != len(log_probs) or len(rw) != len(values):
            raise ValueError("store_transitions: %d log-probs, %d values, %d rewards"
                             % (len(log_probs), len(values), len(rw)))
        for buf, t in ((self.log_probs, log_probs), (self.values, values)):
            if isinstance(buf, TensorSeq):
                buf.add_batch(t.detach().reshape(-1))
            else:
                buf.extend(t.detach().reshape(-1).unbind(0))
        for r in rw:
            self.store_reward(float(r))

    def _step(self, loss: torch.Tensor, collective: bool):
        self.optimizer.zero_grad()
        loss.backward()
        params = list(self.network.parameters())
        if collective:
            dist_utils.allreduce_grads(params)  # identical on every rank already: keeps them bit-equal
        nn.utils.clip_grad_norm_(params, 0.5)
        self.optimizer.step()

    def update(self, collective: Optional[bool] = None) -> Dict[str, float]:  # agents/architect.py:91-155
        """The reference's "simplified PPO" step on the buffered transitions.

        collective (default: inside a process group): every rank must call it, with any
        number (also zero) of local transitions; the statistics of the union are
        all-reduced and the step is skipped on every rank when the union is empty."""
        multi = dist_utils.is_multi() if collective is None else (collective and dist_utils.is_multi())
        if not multi:
            return self._update_local()
        n = min(len(self.rewards), len(self.log_probs), len(self.values))
        d = self.device
        # sums over the union: [k, sum r, sum r^2, sum lp, sum lp*r, sum lp*v, sum v]
        st = torch.zeros(7, dtype=torch.float64, device=d)
        if n:
            r = torch.tensor(self.rewards[:n], dtype=torch.float64, device=d)
            lp = torch.stack(self.log_probs[:n]).to(d).detach().double().reshape(-1)
            v = torch.stack([x.squeeze() for x in self.values[:n]]).to(d).detach().double().reshape(-1)
            st = torch.stack([torch.tensor(float(n), dtype=torch.float64, device=d), r.sum(), (r * r).sum(),
                              lp.sum(), (lp * r).sum(), (lp * v).sum(), v.sum()])
        dist_utils.allreduce_(st)
        k, sr, sr2, slp, slpr, slpv, _ = st.tolist()
        self._clear()
        if k == 0:
            return {"architect_loss": 0.0}
        self.network.train()
        mean = sr / k
        if k > 1:  # (r - mean) / (std_unbiased + 1e-8): the normalised rewards average to 0
            std = max((sr2 - k * mean * mean) / (k - 1), 0.0) ** 0.5
            target, scale = 0.0, 1.0 / (std + 1e-8)
        else:
            target, scale = mean, None
        # policy_loss = -mean(lp * (r_norm - v)), no gradient path (as in the reference)
        s_lp_rn = (slpr - mean * slp) * scale if scale is not None else slpr
        policy_loss = -(s_lp_rn - slpv) / k
        new_value = self.network.value(self.grid_state()).squeeze()
        value_loss = F.mse_loss(new_value, torch.tensor(target, dtype=new_value.dtype, device=d))
        total = policy_loss + self.value_coeff * value_loss
        self._step(total, collective=True)
        return {"architect_policy_loss": float(policy_loss), "architect_value_loss": float(value_loss.item()),
                "architect_total_loss": float(total.item()), "architect_layouts": int(k),
                "architect_avg_reward": self.total_reward / max(self.episode_count, 1)}

    def _update_local(self) -> Dict[str, float]:
        if len(self.rewards) == 0:
            return {"architect_loss": 0.0}
        self.network.train()
        n = min(len(self.rewards), len(self.log_probs), len(self.values))
        rewards = torch.tensor(self.rewards[:n], dtype=torch.float32, device=self.device)
        old_log_probs = torch.stack(self.log_probs[:n]).to(self.device).detach().float()
        old_values = torch.stack([v.squeeze() for v in self.values[:n]]).to(self.device).detach()
        if len(rewards) > 1:
            rewards = (rewards - rewards.mean()) / (rewards.std() + 1e-8)
        advantages = rewards - old_values
        new_value = self.network.value(self.grid_state()).squeeze()  # = forward()'s state_value
        value_loss = F.mse_loss(new_value, rewards.mean())
        policy_loss = -(old_log_probs * advantages.detach()).mean()  # no gradient path, as in the reference
        total_loss = policy_loss + self.value_coeff * value_loss
        self._step(total_loss, collective=False)
        metrics = {"architect_policy_loss": float(policy_loss.item()), "architect_value_loss": float(value_loss.item()),
                   "architect_total_loss": float(total_loss.item()), "architect_layouts": int(n),
                   "architect_avg_reward": self.total_reward / max(self.episode_count, 1)}
        self._clear()
        return metrics

    def side_stream(self):
        """The stream the training loop runs this agent's deferred update on (None off a HIP device)."""
        if self.device.type != "cuda":
            return None
        st = getattr(self, "_side", None)
        if st is None:
            # high priority: the persistent update kernel needs 64 whole CUs (its LDS), and the
            # dispatcher hands CUs freed by the Solver's short kernels to this queue first
            lo, hi = torch.cuda.Stream.priority_range()
            st = self._side = torch.cuda.Stream(device=self.device, priority=min(lo, hi))
        return st

    def update_sequence(self, log_probs: torch.Tensor, values: torch.Tensor, rewards: torch.Tensor,
                        defer: bool = False, join=None):
        """k single-transition updates in order: update() called after each layout with one
        (log_prob, value, reward) in its buffer, k times (the reference's cadence,
        training.py:479-480 / :558-559).  With one reward the value target is the raw
        reward and the policy term is a constant, so update i is one Adam step on
        value_coeff * (V(s0) - r_i)^2 (V on the constant grid state, grad-norm clipped to
        0.5).  On a HIP device all k steps run as ONE persistent kernel
        (heist_arch_update_sequence: forward, fp32 backward, clip and Adam per step with the
        weights and moments on chip).  HEIST_ARCH_UPDATE=graph (A/B) or a grid size the
        kernel is not compiled for takes the HIP-graph path instead: the step captured once
        (forward, backward, clip, capturable Adam, the reward index advanced on the device)
        and replayed k times, the first steps eager as the capture's warm-up.  Returns
        update()'s metrics for the last transition.

        defer=True returns instead a callable that produces those metrics, and nothing here
        waits for the GPU on the kernel path: run it with a side stream current (the training
        loop uses side_stream()) so other work (the Solver's PPO update) runs beside it; the
        callable first makes `join` (a stream, e.g. the main one) wait for the launch."""
        k = int(rewards.numel())
        if k == 0:
            m0 = {"architect_loss": 0.0}
            return (lambda: m0) if defer else m0
        d = self.device
        r32 = rewards.to(device=d, dtype=torch.float32).reshape(-1)
        lp = log_probs.to(device=d, dtype=torch.float32).reshape(-1)
        v = values.to(device=d, dtype=torch.float32).reshape(-1)
        self.network.train()

        def metrics(vlast):
            policy_loss = -(lp[k - 1] * (r32[k - 1] - v[k - 1]))
            total = policy_loss + self.value_coeff * vlast
            return {"architect_policy_loss": float(policy_loss), "architect_value_loss": float(vlast),
                    "architect_total_loss": float(total), "architect_layouts": 1,
                    "architect_avg_reward": self.total_reward / max(self.episode_count, 1)}

        if self._kernel_ok():
            if defer:
                vl = self._kernel_steps(r32)
                done = torch.cuda.Event()
                done.record(torch.cuda.current_stream(d))
                side = torch.cuda.current_stream(d)

                def finish():
                    # the launch's status word (copied behind it) is read where the host
                    # waits for the losses anyway; an invalid launch is undone and re-run
                    done.synchronize()
                    vl_ = vl
                    if self._kernel_failed():
                        with torch.cuda.stream(side):
                            vl_ = self._rerun_after_kernel_failure(r32)
                        side.synchronize()
                    if join is not None:
                        join.wait_event(done)
                        join.wait_stream(side)
                    return metrics(vl_[-1])
                return finish
            vl = self._kernel_steps(r32)
            torch.cuda.current_stream(d).synchronize()
            if self._kernel_failed():
                vl = self._rerun_after_kernel_failure(r32)
            vlast = vl[-1]
        else:
            vlast = self._steps_without_kernel(r32)[-1]
        m = metrics(vlast)
        if defer and join is not None and d.type == "cuda":
            join.wait_stream(torch.cuda.current_stream(d))
        return (lambda: m) if defer else m

    def value_parameters(self) -> List[torch.Tensor]:
        """The 12 tensors the value loss reaches (encoder, fc_global, value_head), in
        parameters() order: the ones update() steps (the decoder and camera heads get no
        gradient, so Adam skips them)."""
        n = self.network
        return [n.encoder[0].weight, n.encoder[0].bias, n.encoder[2].weight, n.encoder[2].bias, n.encoder[4].weight,
                n.encoder[4].bias, n.fc_global.weight, n.fc_global.bias, n.value_head[0].weight, n.value_head[0].bias,
                n.value_head[2].weight, n.value_head[2].bias]

    def _kernel_ok(self) -> bool:
        """The persistent update kernel applies: a HIP device, a compiled grid size, the
        default Adam configuration (one group, no weight decay / amsgrad / maximize), equal
        step counts on the value tensors, 128-byte aligned weights."""
        if self.device.type != "cuda" or os.environ.get("HEIST_ARCH_UPDATE", "kernel") != "kernel":
            return False
        if getattr(self, "_kernel_disabled", False):  # a launch of this agent came back invalid
            return False
        from .. import _native
        if not _native.lib().heist_arch_update_supported(self.grid_rows, self.grid_cols):
            return False
        # its 64 workgroups (one CU each: ~141 KB of LDS) must all be resident at once
        if torch.cuda.get_device_properties(self.device).multi_processor_count < 64:
            return False
        if len(self.optimizer.param_groups) != 1:
            return False
        grp = self.optimizer.param_groups[0]
        if grp.get("weight_decay", 0) != 0 or grp.get("amsgrad") or grp.get("maximize") or grp.get("differentiable"):
            return False
        # fused / capturable Adam (the graph path switches capturable on) form the bias
        # corrections on the device in float32: not the foreach scalars the kernel reproduces
        if grp.get("fused") or grp.get("capturable"):
            return False
        ps = self.value_parameters()
        if any(p.data_ptr() % 128 for p in (ps[2], ps[4], ps[8])) or not all(p.is_contiguous() for p in ps):
            return False
        if getattr(self, "_grid_nnz", None) is None:
            self._grid_nnz = int((self.grid_state() != 0).sum())
        if self._grid_nnz > 64:  # the kernel's conv1 walks the input's nonzeros (the state has 2)
            return False
        steps = {float(self.optimizer.state[p]["step"]) for p in ps if "step" in self.optimizer.state[p]}
        return len(steps) <= 1 and (not steps or all("step" in self.optimizer.state[p] for p in ps))

    def _kernel_steps(self, r32: torch.Tensor) -> torch.Tensor:
        """value steps for every reward of r32 [k] in one heist_arch_update_sequence launch;
        returns the k value losses.  Adam's state is created as torch does on a first step
        (zero moments, step 0) and its step counters advance by k."""
        from .. import _native
        d = self.device
        k = int(r32.numel())
        ps = self.value_parameters()
        grp = self.optimizer.param_groups[0]
        for p in ps:
            st = self.optimizer.state[p]
            if "step" not in st:
                st["step"] = (torch.zeros((), dtype=torch.float32, device=d) if grp.get("capturable")
                              else torch.tensor(0.0, dtype=torch.float32))
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        step0 = float(self.optimizer.state[ps[0]]["step"])
        beta1, beta2 = grp["betas"]
        # the per-step scalars as _multi_tensor_adam forms them: Python floats from the step
        # count (numpy's float64 power is C pow, as Python's **), then float32
        steps = step0 + np.arange(1, k + 1, dtype=np.float64)
        bc1, bc2 = 1.0 - np.power(float(beta1), steps), 1.0 - np.power(float(beta2), steps)
        sc = torch.from_numpy(np.stack([(float(grp["lr"]) / bc1) * -1.0, np.sqrt(bc2)], axis=1).astype(np.float32))
        sc = sc.pin_memory().to(d, non_blocking=True)  # pageable copies would wait for an idle device
        ws = getattr(self, "_au_ws", None)
        nb = int(_native.lib().heist_arch_update_workspace_bytes())
        if ws is None or ws.device != d:
            ws = self._au_ws = torch.empty((nb + 3) // 4, dtype=torch.float32, device=d)
        vl = torch.empty(k, dtype=torch.float32, device=d)
        r = r32.to(device=d, dtype=torch.float32).contiguous()
        grid = getattr(self, "_grid_dev", None)
        if grid is None or grid.device != d:
            grid = self._grid_dev = self.grid_state().contiguous()  # the constant input, made once
        arr = lambda ts: (_native._vp * 12)(*[t.data_ptr() for t in ts])  # noqa: E731
        self.optimizer.zero_grad(set_to_none=True)
        # a copy of everything the launch overwrites: restored if its status word says the
        # results are invalid (heist_arch_update_status; a device-side copy, ~4 MB)
        state = [self.optimizer.state[p] for p in ps]
        live = ps + [st["exp_avg"] for st in state] + [st["exp_avg_sq"] for st in state]
        snap = getattr(self, "_au_snap", None)
        if snap is None or len(snap) != len(live) or any(a.shape != b.shape for a, b in zip(snap, live)):
            snap = self._au_snap = [torch.empty_like(t) for t in live]
        torch._foreach_copy_(snap, [t.detach() for t in live])
        _native.check(_native.lib().heist_arch_update_sequence(
            arr(ps), arr([self.optimizer.state[p]["exp_avg"] for p in ps]),
            arr([self.optimizer.state[p]["exp_avg_sq"] for p in ps]), _native.ptr(grid), self.grid_rows,
            self.grid_cols, _native.ptr(r), k, _native.ptr(sc), float(beta1), float(beta2), float(grp["eps"]),
            0.5, float(self.value_coeff), _native.ptr(vl), _native.ptr(ws), _native.stream(d)),
            "heist_arch_update_sequence")
        # the launch's status word behind it, into pinned memory (read by _kernel_failed)
        stw = getattr(self, "_au_status", None)
        if stw is None:
            stw = self._au_status = torch.zeros(1, dtype=torch.int32).pin_memory()
        off = (nb - 252) // 4  # heist.h: the uint32 at byte offset workspace_bytes - 252
        stw.copy_(ws[off:off + 1].view(torch.int32), non_blocking=True)
        self._au_pending = k
        for p in ps:
            self.optimizer.state[p]["step"].add_(float(k))
        return vl

    def _kernel_failed(self) -> bool:
        """True if the last heist_arch_update_sequence launch reported invalid results (its
        status word, copied behind it; the caller has synchronised with the launch)."""
        if not getattr(self, "_au_pending", 0):
            return False
        code = int(self._au_status[0])
        if dist_utils.is_multi():
            # every rank replays the same steps (training.py's per-layout union): one rank's
            # invalid launch must undo the launch on all of them, or the replicas drift apart
            # (the fallback path's Adam forms its scalars differently), so the decision is
            # the OR of the status words over ranks
            t = torch.tensor([code & 1, code & 2], dtype=torch.int64, device=self.device)
            dist_utils.allreduce_(t, "max")
            code = int(t[0].item()) | int(t[1].item())
            self._au_status[0] = code
        return code != 0

    def _rerun_after_kernel_failure(self, r32: torch.Tensor) -> torch.Tensor:
        """Undo an invalid launch (weights, moments and step counters back to the snapshot
        taken before it), stop using the kernel in this agent, and run the same k steps on
        the eager / graph path.  Returns their value losses."""
        import warnings
        k = self._au_pending
        code = int(self._au_status[0])
        ps = self.value_parameters()
        state = [self.optimizer.state[p] for p in ps]
        live = ps + [st["exp_avg"] for st in state] + [st["exp_avg_sq"] for st in state]
        with torch.no_grad():
            torch._foreach_copy_(live, self._au_snap)
        for st in state:
            st["step"].sub_(float(k))
        self._au_pending = 0
        self._kernel_disabled = True
        warnings.warn("heist_arch_update_sequence reported invalid results (status %d: %s); the %d steps were "
                      "undone and re-run on the %s path, which this agent keeps using"
                      % (code, "grid barrier timed out" if code & 1 else "input has > 64 nonzeros", k,
                         "graph" if self.device.type == "cuda" else "eager"), RuntimeWarning)
        return self._steps_without_kernel(r32)

    def _steps_without_kernel(self, r32: torch.Tensor) -> torch.Tensor:
        """update_sequence without the persistent kernel: the first steps eager (the graph
        capture's warm-up), the rest by graph replay; returns the last value loss (or the
        losses of the replayed ones)."""
        d = self.device
        k = int(r32.numel())
        n_eager = k if d.type != "cuda" or k < 8 else 3
        out = []
        for i in range(n_eager):
            out.append(self._value_step(r32[i]).reshape(1))
        if n_eager < k:
            out.append(self._replay_steps(r32[n_eager:]))
        return torch.cat(out)

    def _value_step(self, r: torch.Tensor) -> torch.Tensor:
        """One eager single-reward step (update() with len(rewards) == 1); returns the value loss."""
        new_value = self.network.value(self.grid_state()).squeeze()
        value_loss = F.mse_loss(new_value, r)
        self._step(self.value_coeff * value_loss, collective=False)
        return value_loss.detach()

    def _replay_steps(self, r32: torch.Tensor) -> torch.Tensor:
        """value steps for every reward of r32 [k'] by graph replay; returns the k' value losses."""
        k = r32.numel()
        g = getattr(self, "_graph", None)
        if g is None or self._g_r.numel() < k:
            g = self._capture(max(k, 1024))
        self._g_r[:k].copy_(r32)
        self._g_i.zero_()
        for _ in range(k):
            g.replay()
        return self._g_vl[:k].clone()

    def _capture(self, cap: int):
        d = self.device
        for grp in self.optimizer.param_groups:  # device-side step counters: no host sync in Adam
            grp["capturable"] = True
        for st in self.optimizer.state.values():
            if "step" in st and st["step"].device != d:
                st["step"] = st["step"].to(d, torch.float32)
        self._g_r = torch.zeros(cap, dtype=torch.float32, device=d)
        self._g_vl = torch.zeros(cap, dtype=torch.float32, device=d)
        self._g_i = torch.zeros(1, dtype=torch.int64, device=d)
        self._g_s = self.grid_state()
        params = list(self.network.parameters())
        self.optimizer.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        # HEIST_ARCH_MIOPEN=0 (A/B): the captured batch-1 convolutions on PyTorch's native
        # kernels instead of MIOpen's
        miopen = os.environ.get("HEIST_ARCH_MIOPEN", "1") != "0"
        with torch.backends.cudnn.flags(enabled=miopen), torch.cuda.graph(g):
            r = self._g_r.index_select(0, self._g_i).squeeze()
            value_loss = F.mse_loss(self.network.value(self._g_s).squeeze(), r)
            self._g_vl.index_copy_(0, self._g_i, value_loss.detach().reshape(1))
            (self.value_coeff * value_loss).backward()
            nn.utils.clip_grad_norm_(params, 0.5)
            self.optimizer.step()
            self._g_i.add_(1)
        self._graph = g
        return g

    def _clear(self):
        self.log_probs.clear()
        self.values.clear()
        self.rewards.clear()

    def optimizer_state_dict(self) -> dict:
        """The optimizer state as the reference's eager Adam keeps it: `capturable` off and
        the step counters as CPU scalars, whatever the graph replay (_capture) switched on,
        so a checkpoint loads into the reference's agent on any device
        (agents/architect.py:165-170: map_location=DEVICE, then Adam.step)."""
        sd = self.optimizer.state_dict()
        groups = [dict(g, capturable=False) for g in sd["param_groups"]]
        state = {}
        for k, st in sd["state"].items():
            st = dict(st)
            if torch.is_tensor(st.get("step")):
                st["step"] = st["step"].detach().to("cpu", torch.float32).reshape(())
            state[k] = st
        return {"state": state, "param_groups": groups}

    def save(self, path: str):  # agents/architect.py:157-163
        torch.save({"network": self.network.state_dict(), "optimizer": self.optimizer_state_dict(),
                    "episode_count": self.episode_count}, path)

    def _drop_graph(self):
        """Forget the captured update step (it holds the old optimizer state tensors)."""
        for k in ("_graph", "_g_r", "_g_vl", "_g_i", "_g_s"):
            self.__dict__.pop(k, None)

    def load(self, path: str):
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.network.load_state_dict(ck["network"])
        self.optimizer.load_state_dict(ck["optimizer"])
        self._drop_graph()  # replays would update the replaced exp_avg / exp_avg_sq / step tensors
        self.episode_count = ck.get("episode_count", 0)
