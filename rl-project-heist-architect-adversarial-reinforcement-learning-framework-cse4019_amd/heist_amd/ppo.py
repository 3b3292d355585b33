"""GAE, advantage normalisation and the clipped-PPO loss on HIP kernels.

Reference: heist_architect/agents/solver.py:112-244.  The rollout layout is [T, N]
(time-major, one column per env); a column holds that env's episodes back to back,
exactly like the reference's flat per-layout buffer.
"""
from typing import Optional, Tuple

import torch

from . import _native as nat


def compute_gae(rewards: torch.Tensor, values: torch.Tensor, dones: torch.Tensor,
                last_value: Optional[torch.Tensor] = None, gamma: float = 0.99,
                lam: float = 0.95) -> Tuple[torch.Tensor, torch.Tensor]:
    """SolverAgent._compute_gae + returns on [T, N] (or [T]) tensors -> (adv, ret)."""
    squeeze = rewards.dim() == 1
    r = rewards.reshape(rewards.shape[0], -1).float().contiguous()
    v = values.reshape(r.shape).float().contiguous()
    d = dones.reshape(r.shape).to(torch.uint8).contiguous()
    T, N = r.shape
    lv = None if last_value is None else last_value.reshape(N).float().contiguous()
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    nat.check(nat.lib().heist_gae(nat.ptr(r), nat.ptr(v), nat.ptr(d), nat.ptr(lv), T, N, float(gamma), float(lam),
                                  nat.ptr(adv), nat.ptr(ret), nat.stream(r.device)), "heist_gae")
    if squeeze:
        return adv.reshape(T), ret.reshape(T)
    return adv, ret


def normalize_advantages(adv: torch.Tensor, eps: float = 1e-8, group=None, inplace: bool = False) -> torch.Tensor:
    """(adv - mean) / (std + eps) with unbiased std (agents/solver.py:146-147).

    With torch.distributed initialised (or `group` given) the moments are global over
    all ranks: two tiny all-reduces of float64 sums, nothing else crosses the wire; a
    rank with an empty buffer still takes part.  group="local": this rank's buffer only.
    """
    x = adv if inplace else adv.clone()
    x = x.contiguous()
    flat = x.view(-1)
    n = flat.numel()
    acc = torch.zeros(3, dtype=torch.float64, device=x.device)
    st = nat.stream(x.device)
    dist = torch.distributed
    if group == "local":  # this rank's buffer only, even inside a process group
        multi, group = False, None
    else:
        multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    if not multi:
        nat.check(nat.lib().heist_adv_normalize(nat.ptr(flat), n, nat.ptr(acc), float(eps), st), "heist_adv_normalize")
        return x
    nat.check(nat.lib().heist_adv_moments(nat.ptr(flat), n, 0, nat.ptr(acc), st), "heist_adv_moments")
    head = acc[:2].clone()
    dist.all_reduce(head, group=group)
    acc[:2] = head
    nat.check(nat.lib().heist_adv_moments(nat.ptr(flat), n, 1, nat.ptr(acc), st), "heist_adv_moments")
    tail = acc[2:].clone()
    dist.all_reduce(tail, group=group)
    acc[2:] = tail
    nat.check(nat.lib().heist_adv_apply(nat.ptr(flat), n, nat.ptr(acc), float(eps), st), "heist_adv_apply")
    return x


class _PPOLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, values, actions, old_logp, adv, ret, clip, vcoef, ecoef):
        lg = logits.float().contiguous()
        M, A = lg.shape
        v = values.reshape(M).float().contiguous()
        a = actions.reshape(M).to(torch.int64).contiguous()
        ol, ad, rt = (t.reshape(M).float().contiguous() for t in (old_logp, adv, ret))
        parts = torch.empty(4, dtype=torch.float32, device=lg.device)
        dl = torch.empty_like(lg)
        dv = torch.empty_like(v)
        scratch = torch.empty(3 * ((M + 255) // 256), dtype=torch.float64, device=lg.device)
        nat.check(nat.lib().heist_ppo_loss(nat.ptr(lg), nat.ptr(v), nat.ptr(a), nat.ptr(ol), nat.ptr(ad), nat.ptr(rt),
                                           M, A, float(clip), float(vcoef), float(ecoef), nat.ptr(parts), nat.ptr(dl),
                                           nat.ptr(dv), nat.ptr(scratch), nat.stream(lg.device)), "heist_ppo_loss")
        ctx.save_for_backward(dl, dv)
        ctx.vshape = values.shape
        ctx.ldtype = logits.dtype
        ctx.vdtype = values.dtype
        ctx.mark_non_differentiable(parts)
        return parts[0].clone(), parts

    @staticmethod
    def backward(ctx, g_total, g_parts):
        dl, dv = ctx.saved_tensors
        return ((dl * g_total).to(ctx.ldtype), (dv * g_total).reshape(ctx.vshape).to(ctx.vdtype),
                None, None, None, None, None, None, None)


def ppo_loss(logits: torch.Tensor, values: torch.Tensor, actions: torch.Tensor, old_logp: torch.Tensor,
             adv: torch.Tensor, ret: torch.Tensor, clip: float = 0.2, vcoef: float = 0.5,
             ecoef: float = 0.05) -> Tuple[torch.Tensor, torch.Tensor]:
    """loss = pg + vcoef*vl - ecoef*entropy (agents/solver.py:172-193), fused on the GPU.

    Returns (loss, parts) with parts = [total, policy, value, entropy] (detached).
    Differentiable w.r.t. logits and values.
    """
    return _PPOLoss.apply(logits, values, actions, old_logp, adv, ret, clip, vcoef, ecoef)
