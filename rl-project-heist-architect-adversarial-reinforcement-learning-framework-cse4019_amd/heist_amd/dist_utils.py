"""Collective helpers for env-sharded data-parallel training.

The reference is single-process (utils.py:15-25); the build runs one process per GPU,
each owning its own env shard and a replica of both nets.  Every helper here is a
no-op without an initialised process group, and uses only ``all_reduce`` on tensors of
the caller's device: that one collective exists for device tensors on both the RCCL
("nccl") and the gloo backend, so the same code runs on the GPU box and in the
CPU gloo tests.  Every rank must make the same sequence of calls.
"""
from typing import List, Optional, Tuple

import torch


def _dist():
    d = torch.distributed
    return d if d.is_available() and d.is_initialized() else None


def world_size() -> int:
    d = _dist()
    return d.get_world_size() if d else 1


def rank() -> int:
    d = _dist()
    return d.get_rank() if d else 0


def is_multi() -> bool:
    return world_size() > 1


def allreduce_(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """In-place all-reduce (sum / max / min) of t; identity on one rank."""
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return t
    ops = {"sum": d.ReduceOp.SUM, "max": d.ReduceOp.MAX, "min": d.ReduceOp.MIN}
    d.all_reduce(t, op=ops[op])
    return t


def allgather_counts(k: int, device) -> torch.Tensor:
    """Every rank's integer k as an int64 [world] tensor on the host (one all-reduce of a
    one-hot vector)."""
    w = world_size()
    v = torch.zeros(w, dtype=torch.int64, device=device)
    v[rank()] = int(k)
    return allreduce_(v).cpu()


def allgather_rows(x: torch.Tensor, device) -> Tuple[torch.Tensor, List[int]]:
    """Concatenate every rank's [k_r, ...] float tensor in rank order (two all-reduces:
    the counts, then a zero-padded [world, max_k, ...] block).  Returns (rows, counts)."""
    if not is_multi():
        return x, [int(x.shape[0])]
    counts = allgather_counts(x.shape[0], device).tolist()
    kmax = max(counts)
    buf = torch.zeros((world_size(), kmax) + tuple(x.shape[1:]), dtype=x.dtype, device=device)
    if x.shape[0]:
        buf[rank(), :x.shape[0]] = x.to(device)
    allreduce_(buf)
    return torch.cat([buf[r, :counts[r]] for r in range(len(counts))]), counts


def allreduce_grads(params, weight: Optional[float] = None) -> float:
    """Average the gradients of ``params`` over ranks with ONE flat all-reduce.

    Parameters whose .grad is None count as zero (and receive a gradient), so every rank
    sends the same flat length whatever it back-propagated.  With ``weight`` (the number
    of samples behind this rank's gradient, 0 for a rank that sat the minibatch out) the
    result is the sample-weighted mean sum_r w_r g_r / sum_r w_r, and the summed weight,
    appended to the same buffer, is returned; without it the plain mean over ranks.
    On one rank nothing moves and ``weight`` (or 1) is returned."""
    params = list(params)
    if not is_multi():
        return 1.0 if weight is None else float(weight)
    dev = params[0].device
    parts = []
    for p in params:
        g = p.grad
        parts.append(torch.zeros(p.numel(), dtype=torch.float32, device=dev) if g is None
                     else g.detach().reshape(-1).float())
    w = 1.0 if weight is None else float(weight)
    flat = torch.cat(parts + [torch.full((1,), w, dtype=torch.float32, device=dev)])
    if weight is not None:
        flat[:-1] *= w
    allreduce_(flat)
    total = float(flat[-1].item())
    denom = total if weight is not None else float(world_size())
    if denom > 0:
        flat[:-1] /= denom
    o = 0
    for p in params:
        n = p.numel()
        v = flat[o:o + n].view_as(p).to(p.dtype)
        if p.grad is None:
            p.grad = v.clone()
        else:
            p.grad.copy_(v)
        o += n
    return total
