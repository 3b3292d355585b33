"""Which MIOpen solvers serve the Solver backbone's fp32 training convolutions best?  The
three 3x3 convs of SolverNetwork (networks.py:93-100) at the PPO minibatch (16,384 samples of
20x20), forward + data gradient + weight gradient, timed with HIP events for NHWC
(channels_last, the network's format) and NCHW, each with torch.backends.cudnn.benchmark off
(MIOpen's immediate mode / find-db) and on (MIOpen Find: every applicable solver, Winograd
included, is run and the fastest kept).  Also the largest |difference| of each layout's
outputs and gradients from the NHWC immediate-mode ones (relative to their max).  One JSON
line per configuration.  PROBE_N sets the batch."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

N = int(os.environ.get("PROBE_N", "16384"))
dev = torch.device("cuda", 0)


def run(layout, bench, ref=None):
    torch.backends.cudnn.benchmark = bench
    fmt = torch.channels_last if layout == "NHWC" else torch.contiguous_format
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(N, 3, 20, 20, device=dev, generator=g).contiguous(memory_format=fmt)
    ws = [torch.randn(co, ci, 3, 3, device=dev, generator=g) * 0.1 for ci, co in ((3, 32), (32, 64), (64, 64))]
    bs = [torch.randn(co, device=dev, generator=g) * 0.1 for co in (32, 64, 64)]
    ws = [w.contiguous(memory_format=fmt).requires_grad_() for w in ws]
    bs = [b.requires_grad_() for b in bs]
    V = torch.randn(N, 64, 20, 20, device=dev, generator=g).contiguous(memory_format=fmt)

    def step():
        h = x
        for w, b in zip(ws, bs):
            h = F.relu(F.conv2d(h, w, b, padding=1))
        (h * V).sum().backward()
        return h
    t0 = time.perf_counter()
    for _ in range(2):
        h = step()
    torch.cuda.synchronize()
    warm = time.perf_counter() - t0
    for p in ws + bs:
        p.grad = None
    a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    iters = 5
    for _ in range(iters):
        for p in ws + bs:
            p.grad = None
        h = step()
    b_.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b_) / iters
    out = {"layout": layout, "benchmark": bench, "n": N, "ms_fwd_bwd": ms, "warmup_s": warm,
           "tflops": 3 * 2 * N * 400 * (32 * 27 + 64 * 288 + 64 * 576) / (ms * 1e-3) / 1e12}
    res = [h.detach().contiguous().float()] + [w.grad.contiguous() for w in ws] + [b.grad for b in bs]
    if ref is not None:
        out["max_rel_diff"] = max(float((r - q).abs().max()) / max(float(q.abs().max()), 1e-12) for r, q in zip(res, ref))
    print(json.dumps(out), flush=True)
    return res


ref = run("NHWC", False)
for layout, bench in (("NCHW", False), ("NHWC", True), ("NCHW", True)):
    run(layout, bench, ref)
