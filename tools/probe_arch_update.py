"""The Architect's per-layout update sequence on the GPU: the persistent kernel
(heist_arch_update_sequence) against the HIP-graph replay and the eager update() calls,
at the full-iteration length (3,841 updates, profiles/r03l_probe_train.log), 20x20.

Prints microseconds per update for kernel and graph, the kernel's phase split
(heist_arch_update_stamps: s_memrealtime at the phase points of workgroups 0 and 63,
median over steps 1..15), and the drift of kernel and graph against eager from the same
weights: max |param diff| per tensor and the value-loss trajectories."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd"))
from heist_amd import _native  # noqa: E402
from heist_amd.agents.architect import ArchitectAgent  # noqa: E402

SEGMENTS = [("P1 conv1", 0, 15), ("P1 conv2+store", 15, 1), ("B1", 1, 2),
            ("P2 load a2", 2, 12), ("P2 wv1 issue", 12, 17), ("P2 conv3", 17, 18), ("P2 pool+gp", 18, 3), ("B2", 3, 4),
            ("P3 g", 4, 20), ("P3 h,v,dh,dg", 20, 13), ("P3 dp", 13, 21), ("P3 da3+store", 21, 22),
            ("P3 dW3 wgrad", 22, 16), ("P3 dW3 store", 16, 19), ("P3 sums", 19, 5), ("B3", 5, 6), ("P4 load", 6, 23), ("P4 da2", 23, 14), ("P4 conv1", 14, 24),
            ("P4 dW2 wgrad", 24, 31), ("P4 dW2 store+sums", 31, 7), ("B4", 7, 8), ("P5 loads+sums", 8, 25), ("P5 da1", 25, 26), ("P5 dW1+rec", 26, 9),
            ("B5", 9, 10), ("P6 rec load", 10, 27), ("P6 norms", 27, 28), ("P6 Adam small", 28, 29), ("P6 Adam W2/W3", 29, 30),
            ("P6 Adam Wf/Wv1", 30, 11)]


def agent(sd):
    ag = ArchitectAgent(grid_rows=20, grid_cols=20, device="cuda")
    ag.network.load_state_dict(sd)
    return ag


def timed(mode, sd, r, lp, v, reps=3):
    os.environ["HEIST_ARCH_UPDATE"] = mode
    ag = agent(sd)
    ag.update_sequence(lp[:8], v[:8], r[:8])  # warm-up (graph capture / first launch)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ag.update_sequence(lp, v, r)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def stamps(sd, r, lp, v):
    os.environ["HEIST_ARCH_UPDATE"] = "kernel"
    ag = agent(sd)
    buf = torch.zeros(2 * 16 * 32 + 16 * 5 * 64, dtype=torch.int64, device="cuda")
    _native.lib().heist_arch_update_stamps(_native.ptr(buf))
    ag.update_sequence(lp[:16], v[:16], r[:16])
    torch.cuda.synchronize()
    _native.lib().heist_arch_update_stamps(None)
    allst = buf.cpu().numpy().astype(np.float64) * 10e-3  # 100 MHz ticks -> us
    st = allst[:1024].reshape(2, 16, 32)
    ready = allst[1024:].reshape(16, 5, 64)
    exit_slot = (2, 4, 6, 8, 10)
    print("barriers (steps 1..15, median): skew = last - first workgroup ready (stores drained); "
          "release = workgroup 0 leaving - last ready; slowest workgroups", flush=True)
    for b in range(5):
        rd = ready[1:, b, :]
        skew = np.median(rd.max(1) - rd.min(1))
        rel = np.median(st[0, 1:, exit_slot[b]] - rd.max(1))
        late = np.bincount(rd.argmax(1), minlength=64).argsort()[::-1][:4]
        wg0_wait = np.median(rd.max(1) - rd[:, 0])
        print("   B%d  skew %5.2f  release %5.2f  wg0 waits %5.2f for the last  slowest wgs %s"
              % (b + 1, skew, rel, wg0_wait, list(late)), flush=True)
    for wi, wname in enumerate(("wg0", "wg63")):
        step = np.median(st[wi, 2:, 0] - st[wi, 1:-1, 0])
        print("%s step %.2f us:" % (wname, step), flush=True)
        for name, a, b in SEGMENTS:
            print("   %-16s %6.2f" % (name, np.median(st[wi, 1:, b] - st[wi, 1:, a])))


def drift(sd, r, lp, v):
    out = {}
    for mode in ("kernel", "graph"):
        os.environ["HEIST_ARCH_UPDATE"] = mode
        ag = agent(sd)
        m = ag.update_sequence(lp, v, r)
        out[mode] = (ag, m["architect_value_loss"])
    e = agent(sd)
    for i in range(len(r)):
        e.log_probs, e.values, e.rewards = [torch.tensor(float(lp[i]), device="cuda")], [torch.tensor(float(v[i]), device="cuda")], [float(r[i])]
        me = e.update(collective=False)
    for mode, (ag, vl) in out.items():
        diffs = {n: float((p - q).abs().max()) for (n, p), q in zip(ag.network.state_dict().items(),
                                                                    e.network.state_dict().values())}
        worst = max(diffs.items(), key=lambda kv: kv[1])
        print("%s vs eager after %d updates: value loss %.9g vs %.9g; max |param diff| %.3g (%s)"
              % (mode, len(r), vl, me["architect_value_loss"], worst[1], worst[0]), flush=True)
        print("  per tensor: " + ", ".join("%s %.2g" % (n, d) for n, d in diffs.items() if d > 0))


def main():
    torch.manual_seed(0)
    k = int(os.environ.get("K", "3841"))
    sd = {n: t.detach().clone() for n, t in agent({**ArchitectAgent(device="cuda").network.state_dict()}).network.state_dict().items()}
    g = torch.Generator().manual_seed(1)
    r = torch.rand(k, generator=g, dtype=torch.float64) * 2 - 1
    lp, v = torch.randn(k, generator=g, dtype=torch.float64), torch.randn(k, generator=g, dtype=torch.float64)
    for mode in ("kernel", "graph"):
        dt = timed(mode, sd, r, lp, v)
        print("%-6s k=%d: %.3f ms total, %.2f us per update" % (mode, k, dt * 1e3, dt / k * 1e6), flush=True)
    stamps(sd, r, lp, v)
    if os.environ.get("DRIFT", "0") == "1":
        drift(sd, r, lp, v)


if __name__ == "__main__":
    main()
