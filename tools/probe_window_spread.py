"""Why one 20-tick window in five of the headline runs slow (What's weak 2): the
bench's workload (4096 envs, C2 Architect-checkpoint layouts, K = 20 ticks per launch, after
the same clock settle), every launch timed alone with HIP events, 400 launches.  Per launch:
its duration, the ticks it covers (the shared fan table's offset), the episodes it finishes
(auto-resets, from its done flags) and the camera heading at its first tick (every camera of
an Architect batch shares fov, speed and heading, networks.py:283-322, so all envs' fans
rotate in lockstep).  Prints one JSON line: the per-launch series and their correlations."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402
from heist_amd.layouts import architect_checkpoint_layouts  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n, K, L = 4096, 20, int(os.environ.get("PROBE_LAUNCHES", "400"))
    env = HeistEnv(n, EnvironmentConfig(architect_budget=15), max_cams=5, max_guards=3, max_path=16, device=dev)
    lb, _ = architect_checkpoint_layouts(env, 15, seed=1234, ckpt=os.path.join(ROOT, "checkpoints", "architect_c2_fixed.pt"))
    env.reset()
    cp = lb.cam_params.cpu().numpy()
    nc = lb.n_cams.cpu().numpy()
    live = cp[np.arange(cp.shape[1])[None, :] < nc[:, None]]
    h0, speed = float(live[0, 3]), float(live[0, 4])
    g = torch.Generator(device=dev)
    g.manual_seed(4321)
    acts = torch.randint(0, 5, (L * K, n), device=dev, generator=g, dtype=torch.int64)
    bufs = (torch.empty((K, n, 3, 20, 20), device=dev), torch.empty((K, n), device=dev),
            torch.empty((K, n), dtype=torch.uint8, device=dev), torch.empty((K, n), dtype=torch.int8, device=dev))
    launches = [env.step_multi_launcher(K, acts[i * K:(i + 1) * K], *bufs) for i in range(L)]
    t0 = time.perf_counter()  # clock settle, as bench.py's
    while (time.perf_counter() - t0) < 0.03:
        launches[0]()
    torch.cuda.synchronize(dev)
    env.set_ray_mode(env.kernel_config()["ray_mode"])  # fan table stale: launch 0 refills, then every 51st
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(L + 1)]
    done = torch.zeros(L, dtype=torch.int64, device=dev)
    ev[0].record()
    for i in range(L):
        launches[i]()
        ev[i + 1].record()
        done[i] = bufs[2].sum()  # episodes finished in this launch (on the stream, after it)
    torch.cuda.synchronize(dev)
    ms_all = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(L)])
    refill = np.arange(L) % 51 == 0  # launches that ran fan_kernel first (1,024-tick table, K = 20)
    keep = ~refill
    # the done-count kernel runs between the launches and is inside each event pair: subtract
    # nothing (it is the same small kernel every time); report the relative spread
    resets = done.cpu().numpy().astype(float)[keep]
    tick0 = np.arange(L)[keep] * K
    heading = np.mod(h0 + speed * (tick0 + 1), 360.0)
    ms = ms_all[keep]
    out = {"launches": L, "K": K, "refill_launch_ms": float(ms_all[refill].mean()), "ms_mean": float(ms.mean()), "ms_std": float(ms.std()),
           "ms_min": float(ms.min()), "ms_max": float(ms.max()),
           "ms_p10_p50_p90": [float(np.percentile(ms, p)) for p in (10, 50, 90)],
           "camera": {"heading0": h0, "speed": speed},
           "corr_resets": float(np.corrcoef(ms, resets)[0, 1]),
           "resets_mean": float(resets.mean()),
           "ms": [round(float(x), 4) for x in ms], "resets": resets.astype(int).tolist(),
           "heading": [round(float(x), 2) for x in heading]}
    # mean duration by heading bucket (30 degrees)
    b = (heading // 30).astype(int)
    out["ms_by_heading_bucket"] = {int(k): float(ms[b == k].mean()) for k in np.unique(b)}
    # 5 windows of 20 ticks = one launch each, as the bench times them: spread of 5 consecutive launches
    out["fast_slow_ratio"] = float(np.percentile(ms, 90) / np.percentile(ms, 10))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
