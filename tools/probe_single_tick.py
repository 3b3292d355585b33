"""One heist_step launch per tick (the training rollout's form) on the bench's C2 workload
(4096 envs, Architect-checkpoint layouts): the single-tick step kernel (HEIST_STEP_LEAN=0)
against a one-tick heist_step_multi launch of the lean kernel (the default), HIP events
around `steps` ticks after a clock-settle phase; also the lean kernel's K-tick launches for
K = 2, 4, 20 (per-launch overhead = t(K=1) - t(K=20)).  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402
from heist_amd.layouts import architect_checkpoint_layouts  # noqa: E402


def make_env(dev, lean):
    os.environ["HEIST_STEP_LEAN"] = "1" if lean else "0"
    try:
        env = HeistEnv(4096, EnvironmentConfig(architect_budget=15), max_cams=5, max_guards=3, max_path=16, device=dev)
    finally:
        del os.environ["HEIST_STEP_LEAN"]
    _, ok = architect_checkpoint_layouts(env, 15, seed=1234, ckpt=os.path.join(ROOT, "checkpoints", "architect_c2_fixed.pt"))
    env.reset()
    return env


def time_ticks(dev, fn, steps, settle_ms=100.0):
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < settle_ms:
        fn(0)
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for k in range(steps):
        fn(k)
    b.record()
    torch.cuda.synchronize(dev)
    return a.elapsed_time(b)


def main():
    dev = torch.device("cuda:0")
    steps = 200
    acts = torch.randint(0, 5, (steps, 4096), device=dev)
    out = {}
    for lean in (False, True):
        env = make_env(dev, lean)
        name = "lean_k1" if lean else "step_kernel"
        out[name] = {"step_lean": env.kernel_config()["step_lean"],
                     "us_per_tick": time_ticks(dev, lambda k: env.step(acts[k % steps]), steps) / steps * 1e3}
        if lean:
            for K in (1, 2, 4, 20):
                bufs = (torch.empty((K, 4096, 3, 20, 20), device=dev), torch.empty((K, 4096), device=dev),
                        torch.empty((K, 4096), dtype=torch.uint8, device=dev),
                        torch.empty((K, 4096), dtype=torch.int8, device=dev))
                launches = [env.step_multi_launcher(K, acts[j * K:(j + 1) * K], *bufs) for j in range(steps // K)]
                ms = time_ticks(dev, lambda k: launches[k % len(launches)](), len(launches))
                out["multi_K%d" % K] = {"us_per_tick": ms / (len(launches) * K) * 1e3}
        env.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
