"""Time the K-tick lean kernel under the current HEIST_* knobs (profiling modes 21-28 need a
library built with tools/build_variant.sh probes -DHEIST_LEAN_PROBES, loaded with
HEIST_LIB=tools/variants/libheist_hip_probes.so; their results are wrong: timing only) on
bench.py's env workload: 4096 envs, K = 20,
PROBE_LAYOUTS architect (the headline) or synthetic.  HIP events around 100 launches after
a clock settle; prints one JSON line (us per tick, median of 3 windows)."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402


def main():
    import bench
    n, K = 4096, int(os.environ.get("PROBE_K", "20"))
    lay = os.environ.get("PROBE_LAYOUTS", "architect")
    env = HeistEnv(n, EnvironmentConfig(architect_budget=15), max_cams=5, max_guards=3, max_path=16, device="cuda")
    if lay == "synthetic":
        from heist_amd.layouts import valid_synthetic_layouts
        valid_synthetic_layouts(env, 15, seed=1234)
    else:
        bench.architect_layouts(env, 15, seed=1234)
    env.reset()
    acts = torch.randint(0, 5, (K, n), device="cuda")
    obs = torch.empty((K, n, 3, 20, 20), device="cuda")
    rew = torch.empty((K, n), device="cuda")
    done = torch.empty((K, n), dtype=torch.uint8, device="cuda")
    st = torch.empty((K, n), dtype=torch.int8, device="cuda")
    t0 = time.time()
    while time.time() - t0 < 0.05:
        env.step_multi_raw(K, acts, obs, rew, done, st)
    torch.cuda.synchronize()
    wins = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(100):
            env.step_multi_raw(K, acts, obs, rew, done, st)
        b.record()
        torch.cuda.synchronize()
        wins.append(a.elapsed_time(b) * 1e3 / (100 * K))
    # the single-tick form (heist_step, what a rollout calls) on the same handle
    single = []
    if os.environ.get("PROBE_SINGLE"):
        for _ in range(3):
            a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a_.record()
            for _ in range(100):
                env.step(acts[0])
            b_.record()
            torch.cuda.synchronize()
            single.append(a_.elapsed_time(b_) * 1e3 / 100)
    print(json.dumps({"layouts": lay, "K": K, "us_per_tick": statistics.median(wins), "windows": wins,
                      "single_tick_us": statistics.median(single) if single else None,
                      "knobs": {k: v for k, v in os.environ.items() if k.startswith("HEIST_")}}), flush=True)


if __name__ == "__main__":
    main()
