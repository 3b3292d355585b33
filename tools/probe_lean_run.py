"""A fixed stream of step_multi launches for profilers (PC sampling, counters): bench.py's
env workload (4096 envs, K = 20 ticks per launch, auto-reset), PROBE_LAYOUTS = architect
(the C2 checkpoint, the headline) or synthetic; PROBE_LAUNCHES launches after 10 warm-up."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402


def main():
    import bench
    n, K = int(os.environ.get("PROBE_N", "4096")), int(os.environ.get("PROBE_K", "20"))
    env = HeistEnv(n, EnvironmentConfig(architect_budget=15), max_cams=5, max_guards=3, max_path=16, device="cuda")
    if os.environ.get("PROBE_LAYOUTS", "architect") == "synthetic":
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
    launches = int(os.environ.get("PROBE_LAUNCHES", "200"))
    for i in range(10 + launches):
        env.step_multi_raw(K, acts, obs, rew, done, st)
    torch.cuda.synchronize()
    print("launches", launches, flush=True)


if __name__ == "__main__":
    main()
