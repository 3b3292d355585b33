"""Where does heist_step's time go?  Times the step kernel at 4096 envs (bench layouts)
with HEIST_PROBE_MODE = 0 (normal), 1 (no rays), 2 (ray angles + sin/cos only),
3 (marching with a fixed direction, no sin/cos), 4 (no observation write), 5 (neither
rays nor observation write), 6 (return at entry: launch + dispatch floor), 7 (return after
the raycast), 8 (return after the prefetch issue and plane clears), 9 (return before the
raycast barrier: + camera/guard update and emitter table).  Modes 1-7 give wrong results on
purpose; they only bound the cost of each part.  One JSON line per mode."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402
from heist_amd.layouts import valid_synthetic_layouts  # noqa: E402


def bench_layouts(env, seed=1234):
    """bench.py's headline layouts (PROBE_LAYOUTS=architect, default: the fixed Architect
    checkpoint at T=1.0, budget 15) or its synthetic mix (PROBE_LAYOUTS=synthetic)."""
    if os.environ.get("PROBE_LAYOUTS", "architect") == "architect":
        import bench
        bench.architect_layouts(env, 15, seed=seed)
    else:
        valid_synthetic_layouts(env, 15, seed=seed)


def main():
    n = int(os.environ.get("PROBE_N", "4096"))
    envs = {}
    for mode in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9):
        os.environ["HEIST_PROBE_MODE"] = str(mode)
        env = HeistEnv(n, EnvironmentConfig(), max_cams=8, max_guards=4, max_path=16, device="cuda", auto_reset=True)
        bench_layouts(env)
        env.reset()
        envs[mode] = env
    os.environ.pop("HEIST_PROBE_MODE")
    acts = torch.randint(0, 5, (64, n), device="cuda")
    st = torch.cuda.current_stream()
    res = {m: [] for m in envs}
    for rnd in range(5):
        for m, env in envs.items():
            for k in range(5):
                env.step(acts[k])
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for k in range(50):
                env.step(acts[k % 64])
            b.record(st)
            torch.cuda.synchronize()
            res[m].append(a.elapsed_time(b) / 50 * 1e3)
    for m, v in res.items():
        v = sorted(v)
        print(json.dumps({"probe_mode": m, "n": n, "us_per_step_median": round(v[len(v) // 2], 2)}), flush=True)


if __name__ == "__main__":
    main()
