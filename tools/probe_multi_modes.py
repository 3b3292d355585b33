"""Where does a heist_step_multi tick's work go?  The K-tick kernel's profiling variants
(HEIST_PROBE_MODE at heist_create; results wrong on purpose): 0 normal, 1 no raycast / cone
stamps, 2 no observation stores, 3 neither, 4 no ray marches (directions + tie screens).  Workload: bench.py's headline (4096 envs, C2
checkpoint layouts, K = 20).  Launches come in blocks of PER_MODE per mode, modes cycling
0..3 for ROUNDS rounds, so a rocprofv3 --pmc CSV of this script splits by dispatch order
(tools/pmc_summary.py --modes).  Prints one JSON line per mode with the median us per tick."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402

MODES = (0, 1, 2, 3, 4)
PER_MODE = 3
ROUNDS = 3
K = 20


def main():
    import bench
    n = int(os.environ.get("PROBE_N", "4096"))
    envs = {}
    for mode in MODES:
        os.environ["HEIST_PROBE_MODE"] = str(mode)
        env = HeistEnv(n, EnvironmentConfig(architect_budget=15), max_cams=5, max_guards=3, max_path=16, device="cuda")
        bench.architect_layouts(env, 15, seed=1234)
        env.reset()
        envs[mode] = env
    os.environ.pop("HEIST_PROBE_MODE")
    acts = torch.randint(0, 5, (K, n), device="cuda")
    bufs = (torch.empty((K, n, 3, 20, 20), device="cuda"), torch.empty((K, n), device="cuda"),
            torch.empty((K, n), dtype=torch.uint8, device="cuda"), torch.empty((K, n), dtype=torch.int8, device="cuda"))
    res = {m: [] for m in MODES}
    for _ in range(ROUNDS):
        for m in MODES:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(PER_MODE):
                envs[m].step_multi_raw(K, acts, *bufs)
            b.record()
            torch.cuda.synchronize()
            res[m].append(a.elapsed_time(b) / (PER_MODE * K) * 1e3)
    for m in MODES:
        v = sorted(res[m])
        print(json.dumps({"probe_mode": m, "n": n, "K": K, "us_per_tick_median": round(v[len(v) // 2], 3)}), flush=True)


if __name__ == "__main__":
    main()
