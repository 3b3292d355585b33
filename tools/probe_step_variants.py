"""heist_step timing across the compiled launch variants at 4096 envs (bench layouts):
waves per env, samples per ray chunk, the waves-per-SIMD bound the kernel is compiled for.
Env vars are read at heist_create.  One JSON line per variant."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402
from heist_amd.layouts import valid_synthetic_layouts  # noqa: E402

VARIANTS = {  # the compiled variants (HEIST_ENV_VARIANTS in heist_env.hip)
    "w2_u4_o8": {"HEIST_STEP_WAVES": "2", "HEIST_STEP_OCC": "8"},
    "w2_u4_o8_exact": {"HEIST_STEP_WAVES": "2", "HEIST_EXACT_RAYS": "1"},
    "w4_u4_o8": {"HEIST_STEP_WAVES": "4", "HEIST_STEP_OCC": "8"},
    "w1_u4_o8": {"HEIST_STEP_WAVES": "1", "HEIST_STEP_OCC": "8"},
}


def main():
    n = int(os.environ.get("PROBE_N", "4096"))
    envs = {}
    for name, ev in VARIANTS.items():
        for k in ("HEIST_STEP_WAVES", "HEIST_RAY_CHUNK", "HEIST_STEP_OCC", "HEIST_EXACT_RAYS"):
            os.environ.pop(k, None)
        os.environ.update(ev)
        env = HeistEnv(n, EnvironmentConfig(), max_cams=8, max_guards=4, max_path=16, device="cuda", auto_reset=True)
        valid_synthetic_layouts(env, 15, seed=1234)
        env.reset()
        envs[name] = env
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
    # all variants must agree bit for bit on the same action stream
    ref = None
    for m, env in envs.items():
        o = env.obs.clone()
        if ref is None:
            ref = o
        same = bool(torch.equal(o, ref))
        v = sorted(res[m])
        print(json.dumps({"variant": m, "n": n, "us_per_step_median": round(v[len(v) // 2], 2),
                          "obs_equal_to_first": same}), flush=True)


if __name__ == "__main__":
    main()
