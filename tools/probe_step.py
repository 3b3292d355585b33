"""Timing probe for heist_step: env count sweep and layout-composition sweep.
Interleaved rounds in one process; prints one JSON line per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402
from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402
from heist_amd.layouts import synthetic_layouts  # noqa: E402


def make(n, budget, n_cams, n_guards, R=20, waves=4, chunk=4, occ=1):
    os.environ["HEIST_STEP_WAVES"] = str(waves)
    os.environ["HEIST_RAY_CHUNK"] = str(chunk)
    os.environ["HEIST_STEP_OCC"] = str(occ)
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R)
    env = HeistEnv(n, cfg, device="cuda")
    lays = synthetic_layouts(n, R, R, budget, seed=1, n_cams=n_cams, n_guards=n_guards)
    env.set_layouts(lays, budget=budget)
    env.reset()
    acts = torch.randint(0, 5, (64, n), device="cuda")
    return env, acts


def time_env(env, acts, iters=40):
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for k in range(5):
        env.step(acts[k])
    a.record(st)
    for k in range(iters):
        env.step(acts[k % 64])
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us per step


cases = {}
for occ in (1, 8):  # min waves per SIMD the step kernel is compiled for
    for n in (4096, 16384):
        cases["o%d_n%d_b15" % (occ, n)] = make(n, 15, None, None, occ=occ)
    cases["o%d_n4096_c4_g0" % occ] = make(4096, 14, 4, 0, occ=occ)
    cases["o%d_n4096_c0_g2" % occ] = make(4096, 12, 0, 2, occ=occ)
for k in ("HEIST_RAY_CHUNK", "HEIST_STEP_WAVES", "HEIST_STEP_OCC"):
    os.environ.pop(k, None)
res = {k: [] for k in cases}
for rnd in range(5):
    for k, (env, acts) in cases.items():
        res[k].append(time_env(env, acts))
for k, v in res.items():
    n = cases[k][0].n_envs
    med = sorted(v)[len(v) // 2]
    print(json.dumps({"case": k, "us_per_step_median": round(med, 2), "us_min": round(min(v), 2),
                      "Msteps_per_s": round(n / med, 2)}))
