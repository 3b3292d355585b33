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


def make(n, budget, n_cams, n_guards, R=20, waves=4, trig=1):
    os.environ["HEIST_STEP_WAVES"] = str(waves)
    os.environ["HEIST_TRIG_MODE"] = str(trig)
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
for trig in (0, 1):
    for n in (1024, 4096, 16384):
        cases["t%d_n%d_b15" % (trig, n)] = make(n, 15, None, None, trig=trig)
    for nc, ng in ((4, 0), (0, 2)):
        cases["t%d_n4096_c%d_g%d" % (trig, nc, ng)] = make(4096, 3 * nc + 5 * ng + 2, nc, ng, trig=trig)
    cases["t%d_n4096_32x32_c4_g3" % trig] = make(4096, 40, 4, 3, R=32, trig=trig)
res = {k: [] for k in cases}
for rnd in range(5):
    for k, (env, acts) in cases.items():
        res[k].append(time_env(env, acts))
for k, v in res.items():
    n = cases[k][0].n_envs
    med = sorted(v)[len(v) // 2]
    print(json.dumps({"case": k, "us_per_step_median": round(med, 2), "us_min": round(min(v), 2),
                      "Msteps_per_s": round(n / med, 2)}))
