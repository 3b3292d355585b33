"""C-oracle vs Python-reference speed on identical layouts, in THIS container (the Python
reference lives at /root/reference and never travels to the GPU box).

bench.py's cpu_baseline times the C oracle (oracle/heist_oracle.c) on the GPU box's host
because the Python reference cannot be run there; this script measures, on one core of
the build container, how much faster the C restatement is than the reference's own CPU
path (HeistEnvironment.step + get_state_tensor, environment.py:216-374) on the same
seeded 20x20 budget-15 layouts with random actions and reset-on-done, so that the GPU
box's C-oracle number can be converted into reference steps/s.  It also replays one
action sequence through both and checks rewards and state tensors are identical (the
ratio compares the same work).  Output: profiles/cpu_ratio.json.

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_ratio.py [--seconds 10] [--layouts 64]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]

from heist_amd.layouts import synthetic_layouts  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def cpu_model():
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--layouts", type=int, default=64)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "cpu_ratio.json"))
    a = ap.parse_args()
    sys.path.insert(0, REF)
    from heist_architect.environment import EnvironmentConfig, HeistEnvironment

    lays = synthetic_layouts(a.layouts, 20, 20, 15, seed=1234)

    # parity of the two timed paths on one action sequence
    rng = np.random.default_rng(7)
    for lay in lays[:4]:
        ref = HeistEnvironment(EnvironmentConfig())
        ref.set_layout(*lay)
        ref.reset()
        orc = po.OracleEnv(20, 20, 200, (1, 1), (18, 18), 15)
        orc.set_layout(*lay)
        orc.reset()
        for _ in range(150):
            act = int(rng.integers(0, 5))
            _, r, d, _ = ref.step(act)
            r2, d2, _ = orc.step(act)
            assert r == r2 and d == d2
            assert ref.get_state_tensor().tobytes() == orc.state_tensor().tobytes()
            if d:
                ref.reset()
                orc.reset()

    # Python reference, one core
    envs = []
    for lay in lays:
        e = HeistEnvironment(EnvironmentConfig())
        e.set_layout(*lay)
        e.reset()
        envs.append(e)
    rng = np.random.default_rng(1)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        for e in envs:
            _, _, d, _ = e.step(int(rng.integers(0, 5)))
            e.get_state_tensor()
            if d:
                e.reset()
        n += len(envs)
    ref_dt = time.perf_counter() - t0
    ref_rate = n / ref_dt

    # C oracle, one thread, same layouts
    def make():
        out = []
        for lay in lays:
            o = po.OracleEnv(20, 20, 200, (1, 1), (18, 18), 15)
            o.set_layout(*lay)
            o.reset()
            out.append(o)
        return out
    orcs = make()
    t0 = time.perf_counter()
    m = po.run_random(orcs, 8, seed=1, n_threads=1)
    dt = time.perf_counter() - t0
    ticks = max(8, int(8 * a.seconds / max(dt, 1e-6)))
    orcs = make()
    t0 = time.perf_counter()
    m = po.run_random(orcs, ticks, seed=2, n_threads=1)
    orc_dt = time.perf_counter() - t0
    orc_rate = m / orc_dt

    res = {"reference_env_steps_per_s_1core": ref_rate, "reference_sample": "%d env-steps in %.1f s" % (n, ref_dt),
           "oracle_env_steps_per_s_1thread": orc_rate, "oracle_sample": "%d env-steps in %.1f s" % (m, orc_dt),
           "oracle_over_reference": orc_rate / ref_rate,
           "workload": "%d synthetic 20x20 budget-15 layouts (SURVEY 8d generator ii, seed 1234), random actions, "
                       "reset on done, get_state_tensor every tick" % len(lays),
           "parity": "4 layouts x 150 ticks replayed through both: rewards, dones and state tensors identical",
           "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "python": platform.python_version(),
           "numpy": np.__version__}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
