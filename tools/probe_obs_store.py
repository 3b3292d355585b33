"""heist_step timing by a handle knob read at heist_create (PROBE_VAR, default
HEIST_OBS_STORE: 0 plain, 1 write-through sc1, 2 nt, 3 sc1 nt observation stores; or e.g.
HEIST_DISPATCH_ORDER 0/1) at 4096 envs on the bench's C2 layouts (fixed Architect
checkpoint, budget 15).  Rounds interleave the policies so clock
and thermal drift hit all of them alike; every policy must give the same observations.
One JSON line per policy."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402


def main():
    n = int(os.environ.get("PROBE_N", "4096"))
    var = os.environ.get("PROBE_VAR", "HEIST_OBS_STORE")
    pols = [int(x) for x in os.environ.get("PROBE_POLICIES", "0,1,2,3").split(",")]
    envs = {}
    for pol in pols:
        os.environ[var] = str(pol)
        env = HeistEnv(n, EnvironmentConfig(), max_cams=8, max_guards=4, max_path=16, device="cuda", auto_reset=True)
        bench.architect_layouts(env, 15, seed=1234)
        env.reset()
        envs[pol] = env
    acts = torch.randint(0, 5, (64, n), device="cuda")
    st = torch.cuda.current_stream()
    res = {m: [] for m in envs}
    for rnd in range(7):
        for m, env in envs.items():
            for k in range(5):
                env.step(acts[k])
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for k in range(100):
                env.step(acts[k % 64])
            b.record(st)
            torch.cuda.synchronize()
            res[m].append(a.elapsed_time(b) / 100 * 1e3)
    ref = None
    for m, env in envs.items():
        o = env.obs.clone()
        if ref is None:
            ref = o
        v = sorted(res[m])
        print(json.dumps({"var": var, "value": m, "n": n, "us_per_step_median": round(v[len(v) // 2], 2),
                          "us_all": [round(x, 2) for x in res[m]], "obs_equal_to_first": bool(torch.equal(o, ref))}),
              flush=True)


if __name__ == "__main__":
    main()
