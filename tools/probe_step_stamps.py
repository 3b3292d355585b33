"""Where does one heist_step launch spend its time?  In-kernel phase stamps
(heist_step_stamps: s_memtime at 8 phase boundaries of every wave) over one step of the
bench workload (4096 envs, 20x20, budget-15 layouts, random actions, auto-reset).

Prints one JSON line: per-phase cycles (median / p90 over waves), block lifetime, the
spread of block start times within each XCD (blocks go to XCDs round-robin, and the clock
is compared only within one XCD), and the fraction of envs that auto-reset in the step."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402
from heist_amd import _native as nat  # noqa: E402
from heist_amd.layouts import valid_synthetic_layouts  # noqa: E402


def bench_layouts(env, seed=1234):
    """bench.py's headline layouts (PROBE_LAYOUTS=architect, default: the fixed Architect
    checkpoint at T=1.0, budget 15) or its synthetic mix (PROBE_LAYOUTS=synthetic)."""
    if os.environ.get("PROBE_LAYOUTS", "architect") == "architect":
        import bench
        bench.architect_layouts(env, 15, seed=seed)
    else:
        valid_synthetic_layouts(env, 15, seed=seed)

PHASES = ["prefetch", "update+publish", "raycast", "reward", "auto_reset", "obs_write", "store"]


def q(x, p):
    return float(np.percentile(x, p)) if len(x) else 0.0


def main():
    n = int(os.environ.get("PROBE_N", "4096"))
    env = HeistEnv(n, EnvironmentConfig(), max_cams=8, max_guards=4, max_path=16, device="cuda", auto_reset=True)
    waves = nat.lib().heist_step_waves(env._h)
    bench_layouts(env)
    env.reset()
    acts = torch.randint(0, 5, (16, n), device="cuda")
    for k in range(10):
        env.step(acts[k])
    buf = torch.zeros((n, waves, 10), dtype=torch.int64, device="cuda")
    out = {"n": n, "waves": waves, "steps": []}
    for k in range(3):
        nat.check(nat.lib().heist_step_stamps(env._h, nat.ptr(buf), buf.numel()), "heist_step_stamps")
        _, _, done, _ = env.step(acts[10 + k])
        nat.check(nat.lib().heist_step_stamps(env._h, None, 0), "heist_step_stamps")
        torch.cuda.synchronize()
        s = buf.cpu().numpy().astype(np.int64)
        d = done.cpu().numpy().astype(bool)
        ph = np.diff(s[:, :, :8], axis=2)  # [n, waves, 7]
        rec = {"auto_reset_frac": float(d.mean())}
        rec["phase_cycles_median"] = {nm: q(ph[:, :, i].ravel(), 50) for i, nm in enumerate(PHASES)}
        rec["phase_cycles_p90"] = {nm: q(ph[:, :, i].ravel(), 90) for i, nm in enumerate(PHASES)}
        rec["raycast_cycles_median_reset_envs"] = q(ph[d][:, :, 2].ravel(), 50)
        rec["auto_reset_cycles_median_reset_envs"] = q(ph[d][:, :, 4].ravel(), 50)
        life = s[:, 0, 7] - s[:, 0, 0]
        rec["block_lifetime_cycles"] = {"p10": q(life, 10), "p50": q(life, 50), "p90": q(life, 90), "max": float(life.max())}
        # per-CU timeline (the clock is per CU): HW_ID CU_ID[11:8] SH_ID[12] SE_ID[15:13], XCC_ID[3:0]
        hw = s[:, 0, 8]
        cu = (s[:, 0, 9] & 0xF) * 1024 + ((hw >> 8) & 0xFF)
        spans, counts, first_end = [], [], []
        for c in np.unique(cu):
            idx = np.nonzero(cu == c)[0]
            t0 = s[idx, :, 0].min()
            t1 = s[idx, :, 7].max()
            spans.append(t1 - t0)
            counts.append(len(idx))
            first_end.append(np.sort(s[idx, 0, 0] - t0))
        rec["cus"] = len(spans)
        rec["blocks_per_cu"] = {"min": int(min(counts)), "max": int(max(counts)), "p50": q(counts, 50)}
        rec["cu_span_cycles"] = {"p10": q(spans, 10), "p50": q(spans, 50), "p90": q(spans, 90), "max": float(max(spans))}
        starts = np.concatenate([f for f in first_end])
        rec["block_start_within_cu_cycles"] = {p: q(starts, p) for p in (10, 25, 50, 60, 75, 90, 100)}
        busy = []
        for c in np.unique(cu):
            idx = np.nonzero(cu == c)[0]
            life = (s[idx, 0, 7] - s[idx, 0, 0]).sum()
            t0 = s[idx, :, 0].min()
            t1 = s[idx, :, 7].max()
            busy.append(life / float(t1 - t0))
        rec["mean_resident_blocks_per_cu"] = q(busy, 50)
        out["steps"].append(rec)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
