"""Where does a heist_step_multi launch spend its time?  The STAMP variant of the K-tick
kernel (heist_step_stamps armed) sums the shader clock each wave spends in 7 tick segments
over the launch (SEGS below; "a|b": wave 0 does a, waves 1.. do b).  Workload:
bench.py's headline (4096 envs, C2 checkpoint layouts, K ticks per launch), or with
PROBE_LAYOUTS=synthetic the synthetic mix (SURVEY 8d generator ii).

Prints one JSON line: per-segment cycles per tick (mean over waves, by wave index),
launch lifetime per tick, effective clock (cycles per tick x ticks / launch time)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

from heist_amd import EnvironmentConfig, HeistEnv  # noqa: E402
from heist_amd import _native as nat  # noqa: E402

SEGS = ["move+shaping", "emitters|static", "publish|clear", "wait_raycast_barrier", "raycast", "wait_raycast_end",
        "detect+reset", "out|ch1", "tick_end_barrier"]
# step_lean_kernel's segments (20 x 20 / 32 x 32 one wave per env, HEIST_LEAN=1, the default)
LEAN_SEGS = ["dma_wait+fan_hdr", "move+rotate+patrol", "cameras", "guard_cones", "fan_dma+ch1_reads",
             "detect+vault+timeout", "auto_reset", "stores", "-"]


def main():
    import bench
    n = int(os.environ.get("PROBE_N", "4096"))
    K = int(os.environ.get("PROBE_K", "20"))
    env = HeistEnv(n, EnvironmentConfig(architect_budget=15), max_cams=5, max_guards=3, max_path=16, device="cuda")
    if os.environ.get("PROBE_LAYOUTS", "architect") == "synthetic":
        from heist_amd.layouts import valid_synthetic_layouts
        valid_synthetic_layouts(env, 15, seed=1234)
    else:
        bench.architect_layouts(env, 15, seed=1234)
    env.reset()
    kc = env.kernel_config()
    W = kc["multi_waves"]
    segs = LEAN_SEGS if kc["lean"] and W == 1 else SEGS
    acts = torch.randint(0, 5, (4 * K, n), device="cuda")
    for j in range(2):
        env.step_multi(acts[j * K:(j + 1) * K])
    # heist_step_multi checks the buffer against both kernels' needs (a launch without a
    # K-tick variant runs single ticks): n x 10 x step_waves words for heist_step
    words = max(int(nat.lib().heist_stamp_words(env._h, 0)), int(nat.lib().heist_stamp_words(env._h, 1)))
    buf = torch.zeros(max(words, n * W * 16), dtype=torch.int64, device="cuda")
    out = {"layouts": os.environ.get("PROBE_LAYOUTS", "architect"), "n": n, "K": K, "waves": W, "launches": []}
    for j in range(2, 4):
        nat.check(nat.lib().heist_step_stamps(env._h, nat.ptr(buf), buf.numel()), "heist_step_stamps")
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        env.step_multi(acts[j * K:(j + 1) * K])
        ev1.record()
        nat.check(nat.lib().heist_step_stamps(env._h, None, 0), "heist_step_stamps")
        torch.cuda.synchronize()
        s = buf[:n * W * 16].reshape(n, W, 16).cpu().numpy().astype(np.int64)
        rec = {"launch_ms": ev0.elapsed_time(ev1)}
        for w in range(W):
            rec["wave%d_cycles_per_tick" % w] = {nm: float(s[:, w, i].mean()) / K for i, nm in enumerate(segs)}
            # the heaviest envs (top 5 % by lifetime): what sets the launch's length
            top = s[:, w, 9] >= np.percentile(s[:, w, 9], 95)
            rec["wave%d_top5pct_cycles_per_tick" % w] = {nm: float(s[top, w, i].mean()) / K for i, nm in enumerate(segs)}
        life = s[:, 0, 9]
        rec["lifetime_cycles_per_tick"] = {"p10": float(np.percentile(life, 10)) / K, "p50": float(np.median(life)) / K,
                                           "p90": float(np.percentile(life, 90)) / K, "max": float(life.max()) / K}
        rec["effective_clock_ghz_from_max_lifetime"] = float(life.max()) / (rec["launch_ms"] * 1e6)
        # residency: blocks alive at once per CU (the clock is per CU: compare within one)
        hw, xcc, start = s[:, 0, 11], s[:, 0, 12], s[:, 0, 10]
        cu = (xcc & 0xF) * 1024 + ((hw >> 8) & 0xFF)
        conc, per_cu = [], []
        for c in np.unique(cu):
            idx = np.nonzero(cu == c)[0]
            st, en = start[idx], start[idx] + s[idx, 0, 9]
            per_cu.append(len(idx))
            ev = sorted([(x, 1) for x in st] + [(x, -1) for x in en])
            cur = best = 0
            for _, dlt in ev:
                cur += dlt
                best = max(best, cur)
            conc.append(best)
        rec["blocks_per_cu"] = {"min": int(min(per_cu)), "max": int(max(per_cu)), "p50": float(np.median(per_cu))}
        rec["max_concurrent_blocks_per_cu"] = {"min": int(min(conc)), "max": int(max(conc)),
                                               "p50": float(np.median(conc))}
        rec["cus"] = int(len(per_cu))
        out["launches"].append(rec)
        if os.environ.get("PROBE_DUMP"):
            np.savez(os.environ["PROBE_DUMP"] + "_%d.npz" % j, stamps=s, launch_ms=rec["launch_ms"])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
