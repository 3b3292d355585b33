"""Env-only K-tick throughput at the bench's secondary configs, one JSON line each (the same
measure_env_config bench.py runs: K = 20 ticks per launch, clock settle, HIP events):
synthetic 20x20 (4096 envs, budget 15), C4 (8192 envs, budget 40, Architect layouts), C5
(2048 envs of 32x32, 4 cameras + 3 guards).  PROBE_CONFIGS selects (comma list of syn, c4,
c5); HEIST_* knobs in the environment apply (A/B runs)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda", 0)
CONFIGS = {"syn": ((20, 4096, 15), {}), "c4": ((20, 8192, 40), {"architect": True}),
           "c5": ((32, 2048, 40), {"n_cams": 4, "n_guards": 3})}
for name in os.environ.get("PROBE_CONFIGS", "syn,c4,c5").split(","):
    args, kw = CONFIGS[name]
    r = bench.measure_env_config(dev, *args, K=20, **kw)
    print(json.dumps({"config": name, "value": r["value"], "kernel_ms": r["kernel_ms"], "frac": r["roofline"]["frac"],
                      "kernel": r["kernel"], "mean_cameras": r["mean_cameras"], "mean_guards": r["mean_guards"],
                      "knobs": {k: v for k, v in os.environ.items() if k.startswith("HEIST_")}}), flush=True)
