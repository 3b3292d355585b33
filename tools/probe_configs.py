"""Env-only step time at the BASELINE secondary configs (C4: 8192 envs, budget 40; C5:
2048 envs of 32x32 with 4 cameras + 3 guards) for each compiled waves-per-env variant
(HEIST_STEP_WAVES, read at heist_create).  One JSON line per (config, waves)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda", 0)
for waves in ("2", "4"):
    os.environ["HEIST_STEP_WAVES"] = waves
    for name, args, kw in (("c4", (20, 8192, 40), {"architect": True}),
                           ("c5", (32, 2048, 40), {"n_cams": 4, "n_guards": 3})):
        r = bench.measure_env_config(dev, *args, **kw)
        print(json.dumps({"config": name, "waves": int(waves), "value": r["value"], "kernel_ms": r["kernel_ms"]}),
              flush=True)
