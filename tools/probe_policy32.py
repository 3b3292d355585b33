"""Times the fused Solver select_action and backbone at 20x20 (4096 envs) and 32x32 (2048
envs, row-band kernel) with bench.py's measure_policy; prints one JSON line per grid."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda", 0)
for R, n in ((20, 4096), (32, 2048)):
    print(json.dumps(bench.measure_policy(dev, n, R=R)), flush=True)
