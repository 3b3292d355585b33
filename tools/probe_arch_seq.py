"""Per-update cost of ArchitectAgent.update_sequence (graph replay of the per-layout
Architect steps) with MIOpen convolutions vs PyTorch's native (im2col + GEMM)
convolutions (HEIST_ARCH_MIOPEN=0).  One JSON line per setting."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

from heist_amd.agents.architect import ArchitectAgent  # noqa: E402


def run(k, miopen):
    os.environ["HEIST_ARCH_MIOPEN"] = "1" if miopen else "0"
    dev = torch.device("cuda")
    torch.manual_seed(5)
    a = ArchitectAgent(grid_rows=20, grid_cols=20, device=dev)
    g = torch.Generator().manual_seed(9)
    lp, v, r = (torch.randn(k, generator=g, dtype=torch.float64) for _ in range(3))
    a.update_sequence(lp[:64], v[:64], r[:64])  # capture + warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a.update_sequence(lp, v, r)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"k": k, "miopen": miopen, "ms_per_update": dt / k * 1e3}), flush=True)


for m in (True, False, True, False):
    run(2000, m)
