"""Mint the "fixed Architect checkpoint" of BASELINE config 2.

The reference's trained checkpoints are not in the mount (.MISSING_LARGE_BLOBS), so the
fixed Architect that C2's Solver trains against is a seeded, untrained ArchitectNetwork
saved in the reference's checkpoint dict format (agents/architect.py:157-163):
{"network": state_dict, "optimizer": Adam state_dict, "episode_count": 0}.
The initialisation is the reference's (networks.py:205-211 order and init calls), so the
same seed gives the same weights in the reference's own ArchitectNetwork.

    python tools/mint_architect_checkpoint.py [out.pt] [--seed 2026]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]

import torch  # noqa: E402

DEFAULT = os.path.join(ROOT, "checkpoints", "architect_c2_fixed.pt")
SEED = 2026


def mint(path: str = DEFAULT, seed: int = SEED, grid: int = 20) -> str:
    from heist_amd.networks import ArchitectNetwork
    torch.manual_seed(seed)
    net = ArchitectNetwork(grid_rows=grid, grid_cols=grid)  # CPU init: device-independent weights
    opt = torch.optim.Adam(net.parameters(), lr=3e-4)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save({"network": net.state_dict(), "optimizer": opt.state_dict(), "episode_count": 0}, path)
    return path


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?", default=DEFAULT)
    ap.add_argument("--seed", type=int, default=SEED)
    a = ap.parse_args()
    print(mint(a.out, a.seed))
