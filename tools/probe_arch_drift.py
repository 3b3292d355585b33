"""Where does the Architect update kernel part from the eager sequence?  From the nets.npz
weights with kat.json-table rewards (the drift test's sequence): two kernel runs compared
bit for bit (determinism), then kernel vs eager checkpointed every `CH` updates (max |param
diff| and value loss at each checkpoint)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_data as gd  # noqa: E402
from heist_amd.agents.architect import ArchitectAgent  # noqa: E402


def main():
    n_sd = gd.load("nets.npz")
    sd = {k[len("architect/"):]: torch.from_numpy(n_sd[k]) for k in n_sd.files if k.startswith("architect/")}
    table = sorted(set(float(v) for v in gd.load_json("kat.json")["architect_reward"].values())) + [-1.0]
    g = torch.Generator().manual_seed(31)
    k = int(os.environ.get("K", "3841"))
    ch = int(os.environ.get("CH", "200"))
    r = torch.tensor(table, dtype=torch.float64)[torch.randint(0, len(table), (k,), generator=g)]
    lp, v = torch.randn(k, generator=g, dtype=torch.float64), torch.randn(k, generator=g, dtype=torch.float64)

    def agent():
        a = ArchitectAgent(grid_rows=20, grid_cols=20, budget=15, device="cuda")
        a.network.load_state_dict(sd)
        return a

    os.environ["HEIST_ARCH_UPDATE"] = "kernel"
    a1, a2 = agent(), agent()
    a1.update_sequence(lp, v, r)
    a2.update_sequence(lp, v, r)
    same = all(torch.equal(p, q) for p, q in zip(a1.network.state_dict().values(), a2.network.state_dict().values()))
    print("two kernel runs bit-identical:", same, flush=True)
    kern, e = agent(), agent()
    for c0 in range(0, k, ch):
        c1 = min(k, c0 + ch)
        mk = kern.update_sequence(lp[c0:c1], v[c0:c1], r[c0:c1])
        for i in range(c0, c1):
            e.log_probs, e.values = [torch.tensor(float(lp[i]), device="cuda")], [torch.tensor(float(v[i]), device="cuda")]
            e.rewards = [float(r[i])]
            me = e.update(collective=False)
        diffs = [(n, float((p - q).abs().max())) for (n, p), q in zip(kern.network.state_dict().items(),
                                                                        e.network.state_dict().values())]
        worst = max(diffs, key=lambda x: x[1])
        with torch.no_grad():
            vk = float(kern.network.value(kern.grid_state()))
            ve = float(e.network.value(e.grid_state()))
        print("after %4d: max |diff| %.3g (%s)  value loss %.7g / %.7g  V(s0) %.7g / %.7g"
              % (c1, worst[1], worst[0], mk["architect_value_loss"], me["architect_value_loss"], vk, ve), flush=True)


if __name__ == "__main__":
    main()
