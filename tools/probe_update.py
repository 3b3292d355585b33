"""Timing probe: one PPO minibatch step (SolverNetwork forward + backward) at 16384
samples under different precisions / memory formats.  One JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

from heist_amd.networks import SolverNetwork  # noqa: E402


def run(case, net, x, iters=5):
    st = torch.cuda.current_stream()

    def step():
        net.zero_grad(set_to_none=False)
        if case.startswith("bf16"):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                lg, v, _ = net(x)
        else:
            lg, v, _ = net(x)
        (lg.float().square().mean() + v.float().square().mean()).backward()
    for _ in range(2):
        step()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(iters):
        step()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dev = torch.device("cuda:0")
    n = int(os.environ.get("PROBE_MB", "16384"))
    for case in ("fp32", "fp32_cl", "bf16", "bf16_cl"):
        torch.manual_seed(0)
        net = SolverNetwork().to(dev)
        x = torch.rand(n, 3, 20, 20, device=dev)
        if case.endswith("_cl"):
            net = net.to(memory_format=torch.channels_last)
            x = x.contiguous(memory_format=torch.channels_last)
        ms = run(case, net, x)
        print(json.dumps({"case": case, "n": n, "fwd_bwd_ms": round(ms, 3),
                          "tflops": round(3 * 44.93e6 * n / (ms * 1e-3) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
