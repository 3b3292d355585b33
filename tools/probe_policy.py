"""Timing probe for the Solver policy on one GPU: fused backbone kernel vs the fp32
PyTorch conv stack, and the whole batched act() both ways.  One JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from heist_amd.agents import SolverAgent  # noqa: E402

FLOP_PER_ENV = 2 * 400 * (32 * 27 + 64 * 288 + 64 * 576)  # conv1..3 at 20x20


def timed(fn, iters=20, warm=3):
    st = torch.cuda.current_stream()
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(iters):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for n in [int(x) for x in os.environ.get("PROBE_N", "1024,4096,16384").split(",")]:
        ag = SolverAgent(20, 20, device=dev)
        net = ag.network
        obs = torch.rand(n, 3, 20, 20, device=dev)
        h = c = torch.zeros(1, n, 128, device=dev)
        ms_k = timed(lambda: net.features_fused(obs))

        def tb():
            with torch.no_grad():
                x = F.relu(net.conv3(F.relu(net.conv2(F.relu(net.conv1(obs))))))
                return net.pool(x)
        ms_t = timed(tb, iters=5)
        ms_af = timed(lambda: ag.act(obs, (h, c), fused=True))
        ms_ar = timed(lambda: ag.act(obs, (h, c), fused=False), iters=5)
        tf = FLOP_PER_ENV * n / (ms_k * 1e-3) / 1e12
        print(json.dumps({"n": n, "backbone_kernel_ms": round(ms_k, 4), "backbone_tflops": round(tf, 1),
                          "mfma_frac_of_2500": round(tf / 2500.0, 4), "backbone_torch_fp32_ms": round(ms_t, 3),
                          "act_fused_ms": round(ms_af, 3), "act_fp32_ms": round(ms_ar, 3)}), flush=True)


if __name__ == "__main__" and not os.environ.get("PROBE_STAMPS"):
    main()


def phase_stamps(n=4096):
    """Median cycles per phase of solver_conv_kernel (s_memtime stamps, second env of
    every workgroup): 0 start, 1 after B1, 2 conv1 done, 3 after B2, 4 conv2 MFMAs done,
    5 conv2 epilogue done, 6 after B3, 7 conv3 done, 8 after B4, 9 end."""
    from heist_amd import _native
    from heist_amd.networks import SolverNetwork
    dev = torch.device("cuda:0")
    net = SolverNetwork().to(dev)
    obs = torch.rand(n, 3, 20, 20, device=dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    buf = torch.zeros(min(n, ncu) * 4 * 10, dtype=torch.int64, device=dev)
    net.features_fused(obs)
    _native.check(_native.lib().heist_solver_stamps(_native.ptr(buf)), "stamps")
    net.features_fused(obs)
    torch.cuda.synchronize()
    _native.check(_native.lib().heist_solver_stamps(None), "stamps")
    st = buf.reshape(-1, 4, 10).double()
    d = (st[:, :, 1:] - st[:, :, :-1]).reshape(-1, 9)
    ok = (st[:, :, 0] > 0).reshape(-1)
    med = d[ok].median(0).values.tolist()
    names = ["stage+B1", "conv1", "B2", "conv2_mfma", "conv2_epi", "B3", "conv3", "pool_xchg+B4", "feat_out"]
    tot = (st[:, :, 9] - st[:, :, 0]).reshape(-1)[ok].median().item()
    print(json.dumps({"phase_median_cycles": dict(zip(names, [round(x) for x in med])), "env_cycles_median": tot}))


if __name__ == "__main__" and os.environ.get("PROBE_STAMPS"):
    phase_stamps()
