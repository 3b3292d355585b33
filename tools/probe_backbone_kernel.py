"""Backbone kernel timing three ways at n envs (PROBE_N, default 4096,16384): HIP events
around 50 features_fused() calls (bench.measure_policy's form), events around 50 direct
heist_solver_features C-ABI calls (no per-call Python work), and one event pair per call.
Run under rocprofv3 --kernel-trace --stats to compare with the kernel's own duration."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import torch  # noqa: E402

from heist_amd import _native  # noqa: E402
from heist_amd.networks import SolverNetwork  # noqa: E402

FLOP = 2 * 400 * (32 * 27 + 64 * 288 + 64 * 576)


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = SolverNetwork().to(dev)
    st = torch.cuda.current_stream(dev)
    for n in [int(x) for x in os.environ.get("PROBE_N", "4096,16384").split(",")]:
        obs = torch.rand(n, 3, 20, 20, device=dev)
        out = torch.empty(n, 1024, device=dev)
        packed = net._packed_backbone()
        L = _native.lib()
        sp = _native.stream(dev)

        def direct():
            _native.check(L.heist_solver_features(_native.ptr(obs), n, 20, 20, _native.ptr(packed), _native.ptr(out), sp),
                          "heist_solver_features")

        res = {"n": n}
        for name, fn in (("features_fused", lambda: net.features_fused(obs)), ("direct", direct)):
            for _ in range(5):
                fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(50):
                fn()
            b.record(st)
            torch.cuda.synchronize(dev)
            res[name + "_ms"] = a.elapsed_time(b) / 50
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
        for a, b in evs:
            a.record(st)
            direct()
            b.record(st)
        torch.cuda.synchronize(dev)
        res["per_call_ms"] = sum(a.elapsed_time(b) for a, b in evs) / 50
        for k in ("features_fused_ms", "direct_ms", "per_call_ms"):
            res[k.replace("_ms", "_frac")] = FLOP * n / (res[k] * 1e-3) / 1e12 / 2500.0
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
