"""Per-pass timing of the Solver backbone's fp32 training convolutions at the PPO minibatch
size (16,384 samples of 20 x 20): the hand-written fp32-MFMA kernels (heist_train_conv*,
csrc/heist_train_conv.hip) against MIOpen's (torch.ops.aten.convolution / _backward on
channels-last tensors), HIP events over `iters` launches each after a clock-settle phase,
algorithmic TFLOP/s against the 157.3 TF fp32 matrix peak.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd"))

import torch  # noqa: E402

from heist_amd import _native as nat  # noqa: E402
from heist_amd.networks import SolverNetwork, _tc_act, _tc_queues  # noqa: E402

PEAK = 157.3


def timed(fn, dev, iters=10, settle_ms=200.0):
    fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < settle_ms:
        fn()
        torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize(dev)
    return a.elapsed_time(b) / iters


def main():
    dev = torch.device("cuda:0")
    n = int(os.environ.get("PROBE_N", "16384"))
    R = C = 20
    torch.manual_seed(0)
    net = SolverNetwork(R, R).to(dev)
    L = nat.lib()
    st = nat.stream(dev)
    q = _tc_queues(dev)
    P = lambda t: nat._vp(t.data_ptr())  # noqa: E731
    x = torch.rand(n, 3, R, C, device=dev)
    x4 = _tc_act(n, R, C, 3, dev)
    s = x.stride()
    nat.check(L.heist_train_obs_nhwc4(P(x), n, R, C, s[0], s[1], s[2], s[3], P(x4), st), "obs")
    acts = {32: _tc_act(n, R, C, 32, dev), 64: _tc_act(n, R, C, 64, dev)}
    a3 = _tc_act(n, R, C, 64, dev)
    for t in list(acts.values()) + [a3]:
        t.uniform_(-1, 1)
    frags = {}
    for layer, m in ((1, net.conv1), (2, net.conv2), (3, net.conv3)):
        for mode in ((0,) if layer == 1 else (0, 1)):
            f = torch.empty(L.heist_train_conv_frag_floats(layer, mode), device=dev)
            nat.check(L.heist_train_conv_pack(layer, mode, P(m.weight.detach().contiguous()), P(f), st), "pack")
            frags[(layer, mode)] = f
    part = torch.empty(int(L.heist_train_conv_partial_floats(3, n, R, C)), device=dev)
    out = {}
    flop = {1: 2 * n * R * C * 32 * 27, 2: 2 * n * R * C * 64 * 288, 3: 2 * n * R * C * 64 * 576}

    def conv(layer, mode, xin, fr, bias, mask, y):
        return lambda: nat.check(L.heist_train_conv(layer, mode, P(xin), n, R, C, P(fr), P(bias) if bias is not None else None,
                                                    P(mask) if mask is not None else None, P(y), P(q), st), "conv")

    def wgrad(layer, dy, xin, co, ci):
        dw = torch.empty(co, ci, 3, 3, device=dev)
        db = torch.empty(co, device=dev)
        return lambda: nat.check(L.heist_train_conv_wgrad(layer, P(dy), P(xin), n, R, C, P(part), P(dw), P(db), P(q), st),
                                 "wgrad")
    y32, y64 = _tc_act(n, R, C, 32, dev), _tc_act(n, R, C, 64, dev)
    mk = {c: torch.randint(0, 16, (n, R, C, c // 4), dtype=torch.uint8, device=dev) for c in (32, 64)}
    passes = {
        "conv1_fwd": (conv(1, 0, x4, frags[(1, 0)], net.conv1.bias, mk[32], y32), flop[1]),
        "conv2_fwd": (conv(2, 0, acts[32], frags[(2, 0)], net.conv2.bias, mk[64], y64), flop[2]),
        "conv3_fwd": (conv(3, 0, acts[64], frags[(3, 0)], net.conv3.bias, mk[64], y64), flop[3]),
        "conv3_dgrad": (conv(3, 1, a3, frags[(3, 1)], None, mk[64], y64), flop[3]),
        "conv2_dgrad": (conv(2, 1, a3, frags[(2, 1)], None, mk[32], y32), flop[2]),
        "conv3_wgrad": (wgrad(3, a3, acts[64], 64, 64), flop[3]),
        "conv2_wgrad": (wgrad(2, a3, acts[32], 64, 32), flop[2]),
        "conv1_wgrad": (wgrad(1, acts[32], x4, 32, 3), flop[1]),
    }
    for name, (fn, fl) in passes.items():
        ms = timed(fn, dev)
        out[name] = {"ms": ms, "tflops": fl / ms / 1e9, "frac": fl / ms / 1e9 / PEAK}
    # the adaptive pool and its backward (HBM passes: a3 read / d3 written, 68-float rows)
    feat = torch.empty(n, 1024, device=dev)
    dfeat = torch.rand(n, 1024, device=dev)
    d3 = _tc_act(n, R, C, 64, dev)
    act_bytes = n * R * C * 68 * 4
    mem = {"pool": (lambda: nat.check(L.heist_train_pool(P(a3), n, R, C, P(feat), st), "pool"), act_bytes),
           "pool_bwd": (lambda: nat.check(L.heist_train_pool_bwd(P(dfeat), P(mk[64]), n, R, C, P(d3), st), "pool_bwd"),
                        act_bytes + n * R * C * 16)}
    mem_out = {}
    for name, (fn, b) in mem.items():
        ms = timed(fn, dev)
        mem_out[name] = {"ms": ms, "gbs": b / ms / 1e6}
    # MIOpen on the same shapes (channels-last fp32), the path the MFMA kernels replace
    xs = {c: torch.rand(n, c, R, C, device=dev).contiguous(memory_format=torch.channels_last) for c in (3, 32, 64)}
    gy = {c: torch.rand(n, c, R, C, device=dev).contiguous(memory_format=torch.channels_last) for c in (32, 64)}
    conv_ = torch.ops.aten.convolution
    bwd_ = torch.ops.aten.convolution_backward
    mi = {
        "conv1_fwd": (lambda: conv_(xs[3], net.conv1.weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1), flop[1]),
        "conv2_fwd": (lambda: conv_(xs[32], net.conv2.weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1), flop[2]),
        "conv3_fwd": (lambda: conv_(xs[64], net.conv3.weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1), flop[3]),
        "conv3_dgrad": (lambda: bwd_(gy[64], xs[64], net.conv3.weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                     [True, False, False]), flop[3]),
        "conv2_dgrad": (lambda: bwd_(gy[64], xs[32], net.conv2.weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                     [True, False, False]), flop[2]),
        "conv3_wgrad": (lambda: bwd_(gy[64], xs[64], net.conv3.weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                     [False, True, False]), flop[3]),
        "conv2_wgrad": (lambda: bwd_(gy[64], xs[32], net.conv2.weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                     [False, True, False]), flop[2]),
        "conv1_wgrad": (lambda: bwd_(gy[32], xs[3], net.conv1.weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                     [False, True, False]), flop[1]),
    }
    for name, (fn, fl) in mi.items():
        ms = timed(fn, dev)
        out[name]["miopen_ms"] = ms
        out[name]["miopen_frac"] = fl / ms / 1e9 / PEAK
    tot = sum(v["ms"] for v in out.values())
    tot_mi = sum(v["miopen_ms"] for v in out.values())
    print(json.dumps({"n": n, "passes": out, "pool_passes": mem_out, "sum_ms": tot, "sum_miopen_ms": tot_mi,
                      "flop_per_step": 3 * sum(flop.values()) - flop[1]}), flush=True)


if __name__ == "__main__":
    main()
