"""Pass-by-pass check of the fp32-MFMA training convolutions (heist_train_conv*) against
torch fp32 on a small batch: each forward layer, each data gradient, each weight / bias
gradient, printed as max |diff| / max |ref| (diagnostic; the parity tests are
tests/test_gpu_train_backbone.py)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from heist_amd import _native as nat  # noqa: E402
from heist_amd.networks import SolverNetwork, _tc_act, _tc_queues  # noqa: E402


def rel(a, b):
    return float((a - b).abs().max()) / max(float(b.abs().max()), 1e-12)


def main():
    dev = torch.device("cuda:0")
    n = int(os.environ.get("CHECK_N", "64"))
    R = C = 20
    torch.manual_seed(1)
    net = SolverNetwork(R, R).to(dev)
    for m in (net.conv1, net.conv2, net.conv3):
        m.bias.data.uniform_(-0.1, 0.1)
    L = nat.lib()
    st = nat.stream(dev)
    q = _tc_queues(dev)
    P = lambda t: nat._vp(t.data_ptr())  # noqa: E731
    x = torch.rand(n, 3, R, C, device=dev)
    out = {}
    # torch reference
    z1 = F.conv2d(x, net.conv1.weight, net.conv1.bias, padding=1)
    a1 = F.relu(z1)
    z2 = F.conv2d(a1, net.conv2.weight, net.conv2.bias, padding=1)
    a2 = F.relu(z2)
    z3 = F.conv2d(a2, net.conv3.weight, net.conv3.bias, padding=1)
    a3 = F.relu(z3)
    # ours, forward
    x4 = _tc_act(n, R, C, 3, dev)
    s = x.stride()
    nat.check(L.heist_train_obs_nhwc4(P(x), n, R, C, s[0], s[1], s[2], s[3], P(x4), st), "obs")
    out["x4"] = rel(x4[..., :3].permute(0, 3, 1, 2), x)
    ys = {}
    xin = x4
    for layer, m, ch in ((1, net.conv1, 32), (2, net.conv2, 64), (3, net.conv3, 64)):
        f = torch.empty(L.heist_train_conv_frag_floats(layer, 0), device=dev)
        nat.check(L.heist_train_conv_pack(layer, 0, P(m.weight.detach().contiguous()), P(f), st), "pack")
        y = _tc_act(n, R, C, ch, dev)
        nat.check(L.heist_train_conv(layer, 0, P(xin), n, R, C, P(f), P(m.bias.detach()), None, P(y), P(q), st), "conv")
        ys[layer] = y
        xin = y
    fw = dict(ys)
    for layer, ref in ((1, a1), (2, a2), (3, a3)):
        ch = ref.shape[1]
        out["fwd%d" % layer] = rel(ys[layer][..., :ch].permute(0, 3, 1, 2), ref)
    # backward from a random gradient at a3
    g3 = torch.randn_like(a3)
    d3 = g3 * (a3 > 0)
    d3t = _tc_act(n, R, C, 64, dev)
    d3t[..., :64] = d3.permute(0, 2, 3, 1)
    gi2, gw3, gb3 = torch.ops.aten.convolution_backward(d3, a2, net.conv3.weight, [64], [1, 1], [1, 1], [1, 1], False,
                                                        [0, 0], 1, [True, True, True])
    d2 = gi2 * (a2 > 0)
    gi1, gw2, gb2 = torch.ops.aten.convolution_backward(d2, a1, net.conv2.weight, [64], [1, 1], [1, 1], [1, 1], False,
                                                        [0, 0], 1, [True, True, True])
    d1 = gi1 * (a1 > 0)
    _, gw1, gb1 = torch.ops.aten.convolution_backward(d1, x, net.conv1.weight, [32], [1, 1], [1, 1], [1, 1], False,
                                                      [0, 0], 1, [False, True, True])
    part = torch.empty(int(max(L.heist_train_conv_partial_floats(k, n, R, C) for k in (1, 2, 3))), device=dev)

    def dgrad(layer, w, dy, mask, ch):
        f = torch.empty(L.heist_train_conv_frag_floats(layer, 1), device=dev)
        nat.check(L.heist_train_conv_pack(layer, 1, P(w.detach().contiguous()), P(f), st), "pack")
        y = _tc_act(n, R, C, ch, dev)
        nat.check(L.heist_train_conv(layer, 1, P(dy), n, R, C, P(f), None, P(mask), P(y), P(q), st), "dgrad")
        torch.cuda.synchronize()
        return y

    def wgrad(layer, dy, xin, co, ci):
        dw = torch.empty(co, ci, 3, 3, device=dev)
        db = torch.empty(co, device=dev)
        nat.check(L.heist_train_conv_wgrad(layer, P(dy), P(xin), n, R, C, P(part), P(dw), P(db), P(q), st), "wgrad")
        torch.cuda.synchronize()
        return dw, db
    # each pass from the torch reference's inputs and masks (so errors do not compound, and a
    # ReLU mask that flips between two fp32 summation orders does not count as an error)
    def ours(t, ch):
        o = _tc_act(n, R, C, ch, dev)
        o[..., :ch] = t.permute(0, 2, 3, 1)
        return o
    ys = {1: ours(a1.detach(), 32), 2: ours(a2.detach(), 64)}
    d2m = dgrad(3, net.conv3.weight, d3t, ys[2], 64)
    out["dgrad3"] = rel(d2m[..., :64].permute(0, 3, 1, 2), d2)
    d2t = _tc_act(n, R, C, 64, dev)
    d2t[..., :64] = d2.permute(0, 2, 3, 1)
    d1m = dgrad(2, net.conv2.weight, d2t, ys[1], 32)
    out["dgrad2"] = rel(d1m[..., :32].permute(0, 3, 1, 2), d1)
    dw3, db3 = wgrad(3, d3t, ys[2], 64, 64)
    # our own forward's masks against torch's (how many ReLU decisions differ between the two
    # fp32 summation orders)
    out["mask_flips"] = {k: int(((yy[..., :r.shape[1]].permute(0, 3, 1, 2) > 0) != (r > 0)).sum())
                         for k, yy, r in (("a1", fw[1], a1), ("a2", fw[2], a2), ("a3", fw[3], a3))}
    out["wgrad3"], out["bgrad3"] = rel(dw3, gw3), rel(db3, gb3)
    dw2, db2 = wgrad(2, d2t, ys[1], 64, 32)
    out["wgrad2"], out["bgrad2"] = rel(dw2, gw2), rel(db2, gb2)
    d1t = _tc_act(n, R, C, 32, dev)
    d1t[..., :32] = d1.permute(0, 2, 3, 1)
    dw1, db1 = wgrad(1, d1t, x4, 32, 3)
    out["wgrad1"], out["bgrad1"] = rel(dw1, gw1), rel(db1, gb1)
    if out["wgrad1"] > 1e-4:  # where: per tap / input channel
        err = (dw1 - gw1).abs().amax(dim=0)
        out["wgrad1_err_ci_tap"] = err.reshape(3, 9).tolist()
    print(json.dumps({"n": n, "rel_err": out}), flush=True)


if __name__ == "__main__":
    main()
