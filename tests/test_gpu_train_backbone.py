"""The Solver backbone's fp32 training paths against the plain torch ops of the reference
forward (networks.py:93-100) and autograd's backward: pooled features, every conv weight /
bias gradient, and a whole PPO minibatch step of SolverAgent (agents/solver.py:157-199),
within the north_star 1e-4.  Two paths:
  mfma   networks.py _BackboneMFMA32 (20 x 20, the default): every convolution pass on the
         hand-written fp32-MFMA kernels (csrc/heist_train_conv.hip);
  tail   _BackboneF32 (other grids, or HEIST_TRAIN_CONV=0): MIOpen convolutions without bias,
         the bias / ReLU / pool tail fused (csrc/heist_train.hip)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import golden_data as gd
from heist_amd.agents import SolverAgent
from heist_amd.networks import SolverNetwork

pytestmark = pytest.mark.gpu


def _twins(R, dev, sd=None, seed=0, mfma=True):
    torch.manual_seed(seed)
    a = SolverNetwork(R, R).to(dev).to(memory_format=torch.channels_last)
    a.mfma_train = mfma
    if sd is not None:
        a.load_state_dict(sd)
    b = SolverNetwork(R, R).to(dev).to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    b.fused_tail = False
    return a, b


def _states(n, R, dev, seed):
    """observation-like planes: tile / 5, 0/1 visibility, position channel (environment.py:305-374)"""
    g = torch.Generator().manual_seed(seed)
    x = torch.zeros(n, 3, R, R)
    x[:, 0] = torch.randint(0, 6, (n, R, R), generator=g).float() / 5
    x[:, 1] = (torch.rand(n, R, R, generator=g) < 0.3).float()
    x[:, 2] = -0.3 * torch.rand(n, R, R, generator=g)
    return x.to(dev).contiguous(memory_format=torch.channels_last)


def _close(got, want, tol, what):
    scale = max(float(want.abs().max()), 1e-6)
    err = float((got - want).abs().max())
    assert err <= tol * scale, "%s: max |diff| %.3g vs scale %.3g" % (what, err, scale)
    return err / scale


@pytest.mark.parametrize("R", [20, 10, 32])
def test_fused_tail_forward_backward_matches_torch(gpu_device, R):
    """The MIOpen + fused-tail path (_BackboneF32; the MFMA path off): features() and every
    backbone gradient of sum(features * V) (V fixed random) on 384 states vs plain torch,
    relative to each tensor's max within 1e-5 (forward) and 1e-4 (gradients).  R = 10 has
    overlapping pool windows (10 % 4 != 0).  Both sides run MIOpen's convolutions, so their
    ReLU masks agree."""
    n = 384
    a, b = _twins(R, gpu_device, seed=R, mfma=False)
    x2 = _states(2, R, gpu_device, 0)
    assert a._fused_tail_ok(x2) and not b._fused_tail_ok(x2) and not a._train_conv_ok(x2)
    x = _states(n, R, gpu_device, seed=R + 1)
    V = torch.randn(n, 256, device=gpu_device, generator=torch.Generator(device=gpu_device).manual_seed(3))
    fa, fb = a.features(x), b.features(x)
    _close(fa, fb, 1e-5, "features")
    (fa * V).sum().backward()
    (fb * V).sum().backward()
    worst = 0.0
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        if n.startswith(("conv", "fc_spatial")):
            worst = max(worst, _close(p.grad, q.grad, 1e-4, n))
    print("R=%d worst relative gradient difference %.3g" % (R, worst))


def _mfma_forward(net, x):
    """The fp32-MFMA forward through the C ABI (the passes _BackboneMFMA32 runs, deterministic):
    the [n][R][C][P] activations a1, a2, a3."""
    from heist_amd import _native as nat
    from heist_amd.networks import _tc_act, _tc_queues
    L, st, dev = nat.lib(), nat.stream(x.device), x.device
    n, _, R, C = x.shape
    P = lambda t: nat._vp(t.data_ptr())  # noqa: E731
    q = _tc_queues(dev)
    x4 = _tc_act(n, R, C, 3, dev)
    s = x.stride()
    nat.check(L.heist_train_obs_nhwc4(P(x), n, R, C, s[0], s[1], s[2], s[3], P(x4), st), "obs")
    ys, xin = [], x4
    for layer, m, ch in ((1, net.conv1, 32), (2, net.conv2, 64), (3, net.conv3, 64)):
        f = torch.empty(L.heist_train_conv_frag_floats(layer, 0), device=dev)
        nat.check(L.heist_train_conv_pack(layer, 0, P(m.weight.detach().contiguous()), P(f), st), "pack")
        y = _tc_act(n, R, C, ch, dev)
        nat.check(L.heist_train_conv(layer, 0, P(xin), n, R, C, P(f), P(m.bias.detach().contiguous()), None, P(y),
                                     P(q), st), "conv")
        ys.append(y[..., :ch].permute(0, 3, 1, 2))
        xin = y
    torch.cuda.synchronize(dev)
    return ys


def _ref64(net, x, U, masks=None):
    """float64 backbone (CPU) of sum(pool(relu(conv3(relu(conv2(relu(conv1 x)))))) * U): the
    pooled features and the six conv parameter gradients.  masks = the three ReLU masks to use
    (those of the fp32 path under test), else float64's own."""
    ps = [t.detach().double().cpu().requires_grad_() for m in (net.conv1, net.conv2, net.conv3)
          for t in (m.weight, m.bias)]
    a = x.detach().double().cpu()
    own = []
    for k in range(3):
        z = torch.nn.functional.conv2d(a, ps[2 * k], ps[2 * k + 1], padding=1)
        own.append(z > 0)
        a = z * (masks[k].cpu().double() if masks is not None else (z > 0).double())
    f = torch.nn.functional.adaptive_avg_pool2d(a, (4, 4)).reshape(x.shape[0], -1)
    (f * U.double().cpu()).sum().backward()
    return f.detach(), [p.grad for p in ps], own


@pytest.mark.parametrize("n", [384, 257, 2061])
def test_mfma_backbone_matches_float64(gpu_device, n):
    """The fp32-MFMA path (_BackboneMFMA32, the default at 20 x 20) against a float64 reference:
    pooled features within 1e-5 of their max; every conv weight / bias gradient of
    sum(features * U) within 1e-4 of its max against float64 run with the MFMA forward's own
    ReLU masks (two fp32 summation orders can disagree on the sign of a pre-activation within
    rounding of 0 -- a ReLU decision, where the gradient is discontinuous -- so the arithmetic
    is held to the reference where it is defined, and the disagreements are counted: at most
    1e-5 of the pre-activations differ from float64's own masks).  Odd batch sizes: a last
    work unit with one band, a last weight-gradient chunk of 5 bands."""
    from heist_amd.networks import _BackboneMFMA32
    torch.manual_seed(n)
    net = SolverNetwork(20, 20).to(gpu_device).to(memory_format=torch.channels_last)
    for m in (net.conv1, net.conv2, net.conv3):
        torch.nn.init.uniform_(m.bias, -0.05, 0.05)
    x = _states(n, 20, gpu_device, seed=n + 1)
    assert net._train_conv_ok(x)
    U = torch.randn(n, 1024, generator=torch.Generator().manual_seed(5)).to(gpu_device)
    ps = [t for m in (net.conv1, net.conv2, net.conv3) for t in (m.weight, m.bias)]
    feat = _BackboneMFMA32.apply(x, *ps)
    (feat * U).sum().backward()
    masks = [a > 0 for a in _mfma_forward(net, x)]
    f64, g64, own = _ref64(net, x, U, masks)
    _close(feat.detach().cpu().double(), f64, 1e-5, "features")
    flips = sum(int((m.cpu() != o).sum()) for m, o in zip(masks, own))
    total = sum(m.numel() for m in masks)
    assert flips <= 1e-5 * total, (flips, total)
    errs = {name: float((p.grad.detach().cpu().double() - g).abs().max()) / max(float(g.abs().max()), 1e-12)
            for name, p, g in zip(("w1", "b1", "w2", "b2", "w3", "b3"), ps, g64)}
    print("n=%d ReLU decisions differing from float64: %d of %d; gradient errors %s" % (n, flips, total, errs))
    assert max(errs.values()) <= 1e-4, errs


@pytest.mark.parametrize("n", [1, 3, 64, 257, 2061])
def test_mfma_passes_match_torch(gpu_device, n):
    """Each fp32-MFMA pass alone against torch fp32 on the same inputs and masks (so a ReLU
    decision of the forward cannot differ): the three forward layers (bias + ReLU), the data
    gradients of conv3 and conv2 (with the ReLU masks of their inputs), the weight and bias
    gradients of all three, each within 1e-5 of its max (fp32 summation order only).  n = 1 and 3:
    most workgroups draw no unit at all and the last unit holds one band (the dropped
    epilogue stores of the counted-wait scheme); n = 64 gives every workgroup at most one work
    unit; 2061 several units per workgroup (the double-buffered pipeline with its counted DMA
    waits, the k-split hand-off) and several weight-gradient chunks."""
    from heist_amd import _native as nat
    from heist_amd.networks import _tc_act, _tc_queues
    F = torch.nn.functional
    dev = gpu_device
    torch.manual_seed(n)
    net = SolverNetwork(20, 20).to(dev)
    for m in (net.conv1, net.conv2, net.conv3):
        torch.nn.init.uniform_(m.bias, -0.1, 0.1)
    L, st, q = nat.lib(), nat.stream(dev), _tc_queues(dev)
    P = lambda t: nat._vp(t.data_ptr())  # noqa: E731
    R = C = 20
    x = torch.rand(n, 3, R, C, device=dev)
    w = [m.weight.detach() for m in (net.conv1, net.conv2, net.conv3)]
    b = [m.bias.detach() for m in (net.conv1, net.conv2, net.conv3)]
    a1 = F.relu(F.conv2d(x, w[0], b[0], padding=1))
    a2 = F.relu(F.conv2d(a1, w[1], b[1], padding=1))
    a3 = F.relu(F.conv2d(a2, w[2], b[2], padding=1))

    def ours(t, ch):  # [n][R][C][ch + 4]
        o = _tc_act(n, R, C, ch, dev)
        o[..., :ch] = t.permute(0, 2, 3, 1)
        return o

    def back(t, ch):
        return t[..., :ch].permute(0, 3, 1, 2)

    x4 = _tc_act(n, R, C, 3, dev)
    s = x.stride()
    nat.check(L.heist_train_obs_nhwc4(P(x), n, R, C, s[0], s[1], s[2], s[3], P(x4), st), "obs")
    ins = {1: x4, 2: ours(a1, 32), 3: ours(a2, 64)}
    refs = {1: a1, 2: a2, 3: a3}
    for layer, ch in ((1, 32), (2, 64), (3, 64)):
        f = torch.empty(L.heist_train_conv_frag_floats(layer, 0), device=dev)
        nat.check(L.heist_train_conv_pack(layer, 0, P(w[layer - 1].contiguous()), P(f), st), "pack")
        y = _tc_act(n, R, C, ch, dev)
        mo = torch.empty((n, R, C, ch // 4), dtype=torch.uint8, device=dev)
        nat.check(L.heist_train_conv(layer, 0, P(ins[layer]), n, R, C, P(f), P(b[layer - 1]), P(mo), P(y), P(q), st),
                  "conv")
        _close(back(y, ch), refs[layer], 1e-5, "forward %d" % layer)
        got = mo.to(torch.int32)[..., None] >> torch.arange(4, device=dev, dtype=torch.int32) & 1
        assert torch.equal(got.reshape(n, R, C, ch).bool(), (back(y, ch) > 0).permute(0, 2, 3, 1)), layer
    # the pool of conv3's output (the training forward's form)
    feat = torch.empty(n, 1024, device=dev)
    nat.check(L.heist_train_pool(P(ours(a3, 64)), n, R, C, P(feat), st), "pool")
    _close(feat, F.adaptive_avg_pool2d(a3, (4, 4)).reshape(n, -1), 1e-5, "pool")
    # its backward with conv3's ReLU mask (written by the forward above): window / area, masked
    dfeat = torch.randn(n, 1024, device=dev)
    m3 = torch.empty((n, R, C, 16), dtype=torch.uint8, device=dev)
    nat.check(L.heist_train_conv(3, 0, P(ins[3]), n, R, C, P(f), P(b[2]), P(m3), P(_tc_act(n, R, C, 64, dev)), P(q), st),
              "conv3 mask")
    dp = _tc_act(n, R, C, 64, dev)
    nat.check(L.heist_train_pool_bwd(P(dfeat), P(m3), n, R, C, P(dp), st), "pool_bwd")
    ap = a3.detach().clone().requires_grad_(True)
    F.adaptive_avg_pool2d(ap, (4, 4)).reshape(n, -1).backward(dfeat)
    mask3 = (m3.to(torch.int32)[..., None] >> torch.arange(4, device=dev, dtype=torch.int32) & 1).reshape(n, R, C, 64)
    # (torch divides by the window's height, then its width: a last-bit difference)
    _close(back(dp, 64), ap.grad * mask3.permute(0, 3, 1, 2).to(ap.grad.dtype), 1e-6, "pool backward")
    assert torch.equal(back(dp, 64) != 0, (ap.grad * mask3.permute(0, 3, 1, 2)) != 0), "pool backward mask"
    d3 = torch.randn_like(a3) * (a3 > 0)
    gi2, gw3, gb3 = torch.ops.aten.convolution_backward(d3, a2, w[2], [64], [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                        [True, True, True])
    d2 = gi2 * (a2 > 0)
    gi1, gw2, gb2 = torch.ops.aten.convolution_backward(d2, a1, w[1], [64], [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                        [True, True, True])
    d1 = gi1 * (a1 > 0)
    _, gw1, gb1 = torch.ops.aten.convolution_backward(d1, x, w[0], [32], [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                      [False, True, True])
    def bits(t):  # [n][ch][R][C] -> the ReLU mask bits [n][R][C][ch / 4] (uint8: bit r = channel 4 k + r)
        b = (t > 0).permute(0, 2, 3, 1).reshape(n, R, C, t.shape[1] // 4, 4).to(torch.int32)
        return (b << torch.arange(4, device=dev, dtype=torch.int32)).sum(-1).to(torch.uint8).contiguous()

    for layer, dy, mask, ch, ref in ((3, ours(d3, 64), bits(a2), 64, d2), (2, ours(d2, 64), bits(a1), 32, d1)):
        f = torch.empty(L.heist_train_conv_frag_floats(layer, 1), device=dev)
        nat.check(L.heist_train_conv_pack(layer, 1, P(w[layer - 1].contiguous()), P(f), st), "pack")
        y = _tc_act(n, R, C, ch, dev)
        nat.check(L.heist_train_conv(layer, 1, P(dy), n, R, C, P(f), None, P(mask), P(y), P(q), st), "dgrad")
        _close(back(y, ch), ref, 1e-5, "data gradient %d" % layer)
    part = torch.empty(int(max(L.heist_train_conv_partial_floats(k, n, R, C) for k in (1, 2, 3))), device=dev)
    for layer, dy, xin, co, ci, gw, gb in ((3, ours(d3, 64), ins[3], 64, 64, gw3, gb3),
                                           (2, ours(d2, 64), ins[2], 64, 32, gw2, gb2),
                                           (1, ours(d1, 32), x4, 32, 3, gw1, gb1)):
        dw = torch.empty(co, ci, 3, 3, device=dev)
        db = torch.empty(co, device=dev)
        nat.check(L.heist_train_conv_wgrad(layer, P(dy), P(xin), n, R, C, P(part), P(dw), P(db), P(q), st), "wgrad")
        _close(dw, gw, 1e-5, "weight gradient %d" % layer)
        _close(db, gb, 1e-5, "bias gradient %d" % layer)


@pytest.mark.parametrize("path", ["mfma", "tail"])
def test_fused_tail_ppo_minibatch_golden_weights(gpu_device, path):
    """One PPO minibatch (agents/solver.py:172-199: zero-hidden forward, clipped loss,
    backward) of SolverAgent from the reference's seeded weights (nets.npz) on 2,048 states
    (the six golden inputs first): the loss parts and every parameter gradient, fused vs plain
    torch fp32, within 1e-4 (relative to each gradient's max); then the clipped Adam step."""
    z = gd.load("nets.npz")
    sd = {k[len("solver/"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("solver/")}
    ags = []
    for fused in (True, False):
        ag = SolverAgent(20, 20, device=gpu_device)
        ag.network.load_state_dict(sd)
        ag.network.fused_tail = fused
        ag.network.mfma_train = path == "mfma"
        ags.append(ag)
    n = 2048
    x = _states(n, 20, gpu_device, seed=7)
    x[:6] = torch.from_numpy(z["solver_in"]).to(gpu_device)
    g = torch.Generator().manual_seed(8)
    actions = torch.randint(0, 5, (n,), generator=g).to(gpu_device)
    old_logp = (-1.6 + 0.1 * torch.randn(n, generator=g)).to(gpu_device)
    adv = torch.randn(n, generator=g).to(gpu_device)
    ret = torch.randn(n, generator=g).to(gpu_device)
    from heist_amd.ppo import ppo_loss
    outs = []
    for ag in ags:
        ag.network.train()
        ag.optimizer.zero_grad()
        logits, values, _ = ag.network(x)
        loss, parts = ppo_loss(logits, values.reshape(-1), actions, old_logp, adv, ret, ag.clip_epsilon,
                               ag.value_coeff, ag.entropy_coeff)
        loss.backward()
        outs.append((float(loss), parts.detach().cpu().numpy(),
                     {k: p.grad.detach().clone() for k, p in ag.network.named_parameters()}))
    assert ags[0].network._train_conv_ok(x) == (path == "mfma")
    (la, pa, ga), (lb, pb, gb) = outs
    assert abs(la - lb) <= 1e-4 * max(1.0, abs(lb))
    np.testing.assert_allclose(pa, pb, rtol=0, atol=1e-4)
    for k in gb:
        if path == "mfma" and k.startswith("conv"):
            # a ReLU decision within fp32 rounding of 0 may differ between the two summation
            # orders (test_mfma_backbone_matches_float64 holds these to float64 with the
            # MFMA forward's own masks); here: the gradient as a whole within 1 % (L2)
            err = float((ga[k] - gb[k]).norm()) / max(float(gb[k].norm()), 1e-12)
            assert err <= 1e-2, (k, err)
        else:
            _close(ga[k], gb[k], 1e-4, k)
    for ag in ags:
        torch.nn.utils.clip_grad_norm_(list(ag.network.parameters()), ag.max_grad_norm)
        ag.optimizer.step()
    # Adam's first step is lr * sign(g) per element: equal steps, except that an element whose
    # gradient is at rounding-noise level may step the other way (2 lr apart)
    lr = ags[0].optimizer.param_groups[0]["lr"]
    for (k, p), q in zip(ags[0].network.named_parameters(), ags[1].network.parameters()):
        d = (p - q).abs()
        assert float(d.max()) <= 2.01 * lr, k
        assert float((d > 1e-6).float().mean()) <= 0.01, k


def test_fused_tail_used_by_default_and_knob(gpu_device, monkeypatch):
    """The fp32 PPO path takes the fused tail on a HIP device; HEIST_FUSED_TRAIN=0 and
    bf16 autocast (update_precision="bf16") take the plain ops."""
    net = SolverNetwork(20, 20).to(gpu_device).to(memory_format=torch.channels_last)
    x = _states(4, 20, gpu_device, 1)
    assert net._fused_tail_ok(x)
    monkeypatch.setenv("HEIST_FUSED_TRAIN", "0")
    assert not net._fused_tail_ok(x)
    monkeypatch.delenv("HEIST_FUSED_TRAIN")
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert not net._fused_tail_ok(x)
    assert not net._fused_tail_ok(x.cpu())


def test_mfma_backbone_deterministic_and_default(gpu_device, monkeypatch):
    """The fp32-MFMA path is the default at 20 x 20 (HEIST_TRAIN_CONV=0 returns to MIOpen);
    two forward + backward passes on the same input give bit-identical features and gradients
    (dynamic work queues, fixed-order weight-gradient sums); a channels-last input equals the
    NCHW one."""
    net = SolverNetwork(20, 20).to(gpu_device).to(memory_format=torch.channels_last)
    x = _states(1000, 20, gpu_device, 5)
    assert net._train_conv_ok(x)
    monkeypatch.setenv("HEIST_TRAIN_CONV", "0")
    assert not net._train_conv_ok(x) and net._fused_tail_ok(x)
    monkeypatch.delenv("HEIST_TRAIN_CONV")
    outs = []
    for xi in (x, x, x.contiguous()):
        net.zero_grad()
        f = net.features(xi)
        f.square().sum().backward()
        outs.append([f.detach().clone()] + [p.grad.clone() for p in net.parameters() if p.grad is not None])
    for o in outs[1:]:
        for u, v in zip(outs[0], o):
            assert torch.equal(u, v)
