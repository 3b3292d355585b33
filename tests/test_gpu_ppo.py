"""GPU parity of the GAE scan, advantage normalisation and fused clipped-PPO loss.

Floating point: within 1e-4 of the reference (north star), checked against the
reference's golden vectors, the C oracle and a plain PyTorch fp32 autograd
restatement of agents/solver.py:172-193.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import golden_data as gd
from oracle import pyoracle as po
from heist_amd.ppo import compute_gae, normalize_advantages, ppo_loss

pytestmark = pytest.mark.gpu
TOL = 1e-4


def test_gae_golden(gpu_device):
    z = gd.load("ppo.npz")
    for i in range(int(z["n_gae"])):
        r, v, d = (torch.tensor(z["gae%d_%s" % (i, k)], device=gpu_device) for k in "rvd")
        adv, ret = compute_gae(r, v, d)
        np.testing.assert_allclose(adv.cpu().numpy(), z["gae%d_adv" % i], atol=TOL, rtol=0)
        np.testing.assert_allclose(ret.cpu().numpy(), z["gae%d_ret" % i], atol=TOL, rtol=0)
        norm = normalize_advantages(adv)
        np.testing.assert_allclose(norm.cpu().numpy(), z["gae%d_norm" % i], atol=TOL, rtol=0)


def test_gae_columns_vs_oracle(gpu_device):
    rng = np.random.default_rng(0)
    T, N = 203, 4096
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    d = (rng.random((T, N)) < 0.03).astype(np.uint8)
    adv, ret = compute_gae(*(torch.from_numpy(x).to(gpu_device) for x in (r, v, d)))
    adv = adv.cpu().numpy()
    for n in rng.choice(N, 64, replace=False):
        exp = po.gae(r[:, n], v[:, n], d[:, n].astype(np.float32))
        np.testing.assert_array_equal(adv[:, n], exp)  # same float32 op order: bit-exact
    np.testing.assert_array_equal(ret.cpu().numpy(), adv + v)


def test_gae_bootstrap(gpu_device):
    r = torch.zeros(3, 1, device=gpu_device)
    v = torch.zeros(3, 1, device=gpu_device)
    d = torch.zeros(3, 1, dtype=torch.uint8, device=gpu_device)
    lv = torch.ones(1, device=gpu_device)
    adv, _ = compute_gae(r, v, d, last_value=lv)
    g, lam = 0.99, 0.95
    assert abs(float(adv[2, 0]) - g) < 1e-6
    assert abs(float(adv[0, 0]) - g * (g * lam) ** 2) < 1e-6


def test_normalize_large(gpu_device):
    x = torch.randn(1 << 22, device=gpu_device) * 3 + 5
    y = normalize_advantages(x)
    ref = (x - x.mean()) / (x.std() + 1e-8)
    assert float((y - ref).abs().max()) < 1e-4


def _torch_reference_loss(logits, values, actions, old, adv, ret, clip=0.2, vc=0.5, ec=0.05):
    """agents/solver.py:175-193 in plain PyTorch fp32."""
    probs = F.softmax(logits, dim=-1)
    dist = torch.distributions.Categorical(probs)
    nl = dist.log_prob(actions)
    ent = dist.entropy().mean()
    ratio = torch.exp(nl - old)
    pl = -torch.min(ratio * adv, torch.clamp(ratio, 1 - clip, 1 + clip) * adv).mean()
    vl = F.mse_loss(values.squeeze(), ret)
    return pl + vc * vl - ec * ent, pl, vl, ent


def test_ppo_loss_golden(gpu_device):
    z = gd.load("ppo.npz")
    for i in range(int(z["n_loss"])):
        g = lambda k: torch.tensor(z["loss%d_%s" % (i, k)], device=gpu_device)  # noqa: E731
        logits = g("logits").requires_grad_(True)
        values = g("values").requires_grad_(True)
        loss, parts = ppo_loss(logits, values, g("actions"), g("old"), g("adv"), g("ret"))
        loss.backward()
        p = parts.cpu().numpy()
        assert abs(p[1] - float(z["loss%d_pg" % i])) < TOL
        assert abs(p[2] - float(z["loss%d_vl" % i])) < TOL
        assert abs(p[3] - float(z["loss%d_ent" % i])) < TOL
        np.testing.assert_allclose(logits.grad.cpu().numpy(), z["loss%d_dlogits" % i], atol=1e-6, rtol=TOL)
        np.testing.assert_allclose(values.grad.cpu().numpy(), z["loss%d_dvalues" % i], atol=1e-6, rtol=TOL)


@pytest.mark.parametrize("M", [1, 64, 1000, 65536])
def test_ppo_loss_vs_torch_autograd(M, gpu_device):
    gen = torch.Generator(device="cpu").manual_seed(M)
    logits = (torch.randn(M, 5, generator=gen) * 2).to(gpu_device)
    logits[0, 0] = 40.0  # clamp branch
    values = torch.randn(M, 1, generator=gen).to(gpu_device)
    actions = torch.randint(0, 5, (M,), generator=gen).to(gpu_device)
    with torch.no_grad():
        old = torch.distributions.Categorical(F.softmax(logits, -1)).log_prob(actions) + \
            torch.randn(M, generator=gen).to(gpu_device) * 0.3
    adv = torch.randn(M, generator=gen).to(gpu_device)
    ret = torch.randn(M, generator=gen).to(gpu_device)
    l1, v1 = logits.clone().requires_grad_(True), values.clone().requires_grad_(True)
    loss, parts = ppo_loss(l1, v1, actions, old, adv, ret)
    loss.backward()
    l2, v2 = logits.clone().requires_grad_(True), values.clone().requires_grad_(True)
    ref, pl, vl, ent = _torch_reference_loss(l2, v2, actions, old, adv, ret)
    ref.backward()
    assert abs(float(loss) - float(ref)) < TOL
    assert abs(float(parts[3]) - float(ent)) < TOL
    torch.testing.assert_close(l1.grad, l2.grad, atol=1e-6, rtol=1e-3)
    torch.testing.assert_close(v1.grad, v2.grad, atol=1e-6, rtol=1e-4)


def test_ppo_loss_vs_oracle(gpu_device):
    rng = np.random.default_rng(9)
    M = 4096
    logits = rng.normal(0, 2, (M, 5)).astype(np.float32)
    values = rng.normal(size=M).astype(np.float32)
    actions = rng.integers(0, 5, M)
    old = rng.normal(-1.6, 0.5, M).astype(np.float32)
    adv = rng.normal(size=M).astype(np.float32)
    ret = rng.normal(size=M).astype(np.float32)
    parts_o, dl_o, dv_o = po.ppo_loss(logits, values, actions, old, adv, ret)
    t = lambda a: torch.from_numpy(a).to(gpu_device)  # noqa: E731
    lg = t(logits).requires_grad_(True)
    vv = t(values).requires_grad_(True)
    loss, parts = ppo_loss(lg, vv, t(actions), t(old), t(adv), t(ret))
    loss.backward()
    np.testing.assert_allclose(parts.cpu().numpy(), parts_o, atol=TOL, rtol=0)
    np.testing.assert_allclose(lg.grad.cpu().numpy(), dl_o, atol=1e-7, rtol=1e-4)
    np.testing.assert_allclose(vv.grad.cpu().numpy(), dv_o, atol=1e-7, rtol=1e-5)
