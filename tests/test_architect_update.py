"""ArchitectAgent.update and the Architect reward against the reference's golden vectors.

arch_update.npz holds ArchitectAgent.update (agents/architect.py:91-155) run by the
Python reference on the nets.npz seed-32 ArchitectNetwork: buffered transitions in,
losses out, and per parameter tensor the post-update (clipped) gradient and the
parameter change as norms + fixed random projections.  Tolerance 1e-4 (north star) on
the losses; the gradient / step summaries to 1e-4 relative (fp32 conv backward on a
different device and library); parameters whose gradient is cancellation noise (below
1e-6 of the largest), and every parameter of a case whose value loss is itself rounding
noise, get only Adam's lr bound on their step.  kat.json's architect_reward table pins
calculate_architect_reward (rewards.py:43-73).
"""
import numpy as np
import pytest
import torch

import golden_data as gd
from heist_amd.agents.architect import ArchitectAgent
from heist_amd.rewards import RewardCalculator


def proj_vectors(i, n, k=4):  # tests/golden/make_golden.py:proj_vectors
    return np.random.default_rng(7000 + i).standard_normal((k, n))


def _check_cases(device):
    z = gd.load("arch_update.npz")
    n_sd = gd.load("nets.npz")
    sd = {k[len("architect/"):]: torch.from_numpy(n_sd[k]) for k in n_sd.files if k.startswith("architect/")}
    for ci in range(int(z["n_cases"])):
        ag = ArchitectAgent(grid_rows=20, grid_cols=20, budget=15, device=device)
        ag.network.load_state_dict(sd)
        for ui in range(int(z["c%d_n" % ci])):
            key = "c%d_u%d_" % (ci, ui)
            p0 = [p.detach().clone() for p in ag.network.parameters()]
            ag.log_probs = [torch.tensor(float(x), device=device) for x in z[key + "lp"]]
            ag.values = [torch.tensor([[float(x)]], device=device) for x in z[key + "v"]]
            ag.rewards = []
            ag.store_rewards([float(r) for r in z[key + "r"]])
            m = ag.update(collective=False)
            got = [m["architect_policy_loss"], m["architect_value_loss"], m["architect_total_loss"]]
            np.testing.assert_allclose(got, z[key + "loss"], rtol=1e-4, atol=1e-4, err_msg=key)
            gmax = float(np.max(z[key + "gnorm"]))
            # a case whose value loss is rounding noise (normalised rewards average to 0 and
            # the value head already sits at that target): every gradient is fp32
            # cancellation noise, which Adam (|g| ~ eps) turns into device-dependent steps
            noise_case = float(z[key + "loss"][1]) < 1e-12
            for i, (p, q) in enumerate(zip(ag.network.parameters(), p0)):
                g = (p.grad if p.grad is not None else torch.zeros_like(p)).detach().double().reshape(-1).cpu().numpy()
                d = (p.detach() - q).double().reshape(-1).cpu().numpy()
                P = proj_vectors(i, g.size)
                gscale = max(float(z[key + "gnorm"][i]), 1e-12)
                if noise_case:  # gradients scale with a rounding-noise residual: bounded, not compared
                    assert np.linalg.norm(g) < 1e-6, (key, i)
                    assert np.abs(d).max() <= ag.optimizer.param_groups[0]["lr"] * 3.17, (key, i)
                    continue
                np.testing.assert_allclose(np.linalg.norm(g), z[key + "gnorm"][i], rtol=1e-4, atol=1e-9,
                                           err_msg="%s grad norm %d" % (key, i))
                np.testing.assert_allclose(P @ g, z[key + "gproj"][i], rtol=0, atol=4e-4 * gscale + 1e-9,
                                           err_msg="%s grad proj %d" % (key, i))
                if float(z[key + "gnorm"][i]) < 1e-6 * gmax:
                    # a gradient at fp32 cancellation-noise level (both sides): Adam turns it
                    # into a step of noise, |m_hat / sqrt(v_hat)| <= (1 - b1) / sqrt(1 - b2) per element
                    assert np.abs(d).max() <= ag.optimizer.param_groups[0]["lr"] * 3.17, (key, i)
                    continue
                dscale = max(float(z[key + "dnorm"][i]), 1e-12)
                np.testing.assert_allclose(np.linalg.norm(d), z[key + "dnorm"][i], rtol=1e-3, atol=1e-9,
                                           err_msg="%s step norm %d" % (key, i))
                np.testing.assert_allclose(P @ d, z[key + "dproj"][i], rtol=0, atol=1e-3 * dscale + 1e-9,
                                           err_msg="%s step proj %d" % (key, i))


def test_architect_update_golden_cpu():
    _check_cases(torch.device("cpu"))


@pytest.mark.gpu
def test_architect_update_golden_gpu(gpu_device):
    _check_cases(gpu_device)


def test_architect_reward_kat():
    """calculate_architect_reward (rewards.py:43-73) at the solve rates kat.json holds."""
    table = gd.load_json("kat.json")["architect_reward"]
    rc = RewardCalculator()
    for s, want in table.items():
        assert rc.architect_reward_from_rate(True, float(s)) == want, s
    assert rc.architect_reward_from_rate(False, 0.3) == -1.0


def _sequence_vs_updates(device, ks=(12,)):
    """update_sequence (the per-layout cadence; graph-replayed on a HIP device) equals k
    calls of update() with one transition each (agents/architect.py:91-155, one reward),
    over consecutive sequences of lengths ks on the same agents."""
    torch.manual_seed(5)
    a, b = (ArchitectAgent(grid_rows=12, grid_cols=12, device=device) for _ in range(2))
    b.network.load_state_dict(a.network.state_dict())
    g = torch.Generator().manual_seed(9)
    for k in ks:
        lp, v, r = (torch.randn(k, generator=g, dtype=torch.float64) for _ in range(3))
        for i in range(k):
            b.log_probs.append(torch.tensor(float(lp[i]), device=device))
            b.values.append(torch.tensor(float(v[i]), device=device))
            b.rewards.append(float(r[i]))
            mb = b.update(collective=False)
        ma = a.update_sequence(lp, v, r)
        for key in ("architect_policy_loss", "architect_value_loss", "architect_total_loss"):
            assert abs(ma[key] - mb[key]) < 1e-6, (k, key)
        # parameters: within fp32 noise amplified by Adam (a gradient element at rounding-noise
        # level takes a step of up to lr whatever its size; the graph's backward and capturable
        # Adam round differently from the eager ones: measured max 4.2e-6 = 0.014 lr over 40
        # steps, profiles/r03c_probe_arch_graph.log); exact equality on CPU (both eager)
        tol = 1e-5 if device.type == "cuda" else 1e-6
        for (n, p), q in zip(a.network.state_dict().items(), b.network.state_dict().values()):
            d = float((p - q).abs().max())
            assert d <= tol, (k, n, d)


def test_architect_update_sequence_cpu():
    _sequence_vs_updates(torch.device("cpu"), ks=(12, 5))


@pytest.mark.gpu
def test_architect_update_sequence_gpu_graph(gpu_device):
    # 40: the first capture (1,024 slots); 5: eager only; 1500: past the slots, captured again
    _sequence_vs_updates(gpu_device, ks=(40, 5, 1500))


def _checkpoint_after_sequence_loads_on_cpu(device, tmp_path):
    """A checkpoint written after update_sequence (graph replay: capturable Adam on the
    device) loads into a CPU agent, as the reference's load does (map_location=DEVICE,
    agents/architect.py:165-170), and that agent's update() steps (Adam's capturable-device
    check would fail on a saved capturable=True); the saved state is the live one."""
    torch.manual_seed(3)
    a = ArchitectAgent(grid_rows=12, grid_cols=12, device=device)
    g = torch.Generator().manual_seed(4)
    lp, v, r = (torch.randn(30, generator=g, dtype=torch.float64) for _ in range(3))
    a.update_sequence(lp, v, r)
    path = str(tmp_path / "architect_ep1.pt")
    a.save(path)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert all(not grp.get("capturable", False) for grp in ck["optimizer"]["param_groups"])
    cpu = ArchitectAgent(grid_rows=12, grid_cols=12, device=torch.device("cpu"))
    cpu.load(path)
    for (n, p), q in zip(cpu.network.state_dict().items(), a.network.state_dict().values()):
        assert torch.equal(p, q.cpu()), n
    before = [p.detach().clone() for p in cpu.network.parameters()]
    cpu.log_probs, cpu.values = [torch.tensor(0.1)], [torch.tensor(0.2)]
    cpu.store_reward(0.5)
    cpu.update(collective=False)
    assert any(not torch.equal(p, q) for p, q in zip(cpu.network.parameters(), before))
    # the source agent keeps replaying after a load (its graph dropped and re-captured)
    a.load(path)
    assert getattr(a, "_graph", None) is None
    a.update_sequence(lp[:12], v[:12], r[:12])


def test_architect_checkpoint_after_sequence_cpu(tmp_path):
    _checkpoint_after_sequence_loads_on_cpu(torch.device("cpu"), tmp_path)


@pytest.mark.gpu
def test_architect_checkpoint_after_sequence_gpu(gpu_device, tmp_path):
    _checkpoint_after_sequence_loads_on_cpu(gpu_device, tmp_path)
