"""The Solver's fp32 training forward with the split-K weight gradients (networks._linear:
fc_spatial, the LSTM's two gate GEMMs, the heads' first layers; reference networks.py:76-131
trained by agents/solver.py:157-199) against the same forward and backward with plain
F.linear (HEIST_SPLITK_WGRAD=0): outputs bit-identical (the forward is the same GEMM), every
parameter gradient within 1e-5 of its largest entry (only the order of the fp32 sums over
the minibatch rows differs); a ragged row count takes the remainder GEMM."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [4096, 5000])
def test_splitk_wgrad_matches_plain_linear(gpu_device, monkeypatch, n):
    from heist_amd.networks import SolverNetwork
    torch.manual_seed(3)
    net = SolverNetwork().to(gpu_device)
    x = torch.rand(n, 3, 20, 20, device=gpu_device)
    outs, grads = [], []
    for flag in ("1", "0"):
        monkeypatch.setenv("HEIST_SPLITK_WGRAD", flag)
        net.zero_grad(set_to_none=True)
        logits, value, _ = net(x)
        (logits.square().mean() + value.square().mean()).backward()
        outs.append((logits.detach(), value.detach()))
        grads.append({k: p.grad.clone() for k, p in net.named_parameters()})
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    for k in grads[1]:
        a, b = grads[0][k], grads[1][k]
        assert float((a - b).abs().max()) <= 1e-5 * max(float(b.abs().max()), 1e-30), k
