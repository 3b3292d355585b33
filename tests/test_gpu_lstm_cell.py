"""heist_lstm_cell (the rollout's LSTM cell pointwise part, SolverNetwork.lstm_step under
no_grad; reference networks.py:90-100, nn.LSTM one step) against the ten torch kernels it
replaces (the same lstm_step with grad enabled), bit for bit: random gates at several scales
(saturated sigmoids and tanhs, tiny arguments), negative cell states."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,scale", [(1, 1.0), (4097, 3.0), (300, 30.0), (64, 1e-6)])
def test_lstm_cell_matches_torch(gpu_device, n, scale):
    from heist_amd.networks import SolverNetwork
    torch.manual_seed(n)
    net = SolverNetwork().to(gpu_device)
    H = net.lstm_hidden
    with torch.no_grad():
        for p in (net.lstm.weight_ih_l0, net.lstm.weight_hh_l0, net.lstm.bias_ih_l0, net.lstm.bias_hh_l0):
            p.mul_(scale)
    x = torch.randn(n, net.lstm.input_size, device=gpu_device)
    h = torch.randn(1, n, H, device=gpu_device)
    c = torch.randn(1, n, H, device=gpu_device) * 4
    with torch.no_grad():
        h1, (hh, cc) = net.lstm_step(x, (h, c))  # heist_lstm_cell
    with torch.enable_grad():
        h2, (hh2, cc2) = net.lstm_step(x, (h, c))  # the torch kernels
    assert torch.equal(h1, h2.detach()) and torch.equal(cc, cc2.detach())
    assert torch.equal(torch.signbit(h1), torch.signbit(h2.detach()))
