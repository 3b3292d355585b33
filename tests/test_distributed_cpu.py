"""world_size-2 gloo tests of the data-parallel pieces (CPU, no GPU needed)."""
import os
import socket

import torch
import torch.multiprocessing as mp

import dist_workers


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_allreduce_grads_two_ranks(tmp_path, monkeypatch):
    import sys
    monkeypatch.setenv("HEIST_TEST_PATHS", os.pathsep.join(sys.path))
    mp.spawn(dist_workers.grads_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    g0 = torch.load(tmp_path / "g0.pt")
    g1 = torch.load(tmp_path / "g1.pt")
    refs = []
    for rank in range(2):  # each rank's single-process gradient, replayed here
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
        x = torch.randn(11, 7) * (rank + 1)
        net(x).square().sum().backward()
        refs.append([p.grad.clone() for p in net.parameters()])
    for a, b, r0, r1 in zip(g0, g1, *refs):
        assert torch.equal(a, b)  # every rank holds the same averaged gradient
        torch.testing.assert_close(a, (r0 + r1) / 2, rtol=1e-6, atol=1e-6)


def test_weighted_allreduce_grads(tmp_path, monkeypatch):
    import sys
    monkeypatch.setenv("HEIST_TEST_PATHS", os.pathsep.join(sys.path))
    mp.spawn(dist_workers.weighted_grads_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    a = torch.load(tmp_path / "w0.pt")
    b = torch.load(tmp_path / "w1.pt")
    assert a["total"] == b["total"] == 11.0
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    x = torch.randn(11, 7)
    net(x).square().mean().backward()
    for ga, gb, p in zip(a["g"], b["g"], net.parameters()):
        assert torch.equal(ga, gb)
        torch.testing.assert_close(ga, p.grad, rtol=1e-6, atol=1e-7)  # the only contributing rank's mean


def test_architect_update_collective(tmp_path, monkeypatch):
    """Every rank calls ArchitectAgent.update(); the one with no transitions steps too,
    and the step equals a single-process update on the union (agents/architect.py:91-155)."""
    import sys
    monkeypatch.setenv("HEIST_TEST_PATHS", os.pathsep.join(sys.path))
    mp.spawn(dist_workers.architect_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    a = torch.load(tmp_path / "arch0.pt")
    b = torch.load(tmp_path / "arch1.pt")
    for x, y in zip(a["params"], b["params"]):
        assert torch.equal(x, y)
    from heist_amd.agents.architect import ArchitectAgent
    torch.manual_seed(7)
    ag = ArchitectAgent(grid_rows=10, grid_cols=10, device="cpu")
    p0 = [p.detach().clone() for p in ag.network.parameters()]
    ag.store_transitions(torch.tensor([-3.0, -4.0, -5.0]), torch.tensor([0.1, 0.1, 0.1]), [1.0, -1.0, 0.5])
    m = ag.update()
    assert abs(a["m"]["architect_policy_loss"] - m["architect_policy_loss"]) < 1e-5
    assert abs(a["m"]["architect_value_loss"] - m["architect_value_loss"]) < 1e-6
    moved = 0
    for x, y, z in zip(a["params"], ag.network.parameters(), p0):
        torch.testing.assert_close(x, y.detach(), rtol=0, atol=1e-6)
        moved += int(not torch.equal(x, z))
    assert moved > 0
