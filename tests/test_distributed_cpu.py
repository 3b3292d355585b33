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
