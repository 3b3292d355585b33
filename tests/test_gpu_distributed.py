"""Two ranks sharing the one GPU over gloo: the distributed advantage normalisation
(HIP moments, float64 all-reduce between phases) equals normalising the concatenation."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

import dist_workers

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_global_advantage_normalisation(tmp_path, monkeypatch, gpu_device):
    monkeypatch.setenv("HEIST_TEST_PATHS", os.pathsep.join(sys.path))
    mp.spawn(dist_workers.advnorm_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    x0, y0 = torch.load(tmp_path / "a0.pt")
    x1, y1 = torch.load(tmp_path / "a1.pt")
    x = torch.cat([x0, x1]).double()
    ref = (x - x.mean()) / (x.std() + 1e-8)
    got = torch.cat([y0, y1]).double()
    assert float((got - ref).abs().max()) < 1e-4
