"""Two ranks sharing the one GPU over gloo: the distributed advantage normalisation
(HIP moments, float64 all-reduce between phases) equals normalising the concatenation."""
import json
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


def test_trainer_two_ranks_unequal_shards(tmp_path, monkeypatch, gpu_device):
    """train_iteration x3 on 2 ranks with unequal valid masks, rollout lengths, attempt
    counts and finished-layout counts completes, and leaves both replicas bit-identical."""
    monkeypatch.setenv("HEIST_TEST_PATHS", os.pathsep.join(sys.path))
    mp.spawn(dist_workers.trainer_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    a = torch.load(tmp_path / "t0.pt")
    b = torch.load(tmp_path / "t1.pt")
    for k in ("solver", "architect"):
        assert len(a[k]) == len(b[k])
        for x, y in zip(a[k], b[k]):
            assert torch.equal(x, y), k
    assert a["global_episode"] == b["global_episode"]
    assert not set(a["episodes"]) & set(b["episodes"])  # episode numbers are global
    assert a["scored"] != b["scored"] or sum(a["scored"]) > 0
    # seed=5 on both ranks still gives each rank its own layouts and actions
    assert not torch.equal(a["first_grids"], b["first_grids"])
    assert not torch.equal(a["first_actions"], b["first_actions"])
    logs = json.load(open(tmp_path / "logs" / "game_log.json"))
    assert sorted(e["episode"] for e in logs) == sorted(a["episodes"] + b["episodes"])
