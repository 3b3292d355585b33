"""Worker bodies for the multi-process tests (spawned; importable by child processes)."""
import os
import sys

import torch
import torch.distributed as dist


def _init(rank, world, port, backend):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group(backend, rank=rank, world_size=world)


def grads_worker(rank, world, port, out_dir):
    """allreduce_grads: one flat all-reduce averages every parameter's gradient."""
    sys.path[:0] = [p for p in os.environ.get("HEIST_TEST_PATHS", "").split(os.pathsep) if p]
    _init(rank, world, port, "gloo")
    from heist_amd.agents.solver import allreduce_grads
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    x = torch.randn(11, 7) * (rank + 1)
    net(x).square().sum().backward()
    allreduce_grads(list(net.parameters()))
    torch.save([p.grad.clone() for p in net.parameters()], os.path.join(out_dir, "g%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


def advnorm_worker(rank, world, port, out_dir):
    """normalize_advantages across ranks (HIP moments + all-reduce) == global normalisation."""
    sys.path[:0] = [p for p in os.environ.get("HEIST_TEST_PATHS", "").split(os.pathsep) if p]
    _init(rank, world, port, "gloo")
    from heist_amd.ppo import normalize_advantages
    g = torch.Generator().manual_seed(rank)
    x = (torch.randn(1000 + 37 * rank, generator=g) * (rank + 2) + rank).cuda()
    y = normalize_advantages(x)
    torch.save((x.cpu(), y.cpu()), os.path.join(out_dir, "a%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()
