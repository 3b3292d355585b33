"""heist_rollout_tally (the batched trainer's per-tick attempt bookkeeping, training.py:515-544
per env, and the fresh LSTM state per attempt, :517) against the torch expressions it
replaces, bit for bit: random valid masks, attempt counts around the cap, every status code,
rewards with both signs (the float64 sum), LSTM states with negative entries (h * 0 = -0.0)."""
import pytest
import torch

from heist_amd.vec_env import STATUS_CODES

pytestmark = pytest.mark.gpu


def _torch_tally(valid, attempts, A, done, status, r64, steps, rsum, solve, detect, timeout, h, c):
    vault, det = STATUS_CODES["vault_reached"], STATUS_CODES["detected"]
    counting = valid & (attempts < A)
    steps = steps + counting.int()
    rsum = rsum + torch.where(counting, r64, torch.zeros_like(rsum))
    fin = counting & done
    st = status.to(torch.int32)
    solve = solve + (fin & (st == vault)).int()
    detect = detect + (fin & (st == det)).int()
    timeout = timeout + (fin & (st != vault) & (st != det)).int()
    attempts = attempts + fin.int()
    keep = (~done).to(h.dtype).reshape(1, -1, 1)
    return attempts, steps, rsum, solve, detect, timeout, h * keep, c * keep


@pytest.mark.parametrize("n,hidden", [(1, 128), (4097, 128), (300, 5)])
def test_rollout_tally_matches_torch(gpu_device, n, hidden):
    from heist_amd import _native as nat
    g = torch.Generator().manual_seed(n + hidden)
    dev = gpu_device
    A = 4
    valid = (torch.rand(n, generator=g) < 0.8).to(dev)
    done = (torch.rand(n, generator=g) < 0.4).to(dev)
    status = torch.randint(0, 5, (n,), generator=g, dtype=torch.int8).to(dev)
    r64 = (torch.randn(n, generator=g, dtype=torch.float64) * 3).to(dev)
    ints = [torch.randint(0, 6, (n,), generator=g, dtype=torch.int32).to(dev) for _ in range(5)]  # attempts .. timeout
    steps, solve, detect, timeout = ints[1], ints[2], ints[3], ints[4]
    attempts = ints[0]
    rsum = torch.randn(n, generator=g, dtype=torch.float64).to(dev)
    h = torch.randn(1, n, hidden, generator=g).to(dev)
    c = torch.randn(1, n, hidden, generator=g).to(dev)
    want = _torch_tally(valid, attempts, A, done, status, r64, steps, rsum, solve, detect, timeout, h, c)
    got = [t.clone() for t in (attempts, steps, rsum, solve, detect, timeout, h, c)]
    P = nat.ptr
    nat.check(nat.lib().heist_rollout_tally(P(valid), P(got[0]), A, P(done), P(status), P(r64), P(got[1]), P(got[2]),
                                            P(got[3]), P(got[4]), P(got[5]), P(got[6]), P(got[7]), hidden, n,
                                            nat.stream(dev)), "heist_rollout_tally")
    torch.cuda.synchronize(dev)
    for name, x, y in zip(("attempts", "steps", "reward", "solve", "detect", "timeout", "h", "c"), got, want):
        assert torch.equal(x, y), name
        if x.is_floating_point():  # signed zeros too
            assert torch.equal(torch.signbit(x), torch.signbit(y)), name
