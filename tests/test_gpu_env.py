"""GPU parity of the environment path (heist_set_layout / heist_reset / heist_step /
heist_cones / heist_bfs_valid) against the reference's golden vectors and the C oracle.

Bar: bit-exact.  Integer state, visibility and the float32 observation must match
byte for byte; the float64 reward must match exactly (reward64_out).  The golden
vectors come from the Python reference (tests/golden/make_golden.py); the oracle
(oracle/heist_oracle.c) is pinned to them by tests/test_oracle_golden.py.
"""
import numpy as np
import pytest
import torch

import golden_data as gd
from oracle import pyoracle as po
from heist_amd import EnvironmentConfig, HeistEnv
from heist_amd.layouts import synthetic_layouts, valid_synthetic_layouts

pytestmark = pytest.mark.gpu

STATUS_RESET = 5


def _cfg(tr):
    return EnvironmentConfig(grid_rows=tr["R"], grid_cols=tr["C"], max_steps=tr["max_steps"], start_pos=tr["start"],
                             vault_pos=tr["vault"], architect_budget=tr["budget"])


@pytest.mark.parametrize("path", ["step_kernel", "lean_k1"])
@pytest.mark.parametrize("cones", [True, False], ids=["guard_cones", "live_guards"])
@pytest.mark.parametrize("tr", list(gd.env_traces()), ids=lambda t: t["name"])
def test_golden_trace_bit_exact(tr, cones, path, gpu_device, monkeypatch):
    """Every golden trace on both single-tick paths: the step kernel (HEIST_STEP_LEAN=0) and,
    where the lean K-tick kernel serves the grid (20 x 20 at one wave per env, 32 x 32),
    heist_step as a one-tick heist_step_multi launch (the training rollout's tick)."""
    if path == "lean_k1":
        monkeypatch.setenv("HEIST_MULTI_WAVES", "1")
        monkeypatch.setenv("HEIST_STEP_LEAN", "1")
    else:
        monkeypatch.setenv("HEIST_STEP_LEAN", "0")
    env = HeistEnv(1, _cfg(tr), max_cams=16, max_guards=8, max_path=64, device=gpu_device, auto_reset=False)
    lean_grid = (tr["R"], tr["C"]) in ((20, 20), (32, 32))
    assert env.kernel_config()["step_lean"] == (1 if path == "lean_k1" and lean_grid else 0)
    env.set_guard_cones(cones)
    valid = env.set_layouts([(tr["walls"], tr["cams"], tr["guards"])], budget=tr["budget"])
    assert bool(valid[0]) == tr["valid"]
    st = env.export(grid=True)
    np.testing.assert_array_equal(st["grid"][0].cpu().numpy(), tr["grid"])
    acc = [int(st[k][0]) for k in ("n_walls", "n_cams", "n_guards", "spent")]
    assert acc == tr["accepted"]
    nc, ng = tr["accepted"][1], tr["accepted"][2]
    for k, op in enumerate(tr["ops"]):
        ctx = "%s op#%d" % (tr["name"], k)
        if op == -1:
            obs = env.reset()
            r, d, s = 0.0, None, STATUS_RESET
        else:
            obs, _, dn, stt = env.step(torch.tensor([op]))
            r, d, s = float(env.reward64[0]), bool(dn[0]), int(stt[0])
        st = env.export()
        assert r == tr["reward"][k], ctx
        if d is not None:
            assert d == tr["done"][k], ctx
        assert s == tr["status"][k], ctx
        assert (int(st["pos_r"][0]), int(st["pos_c"][0])) == tuple(tr["pos"][k]), ctx
        assert int(st["tick"][0]) == tr["tick"][k], ctx
        assert bool(st["done"][0]) == tr["done"][k], ctx
        np.testing.assert_array_equal(st["cam_heading"][0, :nc].cpu().numpy(), tr["cam_h"][k], err_msg=ctx)
        np.testing.assert_array_equal(st["guard_idx"][0, :ng].cpu().numpy(), tr["g_idx"][k], err_msg=ctx)
        np.testing.assert_array_equal(st["guard_heading"][0, :ng].cpu().numpy(), tr["g_h"][k], err_msg=ctx)
        o = obs[0].cpu().numpy()
        np.testing.assert_array_equal(o[1] > 0.5, tr["vis"][k], err_msg=ctx)
        if k < len(tr["state"]):
            assert o.tobytes() == tr["state"][k].tobytes(), ctx


def test_cones_bit_exact(gpu_device):
    groups = {}
    for c in gd.cones():
        groups.setdefault((c["R"], c["C"]), []).append(c)
    n = 0
    for (R, C), cs in groups.items():
        walls = torch.tensor(np.stack([c["walls"] for c in cs]).astype(np.uint8), device=gpu_device)
        meta = torch.tensor([[1 if c["kind"] == 2 else 0, c["row"], c["col"], c["range"]] for c in cs],
                            dtype=torch.int32, device=gpu_device)
        par = torch.tensor([[c["fov"], c["heading"]] for c in cs], dtype=torch.float64, device=gpu_device)
        out = torch.empty((len(cs), R, C), dtype=torch.uint8, device=gpu_device)
        from heist_amd import _native as nat
        nat.check(nat.lib().heist_cones(len(cs), R, C, nat.ptr(walls), nat.ptr(meta), nat.ptr(par), nat.ptr(out),
                                        nat.stream(gpu_device)), "heist_cones")
        got = out.bool().cpu().numpy()
        for i, c in enumerate(cs):
            np.testing.assert_array_equal(got[i], c["tiles"], err_msg=str((c["kind"], c["fov"], c["heading"])))
            n += 1
    assert n >= 1000


def test_cone_order_matches_reference_list(gpu_device):
    """heist_cone_order first-visit keys give get_vision_cone_tiles / get_visible_tiles'
    list order (security.py:53-101, :161-192) on 600 reference-generated cases, through
    the component classes (batched ABI call for each grid size, then the class methods)."""
    from heist_amd import _native as nat
    from heist_amd.components.security import Camera, Guard
    groups = {}
    for c in gd.cone_orders():
        groups.setdefault((c["R"], c["C"]), []).append(c)
    n = 0
    for (R, C), cs in groups.items():
        walls = torch.tensor(np.stack([c["walls"] for c in cs]).astype(np.uint8), device=gpu_device)
        meta = torch.tensor([[c["kind"], c["row"], c["col"], c["range"]] for c in cs], dtype=torch.int32,
                            device=gpu_device)
        par = torch.tensor([[c["fov"], c["heading"]] for c in cs], dtype=torch.float64, device=gpu_device)
        keys = torch.empty((len(cs), R, C), dtype=torch.int32, device=gpu_device)
        nat.check(nat.lib().heist_cone_order(len(cs), R, C, nat.ptr(walls), nat.ptr(meta), nat.ptr(par),
                                             nat.ptr(keys), nat.stream(gpu_device)), "heist_cone_order")
        k = keys.cpu().numpy().view(np.uint32).reshape(len(cs), -1)
        for i, c in enumerate(cs):
            hit = np.nonzero(k[i] != 0xFFFFFFFF)[0]
            got = [(int(j) // C, int(j) % C) for j in hit[np.argsort(k[i][hit], kind="stable")]]
            assert got == c["order"], (c["kind"], c["fov"], c["heading"])
            n += 1
    assert n == 600
    for c in list(gd.cone_orders())[:30]:  # the class methods return the same lists
        if c["kind"] == 0:
            got = Camera(row=c["row"], col=c["col"], fov_angle=c["fov"], heading=c["heading"],
                         vision_range=c["range"]).get_vision_cone_tiles(c["R"], c["C"], c["walls"])
        else:
            got = Guard(patrol_path=[(c["row"], c["col"])], vision_range=c["range"], fov_angle=c["fov"],
                        heading=c["heading"]).get_visible_tiles(c["R"], c["C"], c["walls"])
        assert got == c["order"]


def test_bfs_bit_exact(gpu_device):
    from heist_amd.utils import bfs_valid_batch
    groups = {}
    for c in gd.bfs_cases():
        key = (c["grid"].shape, c["start"], c["goal"])
        groups.setdefault(key, []).append(c)
    n = 0
    for (shape, start, goal), cs in groups.items():
        g = torch.tensor(np.stack([c["grid"] for c in cs]).astype(np.int32), device=gpu_device)
        got = bfs_valid_batch(g, start, goal).cpu().numpy()
        np.testing.assert_array_equal(got, np.array([c["valid"] for c in cs]))
        n += len(cs)
    assert n >= 1000


def _oracle_envs(cfg, layouts, budget):
    envs = []
    for lay in layouts:
        o = po.OracleEnv(cfg.grid_rows, cfg.grid_cols, cfg.max_steps, cfg.start_pos, cfg.vault_pos, budget)
        o.set_layout(*lay)
        o.reset()
        envs.append(o)
    return envs


@pytest.mark.parametrize("R,C,budget,n,T", [(20, 20, 15, 192, 260), (32, 32, 40, 64, 120), (13, 17, 25, 64, 150),
                                             (64, 64, 60, 16, 80), (6, 48, 12, 32, 80)])
def test_batched_auto_reset_vs_oracle(R, C, budget, n, T, gpu_device):
    """Every env of a batch, with in-kernel auto-reset, equals its own oracle replay."""
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=C, max_steps=60 if R != 20 else 200)
    env = HeistEnv(n, cfg, max_cams=24, max_guards=12, max_path=16, device=gpu_device, auto_reset=True)
    lays = synthetic_layouts(n, R, C, budget, seed=R * 1000 + C)
    env.set_layouts(lays, budget=budget)
    obs = env.reset().cpu().numpy()
    oracles = _oracle_envs(cfg, lays, budget)
    for i, o in enumerate(oracles):
        assert obs[i].tobytes() == o.state_tensor().tobytes()
    rng = np.random.default_rng(7)
    for t in range(T):
        acts = rng.integers(0, 5, n)
        acts[rng.random(n) < 0.4] = rng.choice([2, 4])
        obs, rew, done, status = env.step(torch.from_numpy(acts))
        obs, r64, done, status = (x.cpu().numpy() for x in (obs, env.reward64, done, status))
        for i, o in enumerate(oracles):
            r, d, s = o.step(int(acts[i]))
            if d:
                o.reset()
            assert (r64[i], bool(done[i]), int(status[i])) == (r, d, s), "env %d t %d" % (i, t)
            assert obs[i].tobytes() == o.state_tensor().tobytes(), "env %d t %d" % (i, t)


def test_full_size_sampled_vs_oracle(gpu_device):
    """BASELINE config size (4096 envs, 20x20): a sample of envs matches the oracle exactly
    and batch-wide invariants hold for every env."""
    n, R = 4096, 20
    cfg = EnvironmentConfig()
    env = HeistEnv(n, cfg, device=gpu_device)
    lays = valid_synthetic_layouts(env, 15, seed=1234)
    assert bool(env.valid.bool().all())
    env.reset()
    pick = np.random.default_rng(3).choice(n, 48, replace=False)
    oracles = _oracle_envs(cfg, [lays[i] for i in pick], 15)
    grid = env.export(grid=True)["grid"].float() / 5.0
    g = torch.Generator(device="cpu").manual_seed(11)
    for t in range(120):
        acts = torch.randint(0, 5, (n,), generator=g)
        obs, rew, done, status = env.step(acts)
        assert torch.equal(obs[:, 0], grid)  # occupancy channel is static
        assert bool(((obs[:, 1] == 0) | (obs[:, 1] == 1)).all())
        o_np = obs[torch.from_numpy(pick).to(gpu_device)].cpu().numpy()
        r64 = env.reward64.cpu().numpy()
        for j, i in enumerate(pick):
            r, d, s = oracles[j].step(int(acts[i]))
            if d:
                oracles[j].reset()
            assert r64[i] == r
            assert o_np[j].tobytes() == oracles[j].state_tensor().tobytes()


@pytest.mark.parametrize("step_lean", [0, 1], ids=["step_kernel", "lean_k1"])
def test_full_size_c2_checkpoint_layouts_vs_oracle(gpu_device, monkeypatch, step_lean):
    """The bench's headline workload (BASELINE config 2: 4096 envs, 20x20, layouts sampled
    from checkpoints/architect_c2_fixed.pt at T = 1.0, budget 15): 48 envs replayed through
    the oracle for 120 ticks with auto-reset, bit-exact, and batch-wide invariants for all;
    heist_step on the single-tick step kernel and as a one-tick launch of the lean K-tick
    kernel (HEIST_STEP_LEAN=1)."""
    monkeypatch.setenv("HEIST_STEP_LEAN", str(step_lean))
    import os
    from heist_amd.layouts import architect_checkpoint_layouts
    from heist_amd.training import _lb_rows
    ckpt = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "checkpoints",
                        "architect_c2_fixed.pt")
    n, budget = 4096, 15
    cfg = EnvironmentConfig(architect_budget=budget)
    env = HeistEnv(n, cfg, max_cams=5, max_guards=3, max_path=16, device=gpu_device)
    assert env.kernel_config()["step_lean"] == step_lean
    lb, all_valid = architect_checkpoint_layouts(env, budget, seed=1234, ckpt=ckpt)
    assert all_valid
    env.reset()
    st = env.export(grid=True)
    assert float(st["n_cams"].double().mean()) > 1.0 and int(st["n_guards"].max()) >= 1
    pick = np.random.default_rng(5).choice(n, 48, replace=False)
    lays = _lb_rows(lb, pick).to_lists()
    oracles = _oracle_envs(cfg, lays, budget)
    grid = st["grid"].float() / 5.0
    g = torch.Generator(device="cpu").manual_seed(12)
    for t in range(120):
        acts = torch.randint(0, 5, (n,), generator=g)
        obs, rew, done, status = env.step(acts)
        assert torch.equal(obs[:, 0], grid)
        o_np = obs[torch.from_numpy(pick).to(gpu_device)].cpu().numpy()
        r64, dn, stt = (x.cpu().numpy() for x in (env.reward64, done, status))
        for j, i in enumerate(pick):
            r, d, s = oracles[j].step(int(acts[i]))
            if d:
                oracles[j].reset()
            assert (r64[i], bool(dn[i]), int(stt[i])) == (r, d, s), "env %d t %d" % (i, t)
            assert o_np[j].tobytes() == oracles[j].state_tensor().tobytes(), "env %d t %d" % (i, t)


def test_step_after_done_without_auto_reset(gpu_device):
    cfg = EnvironmentConfig(grid_rows=6, grid_cols=6, max_steps=3)
    env = HeistEnv(2, cfg, device=gpu_device, auto_reset=False)
    env.set_layouts([([], [], []), ([], [], [])])
    env.reset()
    for _ in range(3):
        env.step(torch.zeros(2, dtype=torch.int64))
    obs_before = env.obs.clone()
    _, rew, done, status = env.step(torch.zeros(2, dtype=torch.int64))
    assert bool(done.all()) and (status == 4).all() and float(rew.abs().sum()) == 0.0
    assert torch.equal(env.obs, obs_before)


def test_step_stamps_instrumentation(gpu_device):
    """heist_step_stamps: the stamped kernel variant gives the same results as the plain
    one, every wave records 8 non-decreasing clock stamps, and HW_ID / XCC_ID are filled."""
    from heist_amd import _native as nat
    n = 256
    cfg = EnvironmentConfig()
    lays = synthetic_layouts(n, 20, 20, 15, seed=31)
    envs = [HeistEnv(n, cfg, device=gpu_device) for _ in range(2)]
    for e in envs:
        e.set_layouts(lays, budget=15)
        e.reset()
    w = nat.lib().heist_step_waves(envs[0]._h)
    assert w in (1, 2, 4)
    buf = torch.zeros((n, w, 10), dtype=torch.int64, device=gpu_device)
    g = torch.Generator(device="cpu").manual_seed(3)
    for t in range(20):
        a = torch.randint(0, 5, (n,), generator=g)
        nat.check(nat.lib().heist_step_stamps(envs[0]._h, nat.ptr(buf), buf.numel()), "heist_step_stamps")
        r0 = envs[0].step(a)
        nat.check(nat.lib().heist_step_stamps(envs[0]._h, None, 0), "heist_step_stamps")
        r1 = envs[1].step(a)
        for x, y in zip(r0, r1):
            assert torch.equal(x, y), t
    s = buf.cpu().numpy()
    assert (s[:, :, :8] > 0).all()
    assert (np.diff(s[:, :, :8], axis=2) >= 0).all()
    assert (s[:, :, 8] != 0).any()
    # a buffer too small for the kernel a call runs is refused, not overrun
    L = nat.lib()
    need0, need1 = L.heist_stamp_words(envs[0]._h, 0), L.heist_stamp_words(envs[0]._h, 1)
    assert need0 == n * 10 * w and need1 == n * 16 * envs[0].kernel_config()["multi_waves"]
    small = torch.zeros(min(need0, need1) - 1, dtype=torch.int64, device=gpu_device)
    nat.check(L.heist_step_stamps(envs[0]._h, nat.ptr(small), small.numel()), "heist_step_stamps")
    acts = torch.zeros((2, n), dtype=torch.int64, device=gpu_device)
    with pytest.raises(nat.HeistError):
        envs[0].step_multi(acts)
    with pytest.raises(nat.HeistError):
        envs[0].step(acts[0])
    nat.check(L.heist_step_stamps(envs[0]._h, None, 0), "heist_step_stamps")
    envs[0].step_multi(acts)


@pytest.mark.parametrize("R", [20, 32])
def test_step_multi_stamps_lean(gpu_device, R):
    """heist_step_stamps on the K-tick path: the stamped step_lean_kernel instance gives the
    same results as the plain one, and each env's per-segment cycle sums (words 0..8) add up
    to no more than its lifetime (word 9)."""
    from heist_amd import _native as nat
    n, K = 512, 8
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R)
    lays = synthetic_layouts(n, R, R, 15, seed=5)
    envs = [HeistEnv(n, cfg, device=gpu_device) for _ in range(2)]
    for e in envs:
        e.set_layouts(lays, budget=15)
        e.reset()
    kc = envs[0].kernel_config()
    if not kc["lean"]:
        pytest.skip("lean K-tick kernel disabled")
    W = kc["multi_waves"]
    L = nat.lib()
    words = max(int(L.heist_stamp_words(envs[0]._h, 0)), int(L.heist_stamp_words(envs[0]._h, 1)))
    buf = torch.zeros(words, dtype=torch.int64, device=gpu_device)
    g = torch.Generator(device="cpu").manual_seed(9)
    for it in range(3):
        acts = torch.randint(0, 5, (K, n), generator=g).to(gpu_device)
        nat.check(L.heist_step_stamps(envs[0]._h, nat.ptr(buf), buf.numel()), "heist_step_stamps")
        r0 = envs[0].step_multi(acts, reward64=True)
        nat.check(L.heist_step_stamps(envs[0]._h, None, 0), "heist_step_stamps")
        r1 = envs[1].step_multi(acts, reward64=True)
        for x, y in zip(r0, r1):
            assert torch.equal(x, y), it
    s = buf[:n * W * 16].reshape(n, W, 16)[:, 0].cpu().numpy()
    assert (s[:, :9] >= 0).all() and (s[:, 9] > 0).all()
    assert (s[:, :9].sum(axis=1) <= s[:, 9]).all()
    assert (s[:, 2] > 0).any() and (s[:, 7] > 0).all()


@pytest.mark.parametrize("cones", [False, True], ids=["live_guards", "guard_cones"])
def test_sample_counter_work_figure(cones, gpu_device):
    """heist_count_samples: an unobstructed camera ray evaluates all 2*range samples, a guard
    ray all range samples (none with the guard cone cache); counting leaves the results
    unchanged."""
    cfg = EnvironmentConfig()
    fov = 60.0
    lay = ([], [{"row": 10, "col": 10, "fov_angle": fov, "heading": 0.0, "rotation_speed": 15.0,
                 "vision_range": 6}],
           [{"patrol_path": [(5, 5), (5, 6)], "speed": 1, "vision_range": 4, "fov_angle": 90.0}])
    envs = [HeistEnv(2, cfg, device=gpu_device) for _ in range(2)]
    for e in envs:
        e.set_guard_cones(cones)
        e.set_layouts([lay, lay], budget=40)
    cnt = torch.zeros(2, dtype=torch.int64, device=gpu_device)
    envs[0].count_samples(cnt)
    per_pass = (max(int(fov * 2), 30) + 1) * 12 + (0 if cones else (max(int(90.0 * 2), 30) + 1) * 4)
    outs = []
    for e in envs:
        e.reset()
        seq = [e.obs.clone()]
        for _ in range(3):
            obs, _, done, _ = e.step(torch.tensor([0, 4]))
            assert not bool(done.any())  # no auto-reset pass in the count
            seq.append(obs.clone())
        outs.append(seq)
    assert cnt.tolist() == [4 * per_pass] * 2
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    envs[0].count_samples(None)
    envs[0].step(torch.tensor([0, 0]))
    assert cnt.tolist() == [4 * per_pass] * 2


# --- fp32 fast raycast vs exact fp64 raycast ------------------------------------------

def _fast_dir(deg, dev):
    from heist_amd import _native as nat
    x = torch.as_tensor(deg, dtype=torch.float64, device=dev).contiguous()
    co = torch.empty(x.numel(), dtype=torch.float32, device=dev)
    so = torch.empty_like(co)
    nat.check(nat.lib().heist_fast_dir(nat.ptr(x), x.numel(), nat.ptr(co), nat.ptr(so), nat.stream(dev)),
              "heist_fast_dir")
    return co, so


def _exact_dir(deg, dev):
    from heist_amd import _native as nat
    rad = torch.as_tensor(deg, dtype=torch.float64, device=dev) * (np.pi / 180.0)  # math.radians
    rad = rad.contiguous()
    so = torch.empty_like(rad)
    co = torch.empty_like(rad)
    nat.check(nat.lib().heist_sincos(nat.ptr(rad), rad.numel(), nat.ptr(so), nat.ptr(co), nat.stream(dev)),
              "heist_sincos")
    return co, so


def test_fast_direction_error(gpu_device):
    """The fast path's fp32 direction is within 3e-7 of the exact (glibc) one; the near-tie
    screen assumes kDirErr = 1e-6, so this keeps a >3x margin."""
    rng = np.random.default_rng(0)
    deg = np.concatenate([
        rng.uniform(-200.0, 560.0, 4_000_000),
        np.arange(-180.0, 540.0, 0.25),                                   # integer / quarter headings
        (np.arange(-8, 13)[:, None] * 45.0 + rng.uniform(-1e-3, 1e-3, (21, 2000))).ravel(),  # octant edges
        rng.uniform(0, 360, 200_000).astype(np.float32).astype(np.float64),  # f32 Architect params
    ])
    cf, sf = _fast_dir(deg, gpu_device)
    ce, se = _exact_dir(deg, gpu_device)
    err = max(float((cf.double() - ce).abs().max()), float((sf.double() - se).abs().max()))
    assert err < 3e-7, err


def _cones(n, R, C, walls, meta, par, mode, dev):
    from heist_amd import _native as nat
    out = torch.empty((n, R, C), dtype=torch.uint8, device=dev)
    nat.check(nat.lib().heist_cones_mode(n, R, C, nat.ptr(walls), nat.ptr(meta), nat.ptr(par), mode, nat.ptr(out),
                                         nat.stream(dev)), "heist_cones_mode")
    return out


@pytest.mark.parametrize("R,C", [(20, 20), (32, 32), (64, 64), (9, 23)])
def test_cones_fast_equals_exact(R, C, gpu_device):
    """heist_cones_mode 0 (fp32 fast + exact re-cast) == mode 1 (exact fp64) bit for bit on
    random emitters, including exact-tie headings (integer and half degrees, the reference's
    defaults), ranges above the fast path's limit, and random wall maps."""
    rng = np.random.default_rng(R * 100 + C)
    n = 20000
    walls = (rng.random((n, R, C)) < rng.uniform(0.0, 0.35, (n, 1, 1))).astype(np.uint8)
    kind = rng.integers(0, 2, n)
    row = rng.integers(0, R, n)
    col = rng.integers(0, C, n)
    rng_ = np.where(rng.random(n) < 0.9, np.where(kind == 0, 6, 4), rng.integers(1, 12, n))
    fov = np.where(rng.random(n) < 0.3, rng.choice([30.0, 45.0, 60.0, 90.0, 120.0], n),
                   rng.uniform(30.0, 120.0, n).astype(np.float32).astype(np.float64))
    head = np.select([rng.random(n) < 0.3, rng.random(n) < 0.5],
                     [rng.integers(0, 72, n) * 5.0, rng.integers(0, 720, n) * 0.5],
                     rng.uniform(0.0, 360.0, n).astype(np.float32).astype(np.float64))
    # axis-grazing rays: fov 60 puts ray 60 of 120 exactly on the heading, which sits within
    # 1e-12 .. 1e-2 degrees of a multiple of 90 (cos or sin within ~1e-20 .. 1e-8 of +-1)
    graze = rng.random(n) < 0.25
    tiny = 10.0 ** rng.uniform(-12, -2, n) * rng.choice([-1.0, 1.0], n)
    head = np.where(graze, rng.integers(0, 5, n) * 90.0 + tiny, head)
    fov = np.where(graze, 60.0, fov)
    walls[np.arange(n), row, col] = 0
    dev = gpu_device
    wt = torch.tensor(walls, device=dev)
    meta = torch.tensor(np.stack([kind, row, col, rng_], 1).astype(np.int32), device=dev)
    par = torch.tensor(np.stack([fov, head], 1), dtype=torch.float64, device=dev)
    fast = _cones(n, R, C, wt, meta, par, 0, dev)
    exact = _cones(n, R, C, wt, meta, par, 1, dev)
    bad = (fast != exact).flatten(1).any(1).nonzero().flatten().tolist()
    assert not bad, [(int(kind[i]), int(row[i]), int(col[i]), int(rng_[i]), fov[i], head[i]) for i in bad[:5]]


def test_step_fast_equals_exact_and_redo_rate(gpu_device):
    """Three handles on the same layouts: fast raycast (mode 0) with the guard cone cache,
    fast with live guards, and exact (mode 1) with live guards: every observation, reward
    and status is identical over 150 ticks with auto-reset.  Synthetic (f32-random)
    headings re-cast only a small fraction of rays exactly; the reference's default
    cameras (heading 0, fov 60, speed 15: half-degree ray angles) re-cast many."""
    n = 1024
    cfg = EnvironmentConfig()
    lays = synthetic_layouts(n - 64, 20, 20, 15, seed=77)
    cam = {"row": 10, "col": 10, "fov_angle": 60.0, "heading": 0.0, "rotation_speed": 15.0, "vision_range": 6}
    for k in range(64):
        c = dict(cam, row=3 + k % 14, col=2 + (k * 7) % 15)
        lays.append(([(5, 5 + k % 10)], [c], [{"patrol_path": [(15, 3), (15, 4), (14, 4)], "speed": 1,
                                                 "vision_range": 4, "fov_angle": 90.0}]))
    envs = [HeistEnv(n, cfg, device=gpu_device) for _ in range(3)]
    envs[1].set_ray_mode(1)
    envs[1].set_guard_cones(False)
    envs[2].set_guard_cones(False)
    envs = [envs[2], envs[1], envs[0]]  # [fast live, exact live, fast cached]
    cnt = [torch.zeros(n, dtype=torch.int64, device=gpu_device) for _ in range(2)]
    for e in envs:
        e.set_layouts(lays, budget=15)
    for e, c in zip(envs, cnt):
        e.count_exact_rays(c)
    o = [e.reset() for e in envs]
    assert torch.equal(o[0], o[1]) and torch.equal(o[0], o[2])
    cnt_s = [torch.zeros(n, dtype=torch.int64, device=gpu_device) for _ in range(2)]
    envs[0].count_samples(cnt_s[0])
    envs[1].count_samples(cnt_s[1])
    g = torch.Generator(device="cpu").manual_seed(5)
    for t in range(150):
        a = torch.randint(0, 5, (n,), generator=g)
        r = [e.step(a) for e in envs]
        for k in (1, 2):
            for x, y in zip(r[0], r[k]):
                assert torch.equal(x, y), (t, k)
            assert torch.equal(envs[0].reward64, envs[k].reward64), (t, k)
    assert torch.equal(cnt_s[0], cnt_s[1])
    exact_all = cnt[1].double()
    frac_syn = float(cnt[0][: n - 64].sum()) / float(exact_all[: n - 64].sum())
    frac_def = float(cnt[0][n - 64:].sum()) / float(exact_all[n - 64:].sum())
    assert frac_syn < 0.01, frac_syn
    assert frac_def > frac_syn, (frac_def, frac_syn)
    for e in envs:
        e.count_exact_rays(None)
        e.count_samples(None)


def _guard_variety_layouts(n, R, rng):
    """Guards of every shape the cone cache must handle or refuse: Architect rings, long
    diagonal patrols with more than 8 distinct move headings (not cached), speeds 0..3 and
    negative, duplicate points, single points, ranges 1..9 (above 7: not cached), fovs
    30..200, plus a camera or two."""
    lays = []
    for i in range(n):
        guards = []
        for _ in range(int(rng.integers(1, 5))):
            kind = int(rng.integers(0, 5))
            r0, c0 = int(rng.integers(1, R - 1)), int(rng.integers(1, R - 1))
            if kind == 0:
                from heist_amd.layouts import architect_patrol
                path = architect_patrol(r0, c0, R, R)
            elif kind == 1:  # random walk with diagonal and long moves
                path = [(r0, c0)]
                for _ in range(int(rng.integers(2, 20))):
                    r0 = int(np.clip(r0 + rng.integers(-2, 3), 0, R - 1))
                    c0 = int(np.clip(c0 + rng.integers(-2, 3), 0, R - 1))
                    path.append((r0, c0))
            elif kind == 2:
                path = [(r0, c0)]
            elif kind == 3:  # back and forth with duplicates
                path = [(r0, c0), (r0, c0), (r0, min(c0 + 1, R - 2)), (r0, min(c0 + 1, R - 2))]
            else:
                path = [(int(rng.integers(0, R)), int(rng.integers(0, R))) for _ in range(int(rng.integers(2, 9)))]
            guards.append({"patrol_path": path, "speed": int(rng.choice([1, 1, 1, 2, 3, -1, 0])),
                           "vision_range": int(rng.choice([4, 4, 4, 1, 3, 7, 8, 9])),
                           "fov_angle": float(rng.choice([90.0, 90.0, 30.0, 120.0, 200.0,
                                                          float(np.float32(rng.uniform(30, 180)))]))})
        cams = [{"row": int(rng.integers(1, R - 1)), "col": int(rng.integers(1, R - 1)),
                 "fov_angle": float(np.float32(rng.uniform(30, 120))), "heading": float(np.float32(rng.uniform(0, 360))),
                 "rotation_speed": float(np.float32(rng.uniform(5, 35))), "vision_range": 6}
                for _ in range(int(rng.integers(0, 3)))]
        walls = [(int(rng.integers(1, R - 1)), int(rng.integers(1, R - 1))) for _ in range(int(rng.integers(0, 25)))]
        lays.append((walls, cams, guards))
    return lays


@pytest.mark.parametrize("R", [12, 20, 32])
def test_guard_cone_cache_equals_live_raycast(R, gpu_device):
    """The guard cone cache (heist_set_guard_cones) against live raycasting and the C
    oracle: same observations, rewards, statuses and guard headings over 200 ticks with
    auto-reset, on guards the cache takes and guards it must refuse."""
    n = 512
    rng = np.random.default_rng(R)
    lays = _guard_variety_layouts(n, R, rng)
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R, max_steps=60)
    envs = [HeistEnv(n, cfg, max_cams=2, max_guards=4, max_path=24, device=gpu_device) for _ in range(2)]
    envs[1].set_guard_cones(False)
    for e in envs:
        e.set_layouts(lays, budget=60)
    o = [e.reset() for e in envs]
    assert torch.equal(o[0], o[1])
    sample = rng.choice(n, 24, replace=False)
    oracles = []
    for i in sample:
        ob = po.OracleEnv(R, R, 60, (1, 1), (R - 2, R - 2), 60)
        ob.set_layout(*lays[i])
        ob.reset()
        oracles.append(ob)
    g = torch.Generator(device="cpu").manual_seed(R)
    for t in range(200):
        a = torch.randint(0, 5, (n,), generator=g)
        r = [e.step(a) for e in envs]
        for x, y in zip(r[0], r[1]):
            assert torch.equal(x, y), t
        assert torch.equal(envs[0].reward64, envs[1].reward64), t
        obs = r[0][0].cpu().numpy()
        r64 = envs[0].reward64.cpu().numpy()
        for i, ob in zip(sample, oracles):
            rr, d, _ = ob.step(int(a[i]))
            if d:
                ob.reset()
            assert r64[i] == rr, (t, i)
            assert obs[i].tobytes() == ob.state_tensor().tobytes(), (t, i)
    s0, s1 = envs[0].export(), envs[1].export()
    assert torch.equal(s0["guard_idx"], s1["guard_idx"]) and torch.equal(s0["guard_heading"], s1["guard_heading"])


@pytest.mark.parametrize("R,n", [(20, 4096), (20, 256), (32, 512)])
def test_observation_store_forms_agree(R, n, gpu_device, monkeypatch):
    """The observation write's forms (handle knobs read at heist_create): non-temporal
    stores with channels 0/2 written before the raycast (the default), plain stores in one
    piece after it, write-through (sc1) and sc1+nt stores, give byte-identical observations,
    rewards and statuses over 80 ticks with auto-reset.  n = 256 runs 4 waves per env (the
    pre-raycast writers are waves 1-3), n = 4096 two."""
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R)
    lays = synthetic_layouts(n, R, R, 15 if R == 20 else 40, seed=300 + R + n)
    envs = []
    for store, split in ((2, 1), (0, 0), (1, 1), (3, 0), (0, 1)):
        monkeypatch.setenv("HEIST_OBS_STORE", str(store))
        monkeypatch.setenv("HEIST_SPLIT_OBS", str(split))
        e = HeistEnv(n, cfg, max_cams=16, max_guards=8, max_path=16, device=gpu_device)
        e.set_layouts(lays, budget=15 if R == 20 else 40)
        envs.append(e)
    o = [e.reset() for e in envs]
    for k in range(1, len(envs)):
        assert torch.equal(o[0], o[k]), k
    g = torch.Generator(device="cpu").manual_seed(R + n)
    for t in range(80):
        a = torch.randint(0, 5, (n,), generator=g)
        r = [e.step(a) for e in envs]
        for k in range(1, len(envs)):
            for x, y in zip(r[0], r[k]):
                assert torch.equal(x, y), (t, k)
            assert torch.equal(envs[0].reward64, envs[k].reward64), (t, k)


def _step_kernel_env(*args, **kw):
    """A handle whose heist_step runs the single-tick step kernel (HEIST_STEP_LEAN=0), the
    independent reference of the K-tick comparisons (else heist_step is itself a one-tick
    launch of the lean K-tick kernel wherever that kernel serves the handle)."""
    import os
    os.environ["HEIST_STEP_LEAN"] = "0"
    try:
        env = HeistEnv(*args, **kw)
    finally:
        del os.environ["HEIST_STEP_LEAN"]
    assert env.kernel_config()["step_lean"] == 0
    return env


def _twin_envs(n, cfg, lays, budget, gpu_device, cones=True, **kw):
    envs = []
    for i in range(2):
        env = (HeistEnv if i == 0 else _step_kernel_env)(n, cfg, device=gpu_device, **kw)
        env.set_guard_cones(cones)
        v = env.set_layouts(lays, budget=budget)
        env.reset()
        envs.append((env, v.clone()))
    assert torch.equal(envs[0][1], envs[1][1])
    return envs[0][0], envs[1][0]


def _compare_multi_vs_single(a, b, acts, chunks, auto_reset=True):
    """env a: heist_step_multi over `chunks` (tick counts per launch); env b: one heist_step
    per tick.  Every tick's obs, float64 reward, done and status must be bit-identical,
    and so must the state both end in."""
    k0 = 0
    for K in chunks:
        obs, rew, done, status, r64 = a.step_multi(acts[k0:k0 + K], auto_reset=auto_reset, reward64=True)
        for k in range(K):
            o, r, d, s = b.step(acts[k0 + k], auto_reset=auto_reset)
            ctx = "tick %d" % (k0 + k)
            assert torch.equal(obs[k], o), ctx
            assert torch.equal(r64[k], b.reward64), ctx
            assert torch.equal(rew[k], r), ctx
            assert torch.equal(done[k], d), ctx
            assert torch.equal(status[k], s), ctx
        k0 += K
    sa, sb = a.export(grid=True), b.export(grid=True)
    for key in sb:
        assert torch.equal(sa[key], sb[key]), key


@pytest.mark.parametrize("cones", [True, False], ids=["guard_cones", "live_guards"])
@pytest.mark.parametrize("auto_reset", [True, False], ids=["auto_reset", "no_reset"])
def test_step_multi_equals_single_steps(gpu_device, cones, auto_reset):
    """heist_step_multi (K ticks per launch, state on chip) == K heist_step launches, bit for
    bit, over 60 ticks in launches of 1, 17 and 42 ticks, with short episodes (max_steps
    25) so that timeouts, detections and auto-resets with guards off their start happen
    inside a launch."""
    n, R = 512, 20
    cfg = EnvironmentConfig(max_steps=25)
    lays = synthetic_layouts(n, R, R, 15, seed=61)
    a, b = _twin_envs(n, cfg, lays, 15, gpu_device, cones=cones)
    g = torch.Generator(device="cpu").manual_seed(62)
    acts = torch.randint(0, 5, (60, n), generator=g).to(gpu_device)
    acts[::7, ::3] = 7  # out-of-range actions do not move
    _compare_multi_vs_single(a, b, acts, [1, 17, 42], auto_reset=auto_reset)


def test_step_multi_c5_32x32_four_waves(gpu_device):
    """BASELINE config 5 geometry (32x32, 4 cameras + 3 guards, 2048 envs: 4 waves per env)."""
    n, R = 2048, 32
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R, max_steps=40, architect_budget=40)
    lays = synthetic_layouts(n, R, R, 40, seed=63, n_cams=4, n_guards=3)
    a, b = _twin_envs(n, cfg, lays, 40, gpu_device, max_cams=13, max_guards=8)
    assert a.kernel_config()["step_waves"] in (2, 4)
    g = torch.Generator(device="cpu").manual_seed(64)
    acts = torch.randint(0, 5, (50, n), generator=g).to(gpu_device)
    _compare_multi_vs_single(a, b, acts, [50])


def test_step_multi_c2_checkpoint_layouts(gpu_device):
    """The headline workload (4096 envs, C2 checkpoint layouts): K-tick launches == single
    ticks, plus 32 envs replayed through the oracle."""
    import os
    from heist_amd.layouts import architect_checkpoint_layouts
    from heist_amd.training import _lb_rows
    ckpt = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "checkpoints",
                        "architect_c2_fixed.pt")
    n, budget = 4096, 15
    cfg = EnvironmentConfig(architect_budget=budget)
    envs = []
    for _ in range(2):
        env = HeistEnv(n, cfg, max_cams=5, max_guards=3, max_path=16, device=gpu_device)
        lb, ok = architect_checkpoint_layouts(env, budget, seed=1234, ckpt=ckpt)
        assert ok
        env.reset()
        envs.append(env)
    a, b = envs
    g = torch.Generator(device="cpu").manual_seed(65)
    acts = torch.randint(0, 5, (80, n), generator=g).to(gpu_device)
    pick = np.random.default_rng(66).choice(n, 32, replace=False)
    oracles = _oracle_envs(cfg, _lb_rows(lb, pick).to_lists(), budget)
    obs, rew, done, status, r64 = a.step_multi(acts[:80], reward64=True)
    r64n, dn, stn = (x.cpu().numpy() for x in (r64, done, status))
    obs_p = obs[:, torch.from_numpy(pick).to(gpu_device)].cpu().numpy()
    for k in range(80):
        for j, i in enumerate(pick):
            r, d, s = oracles[j].step(int(acts[k, i]))
            if d:
                oracles[j].reset()
            assert (r64n[k, i], bool(dn[k, i]), int(stn[k, i])) == (r, d, s), "env %d t %d" % (i, k)
            assert obs_p[k, j].tobytes() == oracles[j].state_tensor().tobytes(), "env %d t %d" % (i, k)
    for k in range(80):
        o, r, d, s = b.step(acts[k])
        assert torch.equal(obs[k], o) and torch.equal(done[k], d) and torch.equal(status[k], s), k


def test_step_multi_bench_launch_sequence_with_fan_refill(gpu_device):
    """The headline launch sequence exactly as bench.py issues it (4096 C2-checkpoint envs,
    a 5-tick warm-up launch, then 20-tick launches read the shared fan table at offsets 5,
    25, ...), continued for 1,045 ticks so that the table is refilled once (the 51st 20-tick
    launch, ticks 1005-1024: fan_pos 1005 + 20 > kFanTicks, heist_capi.hip heist_step_multi)
    and read again after the refill.  Every tick of every env == single ticks bit for bit,
    and 32 envs == the C oracle on every tick's reward/done/status, with their observation
    rows compared byte for byte on the ticks around the refill (reference
    environment.py:216-299, security.py:49-101)."""
    import os
    from heist_amd.layouts import architect_checkpoint_layouts
    from heist_amd.training import _lb_rows
    ckpt = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "checkpoints",
                        "architect_c2_fixed.pt")
    n, budget = 4096, 15
    cfg = EnvironmentConfig(architect_budget=budget)
    envs = []
    for _ in range(2):  # the bench's handle shape (bench.py: max_cams = budget // 3, max_guards = budget // 5)
        env = HeistEnv(n, cfg, max_cams=5, max_guards=3, max_path=16, device=gpu_device)
        lb, ok = architect_checkpoint_layouts(env, budget, seed=1234, ckpt=ckpt)
        assert ok
        env.reset()
        envs.append(env)
    a, b = envs
    assert a.kernel_config()["multi_waves"] == 1 and a.kernel_config()["fan_on"] == 1
    chunks = [5] + [20] * 52
    T = sum(chunks)
    assert T >= 1040
    g = torch.Generator(device=gpu_device).manual_seed(4321)
    acts = torch.randint(0, 5, (T, n), device=gpu_device, generator=g, dtype=torch.int64)
    pick = np.random.default_rng(67).choice(n, 32, replace=False)
    pick_t = torch.from_numpy(pick).to(gpu_device)
    oracles = _oracle_envs(cfg, _lb_rows(lb, pick).to_lists(), budget)
    acts_p = acts[:, pick_t].cpu().numpy()
    window = range(985, 1045)  # the refill launch is ticks 1005-1024
    k0 = 0
    for K in chunks:
        obs, rew, done, status, r64 = a.step_multi(acts[k0:k0 + K], reward64=True)
        for k in range(K):
            o, r, d, s = b.step(acts[k0 + k])
            ctx = "tick %d" % (k0 + k)
            assert torch.equal(obs[k], o), ctx
            assert torch.equal(r64[k], b.reward64), ctx
            assert torch.equal(rew[k], r) and torch.equal(done[k], d) and torch.equal(status[k], s), ctx
        r64p, dp, sp = (x[:, pick_t].cpu().numpy() for x in (r64, done, status))
        need_obs = any(k0 + k in window for k in range(K))
        obs_p = obs[:, pick_t].cpu().numpy() if need_obs else None
        for k in range(K):
            for j in range(len(pick)):
                r, d, s = oracles[j].step(int(acts_p[k0 + k, j]))
                if d:
                    oracles[j].reset()
                assert (r64p[k, j], bool(dp[k, j]), int(sp[k, j])) == (r, d, s), "env %d t %d" % (pick[j], k0 + k)
                if need_obs and k0 + k in window:
                    assert obs_p[k, j].tobytes() == oracles[j].state_tensor().tobytes(), "env %d t %d" % (pick[j], k0 + k)
        k0 += K
    sa, sb = a.export(grid=True), b.export(grid=True)
    for key in sb:
        assert torch.equal(sa[key], sb[key]), key


def _shared_camera_layouts(n, R, budget, seed, fov, speed, heading, **kw):
    """Synthetic layouts whose cameras all share one (fov, speed, heading), as an Architect
    batch's do (reference networks.py:283-322): the lean K-tick kernel's fan-served form."""
    lays = synthetic_layouts(n, R, R, budget, seed=seed, **kw)
    out = []
    for walls, cams, guards in lays:
        cams = [dict(c, fov_angle=fov, rotation_speed=speed, heading=heading) for c in cams]
        out.append((walls, cams, guards))
    return out


@pytest.mark.parametrize("auto_reset", [True, False], ids=["auto_reset", "no_reset"])
@pytest.mark.parametrize("fov", [120.0, 126.5, 33.25], ids=["fov120", "fov126", "fov33"])
def test_step_lean_wide_fans_and_many_guards(gpu_device, monkeypatch, fov, auto_reset):
    """The lean one-wave K-tick kernel (step_lean_kernel) on shared-camera layouts with wide
    fans (more than 64 unique directions: the second staged chunk, and the chunk the
    previous tick did not stage), budget 40 (up to 13 cameras, 8 guards: two cone-stamp
    passes), short episodes, launches of 1, 63, 70 and 66 ticks (the 64-tick action chunk
    and the table's refill) == single ticks and == the generic K-tick body (HEIST_LEAN=0),
    bit for bit."""
    n, R, budget = 512, 20, 40
    cfg = EnvironmentConfig(max_steps=30, architect_budget=budget)
    f32 = lambda x: float(np.float32(x))  # noqa: E731
    lays = _shared_camera_layouts(n, R, budget, 77, f32(fov), f32(23.7), f32(301.3))
    envs = []
    monkeypatch.setenv("HEIST_MULTI_WAVES", "1")  # one wave per env at n = 512, as at the bench's 4,096
    for lean in ("1", "0", "1"):
        monkeypatch.setenv("HEIST_LEAN", lean)
        env = HeistEnv(n, cfg, max_cams=13, max_guards=8, max_path=16, device=gpu_device)
        monkeypatch.delenv("HEIST_LEAN")
        v = env.set_layouts(lays, budget=budget)
        env.reset()
        envs.append((env, v))
    (a, va), (c, vc), (b, vb) = envs
    assert torch.equal(va, vb) and torch.equal(va, vc)
    assert a.kernel_config()["lean"] == 1 and c.kernel_config()["lean"] == 0
    assert a.kernel_config()["multi_waves"] == 1
    g = torch.Generator(device="cpu").manual_seed(78)
    acts = torch.randint(0, 5, (200, n), generator=g).to(gpu_device)
    k0 = 0
    for kk in (1, 63, 70, 66):
        oa = a.step_multi(acts[k0:k0 + kk], auto_reset=auto_reset, reward64=True)
        oc = c.step_multi(acts[k0:k0 + kk], auto_reset=auto_reset, reward64=True)
        for x, y in zip(oa, oc):
            assert torch.equal(x, y), k0
        for k in range(kk):
            o, r, d, s = b.step(acts[k0 + k], auto_reset=auto_reset)
            ctx = "tick %d" % (k0 + k)
            assert torch.equal(oa[0][k], o), ctx
            assert torch.equal(oa[4][k], b.reward64) and torch.equal(oa[2][k], d) and torch.equal(oa[3][k], s), ctx
        k0 += kk
    sa, sb = a.export(grid=True), b.export(grid=True)
    for key in sb:
        assert torch.equal(sa[key], sb[key]), key


def _interval_fan_layouts(n, R, budget, seed, **kw):
    """Synthetic layouts (every camera its own fov, heading, speed: the shared fan serves
    none) with some cameras forced onto the hard cases of the interval fans: the reference's
    default camera (heading 0, fov 60, speed 15: rays on whole and half degrees, on the axes),
    rays a few angle units from a cut, fovs up to 120 degrees (two 64-lane interval chunks)."""
    from heist_amd.layouts import synthetic_layouts
    rng = np.random.default_rng(seed)
    cuts = [0.0, 4.7885, 30.0, 41.4096, 45.0, 60.0, 90.0, 135.0, 180.0, 270.0]
    out = []
    for walls, cams, guards in synthetic_layouts(n, R, R, budget, seed=seed, **kw):
        cams = [dict(c) for c in cams]
        for c in cams:
            u = rng.random()
            if u < 0.15:
                c.update(fov_angle=60.0, heading=0.0, rotation_speed=15.0)
            elif u < 0.3:  # ray i on (about) a cut angle at the first K-tick tick (one rotation)
                fov = float(np.float32(rng.uniform(30, 120)))
                nr = max(int(fov * 2), 30)
                i = int(rng.integers(0, nr + 1))
                cut = float(rng.choice(cuts)) + float(rng.choice([0.0, 3e-6, -3e-6, 1e-7]))
                c.update(fov_angle=fov, heading=(cut + fov / 2.0 - fov * i / nr - c["rotation_speed"]) % 360.0)
            elif u < 0.4:
                c.update(fov_angle=float(np.float32(rng.uniform(100, 120))))
        out.append((walls, cams, guards))
    return out


@pytest.mark.parametrize("auto_reset", [True, False], ids=["auto_reset", "no_reset"])
@pytest.mark.parametrize("R,n,budget,kw,waves", [(20, 4096, 15, {}, None), (20, 512, 40, {}, None),
                                                 (32, 2048, 40, {"n_cams": 4, "n_guards": 3}, None),
                                                 (32, 2048, 40, {"n_cams": 4, "n_guards": 3}, 1)],
                         ids=["bench4096", "budget40", "c5_32x32", "c5_32x32_one_wave"])
def test_step_lean_interval_fans(gpu_device, monkeypatch, R, n, budget, kw, waves, auto_reset):
    """step_lean_kernel's interval fans (cameras the shared fan does not serve: the synthetic
    mix) == single ticks of the step kernel, == the generic K-tick body (HEIST_INTERVAL_FANS=0),
    and 32 envs == the C oracle (reward, done, status, observation bytes) on every tick; short
    episodes, launches of 1, 20, 63 and 70 ticks; 20 x 20 and BASELINE C5's 32 x 32 (2048 envs,
    exactly 4 cameras + 3 guards, budget 40: four observation quads per lane, 19 stores per
    row; at 2,048 envs two waves per env, HEIST_LEAN_WAVES=1 the one-wave form).  Cameras forced
    onto the default heading, cuts, axes and wide fovs (_interval_fan_layouts).  Reference
    environment.py:216-299, security.py:53-101."""
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R, max_steps=40, architect_budget=budget)
    lays = _interval_fan_layouts(n, R, budget, 300 + budget + R, **kw)
    envs = []
    monkeypatch.setenv("HEIST_MULTI_WAVES", "1")
    if waves is not None:
        monkeypatch.setenv("HEIST_LEAN_WAVES", str(waves))
    for i, ivl in enumerate(("1", "0", "1")):
        monkeypatch.setenv("HEIST_INTERVAL_FANS", ivl)
        env = (HeistEnv if i < 2 else _step_kernel_env)(n, cfg, max_cams=max(1, budget // 3),
                                                        max_guards=max(1, budget // 5), max_path=16, device=gpu_device)
        v = env.set_layouts(lays, budget=budget)
        env.reset()
        envs.append((env, v))
    monkeypatch.delenv("HEIST_INTERVAL_FANS")
    (a, va), (c, vc), (b, vb) = envs
    assert torch.equal(va, vb) and torch.equal(va, vc)
    assert a.kernel_config()["interval_fans"] == 1 and c.kernel_config()["interval_fans"] == 0
    assert a.kernel_config()["lean"] == 1 and a.kernel_config()["multi_waves"] == 1
    if R == 32 and torch.cuda.get_device_properties(gpu_device).multi_processor_count >= 256:
        assert a.kernel_config()["lean_waves"] == (waves or 2)
    valid = va.cpu().numpy().astype(bool)
    pick = np.random.default_rng(budget).choice(np.nonzero(valid)[0], 32, replace=False)
    pick_t = torch.from_numpy(pick).to(gpu_device)
    oracles = _oracle_envs(cfg, [lays[i] for i in pick], budget)
    g = torch.Generator(device="cpu").manual_seed(79)
    acts = torch.randint(0, 5, (160, n), generator=g).to(gpu_device)
    k0 = 0
    for kk in (1, 20, 63, 70):
        oa = a.step_multi(acts[k0:k0 + kk], auto_reset=auto_reset, reward64=True)
        oc = c.step_multi(acts[k0:k0 + kk], auto_reset=auto_reset, reward64=True)
        for x, y in zip(oa, oc):
            assert torch.equal(x, y), k0
        obs_p = oa[0][:, pick_t].cpu().numpy()
        r64p, dp, sp = (x[:, pick_t].cpu().numpy() for x in (oa[4], oa[2], oa[3]))
        ap = acts[k0:k0 + kk, pick_t].cpu().numpy()
        for k in range(kk):
            o, r, d, s = b.step(acts[k0 + k], auto_reset=auto_reset)
            ctx = "tick %d" % (k0 + k)
            assert torch.equal(oa[0][k], o), ctx
            assert torch.equal(oa[4][k], b.reward64) and torch.equal(oa[2][k], d) and torch.equal(oa[3][k], s), ctx
            for j in range(len(pick)):
                r_, d_, s_ = oracles[j].step(int(ap[k, j]))
                if d_ and auto_reset:
                    oracles[j].reset()
                assert (r64p[k, j], bool(dp[k, j]), int(sp[k, j])) == (r_, d_, s_), "env %d %s" % (pick[j], ctx)
                assert obs_p[k, j].tobytes() == oracles[j].state_tensor().tobytes(), "env %d %s" % (pick[j], ctx)
        k0 += kk
    sa, sb = a.export(grid=True), b.export(grid=True)
    for key in sb:
        assert torch.equal(sa[key], sb[key]), key


@pytest.mark.parametrize("R,n,budget,kw", [(20, 512, 15, {}), (32, 2048, 40, {"n_cams": 4, "n_guards": 3})],
                         ids=["20x20", "c5_32x32"])
def test_step_lean_interval_fans_narrow_fovs(gpu_device, monkeypatch, R, n, budget, kw):
    """Cameras around the interval fans' ray-spacing bound (su >= 2^21 angle units: the integer
    pair bounds need rint(2^52 / su) in an int32; fov / 30 rays below ~5.27 degrees sends the
    env to the generic body): fovs 2 .. 16 degrees mixed with ordinary ones, 512 envs at 20 x 20
    and 2048 C5 envs at 32 x 32, == single ticks of the step kernel and 16 envs == the C oracle
    over 60 ticks in launches of 20 and 40."""
    rng = np.random.default_rng(17 + R)
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R, max_steps=30)
    lays = []
    for walls, cams, guards in synthetic_layouts(n, R, R, budget, seed=171 + R, **kw):
        cams = [dict(c) for c in cams]
        for c in cams:
            if rng.random() < 0.6:
                c.update(fov_angle=float(rng.choice([2.0, 5.0, 5.25, 5.2734375, 5.3, 6.0, 10.0, 15.5])))
        lays.append((walls, cams, guards))
    monkeypatch.setenv("HEIST_MULTI_WAVES", "1")
    envs = []
    for i in range(2):
        env = (HeistEnv if i == 0 else _step_kernel_env)(n, cfg, max_cams=max(5, budget // 3),
                                                        max_guards=max(3, budget // 5), max_path=16, device=gpu_device)
        v = env.set_layouts(lays, budget=budget)
        env.reset()
        envs.append((env, v))
    (a, va), (b, vb) = envs
    assert torch.equal(va, vb)
    assert a.kernel_config()["lean"] == 1 and a.kernel_config()["multi_waves"] == 1
    pick = np.random.default_rng(3).choice(np.nonzero(va.cpu().numpy().astype(bool))[0], 16, replace=False)
    oracles = _oracle_envs(cfg, [lays[i] for i in pick], budget)
    g = torch.Generator(device="cpu").manual_seed(91)
    acts = torch.randint(0, 5, (60, n), generator=g).to(gpu_device)
    k0 = 0
    for kk in (20, 40):
        obs, rew, done, status, r64 = a.step_multi(acts[k0:k0 + kk], reward64=True)
        for k in range(kk):
            o, r, d, s = b.step(acts[k0 + k])
            assert torch.equal(obs[k], o) and torch.equal(r64[k], b.reward64), k0 + k
            assert torch.equal(done[k], d) and torch.equal(status[k], s), k0 + k
            for i, o_env in zip(pick, oracles):
                r_, d_, s_ = o_env.step(int(acts[k0 + k, i]))
                if d_:
                    o_env.reset()
                assert (float(r64[k, i]), bool(done[k, i]), int(status[k, i])) == (r_, d_, s_), (k0 + k, i)
                assert obs[k, i].cpu().numpy().tobytes() == o_env.state_tensor().tobytes(), (k0 + k, i)
        k0 += kk


@pytest.mark.parametrize("waves", [1, 2])
def test_step_lean_32x32_shared_fan_and_interval_mix(gpu_device, monkeypatch, waves):
    """The 32 x 32 lean kernel with one and two waves per env on a batch that mixes envs the
    shared fan serves (every camera the batch's first camera's twin: in the two-wave form wave
    0 casts them) with interval-fan envs (the casts split over the waves) and envs the generic
    body takes (a 4-degree fov: wave 1 leaves): K-tick launches with auto-reset == single ticks
    of the step kernel, and 12 envs == the C oracle, over 60 ticks."""
    n, R, budget = 512, 32, 40
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R, max_steps=30, architect_budget=budget)
    rng = np.random.default_rng(29 + waves)
    lays = []
    for walls, cams, guards in synthetic_layouts(n, R, R, budget, seed=131, n_cams=4, n_guards=3):
        cams = [dict(c) for c in cams]
        u = rng.random()
        for c in cams:
            if u < 0.5:  # the shared fan's source camera's twin
                c.update(fov_angle=60.0, heading=30.0, rotation_speed=15.0)
            elif u < 0.6:
                c.update(fov_angle=4.0)
        lays.append((walls, cams, guards))
    first = lays[0][1][0]
    first.update(fov_angle=60.0, heading=30.0, rotation_speed=15.0)
    monkeypatch.setenv("HEIST_LEAN_WAVES", str(waves))
    a = HeistEnv(n, cfg, max_cams=13, max_guards=8, max_path=16, device=gpu_device)
    monkeypatch.delenv("HEIST_LEAN_WAVES")
    b = _step_kernel_env(n, cfg, max_cams=13, max_guards=8, max_path=16, device=gpu_device)
    va, vb = a.set_layouts(lays, budget=budget), b.set_layouts(lays, budget=budget)
    assert torch.equal(va, vb)
    a.reset()
    b.reset()
    assert a.kernel_config()["lean"] == 1 and a.kernel_config()["lean_waves"] == waves
    pick = np.random.default_rng(5).choice(np.nonzero(va.cpu().numpy().astype(bool))[0], 12, replace=False)
    oracles = _oracle_envs(cfg, [lays[i] for i in pick], budget)
    g = torch.Generator(device="cpu").manual_seed(97)
    acts = torch.randint(0, 5, (60, n), generator=g).to(gpu_device)
    k0 = 0
    for kk in (1, 20, 39):
        obs, rew, done, status, r64 = a.step_multi(acts[k0:k0 + kk], reward64=True)
        for k in range(kk):
            o, r, d, s = b.step(acts[k0 + k])
            assert torch.equal(obs[k], o) and torch.equal(r64[k], b.reward64), k0 + k
            assert torch.equal(done[k], d) and torch.equal(status[k], s), k0 + k
            for i, o_env in zip(pick, oracles):
                r_, d_, s_ = o_env.step(int(acts[k0 + k, i]))
                if d_:
                    o_env.reset()
                assert (float(r64[k, i]), bool(done[k, i]), int(status[k, i])) == (r_, d_, s_), (k0 + k, i)
                assert obs[k, i].cpu().numpy().tobytes() == o_env.state_tensor().tobytes(), (k0 + k, i)
        k0 += kk
    sa, sb = a.export(grid=True), b.export(grid=True)
    for key in sb:
        assert torch.equal(sa[key], sb[key]), key


def test_step_lean_interval_fans_on_architect_layouts(gpu_device, monkeypatch):
    """The headline's Architect layouts with the shared fan table off (HEIST_SHARED_FAN=0):
    every env takes the interval fans instead; == single ticks, 60 ticks."""
    import os
    from heist_amd.layouts import architect_checkpoint_layouts
    ckpt = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "checkpoints",
                        "architect_c2_fixed.pt")
    n, budget = 4096, 15
    cfg = EnvironmentConfig(architect_budget=budget, max_steps=30)
    envs = []
    for fan in ("0", "1"):
        monkeypatch.setenv("HEIST_SHARED_FAN", fan)
        env = HeistEnv(n, cfg, max_cams=5, max_guards=3, max_path=16, device=gpu_device)
        _, ok = architect_checkpoint_layouts(env, budget, seed=1234, ckpt=ckpt)
        assert ok
        env.reset()
        envs.append(env)
    monkeypatch.delenv("HEIST_SHARED_FAN")
    a, b = envs
    assert a.kernel_config()["fan_on"] == 0 and a.kernel_config()["multi_waves"] == 1
    g = torch.Generator(device="cpu").manual_seed(81)
    acts = torch.randint(0, 5, (60, n), generator=g).to(gpu_device)
    oa = a.step_multi(acts[:60], reward64=True)
    for k in range(60):
        o, r, d, s = b.step(acts[k])
        assert torch.equal(oa[0][k], o) and torch.equal(oa[4][k], b.reward64), k
        assert torch.equal(oa[2][k], d) and torch.equal(oa[3][k], s), k


@pytest.mark.parametrize("waves", [1, 2])
@pytest.mark.parametrize("cones", [True, False], ids=["guard_cones", "live_guards"])
def test_step_multi_one_wave_per_env(gpu_device, monkeypatch, cones, waves):
    """The K-tick kernel's one-wave-per-env form (HEIST_MULTI_WAVES=1: every role on one
    wave, the default from 16 envs per CU) and its two-wave form == single ticks, bit for
    bit, with short episodes."""
    n, R = 384, 20
    cfg = EnvironmentConfig(max_steps=25)
    lays = synthetic_layouts(n, R, R, 15, seed=67)
    monkeypatch.setenv("HEIST_MULTI_WAVES", str(waves))
    a = HeistEnv(n, cfg, device=gpu_device)
    monkeypatch.delenv("HEIST_MULTI_WAVES")
    b = HeistEnv(n, cfg, device=gpu_device)
    assert a.kernel_config()["multi_waves"] == waves
    for env in (a, b):
        env.set_guard_cones(cones)
        env.set_layouts(lays, budget=15)
        env.reset()
    g = torch.Generator(device="cpu").manual_seed(68)
    acts = torch.randint(0, 5, (60, n), generator=g).to(gpu_device)
    _compare_multi_vs_single(a, b, acts, [13, 47])


@pytest.mark.parametrize("waves", [1, 2])
@pytest.mark.parametrize("R,C", [(13, 17), (9, 23), (16, 20)])
def test_step_multi_any_grid_width(gpu_device, monkeypatch, waves, R, C):
    """heist_step_multi on grids whose width is not a multiple of 4 (the K-tick kernel's
    float4 rows need C % 4 == 0; other widths run K single ticks) and on a 16 x 20 grid (the
    kernel itself) == single ticks."""
    n = 256
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=C, max_steps=30)
    lays = synthetic_layouts(n, R, C, 15, seed=69)
    monkeypatch.setenv("HEIST_MULTI_WAVES", str(waves))
    a = HeistEnv(n, cfg, device=gpu_device)
    monkeypatch.delenv("HEIST_MULTI_WAVES")
    b = HeistEnv(n, cfg, device=gpu_device)
    for env in (a, b):
        env.set_layouts(lays, budget=15)
        env.reset()
    g = torch.Generator(device="cpu").manual_seed(70)
    acts = torch.randint(0, 5, (45, n), generator=g).to(gpu_device)
    _compare_multi_vs_single(a, b, acts, [20, 25])


@pytest.mark.parametrize("waves", [1, 2])
@pytest.mark.parametrize("auto_reset", [True, False], ids=["auto_reset", "no_reset"])
def test_step_multi_shared_fan(gpu_device, monkeypatch, waves, auto_reset):
    """Architect-checkpoint layouts (every camera of the batch shares one fan, so the K-tick
    kernel takes its rays from the shared fan table, FanTick) with short episodes: timeouts,
    detections and resets inside a launch, and without auto-reset finished envs stop
    rotating and fall back to their own fan -- bit-identical to single ticks, and to the
    same launches with the table off (HEIST_SHARED_FAN=0)."""
    import os
    from heist_amd.layouts import architect_checkpoint_layouts
    ckpt = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "checkpoints",
                        "architect_c2_fixed.pt")
    n, budget = 512, 15
    cfg = EnvironmentConfig(architect_budget=budget, max_steps=25)
    envs = []
    for fan in ("1", "0", "1"):
        monkeypatch.setenv("HEIST_MULTI_WAVES", str(waves))
        monkeypatch.setenv("HEIST_SHARED_FAN", fan)
        env = HeistEnv(n, cfg, max_cams=5, max_guards=3, max_path=16, device=gpu_device)
        monkeypatch.delenv("HEIST_MULTI_WAVES")
        monkeypatch.delenv("HEIST_SHARED_FAN")
        _, ok = architect_checkpoint_layouts(env, budget, seed=1234, ckpt=ckpt)
        assert ok
        env.reset()
        envs.append(env)
    a, c, b = envs
    assert a.kernel_config()["fan_on"] == 1 and c.kernel_config()["fan_on"] == 0
    g = torch.Generator(device="cpu").manual_seed(71)
    acts = torch.randint(0, 5, (60, n), generator=g).to(gpu_device)
    for k0, kk in ((0, 20), (20, 40)):
        oa = a.step_multi(acts[k0:k0 + kk], auto_reset=auto_reset, reward64=True)
        oc = c.step_multi(acts[k0:k0 + kk], auto_reset=auto_reset, reward64=True)
        for x, y in zip(oa, oc):
            assert torch.equal(x, y)
        for k in range(kk):
            o, r, d, s = b.step(acts[k0 + k], auto_reset=auto_reset)
            assert torch.equal(oa[0][k], o) and torch.equal(oa[2][k], d) and torch.equal(oa[3][k], s), (k0 + k)


def test_step_multi_shared_fan_across_layout_changes(gpu_device):
    """The shared fan table across heist_set_layout / single ticks between K-tick launches:
    new Architect cameras (a second checkpoint draw) and headings advanced by single ticks
    make the table stale; results stay equal to single ticks throughout."""
    import os
    from heist_amd.layouts import architect_checkpoint_layouts
    ckpt = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "checkpoints",
                        "architect_c2_fixed.pt")
    n, budget = 512, 15
    cfg = EnvironmentConfig(architect_budget=budget, max_steps=30)
    a, b = (HeistEnv(n, cfg, max_cams=5, max_guards=3, max_path=16, device=gpu_device) for _ in range(2))
    g = torch.Generator(device="cpu").manual_seed(72)
    acts = torch.randint(0, 5, (90, n), generator=g).to(gpu_device)
    t = 0
    for seed, kk, single in ((1234, 25, 3), (99, 30, 2), (99, 20, 0)):
        if seed != 99 or kk == 30:
            for env in (a, b):
                _, ok = architect_checkpoint_layouts(env, budget, seed=seed, ckpt=ckpt)
                assert ok
                env.reset()
        oa = a.step_multi(acts[t:t + kk])
        for k in range(kk):
            o, r, d, s = b.step(acts[t + k])
            assert torch.equal(oa[0][k], o) and torch.equal(oa[2][k], d) and torch.equal(oa[3][k], s), (t + k)
        t += kk
        for k in range(single):  # single ticks on both: headings move outside the launches
            oa1 = a.step(acts[t])
            ob1 = b.step(acts[t])
            assert torch.equal(oa1[0], ob1[0])
            t += 1
