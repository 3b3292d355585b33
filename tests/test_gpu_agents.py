"""GPU tests of the layers above the kernels: Architect decode, masked re-layout, the
single-env HeistEnvironment compatibility class, agents and the batched trainer."""
import json
import os

import numpy as np
import pytest
import torch

import golden_data as gd
from heist_amd import EnvironmentConfig, HeistEnv, HeistEnvironment
from heist_amd.architect_decode import decode_layouts
from heist_amd.layouts import synthetic_layouts

pytestmark = pytest.mark.gpu


def test_architect_decode_golden(gpu_device):
    """heist_architect_decode == ArchitectNetwork.generate_layout's decode on the
    reference's recorded asset maps (networks.py:283-335)."""
    z = gd.load("nets.npz")
    dec = gd.load_json("architect_decode.json")
    cur = 0
    for (R, C, budget, nw, nc, ng), case in zip(z["dec_meta"], dec):
        amap = torch.tensor(z["dec_maps"][cur:cur + R * C].reshape(1, R, C).astype(np.int64), device=gpu_device)
        cur += R * C
        fov, speed, heading = case["cam_params"]
        cp = torch.tensor([[fov, speed, heading]], dtype=torch.float32, device=gpu_device)
        lb = decode_layouts(amap, cp, int(budget))
        walls, cams, guards = lb.to_lists()[0]
        assert [list(w) for w in walls] == case["walls"]
        assert [(c["row"], c["col"]) for c in cams] == [tuple(c) for c in case["cams"]]
        for c in cams:
            assert (c["fov_angle"], c["rotation_speed"], c["heading"], c["vision_range"]) == (fov, speed, heading, 6)
        assert [[list(p) for p in g["patrol_path"]] for g in guards] == case["guards"]
        assert all(g["speed"] == 1 and g["vision_range"] == 4 and g["fov_angle"] == 90.0 for g in guards)


def test_masked_set_layout_and_reset(gpu_device):
    cfg = EnvironmentConfig()
    n = 16
    env = HeistEnv(n, cfg, device=gpu_device)
    lays = synthetic_layouts(n, 20, 20, 15, seed=2)
    env.set_layouts(lays)
    env.reset()
    grid0 = env.export(grid=True)["grid"].clone()
    new = synthetic_layouts(3, 20, 20, 15, seed=99)
    env.set_layouts(new, env_ids=[1, 5, 9])
    grid1 = env.export(grid=True)["grid"]
    keep = [i for i in range(n) if i not in (1, 5, 9)]
    assert torch.equal(grid1[keep], grid0[keep])
    ref = HeistEnv(3, cfg, device=gpu_device)
    ref.set_layouts(new)
    assert torch.equal(grid1[[1, 5, 9]], ref.export(grid=True)["grid"])
    for _ in range(7):
        env.step(torch.full((n,), 4))
    obs_before = env.obs.clone()
    tick_before = env.export()["tick"].clone()
    m = torch.zeros(n, dtype=torch.uint8, device=gpu_device)
    m[[1, 5, 9]] = 1
    env.reset(m)
    assert torch.equal(env.obs[keep], obs_before[keep])
    st = env.export()
    assert (st["tick"][[1, 5, 9]] == 0).all() and torch.equal(st["tick"][keep], tick_before[keep])


def test_single_env_class_matches_golden_traces(gpu_device):
    """HeistEnvironment (reference API, GPU-backed) replays golden traces exactly."""
    for tr in list(gd.env_traces())[:12]:
        cfg = EnvironmentConfig(grid_rows=tr["R"], grid_cols=tr["C"], max_steps=tr["max_steps"],
                                start_pos=tr["start"], vault_pos=tr["vault"], architect_budget=tr["budget"])
        env = HeistEnvironment(cfg, device=gpu_device)
        assert env.set_layout(tr["walls"], tr["cams"], tr["guards"]) == tr["valid"]
        assert (len(env.walls), len(env.cameras), len(env.guards), env.budget.spent) == tuple(tr["accepted"])
        np.testing.assert_array_equal(env.grid, tr["grid"])
        for k, op in enumerate(tr["ops"][:150]):
            if op == -1:
                env.reset()
                r = 0.0
            else:
                _, r, d, info = env.step(int(op))
                assert d == tr["done"][k]
            assert r == tr["reward"][k]
            assert env.solver_pos == tuple(tr["pos"][k]) and env.tick == tr["tick"][k]
            assert [c.heading for c in env.cameras] == list(tr["cam_h"][k])
            assert [g.current_idx for g in env.guards] == list(tr["g_idx"][k])
            np.testing.assert_array_equal(env.visibility_map.visibility > 0.5, tr["vis"][k])
            if k < len(tr["state"]):
                assert env.get_state_tensor().tobytes() == tr["state"][k].tobytes()


def test_reference_kats_through_single_env_class(gpu_device):
    kat = gd.load_json("kat.json")
    s = kat["sanity"]
    env = HeistEnvironment(EnvironmentConfig(grid_rows=10, grid_cols=10, start_pos=(1, 1), vault_pos=(8, 8)),
                           device=gpu_device)
    assert env.set_layout([(3, 3), (3, 4), (3, 5)],
                          [{"row": 5, "col": 5, "fov_angle": 60, "heading": 0, "rotation_speed": 15,
                            "vision_range": 4}],
                          [{"patrol_path": [(7, 2), (7, 3), (7, 4), (7, 5)], "speed": 1, "vision_range": 3,
                            "fov_angle": 90}]) == s["valid"]
    env.reset()
    rews = []
    for _ in range(5):
        _, r, d, info = env.step(4)
        rews.append(r)
        if d:
            break
    assert rews == s["rewards"] and info["status"] == s["status"] and env.tick == s["tick"]
    assert list(env.solver_pos) == s["pos"]
    assert int(np.sum(env.visibility_map.visibility > 0.5)) == s["surveilled"]
    assert env.render_text() == s["render"]
    assert env.detection_events and env.get_architect_reward() == 1.0
    env = HeistEnvironment(EnvironmentConfig(grid_rows=10, grid_cols=10), device=gpu_device)
    env.set_layout([], [], [])
    env.reset()
    tot = sum(env.step(2)[1] for _ in range(7))
    assert tot == kat["fixes_down"]
    for _ in range(7):
        _, r, d, info = env.step(4)
        tot += r
        if d:
            break
    assert tot == kat["fixes_right"] and info["status"] == kat["fixes_status"]
    st = env.get_environment_state()
    json.dumps(st)  # the dashboard's frame format must serialise
    assert st["done"] and st["solver_pos"] == (8, 8)


def test_solver_agent_reference_api(gpu_device, tmp_path):
    from heist_amd.agents import SolverAgent
    env = HeistEnvironment(EnvironmentConfig(grid_rows=10, grid_cols=10), device=gpu_device)
    env.set_layout([(3, 3)], [], [])
    ag = SolverAgent(grid_rows=10, grid_cols=10, device=gpu_device)
    for _ in range(2):
        env.reset()
        ag.reset()
        state = env.get_state_tensor()
        for _ in range(40):
            a = ag.select_action(state)
            _, r, d, _ = env.step(a)
            ag.store_transition(r, d)
            state = env.get_state_tensor()
            if d:
                break
        ag.end_episode(0.0)
    m = ag.update()
    assert set(m) >= {"solver_policy_loss", "solver_value_loss", "solver_entropy"}
    assert all(np.isfinite(v) for v in m.values())
    p = tmp_path / "solver_ep1.pt"
    ag.save(str(p))
    ck = torch.load(str(p), weights_only=True)
    assert set(ck) == {"network", "optimizer", "episode_count"} and ck["episode_count"] == 2
    ag2 = SolverAgent(grid_rows=10, grid_cols=10, device=gpu_device)
    ag2.load(str(p))
    for k, v in ag.network.state_dict().items():
        assert torch.equal(v, ag2.network.state_dict()[k])


def test_trainer_runs_and_logs(gpu_device, tmp_path):
    from heist_amd.training import AdversarialTrainer
    cfg = EnvironmentConfig(grid_rows=12, grid_cols=12, max_steps=40)
    tr = AdversarialTrainer(cfg, solver_episodes_per_layout=2, total_episodes=96, save_dir=str(tmp_path / "ck"),
                            log_dir=str(tmp_path / "logs"), n_envs=32, rollout_len=40, minibatch=256,
                            device=gpu_device, seed=0)
    tr.train(warmup_rollouts=1)
    logs = json.load(open(tmp_path / "logs" / "game_log.json"))
    assert len(logs) >= 1
    keys = {"episode", "phase", "budget", "walls", "cameras", "guards", "solve_rate", "detection_rate",
            "timeout_rate", "architect_reward", "solver_reward", "avg_steps", "level_valid", "is_interactive",
            "freeze_architect", "freeze_solver", "temperature", "timestamp"}
    assert set(logs[0]) == keys
    for e in logs:
        if e["level_valid"]:
            assert abs(e["solve_rate"] + e["detection_rate"] + e["timeout_rate"] - 1.0) < 1e-6
    met = json.load(open(tmp_path / "logs" / "training_metrics.json"))
    assert set(met) == set(("episode", "solve_rate", "detection_rate", "timeout_rate", "architect_reward",
                            "solver_reward", "architect_loss", "solver_loss", "avg_steps", "budget", "phase"))
    last = tr.find_latest_checkpoint()
    assert last is not None and tr.list_checkpoints()[-1] == last
    tr2 = AdversarialTrainer(cfg, solver_episodes_per_layout=2, total_episodes=8, save_dir=str(tmp_path / "ck"),
                             log_dir=str(tmp_path / "logs"), n_envs=8, rollout_len=40, device=gpu_device)
    assert tr2.resume_from_checkpoint() == last
    n0 = len(tr2.game_log)
    res = tr2.run_interactive_episodes(num_episodes=2, budget=9, solver_attempts=2)
    assert len(res) == 2 and all(r["budget"] == 9 for r in res)  # the reference's ep_metrics dicts
    assert all(e.to_dict()["is_interactive"] for e in tr2.game_log[n0:])
    sim = tr2.simulate_episode(budget=8, solver_attempts=2)
    assert sim["outcome"] in ("vault_reached", "detected", "timeout") and len(sim["frames"]) >= 2
