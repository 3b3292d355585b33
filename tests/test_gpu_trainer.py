"""GPU tests of the batched AdversarialTrainer (training.py:277-600 replaced):

* the rollout's rewards / dones / statuses replayed through the C oracle, the GAE of its
  complete episodes equal to the reference's _compute_gae (agents/solver.py:228-244), and
  the V(s_T) bootstrap where the rollout cuts an attempt;
* BASELINE config 3 (4096 envs, 20x20, alternating Architect/Solver self-play) and
  config 4 (8192 envs, curriculum budget 10 -> 40) iterations with sampled oracle replay;
* interactive episodes masking the training envs; callbacks with the reference's frame.
RNG streams differ from the reference (device sampling), so trajectories are compared by
action replay, as SURVEY 7 states.
"""
import json
import os

import numpy as np
import pytest
import torch

from heist_amd import EnvironmentConfig
from heist_amd.training import CURRICULA, AdversarialTrainer
from oracle import pyoracle as po
from trainer_replay import replay

pytestmark = pytest.mark.gpu


def _trainer(tmp_path, n, R=20, T=48, A=3, episode0=200, **kw):
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R, max_steps=200)
    tr = AdversarialTrainer(cfg, solver_episodes_per_layout=A, total_episodes=10 ** 6, save_dir=str(tmp_path / "ck"),
                            log_dir=str(tmp_path / "logs"), n_envs=n, rollout_len=T, device=kw.pop("device"),
                            seed=kw.pop("seed", 0), **kw)
    tr.global_episode = episode0  # curriculum phase with cameras and guards
    tr._assign_layouts(np.arange(n))
    return tr


def test_rollout_replay_and_gae_bootstrap(gpu_device, tmp_path):
    tr = _trainer(tmp_path, 24, T=64, device=gpu_device, minibatch=512)
    ids = np.nonzero(tr.b_valid.cpu().numpy())[0]
    assert len(ids) >= 12
    tr._trace = []
    ro = tr._rollout(64)
    assert replay(tr, ids, tr._trace) == 64 * len(ids)
    r64 = torch.stack([x[1] for x in tr._trace])
    assert torch.equal(ro.rewards, r64.float())
    assert torch.equal(ro.dones.bool(), torch.stack([x[2] for x in tr._trace]))
    # V(s_T) under the carried LSTM state, recomputed independently
    with torch.no_grad():
        _, v_T, _ = tr.solver.network(tr.env.obs, (tr.h, tr.c))
    torch.testing.assert_close(ro.last_value, v_T.reshape(-1), rtol=0, atol=1e-5)
    adv, ret = tr.solver.rollout_advantages(ro)
    r, v, d = (x.cpu().numpy() for x in (ro.rewards, ro.values, ro.dones))
    adv, ret, lv = adv.cpu().numpy(), ret.cpu().numpy(), ro.last_value.cpu().numpy()
    np.testing.assert_array_equal(ret, adv + v)
    n_complete = n_cut = 0
    g, lam = tr.solver.gamma, tr.solver.gae_lambda
    for e in ids:
        ends = list(np.nonzero(d[:, e])[0])
        s = 0
        for t_end in ends:  # complete attempts: the reference's per-buffer GAE, bootstrap 0
            exp = po.gae(r[s:t_end + 1, e], v[s:t_end + 1, e], d[s:t_end + 1, e].astype(np.float32))
            np.testing.assert_allclose(adv[s:t_end + 1, e], exp, rtol=0, atol=1e-5)
            n_complete += 1
            s = t_end + 1
        if s < 64:  # the attempt the rollout cuts: bootstrapped from V(s_T)
            T1 = 63
            exp_last = r[T1, e] + g * lv[e] - v[T1, e]
            assert abs(adv[T1, e] - exp_last) < 1e-6
            # and the whole cut segment equals GAE on [s, T) with one extra step of value V(s_T)
            rr = np.append(r[s:, e], 0.0).astype(np.float32)
            vv = np.append(v[s:, e], lv[e]).astype(np.float32)
            dd = np.zeros(len(rr), np.float32)
            dd[-1] = 1.0
            exp = po.gae(rr, vv, dd, g, lam)[:-1]
            np.testing.assert_allclose(adv[s:, e], exp, rtol=0, atol=1e-5)
            n_cut += 1
    assert n_complete > 0 and n_cut > 0


def _check_scored(tr):
    for e in tr.game_log:
        d = e.to_dict()
        if d["level_valid"]:
            assert abs(d["solve_rate"] + d["detection_rate"] + d["timeout_rate"] - 1.0) < 1e-6
    eps = [e.to_dict()["episode"] for e in tr.game_log]
    assert len(eps) == len(set(eps))


def _roundtrip(tr, tmp_path):
    tr._save_checkpoint(tr.global_episode)
    cfg = tr.config
    tr2 = AdversarialTrainer(cfg, solver_episodes_per_layout=tr.solver_episodes, total_episodes=10,
                             save_dir=tr.save_dir, log_dir=tr.log_dir, n_envs=4, device=tr.device,
                             curriculum=tr.CURRICULUM)
    assert tr2.resume_from_checkpoint() == tr.global_episode
    for a, b in ((tr.solver.network, tr2.solver.network), (tr.architect.network, tr2.architect.network)):
        for k, v in a.state_dict().items():
            assert torch.equal(v, b.state_dict()[k]), k
    logs = json.load(open(os.path.join(tr.log_dir, "game_log.json")))
    assert len(logs) == len(tr.game_log)
    tr2.env.close()


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_c3_selfplay_4096_envs(gpu_device, tmp_path, precision):
    """BASELINE config 3: 4096 envs/GPU, 20x20, alternating Architect/Solver PPO, on the
    parity-default fp32 rollout (the reference's forward) and on the opt-in bf16 kernels."""
    n = 4096
    tr = _trainer(tmp_path, n, T=48, A=2, device=gpu_device, minibatch=16384, rollout_precision=precision)
    assert tr.solver.rollout_precision == precision
    rng = np.random.default_rng(3)
    valid = np.nonzero(tr.b_valid.cpu().numpy())[0]
    sample = rng.choice(valid, 32, replace=False)
    tr._trace = []
    from trainer_replay import oracle_envs
    envs = oracle_envs(tr, sample)
    arch0 = [p.detach().clone() for p in tr.architect.network.parameters()]
    out = tr.train_iteration()
    assert replay(tr, sample, tr._trace, envs) == 48 * 32
    assert out["layouts_scored"] > 0 and out["solver_updates"] == 3 * ((out["solver_samples"] + 16383) // 16384)
    assert np.isfinite(out["solver_policy_loss"]) and np.isfinite(out["architect_value_loss"])
    moved = [not torch.equal(a, b) for a, b in zip(arch0, tr.architect.network.parameters())]
    assert any(moved)  # the Architect took its step on the scored layouts
    _check_scored(tr)
    tr._trace = None
    out2 = tr.train_iteration()  # the re-laid-out envs play their new layouts
    assert out2["layouts_scored"] >= 0
    _check_scored(tr)
    _roundtrip(tr, tmp_path)


def test_c4_8192_envs_budget_40(gpu_device, tmp_path):
    """BASELINE config 4 on one GPU: 8192 envs, the c4 curriculum at its top (budget 40)."""
    n = 8192
    tr = _trainer(tmp_path, n, T=32, A=2, episode0=400, device=gpu_device, minibatch=16384,
                  curriculum="c4", rollout_precision="bf16")
    assert tr.get_curriculum_phase(401)[1] == 40 and tr.CURRICULUM == CURRICULA["c4"]
    assert tr.env.max_cams == 13 and tr.env.max_guards == 8
    budgets = {tr.b_meta[e][1] for e in range(0, n, 97)}
    assert budgets == {40}
    st = tr.env.export()
    assert int(st["n_guards"].max()) >= 2 and int(st["n_cams"].max()) >= 2
    valid = np.nonzero(tr.b_valid.cpu().numpy())[0]
    sample = np.random.default_rng(4).choice(valid, 32, replace=False)
    from trainer_replay import oracle_envs
    envs = oracle_envs(tr, sample)
    tr._trace = []
    out = tr.train_iteration()
    assert replay(tr, sample, tr._trace, envs) == 32 * 32
    assert np.isfinite(out["solver_value_loss"])
    _check_scored(tr)


def test_interactive_episodes_mask_training_envs(gpu_device, tmp_path):
    tr = _trainer(tmp_path, 16, R=12, T=40, A=2, device=gpu_device, minibatch=256)
    n_before = len(tr.game_log)
    frames = []
    res = tr.run_interactive_episodes(num_episodes=3, budget=9, solver_attempts=2,
                                      callback=lambda ep, m, st: frames.append((ep, m, st)))
    assert len(res) == 3
    assert set(res[0]) == {"solve_rate", "detection_rate", "timeout_rate", "architect_reward", "solver_reward",
                           "avg_steps", "budget", "phase"}
    new = [e.to_dict() for e in tr.game_log[n_before:]]
    assert all(e["is_interactive"] and e["budget"] == 9 for e in new)  # no training layout was scored meanwhile
    assert len(frames) == len(new) and all(f[1]["budget"] == 9 for f in frames)
    st = frames[-1][2]
    json.dumps(st)
    assert set(st) == {"grid", "visibility", "solver_pos", "solver_path", "vault_pos", "start_pos", "tick", "done",
                       "cameras", "guards", "detection_events"}
    assert tr.b_valid.any()  # training resumes on every env afterwards


def test_layout_batch_cadence_reference_buffers(gpu_device, tmp_path):
    """solver_cadence="layout_batch" (SURVEY 8 a20's parity mode): every env plays its
    layout's A attempts to done, and the one Solver update runs on exactly those
    transitions -- the reference's per-layout buffer (training.py:515-565) -- with GAE
    bootstrapping 0 at the buffer end and advantages normalised over the buffer
    (agents/solver.py:142-147, :228-244): equal to the oracle's GAE over each env's
    concatenated attempts, normalised in float32, within 1e-5; no V(s_T) bootstrap."""
    A = 3
    tr = _trainer(tmp_path, 24, R=12, T=40, A=A, device=gpu_device, minibatch=512, solver_cadence="layout_batch")
    ids = np.nonzero(tr.b_valid.cpu().numpy())[0]
    assert len(ids) >= 12
    from trainer_replay import oracle_envs
    envs = oracle_envs(tr, ids)
    tr._trace = []
    out = tr.train_iteration()
    assert replay(tr, ids, tr._trace, envs) == out["rollout_ticks"] * len(ids)
    ro, sel = tr._last_layout_batch
    assert ro.last_value is None  # bootstrap 0
    an, ret, e_i, t_i = (x.cpu().numpy() for x in tr.solver.last_layout_batch)
    r, v, d, s = (x.cpu().numpy() for x in (ro.rewards, ro.values, ro.dones, sel))
    assert out["solver_samples"] == len(an) == int(s[:, ids].sum())
    assert out["layouts_scored"] == len(ids)
    for e in ids:
        rows = np.nonzero(s[:, e])[0]
        assert len(rows) and rows[0] == 0 and np.all(np.diff(rows) == 1)  # one contiguous buffer from tick 0
        de = d[rows, e]
        assert de[-1] == 1 and int(de.sum()) == A  # exactly A attempts, the last one ended
        ref = po.gae(r[rows, e], v[rows, e], de)
        mine = e_i == e
        np.testing.assert_array_equal(t_i[mine], rows)
        np.testing.assert_allclose(ret[mine], ref + v[rows, e], rtol=0, atol=1e-5)
        if len(ref) > 1:
            ref32 = ref.astype(np.float32)
            refn = (ref32 - ref32.mean(dtype=np.float32)) / (np.float32(ref32.std(ddof=1, dtype=np.float32)) + np.float32(1e-8))
        else:
            refn = ref
        np.testing.assert_allclose(an[mine], refn, rtol=0, atol=1e-5)
    assert np.isfinite(out["solver_policy_loss"])


def test_interactive_episodes_more_than_envs(gpu_device, tmp_path):
    """num_episodes > n_envs: the layouts are played in blocks of n_envs, every one of them."""
    tr = _trainer(tmp_path, 6, R=10, T=30, A=1, device=gpu_device, minibatch=256)
    n_before = len(tr.game_log)
    res = tr.run_interactive_episodes(num_episodes=14, budget=5, solver_attempts=1, allow_cameras=False,
                                      allow_guards=False)
    assert len(res) == 14
    new = [e.to_dict() for e in tr.game_log[n_before:]]
    assert len(new) >= 14 and all(e["is_interactive"] for e in new)
    assert len({e["episode"] for e in new}) == len(new)


def test_per_layout_architect_updates(gpu_device, tmp_path):
    """architect_update="per_layout": one single-reward reference update per layout
    (agents/architect.py:91-155 with one reward) -- equal to replaying them one by one."""
    tr = _trainer(tmp_path, 64, R=12, T=40, A=1, device=gpu_device, minibatch=1024, architect_update="per_layout")
    import copy
    tr.solver.ppo_epochs = 1
    sd0 = copy.deepcopy(tr.architect.network.state_dict())
    ro = tr._rollout(40)
    tr._score_finished()
    A = tr.architect
    trip = sorted(zip(tr._arch_eps, [float(x) for x in torch.stack(A.log_probs)],
                      [float(x) for x in torch.stack([v.squeeze() for v in A.values])], list(A.rewards)))
    assert len(trip) > 1
    tr._architect_step()
    got = {k: v.clone() for k, v in A.network.state_dict().items()}
    from heist_amd.agents import ArchitectAgent
    ref = ArchitectAgent(grid_rows=12, grid_cols=12, device=gpu_device)
    ref.network.load_state_dict(sd0)
    for _, lp, v, r in trip:
        ref.log_probs.append(torch.tensor(lp, device=gpu_device))
        ref.values.append(torch.tensor(v, device=gpu_device))
        ref.rewards.append(r)
        ref.update()
    # the trainer replays the updates from a HIP graph (ArchitectAgent.update_sequence):
    # equal to the eager replay within Adam-amplified fp32 noise (test_architect_update.py)
    for k, v in ref.network.state_dict().items():
        torch.testing.assert_close(got[k], v, rtol=0, atol=1e-5)
    del ro
