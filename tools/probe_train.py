"""Timing probe for one batched training iteration at 4096 envs: rollout (env + fused
policy + bookkeeping) vs PPO update vs the rest.  One JSON line."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from heist_amd import EnvironmentConfig  # noqa: E402
from heist_amd.training import AdversarialTrainer  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n = int(os.environ.get("PROBE_N", "4096"))
    T = int(os.environ.get("PROBE_T", "32"))
    mb = int(os.environ.get("PROBE_MB", "16384"))
    d = tempfile.mkdtemp()
    tr = AdversarialTrainer(EnvironmentConfig(), solver_episodes_per_layout=4, total_episodes=10 ** 9, save_dir=d,
                            log_dir=d, n_envs=n, rollout_len=T, minibatch=mb, device=dev, seed=0)
    tr.global_episode = int(os.environ.get("PROBE_EPISODE", "200"))  # bench.py's measure_train phase
    tr._assign_layouts(np.arange(n))
    tr.train_iteration()
    torch.cuda.synchronize()
    res = {"n": n, "T": T, "minibatch": mb}
    t0 = time.perf_counter()
    ro = tr._rollout(T)
    torch.cuda.synchronize()
    res["rollout_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    tr.solver.update_rollout(ro, minibatch=mb)
    torch.cuda.synchronize()
    res["update_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    tr.train_iteration()
    torch.cuda.synchronize()
    res["iteration_s"] = time.perf_counter() - t0
    # one iteration's parts, in train_iteration's order
    parts = {}
    t0 = time.perf_counter()
    ro = tr._rollout(T)
    torch.cuda.synchronize()
    parts["rollout"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    tr.solver.update_rollout(ro, minibatch=mb)
    torch.cuda.synchronize()
    parts["solver_update"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    done_ids = tr._score_finished()
    torch.cuda.synchronize()
    parts["score"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    tr._architect_step()
    tr._arch_eps = []
    torch.cuda.synchronize()
    parts["architect_updates"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    tr._assign_layouts(done_ids)
    torch.cuda.synchronize()
    parts["assign_layouts"] = time.perf_counter() - t0
    res["architect_updates_per_iteration"] = len(tr.architect.rewards)
    t0 = time.perf_counter()
    tr.train_iteration()  # the loop's own order: Solver update and Architect sequence overlapped
    torch.cuda.synchronize()
    parts["train_iteration_overlapped"] = time.perf_counter() - t0
    res["parts_s"] = parts
    res["layouts_scored"] = int(len(done_ids))
    res["rollout_steps_per_s"] = n * T / res["rollout_s"]
    res["train_steps_per_s"] = n * T / res["iteration_s"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
