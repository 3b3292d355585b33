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
    # CU theft: the Architect's sequence holds 64 whole CUs while the Solver's update runs on
    # the rest.  The update by HIP events on the main stream, alone (the Architect's sequence
    # after it) and with the sequence launched just before it on the side stream (the
    # iteration's order); the sequence by events on its own stream.
    main = torch.cuda.current_stream(dev)
    theft = {}
    for mode in ("alone", "beside_architect", "alone", "beside_architect"):
        ro = tr._rollout(T)
        done = tr._score_finished()
        k = len(tr.architect.rewards)
        torch.cuda.synchronize()
        side = tr.architect.side_stream()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        pend = None
        if mode == "beside_architect" and side is not None:
            side.wait_stream(main)
            for buf in (tr.architect.log_probs, tr.architect.values):
                ts = buf.tensors() if hasattr(buf, "tensors") else [x for x in buf if torch.is_tensor(x)]
                for t_ in ts:
                    if t_.is_cuda:
                        t_.record_stream(side)
            with torch.cuda.stream(side):
                e[2].record(side)
                pend = tr._architect_step(defer=True, join=main)
                e[3].record(side)
        e[0].record(main)
        tr.solver.update_rollout(ro, minibatch=mb)
        e[1].record(main)
        torch.cuda.synchronize()
        row = {"solver_update_ms": e[0].elapsed_time(e[1]), "architect_updates": k}
        if pend is not None:
            pend()
            row["architect_ms"] = e[2].elapsed_time(e[3])
        else:
            t0 = time.perf_counter()
            tr._architect_step()
            torch.cuda.synchronize()
            row["architect_ms_serial_wall"] = (time.perf_counter() - t0) * 1e3
        tr._arch_eps = []
        tr._assign_layouts(done)
        theft.setdefault(mode, []).append(row)
    res["cu_theft"] = theft
    res["rollout_steps_per_s"] = n * T / res["rollout_s"]
    res["train_steps_per_s"] = n * T / res["iteration_s"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
