"""Headline benchmark: Solver env-steps/sec at 20x20, 4096 envs/GPU (BASELINE.json metric).

One "step" = one heist_step launch over all envs of the rank: move, camera/guard
update, raycast visibility, reward/termination, in-kernel auto-reset, and the
[N,3,20,20] float32 observation write.  Inputs (layouts, per-step actions) are
resident in HBM before the timed region.  Multi-GPU: one process per GPU (torchrun),
envs sharded by rank with no data-path collective (weak scaling); the only RCCL
calls are the barrier and the max-over-ranks of the elapsed time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 4096] [--no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")
sys.path[:0] = [ROOT, PKG]

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "Solver env-steps/sec at 20×20, 4096 envs/GPU, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(msg):
    """Progress on stderr (stdout carries only the one JSON result line)."""
    print("[bench %s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def algorithmic_bytes_per_env_step(R, C, ncam, nguard):
    """obs f32 write + grid u8 read + action i64 + reward f32 + done + status
    + read and write of the dynamic per-env state (24 + 8*ncam + 12*nguard bytes)."""
    return 12 * R * C + R * C + 8 + 4 + 1 + 1 + 2 * (24 + 8 * ncam + 12 * nguard)


def cpu_baseline(layouts, cfg, budget, target_s=10.0, threads=1):
    """The C oracle (restatement of the reference CPU path) on a bounded sample of the
    same workload: env.step + get_state_tensor with random actions, auto-reset."""
    from oracle import pyoracle as po
    sample = layouts[:256]

    def make():
        envs = []
        for lay in sample:
            o = po.OracleEnv(cfg.grid_rows, cfg.grid_cols, cfg.max_steps, cfg.start_pos, cfg.vault_pos, budget)
            o.set_layout(*lay)
            o.reset()
            envs.append(o)
        return envs

    envs = make()
    t0 = time.perf_counter()
    n = po.run_random(envs, 4, seed=1, n_threads=threads)
    dt = time.perf_counter() - t0
    steps = max(4, int(4 * target_s / max(dt, 1e-6)))
    envs = make()
    t0 = time.perf_counter()
    n = po.run_random(envs, steps, seed=2, n_threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": "%d of the same synthetic 20x20 layouts x %d ticks (%d env-steps, %.1f s), random actions, "
                      "auto-reset, state tensor each tick; C oracle (oracle/heist_oracle.c) with host libm"
                      % (len(sample), steps, n, dt)}


def measure_rollout(env, dev, steps=20, warmup=3):
    """env step + batched Solver select_action on the fused kernels (carried LSTM state)."""
    from heist_amd.agents import SolverAgent
    ag = SolverAgent(env.rows, env.cols, device=dev)
    h = c = torch.zeros(1, env.n_envs, 128, device=dev)
    for k in range(warmup + steps):
        if k == warmup:
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
        a, lp, v, (h, c) = ag.act(env.obs, (h, c))
        env.step(a)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    return {"value": steps * env.n_envs / dt, "unit": "env-steps/s", "ms_per_step": dt / steps * 1e3,
            "dtype": "bf16 MFMA policy (fp32 accumulate)",
            "note": "heist_step + fused Solver select_action (backbone + head kernels), carried LSTM state"}


def measure_env_config(dev, R, n, budget, steps=100, warmup=10, **kw):
    """env-only heist_step at another BASELINE config (C4: 8192 envs/GPU at the top of the
    budget schedule; C5: 2048 envs/GPU, 32x32, exactly 4 cameras + 3 guards), timed like
    the headline number (HIP events around `steps` launches)."""
    from heist_amd import EnvironmentConfig, HeistEnv
    from heist_amd.layouts import valid_synthetic_layouts
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R, max_steps=200, architect_budget=budget)
    # capacity for whatever the budget can buy (cameras cost 3, guards 5: budget.py:13-17)
    env = HeistEnv(n, cfg, max_cams=budget // 3, max_guards=budget // 5, max_path=16, device=dev, auto_reset=True)
    lays = valid_synthetic_layouts(env, budget, seed=99, **kw)
    env.reset()
    acts = torch.randint(0, 5, (warmup + steps, n), device=dev, dtype=torch.int64)
    for k in range(warmup):
        env.step(acts[k])
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    e0.record(st)
    for k in range(steps):
        env.step(acts[warmup + k])
    e1.record(st)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    ncam = float(np.mean([len(c) for _, c, _ in lays]))
    ngu = float(np.mean([len(g) for _, _, g in lays]))
    b = algorithmic_bytes_per_env_step(R, R, ncam, ngu)
    gbs = b * n / (ms * 1e-3) / 1e9
    return {"value": n / (ms * 1e-3), "unit": "env-steps/s", "kernel_ms": ms, "envs": n, "grid": "%dx%d" % (R, R),
            "budget": budget, "mean_cameras": ncam, "mean_guards": ngu,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_env_step": b}}


SOLVER_BACKBONE_FLOP = 2 * 400 * (32 * 27 + 64 * 288 + 64 * 576)  # conv1..3 MACs x 2 at 20x20, per env
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md)


def measure_policy(dev, n, iters=50, warmup=5):
    """Batched Solver select_action on the fused kernels (heist_solver_features +
    heist_solver_head) and the backbone kernel alone, timed with HIP events."""
    from heist_amd.agents import SolverAgent
    ag = SolverAgent(20, 20, device=dev)
    net = ag.network
    obs = torch.rand(n, 3, 20, 20, device=dev)
    h = c = torch.zeros(1, n, 128, device=dev)
    st = torch.cuda.current_stream(dev)

    def timed(fn):
        for _ in range(warmup):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(iters):
            fn()
        b.record(st)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) / iters
    ms_bb = timed(lambda: net.features_fused(obs))
    ms_act = timed(lambda: ag.act(obs, (h, c)))
    tf = SOLVER_BACKBONE_FLOP * n / (ms_bb * 1e-3) / 1e12
    return {"value": n / (ms_act * 1e-3), "unit": "env-steps/s", "ms_per_step": ms_act,
            "dtype": "bf16 MFMA (fp32 accumulate)",
            "note": "batched SolverAgent.act: fused conv backbone + fc/LSTM/heads/sample kernels",
            "backbone_roofline": {"bound": "mfma", "kernel": "heist::solver_conv_kernel<20,20>",
                                  "kernel_ms": ms_bb, "achieved": tf, "peak": MFMA_BF16_PEAK_TFLOPS,
                                  "unit": "TFLOP/s", "frac": tf / MFMA_BF16_PEAK_TFLOPS,
                                  "flop_per_env": SOLVER_BACKBONE_FLOP}}


def measure_train(cfg, dev, n_envs, rollout_len=32, minibatch=16384, update_precision="fp32"):
    """Batched AdversarialTrainer iteration: rollout + heist_gae + adv-norm + 3 PPO epochs
    (heist_ppo_loss, Adam) + Architect scoring/update/re-layout."""
    from heist_amd.training import AdversarialTrainer
    import tempfile
    d = tempfile.mkdtemp()
    tr = AdversarialTrainer(cfg, solver_episodes_per_layout=4, total_episodes=10 ** 9, save_dir=d, log_dir=d,
                            n_envs=n_envs, rollout_len=rollout_len, minibatch=minibatch, device=dev, seed=0,
                            update_precision=update_precision)
    tr._assign_layouts(np.arange(n_envs))
    log("  warm-up iteration")
    tr.train_iteration()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    tr.train_iteration()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    return {"value": rollout_len * n_envs / dt, "unit": "env-steps/s", "s_per_iteration": dt,
            "config": "T=%d x %d envs, 3 epochs, minibatch %d; rollout policy bf16 fused kernels, PPO update %s "
                      "(NHWC MIOpen convs)" % (rollout_len, n_envs, minibatch, update_precision)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--budget", type=int, default=15)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-secondary", action="store_true", help="skip the rollout / full-train numbers")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = torch.distributed
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from heist_amd import EnvironmentConfig, HeistEnv
    from heist_amd.layouts import valid_synthetic_layouts

    cfg = EnvironmentConfig(grid_rows=20, grid_cols=20, max_steps=200, architect_budget=args.budget)
    N = args.envs
    env = HeistEnv(N, cfg, max_cams=8, max_guards=4, max_path=16, device=dev, auto_reset=True)
    layouts = valid_synthetic_layouts(env, args.budget, seed=1234 + rank)
    env.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(4321 + rank)
    actions = torch.randint(0, 5, (args.warmup + args.steps, N), device=dev, generator=gen, dtype=torch.int64)
    stream = torch.cuda.current_stream(dev)

    for k in range(args.warmup):
        env.step(actions[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # HIP events bracket the timed launches on the stream they run on; their span / K is the
    # mean launch duration (it includes the small inter-launch gaps, so it is conservative)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for k in range(args.steps):
        env.step(actions[args.warmup + k])
    e1.record(stream)
    issue_s = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / args.steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ALU work figure: ray samples evaluated per env-step, counted by the
    # kernel on extra steps after the timed region
    cnt = torch.zeros(N, dtype=torch.int64, device=dev)
    cnt_x = torch.zeros(N, dtype=torch.int64, device=dev)
    env.count_samples(cnt)
    env.count_exact_rays(cnt_x)
    n_count = 8
    for k in range(n_count):
        env.step(actions[k])
    env.count_samples(None)
    env.count_exact_rays(None)
    samples_per_step = float(cnt.sum().item()) / (n_count * N)
    exact_rays_per_step = float(cnt_x.sum().item()) / (n_count * N)

    ncam = float(np.mean([len(c) for _, c, _ in layouts]))
    ngu = float(np.mean([len(g) for _, _, g in layouts]))
    b_step = algorithmic_bytes_per_env_step(20, 20, ncam, ngu)
    achieved = b_step * N / (kern_ms * 1e-3) / 1e9  # GB/s, per launch / launch duration
    total_steps = args.steps * N * world
    value = total_steps / elapsed

    if rank == 0:
        traffic = None
        tf = os.path.join(ROOT, "profiles", "heist_step_traffic.json")
        if os.path.exists(tf) and N == 4096:
            with open(tf) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        line = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "env-only heist_step, 20x20 grid, %d envs/GPU, synthetic budget-%d layouts "
                                   "(mean %.2f cameras, %.2f guards/env), uniform random actions, auto-reset"
                                   % (N, args.budget, ncam, ngu),
                       "envs_per_gpu": N, "grid": "20x20", "parallelism": "env-sharded x%d" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "heist::step_kernel", "kernel_ms": kern_ms,
                         "algorithmic_bytes_per_env_step": b_step,
                         "ray_samples_per_env_step": samples_per_step,
                         "exact_path_rays_per_env_step": exact_rays_per_step,
                         "host_issue_us_per_step": issue_s / args.steps * 1e6},
            "cpu_baseline": None,
        }
        log("env-only: %.1f M env-steps/s, step kernel %.1f us" % (value / 1e6, kern_ms * 1e3))
        # single-GPU figures: the secondary numbers and the CPU baseline run on rank 0 at N=1
        # only (at N>1 the other ranks would idle at the closing barrier meanwhile)
        if not args.no_secondary and world == 1:
            sec = {}
            log("env-only at the other BASELINE configs")
            sec["env_only_c4_8192envs_budget40"] = measure_env_config(dev, 20, 8192, 40)
            sec["env_only_c5_32x32_2048envs_4cams_3guards"] = measure_env_config(dev, 32, 2048, 40, n_cams=4,
                                                                                 n_guards=3)
            log("rollout")
            sec["rollout"] = measure_rollout(env, dev)
            log("policy inference")
            sec["policy_inference"] = measure_policy(dev, N)
            log("full train (fp32 update)")
            sec["full_train"] = measure_train(cfg, dev, N)
            log("full train (bf16 update)")
            sec["full_train_bf16_update"] = measure_train(cfg, dev, N, update_precision="bf16")
            line["secondary"] = sec
        if not args.no_cpu_baseline and world == 1:
            log("cpu baseline")
            line["cpu_baseline"] = cpu_baseline(layouts, cfg, args.budget, target_s=args.cpu_seconds, threads=1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
