"""Headline benchmark: Solver env-steps/sec at 20x20, 4096 envs/GPU (BASELINE.json metric).

One "step" = one env tick over all envs of the rank: move, camera/guard update, raycast
visibility, reward/termination, in-kernel auto-reset, and the [N,3,20,20] float32
observation write, reward, done and status of that tick to HBM.  The timed ticks run in
heist_step_multi launches of K = --ticks-per-launch ticks each (default 20; named in
config.workload), K = 1 being one heist_step launch per tick (also reported as the
secondary env_only_single_tick).  Inputs (layouts, per-tick actions) are resident in HBM
before the timed region, and every launch's arguments are resolved before it.  The headline layouts are BASELINE config 2's:
sampled at temperature 1.0 and budget 15 from the fixed Architect checkpoint
(checkpoints/architect_c2_fixed.pt, tools/mint_architect_checkpoint.py), resampled until
BFS-valid; the round-1 synthetic mix (SURVEY 8d generator (ii)) is a secondary line.
Multi-GPU: one process per GPU, envs sharded by rank with no data-path collective (weak
scaling); the only RCCL calls are the barrier and the max-over-ranks of the elapsed time.
`--gpus N` without torchrun's WORLD_SIZE spawns the N ranks itself (before any GPU call);
under torchrun WORLD_SIZE must equal N.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 4096] [--no-cpu-baseline]
                    [--no-secondary] [--backend nccl|gloo] [--train-envs 8192]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd")
sys.path[:0] = [ROOT, PKG]
# MIOpen's find results and compiled kernels for the full-train secondaries' convolutions
# (miopen_cache/, recorded by a bench run on MI355X): without them a fresh box spends
# ~2 min per precision searching solvers before the first PPO update
for _k, _v in (("MIOPEN_USER_DB_PATH", "miopen_cache"), ("MIOPEN_CUSTOM_CACHE_DIR", "miopen_cache")):
    os.environ.setdefault(_k, os.path.join(ROOT, _v))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "Solver env-steps/sec at 20×20, 4096 envs/GPU, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(msg):
    """Progress on stderr (stdout carries only the one JSON result line)."""
    print("[bench %s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def multi_kernel_name(kcfg, R, C):
    """The K-tick launch's kernel: the lean one-wave kernel for 20 x 20 grids at one wave per env
    and for 32 x 32 grids (heist_env.hip step_lean_kernel; envs it cannot serve take the generic
    body inside the same launch), else step_multi_kernel."""
    lean = kcfg.get("lean", 0) and ((kcfg.get("multi_waves") == 1 and R == 20 and C == 20) or (R == 32 and C == 32))
    return "heist::step_lean_kernel" if lean else "heist::step_multi_kernel"


def algorithmic_bytes_per_env_step(R, C, ncam, nguard):
    """obs f32 write + grid u8 read + action i64 + reward f32 + done + status
    + read and write of the dynamic per-env state (24 + 8*ncam + 12*nguard bytes)."""
    return 12 * R * C + R * C + 8 + 4 + 1 + 1 + 2 * (24 + 8 * ncam + 12 * nguard)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(layouts, cfg, budget, target_s=10.0, threads=1):
    """The C oracle (restatement of the reference CPU path) on a bounded sample of the
    same workload: env.step + get_state_tensor with random actions, auto-reset; one
    pthread per core over disjoint envs when threads > 1."""
    from oracle import pyoracle as po
    sample = layouts[:max(256, 16 * threads)]

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
    out = {"value": n / dt, "unit": "env-steps/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
           "host_cpus": os.cpu_count(),
            "sample": "%d of the bench's layouts x %d ticks (%d env-steps, %.1f s wall), random actions, "
                      "auto-reset, state tensor each tick; C oracle (oracle/heist_oracle.c, host libm), %d thread%s"
                      % (len(sample), steps, n, dt, threads, "s" if threads > 1 else "")}
    rf = os.path.join(ROOT, "profiles", "cpu_ratio.json")
    if os.path.exists(rf):  # tools/cpu_ratio.py: C oracle vs the Python reference on one build-container core
        with open(rf) as f:
            ratio = json.load(f)["oracle_over_reference"]
        out["python_reference_equivalent"] = {
            "value": out["value"] / ratio, "unit": "env-steps/s", "oracle_over_reference": ratio, "estimate": True,
            "source": "profiles/cpu_ratio.json (tools/cpu_ratio.py: same layouts, one core of the build container)",
            "note": "derived, not timed here: this host's C-oracle rate divided by the oracle / Python-reference "
                    "speed ratio measured on another machine (the reference itself cannot run on the GPU box)"}
    return out


def architect_layouts(env, budget, seed, ckpt=None):
    """BASELINE config 2's layouts (heist_amd.layouts.architect_checkpoint_layouts): the
    fixed Architect checkpoint sampled at T = 1.0, every env resampled until BFS-valid."""
    from heist_amd.layouts import architect_checkpoint_layouts
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import mint_architect_checkpoint as mint
    path = ckpt or mint.DEFAULT
    if not os.path.exists(path):
        mint.mint(path)
    return architect_checkpoint_layouts(env, budget, seed, path)


def shared_fan_fraction(cam_params, n_cams):
    """Share of the envs with cameras whose cameras all cast the shared fan (heist_env.hip
    fan_kernel: the K-tick kernel takes a camera direction group's rays from the table when
    its emitter equals the table's, i.e. every camera has the (fov, heading, speed, range) of
    the first env's first camera, range <= 6).  Architect batches share one camera parameter
    set per forward (reference networks.py:283-322); the synthetic mix draws its own per
    camera.  cam_params [N, max_cams, 6] (row, col, fov, heading, speed, range), n_cams [N]."""
    cp, nc = np.asarray(cam_params, np.float64), np.asarray(n_cams)
    has = nc > 0
    if not has.any():
        return 0.0
    e0 = int(np.nonzero(has)[0][0])
    ref = cp[e0, 0, 2:6]
    if ref[3] > 6:
        return 0.0
    served = [bool(np.all(cp[e, :nc[e], 2:6] == ref)) for e in np.nonzero(has)[0]]
    return float(np.mean(served))


def synthetic_fan_fraction(layouts, env, budget):
    """shared_fan_fraction of layouts in the reference's list format."""
    from heist_amd.vec_env import LayoutBatch
    lb = LayoutBatch.from_lists(layouts, budget, env.max_cams, env.max_guards, env.max_path, "cpu", env.rows, env.cols)
    return shared_fan_fraction(lb.cam_params.numpy(), lb.n_cams.numpy())


def measure_fan_fill(env, actions, K, bufs, reps=5):
    """The shared fan table's fill (fan_kernel: kFanTicks = 1,024 entries, run on the launch's
    stream before a K-tick launch that finds the table stale) priced by HIP events: a K-tick
    launch after the table was marked stale minus the same launch reading the table.  The
    timed ticks read a table an earlier launch filled; amortised over the 1,024 ticks one fill
    serves, its cost per tick is fill / 1,024."""
    stream = torch.cuda.current_stream(env.device)
    acts = actions[:K]

    def one(stale):
        if stale:
            env.set_ray_mode(env.kernel_config()["ray_mode"])  # marks the table stale (heist_set_ray_mode)
        launch = env.step_multi_launcher(K, acts, *bufs)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        launch()
        b.record(stream)
        torch.cuda.synchronize(env.device)
        return a.elapsed_time(b)
    one(False)
    fill = [one(True) for _ in range(reps)]
    plain = [one(False) for _ in range(reps)]
    return max(0.0, float(np.median(fill) - np.median(plain)))


def time_env(env, actions, warmup, steps, K, world, settle_ms=0.0, extra_windows=0):
    """Time `steps` env ticks over all envs after `warmup` untimed ones: K = 1 one heist_step
    launch per tick, K > 1 heist_step_multi launches of K ticks (the last one shorter), every
    tick's observation rows going to an [K, N, 3, R, C] buffer.  HIP events bracket the
    timed launches on the stream they run on, so their span / steps is the mean tick
    duration (inter-launch gaps included); the wall clock runs between two barriers and at
    N > 1 is the max over ranks.  K > 1: an untimed clock-settle phase of settle_ms of K-tick
    launches precedes the window (then the fan table is refilled by the warm-up ticks, as
    without it), and extra_windows more windows (HIP events only) give the spread
    (time_env.windows).  Returns (elapsed_s, kernel_ms_per_tick, issue_s, launches)."""
    dev, N = env.device, env.n_envs
    dist = torch.distributed
    stream = torch.cuda.current_stream(dev)
    if K > 1:
        shape = (K, N, 3, env.rows, env.cols)
        bufs = (torch.empty(shape, dtype=torch.float32, device=dev), torch.empty((K, N), device=dev),
                torch.empty((K, N), dtype=torch.uint8, device=dev), torch.empty((K, N), dtype=torch.int8, device=dev))

        def prepare(k0, n):  # the launches of ticks k0 .. k0+n-1, arguments resolved before any timing
            return [env.step_multi_launcher(min(K, n - j), actions[k0 + j:k0 + j + min(K, n - j)], *bufs)
                    for j in range(0, n, K)]

        def run(k0, n, ready=None):
            ls = ready if ready is not None else prepare(k0, n)
            for launch in ls:
                launch()
            return len(ls)
    else:
        bufs = None

        def prepare(k0, n):
            return None

        def run(k0, n, ready=None):
            for k in range(n):
                env.step(actions[k0 + k])
            return n
    run(0, warmup)
    time_env.settle = None
    if K > 1 and settle_ms > 0:
        # clock settle (untimed): K-tick launches on the same handle for settle_ms, so the
        # timed window does not start on a cold / boosting clock; then the shared fan table is
        # marked stale and the warm-up launches refill it, so the timed launches read the table
        # at the same offsets as without the settle phase (no refill inside the window)
        settle = prepare(0, K)
        torch.cuda.synchronize(dev)
        ts = time.perf_counter()
        n_settle = 0
        while (time.perf_counter() - ts) * 1e3 < settle_ms or n_settle < 8:
            for launch in settle:
                launch()
            n_settle += 1
            if n_settle % 16 == 0:
                torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        env.set_ray_mode(env.kernel_config()["ray_mode"])  # marks the fan table stale (heist_set_ray_mode)
        run(0, warmup)
        time_env.settle = {"launches": n_settle, "ms": (time.perf_counter() - ts) * 1e3}
    ready = prepare(warmup, steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)  # a marker on the idle stream (no work): the wall clock starts after its host call
    t0 = time.perf_counter()
    launches = run(warmup, steps, ready)
    e1.record(stream)
    issue_s = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    if world > 1:  # one rank: no barrier, so the one synchronize closes the window
        dist.barrier()
        torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / steps
    windows = []
    for _ in range(extra_windows if K > 1 else 0):
        # the same window again (after the same stale-table warm-up), HIP events only: the
        # spread of the headline's kernel time on this box
        env.set_ray_mode(env.kernel_config()["ray_mode"])
        run(0, warmup)
        ready_x = prepare(warmup, steps)
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        run(warmup, steps, ready_x)
        b.record(stream)
        torch.cuda.synchronize(dev)
        windows.append(a.elapsed_time(b) / steps)
    time_env.windows = windows
    per_rank = [(elapsed, kern_ms)]
    if world > 1:  # every rank's wall time and kernel time per tick; the line's time is the max
        t = torch.zeros((world, 2), dtype=torch.float64, device=dev)
        t[dist.get_rank()] = torch.tensor([elapsed, kern_ms], dtype=torch.float64)
        dist.all_reduce(t)
        per_rank = [tuple(r) for r in t.tolist()]
        elapsed = max(r[0] for r in per_rank)
    time_env.last_bufs = bufs if K > 1 else None
    time_env.per_rank = per_rank
    return elapsed, kern_ms, issue_s, launches


def measure_rollout(env, dev, steps=20, warmup=3, precision="bf16"):
    """env step + batched Solver select_action (carried LSTM state): "bf16" on the fused
    kernels (opt-in), "fp32" on the reference's fp32 forward (the parity default)."""
    from heist_amd.agents import SolverAgent
    ag = SolverAgent(env.rows, env.cols, device=dev, rollout_precision=precision)
    h = c = torch.zeros(1, env.n_envs, 128, device=dev)
    for k in range(warmup + steps):
        if k == warmup:
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
        a, lp, v, (h, c) = ag.act(env.obs, (h, c))
        env.step(a)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    tf = solver_backbone_flop(env.rows) * steps * env.n_envs / dt / 1e12  # rollout MFMA fraction
    peak = MFMA_BF16_PEAK_TFLOPS if precision == "bf16" else MFMA_FP32_PEAK_TFLOPS
    return {"value": steps * env.n_envs / dt, "unit": "env-steps/s", "ms_per_step": dt / steps * 1e3,
            "mfma_roofline": {"achieved": tf, "peak": peak, "unit": "TFLOP/s", "frac": tf / peak,
                              "peak_dtype": precision,
                              "note": "algorithmic conv-backbone flops of the policy forward per env-step"},
            "dtype": "bf16 MFMA policy (fp32 accumulate)" if precision == "bf16" else
                     "fp32 policy (exact-fp32 MFMA conv backbone)",
            "note": ("heist_step + fused Solver select_action (backbone + head kernels)" if precision == "bf16" else
                     "heist_step + fp32 select_action (conv backbone on the fp32-MFMA training kernels at "
                     "20x20, fused-gate LSTM; the fp32 matrix peak bounds it at ~3.5 M env-steps/s)") +
                    ", carried LSTM state"}


def measure_env_config(dev, R, n, budget, steps=100, warmup=10, K=1, **kw):
    """env-only throughput at another BASELINE config (C4: 8192 envs/GPU at the top of the
    budget schedule; C5: 2048 envs/GPU, 32x32, exactly 4 cameras + 3 guards), timed like
    the headline (time_env: K ticks per launch)."""
    from heist_amd import EnvironmentConfig, HeistEnv
    from heist_amd.layouts import valid_synthetic_layouts
    cfg = EnvironmentConfig(grid_rows=R, grid_cols=R, max_steps=200, architect_budget=budget)
    # capacity for whatever the budget can buy (cameras cost 3, guards 5: budget.py:13-17)
    env = HeistEnv(n, cfg, max_cams=max(1, budget // 3), max_guards=max(1, budget // 5), max_path=16, device=dev,
                   auto_reset=True)
    if kw.pop("architect", False):
        lb, _ = architect_layouts(env, budget, seed=99)
        fan = shared_fan_fraction(lb.cam_params.cpu().numpy(), lb.n_cams.cpu().numpy())
    else:
        fan = synthetic_fan_fraction(valid_synthetic_layouts(env, budget, seed=99, **kw), env, budget)
    env.reset()
    acts = torch.randint(0, 5, (warmup + steps, n), device=dev, dtype=torch.int64)
    K = max(1, min(K, steps))
    _, ms, _, _ = time_env(env, acts, warmup, steps, K, 1, settle_ms=10.0)
    cnt = torch.zeros(n, dtype=torch.int64, device=dev)  # ray samples per env-step (SURVEY 8(d)'s ALU figure)
    env.count_samples(cnt)
    n_count = 20
    for k in range(n_count):
        env.step(acts[k])
    env.count_samples(None)
    samples = float(cnt.sum().item()) / (n_count * n)
    st = env.export()
    ncam, ngu = float(st["n_cams"].double().mean()), float(st["n_guards"].double().mean())
    b = algorithmic_bytes_per_env_step(R, R, ncam, ngu)
    gbs = b * n / (ms * 1e-3) / 1e9
    kcfg = env.kernel_config()
    kname = multi_kernel_name(kcfg, R, R) if K > 1 else "heist::step_kernel"
    env.close()
    return {"value": n / (ms * 1e-3), "unit": "env-steps/s", "kernel_ms": ms, "envs": n, "grid": "%dx%d" % (R, R),
            "budget": budget, "mean_cameras": ncam, "mean_guards": ngu, "ticks_per_launch": K,
            "shared_fan_frac": fan, "waves_per_env": kcfg["lean_waves"] if R == 32 and kcfg["lean"] else 1,
            "ray_samples_per_env_step": samples, "ray_samples_per_s": samples * n / (ms * 1e-3),
            "kernel": kname,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_env_step": b}}


def solver_backbone_flop(R):  # conv1..3 MACs x 2 per env at R x R (algorithmic, no band halo)
    return 2 * R * R * (32 * 27 + 64 * 288 + 64 * 576)


SOLVER_BACKBONE_FLOP = solver_backbone_flop(20)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md)
MFMA_FP32_PEAK_TFLOPS = 157.3   # MI355X fp32 matrix (v_mfma_f32_*_f32)


def measure_policy(dev, n, iters=50, warmup=5, R=20, settle_ms=100.0):
    """Batched Solver select_action on the fused kernels (heist_solver_features +
    heist_solver_head) and the backbone kernel alone, timed with HIP events.  R = 32 runs
    the row-band backbone (BASELINE C5's grid).  Each timed form runs after an untimed
    clock-settle phase of settle_ms (as time_env's): the setup before it leaves the GPU
    idle, and a 4096-env backbone launch timed from idle measured 0.184-0.19 ms against
    0.158 ms once the clock had ramped (profiles/r05az_backbone_sweep.log)."""
    from heist_amd.agents import SolverAgent
    ag = SolverAgent(R, R, device=dev, rollout_precision="bf16")
    net = ag.network
    obs = torch.rand(n, 3, R, R, device=dev)
    h = c = torch.zeros(1, n, 128, device=dev)
    st = torch.cuda.current_stream(dev)

    settle = {}

    def timed(fn):
        for _ in range(warmup):
            fn()
        ts, k = time.perf_counter(), 0
        while (time.perf_counter() - ts) * 1e3 < settle_ms:
            fn()
            k += 1
            if k % 8 == 0:
                torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        settle[fn] = k
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(iters):
            fn()
        b.record(st)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) / iters
    f_bb, f_act = (lambda: net.features_fused(obs)), (lambda: ag.act(obs, (h, c)))
    ms_bb = timed(f_bb)
    ms_act = timed(f_act)
    tf = solver_backbone_flop(R) * n / (ms_bb * 1e-3) / 1e12
    kern = "heist::solver_conv_kernel<20,20>" if R == 20 else "heist::solver_conv_band_kernel<32,8>"
    return {"value": n / (ms_act * 1e-3), "unit": "env-steps/s", "ms_per_step": ms_act, "envs": n,
            "grid": "%dx%d" % (R, R), "dtype": "bf16 MFMA (fp32 accumulate)",
            "note": "batched SolverAgent.act: fused conv backbone + fc/LSTM/heads/sample kernels",
            "clock_settle": {"ms": settle_ms, "act_calls": settle[f_act], "backbone_calls": settle[f_bb]},
            "backbone_roofline": {"bound": "mfma", "kernel": kern,
                                  "kernel_ms": ms_bb, "achieved": tf, "peak": MFMA_BF16_PEAK_TFLOPS,
                                  "unit": "TFLOP/s", "frac": tf / MFMA_BF16_PEAK_TFLOPS,
                                  "flop_per_env": solver_backbone_flop(R)}}


def measure_train(cfg, dev, n_envs, rollout_len=32, minibatch=16384, update_precision="fp32",
                  rollout_precision="fp32", curriculum=None, episode0=200, iters=1):
    """Batched AdversarialTrainer iterations (self-play at the curriculum phase of episode0):
    rollout + heist_gae (V(s_T) bootstrap) + adv-norm + 3 PPO epochs (heist_ppo_loss, Adam;
    inside a process group every optimizer step averages the Solver's gradients with one
    flat all-reduce) + Architect scoring/update/re-layout.  Collective at N > 1: every rank
    runs it; the time is the max over ranks between two barriers and the value counts the
    env-steps of all ranks."""
    from heist_amd.training import AdversarialTrainer
    import tempfile
    dist = torch.distributed
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    world = dist.get_world_size() if multi else 1
    d = tempfile.mkdtemp()
    tr = AdversarialTrainer(cfg, solver_episodes_per_layout=4, total_episodes=10 ** 9, save_dir=d, log_dir=d,
                            n_envs=n_envs, rollout_len=rollout_len, minibatch=minibatch, device=dev, seed=0,
                            update_precision=update_precision, rollout_precision=rollout_precision,
                            curriculum=curriculum)
    tr.global_episode = episode0
    tr._assign_layouts(np.arange(n_envs))
    log("  warm-up iteration")
    tr.train_iteration()
    torch.cuda.synchronize(dev)
    if multi:
        dist.barrier()
    t0 = time.perf_counter()
    outs = [tr.train_iteration() for _ in range(iters)]
    torch.cuda.synchronize(dev)
    if multi:
        dist.barrier()
    dt = time.perf_counter() - t0
    if multi:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    _, budget, _, _, phase = tr.get_curriculum_phase(episode0 + 1)
    return {"value": iters * rollout_len * n_envs * world / dt, "unit": "env-steps/s", "n_gpus": world,
            "s_per_iteration": dt / iters, "iterations": iters,
            "dtype": "rollout %s, update %s" % (rollout_precision, update_precision),
            "solver_optimizer_steps_per_iteration": outs[-1].get("solver_updates"),
            "config": "T=%d x %d envs/GPU x %d GPU%s, %s phase (budget %d), 3 epochs, minibatch %d per rank; rollout "
                      "policy %s, PPO update %s%s"
                      % (rollout_len, n_envs, world, "s" if world > 1 else "", phase, budget, minibatch,
                         "bf16 fused kernels" if rollout_precision == "bf16" else
                         "fp32 (conv backbone on the fp32-MFMA kernels at 20x20)", update_precision +
                         (" (conv backbone forward + backward on the hand-written fp32-MFMA kernels, heist_train_conv*, "
                          "at 20x20; MIOpen elsewhere)" if update_precision == "fp32" else
                          " (autocast: NHWC MIOpen convs)"),
                         "; one flat RCCL/gloo all-reduce of the Solver gradients per optimizer step" if multi
                         else "")}


def measure_allreduce_grads(dev, iters=20, warmup=3):
    """Mean microseconds of dist_utils.allreduce_grads (the training path's ONE exchange per
    optimizer step: a flat all-reduce of the Solver's 550,150 gradient floats plus its weight,
    reference agents/solver.py:191-199) on this process group, max over ranks."""
    from heist_amd import dist_utils
    from heist_amd.networks import SolverNetwork
    net = SolverNetwork(20, 20).to(dev)
    for p in net.parameters():
        p.grad = torch.randn_like(p)
    params = list(net.parameters())
    dist = torch.distributed
    for _ in range(warmup):
        dist_utils.allreduce_grads(params, weight=1.0)
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist_utils.allreduce_grads(params, weight=1.0)
    torch.cuda.synchronize(dev)
    us = (time.perf_counter() - t0) / iters * 1e6
    t = torch.tensor([us], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _spawned_rank(rank, world, port, argv):
    """Body of a rank started by `bench.py --gpus N` (torch.multiprocessing spawn)."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.argv = [sys.argv[0]] + list(argv)
    main()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--budget", type=int, default=15)
    ap.add_argument("--layouts", choices=("architect", "synthetic"), default="architect",
                    help="headline layout source: the fixed Architect checkpoint (C2) or the synthetic mix")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-secondary", action="store_true", help="skip the rollout / full-train numbers")
    ap.add_argument("--ticks-per-launch", type=int, default=20,
                    help="K: env ticks per heist_step_multi launch in the timed region (1: one heist_step per tick)")
    ap.add_argument("--train-envs", type=int, default=8192, help="envs per GPU of the N > 1 full-train line (C4)")
    ap.add_argument("--settle-ms", type=float, default=30.0,
                    help="untimed K-tick launches before the timed window (clock settle), milliseconds")
    ap.add_argument("--extra-windows", type=int, default=4,
                    help="extra timed windows after the headline one (HIP events): median / spread fields")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend at N > 1 (nccl = RCCL over xGMI; gloo lets several ranks share "
                         "one GPU, for tests)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launch the N ranks here (spawned interpreters; this process never touches the GPU)
        import socket
        import torch.multiprocessing as tmp
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        tmp.spawn(_spawned_rank, args=(args.gpus, port, sys.argv[1:]), nprocs=args.gpus, join=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d (launch N ranks with torchrun --nproc-per-node N, or run "
              "without torchrun and let --gpus spawn them)" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = torch.distributed
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        ndev = torch.cuda.device_count()
        if args.backend == "nccl" and ndev < world:
            # one process per GPU: RCCL needs N distinct devices (gloo may share one, for tests)
            print("bench.py: --gpus %d with the nccl (RCCL) backend needs %d visible GPUs, this node shows %d "
                  "(HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES = %r / %r); run with --gpus %d or --backend gloo"
                  % (world, world, ndev, os.environ.get("HIP_VISIBLE_DEVICES"),
                     os.environ.get("ROCR_VISIBLE_DEVICES"), ndev), file=sys.stderr, flush=True)
            sys.exit(2)
        local %= max(1, ndev)  # gloo: several ranks may share one GPU
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from heist_amd import EnvironmentConfig, HeistEnv
    from heist_amd.layouts import valid_synthetic_layouts

    cfg = EnvironmentConfig(grid_rows=20, grid_cols=20, max_steps=200, architect_budget=args.budget)
    N = args.envs
    env = HeistEnv(N, cfg, max_cams=max(1, args.budget // 3), max_guards=max(1, args.budget // 5), max_path=16,
                   device=dev, auto_reset=True)
    if args.layouts == "architect":
        lb, all_valid = architect_layouts(env, args.budget, seed=1234 + rank)
        layouts = None
        if not all_valid:
            log("warning: some Architect layouts stayed BFS-invalid after resampling")
    else:
        layouts = valid_synthetic_layouts(env, args.budget, seed=1234 + rank)
    env.reset()
    kcfg = env.kernel_config()
    if kcfg["probe_mode"] != 0:  # the profiling kernel skips phases: its numbers are not the step's
        print("bench.py: HEIST_PROBE_MODE=%d selects the profiling step kernel (phases skipped, results wrong); "
              "refusing to time it" % kcfg["probe_mode"], file=sys.stderr)
        sys.exit(2)
    knobs = {k: v for k, v in os.environ.items() if k.startswith("HEIST_")}
    gen = torch.Generator(device=dev)
    gen.manual_seed(4321 + rank)
    actions = torch.randint(0, 5, (args.warmup + args.steps, N), device=dev, generator=gen, dtype=torch.int64)
    K = max(1, min(args.ticks_per_launch, args.steps))
    elapsed, kern_ms, issue_s, launches = time_env(env, actions, args.warmup, args.steps, K, world,
                                                   settle_ms=args.settle_ms, extra_windows=args.extra_windows)
    per_rank = time_env.per_rank
    windows, settle_info = list(time_env.windows), time_env.settle
    fan_fill_ms = 0.0
    if K > 1 and kcfg["fan_on"]:  # the table fill the timed launches did not pay (read from an earlier fill)
        fan_fill_ms = measure_fan_fill(env, actions, K, time_env.last_bufs)
    # the rollout's form (the policy needs each observation before the next action): one
    # heist_step launch per tick, timed the same way at every N (collective at N > 1)
    e1, k1, i1, _ = time_env(env, actions, args.warmup, args.steps, 1, world) if K > 1 else (elapsed, kern_ms,
                                                                                               issue_s, launches)
    per_rank_1 = time_env.per_rank
    allreduce_us = None
    if world > 1:  # the training path's one exchange step: a flat Solver-gradient all-reduce per optimizer step
        allreduce_us = measure_allreduce_grads(dev)

    # ALU work figure: ray samples evaluated per env-step, counted by the
    # kernel on extra steps after the timed region
    cnt = torch.zeros(N, dtype=torch.int64, device=dev)
    cnt_x = torch.zeros(N, dtype=torch.int64, device=dev)
    env.count_samples(cnt)
    env.count_exact_rays(cnt_x)
    n_count = 40  # Architect cameras share their parameters, so the work per tick cycles with the headings
    count_actions = torch.randint(0, 5, (n_count, N), device=dev, generator=gen, dtype=torch.int64)
    for k in range(n_count):
        env.step(count_actions[k])
    env.count_samples(None)
    env.count_exact_rays(None)
    samples_per_step = float(cnt.sum().item()) / (n_count * N)
    exact_rays_per_step = float(cnt_x.sum().item()) / (n_count * N)

    st = env.export()  # accepted placements (set_layout's rules), not the requested lists
    ncam, ngu = float(st["n_cams"].double().mean()), float(st["n_guards"].double().mean())
    b_step = algorithmic_bytes_per_env_step(20, 20, ncam, ngu)
    achieved = b_step * N / (kern_ms * 1e-3) / 1e9  # GB/s: algorithmic bytes per tick / mean tick duration
    total_steps = args.steps * N * world
    value = total_steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    fan_ms_tick = fan_fill_ms / 1024.0  # one fill serves kFanTicks = 1,024 ticks
    achieved_fan = b_step * N / ((kern_ms + fan_ms_tick) * 1e-3) / 1e9
    achieved_wall = b_step * N / (ms_per_step * 1e-3) / 1e9
    fan_frac = shared_fan_fraction(lb.cam_params.cpu().numpy(), lb.n_cams.cpu().numpy()) if layouts is None else \
        synthetic_fan_fraction(layouts, env, args.budget)

    if rank == 0:
        traffic, traffic_src = None, None
        tf = os.path.join(ROOT, "profiles", "heist_step_multi_traffic.json" if K > 1 else "heist_step_traffic.json")
        if os.path.exists(tf) and N == 4096:
            with open(tf) as f:
                tj = json.load(f)
            if tj.get("workload") == args.layouts and tj.get("ticks_per_launch", 1) == K:
                traffic = tj.get("hbm_bytes_per_tick", tj.get("hbm_bytes_per_launch"))
                traffic_src = "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this command (%s), corrected per " \
                              "MI355X_MICROARCH.md, per tick: profiles/%s" % (tj.get("profile", "?"), os.path.basename(tf))
        line = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "env-only action replay (the K ticks' actions known up front) %s, 20x20 grid, "
                                   "%d envs/GPU, %s budget-%d layouts "
                                   "(mean %.2f cameras, %.2f guards/env accepted), uniform random actions pre-generated "
                                   "in HBM, auto-reset, every tick's [N,3,20,20] f32 observation, reward, done and "
                                   "status written to HBM"
                                   % ("heist_step_multi, K=%d ticks per launch (state on chip between ticks)" % K
                                      if K > 1 else "heist_step, one tick per launch", N,
                                      "BASELINE C2: fixed Architect checkpoint (T=1.0)" if args.layouts == "architect"
                                      else "synthetic (SURVEY 8d generator ii)", args.budget, ncam, ngu),
                       "ticks_per_launch": K,
                       "envs_per_gpu": N, "grid": "20x20", "layouts": args.layouts,
                       "parallelism": "env-sharded x%d" % world, "kernel_config": kcfg, "env_knobs": knobs,
                       "backend": args.backend if world > 1 else None},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "frac_wall": achieved_wall / HBM_PEAK_GBS,
                         "frac_with_fan_fill": achieved_fan / HBM_PEAK_GBS,
                         "fan_fill_ms_per_fill": fan_fill_ms, "fan_fill_ms_per_tick_amortised": fan_ms_tick,
                         "shared_fan_frac": fan_frac,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": multi_kernel_name(kcfg, 20, 20) if K > 1 else "heist::step_kernel",
                         "kernel_ms": kern_ms, "kernel_ms_per_launch": kern_ms * K, "launches": launches,
                         "clock_settle": settle_info,
                         "extra_windows_kernel_ms": windows,
                         "windows_frac": None if not windows else {
                             "n": len(windows) + 1,
                             "median": float(np.median([b_step * N / (w * 1e-3) / 1e9 / HBM_PEAK_GBS
                                                        for w in windows + [kern_ms]])),
                             "min": min(b_step * N / (w * 1e-3) / 1e9 / HBM_PEAK_GBS for w in windows + [kern_ms]),
                             "max": max(b_step * N / (w * 1e-3) / 1e9 / HBM_PEAK_GBS for w in windows + [kern_ms])},
                         "algorithmic_bytes_per_env_step": b_step,
                         "ray_samples_per_env_step": samples_per_step,
                         "ray_samples_per_s": samples_per_step * N / (kern_ms * 1e-3),
                         "exact_path_rays_per_env_step": exact_rays_per_step,
                         "host_issue_us_per_step": issue_s / args.steps * 1e6,
                         "note": "achieved = algorithmic bytes per env-step (SURVEY 8d) x envs / mean tick duration "
                                 "(kernel_ms: HIP events around the timed launches); frac_wall uses ms_per_step (the "
                                 "wall clock between the barriers), frac_with_fan_fill adds the shared fan table's "
                                 "fill amortised over the 1,024 ticks it serves (the timed launches read a table "
                                 "an earlier launch filled); shared_fan_frac = share of the envs with cameras whose "
                                 "camera group the table serves; with K > 1 the per-env state stays on chip between "
                                 "ticks, so the kernel moves fewer bytes than the formula counts (see traffic)"},
            # the rollout cannot replay K known actions (the policy needs each
            # observation), so its env figure -- one heist_step launch per tick -- sits beside
            # the headline at every N
            "env_only_single_tick": {
                "value": args.steps * N * world / e1, "unit": "env-steps/s", "kernel_ms": k1,
                "ms_per_step": e1 / args.steps * 1e3, "host_issue_us_per_step": i1 / args.steps * 1e6,
                "kernel": "heist::step_kernel", "workload": "one heist_step launch per tick (the rollout's form)",
                "roofline": {"bound": "hbm", "achieved": b_step * N / (k1 * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": b_step * N / (k1 * 1e-3) / 1e9 / HBM_PEAK_GBS}},
            "cpu_baseline": None,
        }
        log("env-only: %.1f M env-steps/s, %.2f us per tick (K=%d)" % (value / 1e6, kern_ms * 1e3, K))
        # single-GPU figures: the secondary numbers and the CPU baseline run on rank 0 at N=1
        # only (at N>1 the other ranks would idle at the closing barrier meanwhile)
        if world > 1:  # attribution for a 1 -> N curve: every rank's env-only time, the exchange step's cost
            line["per_rank"] = {"elapsed_s": [r[0] for r in per_rank], "kernel_ms_per_tick": [r[1] for r in per_rank],
                                "single_tick_elapsed_s": [r[0] for r in per_rank_1],
                                "single_tick_kernel_ms": [r[1] for r in per_rank_1]}
            line["allreduce_grads_us_per_optimizer_step"] = allreduce_us
        if not args.no_secondary and world == 1:
            sec = {}
            log("env-only at the other BASELINE configs / layout sources")
            other = "synthetic" if args.layouts == "architect" else "architect"
            sec["env_only_%s_layouts" % other] = measure_env_config(dev, 20, N, args.budget, K=K,
                                                                    architect=other == "architect")
            sec["env_only_c4_8192envs_budget40"] = measure_env_config(dev, 20, 8192, 40, K=K, architect=True)
            sec["env_only_c5_32x32_2048envs_4cams_3guards"] = measure_env_config(dev, 32, 2048, 40, K=K, n_cams=4,
                                                                                 n_guards=3)
            log("rollout")
            sec["rollout_bf16"] = measure_rollout(env, dev, precision="bf16")
            sec["rollout_fp32"] = measure_rollout(env, dev, steps=10, precision="fp32")
            log("policy inference")
            sec["policy_inference"] = measure_policy(dev, N)
            sec["policy_inference_c5_32x32"] = measure_policy(dev, 2048, R=32)
            log("full train (fp32 rollout + fp32 update: the parity mode)")
            sec["full_train_fp32"] = measure_train(cfg, dev, N)
            log("full train (bf16 rollout + bf16 update)")
            sec["full_train_bf16"] = measure_train(cfg, dev, N, update_precision="bf16", rollout_precision="bf16")
            line["secondary"] = sec
        if not args.no_cpu_baseline and world == 1:
            log("cpu baseline")
            if layouts is None:
                from heist_amd.training import _lb_rows
                layouts = _lb_rows(lb, np.arange(min(N, 512))).to_lists()
            cores = max(1, min(os.cpu_count() or 1, 16))  # the GPU box's CPU share is 16 threads per GPU
            line["cpu_baseline"] = cpu_baseline(layouts, cfg, args.budget, target_s=args.cpu_seconds, threads=cores)
            line["cpu_baseline_1core"] = cpu_baseline(layouts, cfg, args.budget, target_s=args.cpu_seconds / 2,
                                                      threads=1)
    if world > 1 and not args.no_secondary:
        # BASELINE config 4 at N > 1: 8192 envs/GPU, the c4 curriculum at its top (budget 40),
        # every optimizer step averaging gradients with one all-reduce (collective: all ranks)
        if rank == 0:
            log("multi-GPU full train (C4: 8192 envs/GPU, budget 40, fp32 rollout + update)")
        cfg4 = EnvironmentConfig(grid_rows=20, grid_cols=20, max_steps=200, architect_budget=40)
        train = measure_train(cfg4, dev, args.train_envs, curriculum="c4", episode0=400,
                              minibatch=min(16384, 4 * args.train_envs))
        if rank == 0:
            line["full_train_c4_multi_gpu"] = train
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
