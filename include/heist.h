/* heist.h -- C ABI of the MI355X-native Heist Architect hot path (libheist_hip.so).
 *
 * The reference (a pure-Python package) has no FFI for this path; its boundary is the
 * Python class API that training and the UI call.  Each entry point below replaces one
 * reference interface (paths relative to the reference repository root) and is bound
 * by the Python mirror package heist_amd (see INTEGRATION.md for the ctypes binding).
 *
 * Conventions
 *  - All array pointers are DEVICE pointers owned by the caller (e.g. torch tensors on
 *    the same HIP device), except `reward_consts` in heist_create (host).
 *  - Every call is enqueued on `stream` and is asynchronous; nothing synchronises.
 *  - Return 0 on success, HEIST_EINVAL for bad arguments, else a hipError_t value.
 *    heist_last_error() gives a message for the calling thread's last failure.
 *  - A heist_t handle is bound to the device that was current at heist_create and is
 *    not thread-safe: use one handle per device/thread.
 *  - Layouts are [env][...] row-major; grids are [env][row][col]; obs is [env][3][R][C].
 */
#ifndef HEIST_H
#define HEIST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: heist_step_stamps takes the buffer size; heist_stamp_words; 3: heist_arch_update_*;
 * 4: heist_arch_update_status, the heist_*_nhwc training passes, heist_get_config's 15th word
 *    (heist_step on the lean kernel), the heist_train_* fp32-MFMA training convolutions,
 *    heist_rollout_tally; 5: heist_get_config's 16th word (lean_waves), heist_lstm_cell */
#define HEIST_ABI_VERSION 5
#define HEIST_EINVAL 100000

/* status_out codes of heist_step (environment.py:236-297 info["status"]). */
#define HEIST_RUNNING 0
#define HEIST_DETECTED 1
#define HEIST_VAULT_REACHED 2
#define HEIST_TIMEOUT 3
#define HEIST_ALREADY_DONE 4

typedef struct heist_env* heist_t;
typedef struct ihipStream_t* heist_stream_t; /* == hipStream_t */

int heist_abi_version(void);
const char* heist_last_error(void);

/* Replaces HeistEnvironment.__init__ / EnvironmentConfig (environment.py:18-97) for a
 * batch of n_envs independent environments (1 <= n_envs <= 2^24).  R, C <= 64.  reward_consts (host) =
 * {reward_step, reward_detection, reward_vault}.  max_cams / max_guards / max_path bound
 * the per-env layout capacity. */
int heist_create(int rows, int cols, int max_steps, int start_r, int start_c, int vault_r, int vault_c,
                 const double* reward_consts, int n_envs, int max_cams, int max_guards, int max_path,
                 heist_t* out);
int heist_destroy(heist_t h);

/* Replaces HeistEnvironment.set_layout + _reset_layout + is_level_valid
 * (environment.py:102-177) and BudgetManager.purchase (budget.py:48-58), per env:
 *   wall_rc     [N][max_walls][2]      int32   walls in list order (first n_walls[e] used)
 *   cam_params  [N][max_cams][6]       float64 row, col, fov_angle, heading, rotation_speed, vision_range
 *   guard_paths [N][max_guards][max_path][2] int32 patrol_path points
 *   guard_meta  [N][max_guards][3]     int32   path length, speed, vision_range
 *   guard_fov   [N][max_guards]        float64 fov_angle
 *   budget      [N]                    int32   BudgetManager.total_budget
 *   mask        [N]                    uint8   only envs with mask[e] != 0 are re-laid out (NULL: all)
 *   valid_out   [N]                    uint8   bfs_path_exists(start, vault) (written for masked envs)
 * Guard path points must lie inside the grid.  Solver state is left untouched (call
 * heist_reset next, as training.py:516 does). */
int heist_set_layout(heist_t h, int max_walls, const int32_t* wall_rc, const int32_t* n_walls,
                     const double* cam_params, const int32_t* n_cams, const int32_t* guard_paths,
                     const int32_t* guard_meta, const double* guard_fov, const int32_t* n_guards,
                     const int32_t* budget, const uint8_t* mask, uint8_t* valid_out, heist_stream_t stream);

/* Replaces HeistEnvironment.reset + get_state_tensor (environment.py:183-214, :347-374)
 * for envs with mask[e] != 0 (mask == NULL: all).  obs_out [N][3][R][C] float32; rows of
 * unmasked envs are not written. */
int heist_reset(heist_t h, const uint8_t* mask, float* obs_out, heist_stream_t stream);

/* Replaces HeistEnvironment.step + get_state_tensor (environment.py:216-299, :347-374).
 *   actions [N] int64 in 0..4;  obs_out [N][3][R][C] float32;  reward_out [N] float32
 *   (the float64 reward rounded, as agents/solver.py:138 stores it); reward64_out [N]
 *   float64 or NULL; done_out [N] uint8; status_out [N] int8 (HEIST_* codes).
 * With HEIST_STEP_LEAN=1 at heist_create, where the lean K-tick kernel serves the handle
 * (20 x 20 at one wave per env, 32 x 32; no instrumentation armed) the tick runs as
 * heist_step_multi with K = 1, bit-identical (off by default: slower per tick).
 * auto_reset != 0: an env that finishes this tick is reset in the same launch and its
 * obs row holds the reset observation (training.py:515-520 next attempt), while reward,
 * done and status describe the finishing tick.  auto_reset == 0: finished envs answer
 * later steps with reward 0 / HEIST_ALREADY_DONE (environment.py:232-233). */
int heist_step(heist_t h, const int64_t* actions, float* obs_out, float* reward_out, double* reward64_out,
               uint8_t* done_out, int8_t* status_out, int auto_reset, heist_stream_t stream);

/* K consecutive heist_step calls in one launch, for actions known in advance (env-only
 * throughput, action replay; no reference counterpart as an entry point -- it is
 * environment.py:216-299 + :347-374 applied K times).  Equivalent, bit for bit, to
 *   for k in 0..K-1: heist_step(h, actions + k*N, obs_out + k*N*3*R*C, reward_out + k*N,
 *                               reward64_out ? reward64_out + k*N : NULL, done_out + k*N,
 *                               status_out + k*N, auto_reset, stream)
 * with every per-tick output written (tick-major: actions [K][N] int64, obs_out
 * [K][N][3][R][C] float32, reward_out [K][N] float32, reward64_out [K][N] float64 or NULL,
 * done_out [K][N] uint8, status_out [K][N] int8); the per-env state stays on chip between
 * the ticks.  1 <= K <= 1024.  Launches read a table of the shared camera fan that a launch
 * refills when it is stale; a launch on another stream than the previous one refills it
 * after waiting, on the device, for that launch (no host synchronisation). */
int heist_step_multi(heist_t h, int K, const int64_t* actions, float* obs_out, float* reward_out,
                     double* reward64_out, uint8_t* done_out, int8_t* status_out, int auto_reset,
                     heist_stream_t stream);

/* Copies per-env state out for get_environment_state / the single-env compatibility
 * class (environment.py:388-417).  Any pointer may be NULL.
 *   scalars [N][12] int32: pos_r, pos_c, tick, done, detected, vault_reached, prev_dist,
 *                          initial_dist, n_cams, n_guards, n_walls, budget_spent
 *   grid [N][R][C] int8;  cam_heading [N][max_cams] f64;  guard_idx [N][max_guards] int32;
 *   guard_heading [N][max_guards] f64 */
int heist_export(heist_t h, int32_t* scalars, int8_t* grid, double* cam_heading, int32_t* guard_idx,
                 double* guard_heading, heist_stream_t stream);

/* Instrumentation, no reference counterpart: with counter a device array of n_envs uint64,
 * every later heist_step / heist_reset on h adds to counter[e] the number of ray samples
 * env e evaluated (the ALU work figure of SURVEY 8(d)); NULL switches counting off (default). */
int heist_count_samples(heist_t h, uint64_t* counter);

/* Instrumentation, no reference counterpart: like heist_count_samples, counter[e] += the
 * number of env e's rays whose fp32 fast path met a near .5 tie and were re-cast on the
 * exact fp64 path. */
int heist_count_redo(heist_t h, uint64_t* counter);

/* Instrumentation, no reference counterpart: later heist_step calls on h record the shader
 * clock (s_memtime) at 8 phase boundaries of every wavefront into buf[env][wave][10] (waves
 * per env: heist_step_waves(h); slots 8 and 9 hold HW_ID and XCC_ID): 0 entry, 1 prefetch
 * landed, 2 emitter table published, 3 raycast done, 4 reward done, 5 auto-reset done, 6
 * observation written, 7 exit.  heist_step_multi writes buf[env][multi_waves][16] instead:
 * clock cycles summed per tick segment 0..8 over the launch, lifetime, start clock, HW_ID,
 * XCC_ID.  n_words is buf's size in uint64 words: a call whose kernel needs more
 * (n_envs * 10 * step_waves, resp. n_envs * 16 * multi_waves; heist_stamp_words reports both)
 * fails with HEIST_EINVAL instead of writing past it.  NULL switches stamping off (default). */
int heist_step_stamps(heist_t h, uint64_t* buf, int64_t n_words);

/* uint64 words of a stamp buffer for heist_step (which = 0) or heist_step_multi (which = 1)
 * on h; no reference counterpart. */
int64_t heist_stamp_words(heist_t h, int which);

/* Wavefronts per env of h's step / reset kernels (2 unless HEIST_STEP_WAVES chose 1 or 4
 * at heist_create); no reference counterpart. */
int heist_step_waves(heist_t h);

/* The handle's effective kernel configuration, no reference counterpart (what a benchmark
 * records next to its numbers): out[0..n) with n <= 16 receives step_waves, ray_chunk,
 * step_occ, vis_gap, obs_store, ray_mode, probe_mode, dispatch_order, split_obs,
 * guard_cones, multi_waves, fan_on, lean, interval_fans (the HEIST_* environment knobs as heist_create resolved them,
 * then any heist_set_* calls), step_lean (1: heist_step currently runs as a one-tick
 * heist_step_multi launch on the lean kernel; HEIST_STEP_LEAN=1 at heist_create turns it on),
 * lean_waves (waves per env of the 32 x 32 lean kernel: 2 when the batch's doubled waves fit
 * the chip, HEIST_LEAN_WAVES=1/2 forces).  probe_mode != 0 selects the profiling step kernel, whose results are
 * wrong by design (phases skipped). */
int heist_get_config(heist_t h, int32_t* out, int n);

/* Raycast arithmetic of later heist_step / heist_reset calls on h: 0 (default) = fp32 fast
 * path with exact fp64 re-cast of every ray that comes within a bounded error of a .5 tie,
 * 1 = exact fp64 path for every ray.  Both give bit-identical visibility; 1 exists for
 * parity tests and A/B timing.  The environment variable HEIST_EXACT_RAYS=1 sets 1 at
 * heist_create. */
int heist_set_ray_mode(heist_t h, int ray_mode);

/* Guard cone cache, no reference counterpart (a precomputation of Guard.get_visible_tiles,
 * security.py:161-192): with on = 1 (default; HEIST_GUARD_CONES=0 at heist_create turns
 * it off) every later heist_set_layout casts each guard's vision cone once per (patrol
 * index, heading) on the exact fp64 path, and heist_step / heist_reset OR the cached cone
 * instead of raycasting the guard (guards with a patrol of more than 16 points, more than
 * 8 distinct headings or a vision range above 7 are always raycast).  Results are
 * identical either way; on = 0 raycasts every guard every tick.  Takes effect at the next
 * heist_set_layout. */
int heist_set_guard_cones(heist_t h, int on);

/* Replaces bfs_path_exists (utils.py:52-85) on a batch of grids [N][R][C] int32. */
int heist_bfs_valid(const int32_t* grid, int n, int rows, int cols, int start_r, int start_c, int goal_r,
                    int goal_c, uint8_t* valid_out, heist_stream_t stream);

/* Replaces Camera.get_vision_cone_tiles (security.py:53-101, kind 0) and
 * Guard.get_visible_tiles (security.py:161-192, kind 1) for n independent emitters:
 *   walls [n][R][C] uint8 (nonzero = wall); meta [n][4] int32 = kind, row, col, range;
 *   params [n][2] f64 = fov_angle, heading;  tiles_out [n][R][C] uint8 (1 = visible). */
int heist_cones(int n, int rows, int cols, const uint8_t* walls, const int32_t* meta, const double* params,
                uint8_t* tiles_out, heist_stream_t stream);

/* The reference's LIST ORDER of the same cones (get_vision_cone_tiles / get_visible_tiles
 * append a tile when a ray first reaches it, rays in index order, samples in distance
 * order): keys_out [n][R][C] uint32 = (ray << 12 | sample) of the first visit on the exact
 * fp64 path, 0xFFFFFFFF where no ray reaches the tile.  Same inputs as heist_cones. */
int heist_cone_order(int n, int rows, int cols, const uint8_t* walls, const int32_t* meta, const double* params,
                     uint32_t* keys_out, heist_stream_t stream);

/* heist_cones with an explicit ray_mode (0 fast + exact re-cast, 1 exact only; see
 * heist_set_ray_mode).  heist_cones is ray_mode 0. */
int heist_cones_mode(int n, int rows, int cols, const uint8_t* walls, const int32_t* meta, const double* params,
                     int ray_mode, uint8_t* tiles_out, heist_stream_t stream);

/* The fast path's fp32 ray direction for angles in degrees (parity tooling: its error
 * against the exact glibc direction bounds the near-tie tolerance).  [n] f64 in,
 * cos_out, sin_out [n] f32. */
int heist_fast_dir(const double* angle_deg, int64_t n, float* cos_out, float* sin_out, heist_stream_t stream);

/* Replaces the decode half of ArchitectNetwork.generate_layout (networks.py:283-335) and
 * the curriculum filter of training.py:464-467 for n sampled layouts:
 *   asset_map [n][R][C] int64 per-cell class (0 none, 1 wall, 2 camera, 3 guard);
 *   cam_params [3] or [n][3] float32 = fov, speed, heading (cam_stride 0 or 3);
 *   budget [n] int32.  Outputs are the heist_set_layout input arrays with capacities
 *   max_walls / max_cams / max_guards / max_path (max_path >= 8); lists longer than a
 *   capacity are truncated, so size capacities from the budget (budget, /3, /5). */
int heist_architect_decode(const int64_t* asset_map, int n, int rows, int cols, const float* cam_params,
                           int cam_stride, const int32_t* budget, int allow_cams, int allow_guards, int max_walls,
                           int max_cams, int max_guards, int max_path, int32_t* wall_rc, int32_t* n_walls,
                           double* cam_out, int32_t* n_cams, int32_t* guard_paths, int32_t* guard_meta,
                           double* guard_fov, int32_t* n_guards, heist_stream_t stream);

/* math.sin / math.cos of the reference's raycast (security.py:74-75, :174-175) as the GPU
 * evaluates them: glibc 2.35's dbl-64 algorithm, bit-exact to the host libm for
 * |x| < 105414350.  x, sin_out, cos_out [n] float64 (parity checks and tooling). */
int heist_sincos(const double* x, int64_t n, double* sin_out, double* cos_out, heist_stream_t stream);

/* Replaces the Architect's per-layout update cadence (training.py:479-480 / :558-559:
 * ArchitectAgent.update after every layout with ONE transition, agents/architect.py:91-155)
 * for k consecutive rewards, as one persistent launch (64 workgroups, one per CU, grid
 * barriers between phases).  With one transition update i is an Adam step on
 * value_coeff * (V(s0) - rewards[i])^2, V = ArchitectNetwork's value path (encoder ->
 * adaptive pool -> fc_global -> value_head, networks.py:159-188) on the constant grid s0,
 * after clip_grad_norm_(max_norm) over the 12 value-path tensors.  Workgroup w owns conv2 /
 * conv3 channels 4(w%16)..+3 on pool-cell row band w/16 of the image.
 *   params / exp_avg / exp_avg_sq: HOST arrays of 12 device pointers each, in
 *     ArchitectNetwork.parameters() order restricted to the value path: encoder.0.weight
 *     [32][1][3][3], encoder.0.bias, encoder.2.weight [64][32][3][3], encoder.2.bias,
 *     encoder.4.weight [64][64][3][3], encoder.4.bias, fc_global.weight [256][1024],
 *     fc_global.bias, value_head.0.weight [128][256], value_head.0.bias,
 *     value_head.2.weight [1][128], value_head.2.bias; float32, contiguous; the weights of
 *     encoder.2 / encoder.4 / value_head.0 128-byte aligned.  Updated in place.
 *   grid [rows][cols] float32 = s0 with at most 64 nonzero pixels (the Architect's state
 *     has 2);  rewards [k] float32;  value_loss [k] float32 out
 *     (mse of each step, before its update).
 *   step_scalars [k][2] float32 (device): per update, the two scalars torch.optim.Adam forms
 *     in float64 from the step count and casts to float: -lr / (1 - beta1^step) and
 *     sqrt(1 - beta2^step); beta1, beta2, eps as torch.optim.Adam (amsgrad, weight_decay,
 *     maximize off; the foreach arithmetic).
 *   workspace: heist_arch_update_workspace_bytes() device bytes, not shared by launches in
 *     flight.  rows x cols in {8, 12, 16, 20} squared (heist_arch_update_supported). */
int64_t heist_arch_update_workspace_bytes(void);
int heist_arch_update_supported(int rows, int cols);
int heist_arch_update_sequence(float* const* params, float* const* exp_avg, float* const* exp_avg_sq,
                               const float* grid, int rows, int cols, const float* rewards, int k,
                               const float* step_scalars, double beta1, double beta2, double eps, double max_norm,
                               double value_coeff, float* value_loss, void* workspace, heist_stream_t stream);
/* Status of the last launch on `workspace`, a bit mask; any bit set means its results --
 * the updated params, exp_avg, exp_avg_sq and value_loss -- are INVALID (the caller restores
 * its own copy and re-runs the steps another way):
 *   bit 0: a grid barrier gave up waiting (the 64 workgroups were not co-resident; the spin
 *          bound is 2^25 polls, HEIST_ARCH_SPIN_LIMIT overrides it, e.g. to test this path);
 *   bit 1: grid has more than 64 nonzero pixels.
 * The word is the uint32 at byte offset heist_arch_update_workspace_bytes() - 252 of the
 * workspace (zeroed at each launch), so a caller can also copy it asynchronously.
 * Synchronises `stream`.  heist_arch_update_timed_out reports bit 0 alone. */
int heist_arch_update_status(const void* workspace, int* status, heist_stream_t stream);
int heist_arch_update_timed_out(const void* workspace, int* timed_out, heist_stream_t stream);
/* Instrumentation, no reference counterpart: with buf a device array of 2 * 16 * 32 + 16 * 5 * 64
 * uint64, later heist_arch_update_sequence launches record s_memrealtime (100 MHz) at up to 32
 * phase points of steps 0..15 in workgroups 0 and 63, then every workgroup's arrival (stores
 * drained) at each of the 5 grid barriers of steps 0..15 (tools/probe_arch_update.py); NULL: off. */
int heist_arch_update_stamps(uint64_t* buf);

/* The batched trainer's per-tick attempt bookkeeping over n envs (the per-episode counters of
 * training.py:515-544 -- steps, reward, outcome per attempt -- and solver.reset() per attempt,
 * :517), replacing ~20 tensor ops per tick: counting = valid[e] && attempts[e] <
 * attempts_per_layout; steps += counting; reward_sum += counting ? reward64 : 0.0 (float64);
 * an attempt that ends (counting && done) adds 1 to solve (status 2 = vault_reached), detect
 * (status 1) or timeout (any other status) and to attempts; h, c [n][hidden] float32 (the
 * LSTM state, layer dimension 1) are multiplied by (done ? 0 : 1).  valid, done uint8 (bool),
 * status int8, the counters int32. */
/* The Solver's LSTM cell after its gate GEMMs (reference networks.py:90-100, nn.LSTM one time
 * step, gate order i, f, g, o; replaces the ten pointwise torch kernels of
 * SolverNetwork.lstm_step in the rollout): gates = gates_x + gates_h ([n][4 hidden] float32
 * each), c_out = sigmoid(f) * c + sigmoid(i) * tanh(g), h_out = sigmoid(o) * tanh(c_out)
 * ([n][hidden]), every operation rounded to float32 in that order (bit-identical to torch's
 * kernels). */
int heist_lstm_cell(const float* gates_x, const float* gates_h, const float* c, float* h_out, float* c_out, int hidden,
                    int n, heist_stream_t stream);

int heist_rollout_tally(const uint8_t* valid, int32_t* attempts, int attempts_per_layout, const uint8_t* done,
                        const int8_t* status, const double* reward64, int32_t* steps, double* reward_sum, int32_t* solve,
                        int32_t* detect, int32_t* timeout, float* h, float* c, int hidden, int n, heist_stream_t stream);

/* Replaces SolverAgent._compute_gae + returns (agents/solver.py:142-143, :228-244) on a
 * [T][N] rollout (column e = env e's concatenated episodes).  dones [T][N] uint8.
 * last_value [N] bootstraps t = T-1 (NULL = 0, the reference's buffer-end rule).  gamma and
 * lam are taken in float64 because the reference forms gamma*lam in Python floats. */
int heist_gae(const float* rewards, const float* values, const uint8_t* dones, const float* last_value,
              int T, int n, double gamma, double lam, float* adv_out, float* ret_out, heist_stream_t stream);

/* Advantage normalisation (agents/solver.py:146-147): x <- (x - mean) / (std + eps),
 * unbiased std; skipped when the global count is <= 1.  acc is a device float64[3] the
 * caller zeroes.  Phases (multi-GPU callers all-reduce acc between them):
 *   phase 0: acc[0] += sum(x), acc[1] += n            -> all-reduce acc[0..1]
 *   phase 1: acc[2] += sum((x - acc[0]/acc[1])^2)     -> all-reduce acc[2]
 *   heist_adv_apply(x, n, acc, eps)
 * heist_adv_normalize runs both phases and the apply on one device (acc = scratch3). */
int heist_adv_moments(const float* x, int64_t n, int phase, double* acc, heist_stream_t stream);
int heist_adv_apply(float* x, int64_t n, const double* acc, float eps, heist_stream_t stream);
int heist_adv_normalize(float* x, int64_t n, double* scratch3, float eps, heist_stream_t stream);

/* Clipped PPO loss of SolverAgent.update (agents/solver.py:172-193) over M samples with
 * Categorical(probs=softmax(logits)) semantics, fused forward + backward:
 *   logits [M][A] f32 (A <= 16), values [M] f32, actions [M] int64, old_logp/adv/ret [M] f32;
 *   loss_parts [4] f32 = total, policy, value, entropy (means over M);
 *   dlogits [M][A], dvalues [M] = d(total)/d(input);  scratch >= 3*ceil(M/256) float64. */
int heist_ppo_loss(const float* logits, const float* values, const int64_t* actions, const float* old_logp,
                   const float* adv, const float* ret, int M, int A, double clip, double vcoef, double ecoef,
                   float* loss_parts, float* dlogits, float* dvalues, double* scratch, heist_stream_t stream);

/* Fused batched SolverNetwork backbone (networks.py:93-100: relu(conv1) -> relu(conv2) ->
 * relu(conv3) -> AdaptiveAvgPool2d(4,4) -> flatten) on bf16 MFMA with fp32 accumulation,
 * for SolverAgent.select_action (agents/solver.py:75-99) over a batch.
 * heist_solver_pack converts the float32 torch parameters conv{1,2,3}.weight [co][ci][3][3]
 * and .bias [co] (3->32->64->64) into the kernel's fragment layout in `packed`
 * (heist_solver_packed_bytes() bytes, 16-byte aligned); call it after every weight update.
 * heist_solver_features: obs [n][3][rows][cols] float32 -> feat_out [n][1024] float32
 * (channel-major 64 x 4 x 4, the x.view(batch, -1) order).  rows x cols in {20x20, 10x10, 32x32};
 * other sizes return HEIST_EINVAL (callers use the PyTorch path). */
int heist_solver_packed_bytes(void);
int heist_solver_pack(const float* conv1_w, const float* conv1_b, const float* conv2_w, const float* conv2_b,
                      const float* conv3_w, const float* conv3_b, void* packed, heist_stream_t stream);
int heist_solver_features(const float* obs, int n, int rows, int cols, const void* packed, float* feat_out,
                          heist_stream_t stream);

/* Fused batched Solver head (networks.py:102-131 + agents/solver.py:75-99 select_action):
 * x = relu(fc_spatial(feat)); one LSTM cell step (gate order i, f, g, o); logits =
 * policy_head(h'), value = value_head(h'); action ~ Categorical(softmax(logits)) and its
 * log_prob with torch's probs semantics.  GEMMs on bf16 MFMA (fp32 accumulate), cell
 * update, last layers and sampling in fp32.  Requires hidden_dim 256, lstm_hidden 128,
 * head width 128, 1 <= num_actions <= 7.
 * heist_solver_head_pack: float32 parameters (torch layouts: fc_spatial.weight [256][1024],
 * lstm.weight_ih_l0 [512][256], weight_hh_l0 [512][128], policy_head.0 / value_head.0
 * .weight [128][128], policy_head.2.weight [A][128], value_head.2.weight [1][128], biases)
 * -> packed (heist_solver_head_packed_bytes() bytes); call after every weight update.
 * heist_solver_head: feat [n][1024] (heist_solver_features), h_in / c_in [n][128] or NULL
 * (zero state); seed / counter select the sample (counter-based hash, one uniform per env);
 * outputs logits [n][A] (may be NULL), value [n], action [n] int64, logp [n],
 * h_out / c_out [n][128] (must not alias h_in / c_in). */
/* Instrumentation, no reference counterpart: with buf a device array of
 * n_workgroups * 4 * 10 uint64, later heist_solver_features launches record s_memtime at
 * 10 phase points of each wave for its workgroup's second env (tools/probe_policy.py);
 * NULL switches it off (default). */
int heist_solver_stamps(uint64_t* buf);

int heist_solver_head_packed_bytes(void);
int heist_solver_head_pack(const float* fc_w, const float* fc_b, const float* w_ih, const float* w_hh,
                           const float* b_ih, const float* b_hh, const float* p1_w, const float* p1_b,
                           const float* v1_w, const float* v1_b, const float* p2_w, const float* p2_b,
                           const float* v2_w, const float* v2_b, int num_actions, void* packed,
                           heist_stream_t stream);
int heist_solver_head(const float* feat, const float* h_in, const float* c_in, int n, const void* packed,
                      int num_actions, uint64_t seed, uint64_t counter, float* logits_out, float* value_out,
                      int64_t* action_out, float* logp_out, float* h_out, float* c_out, heist_stream_t stream);

/* The Solver backbone's fp32 training step (agents/solver.py:157-199 over networks.py:93-100:
 * relu(conv1) -> relu(conv2) -> relu(conv3) -> AdaptiveAvgPool2d(4, 4), forward and backward)
 * with the convolutions run without bias (MIOpen) and everything between them fused into one
 * pass per layer.  Tensors are NHWC (channels_last) fp32, 16-byte aligned; n samples of rows x
 * cols positions.
 *   heist_bias_relu_nhwc: x[p][c] = relu(x[p][c] + bias[c]) in place (F.relu(conv + b)).
 *   heist_bias_relu_pool_nhwc: the same for conv3 (64 channels) plus feat_out [n][64 * 16] =
 *     adaptive_avg_pool2d(., (4, 4)) flattened C-major (the view fc_spatial reads).
 *   heist_pool_relu_bwd_nhwc: the backward of the two: d_out = (y > 0) * (the pool's input
 *     gradient of dfeat [n][1024]) (conv3's grad_output), dbias_out [64] = its sum over
 *     samples and positions; partial: [n][64] floats of scratch.
 *   heist_relu_bwd_nhwc: g = (y > 0) ? g : 0 in place (threshold_backward on the saved output)
 *     and dbias_out [channels] its sum; partial [n][channels] scratch; 32 or 64 channels.
 * Sums run in a fixed order (deterministic; fp32 rounding differs from torch's order). */
int heist_bias_relu_nhwc(float* x, const float* bias, int64_t n_pos, int channels, heist_stream_t stream);
int heist_bias_relu_pool_nhwc(float* x, const float* bias, int n, int rows, int cols, int channels, float* feat_out,
                              heist_stream_t stream);
int heist_pool_relu_bwd_nhwc(const float* dfeat, const float* y, int n, int rows, int cols, int channels, float* d_out,
                             float* partial, float* dbias_out, heist_stream_t stream);
int heist_relu_bwd_nhwc(float* g, const float* y, int n, int positions, int channels, float* partial, float* dbias_out,
                        heist_stream_t stream);

/* The Solver backbone's fp32 training convolutions on fp32 MFMA (v_mfma_f32_16x16x4_f32, exact
 * fp32), for the PPO update's forward and backward (agents/solver.py:157-199 over
 * networks.py:93-100): every pass of relu(conv1) -> relu(conv2) -> relu(conv3) -> pool as one
 * persistent kernel with the weights in registers and the activation bands in LDS, replacing
 * MIOpen's convolutions.  20 x 20 grids (heist_train_conv_supported).  Activations are
 * [n][rows][cols][P] float32 with P = channels + 4 (the 4 pad words are never read), the
 * network input [n][rows][cols][4] (heist_train_obs_nhwc4), all 16-byte aligned.
 *   heist_train_conv_pack: torch weights [co][ci][3][3] of layer 1 (3 -> 32, mode 0), 2 (32 -> 64)
 *     or 3 (64 -> 64) -> frag (heist_train_conv_frag_floats floats); mode 0 the forward
 *     convolution, mode 1 its data gradient (transposed, flipped taps).
 *   heist_train_conv: mode 0 y = relu(conv(x) + bias) and, if mask_bits is not NULL, its ReLU
 *     mask as bits (ReLU masks are [n][rows][cols][channels / 4] uint8: bit r of byte k =
 *     channel 4 k + r is > 0); mode 1 (layers 2, 3) y = mask ? conv_data_grad(x) : 0 with x the
 *     gradient at the layer's output (64 channels) and mask_bits the mask of the layer's input
 *     (the forward's bits of the layer below: threshold_backward).  queue: 2 device ints, zero
 *     before the first launch (the kernels leave them zero); one pair per launch in flight.
 *   heist_train_conv_wgrad: dw [co][ci][3][3] and db [co] of layer 1-3 from dy (the gradient at
 *     the layer's pre-activation output) and x (its input); partial:
 *     heist_train_conv_partial_floats(layer, n, ...) floats of scratch.  Sums in a fixed order.
 *   heist_train_obs_nhwc4: obs [n][3][rows][cols] with element strides -> [n][rows][cols][4].
 *   heist_train_pool: feat [n][1024] = adaptive_avg_pool2d(a3, (4, 4)) flattened C-major.
 *   heist_train_pool_bwd: d3 = mask3 * the pool's input gradient of dfeat [n][1024], mask3 the
 *     ReLU mask bits of conv3's forward. */
int heist_train_conv_supported(int rows, int cols);
int heist_train_conv_frag_floats(int layer, int mode);
int heist_train_conv_pack(int layer, int mode, const float* w, float* frag, heist_stream_t stream);
int heist_train_conv(int layer, int mode, const float* x, int n, int rows, int cols, const float* frag,
                     const float* bias, uint8_t* mask_bits, float* y, int* queue, heist_stream_t stream);
int64_t heist_train_conv_partial_floats(int layer, int n, int rows, int cols);
int heist_train_conv_wgrad(int layer, const float* dy, const float* x, int n, int rows, int cols, float* partial,
                           float* dw, float* db, int* queue, heist_stream_t stream);
int heist_train_obs_nhwc4(const float* obs, int n, int rows, int cols, int64_t stride_n, int64_t stride_c,
                          int64_t stride_h, int64_t stride_w, float* x4, heist_stream_t stream);
int heist_train_pool(const float* a3, int n, int rows, int cols, float* feat, heist_stream_t stream);
int heist_train_pool_bwd(const float* dfeat, const uint8_t* mask3_bits, int n, int rows, int cols, float* d3,
                         heist_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif
