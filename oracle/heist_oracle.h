/* heist_oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 *
 * This is the parity checker, never the product: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load liboracle.so.  Every function restates a
 * piece of the Python reference (paths relative to /root/reference) and is pinned
 * against golden vectors generated from that reference (tests/golden/).
 *
 * Numerics: compiled with -O2 -ffp-contract=off; trig goes through the host libm
 * sin/cos exactly as CPython math.sin/cos do (never fused into sincos()).
 */
#ifndef HEIST_ORACLE_H
#define HEIST_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_env oracle_env;

/* EnvironmentConfig (environment.py:18-37) + BudgetManager total (budget.py:36). */
oracle_env* oracle_env_create(int R, int C, int max_steps, int sr, int sc, int vr, int vc,
                              double r_step, double r_detect, double r_vault, int budget);
void oracle_env_destroy(oracle_env* e);
void oracle_env_set_budget(oracle_env* e, int total); /* budget.py:64-67 scale_budget */

/* HeistEnvironment.set_layout (environment.py:102-152).
 * walls [n_walls][2]; cams [n_cams][6] = row, col, fov, heading, speed, range;
 * guard_i [n_guards][4] = path offset into paths, path length, speed, range;
 * guard_fov [n_guards]; paths [*][2].  Returns is_level_valid(). */
int oracle_env_set_layout(oracle_env* e, int n_walls, const int32_t* walls, int n_cams, const double* cams,
                          int n_guards, const int64_t* guard_i, const double* guard_fov, const int32_t* paths);
void oracle_env_reset(oracle_env* e);                                 /* environment.py:183-214 */
double oracle_env_step(oracle_env* e, int action, int* done, int* status); /* environment.py:216-299 */
void oracle_env_state_tensor(const oracle_env* e, float* out);      /* environment.py:347-374 */

/* Introspection for parity tests. info = pos_r, pos_c, tick, done, detected, vault_reached,
 * n_walls, n_cams, n_guards, spent. */
void oracle_env_info(const oracle_env* e, int32_t* info);
void oracle_env_vis(const oracle_env* e, uint8_t* out);              /* [R*C] */
void oracle_env_grid(const oracle_env* e, int8_t* out);              /* [R*C] */
void oracle_env_headings(const oracle_env* e, double* cam_h, int32_t* g_idx, double* g_h);

/* Camera.get_vision_cone_tiles (security.py:53-101) when kind == 0,
 * Guard.get_visible_tiles (security.py:161-192) when kind == 1. walls/vis [R*C]. */
void oracle_cone(int kind, int R, int C, const uint8_t* walls, int row, int col, double fov,
                 double heading, int range, uint8_t* vis);

/* bfs_path_exists (utils.py:52-85). */
int oracle_bfs(const int8_t* grid, int R, int C, int sr, int sc, int gr, int gc);

/* SolverAgent._compute_gae on one flat buffer (agents/solver.py:228-244). */
void oracle_gae(const float* r, const float* v, const float* d, int T, double gamma, double lam, float* adv);

/* Clipped PPO loss of SolverAgent.update (agents/solver.py:172-193) for one minibatch,
 * with d(loss)/d(logits) and d(loss)/d(values).  parts = total, policy, value, entropy. */
void oracle_ppo_loss(int M, int A, const float* logits, const float* values, const int64_t* actions,
                     const float* old_logp, const float* adv, const float* ret, double clip, double vcoef,
                     double ecoef, float* parts, float* dlogits, float* dvalues);

/* CPU baseline driver: steps n envs (all already laid out) with uniform random actions for
 * n_steps ticks each, auto-resetting finished envs and building the state tensor each tick
 * (the training.py:522-532 inner loop without the policy).  Uses n_threads pthreads.
 * Returns the number of env-steps taken. */
int64_t oracle_run_random(oracle_env** envs, int n, int n_steps, uint64_t seed, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
