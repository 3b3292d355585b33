/* heist_oracle.c -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 * See heist_oracle.h.  Build: oracle/Makefile (gcc -O2 -ffp-contract=off). */
#include "heist_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

enum { T_EMPTY = 0, T_WALL = 1, T_START = 2, T_VAULT = 3, T_CAMERA = 4, T_GUARD = 5 }; /* utils.py:31-37 */
enum { ST_RUNNING = 0, ST_DETECTED = 1, ST_VAULT = 2, ST_TIMEOUT = 3, ST_ALREADY_DONE = 4 };

/* CPython calls math.cos and math.sin separately; keep gcc from merging them into
 * sincos() (a different libm routine) by calling through volatile pointers. */
static double (*volatile p_cos)(double) = cos;
static double (*volatile p_sin)(double) = sin;
static double (*volatile p_atan2)(double, double) = atan2;

static const double kDegToRad = 3.141592653589793 / 180.0; /* CPython math.radians */
static const double kRadToDeg = 180.0 / 3.141592653589793; /* CPython math.degrees */

typedef struct { int row, col, range; double fov, heading, speed; } ocam;
typedef struct { int off, len, speed, range, idx; double fov, heading; } oguard;

struct oracle_env {
  int R, C, max_steps, sr, sc, vr, vc;
  double r_step, r_detect, r_vault;
  int budget_total, spent;
  int8_t* grid;
  uint8_t* vis;
  uint8_t* wall;
  int n_walls, n_cams, n_guards;
  ocam* cams;
  oguard* guards;
  int32_t* paths; /* [n_path_points][2] */
  int pos_r, pos_c, tick, done, detected, vault_reached, prev_dist, initial_dist;
};

/* Python float % 360.0 (floatobject.c float_rem): remainder takes the divisor's sign. */
static double py_mod(double x, double m) {
  double r = fmod(x, m);
  if (r != 0.0) {
    if ((m < 0) != (r < 0)) r += m;
  } else {
    r = copysign(0.0, m);
  }
  return r;
}
static int py_imod(long a, long m) { long r = a % m; if (r != 0 && ((r < 0) != (m < 0))) r += m; return (int)r; }
static int iabs(int a) { return a < 0 ? -a : a; }
static int manhattan(int r0, int c0, int r1, int c1) { return iabs(r0 - r1) + iabs(c0 - c1); } /* utils.py:122-124 */

oracle_env* oracle_env_create(int R, int C, int max_steps, int sr, int sc, int vr, int vc,
                              double r_step, double r_detect, double r_vault, int budget) {
  oracle_env* e = (oracle_env*)calloc(1, sizeof(oracle_env));
  e->R = R; e->C = C; e->max_steps = max_steps; e->sr = sr; e->sc = sc; e->vr = vr; e->vc = vc;
  e->r_step = r_step; e->r_detect = r_detect; e->r_vault = r_vault; e->budget_total = budget;
  e->grid = (int8_t*)calloc((size_t)R * C, 1);
  e->vis = (uint8_t*)calloc((size_t)R * C, 1);
  e->wall = (uint8_t*)calloc((size_t)R * C, 1);
  oracle_env_set_layout(e, 0, NULL, 0, NULL, 0, NULL, NULL, NULL);
  e->pos_r = sr; e->pos_c = sc;
  e->prev_dist = e->initial_dist = manhattan(sr, sc, vr, vc);
  return e;
}

void oracle_env_destroy(oracle_env* e) {
  if (!e) return;
  free(e->grid); free(e->vis); free(e->wall); free(e->cams); free(e->guards); free(e->paths); free(e);
}

void oracle_env_set_budget(oracle_env* e, int total) { e->budget_total = total; e->spent = 0; }

static int purchase(oracle_env* e, int cost) { /* budget.py:48-58 */
  if (e->budget_total - e->spent >= cost) { e->spent += cost; return 1; }
  return 0;
}

static int valid_placement(const oracle_env* e, int r, int c) { /* environment.py:160-167 */
  if (r <= 0 || r >= e->R - 1 || c <= 0 || c >= e->C - 1) return 0;
  return e->grid[r * e->C + c] == T_EMPTY;
}

int oracle_env_set_layout(oracle_env* e, int n_walls, const int32_t* walls, int n_cams, const double* cams,
                          int n_guards, const int64_t* guard_i, const double* guard_fov, const int32_t* paths) {
  int R = e->R, C = e->C;
  /* _reset_layout + create_empty_grid (environment.py:169-177, utils.py:131-139) */
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < C; ++c)
      e->grid[r * C + c] = (r == 0 || r == R - 1 || c == 0 || c == C - 1) ? T_WALL : T_EMPTY;
  e->grid[e->sr * C + e->sc] = T_START;
  e->grid[e->vr * C + e->vc] = T_VAULT;
  e->spent = 0;
  e->n_walls = e->n_cams = e->n_guards = 0;
  free(e->cams); free(e->guards); free(e->paths);
  e->cams = (ocam*)calloc(n_cams > 0 ? n_cams : 1, sizeof(ocam));
  e->guards = (oguard*)calloc(n_guards > 0 ? n_guards : 1, sizeof(oguard));
  int n_pts = 0;
  for (int g = 0; g < n_guards; ++g) n_pts += (int)guard_i[4 * g + 1];
  e->paths = (int32_t*)calloc(2 * (n_pts > 0 ? n_pts : 1), sizeof(int32_t));
  for (int i = 0; i < n_walls; ++i) { /* :118-121 */
    int r = walls[2 * i], c = walls[2 * i + 1];
    if (valid_placement(e, r, c) && purchase(e, 1)) { e->grid[r * C + c] = T_WALL; e->n_walls++; }
  }
  for (int i = 0; i < n_cams; ++i) { /* :124-135 */
    const double* p = cams + 6 * i;
    int r = (int)p[0], c = (int)p[1];
    if (valid_placement(e, r, c) && purchase(e, 3)) {
      ocam* k = &e->cams[e->n_cams++];
      k->row = r; k->col = c; k->fov = p[2]; k->heading = p[3]; k->speed = p[4]; k->range = (int)p[5];
      e->grid[r * C + c] = T_CAMERA;
    }
  }
  int pts = 0;
  for (int i = 0; i < n_guards; ++i) { /* :138-149 -- no placement check */
    int off = (int)guard_i[4 * i], len = (int)guard_i[4 * i + 1];
    if (len > 0 && purchase(e, 5)) {
      oguard* g = &e->guards[e->n_guards++];
      g->off = pts; g->len = len; g->speed = (int)guard_i[4 * i + 2]; g->range = (int)guard_i[4 * i + 3];
      g->fov = guard_fov[i]; g->idx = 0; g->heading = 0.0;
      memcpy(e->paths + 2 * pts, paths + 2 * off, sizeof(int32_t) * 2 * len);
      pts += len;
      e->grid[e->paths[2 * g->off] * C + e->paths[2 * g->off + 1]] = T_GUARD;
    }
  }
  return oracle_bfs(e->grid, R, C, e->sr, e->sc, e->vr, e->vc);
}

/* --- raycasts ------------------------------------------------------------------- */

static void cast_camera(int R, int C, const uint8_t* walls, int row, int col, double fov, double heading,
                        int range, uint8_t* vis) { /* security.py:53-101 */
  double half_fov = fov / 2.0;
  int num_rays = (int)(fov * 2);
  if (num_rays < 30) num_rays = 30;
  static const double subs[3] = {0.0, 0.5, 1.0}; /* np.linspace(0, 1, 3) */
  for (int i = 0; i <= num_rays; ++i) {
    double angle = (heading - half_fov) + (fov * i) / num_rays;
    double rad = angle * kDegToRad;
    double dx = p_cos(rad);
    double dy = -p_sin(rad);
    int blocked = 0;
    for (int step = 1; step <= range && !blocked; ++step) {
      for (int s = 0; s < 3; ++s) {
        double dist = (double)(step - 1) + subs[s] * 1.0;
        if (dist == 0.0) continue;
        double fx = (double)col + dx * dist;
        double fy = (double)row + dy * dist;
        int c = (int)rint(fx), r = (int)rint(fy); /* Python round(): half to even */
        if (r >= 0 && r < R && c >= 0 && c < C) {
          if (walls[r * C + c]) { blocked = 1; break; }
          if (!(r == row && c == col)) vis[r * C + c] = 1;
        } else {
          blocked = 1;
          break;
        }
      }
    }
  }
}

static void cast_guard(int R, int C, const uint8_t* walls, int row, int col, double fov, double heading,
                       int range, uint8_t* vis) { /* security.py:161-192 */
  double half_fov = fov / 2.0;
  int num_rays = (int)(fov * 2);
  if (num_rays < 30) num_rays = 30;
  for (int i = 0; i <= num_rays; ++i) {
    double angle = (heading - half_fov) + (fov * i) / num_rays;
    double rad = angle * kDegToRad;
    double dx = p_cos(rad);
    double dy = -p_sin(rad);
    for (int step = 1; step <= range; ++step) {
      double fx = (double)col + dx * step;
      double fy = (double)row + dy * step;
      int c = (int)rint(fx), r = (int)rint(fy);
      if (r >= 0 && r < R && c >= 0 && c < C) {
        if (walls[r * C + c]) break;
        if (!(r == row && c == col)) vis[r * C + c] = 1;
      } else {
        break;
      }
    }
  }
}

void oracle_cone(int kind, int R, int C, const uint8_t* walls, int row, int col, double fov, double heading,
                 int range, uint8_t* vis) {
  memset(vis, 0, (size_t)R * C);
  if (kind == 0) cast_camera(R, C, walls, row, col, fov, heading, range, vis);
  else cast_guard(R, C, walls, row, col, fov, heading, range, vis);
}

static void update_visibility(oracle_env* e) { /* visibility.py:31-65 */
  int R = e->R, C = e->C;
  for (int i = 0; i < R * C; ++i) e->wall[i] = e->grid[i] == T_WALL;
  memset(e->vis, 0, (size_t)R * C);
  for (int i = 0; i < e->n_cams; ++i) {
    ocam* k = &e->cams[i];
    cast_camera(R, C, e->wall, k->row, k->col, k->fov, k->heading, k->range, e->vis);
  }
  for (int i = 0; i < e->n_guards; ++i) {
    oguard* g = &e->guards[i];
    int gr = e->paths[2 * (g->off + g->idx)], gc = e->paths[2 * (g->off + g->idx) + 1];
    cast_guard(R, C, e->wall, gr, gc, g->fov, g->heading, g->range, e->vis);
    e->vis[gr * C + gc] = 1;
  }
}

/* --- env ------------------------------------------------------------------------ */

void oracle_env_reset(oracle_env* e) { /* environment.py:183-214 */
  e->pos_r = e->sr; e->pos_c = e->sc; e->tick = 0;
  e->done = e->detected = e->vault_reached = 0;
  e->prev_dist = e->initial_dist = manhattan(e->sr, e->sc, e->vr, e->vc);
  for (int i = 0; i < e->n_guards; ++i) e->guards[i].idx = 0; /* headings carry over */
  update_visibility(e);
}

static const int kDR[5] = {0, -1, 1, 0, 0}, kDC[5] = {0, 0, 0, -1, 1}; /* environment.py:52-58 */

double oracle_env_step(oracle_env* e, int a, int* done, int* status) {
  if (e->done) { *done = 1; *status = ST_ALREADY_DONE; return 0.0; }
  double reward = e->r_step;
  int st = ST_RUNNING;
  int nr = e->pos_r + kDR[a], nc = e->pos_c + kDC[a];
  if (nr >= 0 && nr < e->R && nc >= 0 && nc < e->C && e->grid[nr * e->C + nc] != T_WALL) {
    e->pos_r = nr; e->pos_c = nc;
  }
  for (int i = 0; i < e->n_cams; ++i) /* security.py:49-51 */
    e->cams[i].heading = py_mod(e->cams[i].heading + e->cams[i].speed * 1, 360.0);
  for (int i = 0; i < e->n_guards; ++i) { /* security.py:145-159 */
    oguard* g = &e->guards[i];
    if (g->len < 2) continue;
    int old = g->idx;
    g->idx = py_imod((long)g->idx + (long)g->speed * 1, g->len);
    int dr = e->paths[2 * (g->off + g->idx)] - e->paths[2 * (g->off + old)];
    int dc = e->paths[2 * (g->off + g->idx) + 1] - e->paths[2 * (g->off + old) + 1];
    if (dr != 0 || dc != 0) g->heading = py_mod(p_atan2((double)-dr, (double)dc) * kRadToDeg, 360.0);
  }
  update_visibility(e);
  int curr = manhattan(e->pos_r, e->pos_c, e->vr, e->vc);
  reward += (e->prev_dist - curr) * 0.1;
  e->prev_dist = curr;
  if (curr <= 3 && e->initial_dist > 3) reward += 0.05 * (3 - curr);
  if (e->vis[e->pos_r * e->C + e->pos_c]) {
    e->detected = 1; reward += e->r_detect; e->done = 1; st = ST_DETECTED;
  }
  if (e->pos_r == e->vr && e->pos_c == e->vc) {
    e->vault_reached = 1; reward += e->r_vault; e->done = 1; st = ST_VAULT;
  }
  e->tick += 1;
  if (e->tick >= e->max_steps) {
    e->done = 1; st = ST_TIMEOUT;
    double frac = 1.0 - (double)curr / (double)(e->initial_dist > 1 ? e->initial_dist : 1);
    if (frac < 0) frac = 0; /* max(0, ...) yields int 0 -> 0 * 2.0 */
    reward += frac * 2.0;
  }
  *done = e->done;
  *status = st;
  return reward;
}

void oracle_env_state_tensor(const oracle_env* e, float* out) {
  int R = e->R, C = e->C, RC = R * C;
  for (int i = 0; i < RC; ++i) out[i] = (float)e->grid[i] / 5.0f; /* :319, float32 / 5 */
  for (int i = 0; i < RC; ++i) out[RC + i] = e->vis[i] ? 1.0f : 0.0f;
  float* p = out + 2 * RC;
  for (int i = 0; i < RC; ++i) p[i] = 0.0f;
  p[e->pos_r * C + e->pos_c] = 1.0f;
  p[e->vr * C + e->vc] = -1.0f;
  int max_d = R + C;
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < C; ++c) {
      int d = manhattan(r, c, e->vr, e->vc);
      double v = -0.3 * ((double)d / (double)max_d);
      p[r * C + c] = p[r * C + c] + (float)v; /* NEP 50: float32 + weak python float */
    }
}

void oracle_env_info(const oracle_env* e, int32_t* info) {
  info[0] = e->pos_r; info[1] = e->pos_c; info[2] = e->tick; info[3] = e->done; info[4] = e->detected;
  info[5] = e->vault_reached; info[6] = e->n_walls; info[7] = e->n_cams; info[8] = e->n_guards; info[9] = e->spent;
}
void oracle_env_vis(const oracle_env* e, uint8_t* out) { memcpy(out, e->vis, (size_t)e->R * e->C); }
void oracle_env_grid(const oracle_env* e, int8_t* out) { memcpy(out, e->grid, (size_t)e->R * e->C); }
void oracle_env_headings(const oracle_env* e, double* cam_h, int32_t* g_idx, double* g_h) {
  for (int i = 0; i < e->n_cams; ++i) cam_h[i] = e->cams[i].heading;
  for (int i = 0; i < e->n_guards; ++i) { g_idx[i] = e->guards[i].idx; g_h[i] = e->guards[i].heading; }
}

/* --- BFS ------------------------------------------------------------------------ */

int oracle_bfs(const int8_t* grid, int R, int C, int sr, int sc, int gr, int gc) { /* utils.py:52-85 */
  if (sr == gr && sc == gc) return 1;
  int n = R * C;
  uint8_t* seen = (uint8_t*)calloc(n, 1);
  int* q = (int*)malloc(sizeof(int) * n);
  int head = 0, tail = 0, found = 0;
  q[tail++] = sr * C + sc;
  seen[sr * C + sc] = 1;
  static const int dr[4] = {-1, 1, 0, 0}, dc[4] = {0, 0, -1, 1};
  while (head < tail && !found) {
    int r = q[head] / C, c = q[head] % C;
    ++head;
    for (int k = 0; k < 4; ++k) {
      int nr = r + dr[k], nc = c + dc[k];
      if (nr < 0 || nr >= R || nc < 0 || nc >= C || seen[nr * C + nc]) continue;
      if (grid[nr * C + nc] != T_WALL) {
        if (nr == gr && nc == gc) { found = 1; break; }
        seen[nr * C + nc] = 1;
        q[tail++] = nr * C + nc;
      }
    }
  }
  free(seen); free(q);
  return found;
}

/* --- GAE and PPO loss -------------------------------------------------------------- */

void oracle_gae(const float* r, const float* v, const float* d, int T, double gamma, double lam, float* adv) {
  /* torch float32 ops with Python-float scalars cast to float32 (agents/solver.py:234-242) */
  float g = (float)gamma, gl = (float)(gamma * lam), last = 0.0f;
  for (int t = T - 1; t >= 0; --t) {
    float nv = (t == T - 1) ? 0.0f : v[t + 1];
    float nd = 1.0f - d[t];
    float delta = (r[t] + (g * nv) * nd) - v[t];
    last = delta + (gl * nd) * last;
    adv[t] = last;
  }
}

void oracle_ppo_loss(int M, int A, const float* logits, const float* values, const int64_t* actions,
                     const float* old_logp, const float* adv, const float* ret, double clip, double vcoef,
                     double ecoef, float* parts, float* dlogits, float* dvalues) {
  const float eps = 1.1920928955078125e-07f; /* torch.finfo(float32).eps (clamp_probs) */
  double pg_sum = 0, vl_sum = 0, ent_sum = 0;
  float lo = (float)(1.0 - clip), hi = (float)(1.0 + clip);
  float* p = (float*)malloc(sizeof(float) * A);
  float* pn = (float*)malloc(sizeof(float) * A);
  float* lc = (float*)malloc(sizeof(float) * A);
  float* gpn = (float*)malloc(sizeof(float) * A);
  for (int i = 0; i < M; ++i) {
    const float* x = logits + (size_t)i * A;
    float mx = x[0];
    for (int j = 1; j < A; ++j) mx = x[j] > mx ? x[j] : mx;
    float s = 0;
    for (int j = 0; j < A; ++j) { p[j] = expf(x[j] - mx); s += p[j]; }
    for (int j = 0; j < A; ++j) p[j] = p[j] / s;               /* F.softmax */
    float S = 0;
    for (int j = 0; j < A; ++j) S += p[j];
    for (int j = 0; j < A; ++j) pn[j] = p[j] / S;              /* Categorical(probs) normalises */
    float ent = 0;
    for (int j = 0; j < A; ++j) {
      float c = pn[j] < eps ? eps : (pn[j] > 1 - eps ? 1 - eps : pn[j]);
      lc[j] = logf(c);                                           /* probs_to_logits */
      ent -= pn[j] * lc[j];
    }
    int a = (int)actions[i];
    float ratio = expf(lc[a] - old_logp[i]);
    float s1 = ratio * adv[i];
    float rc = ratio < lo ? lo : (ratio > hi ? hi : ratio);
    float s2 = rc * adv[i];
    pg_sum += (s1 < s2 ? s1 : s2);
    float dv = values[i] - ret[i];
    vl_sum += (double)dv * dv;
    ent_sum += ent;
    /* backward: d(min)/d(ratio), ties split evenly like torch.min */
    int in_clip = ratio >= lo && ratio <= hi;
    float dmin = s1 < s2 ? adv[i] : (s2 < s1 ? (in_clip ? adv[i] : 0.0f) : 0.5f * adv[i] + 0.5f * (in_clip ? adv[i] : 0.0f));
    float g_logp = -(dmin * ratio) / (float)M;
    for (int j = 0; j < A; ++j) {
      int unclamped = pn[j] >= eps && pn[j] <= 1 - eps;
      float g = (float)(ecoef / M) * (lc[j] + (unclamped ? 1.0f : 0.0f));
      if (j == a && unclamped) g += g_logp / pn[j];
      gpn[j] = g;
    }
    float dot = 0;
    for (int j = 0; j < A; ++j) dot += gpn[j] * p[j];
    float gp_dot = 0;
    float* gp = lc; /* reuse */
    for (int j = 0; j < A; ++j) { gp[j] = gpn[j] / S - dot / (S * S); gp_dot += gp[j] * p[j]; }
    for (int j = 0; j < A; ++j) dlogits[(size_t)i * A + j] = p[j] * (gp[j] - gp_dot);
    dvalues[i] = (float)(vcoef * 2.0 / M) * dv;
  }
  float pg = (float)(-pg_sum / M), vl = (float)(vl_sum / M), ent = (float)(ent_sum / M);
  parts[0] = pg + (float)vcoef * vl - (float)ecoef * ent;
  parts[1] = pg; parts[2] = vl; parts[3] = ent;
  free(p); free(pn); free(lc); free(gpn);
}

/* --- CPU baseline driver ------------------------------------------------------------ */

typedef struct { oracle_env** envs; int lo, hi, n_steps; uint64_t seed; int64_t steps; } run_arg;

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void* run_worker(void* p) {
  run_arg* a = (run_arg*)p;
  int maxrc = 0;
  for (int i = a->lo; i < a->hi; ++i) if (a->envs[i]->R * a->envs[i]->C > maxrc) maxrc = a->envs[i]->R * a->envs[i]->C;
  float* st = (float*)malloc(sizeof(float) * 3 * (maxrc > 0 ? maxrc : 1));
  uint64_t s = a->seed ^ (uint64_t)a->lo * 0x632BE59BD9B4E019ull;
  for (int t = 0; t < a->n_steps; ++t)
    for (int i = a->lo; i < a->hi; ++i) {
      oracle_env* e = a->envs[i];
      int done, status;
      oracle_env_step(e, (int)(splitmix(&s) % 5), &done, &status);
      if (done) oracle_env_reset(e);
      oracle_env_state_tensor(e, st);
      a->steps++;
    }
  free(st);
  return NULL;
}

int64_t oracle_run_random(oracle_env** envs, int n, int n_steps, uint64_t seed, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > n) n_threads = n;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
  run_arg* args = (run_arg*)calloc(n_threads, sizeof(run_arg));
  for (int k = 0; k < n_threads; ++k) {
    args[k].envs = envs; args[k].lo = (int)((int64_t)n * k / n_threads); args[k].hi = (int)((int64_t)n * (k + 1) / n_threads);
    args[k].n_steps = n_steps; args[k].seed = seed;
    pthread_create(&th[k], NULL, run_worker, &args[k]);
  }
  int64_t total = 0;
  for (int k = 0; k < n_threads; ++k) { pthread_join(th[k], NULL); total += args[k].steps; }
  free(th); free(args);
  return total;
}
