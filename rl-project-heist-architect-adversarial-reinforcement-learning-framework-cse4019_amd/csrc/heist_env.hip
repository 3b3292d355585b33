// heist_env.hip -- CDNA4 kernels for the batched Heist environment.
//
// One 64-lane wavefront (= one workgroup) owns one environment:
//   * the env's tile grid and its visibility plane live in LDS as bytes;
//   * cameras and guards are flattened into one ray list; lane l casts rays
//     l, l+64, ... (security.py:53-101, :161-192) and marks visible tiles with
//     idempotent byte stores (no atomics);
//   * the solver/reward logic (environment.py:216-299) runs wave-uniform;
//   * the [3][R][C] float32 observation (environment.py:347-374) leaves in
//     16-byte coalesced stores.
// Arithmetic follows the reference's IEEE double semantics exactly: no FMA
// contraction, half-to-even rint(), glibc-exact sin/cos (heist_trig.h).
#include "heist_device.h"
#include "heist_trig.h"

#pragma clang fp contract(off)

namespace heist {

__constant__ double kSinCosTab[4 * HEIST_SINCOS_TAB_ROWS] = HEIST_SINCOS_TAB_INIT;
__constant__ int kActDR[5] = {0, -1, 1, 0, 0};  // environment.py:52-58
__constant__ int kActDC[5] = {0, 0, 0, -1, 1};

__device__ __forceinline__ int iabs_(int a) { return a < 0 ? -a : a; }

// Python float % 360.0 (floatobject.c float_rem: remainder takes the divisor's sign).
__device__ __forceinline__ double py_mod360(double x) {
  double r = fmod(x, 360.0);
  if (r != 0.0) {
    if (r < 0.0) r += 360.0;
  } else {
    r = 0.0;
  }
  return r;
}

__device__ __forceinline__ int py_imod(int a, int m) {
  int r = a % m;
  return (r != 0 && ((r < 0) != (m < 0))) ? r + m : r;
}

// Dynamic LDS carve-up for one env: grid bytes, visibility bytes, emitter table.
struct EnvLds {
  uint8_t* grid;
  uint8_t* vis;
  Emit* em;
  int* meta;  // [0] = number of emitters, [1] = total rays
};

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

__host__ inline size_t env_lds_bytes(int RC, int n_emit) {
  return align16(RC) * 2 + align16(sizeof(Emit) * (n_emit > 0 ? n_emit : 1)) + 16;
}

__device__ __forceinline__ EnvLds carve(unsigned char* smem, int RC, int n_emit) {
  EnvLds L;
  L.grid = smem;
  L.vis = smem + align16(RC);
  L.em = reinterpret_cast<Emit*>(smem + 2 * align16(RC));
  L.meta = reinterpret_cast<int*>(smem + 2 * align16(RC) + align16(sizeof(Emit) * (n_emit > 0 ? n_emit : 1)));
  return L;
}

// ---------------------------------------------------------------------------
// Raycasting
// ---------------------------------------------------------------------------

// Cast every ray of the env's emitters and mark visible tiles (visibility.py:48-57).
// Camera rays sample dist = 0.5, 1.0, ..., range (np.linspace(0,1,3) sub-steps; the
// duplicated integer samples of security.py:78-82 are idempotent and skipped); guard
// rays sample dist = 1..range.  A wall or the grid edge ends the ray; the emitter's own
// tile is never marked by its rays.
__device__ void cast_rays(const EnvLds& L, int R, int C) {
  const int lane = threadIdx.x & 63;
  const int n_em = L.meta[0];
  const int total = L.meta[1];
  int k = 0;
  for (int j = lane; j < total; j += 64) {
    while (k + 1 < n_em && L.em[k + 1].first <= j) ++k;
    const Emit E = L.em[k];
    const int i = j - E.first;
    const double angle = E.hmh + (E.fov * (double)i) / (double)E.num_rays;  // security.py:70
    const double rad = angle * kDegToRad;                                   // math.radians
    const double dx = heist_trig::cos(rad, kSinCosTab);
    const double dy = -heist_trig::sin(rad, kSinCosTab);
    const double stride = E.kind == 0 ? 0.5 : 1.0;
    const int n_samp = E.kind == 0 ? 2 * E.range : E.range;
    const double col = (double)E.col, row = (double)E.row;
    for (int s = 1; s <= n_samp; ++s) {
      const double dist = stride * (double)s;  // exact
      const double fx = col + dx * dist;
      const double fy = row + dy * dist;
      const int c = (int)rint(fx);  // Python round(): half to even
      const int r = (int)rint(fy);
      if ((unsigned)r >= (unsigned)R || (unsigned)c >= (unsigned)C) break;
      const int cell = r * C + c;
      if (L.grid[cell] == kWall) break;
      if (r != E.row || c != E.col) L.vis[cell] = 1;
    }
  }
}

// Lane 0 turns per-emitter ray counts into the flattened ray index (call between barriers).
__device__ __forceinline__ void index_rays(const EnvLds& L, int n_em) {
  if ((threadIdx.x & 63) == 0) {
    int t = 0;
    for (int k = 0; k < n_em; ++k) {
      L.em[k].first = t;
      t += L.em[k].num_rays + 1;
    }
    L.meta[0] = n_em;
    L.meta[1] = t;
  }
}

__device__ __forceinline__ void guard_pos(const EnvParams& p, int e, int g, int idx, int* r, int* c) {
  const uint16_t pt = p.paths[((size_t)e * p.max_guards + g) * p.max_path + idx];
  *r = pt & 0xff;
  *c = pt >> 8;
}

// Build the emitter table from the env's cameras and guards at their current pose.
// Lanes [0, n_cams) take cameras, [n_cams, n_cams + n_guards) guards.
__device__ __forceinline__ void build_emitters(const EnvParams& p, int e, const EnvScalars& s, const EnvLds& L) {
  const int lane = threadIdx.x & 63;
  if (lane < s.n_cams) {
    const Cam cm = p.cams[(size_t)e * p.max_cams + lane];
    Emit E;
    E.hmh = cm.heading - cm.fov / 2.0;
    E.fov = cm.fov;
    E.row = cm.row; E.col = cm.col; E.range = cm.range; E.num_rays = cm.num_rays;
    E.first = 0; E.kind = 0;
    L.em[lane] = E;
  } else if (lane < s.n_cams + s.n_guards) {
    const int g = lane - s.n_cams;
    const Guard gd = p.guards[(size_t)e * p.max_guards + g];
    int r, c;
    guard_pos(p, e, g, gd.idx, &r, &c);
    Emit E;
    E.hmh = gd.heading - gd.fov / 2.0;
    E.fov = gd.fov;
    E.row = r; E.col = c; E.range = gd.range; E.num_rays = gd.num_rays;
    E.first = 0; E.kind = 1;
    L.em[lane] = E;
  }
}

// Full visibility recompute (visibility.py:31-65) for the env's current pose.
// Must be entered by the whole (single-wave) workgroup.
__device__ __forceinline__ void compute_visibility(const EnvParams& p, int e, const EnvScalars& s, const EnvLds& L) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < p.RC; i += 64) L.vis[i] = 0;
  build_emitters(p, e, s, L);
  __syncthreads();
  index_rays(L, s.n_cams + s.n_guards);
  __syncthreads();
  cast_rays(L, p.R, p.C);
  __syncthreads();
  if (lane >= s.n_cams && lane < s.n_cams + s.n_guards) {  // a guard's own tile (visibility.py:59)
    const Emit E = L.em[lane];
    L.vis[E.row * p.C + E.col] = 1;
  }
  __syncthreads();
}

__device__ __forceinline__ void load_grid(const EnvParams& p, int e, const EnvLds& L) {
  const int lane = threadIdx.x & 63;
  const uint8_t* src = p.grid + (size_t)e * p.RC;
  if ((p.RC & 3) == 0) {
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d4 = reinterpret_cast<uint32_t*>(L.grid);
    for (int i = lane; i < p.RC / 4; i += 64) d4[i] = s4[i];
  } else {
    for (int i = lane; i < p.RC; i += 64) L.grid[i] = src[i];
  }
}

// Observation row [3][R][C] (environment.py:347-374): occupancy / 5, visibility, and the
// position channel (static planes with the solver and vault cells patched).
__device__ __forceinline__ void write_obs(const EnvParams& p, int e, const EnvScalars& s, const EnvLds& L,
                                          float* __restrict__ obs) {
  const int lane = threadIdx.x & 63;
  const int RC = p.RC;
  float* o = obs + (size_t)e * 3 * RC;
  const int solver = s.pos_r * p.C + s.pos_c;
  const int vault = p.vr * p.C + p.vc;
  if ((RC & 3) == 0) {
    const int n4 = 3 * RC / 4;
    for (int q = lane; q < n4; q += 64) {
      const int o4 = q * 4;
      const int ch = o4 / RC;
      const int cell = o4 - ch * RC;
      float4 v;
      if (ch == 0) {
        const uint32_t b = *reinterpret_cast<const uint32_t*>(L.grid + cell);
        v.x = p.tile_lut[b & 7]; v.y = p.tile_lut[(b >> 8) & 7];
        v.z = p.tile_lut[(b >> 16) & 7]; v.w = p.tile_lut[(b >> 24) & 7];
      } else if (ch == 1) {
        const uint32_t b = *reinterpret_cast<const uint32_t*>(L.vis + cell);
        v.x = (b & 0xff) ? 1.0f : 0.0f; v.y = (b & 0xff00) ? 1.0f : 0.0f;
        v.z = (b & 0xff0000) ? 1.0f : 0.0f; v.w = (b & 0xff000000u) ? 1.0f : 0.0f;
      } else {
        v = *reinterpret_cast<const float4*>(p.plane0 + cell);
        if ((unsigned)(solver - cell) < 4u) {
          const int k = solver - cell;
          const float sv = p.plane1[solver];
          if (k == 0) v.x = sv; else if (k == 1) v.y = sv; else if (k == 2) v.z = sv; else v.w = sv;
        }
        if ((unsigned)(vault - cell) < 4u) {  // vault wins if the solver stands on it
          const int k = vault - cell;
          if (k == 0) v.x = p.vault_val; else if (k == 1) v.y = p.vault_val;
          else if (k == 2) v.z = p.vault_val; else v.w = p.vault_val;
        }
      }
      *reinterpret_cast<float4*>(o + o4) = v;
    }
  } else {
    for (int q = lane; q < 3 * RC; q += 64) {
      const int ch = q / RC;
      const int cell = q - ch * RC;
      float v;
      if (ch == 0) v = p.tile_lut[L.grid[cell] & 7];
      else if (ch == 1) v = L.vis[cell] ? 1.0f : 0.0f;
      else v = cell == vault ? p.vault_val : (cell == solver ? p.plane1[cell] : p.plane0[cell]);
      o[q] = v;
    }
  }
}

__device__ __forceinline__ void reset_solver(const EnvParams& p, EnvScalars& s) {  // environment.py:191-202
  s.pos_r = p.sr; s.pos_c = p.sc; s.tick = 0;
  s.done = 0; s.detected = 0; s.vault_reached = 0;
  s.prev_dist = s.initial_dist = iabs_(p.sr - p.vr) + iabs_(p.sc - p.vc);
}

// Same lane -> guard mapping as build_emitters, so each lane re-reads only its own store.
__device__ __forceinline__ void reset_guards(const EnvParams& p, int e, const EnvScalars& s) {
  const int lane = threadIdx.x & 63;
  if (lane >= s.n_cams && lane < s.n_cams + s.n_guards)
    p.guards[(size_t)e * p.max_guards + (lane - s.n_cams)].idx = 0;  // headings carry over
}

// ---------------------------------------------------------------------------
// step / reset
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(64) void step_kernel(EnvParams p, const int64_t* __restrict__ actions,
                                                   float* __restrict__ obs, float* __restrict__ rew,
                                                   double* __restrict__ rew64, uint8_t* __restrict__ done_out,
                                                   int8_t* __restrict__ status_out, int auto_reset) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const EnvLds L = carve(smem, p.RC, p.max_cams + p.max_guards);
  load_grid(p, e, L);
  EnvScalars s = p.scal[e];
  const bool act = !s.done;
  __syncthreads();

  double reward = 0.0;
  int status = kAlreadyDone;
  if (act) {
    // 1. move (environment.py:239-246)
    int a = (int)actions[e];
    if (a < 0 || a > 4) a = 0;
    const int nr = s.pos_r + kActDR[a], nc = s.pos_c + kActDC[a];
    if (nr >= 0 && nr < p.R && nc >= 0 && nc < p.C && L.grid[nr * p.C + nc] != kWall) {
      s.pos_r = nr;
      s.pos_c = nc;
    }
    // 2. cameras rotate, guards patrol (security.py:49-51, :145-159)
    if (lane < s.n_cams) {
      Cam* cm = p.cams + (size_t)e * p.max_cams + lane;
      cm->heading = py_mod360(cm->heading + cm->speed * 1.0);
    } else if (lane < s.n_cams + s.n_guards) {
      const int g = lane - s.n_cams;
      Guard* gd = p.guards + (size_t)e * p.max_guards + g;
      const int len = gd->len;
      if (len >= 2) {
        const int old = gd->idx;
        const int nidx = py_imod(old + gd->speed * 1, len);
        int r0, c0, r1, c1;
        guard_pos(p, e, g, old, &r0, &c0);
        guard_pos(p, e, g, nidx, &r1, &c1);
        const int dr = r1 - r0, dc = c1 - c0;
        if (dr != 0 || dc != 0) gd->heading = p.heading_tab[(dr + p.R - 1) * (2 * p.C - 1) + (dc + p.C - 1)];
        gd->idx = nidx;
      }
    }
  }
  __syncthreads();
  // 3. visibility (environment.py:257-258); an already-done env recomputes the same plane
  compute_visibility(p, e, s, L);

  if (act) {
    // 4-5. shaping, detection, vault, timeout (environment.py:235, :261-297)
    reward = p.r_step;
    status = kRunning;
    const int curr = iabs_(s.pos_r - p.vr) + iabs_(s.pos_c - p.vc);
    reward += (double)(s.prev_dist - curr) * 0.1;
    s.prev_dist = curr;
    if (curr <= 3 && s.initial_dist > 3) reward += 0.05 * (double)(3 - curr);
    if (L.vis[s.pos_r * p.C + s.pos_c]) {
      s.detected = 1;
      reward += p.r_detect;
      s.done = 1;
      status = kDetected;
    }
    if (s.pos_r == p.vr && s.pos_c == p.vc) {
      s.vault_reached = 1;
      reward += p.r_vault;
      s.done = 1;
      status = kVaultReached;
    }
    s.tick += 1;
    if (s.tick >= p.max_steps) {
      s.done = 1;
      status = kTimeout;
      double frac = 1.0 - (double)curr / (double)(s.initial_dist > 1 ? s.initial_dist : 1);
      if (frac < 0.0) frac = 0.0;
      reward += frac * 2.0;
    }
  }
  const int done_now = s.done;
  if (auto_reset && done_now) {  // wave-uniform: the barriers inside are safe
    reset_solver(p, s);
    reset_guards(p, e, s);
    __syncthreads();
    compute_visibility(p, e, s, L);
  }
  write_obs(p, e, s, L, obs);
  if (lane == 0) {
    rew[e] = (float)reward;
    if (rew64) rew64[e] = reward;
    done_out[e] = (uint8_t)done_now;
    status_out[e] = (int8_t)status;
    p.scal[e] = s;
  }
}

__global__ __launch_bounds__(64) void reset_kernel(EnvParams p, const uint8_t* __restrict__ mask,
                                                    float* __restrict__ obs) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = blockIdx.x;
  if (mask && !mask[e]) return;
  const EnvLds L = carve(smem, p.RC, p.max_cams + p.max_guards);
  load_grid(p, e, L);
  EnvScalars s = p.scal[e];
  reset_solver(p, s);
  reset_guards(p, e, s);
  __syncthreads();
  compute_visibility(p, e, s, L);
  write_obs(p, e, s, L, obs);
  if (threadIdx.x == 0) p.scal[e] = s;
}

// ---------------------------------------------------------------------------
// layout placement + BFS
// ---------------------------------------------------------------------------

// 4-neighbour reachability start -> goal over non-wall tiles (utils.py:52-85) as a
// wave-level bitboard flood fill: lane r holds row r as a 64-bit mask.
__device__ bool bfs_wave(uint64_t pass, int sr, int sc, int gr, int gc) {
  const int lane = threadIdx.x & 63;
  if (sr == gr && sc == gc) return true;
  uint64_t reach = lane == sr ? (1ull << sc) : 0ull;
  const uint64_t goal = lane == gr ? (1ull << gc) : 0ull;
  for (int it = 0; it < kMaxDim * kMaxDim; ++it) {
    const uint64_t up = __shfl(reach, lane > 0 ? lane - 1 : 0);
    const uint64_t dn = __shfl(reach, lane < 63 ? lane + 1 : 63);
    const uint64_t nb = (reach | (reach << 1) | (reach >> 1) | (lane > 0 ? up : 0ull) | (lane < 63 ? dn : 0ull)) & pass;
    const uint64_t nxt = reach | nb;
    const bool hit = __any((nxt & goal) != 0ull);
    const bool grew = __any(nxt != reach);
    reach = nxt;
    if (hit) return true;
    if (!grew) return false;
  }
  return false;
}

__device__ __forceinline__ uint64_t row_pass_mask(const uint8_t* g, int R, int C) {
  const int lane = threadIdx.x & 63;
  uint64_t m = 0;
  if (lane < R)
    for (int c = 0; c < C; ++c)
      if (g[lane * C + c] != kWall) m |= 1ull << c;
  return m;
}

__global__ __launch_bounds__(64) void set_layout_kernel(EnvParams p, int max_walls, const int32_t* __restrict__ wall_rc,
                                                         const int32_t* __restrict__ n_walls,
                                                         const double* __restrict__ cam_params,
                                                         const int32_t* __restrict__ n_cams,
                                                         const int32_t* __restrict__ guard_paths,
                                                         const int32_t* __restrict__ guard_meta,
                                                         const double* __restrict__ guard_fov,
                                                         const int32_t* __restrict__ n_guards,
                                                         const int32_t* __restrict__ budget,
                                                         uint8_t* __restrict__ valid_out) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const int R = p.R, C = p.C;
  const EnvLds L = carve(smem, p.RC, p.max_cams + p.max_guards);
  // _reset_layout + create_empty_grid (environment.py:169-177, utils.py:131-139)
  for (int i = lane; i < p.RC; i += 64) {
    const int r = i / C, c = i - (i / C) * C;
    L.grid[i] = (r == 0 || r == R - 1 || c == 0 || c == C - 1) ? kWall : kEmpty;
  }
  __syncthreads();
  if (lane == 0) {
    L.grid[p.sr * C + p.sc] = kStart;
    L.grid[p.vr * C + p.vc] = kVault;
    const int total = budget[e];
    int spent = 0, nw = 0, nc = 0, ng = 0;
    auto placeable = [&](int r, int c) {  // environment.py:160-167
      return r > 0 && r < R - 1 && c > 0 && c < C - 1 && L.grid[r * C + c] == kEmpty;
    };
    const int wn = min(n_walls[e], max_walls);
    for (int i = 0; i < wn; ++i) {  // :118-121
      const int r = wall_rc[((size_t)e * max_walls + i) * 2], c = wall_rc[((size_t)e * max_walls + i) * 2 + 1];
      if (placeable(r, c) && total - spent >= 1) {
        spent += 1;
        L.grid[r * C + c] = kWall;
        ++nw;
      }
    }
    const int cn = min(n_cams[e], p.max_cams);
    for (int i = 0; i < cn; ++i) {  // :124-135
      const double* cp = cam_params + ((size_t)e * p.max_cams + i) * 6;
      const int r = (int)cp[0], c = (int)cp[1];
      if (placeable(r, c) && total - spent >= 3) {
        spent += 3;
        Cam cm;
        cm.fov = cp[2]; cm.heading = cp[3]; cm.speed = cp[4];
        cm.row = (int16_t)r; cm.col = (int16_t)c; cm.range = (int16_t)cp[5];
        cm.num_rays = (int16_t)num_rays_for(cm.fov);
        p.cams[(size_t)e * p.max_cams + nc] = cm;
        L.grid[r * C + c] = kCamera;
        ++nc;
      }
    }
    const int gn = min(n_guards[e], p.max_guards);
    for (int i = 0; i < gn; ++i) {  // :138-149 (no placement check)
      const int32_t* gm = guard_meta + ((size_t)e * p.max_guards + i) * 3;
      const int len = min(gm[0], p.max_path);
      if (len > 0 && total - spent >= 5) {
        spent += 5;
        const int32_t* src = guard_paths + ((size_t)e * p.max_guards + i) * p.max_path * 2;
        uint16_t* dst = p.paths + ((size_t)e * p.max_guards + ng) * p.max_path;
        for (int k = 0; k < len; ++k) {  // points outside the grid are clamped onto it
          const int pr = min(max(src[2 * k], 0), R - 1), pc = min(max(src[2 * k + 1], 0), C - 1);
          dst[k] = (uint16_t)(pr | (pc << 8));
        }
        Guard gd;
        gd.fov = guard_fov[(size_t)e * p.max_guards + i];
        gd.heading = 0.0;
        gd.idx = 0;
        gd.speed = gm[1];
        gd.len = (int16_t)len;
        gd.range = (int16_t)gm[2];
        gd.num_rays = (int16_t)num_rays_for(gd.fov);
        gd.pad = 0;
        p.guards[(size_t)e * p.max_guards + ng] = gd;
        L.grid[(dst[0] & 0xff) * C + (dst[0] >> 8)] = kGuard;
        ++ng;
      }
    }
    L.meta[0] = nw; L.meta[1] = nc; L.meta[2] = ng; L.meta[3] = spent;
  }
  __syncthreads();
  const bool ok = bfs_wave(row_pass_mask(L.grid, R, C), p.sr, p.sc, p.vr, p.vc);
  uint8_t* dst = p.grid + (size_t)e * p.RC;
  for (int i = lane; i < p.RC; i += 64) dst[i] = L.grid[i];
  if (lane == 0) {
    EnvScalars* s = p.scal + e;
    s->n_walls = L.meta[0];
    s->n_cams = L.meta[1];
    s->n_guards = L.meta[2];
    s->spent = L.meta[3];
    valid_out[e] = ok ? 1 : 0;
  }
}

__global__ __launch_bounds__(64) void bfs_kernel(const int32_t* __restrict__ grid, int R, int C, int sr, int sc, int gr,
                                                  int gc, uint8_t* __restrict__ out) {
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const int32_t* g = grid + (size_t)e * R * C;
  uint64_t m = 0;
  if (lane < R)
    for (int c = 0; c < C; ++c)
      if (g[lane * C + c] != kWall) m |= 1ull << c;
  const bool ok = bfs_wave(m, sr, sc, gr, gc);
  if (lane == 0) out[e] = ok ? 1 : 0;
}

__global__ __launch_bounds__(64) void cones_kernel(int R, int C, const uint8_t* __restrict__ walls,
                                                    const int32_t* __restrict__ meta, const double* __restrict__ params,
                                                    uint8_t* __restrict__ out) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const int RC = R * C;
  const EnvLds L = carve(smem, RC, 1);
  for (int i = lane; i < RC; i += 64) {
    L.grid[i] = walls[(size_t)e * RC + i] ? kWall : kEmpty;
    L.vis[i] = 0;
  }
  if (lane == 0) {
    const int kind = meta[e * 4], row = meta[e * 4 + 1], col = meta[e * 4 + 2], range = meta[e * 4 + 3];
    const double fov = params[e * 2], heading = params[e * 2 + 1];
    Emit E;
    E.hmh = heading - fov / 2.0;
    E.fov = fov;
    E.row = row; E.col = col; E.range = range; E.num_rays = num_rays_for(fov);
    E.first = 0; E.kind = kind;
    L.em[0] = E;
    L.meta[0] = 1;
    L.meta[1] = E.num_rays + 1;
  }
  __syncthreads();
  cast_rays(L, R, C);
  __syncthreads();
  for (int i = lane; i < RC; i += 64) out[(size_t)e * RC + i] = L.vis[i];
}

__global__ void init_kernel(EnvParams p) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.n_envs) return;
  EnvScalars s;
  s.pos_r = p.sr; s.pos_c = p.sc; s.tick = 0; s.done = 0; s.detected = 0; s.vault_reached = 0;
  s.prev_dist = s.initial_dist = iabs_(p.sr - p.vr) + iabs_(p.sc - p.vc);
  s.n_cams = 0; s.n_guards = 0; s.n_walls = 0; s.spent = 0;
  p.scal[e] = s;
  uint8_t* g = p.grid + (size_t)e * p.RC;
  for (int i = 0; i < p.RC; ++i) {
    const int r = i / p.C, c = i % p.C;
    g[i] = (r == 0 || r == p.R - 1 || c == 0 || c == p.C - 1) ? kWall : kEmpty;
  }
  g[p.sr * p.C + p.sc] = kStart;
  g[p.vr * p.C + p.vc] = kVault;
}

__global__ void export_kernel(EnvParams p, int32_t* scalars, int8_t* grid, double* cam_heading, int32_t* guard_idx,
                              double* guard_heading) {
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const EnvScalars s = p.scal[e];
  if (scalars && lane == 0) {
    const int32_t v[12] = {s.pos_r, s.pos_c, s.tick, s.done, s.detected, s.vault_reached,
                           s.prev_dist, s.initial_dist, s.n_cams, s.n_guards, s.n_walls, s.spent};
    for (int k = 0; k < 12; ++k) scalars[(size_t)e * 12 + k] = v[k];
  }
  if (grid)
    for (int i = lane; i < p.RC; i += blockDim.x) grid[(size_t)e * p.RC + i] = (int8_t)p.grid[(size_t)e * p.RC + i];
  if (cam_heading && lane < p.max_cams)
    cam_heading[(size_t)e * p.max_cams + lane] = lane < s.n_cams ? p.cams[(size_t)e * p.max_cams + lane].heading : 0.0;
  if (lane < p.max_guards) {
    const bool live = lane < s.n_guards;
    const Guard gd = p.guards[(size_t)e * p.max_guards + lane];
    if (guard_idx) guard_idx[(size_t)e * p.max_guards + lane] = live ? gd.idx : 0;
    if (guard_heading) guard_heading[(size_t)e * p.max_guards + lane] = live ? gd.heading : 0.0;
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------

hipError_t launch_init(const EnvParams& p, hipStream_t st) {
  hipLaunchKernelGGL(init_kernel, dim3((p.n_envs + 255) / 256), dim3(256), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_set_layout(const EnvParams& p, int max_walls, const int32_t* wall_rc, const int32_t* n_walls,
                             const double* cam_params, const int32_t* n_cams, const int32_t* guard_paths,
                             const int32_t* guard_meta, const double* guard_fov, const int32_t* n_guards,
                             const int32_t* budget, uint8_t* valid_out, hipStream_t st) {
  const size_t lds = env_lds_bytes(p.RC, p.max_cams + p.max_guards);
  hipLaunchKernelGGL(set_layout_kernel, dim3(p.n_envs), dim3(64), lds, st, p, max_walls, wall_rc, n_walls, cam_params,
                     n_cams, guard_paths, guard_meta, guard_fov, n_guards, budget, valid_out);
  return hipGetLastError();
}

hipError_t launch_reset(const EnvParams& p, const uint8_t* mask, float* obs, hipStream_t st) {
  const size_t lds = env_lds_bytes(p.RC, p.max_cams + p.max_guards);
  hipLaunchKernelGGL(reset_kernel, dim3(p.n_envs), dim3(64), lds, st, p, mask, obs);
  return hipGetLastError();
}

hipError_t launch_step(const EnvParams& p, const int64_t* actions, float* obs, float* rew, double* rew64,
                       uint8_t* done_out, int8_t* status_out, int auto_reset, hipStream_t st) {
  const size_t lds = env_lds_bytes(p.RC, p.max_cams + p.max_guards);
  hipLaunchKernelGGL(step_kernel, dim3(p.n_envs), dim3(64), lds, st, p, actions, obs, rew, rew64, done_out, status_out,
                     auto_reset);
  return hipGetLastError();
}

hipError_t launch_export(const EnvParams& p, int32_t* scalars, int8_t* grid, double* cam_heading, int32_t* guard_idx,
                         double* guard_heading, hipStream_t st) {
  hipLaunchKernelGGL(export_kernel, dim3(p.n_envs), dim3(64), 0, st, p, scalars, grid, cam_heading, guard_idx,
                     guard_heading);
  return hipGetLastError();
}

hipError_t launch_bfs(const int32_t* grid, int n, int R, int C, int sr, int sc, int gr, int gc, uint8_t* out,
                      hipStream_t st) {
  hipLaunchKernelGGL(bfs_kernel, dim3(n), dim3(64), 0, st, grid, R, C, sr, sc, gr, gc, out);
  return hipGetLastError();
}

hipError_t launch_cones(int n, int R, int C, const uint8_t* walls, const int32_t* meta, const double* params,
                        uint8_t* out, hipStream_t st) {
  const size_t lds = env_lds_bytes(R * C, 1);
  hipLaunchKernelGGL(cones_kernel, dim3(n), dim3(64), lds, st, R, C, walls, meta, params, out);
  return hipGetLastError();
}

}  // namespace heist
