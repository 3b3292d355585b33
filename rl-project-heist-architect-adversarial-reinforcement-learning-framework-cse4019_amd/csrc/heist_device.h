// heist_device.h -- device-side data layout of the batched Heist environment.
//
// HBM layout (all [env]-major, one env is handled by one 64-lane wavefront):
//   EnvScalars [N]                 48 B  solver state + layout counters
//   grid       [N][R*C]            u8    tile types (utils.py:31-37), static per layout
//   stop       [N][stop_bytes]     u8    the raycast's padded stop map, 1 bit per cell (1 = wall or outside),
//                                        static per layout, expanded into LDS by step/reset
//   Cam        [N][max_cams]       32 B  fov, heading, speed (f64), row, col, range, num_rays
//   Guard      [N][max_guards]     32 B  fov, heading (f64), idx, speed, len, range, num_rays
//   paths      [N][max_guards][max_path] u16 (row | col << 8)
//   cones      [N][max_guards][kConePath][kConeSlots] 64 B  each guard's vision cone at
//              every (patrol index, heading slot), built once per layout (guard_cone_kernel)
// Per-handle constant tables: guard heading by (dr, dc) (host libm atan2), the two
// static position-channel planes, the tile->float LUT.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace heist {

enum : int { kEmpty = 0, kWall = 1, kStart = 2, kVault = 3, kCamera = 4, kGuard = 5 };
enum : int { kRunning = 0, kDetected = 1, kVaultReached = 2, kTimeout = 3, kAlreadyDone = 4 };

constexpr int kMaxDim = 64;          // R, C <= 64
constexpr int kMaxEmitters = 64;     // max_cams + max_guards per env
constexpr double kDegToRad = 3.141592653589793 / 180.0;  // CPython math.radians factor
constexpr int kHalfDegN = 2880;      // half-degree sin/cos table: angles -720 .. 719.5

// Guard cone cache (guard_cone_kernel): a guard's visible tiles depend only on its patrol
// index and its heading, and the heading is either the initial one or the direction of
// the move that led to a patrol point (security.py:145-159), so a layout's guard has at
// most len x (len + 1) cones.  Guards with a patrol of at most kConePath points, at most
// kConeSlots distinct headings and a vision range of at most kConeRange get every cone
// precomputed at set_layout; the tick ORs a 32-byte window instead of casting 181 rays.
// Cone entry (64 B, kConeEntry u16): 16 rows of u16, rows 0..14 = tiles (dr, dc) in
// [-7, 7]^2 around the guard (bit dc + 7 of row dr + 7, the guard's own tile included), row
// 15 = the heading slot after the next move from this state; then the pose the entry
// describes, so a tick that moves a cached guard reads its new pose with its cone in one
// load: u16 16..19 = the slot's heading (fp64 bits), u16 20 = the patrol point (r | c << 8).
constexpr int kConeEntry = 32;
constexpr int kConePath = 16;
constexpr int kConeSlots = 8;
constexpr int kConeRange = 7;
constexpr uint8_t kUncached = 0xFF;

struct EnvScalars {
  int32_t pos_r, pos_c, tick, done;
  int32_t detected, vault_reached, prev_dist, initial_dist;
  int32_t n_cams, n_guards, n_walls, spent;
};
static_assert(sizeof(EnvScalars) == 48, "EnvScalars layout");

struct Cam {
  double fov, heading, speed;
  int16_t row, col, range, num_rays;
};
static_assert(sizeof(Cam) == 32, "Cam layout");

struct Guard {
  double fov, heading;
  int16_t idx;       // current_idx
  int16_t step;      // speed mod len (Python %), so idx' = (idx + step) % len
  int16_t len, range, num_rays;
  uint16_t pos;      // patrol_path[idx] packed row | col << 8
  uint16_t pos0;     // patrol_path[0]
  uint8_t hslot;     // heading slot of `heading` in the guard's cone table; kUncached: raycast live
  uint8_t nslot;     // heading slot after the next patrol move (the cone the next tick reads)
};
static_assert(sizeof(Guard) == 32, "Guard layout");

__host__ __device__ inline int pack_rc(int r, int c) { return r | (c << 8); }

// One ray emitter as the raycaster sees it (a camera or a guard at its current pose).
struct Emit {
  double hmh;     // heading - fov / 2.0  (security.py:64, :70)
  double fov;
  double step;    // fov / num_rays: the fast path's ray spacing (approximate angle)
  int32_t row, col, range, num_rays;
  int32_t first;  // index of this emitter's first 64-ray chunk in the env's chunk list
  int32_t kind;   // 0 camera (half-tile sub-steps), 1 guard (whole-tile steps), 2 guard with a cached cone (no rays)
  int32_t members;  // direction group (publish_emitters): a leader's count of consecutive slots sharing its
                    // ray directions (itself included); 0 for the other members (no chunks of their own)
  int32_t pad_;
};
static_assert(sizeof(Emit) == 56, "Emit layout");

// The K-tick kernel's shared camera fan (fan_kernel, heist_env.hip): for tick k of a
// launch, the fast-path fan of the source camera (the first env's first camera) as that tick casts it -- the emitter
// (heading - fov / 2, fov, rays, range) and, computed once for the whole batch, its rays'
// unique fp32 directions (one per dedup key) and its near-tie rays.  A direction group
// whose emitter equals the tick's entry bit for bit takes its rays from the table instead
// of computing them (an Architect batch's cameras share one fan, and their headings advance
// in lockstep); any other group computes its own.  n_uniq < 0: no table for the tick.
// The table covers kFanTicks ticks from the launch that fills it and serves the following
// launches at their offset (fan_base) until it runs out or the handle's cameras change
// other than by K-tick launches (set_layout, reset, single ticks); an entry that no longer
// matches a group's emitter is simply not used, so staleness costs time, never results.
constexpr int kFanRays = 256;   // rays 0 .. num_rays with num_rays < kFanRays
constexpr int kFanTicks = 1024;  // the K-tick launch's K limit
struct FanTick {
  double hmh, fov;
  int num_rays, range, n_uniq, n_tie;
  double heading, speed;     // the source camera's heading at this tick (after its rotation) and speed
  float uniq[2 * kFanRays];  // (dxs, dys) of the unique directions
  uint16_t tie[kFanRays];    // ray indices of the near-tie rays (exact path)
  // The unique directions' sample tiles for the lean K-tick kernel: direction j's sample k
  // (k = 1 .. 12, dist k / 2) lands on tile (row + dr, col + dc) with dc = rint(k * dxs), dr =
  // rint(k * dys) -- exactly the fast path's march, which rounds col + k * dxs once and, the
  // direction screened off every .5 tie, equals col + rint(k * dxs) -- stored as the index of
  // that tile in the padded plane counted from the tile (row - kRing, col - kRing):
  // (dr + kRing) * (C + 2 kRing) + dc + kRing, u16 pairs, samples 1-8 in off4, 9-12 in off2.
  uint4 off4[kFanRays];
  uint2 off2[kFanRays];
};

struct EnvParams {
  int R, C, RC, max_steps;
  int sr, sc, vr, vc;
  double r_step, r_detect, r_vault;
  int n_envs, max_cams, max_guards, max_path;
  EnvScalars* scal;
  uint8_t* grid;
  uint8_t* stop;              // [n_envs][stop_bytes] padded stop maps (set_layout_kernel)
  int stop_bytes;             // per env: (R + 2*kRing)(C + 2*kRing) / 8 rounded up to 16 (bit-packed)
  Cam* cams;
  Guard* guards;
  uint16_t* paths;
  uint16_t* cones;            // [n_envs][max_guards][kConePath][kConeSlots][kConeEntry] guard cone cache
  int guard_cones;            // 1: heist_set_layout builds the cone cache (default); 0: guards raycast live
  const double* heading_tab;  // [(2R-1)*(2C-1)]
  const float* plane0;        // [RC] position channel without the solver
  const float* plane1;        // [RC] position channel value if the solver is on that cell
  float vault_val;            // position channel value on the vault cell
  float tile_lut[8];          // float32(tile) / 5  (environment.py:319)
  double axis_heading[4];     // heading_tab at (dr,dc) = (-1,0), (1,0), (0,-1), (0,1)
  int step_waves;             // wavefronts per env in step/reset (1, 2 or 4)
  int multi_waves;            // wavefronts per env in the K-tick kernel (heist_step_multi; HEIST_MULTI_WAVES)
  int multi_occ;              // min waves per SIMD it is compiled for (8 at 2 or 4 waves, 4 at 1: 128 VGPRs)
  int ray_chunk;              // samples per ray computed together (2, 4)
  int step_occ;               // min waves per SIMD the step kernel is compiled for (1, 8)
  int vis_gap;                // LDS distance stop map -> vis plane (1024, 2048 or 6144), see heist_env.hip
  unsigned long long* sample_counter;  // optional [n_envs]: ray samples evaluated per env, else null
  unsigned long long* redo_counter;    // optional [n_envs]: rays re-cast on the exact fp64 path, else null
  const double* half_deg;      // [2][kHalfDegN] glibc-exact sin, cos of m/2 degrees (m = -1440 .. 1439)
  int32_t* order;              // [n_envs] env of step/reset block b: heaviest raycast first (order_kernel)
  int split_obs;               // 1 (default): step writes obs channels 0/2 before the raycast (HEIST_SPLIT_OBS)
  int dispatch_order;          // 1 (default): step/reset block b runs env order[b] (heaviest first); 2 (opt-in,
                               // HEIST_DISPATCH_ORDER=2, measured and not kept): the same ranks snake-drafted over
                               // the SIMDs (order_kernel); 0: env b
  int n_cu;                    // compute units of the device (the snake draft's SIMD count / 4)
  int prio_mode;               // K-tick lean kernel wave priority by cost rank (order_kernel; HEIST_PRIO_MODE)
  int lean_waves;              // 32 x 32 lean kernel waves per env: 0 auto (2 when they fit the chip), 1, 2
                               // (HEIST_LEAN_WAVES)
  unsigned long long* stamps;          // optional [n_envs][waves][8]: step-kernel phase stamps (s_memtime), else null
  int obs_store;              // observation stores: 0 plain, 1 write-through (sc1), 2 nt, 3 sc1 nt (HEIST_OBS_STORE)
  int ray_mode;               // 0: fp32 fast path with exact fp64 re-cast of near-tie rays; 1: exact fp64 only
  FanTick* fan;               // [kFanTicks] shared camera fan of the current K-tick launch (fan_kernel)
  int fan_on;                 // 1 (default): the K-tick kernel uses the shared fan (HEIST_SHARED_FAN)
  int lean;                   // 1 (default): one-wave 20 x 20 K-tick launches run step_lean_kernel (HEIST_LEAN)
  int interval_fans;          // 1 (default): step_lean_kernel casts cameras the shared fan does not serve from
                              // the ray-direction interval table (heist_fan_intervals.h; HEIST_INTERVAL_FANS)
  int fan_base;               // table entry of the launch's tick 0 (heist_step_multi)
  int fan_fill;               // 1: the launch first refills the table from the cameras' current headings
  int probe_mode;             // profiling only (HEIST_PROBE_MODE): 0 normal, 1 no rays, 2 angles+sin/cos only,
                              // 3 marches with a fixed direction (no sin/cos), 4 no observation write,
                              // 5 neither rays nor observation, 6 return at entry, 7 return after the
                              // raycast; results are wrong for 1-7
};

// security.py:67 max(int(fov * 2), 30); capped at 32000 rays (fov 16000 deg) so the
// count fits the int16 fields and a bad fov cannot blow up a launch.
__host__ __device__ inline int num_rays_for(double fov) {
  if (!(fov * 2 < 32000.0)) return 32000;
  int n = (int)(fov * 2);
  return n > 30 ? n : 30;
}

}  // namespace heist
