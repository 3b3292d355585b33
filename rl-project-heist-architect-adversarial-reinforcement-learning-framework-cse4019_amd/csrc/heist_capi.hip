// heist_capi.hip -- extern "C" entry points of libheist_hip.so (declared in include/heist.h).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "heist.h"
#include "heist_device.h"

#pragma clang fp contract(off)

namespace heist {
hipError_t launch_init(const EnvParams& p, hipStream_t st);
hipError_t launch_order(const EnvParams& p, hipStream_t st);
hipError_t launch_guard_cones(const EnvParams& p, const uint8_t* mask, hipStream_t st);
hipError_t launch_set_layout(const EnvParams& p, int max_walls, const int32_t* wall_rc, const int32_t* n_walls,
                             const double* cam_params, const int32_t* n_cams, const int32_t* guard_paths,
                             const int32_t* guard_meta, const double* guard_fov, const int32_t* n_guards,
                             const int32_t* budget, const uint8_t* mask, uint8_t* valid_out, hipStream_t st);
hipError_t launch_reset(const EnvParams& p, const uint8_t* mask, float* obs, hipStream_t st);
hipError_t launch_step(const EnvParams& p, const int64_t* actions, float* obs, float* rew, double* rew64,
                       uint8_t* done_out, int8_t* status_out, int auto_reset, hipStream_t st);
hipError_t launch_step_multi(const EnvParams& p, int K, const int64_t* actions, float* obs,
                             float* rew, double* rew64, uint8_t* done_out, int8_t* status_out, int auto_reset,
                             hipStream_t st);
hipError_t launch_export(const EnvParams& p, int32_t* scalars, int8_t* grid, double* cam_heading, int32_t* guard_idx,
                         double* guard_heading, hipStream_t st);
hipError_t launch_bfs(const int32_t* grid, int n, int R, int C, int sr, int sc, int gr, int gc, uint8_t* out,
                      hipStream_t st);
int vis_gap_for(int R, int C);
int stop_map_bytes(int R, int C);
bool env_variant_exists(int W, int U, int O, int D);
bool multi_variant_exists(int W, int U, int O, int D);
bool lean_two_waves(const EnvParams& p);
hipError_t launch_cone_order(int n, int R, int C, const uint8_t* walls, const int32_t* meta, const double* params,
                             uint32_t* keys_out, hipStream_t st);
hipError_t launch_cones(int n, int R, int C, const uint8_t* walls, const int32_t* meta, const double* params,
                        uint8_t* out, int ray_mode, hipStream_t st);
hipError_t launch_fast_dir(const double* deg, int64_t n, float* co, float* so, hipStream_t st);
hipError_t launch_arch_decode(const int64_t* amap, int n, int R, int C, const float* cam, int cam_stride,
                              const int32_t* budget, int allow_cams, int allow_guards, int max_walls, int max_cams,
                              int max_guards, int max_path, int32_t* wall_rc, int32_t* n_walls, double* cam_out,
                              int32_t* n_cams, int32_t* guard_paths, int32_t* guard_meta, double* guard_fov,
                              int32_t* n_guards, hipStream_t st);
hipError_t launch_sincos(const double* x, int64_t n, double* so, double* co, hipStream_t st);
int solver_packed_bytes();
bool solver_conv_supported(int R, int C);
hipError_t launch_solver_pack(const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                              const float* b3, void* packed, hipStream_t st);
hipError_t launch_solver_conv(const float* obs, int n, int R, int C, const void* packed, float* feat, int n_cu,
                              hipStream_t st);
int solver_head_packed_bytes();
void set_solver_stamps(unsigned long long* p);
hipError_t launch_solver_head_pack(const float* const* w, int A, void* packed, hipStream_t st);
hipError_t launch_solver_head(const float* feat, const float* h_in, const float* c_in, int n, const void* packed,
                              int A, uint64_t seed, uint64_t counter, float* logits_out, float* value_out,
                              int64_t* action_out, float* logp_out, float* h_out, float* c_out, hipStream_t st);
hipError_t launch_bias_relu(float* x, const float* b, int64_t n_pos, int C, hipStream_t st);
hipError_t launch_bias_relu_pool(float* x, const float* b, int n, int R, int W, int C, float* feat, hipStream_t st);
hipError_t launch_pool_relu_bwd(const float* dfeat, const float* y, int n, int R, int W, int C, float* d, float* part,
                                float* db, hipStream_t st);
hipError_t launch_relu_bwd(float* g, const float* y, int n, int P, int C, float* part, float* db, hipStream_t st);
bool arch_update_supported(int R, int C);
void set_arch_stamps(unsigned long long* p);
int64_t arch_update_workspace_bytes();
hipError_t launch_arch_update(float* const* p, float* const* m, float* const* v, const float* grid, int R, int C,
                              const float* target, int k, const float* adam_sc, float* vloss, void* ws, double beta1,
                              double beta2, double eps, double max_norm, double value_coeff, hipStream_t st);
int train_conv_frag_floats(int layer, int mode);
int64_t train_conv_partial_floats(int layer, int n, int R, int C);
hipError_t launch_train_conv_pack(int layer, int mode, const float* w, float* frag, hipStream_t st);
hipError_t launch_train_conv(int layer, int mode, const float* x, int n, int R, int C, const float* frag,
                             const float* bias, uint8_t* mask_bits, float* y, int* queue, hipStream_t st);
hipError_t launch_train_conv_wgrad(int layer, const float* dy, const float* x, int n, int R, int C, float* partial,
                                   float* dw, float* db, int* queue, hipStream_t st);
hipError_t launch_obs_nhwc4(const float* obs, int n, int R, int C, const int64_t* strides, float* x4, hipStream_t st);
hipError_t launch_train_pool(const float* a3, int n, int R, int C, float* feat, hipStream_t st);
hipError_t launch_train_pool_bwd(const float* dfeat, const uint8_t* m3, int n, int R, int C, float* d3, hipStream_t st);
hipError_t launch_gae(const float* r, const float* v, const uint8_t* d, const float* last_value, int T, int N,
                      double gamma, double lam, float* adv, float* ret, hipStream_t st);
hipError_t launch_rollout_tally(const uint8_t* valid, int32_t* attempts, int A, const uint8_t* done, const int8_t* status,
                                const double* reward64, int32_t* steps, double* reward_sum, int32_t* solve,
                                int32_t* detect, int32_t* timeout, float* h, float* c, int hidden, int n, int vault,
                                int det, hipStream_t st);
hipError_t launch_lstm_cell(const float* gx, const float* gh, const float* c, float* h1, float* c1, int H, int n,
                            hipStream_t st);
hipError_t launch_adv_moments(const float* x, int64_t n, int phase, double* acc, hipStream_t st);
hipError_t launch_adv_apply(float* x, int64_t n, const double* acc, float eps, hipStream_t st);
hipError_t launch_ppo_loss(const float* logits, const float* values, const int64_t* actions, const float* old_logp,
                           const float* adv, const float* ret, int M, int A, double clip, double vcoef, double ecoef,
                           float* parts, float* dlogits, float* dvalues, double* scratch, hipStream_t st);
}  // namespace heist

using heist::EnvParams;

struct heist_env {
  int device;
  EnvParams p;
  void* allocs[12];
  int n_allocs;
  int fan_pos;             // next entry of the shared fan table (FanTick) for a K-tick launch; -1: refill first
  hipStream_t fan_stream;  // stream of the K-tick launch that last used the table (a refill on another stream
                           // could overwrite entries a launch still in flight on this one reads)
  bool fan_used;           // a K-tick launch has been issued on fan_stream
  hipEvent_t fan_done;     // recorded behind every K-tick launch: a refill on another stream waits for it
  int64_t stamp_words;     // size of the stamp buffer armed by heist_step_stamps (uint64 words)
  int step_lean;           // 1 (HEIST_STEP_LEAN=1): heist_step runs as a one-tick heist_step_multi launch wherever
                           // the lean K-tick kernel serves the handle; 0 (default): the single-tick step kernel
                           // (C2, 4096 envs: 15.1 us per tick against 18.9 for the one-tick lean launch, whose
                           // per-launch prologue costs ~12 us: tools/probe_single_tick.py, gpurun_out r06b)
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int check_hip(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  return fail((int)e, std::string(what) + ": " + hipGetErrorString(e));
}

#define HEIST_REQUIRE(cond, msg) \
  do {                           \
    if (!(cond)) return fail(HEIST_EINVAL, msg); \
  } while (0)

int check_handle(heist_t h) {
  HEIST_REQUIRE(h != nullptr, "null heist_t handle");
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != h->device)
    return fail(HEIST_EINVAL, "heist_t used on device " + std::to_string(dev) + " but created on device " +
                                  std::to_string(h->device));
  return 0;
}

double py_mod(double x, double m) {  // Python float %
  double r = std::fmod(x, m);
  if (r != 0.0) {
    if ((m < 0) != (r < 0)) r += m;
  } else {
    r = std::copysign(0.0, m);
  }
  return r;
}

// Guard heading after a move by (dr, dc): math.degrees(math.atan2(-dr, dc)) % 360.0
// (security.py:159), evaluated with the host libm exactly as CPython does.
std::vector<double> heading_table(int R, int C) {
  const double rad_to_deg = 180.0 / 3.141592653589793;  // CPython math.degrees factor
  std::vector<double> t((size_t)(2 * R - 1) * (2 * C - 1), 0.0);
  for (int dr = -(R - 1); dr <= R - 1; ++dr)
    for (int dc = -(C - 1); dc <= C - 1; ++dc) {
      if (dr == 0 && dc == 0) continue;
      const double y = (double)(-dr), x = (double)dc;
      double a;
      if (y == 0.0) a = std::copysign(1.0, x) == 1.0 ? std::copysign(0.0, y) : std::copysign(3.141592653589793, y);
      else a = std::atan2(y, x);  // CPython m_atan2 for finite, nonzero y
      t[(size_t)(dr + R - 1) * (2 * C - 1) + (dc + C - 1)] = py_mod(a * rad_to_deg, 360.0);
    }
  return t;
}

// heist_step's one-tick heist_step_multi route applies: the lean kernel (step_lean_kernel) takes
// the launch (launch_step_multi's lean20 / lean32 test) and no instrumentation is armed (the
// step kernel's stamp and counter layouts differ from the K-tick kernel's)
bool lean_serves(const heist_env* h) {
  const EnvParams& p = h->p;
  const bool lean20 = p.multi_waves == 1 && p.R == 20 && p.C == 20 && p.vis_gap == 1024;
  const bool lean32 = p.R == 32 && p.C == 32 && p.vis_gap == 2048;
  return h->step_lean && p.lean && (lean20 || lean32) && p.probe_mode == 0 && !p.sample_counter &&
         !p.redo_counter && !p.stamps && p.max_cams + p.max_guards <= heist::kMaxEmitters;
}

}  // namespace

extern "C" {

int heist_abi_version(void) { return HEIST_ABI_VERSION; }

const char* heist_last_error(void) { return g_err.c_str(); }

int heist_create(int R, int C, int max_steps, int sr, int sc, int vr, int vc, const double* reward_consts, int n_envs,
                 int max_cams, int max_guards, int max_path, heist_t* out) {
  HEIST_REQUIRE(out != nullptr, "heist_create: out is null");
  *out = nullptr;
  HEIST_REQUIRE(R >= 3 && C >= 3 && R <= heist::kMaxDim && C <= heist::kMaxDim, "heist_create: need 3 <= rows, cols <= 64");
  HEIST_REQUIRE(sr >= 0 && sr < R && sc >= 0 && sc < C && vr >= 0 && vr < R && vc >= 0 && vc < C,
                "heist_create: start/vault outside the grid");
  HEIST_REQUIRE(n_envs >= 1, "heist_create: n_envs must be >= 1");
  // order[] packs the env index in 24 bits (a wave priority above it, order_kernel)
  HEIST_REQUIRE(n_envs <= (1 << 24), "heist_create: n_envs must be <= 16777216");
  HEIST_REQUIRE(max_cams >= 0 && max_guards >= 0 && max_cams + max_guards <= heist::kMaxEmitters,
                "heist_create: need max_cams + max_guards <= 64");
  HEIST_REQUIRE(max_path >= 1 && max_path <= 4096, "heist_create: need 1 <= max_path <= 4096");
  HEIST_REQUIRE(max_steps >= 1, "heist_create: max_steps must be >= 1");
  HEIST_REQUIRE(reward_consts != nullptr, "heist_create: reward_consts is null");

  heist_env* h = new heist_env();
  if (hipGetDevice(&h->device) != hipSuccess) {
    delete h;
    return fail(HEIST_EINVAL, "heist_create: no HIP device");
  }
  EnvParams& p = h->p;
  p.R = R; p.C = C; p.RC = R * C; p.max_steps = max_steps;
  p.sr = sr; p.sc = sc; p.vr = vr; p.vc = vc;
  p.r_step = reward_consts[0]; p.r_detect = reward_consts[1]; p.r_vault = reward_consts[2];
  p.n_envs = n_envs; p.max_cams = max_cams; p.max_guards = max_guards; p.max_path = max_path;

  const size_t n = (size_t)n_envs;
  const std::vector<double> htab = heading_table(R, C);
  std::vector<float> planes((size_t)2 * R * C);
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < C; ++c) {  // environment.py:356-365 with NumPy-2 float32 adds
      const int d = std::abs(r - vr) + std::abs(c - vc);
      const float g = (float)(-0.3 * ((double)d / (double)(R + C)));
      planes[(size_t)r * C + c] = 0.0f + g;
      planes[(size_t)R * C + (size_t)r * C + c] = 1.0f + g;
    }
  p.vault_val = -1.0f + (float)(-0.3 * (0.0 / (double)(R + C)));
  {  // axis-aligned guard moves: heading depends only on the direction
    const int W2 = 2 * C - 1;
    p.axis_heading[0] = htab[(size_t)(-1 + R - 1) * W2 + (C - 1)];
    p.axis_heading[1] = htab[(size_t)(1 + R - 1) * W2 + (C - 1)];
    p.axis_heading[2] = htab[(size_t)(R - 1) * W2 + (-1 + C - 1)];
    p.axis_heading[3] = htab[(size_t)(R - 1) * W2 + (1 + C - 1)];
  }
  // 2 waves per env: 16 blocks resident per CU (LDS ~5 KB each) and half the redundant
  // block-uniform work of 4 waves; 23.0 us per 4096-env step vs 26.8 at 4 waves and 24.1
  // at 1 (C2 Architect layouts with the guard cone cache, gpurun_out r02j).  A batch too
  // small to give every SIMD 8 waves at 2 per env takes 4 per env instead (BASELINE C5:
  // 2048 envs of 32 x 32, 22.7 -> 21.0 us per step; C4's 8192 envs: 2 waves, 44.5 vs
  // 52.1 us; profiles/r02ae_configs.log)
  int n_cu = 0;
  {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n_cu = 256;
    p.step_waves = 2 * (size_t)n_envs < 32 * (size_t)n_cu ? 4 : 2;
  }
  p.ray_chunk = 4;  // tuning knobs; a combination without a compiled variant falls back to (2, 4, 8)
  // 8 waves per SIMD (64 VGPRs): 4096 envs are two full rounds of 8 workgroups per CU
  // (41.4 us per step vs 46.6 at the unbounded 85 VGPRs / 5 waves, profiles/r01m_*)
  p.step_occ = 8;
  if (const char* u = getenv("HEIST_RAY_CHUNK")) p.ray_chunk = atoi(u);
  if (const char* o = getenv("HEIST_STEP_OCC")) p.step_occ = atoi(o);
  if (const char* w = getenv("HEIST_STEP_WAVES")) p.step_waves = atoi(w);
  p.probe_mode = 0;
  if (const char* m = getenv("HEIST_PROBE_MODE")) p.probe_mode = atoi(m);
  p.obs_store = 2;  // nt: 15.4 vs 16.7 us per 4096-env step plain, 16.2 sc1 (profiles/r02ba_probe_obs_store.log)
  if (const char* m = getenv("HEIST_OBS_STORE")) p.obs_store = atoi(m) & 3;
  p.ray_mode = 0;
  if (const char* m = getenv("HEIST_EXACT_RAYS")) p.ray_mode = atoi(m) ? 1 : 0;
  p.sample_counter = nullptr;
  p.redo_counter = nullptr;
  p.stamps = nullptr;
  p.vis_gap = heist::vis_gap_for(R, C);
  if (!heist::env_variant_exists(p.step_waves, p.ray_chunk, p.step_occ, p.vis_gap)) {
    p.step_waves = 2;
    p.ray_chunk = 4;
    p.step_occ = 8;
    p.vis_gap = heist::vis_gap_for(R, C);
  }
  // K-tick kernel: one wave per env (every role in one wave, 96 VGPRs, 5 waves per SIMD, no
  // spills) once the batch gives every SIMD 4 of them -- 4096 envs: 11.9 us per tick vs 13.1
  // at 2 waves per env (8 per SIMD, 64 VGPRs + 52 spilled), profiles/r03d_bench_w*.log --
  // else the step kernel's waves per env; HEIST_MULTI_WAVES overrides
  p.multi_waves = (size_t)n_envs >= 16 * (size_t)n_cu ? 1 : p.step_waves;
  if (const char* m = getenv("HEIST_MULTI_WAVES")) p.multi_waves = atoi(m);
  p.multi_occ = p.multi_waves == 1 ? 4 : 8;
  if (const char* m = getenv("HEIST_MULTI_OCC")) p.multi_occ = atoi(m);  // A/B: waves per SIMD it is built for
  if (!heist::multi_variant_exists(p.multi_waves, p.ray_chunk, p.multi_occ, p.vis_gap)) {
    p.multi_waves = p.step_waves;
    p.multi_occ = 8;
  }
  // Heaviest-raycast-first dispatch (order_kernel) also pays when the whole grid is
  // resident at once: it deals every CU one env of each cost stratum.  Block b = env b
  // (HEIST_DISPATCH_ORDER=0, no order[] load) measured 16.29 vs 15.37 us per 4096-env step
  // (profiles/r02bd_probe_dispatch_order.log).
  p.dispatch_order = 1;
  if (const char* m = getenv("HEIST_DISPATCH_ORDER")) p.dispatch_order = atoi(m) >= 2 ? 2 : (atoi(m) ? 1 : 0);
  p.n_cu = n_cu;
  p.prio_mode = 0;
  if (const char* m = getenv("HEIST_PRIO_MODE")) p.prio_mode = atoi(m) < 0 ? 0 : (atoi(m) > 3 ? 3 : atoi(m));
  p.lean_waves = 0;
  if (const char* m = getenv("HEIST_LEAN_WAVES")) p.lean_waves = atoi(m) == 1 ? 1 : (atoi(m) == 2 ? 2 : 0);
  p.split_obs = 1;
  if (const char* m = getenv("HEIST_SPLIT_OBS")) p.split_obs = atoi(m) ? 1 : 0;
  for (int k = 0; k < 8; ++k) p.tile_lut[k] = k <= 5 ? (float)k / 5.0f : 0.0f;  // environment.py:319

  const size_t sizes[] = {
      sizeof(heist::EnvScalars) * n,
      n * p.RC,
      sizeof(heist::Cam) * n * (max_cams > 0 ? max_cams : 1),
      sizeof(heist::Guard) * n * (max_guards > 0 ? max_guards : 1),
      sizeof(uint16_t) * n * (max_guards > 0 ? max_guards : 1) * max_path,
      sizeof(double) * htab.size(),
      sizeof(float) * planes.size(),
      sizeof(int32_t) * n,
      sizeof(double) * 3 * heist::kHalfDegN,  // [sin | cos | staging radians]
      (size_t)heist::stop_map_bytes(R, C) * n,
      // guard cone cache: 64 B per (guard, patrol index, heading slot)
      sizeof(uint16_t) * heist::kConeEntry * n * (max_guards > 0 ? max_guards : 1) * heist::kConePath * heist::kConeSlots,
      sizeof(heist::FanTick) * heist::kFanTicks,
  };
  static_assert(sizeof(sizes) / sizeof(sizes[0]) <= sizeof(((heist_env*)nullptr)->allocs) / sizeof(void*),
                "heist_env::allocs too small");
  h->n_allocs = 0;
  for (size_t k = 0; k < sizeof(sizes) / sizeof(sizes[0]); ++k) {
    void* ptr = nullptr;
    hipError_t e = hipMalloc(&ptr, sizes[k]);
    if (e != hipSuccess) {
      for (int j = 0; j < h->n_allocs; ++j) (void)hipFree(h->allocs[j]);
      delete h;
      return check_hip(e, "heist_create: hipMalloc");
    }
    h->allocs[h->n_allocs++] = ptr;
  }
  p.scal = (heist::EnvScalars*)h->allocs[0];
  p.grid = (uint8_t*)h->allocs[1];
  p.cams = (heist::Cam*)h->allocs[2];
  p.guards = (heist::Guard*)h->allocs[3];
  p.paths = (uint16_t*)h->allocs[4];
  p.heading_tab = (const double*)h->allocs[5];
  p.plane0 = (const float*)h->allocs[6];
  p.plane1 = p.plane0 + (size_t)R * C;
  p.order = (int32_t*)h->allocs[7];
  p.half_deg = (const double*)h->allocs[8];
  p.stop = (uint8_t*)h->allocs[9];
  p.stop_bytes = heist::stop_map_bytes(R, C);
  p.cones = (uint16_t*)h->allocs[10];
  p.fan = (heist::FanTick*)h->allocs[11];
  h->fan_pos = -1;
  h->fan_stream = nullptr;
  h->fan_used = false;
  h->fan_done = nullptr;
  h->stamp_words = 0;
  p.fan_base = 0;
  p.fan_fill = 0;
  p.fan_on = 1;
  if (const char* f = getenv("HEIST_SHARED_FAN")) p.fan_on = atoi(f) ? 1 : 0;
  p.lean = 1;
  if (const char* f = getenv("HEIST_LEAN")) p.lean = atoi(f) ? 1 : 0;
  p.interval_fans = 1;
  if (const char* f = getenv("HEIST_INTERVAL_FANS")) p.interval_fans = atoi(f) ? 1 : 0;
  p.guard_cones = 1;
  if (const char* gc = getenv("HEIST_GUARD_CONES")) p.guard_cones = atoi(gc) ? 1 : 0;
  h->step_lean = 0;
  if (const char* f = getenv("HEIST_STEP_LEAN")) h->step_lean = atoi(f) ? 1 : 0;
  std::vector<double> hrad(heist::kHalfDegN);
  for (int m = 0; m < heist::kHalfDegN; ++m) hrad[m] = (0.5 * (m - heist::kHalfDegN / 2)) * heist::kDegToRad;

  int rc = check_hip(hipMemcpy(h->allocs[5], htab.data(), sizes[5], hipMemcpyHostToDevice), "heist_create: upload");
  if (!rc) rc = check_hip(hipMemcpy(h->allocs[6], planes.data(), sizes[6], hipMemcpyHostToDevice), "heist_create: upload");
  if (!rc) rc = check_hip(hipMemset(h->allocs[2], 0, sizes[2]), "heist_create: memset");
  // fan table: all 0xFF = NaN emitters and n_uniq = -1, an entry no group can match
  if (!rc) rc = check_hip(hipMemset(h->allocs[11], 0xFF, sizes[11]), "heist_create: memset");
  if (!rc) rc = check_hip(hipMemset(h->allocs[3], 0, sizes[3]), "heist_create: memset");
  if (!rc) rc = check_hip(hipMemset(h->allocs[4], 0, sizes[4]), "heist_create: memset");
  if (!rc) rc = check_hip(hipMemcpy((double*)h->allocs[8] + 2 * heist::kHalfDegN, hrad.data(),
                                    sizeof(double) * heist::kHalfDegN, hipMemcpyHostToDevice), "heist_create: upload");
  if (!rc) {
    double* hd = (double*)h->allocs[8];
    rc = check_hip(heist::launch_sincos(hd + 2 * heist::kHalfDegN, heist::kHalfDegN, hd, hd + heist::kHalfDegN, nullptr),
                   "heist_create: half-degree table");
  }
  if (!rc) rc = check_hip(heist::launch_init(p, nullptr), "heist_create: init");
  if (!rc) rc = check_hip(hipDeviceSynchronize(), "heist_create: init");
  if (rc) {
    heist_destroy(h);
    return rc;
  }
  *out = h;
  return 0;
}

int heist_destroy(heist_t h) {
  if (!h) return 0;
  if (h->fan_done) (void)hipEventDestroy(h->fan_done);
  for (int j = 0; j < h->n_allocs; ++j) (void)hipFree(h->allocs[j]);
  delete h;
  return 0;
}

int heist_set_layout(heist_t h, int max_walls, const int32_t* wall_rc, const int32_t* n_walls, const double* cam_params,
                     const int32_t* n_cams, const int32_t* guard_paths, const int32_t* guard_meta,
                     const double* guard_fov, const int32_t* n_guards, const int32_t* budget, const uint8_t* mask,
                     uint8_t* valid_out, heist_stream_t stream) {
  if (int rc = check_handle(h)) return rc;
  HEIST_REQUIRE(max_walls >= 0, "heist_set_layout: max_walls < 0");
  HEIST_REQUIRE(n_walls && n_cams && n_guards && budget && valid_out, "heist_set_layout: null counts/budget/valid_out");
  HEIST_REQUIRE(max_walls == 0 || wall_rc, "heist_set_layout: wall_rc is null");
  HEIST_REQUIRE(h->p.max_cams == 0 || cam_params, "heist_set_layout: cam_params is null");
  HEIST_REQUIRE(h->p.max_guards == 0 || (guard_paths && guard_meta && guard_fov), "heist_set_layout: guard arrays null");
  h->fan_pos = -1;  // new cameras: the shared fan table is refilled by the next K-tick launch
  if (int rc = check_hip(heist::launch_set_layout(h->p, max_walls, wall_rc, n_walls, cam_params, n_cams, guard_paths,
                                                   guard_meta, guard_fov, n_guards, budget, mask, valid_out,
                                                   (hipStream_t)stream),
                          "heist_set_layout"))
    return rc;
  if (int rc = check_hip(heist::launch_guard_cones(h->p, mask, (hipStream_t)stream), "heist_set_layout: guard cones"))
    return rc;
  return check_hip(heist::launch_order(h->p, (hipStream_t)stream), "heist_set_layout: order");
}

int heist_reset(heist_t h, const uint8_t* mask, float* obs_out, heist_stream_t stream) {
  if (int rc = check_handle(h)) return rc;
  HEIST_REQUIRE(obs_out != nullptr, "heist_reset: obs_out is null");
  h->fan_pos = -1;
  return check_hip(heist::launch_reset(h->p, mask, obs_out, (hipStream_t)stream), "heist_reset");
}

int heist_step(heist_t h, const int64_t* actions, float* obs_out, float* reward_out, double* reward64_out,
               uint8_t* done_out, int8_t* status_out, int auto_reset, heist_stream_t stream) {
  if (int rc = check_handle(h)) return rc;
  HEIST_REQUIRE(actions && obs_out && reward_out && done_out && status_out, "heist_step: null output/input");
  HEIST_REQUIRE(!h->p.stamps || h->stamp_words >= heist_stamp_words(h, 0), "heist_step: stamp buffer too small");
  if (lean_serves(h))  // the training rollout's tick on the lean kernel: heist_step_multi with K = 1 is
    return heist_step_multi(h, 1, actions, obs_out, reward_out, reward64_out, done_out, status_out, auto_reset,
                            stream);  // bit-identical by the heist_step_multi contract (heist.h)
  h->fan_pos = -1;  // headings advanced outside the K-tick launches' accounting
  return check_hip(heist::launch_step(h->p, actions, obs_out, reward_out, reward64_out, done_out, status_out,
                                      auto_reset, (hipStream_t)stream),
                   "heist_step");
}

int heist_step_multi(heist_t h, int K, const int64_t* actions, float* obs_out, float* reward_out,
                     double* reward64_out, uint8_t* done_out, int8_t* status_out, int auto_reset,
                     heist_stream_t stream) {
  if (int rc = check_handle(h)) return rc;
  HEIST_REQUIRE(K >= 1 && K <= 1024, "heist_step_multi: need 1 <= K <= 1024");
  HEIST_REQUIRE(actions && obs_out && reward_out && done_out && status_out, "heist_step_multi: null output/input");
  // (without a K-tick variant the launch runs K single ticks: either kernel's size may apply)
  HEIST_REQUIRE(!h->p.stamps || h->stamp_words >= std::max(heist_stamp_words(h, 1), heist_stamp_words(h, 0)),
                "heist_step_multi: stamp buffer too small");
  hipStream_t st = (hipStream_t)stream;
  // the shared fan table (FanTick): refilled when stale, used up, or last used by a launch on
  // another stream (streams do not order a refill against a launch still reading the table:
  // the new stream waits, on the device, for the event recorded behind the last K-tick
  // launch), else read at the launch's offset -- only when the K-tick kernel runs (otherwise
  // K single ticks advance the headings)
  EnvParams q = h->p;
  const bool kt = heist::multi_variant_exists(q.multi_waves, q.ray_chunk, q.multi_occ, q.vis_gap) && (q.C & 3) == 0 &&
                  (q.probe_mode == 0 || (q.probe_mode >= 21 && q.probe_mode <= 28)) && !q.sample_counter &&
                  !q.redo_counter;  // 21-28: the lean kernel's profiling variants (shared fan kept)
  q.fan_fill = 0;
  q.fan_base = 0;
  int next_pos = -1;
  if (kt && q.fan_on) {
    int pos = h->fan_pos;
    if (pos < 0 || pos + K > heist::kFanTicks || st != h->fan_stream) {
      if (h->fan_used && st != h->fan_stream)  // the refill must not overtake a launch still reading the table
        if (int rc = check_hip(hipStreamWaitEvent(st, h->fan_done, 0), "heist_step_multi: previous stream")) return rc;
      q.fan_fill = 1;
      pos = 0;
    }
    q.fan_base = pos;
    next_pos = pos + K;
  }
  const int rc = check_hip(heist::launch_step_multi(q, K, actions, obs_out, reward_out, reward64_out, done_out,
                                                    status_out, auto_reset, st),
                           "heist_step_multi");
  // the table position advances only with a launch that was issued
  h->fan_pos = rc ? -1 : next_pos;
  if (!rc && kt && q.fan_on) {
    if (!h->fan_done)
      if (int e = check_hip(hipEventCreateWithFlags(&h->fan_done, hipEventDisableTiming), "heist_step_multi: event")) {
        h->fan_pos = -1;
        return e;
      }
    if (int e = check_hip(hipEventRecord(h->fan_done, st), "heist_step_multi: event record")) {
      h->fan_pos = -1;
      return e;
    }
    h->fan_stream = st;
    h->fan_used = true;
  }
  return rc;
}

int heist_export(heist_t h, int32_t* scalars, int8_t* grid, double* cam_heading, int32_t* guard_idx,
                 double* guard_heading, heist_stream_t stream) {
  if (int rc = check_handle(h)) return rc;
  return check_hip(heist::launch_export(h->p, scalars, grid, cam_heading, guard_idx, guard_heading, (hipStream_t)stream),
                   "heist_export");
}

int heist_count_samples(heist_t h, uint64_t* counter) {
  if (int rc = check_handle(h)) return rc;
  h->p.sample_counter = reinterpret_cast<unsigned long long*>(counter);
  return 0;
}

int heist_count_redo(heist_t h, uint64_t* counter) {
  if (int rc = check_handle(h)) return rc;
  h->p.redo_counter = reinterpret_cast<unsigned long long*>(counter);
  return 0;
}

int heist_step_stamps(heist_t h, uint64_t* buf, int64_t n_words) {
  if (int rc = check_handle(h)) return rc;
  HEIST_REQUIRE(buf == nullptr || n_words >= 0, "heist_step_stamps: n_words < 0");
  h->p.stamps = reinterpret_cast<unsigned long long*>(buf);
  h->stamp_words = buf ? n_words : 0;
  return 0;
}

int64_t heist_stamp_words(heist_t h, int which) {
  if (check_handle(h)) return -1;
  return (int64_t)h->p.n_envs * (which ? 16 * h->p.multi_waves : 10 * h->p.step_waves);
}

int heist_step_waves(heist_t h) {
  if (int rc = check_handle(h)) return -rc;
  return h->p.step_waves;
}

int heist_get_config(heist_t h, int32_t* out, int n) {
  if (int rc = check_handle(h)) return rc;
  HEIST_REQUIRE(out != nullptr && n >= 0 && n <= 16, "heist_get_config: need out != NULL and 0 <= n <= 16");
  const EnvParams& p = h->p;
  const int32_t v[16] = {p.step_waves, p.ray_chunk,  p.step_occ,       p.vis_gap,   p.obs_store,  p.ray_mode,
                         p.probe_mode, p.dispatch_order, p.split_obs, p.guard_cones, p.multi_waves, p.fan_on,
                         p.lean,       p.interval_fans,  lean_serves(h) ? 1 : 0,
                         p.R == 32 && p.C == 32 && heist::lean_two_waves(p) ? 2 : 1};
  for (int k = 0; k < n; ++k) out[k] = v[k];
  return 0;
}

int heist_set_ray_mode(heist_t h, int ray_mode) {
  if (int rc = check_handle(h)) return rc;
  h->fan_pos = -1;
  HEIST_REQUIRE(ray_mode == 0 || ray_mode == 1, "heist_set_ray_mode: ray_mode must be 0 or 1");
  h->p.ray_mode = ray_mode;
  return 0;
}

int heist_set_guard_cones(heist_t h, int on) {
  if (int rc = check_handle(h)) return rc;
  h->fan_pos = -1;
  HEIST_REQUIRE(on == 0 || on == 1, "heist_set_guard_cones: on must be 0 or 1");
  h->p.guard_cones = on;
  return 0;
}

int heist_bfs_valid(const int32_t* grid, int n, int rows, int cols, int sr, int sc, int gr, int gc, uint8_t* valid_out,
                    heist_stream_t stream) {
  HEIST_REQUIRE(grid && valid_out, "heist_bfs_valid: null pointer");
  HEIST_REQUIRE(rows >= 1 && cols >= 1 && rows <= heist::kMaxDim && cols <= heist::kMaxDim,
                "heist_bfs_valid: need 1 <= rows, cols <= 64");
  HEIST_REQUIRE(sr >= 0 && sr < rows && sc >= 0 && sc < cols && gr >= 0 && gr < rows && gc >= 0 && gc < cols,
                "heist_bfs_valid: start/goal outside the grid");
  if (n <= 0) return 0;
  return check_hip(heist::launch_bfs(grid, n, rows, cols, sr, sc, gr, gc, valid_out, (hipStream_t)stream),
                   "heist_bfs_valid");
}

int heist_cones(int n, int rows, int cols, const uint8_t* walls, const int32_t* meta, const double* params,
                uint8_t* tiles_out, heist_stream_t stream) {
  HEIST_REQUIRE(walls && meta && params && tiles_out, "heist_cones: null pointer");
  HEIST_REQUIRE(rows >= 1 && cols >= 1 && rows <= heist::kMaxDim && cols <= heist::kMaxDim,
                "heist_cones: need 1 <= rows, cols <= 64");
  if (n <= 0) return 0;
  return check_hip(heist::launch_cones(n, rows, cols, walls, meta, params, tiles_out, 0, (hipStream_t)stream),
                   "heist_cones");
}

int heist_cones_mode(int n, int rows, int cols, const uint8_t* walls, const int32_t* meta, const double* params,
                     int ray_mode, uint8_t* tiles_out, heist_stream_t stream) {
  HEIST_REQUIRE(walls && meta && params && tiles_out, "heist_cones_mode: null pointer");
  HEIST_REQUIRE(rows >= 1 && cols >= 1 && rows <= heist::kMaxDim && cols <= heist::kMaxDim,
                "heist_cones_mode: need 1 <= rows, cols <= 64");
  HEIST_REQUIRE(ray_mode == 0 || ray_mode == 1, "heist_cones_mode: ray_mode must be 0 or 1");
  if (n <= 0) return 0;
  return check_hip(heist::launch_cones(n, rows, cols, walls, meta, params, tiles_out, ray_mode, (hipStream_t)stream),
                   "heist_cones_mode");
}

int heist_cone_order(int n, int rows, int cols, const uint8_t* walls, const int32_t* meta, const double* params,
                     uint32_t* keys_out, heist_stream_t stream) {
  HEIST_REQUIRE(walls && meta && params && keys_out, "heist_cone_order: null pointer");
  HEIST_REQUIRE(rows >= 1 && cols >= 1 && rows <= heist::kMaxDim && cols <= heist::kMaxDim,
                "heist_cone_order: need 1 <= rows, cols <= 64");
  if (n <= 0) return 0;
  return check_hip(heist::launch_cone_order(n, rows, cols, walls, meta, params, keys_out, (hipStream_t)stream),
                   "heist_cone_order");
}

int heist_fast_dir(const double* angle_deg, int64_t n, float* cos_out, float* sin_out, heist_stream_t stream) {
  HEIST_REQUIRE(angle_deg && cos_out && sin_out, "heist_fast_dir: null pointer");
  if (n <= 0) return 0;
  return check_hip(heist::launch_fast_dir(angle_deg, n, cos_out, sin_out, (hipStream_t)stream), "heist_fast_dir");
}

int heist_architect_decode(const int64_t* asset_map, int n, int rows, int cols, const float* cam_params,
                           int cam_stride, const int32_t* budget, int allow_cams, int allow_guards, int max_walls,
                           int max_cams, int max_guards, int max_path, int32_t* wall_rc, int32_t* n_walls,
                           double* cam_out, int32_t* n_cams, int32_t* guard_paths, int32_t* guard_meta,
                           double* guard_fov, int32_t* n_guards, heist_stream_t stream) {
  HEIST_REQUIRE(asset_map && cam_params && budget && n_walls && n_cams && n_guards, "heist_architect_decode: null pointer");
  HEIST_REQUIRE(rows >= 3 && cols >= 3 && rows <= heist::kMaxDim && cols <= heist::kMaxDim,
                "heist_architect_decode: need 3 <= rows, cols <= 64");
  HEIST_REQUIRE(cam_stride == 0 || cam_stride == 3, "heist_architect_decode: cam_stride must be 0 or 3");
  HEIST_REQUIRE(max_walls >= 0 && max_cams >= 0 && max_guards >= 0 && max_path >= 8,
                "heist_architect_decode: bad capacities (max_path >= 8)");
  HEIST_REQUIRE((max_walls == 0 || wall_rc) && (max_cams == 0 || cam_out) &&
                    (max_guards == 0 || (guard_paths && guard_meta && guard_fov)),
                "heist_architect_decode: null output array");
  if (n <= 0) return 0;
  return check_hip(heist::launch_arch_decode(asset_map, n, rows, cols, cam_params, cam_stride, budget, allow_cams,
                                             allow_guards, max_walls, max_cams, max_guards, max_path, wall_rc, n_walls,
                                             cam_out, n_cams, guard_paths, guard_meta, guard_fov, n_guards,
                                             (hipStream_t)stream),
                   "heist_architect_decode");
}

int heist_sincos(const double* x, int64_t n, double* sin_out, double* cos_out, heist_stream_t stream) {
  HEIST_REQUIRE(x && sin_out && cos_out, "heist_sincos: null pointer");
  if (n <= 0) return 0;
  return check_hip(heist::launch_sincos(x, n, sin_out, cos_out, (hipStream_t)stream), "heist_sincos");
}

int64_t heist_arch_update_workspace_bytes(void) { return heist::arch_update_workspace_bytes(); }

int heist_arch_update_supported(int rows, int cols) { return heist::arch_update_supported(rows, cols) ? 1 : 0; }

int heist_arch_update_sequence(float* const* params, float* const* exp_avg, float* const* exp_avg_sq,
                               const float* grid, int rows, int cols, const float* rewards, int k,
                               const float* step_scalars, double beta1, double beta2, double eps, double max_norm,
                               double value_coeff, float* value_loss, void* workspace, heist_stream_t stream) {
  HEIST_REQUIRE(params && exp_avg && exp_avg_sq && grid && workspace, "heist_arch_update_sequence: null pointer");
  HEIST_REQUIRE(heist::arch_update_supported(rows, cols),
                "heist_arch_update_sequence: rows x cols must be 8x8, 12x12, 16x16 or 20x20");
  HEIST_REQUIRE(k >= 0, "heist_arch_update_sequence: negative k");
  if (k == 0) return 0;
  HEIST_REQUIRE(rewards && value_loss && step_scalars, "heist_arch_update_sequence: null rewards / step_scalars / value_loss");
  for (int i = 0; i < 12; ++i)
    HEIST_REQUIRE(params[i] && exp_avg[i] && exp_avg_sq[i], "heist_arch_update_sequence: null tensor pointer");
  for (int i : {2, 4, 8})  // rows handed between workgroups are stored as whole 128-B lines
    HEIST_REQUIRE(((uintptr_t)params[i] & 127) == 0, "heist_arch_update_sequence: weights must be 128-byte aligned");
  HEIST_REQUIRE(((uintptr_t)workspace & 127) == 0, "heist_arch_update_sequence: workspace must be 128-byte aligned");
  HEIST_REQUIRE(beta1 >= 0 && beta1 < 1 && beta2 >= 0 && beta2 < 1 && eps >= 0,
                "heist_arch_update_sequence: bad Adam hyperparameters");
  return check_hip(heist::launch_arch_update(params, exp_avg, exp_avg_sq, grid, rows, cols, rewards, k, step_scalars,
                                             value_loss, workspace, beta1, beta2, eps, max_norm, value_coeff,
                                             (hipStream_t)stream),
                   "heist_arch_update_sequence");
}

int heist_arch_update_stamps(uint64_t* buf) {
  heist::set_arch_stamps(reinterpret_cast<unsigned long long*>(buf));
  return 0;
}

int heist_arch_update_status(const void* workspace, int* status, heist_stream_t stream) {
  HEIST_REQUIRE(workspace && status, "heist_arch_update_status: null pointer");
  unsigned flag[2] = {0, 0};
  const char* ctr = (const char*)workspace + heist::arch_update_workspace_bytes() - 64 * 4;
  hipStream_t st = (hipStream_t)stream;
  if (int rc = check_hip(hipMemcpyAsync(flag, ctr, sizeof(flag), hipMemcpyDeviceToHost, st), "heist_arch_update_status"))
    return rc;
  if (int rc = check_hip(hipStreamSynchronize(st), "heist_arch_update_status")) return rc;
  *status = (int)(flag[1] & 3u);
  return 0;
}

int heist_arch_update_timed_out(const void* workspace, int* timed_out, heist_stream_t stream) {
  HEIST_REQUIRE(workspace && timed_out, "heist_arch_update_timed_out: null pointer");
  int status = 0;
  if (int rc = heist_arch_update_status(workspace, &status, stream)) return rc;
  *timed_out = status & 1;
  return 0;
}

int heist_rollout_tally(const uint8_t* valid, int32_t* attempts, int attempts_per_layout, const uint8_t* done,
                        const int8_t* status, const double* reward64, int32_t* steps, double* reward_sum, int32_t* solve,
                        int32_t* detect, int32_t* timeout, float* h, float* c, int hidden, int n, heist_stream_t stream) {
  HEIST_REQUIRE(valid && attempts && done && status && reward64 && steps && reward_sum && solve && detect && timeout,
                "heist_rollout_tally: null pointer");
  HEIST_REQUIRE(n >= 0 && hidden >= 1 && (n == 0 || (h && c)), "heist_rollout_tally: bad sizes");
  if (n == 0) return 0;
  return check_hip(heist::launch_rollout_tally(valid, attempts, attempts_per_layout, done, status, reward64, steps,
                                               reward_sum, solve, detect, timeout, h, c, hidden, n, HEIST_VAULT_REACHED,
                                               HEIST_DETECTED,
                                               (hipStream_t)stream),
                   "heist_rollout_tally");
}

int heist_lstm_cell(const float* gates_x, const float* gates_h, const float* c, float* h_out, float* c_out, int hidden,
                    int n, heist_stream_t stream) {
  HEIST_REQUIRE(n >= 0 && hidden >= 1, "heist_lstm_cell: bad sizes");
  if (n == 0) return 0;
  HEIST_REQUIRE(gates_x && gates_h && c && h_out && c_out, "heist_lstm_cell: null pointer");
  return check_hip(heist::launch_lstm_cell(gates_x, gates_h, c, h_out, c_out, hidden, n, (hipStream_t)stream),
                   "heist_lstm_cell");
}

int heist_gae(const float* rewards, const float* values, const uint8_t* dones, const float* last_value, int T, int n,
              double gamma, double lam, float* adv_out, float* ret_out, heist_stream_t stream) {
  HEIST_REQUIRE(rewards && values && dones && adv_out && ret_out, "heist_gae: null pointer");
  HEIST_REQUIRE(T >= 0 && n >= 0, "heist_gae: negative size");
  if (T == 0 || n == 0) return 0;
  return check_hip(heist::launch_gae(rewards, values, dones, last_value, T, n, gamma, lam, adv_out, ret_out,
                                     (hipStream_t)stream),
                   "heist_gae");
}

int heist_adv_moments(const float* x, int64_t n, int phase, double* acc, heist_stream_t stream) {
  HEIST_REQUIRE(phase == 0 || phase == 1, "heist_adv_moments: phase must be 0 or 1");
  HEIST_REQUIRE(n >= 0, "heist_adv_moments: negative size");
  if (n == 0) return 0;  // an empty shard adds nothing to the sums (its rank still joins the all-reduce)
  HEIST_REQUIRE(x && acc, "heist_adv_moments: null pointer");
  return check_hip(heist::launch_adv_moments(x, n, phase, acc, (hipStream_t)stream), "heist_adv_moments");
}

int heist_adv_apply(float* x, int64_t n, const double* acc, float eps, heist_stream_t stream) {
  if (n <= 0) return 0;
  HEIST_REQUIRE(x && acc, "heist_adv_apply: null pointer");
  return check_hip(heist::launch_adv_apply(x, n, acc, eps, (hipStream_t)stream), "heist_adv_apply");
}

int heist_adv_normalize(float* x, int64_t n, double* scratch3, float eps, heist_stream_t stream) {
  HEIST_REQUIRE(x && scratch3, "heist_adv_normalize: null pointer");
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (int rc = check_hip(hipMemsetAsync(scratch3, 0, 3 * sizeof(double), st), "heist_adv_normalize")) return rc;
  if (int rc = check_hip(heist::launch_adv_moments(x, n, 0, scratch3, st), "heist_adv_normalize")) return rc;
  if (int rc = check_hip(heist::launch_adv_moments(x, n, 1, scratch3, st), "heist_adv_normalize")) return rc;
  return check_hip(heist::launch_adv_apply(x, n, scratch3, eps, st), "heist_adv_normalize");
}

int heist_ppo_loss(const float* logits, const float* values, const int64_t* actions, const float* old_logp,
                   const float* adv, const float* ret, int M, int A, double clip, double vcoef, double ecoef,
                   float* loss_parts, float* dlogits, float* dvalues, double* scratch, heist_stream_t stream) {
  HEIST_REQUIRE(logits && values && actions && old_logp && adv && ret && loss_parts && dlogits && dvalues && scratch,
                "heist_ppo_loss: null pointer");
  HEIST_REQUIRE(M >= 1, "heist_ppo_loss: M must be >= 1");
  HEIST_REQUIRE(A >= 1 && A <= 16, "heist_ppo_loss: need 1 <= A <= 16");
  return check_hip(heist::launch_ppo_loss(logits, values, actions, old_logp, adv, ret, M, A, clip, vcoef, ecoef,
                                          loss_parts, dlogits, dvalues, scratch, (hipStream_t)stream),
                   "heist_ppo_loss");
}

}  // extern "C"

int heist_solver_packed_bytes(void) { return heist::solver_packed_bytes(); }

int heist_solver_pack(const float* conv1_w, const float* conv1_b, const float* conv2_w, const float* conv2_b,
                      const float* conv3_w, const float* conv3_b, void* packed, heist_stream_t stream) {
  HEIST_REQUIRE(conv1_w && conv1_b && conv2_w && conv2_b && conv3_w && conv3_b && packed,
                "heist_solver_pack: null pointer");
  return check_hip(heist::launch_solver_pack(conv1_w, conv1_b, conv2_w, conv2_b, conv3_w, conv3_b, packed,
                                             (hipStream_t)stream),
                   "heist_solver_pack");
}

int heist_solver_features(const float* obs, int n, int rows, int cols, const void* packed, float* feat_out,
                          heist_stream_t stream) {
  HEIST_REQUIRE(obs && packed && feat_out, "heist_solver_features: null pointer");
  HEIST_REQUIRE(n >= 0, "heist_solver_features: n < 0");
  HEIST_REQUIRE(heist::solver_conv_supported(rows, cols),
                "heist_solver_features: grid " + std::to_string(rows) + "x" + std::to_string(cols) +
                    " not supported (20x20, 10x10)");
  if (n == 0) return 0;
  int dev = 0, n_cu = 0;
  if (int rc = check_hip(hipGetDevice(&dev), "hipGetDevice")) return rc;
  if (int rc = check_hip(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev),
                         "hipDeviceGetAttribute"))
    return rc;
  return check_hip(heist::launch_solver_conv(obs, n, rows, cols, packed, feat_out, n_cu, (hipStream_t)stream),
                   "heist_solver_features");
}

int heist_solver_head_packed_bytes(void) { return heist::solver_head_packed_bytes(); }

int heist_solver_head_pack(const float* fc_w, const float* fc_b, const float* w_ih, const float* w_hh,
                           const float* b_ih, const float* b_hh, const float* p1_w, const float* p1_b,
                           const float* v1_w, const float* v1_b, const float* p2_w, const float* p2_b,
                           const float* v2_w, const float* v2_b, int num_actions, void* packed,
                           heist_stream_t stream) {
  const float* w[14] = {fc_w, fc_b, w_ih, w_hh, b_ih, b_hh, p1_w, p1_b, v1_w, v1_b, p2_w, p2_b, v2_w, v2_b};
  for (const float* x : w) HEIST_REQUIRE(x != nullptr, "heist_solver_head_pack: null pointer");
  HEIST_REQUIRE(packed != nullptr, "heist_solver_head_pack: null packed");
  HEIST_REQUIRE(num_actions >= 1 && num_actions <= 7, "heist_solver_head_pack: need 1 <= num_actions <= 7");
  return check_hip(heist::launch_solver_head_pack(w, num_actions, packed, (hipStream_t)stream),
                   "heist_solver_head_pack");
}

int heist_solver_head(const float* feat, const float* h_in, const float* c_in, int n, const void* packed,
                      int num_actions, uint64_t seed, uint64_t counter, float* logits_out, float* value_out,
                      int64_t* action_out, float* logp_out, float* h_out, float* c_out, heist_stream_t stream) {
  HEIST_REQUIRE(feat && packed && value_out && action_out && logp_out && h_out && c_out,
                "heist_solver_head: null pointer");
  HEIST_REQUIRE(n >= 0, "heist_solver_head: n < 0");
  HEIST_REQUIRE(num_actions >= 1 && num_actions <= 7, "heist_solver_head: need 1 <= num_actions <= 7");
  return check_hip(heist::launch_solver_head(feat, h_in, c_in, n, packed, num_actions, seed, counter, logits_out,
                                             value_out, action_out, logp_out, h_out, c_out, (hipStream_t)stream),
                   "heist_solver_head");
}

int heist_bias_relu_nhwc(float* x, const float* bias, int64_t n_pos, int channels, heist_stream_t stream) {
  HEIST_REQUIRE(x && bias, "heist_bias_relu_nhwc: null pointer");
  HEIST_REQUIRE(n_pos >= 0 && channels > 0 && channels % 4 == 0, "heist_bias_relu_nhwc: need n_pos >= 0, channels % 4 == 0");
  HEIST_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)bias & 15) == 0, "heist_bias_relu_nhwc: 16-byte alignment");
  if (n_pos == 0) return 0;
  return check_hip(heist::launch_bias_relu(x, bias, n_pos, channels, (hipStream_t)stream), "heist_bias_relu_nhwc");
}

int heist_bias_relu_pool_nhwc(float* x, const float* bias, int n, int rows, int cols, int channels, float* feat_out,
                              heist_stream_t stream) {
  HEIST_REQUIRE(x && bias && feat_out, "heist_bias_relu_pool_nhwc: null pointer");
  HEIST_REQUIRE(n >= 0 && rows >= 4 && cols >= 4 && channels == 64, "heist_bias_relu_pool_nhwc: need rows, cols >= 4, 64 channels");
  HEIST_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)bias & 15) == 0, "heist_bias_relu_pool_nhwc: 16-byte alignment");
  if (n == 0) return 0;
  return check_hip(heist::launch_bias_relu_pool(x, bias, n, rows, cols, channels, feat_out, (hipStream_t)stream),
                   "heist_bias_relu_pool_nhwc");
}

int heist_pool_relu_bwd_nhwc(const float* dfeat, const float* y, int n, int rows, int cols, int channels, float* d_out,
                             float* partial, float* dbias_out, heist_stream_t stream) {
  HEIST_REQUIRE(dfeat && y && d_out && partial && dbias_out, "heist_pool_relu_bwd_nhwc: null pointer");
  HEIST_REQUIRE(n >= 1 && rows >= 4 && cols >= 4 && channels == 64, "heist_pool_relu_bwd_nhwc: need n >= 1, rows, cols >= 4, 64 channels");
  HEIST_REQUIRE(((uintptr_t)y & 15) == 0 && ((uintptr_t)d_out & 15) == 0 && ((uintptr_t)partial & 15) == 0,
                "heist_pool_relu_bwd_nhwc: 16-byte alignment");
  return check_hip(heist::launch_pool_relu_bwd(dfeat, y, n, rows, cols, channels, d_out, partial, dbias_out,
                                               (hipStream_t)stream),
                   "heist_pool_relu_bwd_nhwc");
}

int heist_relu_bwd_nhwc(float* g, const float* y, int n, int positions, int channels, float* partial, float* dbias_out,
                        heist_stream_t stream) {
  HEIST_REQUIRE(g && y && partial && dbias_out, "heist_relu_bwd_nhwc: null pointer");
  HEIST_REQUIRE(n >= 1 && positions >= 1 && (channels == 32 || channels == 64), "heist_relu_bwd_nhwc: need n >= 1, 32 or 64 channels");
  HEIST_REQUIRE(((uintptr_t)g & 15) == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)partial & 15) == 0,
                "heist_relu_bwd_nhwc: 16-byte alignment");
  return check_hip(heist::launch_relu_bwd(g, y, n, positions, channels, partial, dbias_out, (hipStream_t)stream),
                   "heist_relu_bwd_nhwc");
}

int heist_train_conv_supported(int rows, int cols) { return rows == 20 && cols == 20 ? 1 : 0; }

int heist_train_conv_frag_floats(int layer, int mode) {
  if (!((layer == 1 && mode == 0) || ((layer == 2 || layer == 3) && (mode == 0 || mode == 1)))) return -1;
  return heist::train_conv_frag_floats(layer, mode);
}

int heist_train_conv_pack(int layer, int mode, const float* w, float* frag, heist_stream_t stream) {
  HEIST_REQUIRE(w && frag, "heist_train_conv_pack: null pointer");
  HEIST_REQUIRE(heist_train_conv_frag_floats(layer, mode) > 0, "heist_train_conv_pack: layer 1 (mode 0), 2 or 3");
  return check_hip(heist::launch_train_conv_pack(layer, mode, w, frag, (hipStream_t)stream), "heist_train_conv_pack");
}

int heist_train_conv(int layer, int mode, const float* x, int n, int rows, int cols, const float* frag,
                     const float* bias, uint8_t* mask_bits, float* y, int* queue, heist_stream_t stream) {
  HEIST_REQUIRE(heist_train_conv_supported(rows, cols), "heist_train_conv: grid must be 20x20");
  HEIST_REQUIRE(heist_train_conv_frag_floats(layer, mode) > 0, "heist_train_conv: layer 1 (mode 0), 2 or 3");
  HEIST_REQUIRE(n >= 0, "heist_train_conv: n < 0");
  HEIST_REQUIRE(x && frag && y && queue, "heist_train_conv: null pointer");
  HEIST_REQUIRE(mode == 0 ? bias != nullptr : mask_bits != nullptr, "heist_train_conv: mode 0 needs bias, mode 1 mask_bits");
  for (const void* p : {(const void*)x, (const void*)frag, (const void*)y, mode ? (const void*)mask_bits : (const void*)bias})
    HEIST_REQUIRE(((uintptr_t)p & 15) == 0, "heist_train_conv: 16-byte alignment");
  if (n == 0) return 0;
  return check_hip(heist::launch_train_conv(layer, mode, x, n, rows, cols, frag, bias, mask_bits, y, queue,
                                            (hipStream_t)stream),
                   "heist_train_conv");
}

int64_t heist_train_conv_partial_floats(int layer, int n, int rows, int cols) {
  return heist::train_conv_partial_floats(layer, n, rows, cols);
}

int heist_train_conv_wgrad(int layer, const float* dy, const float* x, int n, int rows, int cols, float* partial,
                           float* dw, float* db, int* queue, heist_stream_t stream) {
  HEIST_REQUIRE(heist_train_conv_supported(rows, cols), "heist_train_conv_wgrad: grid must be 20x20");
  HEIST_REQUIRE(layer >= 1 && layer <= 3, "heist_train_conv_wgrad: layer 1, 2 or 3");
  HEIST_REQUIRE(n >= 1, "heist_train_conv_wgrad: n < 1");
  HEIST_REQUIRE(dy && x && partial && dw && db && queue, "heist_train_conv_wgrad: null pointer");
  HEIST_REQUIRE(((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)partial & 15) == 0,
                "heist_train_conv_wgrad: 16-byte alignment");
  return check_hip(heist::launch_train_conv_wgrad(layer, dy, x, n, rows, cols, partial, dw, db, queue,
                                                  (hipStream_t)stream),
                   "heist_train_conv_wgrad");
}

int heist_train_obs_nhwc4(const float* obs, int n, int rows, int cols, int64_t stride_n, int64_t stride_c,
                          int64_t stride_h, int64_t stride_w, float* x4, heist_stream_t stream) {
  HEIST_REQUIRE(obs && x4, "heist_train_obs_nhwc4: null pointer");
  HEIST_REQUIRE(n >= 0 && rows >= 1 && cols >= 1, "heist_train_obs_nhwc4: bad sizes");
  HEIST_REQUIRE(((uintptr_t)x4 & 15) == 0, "heist_train_obs_nhwc4: 16-byte alignment");
  if (n == 0) return 0;
  const int64_t st4[4] = {stride_n, stride_c, stride_h, stride_w};
  return check_hip(heist::launch_obs_nhwc4(obs, n, rows, cols, st4, x4, (hipStream_t)stream), "heist_train_obs_nhwc4");
}

int heist_train_pool(const float* a3, int n, int rows, int cols, float* feat, heist_stream_t stream) {
  HEIST_REQUIRE(a3 && feat, "heist_train_pool: null pointer");
  HEIST_REQUIRE(n >= 0 && rows >= 4 && cols >= 4, "heist_train_pool: bad sizes");
  if (n == 0) return 0;
  return check_hip(heist::launch_train_pool(a3, n, rows, cols, feat, (hipStream_t)stream), "heist_train_pool");
}

int heist_train_pool_bwd(const float* dfeat, const uint8_t* mask3_bits, int n, int rows, int cols, float* d3,
                         heist_stream_t stream) {
  HEIST_REQUIRE(dfeat && mask3_bits && d3, "heist_train_pool_bwd: null pointer");
  HEIST_REQUIRE(n >= 0 && rows >= 4 && cols >= 4, "heist_train_pool_bwd: bad sizes");
  HEIST_REQUIRE(((uintptr_t)d3 & 15) == 0, "heist_train_pool_bwd: 16-byte alignment");
  if (n == 0) return 0;
  return check_hip(heist::launch_train_pool_bwd(dfeat, mask3_bits, n, rows, cols, d3, (hipStream_t)stream),
                   "heist_train_pool_bwd");
}

int heist_solver_stamps(uint64_t* buf) {
  heist::set_solver_stamps(reinterpret_cast<unsigned long long*>(buf));
  return 0;
}
