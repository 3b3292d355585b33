// heist_env.hip -- CDNA4 kernels for the batched Heist environment.
//
// step/reset: one workgroup of W wavefronts (W = 1, 2, 4) owns one environment.
//   * Prefetch first: the env's tile grid, padded stop map and guard paths go to LDS,
//     cameras/guards to registers -- all issued together, so the env costs one HBM round
//     trip; a cached guard cone follows its guard record.  The observation's static
//     position plane is the same for every env and is read from L2 by write_obs.
//   * Cameras and guards are updated in registers (no store -> reload) and flattened
//     into one ray list; thread t casts rays t, t + 64W, ... (security.py:53-101,
//     :161-192) with the samples of a ray computed in blocks of four so the wall
//     lookups in LDS overlap; visible tiles are idempotent byte stores (no atomics).
//   * The solver/reward logic (environment.py:216-299) runs block-uniform; the
//     [3][R][C] float32 observation (environment.py:347-374) leaves in 16-byte stores.
// Arithmetic follows the reference's IEEE double semantics exactly: no FMA
// contraction, half-to-even rint(), glibc-exact sin/cos (heist_trig.h).
#include <utility>

#include "heist_device.h"
#include "heist_fan_intervals.h"
#include "heist_trig.h"

#pragma clang fp contract(off)

#ifndef HEIST_LEAN_OCC
#define HEIST_LEAN_OCC 4  // step_lean_kernel's waves per SIMD the compiler budgets registers for (A/B)
#endif

namespace heist {

__constant__ double kSinCosTab[4 * HEIST_SINCOS_TAB_ROWS] = HEIST_SINCOS_TAB_INIT;
constexpr int kTabDoubles = 4 * HEIST_SINCOS_TAB_ROWS;

__device__ __forceinline__ int iabs_(int a) { return a < 0 ? -a : a; }
__device__ __forceinline__ int unpack_r(uint16_t v) { return v & 0xff; }
__device__ __forceinline__ int unpack_c(uint16_t v) { return v >> 8; }

// Python float % 360.0 (floatobject.c float_rem: remainder takes the divisor's sign).
// Headings advance by a positive speed below 360, so x lies in [0, 720) almost always:
// there fmod is x or x - 360, and x - 360 is exact (Sterbenz: 360 <= x < 720), so the
// shortcut returns fmod's value without the library's reduction loop; -0.0 -> +0.0 as
// Python does.
__device__ __forceinline__ double py_mod360(double x) {
  if (x > 0.0 && x < 720.0) return x >= 360.0 ? x - 360.0 : x;
  double r = fmod(x, 360.0);
  if (r != 0.0) {
    if (r < 0.0) r += 360.0;
  } else {
    r = 0.0;
  }
  return r;
}

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

// order[b] = env | wave priority << 24 (order_kernel); the env a step / reset block runs
constexpr int32_t kOrderEnvMask = 0xFFFFFF;
__device__ __forceinline__ int block_env(const EnvParams& p) {
  return p.dispatch_order ? (p.order[blockIdx.x] & kOrderEnvMask) : (int)blockIdx.x;
}

// ---------------------------------------------------------------------------
// LDS carve-up for one env
// ---------------------------------------------------------------------------

struct EnvLds {
  uint8_t* wall;   // LDS offset 0: [(R+2G)(C+2G)] ray stop map, 1 = wall or outside the grid (G = kRing)
  uint8_t* vis;    // LDS offset D: visibility with the same padded geometry (ring bytes unused): camera
                   // rays and live-raycast guards; the cached guard cones are ORed in where read
                   // (cone_vis4).  LDS offset 2D: sink plane, where march_fast sends the stores of
                   // stopped samples (never read)
  uint8_t* grid;   // [RC]
  Emit* em;        // [n_emit]
  uint16_t* path;  // [max_guards][max_path]
  int* queue;      // [W][64] per-wave exact-path ray queues (cast_rays)
  int* meta;       // [0] emitters, [1] total rays
  uint16_t* cone;  // [2][max_guards][16] cached guard cones (kind-2 emitters, heist_device.h): set 0 this
                   // tick's pose, set 1 the pose an auto-reset would give (patrol point 0, same heading)
  uint32_t* rpos;  // [max_guards] patrol point 0 of each guard (row | col << 8), for the reset cones
  int PC;          // padded row stride C + 2G
  int off0;        // padded index of tile (0, 0): G * PC + G
  // r >= 0 and PC < 2^24: one full-rate v_mad_u32_u24 (a 32-bit multiply is quarter rate)
  __device__ __forceinline__ int at(int r, int c) const { return off0 + (int)__umul24((uint32_t)r, (uint32_t)PC) + c; }
};

// Width G of the stop ring around the grid: the longest fp32 fast-path ray (range
// kTieMaxRange = 6) ends at most G tiles from its emitter, so every one of its sample
// addresses lies inside the padded map, stopped or not (march_fast); the exact path's
// U-sample chunks need G >= U.  Even, so the half-to-even rounding can carry the offset.
constexpr int kRing = 6;

// The padded planes hold (R + 2G) x (C + 2G) bytes; D is the compile-time distance from
// the stop map to the visibility plane (so one address serves both), 1024 for grids up to
// 20 x 20, 2048 up to 33 x 33 and 6144 for the 64 x 64 maximum.
__host__ __device__ inline int padded_bytes(int R, int C) { return (R + 2 * kRing) * (C + 2 * kRing); }

__host__ __device__ inline size_t env_lds_bytes(int R, int C, int n_emit, int path_words, int D, int waves,
                                                int cone_guards = 0) {
  const int RC = R * C;
  return 3 * (size_t)D + align16(RC) + align16(sizeof(Emit) * (n_emit > 0 ? n_emit : 1)) +
         align16(sizeof(uint16_t) * (path_words > 0 ? path_words : 1)) +
         sizeof(int) * 64 * (size_t)waves + 32 + 68 * (size_t)cone_guards;
}

template <int D>
__device__ __forceinline__ EnvLds carve(unsigned char* smem, int R, int C, int n_emit, int path_words, int waves,
                                        int cone_guards = 0) {
  const int RC = R * C;
  EnvLds L;
  L.wall = smem;
  L.vis = smem + D;
  size_t o = 3 * (size_t)D;  // [2D, 3D): the fast path's sink for masked stores (never read)
  L.grid = smem + o; o += align16(RC);
  L.em = reinterpret_cast<Emit*>(smem + o); o += align16(sizeof(Emit) * (n_emit > 0 ? n_emit : 1));
  L.path = reinterpret_cast<uint16_t*>(smem + o); o += align16(sizeof(uint16_t) * (path_words > 0 ? path_words : 1));
  L.queue = reinterpret_cast<int*>(smem + o); o += sizeof(int) * 64 * (size_t)waves;
  L.meta = reinterpret_cast<int*>(smem + o); o += 32;
  L.cone = reinterpret_cast<uint16_t*>(smem + o);
  L.rpos = reinterpret_cast<uint32_t*>(L.cone + 32 * cone_guards);
  L.PC = C + 2 * kRing;
  L.off0 = kRing * L.PC + kRing;
  return L;
}

// The padded stop map for tile grid g (stride C bytes in LDS).
template <int NT>
__device__ __forceinline__ void build_wall_map(const uint8_t* g, const EnvLds& L, int R, int C) {
  const int PC = L.PC;
  // i / PC as a multiply-shift: with m = ceil(2^20 / PC) the quotient is exact for
  // i < 2^20 / (m * PC - 2^20), i.e. every i < 2^20 / 75 > 76 * 76 (PC <= 76)
  const uint32_t m = ((1u << 20) + (uint32_t)PC - 1u) / (uint32_t)PC;
  for (int i = threadIdx.x; i < (R + 2 * kRing) * PC; i += NT) {
    const int pr = (int)(((uint32_t)i * m) >> 20);
    const int r = pr - kRing, c = i - pr * PC - kRing;
    const bool out = (unsigned)r >= (unsigned)R || (unsigned)c >= (unsigned)C;
    L.wall[i] = out ? 1 : (g[r * C + c] == kWall ? 1 : 0);
  }
}

// ---------------------------------------------------------------------------
// Raycasting
// ---------------------------------------------------------------------------

// x + 0x1.8p52 rounds x to an integer half-to-even (Python round()) and leaves it in the
// low word, exact for |x| < 2^51.  Adding an EVEN offset k to the constant yields
// round(x) + k with the same tie breaks, which folds the ring offset into the rounding.
template <int K>
__device__ __forceinline__ int round_plus(double x) {
  static_assert((K & 1) == 0, "the offset must be even to keep half-to-even ties");
  constexpr double kMagic = 0x1.8p52 + (double)K;
  return (int)(uint32_t)__builtin_bit_cast(uint64_t, x + kMagic);
}

// U consecutive samples of one ray: positions, U stop-map reads in flight together, then
// branch-free visibility stores (a masked sample writes byte 0 of the vis plane, a ring
// byte nobody reads).  TAIL masks samples past the ray's last one (u >= left).  OWN is the
// number of leading samples that may land on the emitter's own tile (see cast_rays).
// Returns the index of the chunk's first sample that ends the ray (a wall or the grid
// edge; with TAIL also sample `left`), U if none does.
// KEY (heist_cone_order): instead of marking the tile, lower its u32 first-visit key
// keys[address] to kbase + the 1-based sample index (LDS atomic min).
template <int U, int D, bool TAIL, int OWN, bool KEY = false>
__device__ __forceinline__ int sample_chunk(unsigned char* smem, int PC, int own, double col, double row,
                                            double dxs, double dys, double kd, int left, uint32_t* keys = nullptr,
                                            uint32_t kbase = 0) {
  int a[U], w[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const double ku = kd + (double)u;  // exact small integer
    const int c = round_plus<kRing>(col + dxs * ku);  // padded column c + G
    const int r = round_plus<kRing>(row + dys * ku);
    a[u] = __mul24(r, PC) + c;
    w[u] = smem[a[u]];
  }
  bool stop = false;
  int first = U;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool st = w[u] != 0 || (TAIL && u >= left);
    first = (!stop && st) ? u : first;
    stop |= st;
    const bool skip = stop || (u < OWN && a[u] == own);
    if (KEY) {
      if (!skip) atomicMin(&keys[a[u]], kbase + (uint32_t)kd + (uint32_t)u);
    } else {
      smem[D + (skip ? 0 : a[u])] = 1;
    }
  }
  return first;
}

// All samples of one ray from sample s0 = 1 on; the first chunk is peeled so that only it
// carries the own-tile test.  Returns the ray's sample count up to and including the
// sample that ends it (n_samp if none does): the raycast's work figure, the same on the
// fast path.
template <int U, int D, int OWN, bool KEY = false>
__device__ __forceinline__ int march(unsigned char* smem, int PC, int own, double col, double row, double dxs,
                                     double dys, int n_samp, uint32_t* keys = nullptr, uint32_t kbase = 0) {
  if (n_samp < U) {
    const int f = sample_chunk<U, D, true, OWN, KEY>(smem, PC, own, col, row, dxs, dys, 1.0, n_samp, keys, kbase);
    return f + 1 < n_samp ? f + 1 : n_samp;
  }
  int f = sample_chunk<U, D, false, OWN, KEY>(smem, PC, own, col, row, dxs, dys, 1.0, U, keys, kbase);
  if (f < U) return f + 1;
  double kd = 1.0 + U;
  int s0 = 1 + U;
  for (; s0 + U - 1 <= n_samp; s0 += U, kd += (double)U) {
    f = sample_chunk<U, D, false, 0, KEY>(smem, PC, own, col, row, dxs, dys, kd, U, keys, kbase);
    if (f < U) return s0 + f;
  }
  if (s0 > n_samp) return n_samp;
  const int left = n_samp - s0 + 1;
  f = sample_chunk<U, D, true, 0, KEY>(smem, PC, own, col, row, dxs, dys, kd, left, keys, kbase);
  return s0 - 1 + (f + 1 < left ? f + 1 : left);
}

// ---- fp32 fast path -------------------------------------------------------------------
//
// A sample's tile is rint(col + dx*dist) (fp64, glibc dx).  Camera samples are
// dist = k/2 (k = 1 .. 2*range) and guard samples dist = k = (2k)/2 (k = 1 .. range), so
// with K = 2*range every sample is x = (dx/2) * k' for some k' <= K.  x_k sits on a .5 tie iff dx = j/k' with j odd: the
// TIE POINTS of the ray are the fractions j/k', j odd, k' <= K.  Between two tie points
// every rint(x_k) is constant, so for any approximation d of dx with |d - dx| <= E,
// rint(col + k*d/2) equals the exact fp64 result whenever no tie point lies within E of
// d (and the fp64 path itself cannot round differently: that needs dx within ~1e-14 of a
// tie point).  The same holds for dy.
//
// The fast path therefore computes the direction in fp32 (angle reduced to an octant in
// fp64, then the Cephes sinf/cosf polynomials; within ~2e-7 of the true direction, E =
// kDirErr = 1e-6 bounds it with margin, tests/test_gpu_env.py::test_fast_direction_error),
// screens |dx| and |dy| against the tie points once per ray, and marches with one fp32
// fma per sample (magic-constant rounding, exact product, single rounding).  With
// L = lcm(1..12) = 27720 the tie points for K <= 12 are integers of t = |d|*L, flagged in
// a 27721-bit table; a ray is re-cast on the exact path (glibc sin/cos restatement + fp64
// march) when |t - rint(t)| < kTieRad = E*L + (fp32 error of t) and rint(t) is a tie
// point.  Emitters with range > 6 (K > 12) always take the exact path.
//
// The tie point 1 (|d| = 1, an axis-aligned ray) is screened differently: there the
// direction is flat in the angle, so |d| within E of 1 covers an angle window of +-1.5e-3
// rad around every multiple of 90 degrees (most of all re-casts), yet only a far smaller
// window matters.  With x the angle's remainder from the nearest multiple of 90 degrees,
// the exact |d| is 1 - delta, delta ~ x^2/2.  For |x| >= kAxisRad = 1e-6 rad, delta >=
// 5e-13 keeps every fp64 col + (d/2)*k (k <= 12, |col| < 64) strictly below its .5 tie,
// i.e. fp64 rounds as the real numbers do, and so does the fast path once an fp32 |d|
// that rounded to 1.0f is replaced by 1 - 2^-24 (the same side of the tie point; the next
// one, 11/12, is far).  Rays with |x| < kAxisRad take the exact path.  Guard rays (whole
// tiles) have no tie at |d| = 1, and the replacement leaves their samples unchanged.
constexpr float kDirErr = 1e-6f;
constexpr float kAxisRad = 1e-6f;
constexpr float kBelowOne = 0.99999994f;  // 1 - 2^-24
constexpr int kTieMaxRange = 6;
static_assert(kRing >= kTieMaxRange, "march_fast reads every sample of a ray unconditionally");
constexpr int kTieL = 27720;                                  // lcm(1, ..., 12)
constexpr float kTieRad = kDirErr * (float)kTieL + 4e-3f;     // 0.0317 in units of t

struct TieBits {
  uint32_t w[kTieL / 32 + 1];
};
constexpr TieBits make_tie_bits() {
  TieBits t{};
  for (int k = 1; k <= 2 * kTieMaxRange; ++k)
    for (int j = 1; j <= k; j += 2) {
      const int n = j * (kTieL / k);
      t.w[n >> 5] |= 1u << (n & 31);
    }
  t.w[kTieL >> 5] &= ~(1u << (kTieL & 31));  // |d| = 1 is screened by kAxisRad instead
  return t;
}
__constant__ TieBits kTieBits = make_tie_bits();

// The same tie points as one byte per 64-wide bucket of t = |d| * 27720 (tie points are at
// least 27720 / 132 = 210 apart, so a bucket holds at most one): tie[b] = its offset in
// bucket b, 0xFF if none; rank[b] = the tie points in buckets below b.  The K-tick kernel
// keeps both in LDS (868 B): the screen and the dedup key (cast_rays, DEDUP) read them there.
constexpr int kTieBuckets = kTieL / 64 + 1;  // 434
struct TieBuckets {
  uint8_t tie[kTieBuckets];
  uint8_t rank[kTieBuckets];
};
constexpr TieBuckets make_tie_buckets() {
  TieBuckets t{};
  for (int b = 0; b < kTieBuckets; ++b) t.tie[b] = 0xFF;
  const TieBits bits = make_tie_bits();
  int below = 0;
  for (int b = 0; b < kTieBuckets; ++b) {
    t.rank[b] = (uint8_t)below;
    for (int o = 0; o < 64; ++o) {
      const int n = 64 * b + o;
      if (n <= kTieL && ((bits.w[n >> 5] >> (n & 31)) & 1u)) {
        t.tie[b] = (uint8_t)o;
        ++below;
      }
    }
  }
  return t;
}
__constant__ TieBuckets kTieBuckets_ = make_tie_buckets();
static_assert(kTieL / 132 > 64, "at most one tie point per 64-wide bucket");

// 1.5 * 2^23: for |v| < 2^22, fl32(v + kMagic32) = kMagic32 + rint(v), and the low 22 bits
// of its bit pattern hold the integer (plus any offset folded into the constant).
constexpr float kMagic32 = 12582912.0f;

// cos and sin of a (degrees) in fp32: q = rint(a / 90) in fp64, the octant remainder
// (|r| <= 45 deg) to fp32 radians, Cephes sinf/cosf minimax polynomials on [-pi/4, pi/4],
// then the quadrant rotation.  *xr = the remainder in radians (for the axis screen).
__device__ __forceinline__ void fast_dir(double a, float* cs, float* sn, float* xr) {
  const double q = __builtin_rint(a * (1.0 / 90.0));
  const float x = (float)(__builtin_fma(-90.0, q, a) * kDegToRad);
  const float z = x * x;
  const float ps = __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  const float pc = __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                                  4.166664568298827e-2f);
  const float s = __builtin_fmaf(ps * z, x, x);
  const float c = __builtin_fmaf(pc * z, z, __builtin_fmaf(-0.5f, z, 1.0f));
  const int n = (int)q;
  const float s0 = (n & 1) ? c : s;  // sin(a) up to sign
  const float c0 = (n & 1) ? s : c;  // cos(a) up to sign
  *sn = (n & 2) ? -s0 : s0;
  *cs = ((n + 1) & 2) ? -c0 : c0;
  *xr = x;
}

// |d| that rounded to 1.0f in fp32 -> 1 - 2^-24 with its sign (see kAxisRad).
__device__ __forceinline__ float below_one(float d) {
  return __builtin_fabsf(d) == 1.0f ? __builtin_copysignf(kBelowOne, d) : d;
}

// true if |c| or |s| lies within kTieRad / L of a tie point below 1, or a camera ray is
// within kAxisRad of an axis (the ray needs the exact path).
// Scalar code on purpose: the float2 form of this function is miscompiled by the ROCm 7.2
// clang (the two table lookups are merged into one).
__device__ __forceinline__ bool near_tie(float c, float s, float x, bool camera) {
  const float tx = __builtin_fabsf(c) * (float)kTieL, ty = __builtin_fabsf(s) * (float)kTieL;
  const float mx = tx + kMagic32, my = ty + kMagic32;
  const uint32_t nx = __builtin_bit_cast(uint32_t, mx) - 0x4B400000u;
  const uint32_t ny = __builtin_bit_cast(uint32_t, my) - 0x4B400000u;
  const uint32_t wx = kTieBits.w[nx >> 5], wy = kTieBits.w[ny >> 5];
  const bool cx = __builtin_fabsf(tx - (mx - kMagic32)) < kTieRad;
  const bool cy = __builtin_fabsf(ty - (my - kMagic32)) < kTieRad;
  return ((((wx >> (nx & 31)) & (uint32_t)cx) | ((wy >> (ny & 31)) & (uint32_t)cy)) & 1u) ||
         (camera && __builtin_fabsf(x) < kAxisRad);
}

// near_tie with the bucket tables in LDS (tb = TieBuckets copied there), plus the fast
// path's dedup key: rays whose |dx| and |dy| lie in the same intervals between consecutive
// tie points, with the same signs, have the same offsets rint(k dx / 2), rint(k dy / 2) for
// every sample k <= 12 (rint of a non-tie value is translation-invariant by integers), so
// the same tile sequence from any emitter tile (cast_rays, DEDUP).  key = interval of |dx|
// | interval of |dy| << 8 | sign bits << 16.
__device__ __forceinline__ bool near_tie_key(float c, float s, float x, bool camera, const TieBuckets* tb,
                                             uint32_t* key) {
  const float tx = __builtin_fabsf(c) * (float)kTieL, ty = __builtin_fabsf(s) * (float)kTieL;
  const float mx = tx + kMagic32, my = ty + kMagic32;
  const uint32_t nx = __builtin_bit_cast(uint32_t, mx) - 0x4B400000u;
  const uint32_t ny = __builtin_bit_cast(uint32_t, my) - 0x4B400000u;
  const uint32_t bx = tb->tie[nx >> 6], by = tb->tie[ny >> 6];
  const uint32_t rx = tb->rank[nx >> 6], ry = tb->rank[ny >> 6];
  const float fx = mx - kMagic32, fy = my - kMagic32;  // rint(t)
  const bool cx = __builtin_fabsf(tx - fx) < kTieRad, cy = __builtin_fabsf(ty - fy) < kTieRad;
  const uint32_t ox = nx & 63u, oy = ny & 63u;
  // tie points of the bucket below t: those before its offset, and the offset itself when t > it
  const uint32_t kx = rx + (uint32_t)(bx != 0xFFu && (ox > bx || (ox == bx && tx > fx)));
  const uint32_t ky = ry + (uint32_t)(by != 0xFFu && (oy > by || (oy == by && ty > fy)));
  *key = kx | (ky << 8) | ((uint32_t)(c < 0.0f) << 16) | ((uint32_t)(s < 0.0f) << 17);
  return (cx && bx == ox) || (cy && by == oy) || (camera && __builtin_fabsf(x) < kAxisRad);
}

// LDS byte at an absolute LDS address (the dynamic LDS base is folded into the address
// once per ray instead of once per access).
__device__ __forceinline__ uint8_t lds_ld(uint32_t a) {
  return *reinterpret_cast<__attribute__((address_space(3))) uint8_t*>(a);
}
__device__ __forceinline__ void lds_st(uint32_t a, uint8_t v) {
  *reinterpret_cast<__attribute__((address_space(3))) uint8_t*>(a) = v;
}

// 32-bit OR as one v_or_b32: the compiler otherwise narrows the OR of byte loads to a
// 16-bit op and re-extends it with a v_and before every mad_u24 that consumes it.
__device__ __forceinline__ uint32_t or_b32(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_or_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// (x, y) = K * 2^-149 * (dxs, dys) + (mx, my) as ONE v_pk_fma_f32 (two fp32 FMAs, each
// rounded once, as v_fma_f32 does); K is an integer inline constant, i.e. the denormal
// K * 2^-149, applied to both halves (op_sel_hi).  Inline asm: the compiler's own packed
// form of this loop is miscompiled by ROCm 7.2 clang (see march_fast).
// VM: the addend m (the ray origin) per lane in VGPRs instead of wave-uniform in SGPRs.
template <int K, bool VM = false>
__device__ __forceinline__ uint64_t pk_fma_k(uint64_t d, uint64_t m) {
  static_assert(K >= 1 && K <= 12, "inline constant");
  uint64_t r;
#define HEIST_PKC(n)                                                                              \
  if constexpr (K == n) {                                                                         \
    if constexpr (VM) asm("v_pk_fma_f32 %0, %1, " #n ", %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(d), "v"(m)); \
    else asm("v_pk_fma_f32 %0, %1, " #n ", %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(d), "s"(m));  \
  }
  HEIST_PKC(1) HEIST_PKC(2) HEIST_PKC(3) HEIST_PKC(4) HEIST_PKC(5) HEIST_PKC(6)
  HEIST_PKC(7) HEIST_PKC(8) HEIST_PKC(9) HEIST_PKC(10) HEIST_PKC(11) HEIST_PKC(12)
#undef HEIST_PKC
  return r;
}

// row * PC + col as one v_mad_u32_u24 (row < 2^24): with a compile-time PC the compiler
// otherwise forms the product from a 64-bit funnel shift, a mask and an add (3 VALU)
__device__ __forceinline__ uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
  return r;
}

template <int U, bool VM>
__device__ __forceinline__ uint32_t fast_addr(uint32_t PC, uint64_t d, uint64_t m) {
  const uint64_t r = pk_fma_k<U + 1, VM>(d, m);
  return mad_u24((uint32_t)(r >> 32), PC, (uint32_t)r);
}

template <int NS, bool VM, int... Us>
__device__ __forceinline__ void fast_addrs(uint32_t (&a)[NS], uint32_t PC, uint64_t d, uint64_t m,
                                           std::integer_sequence<int, Us...>) {
  ((a[Us] = fast_addr<Us, VM>(PC, d, m)), ...);
}

// Every sample k = 1 .. n_samp of a fast ray in one LDS round trip.  Coordinates are
// computed in units of the smallest fp32 denormal (2^-149; fp32 denormals are preserved):
// k and the padded emitter (col, row) -- the LDS base folded into the column -- enter as
// denormals whose bit patterns are those integers, so fl32(k * dxs + mx) =
// 2^-149 * rint_even(col' + k * dx * stride), one rounding of the exact product-sum (the
// same rint as fp64's), and its bit pattern IS that integer: one mad_u24 (row * PC + col)
// gives the LDS address of the stop byte.  The ring is as wide as the longest fast ray
// (kRing >= kTieMaxRange), so each sample address lies inside the padded stop map whether
// or not the ray has already stopped: all NS wall reads are issued before any is used, and
// a running stop flag sends the visibility store of a stopped sample (and of the emitter's
// own tile) to the sink plane (address + D, i.e. 2D .. 3D, never read) with one more
// mad_u24 instead of a compare and select.  NS = n_samp, or with CLAMP NS >= n_samp and the
// samples past n_samp repeat sample n_samp (k clamped), which changes nothing.  Only the
// first two samples can land on the emitter's own tile (see cast_rays).  Returns the ray's
// sample count up to and including the sample that ends it (n_samp if none does), when
// COUNT.  Scalar fp32 on purpose (and this file builds with -fno-slp-vectorize): ROCm 7.2
// clang miscompiles the float2 / v_pk_fma_f32 form of this loop (a lane's negation is lost).
// VM: the origin (mx, my, own) differs per lane (packed direction-group marches).
template <int D, int NS, bool CLAMP, bool COUNT, bool VM = false>
__device__ __forceinline__ int march_fast(uint32_t PC, uint32_t own, float dxs, float dys, float mx, float my,
                                          int n_samp) {
  uint32_t a[NS], w[NS];
  const uint64_t dv = ((uint64_t)__builtin_bit_cast(uint32_t, dys) << 32) | __builtin_bit_cast(uint32_t, dxs);
  const uint64_t mv = ((uint64_t)__builtin_bit_cast(uint32_t, my) << 32) | __builtin_bit_cast(uint32_t, mx);
  if constexpr (!CLAMP) fast_addrs<NS, VM>(a, PC, dv, mv, std::make_integer_sequence<int, NS>{});
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    if (CLAMP) {
      const uint32_t ki = u > 0 ? (uint32_t)(u + 1 < n_samp ? u + 1 : n_samp) : 1u;
      const float k = __builtin_bit_cast(float, ki);  // ki * 2^-149 (wave-uniform)
      const float yx = __builtin_fmaf(k, dxs, mx), yy = __builtin_fmaf(k, dys, my);
      a[u] = __umul24(__builtin_bit_cast(uint32_t, yy), PC) + __builtin_bit_cast(uint32_t, yx);
    }
    w[u] = lds_ld(a[u]);
  }
  uint32_t stop = 0;
  int cnt = n_samp;
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    if (COUNT) cnt = (stop == 0 && w[u] != 0 && u < n_samp) ? u + 1 : cnt;
    stop = u == 0 ? w[0] : or_b32(stop, w[u]);
    const uint32_t skip = u < 2 ? or_b32(stop, (uint32_t)(a[u] == own)) : stop;  // 0 or 1
    lds_st(__umul24(skip, (uint32_t)D) + a[u] + D, 1);
  }
  return cnt;
}

// One ray on the exact path: security.py:70 angle, glibc-exact sin/cos, fp64 march.
// Returns the ray's sample count (march).
// A ray angle that is a whole number of half degrees (guards after an axis move; the
// reference's default cameras: heading 0, fov 60, speed 15) reads the same glibc-exact
// sin/cos from hd (computed by heist_trig::sincos at heist_create) instead of evaluating it.
template <int U, int D, bool KEY = false>
__device__ __forceinline__ int exact_ray(unsigned char* smem, const Emit& E, int i, int PC, int probe,
                                         const double* hd, uint32_t* keys = nullptr) {
  const double angle = E.hmh + (E.fov * (double)i) / (double)E.num_rays;  // security.py:70
  double sn, cs;
  const double a2 = angle * 2.0;  // exact
  if (probe == 3) {  // profiling: fixed direction, no sin/cos
    sn = 0.3 + 1e-3 * (double)i;
    cs = 0.7;
  } else if (hd && a2 == __builtin_rint(a2) && a2 >= -0.5 * kHalfDegN && a2 < 0.5 * kHalfDegN) {
    const int m = (int)a2 + kHalfDegN / 2;
    sn = hd[m];
    cs = hd[kHalfDegN + m];
  } else {
    const double rad = angle * kDegToRad;  // math.radians
    heist_trig::sincos(rad, kSinCosTab, &sn, &cs);
  }
  const int own = (E.row + kRing) * PC + (E.col + kRing);
  const int n_samp = E.kind == 0 ? 2 * E.range : E.range;
  // dist = stride * s with stride a power of two, so dx * dist == (dx * stride) * s
  // bit for bit; dy = -sin (security.py:72-75).
  const double col = (double)E.col, row = (double)E.row;
  const uint32_t kbase = (uint32_t)i << 12;  // first-visit key: (ray, sample) in ray-major order
  if (E.kind == 0) return march<U, D, 2, KEY>(smem, PC, own, col, row, cs * 0.5, -sn * 0.5, n_samp, keys, kbase);
  return march<U, D, 0, KEY>(smem, PC, own, col, row, cs, -sn, n_samp, keys, kbase);
}

// Wave-uniform values into scalar registers (every lane holds the same copy).
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ double uni(double x) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// lane m's double, wave-uniform
__device__ __forceinline__ double uni_lane(double x, int m) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, m);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), m);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ Emit uni(const Emit& e) {
  Emit u;
  u.hmh = uni(e.hmh); u.fov = uni(e.fov); u.step = uni(e.step);
  u.row = uni(e.row); u.col = uni(e.col); u.range = uni(e.range); u.num_rays = uni(e.num_rays);
  u.first = uni(e.first); u.kind = uni(e.kind); u.members = uni(e.members);
  return u;
}

// An emitter's rays go to the fp32 fast path unless it is exact-only (mode 1, range > 6).
__device__ __forceinline__ bool fast_emitter(const Emit& E, int mode) { return mode == 0 && E.range <= kTieMaxRange; }

// The emitter of ray chunk c (wave-uniform), searching forward from emitter k.
__device__ __forceinline__ int emitter_of_chunk(const EnvLds& L, int n_em, int k, int c) {
  while (k + 1 < n_em && uni(L.em[k + 1].first) <= c) ++k;
  return k;
}

// Cast every ray of the env's emitters and mark visible tiles (visibility.py:48-57).
// Camera rays sample dist = 0.5, 1.0, ..., range (np.linspace(0,1,3) sub-steps; the
// duplicated integer samples of security.py:78-82 are idempotent and skipped); guard
// rays sample dist = 1..range.  A wall or the grid edge ends the ray; the emitter's own
// tile is never marked by its rays.
//
// On the exact path a sample moves at most one tile per axis from the previous one, and a
// chunk of U samples only starts while the ray is still inside the grid, so every sample
// lands within U <= G tiles of the grid; a fast ray stays within its range <= G of its
// emitter (march_fast).  The G-wide ring of stop bytes makes every lookup unconditional,
// with no clamping.  Only a camera's first two samples (dist 0.5, 1) can round back to its
// own tile (|dx|, |dy| < 0.5 cannot both hold beyond dist 1 since dx^2 + dy^2 = 1), and a
// guard's rays never reach it at dist >= 1 (its tile is marked afterwards anyway), so the
// own-tile test is confined to the first two samples.
//
// Work unit: a CHUNK of 64 consecutive rays of one emitter (publish_emitters numbers them),
// one ray per lane; wave w takes chunks w, w + W, ...  Within a chunk the emitter, and so
// its pose, sample count and stride, is wave-uniform and lives in scalar registers; only
// the ray angle differs per lane.  Two passes per wave, so that the exact path's fp64
// registers are not live during the fast one.  Pass 1 casts the fast emitters' rays on the
// fp32 fast path; a ray the tie screen rejects goes to the wave's 64-entry LDS queue
// (ballot + mbcnt, no atomics).  Pass 2 casts the queued rays exactly, one per lane (a wave
// whose queue overflowed re-walks its fast chunks and re-casts every ray the same
// deterministic screen rejects), then every ray of the wave's exact-only chunks.
// Visibility stores are idempotent, so the pass order does not matter.  COUNT: samples (up
// to the one that ends each ray) are summed in LDS meta[2] and exact casts in meta[4] (the
// ALU work figures of SURVEY 8(d)); raycast_pass adds the env's totals to its counters.
// DEDUP (the K-tick kernel): the fast path marches one ray per distinct tile sequence.
// Fast rays of a direction group whose dedup key (near_tie_key) equals the previous
// lane's are dropped -- their sequence, and so the tiles they mark from every member's
// tile, is the previous ray's -- and the others go to the wave's unique queue uq (128
// directions in LDS), which is marched 64 at a time (and whenever the group changes): an
// Architect camera fan of 0.5-degree rays has about a third as many distinct sequences as
// rays.  tb: the tie bucket tables in LDS.
// HEIST_PACK_FLUSH (build-time A/B switch, default 1): with two or more waves per env the
// K-tick kernel's dedup flush packs (member, direction) pairs over the lanes (13.1 vs 13.5 us
// per 4096-env tick at 2 waves); one wave per env keeps one march per member with a
// wave-uniform origin (11.8 vs 12.15 us packed: the per-lane origins cost it registers),
// profiles/r03f_bench_*pack*.log.
#ifndef HEIST_PACK_FLUSH
#define HEIST_PACK_FLUSH 1
#endif

// The shared fan's emitter for one tick (FanTick header), loaded by the K-tick kernel ahead of
// the raycast so that the per-chunk test compares registers (a global load per chunk would put
// its latency on every chunk of every group); n_uniq < 0: no table.
struct FanHdr {
  double hmh, fov;
  int num_rays, range, n_uniq, n_tie;
  float2 dir;  // this lane's unique direction uniq[lane] (loaded with the header; lanes >= n_uniq: unused)
};
__device__ __forceinline__ FanHdr fan_hdr(const FanTick* f) {
  FanHdr h;
  h.hmh = uni(f->hmh); h.fov = uni(f->fov);  // wave-uniform: scalar registers across the tick
  h.num_rays = uni(f->num_rays); h.range = uni(f->range); h.n_uniq = uni(f->n_uniq); h.n_tie = uni(f->n_tie);
  const int lane = threadIdx.x & 63;  // < kFanRays: always inside the table
  h.dir = make_float2(f->uniq[2 * lane], f->uniq[2 * lane + 1]);
  return h;
}

template <int NT, int U, int D, bool COUNT, bool DEDUP = false>
__device__ void cast_rays(unsigned char* smem, const EnvLds& L, int mode, int probe, const double* hd,
                          const TieBuckets* tb = nullptr, float2* uq = nullptr, const FanTick* fan = nullptr,
                          FanHdr fh = FanHdr{0.0, 0.0, 0, 0, -1, 0, {0.0f, 0.0f}}) {
  static_assert(U == 2 || U == 4, "exact-path chunk");
  static_assert(kRing >= U, "the exact path's chunks stay inside the ring");
  constexpr int W = NT / 64;
  const int n_em = uni(L.meta[0]);
  const int n_chunk = uni(L.meta[1]);
  const int PC = L.PC;
  const int lane = threadIdx.x & 63;
  const int wave = uni((int)(threadIdx.x >> 6));
  int* queue = L.queue + wave * 64;
  const uint32_t base = (uint32_t)(uintptr_t)smem;  // LDS address of the stop map
  unsigned int n_eval = 0, n_exact = 0;
  int qn = 0;               // near-tie rays met by this wave (queued while <= 64)
  bool exact_em = false;    // this wave owns chunks of an exact-only emitter
  int k = 0;
  // DEDUP: the unique queue of group uk (uqn entries); flush(n) marches entries 0 .. n-1
  int uqn = 0, uk = -1;
  if (DEDUP) uq += wave * 128;
  constexpr bool kPackFlush = HEIST_PACK_FLUSH != 0 && W >= 2;
  // flush(cnt): the group's cnt unique directions uq[0 .. cnt) from each of its `members`
  // tiles, packed as (member, direction) pairs p = m * cnt + j over the lanes, 64 pairs per
  // march (a 2-camera group of <= 32 unique directions: one march instead of two)
  auto march_uniq = [&](int kk, int cnt, auto src) {  // src(j): unique direction j of group kk
    const Emit Eq = uni(L.em[kk]);
    const int n_samp = Eq.kind == 0 ? 2 * Eq.range : Eq.range;
    const int n_pair = kPackFlush ? Eq.members * cnt : cnt;
    for (int p0 = 0; p0 < n_pair; p0 += 64) {
      int j = p0 + lane, m = 0;
      if (kPackFlush)
        for (int mm = 1; mm < Eq.members; ++mm)  // m = pair / cnt, j = pair % cnt (members is small)
          if (j >= cnt) {
            j -= cnt;
            ++m;
          }
      // src may permute across lanes (the shared fan's directions): every lane calls it, the
      // lanes past n_pair with a valid index, before they drop out (a lane permute reads
      // nothing from an inactive lane)
      const float2 d = src(p0 + lane < n_pair ? j : 0);
      if (p0 + lane >= n_pair) continue;
      auto group = [&](auto ns, auto clamp) {
        constexpr int NS = decltype(ns)::value;
        constexpr bool CL = decltype(clamp)::value;
        if constexpr (kPackFlush) {
          const int row = L.em[kk + m].row, col = L.em[kk + m].col;
          const uint32_t own = base + (uint32_t)((row + kRing) * PC + (col + kRing));
          const float mx = __builtin_bit_cast(float, base + (uint32_t)(col + kRing));
          const float my = __builtin_bit_cast(float, (uint32_t)(row + kRing));
          march_fast<D, NS, CL, false, true>(PC, own, d.x, d.y, mx, my, n_samp);
        } else {  // one march per member, origin in SGPRs
          for (int mm = 0; mm < Eq.members; ++mm) {
            const int row = mm == 0 ? Eq.row : uni(L.em[kk + mm].row);
            const int col = mm == 0 ? Eq.col : uni(L.em[kk + mm].col);
            const uint32_t own = base + (uint32_t)((row + kRing) * PC + (col + kRing));
            const float mx = __builtin_bit_cast(float, base + (uint32_t)(col + kRing));
            const float my = __builtin_bit_cast(float, (uint32_t)(row + kRing));
            march_fast<D, NS, CL, false>(PC, own, d.x, d.y, mx, my, n_samp);
          }
        }
      };
      if (n_samp == 2 * kTieMaxRange)
        group(std::integral_constant<int, 2 * kTieMaxRange>{}, std::false_type{});
      else if (n_samp == 4)
        group(std::integral_constant<int, 4>{}, std::false_type{});
      else if (n_samp < 4)
        group(std::integral_constant<int, 4>{}, std::true_type{});
      else
        group(std::integral_constant<int, 2 * kTieMaxRange>{}, std::true_type{});
    }
  };
  auto flush = [&](int cnt) { march_uniq(uk, cnt, [&](int j) { return uq[j]; }); };
  // pass 1: fp32 fast path
  for (int c = wave; c < n_chunk; c += W) {
    k = emitter_of_chunk(L, n_em, k, c);
    const Emit E = uni(L.em[k]);
    if (!fast_emitter(E, mode)) {
      exact_em = true;
      continue;
    }
    if constexpr (DEDUP) {
      // the tick's shared fan (FanTick): a camera group casting exactly its emitter takes
      // its unique directions and near-tie rays from the table, once, at its first chunk
      if (fh.n_uniq >= 0 && E.kind == 0 && E.hmh == fh.hmh && E.fov == fh.fov && E.num_rays == fh.num_rays &&
          E.range == fh.range) {
        if (c == E.first) {
          if (uqn > 0) {  // another group's queued directions
            flush(uqn);
            uqn = 0;
          }
          const int nt = fh.n_tie;
          for (int b0 = 0; b0 < nt; b0 += 64)
            if (b0 + lane < nt && qn + b0 + lane < 64) queue[qn + b0 + lane] = (k << 16) | (int)fan->tie[b0 + lane];
          qn += nt;
          // directions 0 .. 63 from the registers loaded with the header (a lane permute),
          // the rest of a wide fan from the table
          const float* fu = fan->uniq;
          march_uniq(k, fh.n_uniq, [&](int j) {
            if (j < 64)
              return make_float2(__shfl(fh.dir.x, j, 64), __shfl(fh.dir.y, j, 64));
            return make_float2(fu[2 * j], fu[2 * j + 1]);
          });
        }
        continue;
      }
    }
    const int i = (c - E.first) * 64 + lane;
    const bool active = i <= E.num_rays;  // rays 0 .. num_rays (security.py:68)
    float cf, sf, xr;
    fast_dir(__builtin_fma((double)i, E.step, E.hmh), &cf, &sf, &xr);
    if (probe == 2) {  // profiling: angles and sin/cos only
      if (sf == 12345.0f && cf == 0.0f) L.meta[3] = 1;  // keeps the sin/cos live
      continue;
    }
    if (probe == 3) {  // profiling: fixed direction, no sin/cos
      sf = 0.3f + 1e-3f * (float)i;
      cf = 0.7f;
    }
    uint32_t key = 0;
    const bool tie = active && probe != 3 &&
                     (DEDUP ? near_tie_key(cf, sf, xr, E.kind == 0, tb, &key) : near_tie(cf, sf, xr, E.kind == 0));
    const unsigned long long b = __ballot(tie);
    if (tie) {
      const int pos = qn + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
      if (pos < 64) queue[pos] = (k << 16) | i;
    }
    qn += __popcll(b);
    if constexpr (DEDUP) {
      const uint32_t mine = (active && !tie) ? key : 0xFFFFFFFFu;
      const uint32_t prev = (uint32_t)__shfl_up((int)mine, 1, 64);
      const bool fresh = active && !tie && (lane == 0 || prev != mine);
      if (k != uk && uqn > 0) {  // the queue (< 64 entries) holds another group's rays
        flush(uqn);
        uqn = 0;
      }
      uk = k;
      const unsigned long long fb = __ballot(fresh);
      if (fresh) {
        const int pos = uqn + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(fb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fb, 0u));
        const float h = E.kind == 0 ? 0.5f : 1.0f;
        uq[pos] = make_float2(below_one(cf) * h, -below_one(sf) * h);
      }
      uqn += __popcll(fb);
      if (uqn >= 64) {
        flush(64);
        const float2 d = uq[64 + (lane & 63)];
        if (lane < uqn - 64) uq[lane] = d;
        uqn -= 64;
      }
      continue;
    }
    if (active && !tie) {
      const int n_samp = E.kind == 0 ? 2 * E.range : E.range;  // every member of a group: same range
      const float h = E.kind == 0 ? 0.5f : 1.0f;  // sample stride: camera half tiles, guard whole tiles
      const float dxs = below_one(cf) * h, dys = -below_one(sf) * h;  // exact scalings; dy = -sin (security.py:72-75)
      // the ray of every member of the direction group: same direction, each from its own tile
      auto group = [&](auto ns, auto clamp) {
        constexpr int NS = decltype(ns)::value;
        constexpr bool CL = decltype(clamp)::value;
        for (int m = 0; m < E.members; ++m) {
          const int row = m == 0 ? E.row : uni(L.em[k + m].row);
          const int col = m == 0 ? E.col : uni(L.em[k + m].col);
          const uint32_t own = base + (uint32_t)((row + kRing) * PC + (col + kRing));
          // the padded emitter position as denormal bit patterns (march_fast), LDS base on the column
          const float mx = __builtin_bit_cast(float, base + (uint32_t)(col + kRing));
          const float my = __builtin_bit_cast(float, (uint32_t)(row + kRing));
          n_eval += (unsigned int)march_fast<D, NS, CL, COUNT>(PC, own, dxs, dys, mx, my, n_samp);
        }
      };
      if (n_samp == 2 * kTieMaxRange)  // the reference cameras (range 6)
        group(std::integral_constant<int, 2 * kTieMaxRange>{}, std::false_type{});
      else if (n_samp == 4)  // the reference guards (range 4)
        group(std::integral_constant<int, 4>{}, std::false_type{});
      else if (n_samp < 4)
        group(std::integral_constant<int, 4>{}, std::true_type{});
      else
        group(std::integral_constant<int, 2 * kTieMaxRange>{}, std::true_type{});
    }
  }
  if (DEDUP && uqn > 0) flush(uqn);
  if (probe == 2) return;
  // pass 2: exact path (the wave's own LDS writes to its queue are ordered before its reads)
  __builtin_amdgcn_wave_barrier();
  if (qn <= 64) {
    if (lane < qn) {
      const int v = queue[lane];
      const int kq = v >> 16;
      for (int m = 0; m < L.em[kq].members; ++m) {
        ++n_exact;
        n_eval += (unsigned int)exact_ray<U, D>(smem, L.em[kq + m], v & 0xffff, PC, probe, hd);
      }
    }
  } else {
    k = 0;
    for (int c = wave; c < n_chunk; c += W) {
      k = emitter_of_chunk(L, n_em, k, c);
      const Emit E = uni(L.em[k]);
      if (!fast_emitter(E, mode)) continue;
      const int i = (c - E.first) * 64 + lane;
      float cf, sf, xr;
      fast_dir(__builtin_fma((double)i, E.step, E.hmh), &cf, &sf, &xr);
      if (i <= E.num_rays && near_tie(cf, sf, xr, E.kind == 0))
        for (int m = 0; m < E.members; ++m) {
          ++n_exact;
          n_eval += (unsigned int)exact_ray<U, D>(smem, L.em[k + m], i, PC, probe, hd);
        }
    }
  }
  if (exact_em) {
    k = 0;
    for (int c = wave; c < n_chunk; c += W) {
      k = emitter_of_chunk(L, n_em, k, c);
      const Emit E = uni(L.em[k]);
      if (fast_emitter(E, mode)) continue;
      const int i = (c - E.first) * 64 + lane;
      if (i <= E.num_rays)
        for (int m = 0; m < E.members; ++m) {
          ++n_exact;
          n_eval += (unsigned int)exact_ray<U, D>(smem, L.em[k + m], i, PC, probe, hd);
        }
    }
  }
  if (COUNT) {
    atomicAdd(reinterpret_cast<unsigned int*>(&L.meta[2]), n_eval);
    atomicAdd(reinterpret_cast<unsigned int*>(&L.meta[4]), n_exact);
  }
}

// Publish this tick's emitter table: thread t < n_em holds emitter SLOT t in E (camera
// slots 0 .. max_cams-1, then guard slots; a slot past the env's camera or guard count has
// kind -1 and no rays).  Every slot lives in wave 0 (at most 64 of them), where an
// exclusive lane scan of the emitters' chunk counts (ceil((num_rays + 1) / 64) chunks of
// 64 rays) gives each emitter its first chunk index.
// Direction groups: a camera whose (heading - fov/2, fov, num_rays, range) equal the
// previous slot's casts its rays in the same directions (security.py:70), so it joins that
// slot's group and gets no chunks of its own; the group leader's chunks compute each ray
// direction (and its tie screen) once and march it from every member's tile.  Cameras an
// Architect decodes share one fov/speed/heading per layout (networks.py:283-322), so all
// of a layout's cameras form one group.
static_assert(kMaxEmitters <= 64, "publish_emitters keeps every emitter in wave 0");
__device__ __forceinline__ void publish_emitters(const EnvLds& L, Emit E, int n_em) {
  const int t = threadIdx.x;
  if (t < 64) {
    const double ph = __shfl_up(E.hmh, 1, 64), pf = __shfl_up(E.fov, 1, 64);
    const int pn = __shfl_up(E.num_rays, 1, 64), pr = __shfl_up(E.range, 1, 64), pk = __shfl_up(E.kind, 1, 64);
    const bool cont = t > 0 && t < n_em && E.kind == 0 && pk == 0 && ph == E.hmh && pf == E.fov &&
                      pn == E.num_rays && pr == E.range;
    const unsigned long long lead = __ballot(!cont) | (n_em < 64 ? 1ull << n_em : 0ull);  // + sentinel slot n_em
    const unsigned long long above = t < 63 ? lead >> (t + 1) : 0ull;
    E.members = cont ? 0 : (above ? (int)__builtin_ctzll(above) + 1 : 64 - t);
    const int cnt = (t < n_em && !cont && (E.kind == 0 || E.kind == 1)) ? (E.num_rays + 1 + 63) / 64 : 0;  // 2: cached cone
    // exclusive prefix sum of cnt over the lanes, bit slice by bit slice: lane t's share of
    // slice b is 2^b x (lanes below t with bit b set), one ballot + mbcnt per slice and no
    // LDS round trip (a shuffle scan is six dependent ds_bpermutes); cnt < 2^9
    int excl = 0, total = 0;
    for (int b = 0; b < 9; ++b) {
      const unsigned long long m = __ballot((cnt >> b) & 1);
      excl += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
      total += __popcll(m) << b;
      if (__ballot(cnt >> (b + 1)) == 0ull) break;
    }
    if (t < n_em) {
      E.first = excl;
      L.em[t] = E;
    }
    const unsigned long long cached = __ballot(t < n_em && E.kind == 2);  // guards with a cached cone
    if (t == 63) {
      L.meta[0] = n_em;
      L.meta[1] = total;
      L.meta[2] = 0;
      L.meta[4] = 0;
      L.meta[6] = (int)(uint32_t)cached;
      L.meta[7] = (int)(uint32_t)(cached >> 32);
    }
  }
}

__device__ __forceinline__ Emit cam_emit(const Cam& cm) {
  Emit E;
  E.hmh = cm.heading - cm.fov / 2.0;  // security.py:64, :70
  E.fov = cm.fov;
  E.row = cm.row; E.col = cm.col; E.range = cm.range; E.num_rays = cm.num_rays;
  E.step = cm.fov * __builtin_amdgcn_rcp((double)cm.num_rays);  // fast-path angles only: approximate
  E.first = 0; E.kind = 0; E.members = 1;
  return E;
}

__device__ __forceinline__ Emit guard_emit(const Guard& gd) {
  Emit E;
  E.hmh = gd.heading - gd.fov / 2.0;
  E.fov = gd.fov;
  E.row = unpack_r(gd.pos); E.col = unpack_c(gd.pos); E.range = gd.range; E.num_rays = gd.num_rays;
  E.step = gd.fov * __builtin_amdgcn_rcp((double)gd.num_rays);
  E.first = 0; E.kind = gd.hslot == kUncached ? 1 : 2; E.members = 1;
  return E;
}

// ---- guard cone cache (heist_device.h) --------------------------------------------------

// Element offset (in u16) of the cone entry of guard g of env e at (patrol index, slot).
__device__ __forceinline__ size_t cone_entry(const EnvParams& p, int e, int g, int idx, int slot) {
  return ((((size_t)e * p.max_guards + g) * kConePath + idx) * kConeSlots + slot) * kConeEntry;
}

// One env's records as wave-uniform (SGPR) base pointers, so that per-lane accesses are a
// 32-bit offset from a scalar base (saddr addressing) instead of 64-bit vector index math.
struct EnvBase {
  Cam* cams;
  Guard* guards;
  const uint16_t* paths;
  const uint16_t* cones;
};
__device__ __forceinline__ EnvBase env_base(const EnvParams& p, int e) {
  EnvBase b;
  b.cams = p.cams + (size_t)e * p.max_cams;
  b.guards = p.guards + (size_t)e * p.max_guards;
  b.paths = p.paths + (size_t)e * p.max_guards * p.max_path;
  b.cones = p.cones + (size_t)e * p.max_guards * (kConePath * kConeSlots * kConeEntry);
  return b;
}
// u16 offset of guard g's cone entry (patrol index, slot) from EnvBase::cones
__device__ __forceinline__ uint32_t cone_off(uint32_t g, uint32_t idx, uint32_t slot) {
  return ((g * kConePath + idx) * kConeSlots + slot) * (uint32_t)kConeEntry;  // constant multipliers: shifts
}

// A cached guard's cone for its pose after this tick's move (move: the env acts and the
// patrol has >= 2 points, security.py:147) into LDS cone[g]: the record's nslot names the
// heading slot of the next patrol point, so the entry is known before the barrier.
__device__ __forceinline__ void stage_guard_cone(const EnvParams& p, int e, const EnvLds& L, int g, const Guard& gd,
                                                 bool act) {
  if (gd.hslot == kUncached) return;
  int idx = gd.idx, slot = gd.hslot;
  if (act && gd.len >= 2) {
    idx += gd.step;
    if (idx >= gd.len) idx -= gd.len;
    slot = gd.nslot;
  }
  const uint4* src = reinterpret_cast<const uint4*>(p.cones + cone_entry(p, e, g, idx, slot));
  const uint4 a = src[0], b = src[1];
  uint4* dst = reinterpret_cast<uint4*>(L.cone + 16 * g);
  dst[0] = a;
  dst[1] = b;
}

// Visibility of tiles (r, c0 .. c0 + 3) under the cached guard cones (the kind-2 slots,
// mask in meta[6..7] from publish_emitters) as four 0/1 bytes (byte j = tile c0 + j), read
// straight from the staged 32-byte cone entries instead of stamping them into a plane.
// set 0: this tick's cones (rows L.cone[16 g], guard on its emitter slot's tile); set 1: the
// cones an in-step auto-reset gives (rows L.cone[16 (mg + g)], guard at patrol point 0).
// Bit dc + 7 of row dr + 7 is tile (gr + dr, gc + dc); a cone only names tiles inside the
// grid (guard_cone_kernel), so no bounds test on (r, c) is needed.
__device__ __forceinline__ uint32_t cone_vis4(const EnvLds& L, int mc, int mg, int set, int r, int c0) {
  uint64_t m = ((uint64_t)(uint32_t)uni(L.meta[7]) << 32) | (uint32_t)uni(L.meta[6]);
  uint32_t v = 0;
  while (m) {
    const int k = (int)__builtin_ctzll(m);
    m &= m - 1;
    const int g = k - mc;
    int gr, gc;
    if (set) {
      const int rp = uni((int)L.rpos[g]);
      gr = unpack_r(rp);
      gc = unpack_c(rp);
    } else {
      gr = uni(L.em[k].row);
      gc = uni(L.em[k].col);
    }
    const int dr = r - gr + kConeRange;
    const uint32_t row = (unsigned)dr <= 2u * kConeRange ? (uint32_t)L.cone[16 * (set * mg + g) + dr] : 0u;
    // bits dc .. dc + 3 of the row, dc = c0 - gc + 7 in [-4, 28) after the shift by 4
    const int sh = c0 - gc + kConeRange + 4;
    const uint32_t b = __builtin_amdgcn_ubfe(row << 4, (uint32_t)(sh < 0 ? 0 : (sh > 31 ? 31 : sh)), 4u);
    v |= __umul24(b, 0x204081u) & 0x01010101u;  // bit j -> byte j (24-bit multiply: full rate)
  }
  return v;
}

// Visibility (visibility.py:31-65) once the emitter table (n_slot slots, guards from slot
// mc on) is in LDS and vis is zeroed.  CNT: 1 ray-sample / exact-ray counting compiled in
// (the step kernel's counting variant), 0 not, -1 chosen at run time (reset).
template <int NT, int U, int D, int CNT = -1>
__device__ __forceinline__ void raycast_pass(const EnvParams& p, int e, unsigned char* smem, const EnvLds& L, int n_slot,
                                             int mc, int probe = 0) {
  __syncthreads();  // emitter table, stop map and cleared vis in place
  const int t = threadIdx.x;
  if (t >= mc && t < n_slot) {  // a live guard's own tile (visibility.py:59; a cached cone holds it)
    const Emit E = L.em[t];
    if (E.kind == 1) L.vis[L.at(E.row, E.col)] = 1;
  }
  if (probe != 1 && probe != 5) {
    if (CNT == 1 || (CNT < 0 && (p.sample_counter || p.redo_counter)))
      cast_rays<NT, U, D, true>(smem, L, p.ray_mode, probe, p.half_deg);
    else
      cast_rays<NT, U, D, false>(smem, L, p.ray_mode, probe, p.half_deg);
  }
  __syncthreads();
  if (CNT != 0 && p.sample_counter && t == 0) p.sample_counter[e] += (unsigned int)L.meta[2];
  if (CNT != 0 && p.redo_counter && t == 0) p.redo_counter[e] += (unsigned int)L.meta[4];
}

// Zero the ray plane.
template <int NT>
__device__ __forceinline__ void clear_vis(const EnvParams& p, const EnvLds& L) {
  uint32_t* v4 = reinterpret_cast<uint32_t*>(L.vis);
  for (int i = threadIdx.x; i < (padded_bytes(p.R, p.C) + 3) / 4; i += NT) v4[i] = 0u;
}

// ---------------------------------------------------------------------------
// Prefetch / observation
// ---------------------------------------------------------------------------

// A camera or a guard as two 16-byte register loads; the destination is fixed and the
// type is chosen afterwards by bit-cast (selecting a destination struct member instead
// would defeat SROA and put the whole prefetch in scratch).
struct EmitterRaw {
  uint4 a, b;
};
static_assert(sizeof(EmitterRaw) == sizeof(Cam) && sizeof(EmitterRaw) == sizeof(Guard), "emitter records");

__device__ __forceinline__ Cam as_cam(const EmitterRaw& r) { return __builtin_bit_cast(Cam, r); }
__device__ __forceinline__ Guard as_guard(const EmitterRaw& r) { return __builtin_bit_cast(Guard, r); }

// Issue every per-env HBM read at once: grid and stop map (for LDS), this thread's
// camera/guard record (for registers).  Each thread's first element of every array is loaded before anything is
// stored, so the whole prefetch is one memory round trip; the loops only cover what one
// pass of NT threads cannot (W < 4, grids above 32 x 32, long patrol paths).  Thread t <
// max_cams + max_guards loads emitter slot t (camera t, then guard t - max_cams) whether or
// not the env fills it, so no load waits for the EnvScalars (scalar loads) to arrive.
// Packed stop-map byte j (bits = padded cells 8 j .. 8 j + 7) -> 8 bytes of the LDS wall
// plane: (x * 0x204081) & 0x01010101 spreads 4 bits to bit 0 of 4 bytes (no carries).
__device__ __forceinline__ void expand_stop(uint8_t* wall, int j, uint32_t b) {
  uint2 v;
  v.x = __umul24(b & 15u, 0x204081u) & 0x01010101u;
  v.y = __umul24((b >> 4) & 15u, 0x204081u) & 0x01010101u;
  *reinterpret_cast<uint2*>(wall + 8 * j) = v;
}

template <int NT>
__device__ __forceinline__ void prefetch(const EnvParams& p, int e, const EnvBase& eb, const EnvLds& L,
                                         EmitterRaw& raw) {
  const int t = threadIdx.x;
  const int RC = p.RC;
  const uint8_t* src = p.grid + (size_t)e * RC;
  const bool vec = (RC & 3) == 0;
  const int n4 = vec ? RC / 4 : 0;
  const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d4 = reinterpret_cast<uint32_t*>(L.grid);

  uint32_t gv = 0u;
  if (t < n4) gv = s4[t];
  // the layout's padded stop map, built once by set_layout_kernel (bit-packed)
  const uint8_t* ss = p.stop + (size_t)e * p.stop_bytes;
  const int n_stop = p.stop_bytes;
  uint32_t sv = 0u;
  if (t < n_stop) sv = ss[t];
  raw.a = make_uint4(0u, 0u, 0u, 0u);
  raw.b = raw.a;
  if (t < p.max_cams + p.max_guards) {
    const uint4* rs = t < p.max_cams ? reinterpret_cast<const uint4*>(eb.cams + (uint32_t)t)
                                     : reinterpret_cast<const uint4*>(eb.guards + (uint32_t)(t - p.max_cams));
    raw.a = rs[0];
    raw.b = rs[1];
  }
  if (t < n4) d4[t] = gv;
  if (t < n_stop) expand_stop(L.wall, t, sv);
  for (int i = t + NT; i < n_stop; i += NT) expand_stop(L.wall, i, ss[i]);
  for (int i = t + NT; i < n4; i += NT) {
    d4[i] = s4[i];
  }
  if (!vec) {
    for (int i = t; i < RC; i += NT) {
      L.grid[i] = src[i];
    }
  }
}

// Set lane m (0..3) of v; m outside 0..3 leaves v unchanged (no dynamic indexing:
// that would put the vector in scratch).
__device__ __forceinline__ void patch4(float4& v, int m, float val) {
  if (m == 0) v.x = val;
  else if (m == 1) v.y = val;
  else if (m == 2) v.z = val;
  else if (m == 3) v.w = val;
}

// One 16-byte observation store at byte offset `off` of the env's row (buffer descriptor rs)
// with the handle's cache policy (EnvParams::obs_store, default 2 = nt).  The 20 MB of
// observations per 4096-env step are the launch's largest write; plain stores leave them
// dirty in L2 for the kernel boundary to write back (MI355X_MICROARCH.md, boundary row:
// + dirty bytes / 6 TB/s per dependent launch).  Measured per 4096-env step (C2 layouts,
// profiles/r02ba_probe_obs_store.log): plain 16.66 us, sc1 16.22, nt 15.44, sc1 nt 16.10.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void obs_put(__amdgpu_buffer_rsrc_t rs, int pol, int off, float4 v) {
  const u32x4_t u = __builtin_bit_cast(u32x4_t, v);
  if (pol == 1) __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 16);       // sc1
  else if (pol == 2) __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 2);   // nt
  else if (pol == 3) __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 18);  // sc1 nt
  else __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 0);
}

// Observation row [3][R][C] (environment.py:347-374): occupancy / 5, visibility (ray
// plane | cached guard cones of cone set `cset`, cone_vis4), and the position channel
// (static plane with the solver and vault cells patched; the vault wins if the solver
// stands on it).
template <int NT>
__device__ __forceinline__ void write_obs(const EnvParams& p, int e, const EnvScalars& s, const EnvLds& L, int cset,
                                          float* __restrict__ obs) {
  const int t = threadIdx.x;
  const int RC = p.RC, C = p.C;
  const int mc = p.max_cams, mg = p.max_guards;
  float* o = obs + (size_t)e * 3 * RC;
  const int solver = s.pos_r * C + s.pos_c;
  const int vault = p.vr * C + p.vc;
  const float sv = p.plane1[solver];  // fl32(1 + g) (see heist_create)
  static_assert((kRing & 1) == 0, "padded vis rows of a C % 4 == 0 grid are 2-byte aligned");
  if ((C & 3) == 0) {  // a float4 never crosses a row; 4 vis bytes in two aligned u16 reads
    const int n4 = RC / 4, c4 = C / 4;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(o, (short)0, 12 * RC, 0x00020000);
    const int pol = p.obs_store;
    // the first half of the block writes channels 0 and 2, the second half channel 1
    constexpr int H = NT / 2;
    if (t < H) {
      const int qs = solver >> 2, qv = vault >> 2;
      for (int q = t; q < n4; q += H) {
        const uint32_t b = *reinterpret_cast<const uint32_t*>(L.grid + 4 * q);
        // float32(tile) / 5 == float32(tile) * 0.2f for every tile type 0..7 (checked), and the
        // byte -> float conversion is one v_cvt_f32_ubyteN
        obs_put(rs, pol, 16 * q,
                make_float4((float)(b & 0xff) * 0.2f, (float)((b >> 8) & 0xff) * 0.2f,
                            (float)((b >> 16) & 0xff) * 0.2f, (float)(b >> 24) * 0.2f));
        float4 v = reinterpret_cast<const float4*>(p.plane0)[q];  // the handle's static plane (L2-resident)
        if (q == qs) patch4(v, solver & 3, sv);          // only the solver's and the vault's
        if (q == qv) patch4(v, vault & 3, p.vault_val);  // float4 take these branches
        obs_put(rs, pol, 16 * (2 * n4 + q), v);
      }
    } else {
      for (int q = t - H; q < n4; q += H) {
        const int r = q / c4, c0 = 4 * (q - r * c4);
        const int a = L.at(r, c0);
        uint32_t v;
        if ((kRing & 3) == 0) {
          v = *reinterpret_cast<const uint32_t*>(L.vis + a);
        } else {
          const uint16_t* vp2 = reinterpret_cast<const uint16_t*>(L.vis + a);
          v = (uint32_t)vp2[0] | ((uint32_t)vp2[1] << 16);
        }
        v |= cone_vis4(L, mc, mg, cset, r, c0);
        // visibility bytes are 0 or 1, so they convert directly
        obs_put(rs, pol, 16 * (n4 + q),
                make_float4((float)(v & 0xff), (float)((v >> 8) & 0xff), (float)((v >> 16) & 0xff), (float)(v >> 24)));
      }
    }
  } else {
    for (int q = t; q < 3 * RC; q += NT) {
      const int ch = q / RC;
      const int cell = q - ch * RC;
      float v;
      if (ch == 0) {
        v = p.tile_lut[L.grid[cell] & 7];
      } else if (ch == 1) {
        const int r = cell / C, c = cell - r * C;
        v = (L.vis[L.at(r, c)] | (cone_vis4(L, mc, mg, cset, r, c) & 1u)) ? 1.0f : 0.0f;
      } else {
        v = cell == vault ? p.vault_val : (cell == solver ? sv : p.plane0[cell]);
      }
      o[q] = v;
    }
  }
}

// Step kernel, C % 4 == 0 and two or more waves: the observation in two halves.
// (1) write_obs_static: channel 0 and channel 2 without the solver cell depend on nothing
// this tick computes, so the waves other than wave 0 store them while wave 0 updates the
// emitters (they would otherwise idle at the raycast barrier).  Quad q (4 cells) belongs
// to thread 64 + q % (NT - 64), which reads its grid dword from global memory (L2: the
// prefetch just loaded it; L.grid is not yet visible across waves).
template <int NT>
__device__ __forceinline__ void write_obs_static(const EnvParams& p, int e, float* __restrict__ obs) {
  constexpr int PW = NT > 64 ? NT - 64 : 1;  // NT = 64: never called (split needs two waves)
  const int t = (int)threadIdx.x - 64;
  if (t < 0) return;
  const int RC = p.RC, n4 = RC / 4;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(obs + (size_t)e * 3 * RC, (short)0, 12 * RC, 0x00020000);
  // Both loads go through buffer descriptors sized to their object (the env's grid row,
  // the handle's R*C position plane): the hardware range check returns 0 for an offset past
  // num_records instead of touching memory, so no index here can fault whatever the
  // compiler schedules (the round-2 r02bn fault).
  const __amdgpu_buffer_rsrc_t gs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p.grid + (size_t)e * RC), (short)0, RC, 0x00020000);
  const __amdgpu_buffer_rsrc_t ps =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.plane0), (short)0, 4 * RC, 0x00020000);
  const int vault = p.vr * p.C + p.vc, qv = vault >> 2;
  const int pol = p.obs_store;
  for (int q = t; q < n4; q += PW) {
    const uint32_t b = __builtin_amdgcn_raw_buffer_load_b32(gs, 4 * q, 0, 0);
    float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ps, 16 * q, 0, 0));
    obs_put(rs, pol, 16 * q,
            make_float4((float)(b & 0xff) * 0.2f, (float)((b >> 8) & 0xff) * 0.2f, (float)((b >> 16) & 0xff) * 0.2f,
                        (float)(b >> 24) * 0.2f));
    if (q == qv) patch4(v, vault & 3, p.vault_val);
    obs_put(rs, pol, 16 * (2 * n4 + q), v);
  }
}

// (2) write_obs_dynamic, after the raycast: channel 1 over all NT threads, and the solver's
// quad of channel 2 stored again by its owner from (1) -- the same thread, so its second
// store lands after its first (program order to one address).
template <int NT>
__device__ __forceinline__ void write_obs_dynamic(const EnvParams& p, int e, const EnvScalars& s, const EnvLds& L,
                                                  int cset, float* __restrict__ obs) {
  constexpr int PW = NT > 64 ? NT - 64 : 1;  // NT = 64: never called (split needs two waves)
  const int t = threadIdx.x;
  const int RC = p.RC, C = p.C, n4 = RC / 4, c4 = C / 4;
  const int mc = p.max_cams, mg = p.max_guards;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(obs + (size_t)e * 3 * RC, (short)0, 12 * RC, 0x00020000);
  const int pol = p.obs_store;
  for (int q = t; q < n4; q += NT) {
    const int r = q / c4, c0 = 4 * (q - r * c4);
    const int a = L.at(r, c0);
    uint32_t v;
    if ((kRing & 3) == 0) {
      v = *reinterpret_cast<const uint32_t*>(L.vis + a);
    } else {
      const uint16_t* vp2 = reinterpret_cast<const uint16_t*>(L.vis + a);
      v = (uint32_t)vp2[0] | ((uint32_t)vp2[1] << 16);
    }
    v |= cone_vis4(L, mc, mg, cset, r, c0);
    obs_put(rs, pol, 16 * (n4 + q),
            make_float4((float)(v & 0xff), (float)((v >> 8) & 0xff), (float)((v >> 16) & 0xff), (float)(v >> 24)));
  }
  const int solver = s.pos_r * C + s.pos_c, qs = solver >> 2;
  if (t >= 64 && qs % PW == t - 64) {
    const int vault = p.vr * C + p.vc;
    float4 v = reinterpret_cast<const float4*>(p.plane0)[qs];
    patch4(v, solver & 3, p.plane1[solver]);
    if (qs == (vault >> 2)) patch4(v, vault & 3, p.vault_val);
    obs_put(rs, pol, 16 * (2 * n4 + qs), v);
  }
}

__device__ __forceinline__ void reset_solver(const EnvParams& p, EnvScalars& s) {  // environment.py:191-202
  s.pos_r = p.sr; s.pos_c = p.sc; s.tick = 0;
  s.done = 0; s.detected = 0; s.vault_reached = 0;
  s.prev_dist = s.initial_dist = iabs_(p.sr - p.vr) + iabs_(p.sc - p.vc);
}

__device__ __forceinline__ double guard_heading_after(const EnvParams& p, int dr, int dc, double cur) {
  if (dr == 0 && dc == 0) return cur;  // security.py:158: heading only changes if it moved
  if (dc == 0) return dr < 0 ? p.axis_heading[0] : p.axis_heading[1];
  if (dr == 0) return dc < 0 ? p.axis_heading[2] : p.axis_heading[3];
  return p.heading_tab[(dr + p.R - 1) * (2 * p.C - 1) + (dc + p.C - 1)];
}

// ---------------------------------------------------------------------------
// step / reset
// ---------------------------------------------------------------------------

// Phase stamps (instrumentation, heist_step_stamps): lane 0 of every wave records the
// shader clock at phase boundaries k = 0..7 into stamps[env][wave][k] (10 slots per wave).
// Slot 8 holds HW_ID (CU / SIMD / SE of the wave) and slot 9 XCC_ID, so that clocks are
// compared per CU (the counter is not synchronised across CUs).
#define HEIST_STEP_STAMP(k)                                                                    \
  do {                                                                                         \
    if (STAMP && (threadIdx.x & 63) == 0)                                                      \
      p.stamps[((size_t)e * W + (threadIdx.x >> 6)) * 10 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// COUNT: the counting variant (heist_count_samples / heist_count_redo armed), a kernel of
// its own so profiles of the plain step are not mixed with it.  PROBE: the profiling
// variant that reads EnvParams::probe_mode (HEIST_PROBE_MODE: phases skipped, results
// wrong); the product kernel is compiled with PROBE = false, where every probe test folds
// away, and launch_step only selects the PROBE variant when probe_mode != 0.
template <int W, int U, int O, int D, bool STAMP, bool COUNT, bool PROBE = false>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(O))) void step_kernel(EnvParams p, const int64_t* __restrict__ actions,
                                                       float* __restrict__ obs, float* __restrict__ rew,
                                                       double* __restrict__ rew64, uint8_t* __restrict__ done_out,
                                                       int8_t* __restrict__ status_out, int auto_reset) {
  constexpr int NT = 64 * W;
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = block_env(p);
  const int t = threadIdx.x;
  const int probe = PROBE ? p.probe_mode : 0;
  if (probe == 6) return;  // profiling: launch + dispatch floor
  HEIST_STEP_STAMP(0);
  if (STAMP && (t & 63) == 0) {
    unsigned long long* q = p.stamps + ((size_t)e * W + (t >> 6)) * 10;
    q[8] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    q[9] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  }
  const EnvLds L = carve<D>(smem, p.R, p.C, p.max_cams + p.max_guards, 0, W, p.max_guards);
  const EnvBase eb = env_base(p, e);
  EmitterRaw raw;
  prefetch<NT>(p, e, eb, L, raw);
  if (t == 0) L.meta[5] = 0;  // guards off their patrol start after this tick: bit 0 live, bit 1 cached
  EnvScalars s = p.scal[e];
  const int mc = p.max_cams, n_slot = p.max_cams + p.max_guards;  // emitter slots: cameras, then guards
  const bool live_cam = t < s.n_cams, live_guard = t >= mc && t - mc < s.n_guards;
  const bool act = !s.done;
  const int a_raw = (int)actions[e];
  clear_vis<NT>(p, L);
  if (probe == 8) return;  // profiling: prefetch issue + plane clears only
  HEIST_STEP_STAMP(1);
  // One barrier before the raycast: the emitter slots all live in wave 0, whose lanes
  // update them from their records alone (a guard's next patrol point and its cached
  // cone come straight from HBM, not from LDS), so nothing before it reads another
  // wave's LDS writes; the solver's move, which reads the LDS grid, follows the raycast.
  // 2. cameras rotate, guards patrol (security.py:49-51, :145-159) -- in registers
  uint16_t pos0 = 0;  // a guard thread's patrol start, for the auto-reset below
  bool off_start = false;  // a guard thread's guard stands off its patrol start
  uint8_t gslot = kUncached;  // a guard thread's heading slot after this tick (cached cones)
  Emit E;
  E.kind = -1;  // an empty slot
  if (live_cam) {
    Cam cm = as_cam(raw);
    if (act) {
      cm.heading = py_mod360(cm.heading + cm.speed * 1.0);
      eb.cams[(uint32_t)t].heading = cm.heading;
    }
    E = cam_emit(cm);
  } else if (live_guard) {
    const int g = t - mc;
    Guard gd = as_guard(raw);
    pos0 = gd.pos0;
    const bool moves = act && gd.len >= 2;
    int nidx = gd.idx;
    if (moves) {
      nidx += gd.step;
      if (nidx >= gd.len) nidx -= gd.len;
    }
    // a cached guard: the cone entry of the pose after the move (which names that pose: patrol
    // point and heading) and the cone an auto-reset would give (patrol point 0, the same
    // heading), loaded together straight from the record; a live-raycast guard: the next
    // patrol point, then its heading from the (dr, dc) table
    const bool cached = gd.hslot != kUncached;
    uint16_t np = gd.pos;
    if (moves && !cached) np = eb.paths[__umul24((uint32_t)g, (uint32_t)p.max_path) + (uint32_t)nidx];
    uint4 cm = make_uint4(0u, 0u, 0u, 0u);
    if (cached) {
      const int slot = moves ? gd.nslot : gd.hslot;
      const uint4* src = reinterpret_cast<const uint4*>(eb.cones + cone_off(g, nidx, slot));
      const uint4* rsrc = reinterpret_cast<const uint4*>(eb.cones + cone_off(g, 0, slot));
      const uint4 ca = src[0], cb = src[1], ra = rsrc[0], rb = rsrc[1];
      cm = src[2];
      if (moves) np = (uint16_t)(cm.z & 0xffffu);
      uint4* dst = reinterpret_cast<uint4*>(L.cone + 16 * g);
      uint4* rdst = reinterpret_cast<uint4*>(L.cone + 16 * (p.max_guards + g));
      dst[0] = ca;
      dst[1] = cb;
      rdst[0] = ra;
      rdst[1] = rb;
      L.rpos[g] = pos0;
      if (moves) {  // row 15 of the entry: the slot after the next move
        gd.hslot = gd.nslot;
        gd.nslot = (uint8_t)(cb.w >> 16);
      }
    }
    if (moves) {
      gd.heading = cached ? __builtin_bit_cast(double, ((uint64_t)cm.y << 32) | cm.x)
                          : guard_heading_after(p, unpack_r(np) - unpack_r(gd.pos), unpack_c(np) - unpack_c(gd.pos),
                                                gd.heading);
      gd.idx = (int16_t)nidx;
      gd.pos = np;
      Guard* gp = eb.guards + (uint32_t)g;
      gp->heading = gd.heading;
      gp->idx = gd.idx;
      gp->pos = gd.pos;
      if (gd.hslot != kUncached) {
        gp->hslot = gd.hslot;
        gp->nslot = gd.nslot;
      }
    }
    gslot = gd.hslot;
    off_start = gd.pos != pos0;
    if (off_start) atomicOr(reinterpret_cast<unsigned int*>(&L.meta[5]), gslot == kUncached ? 1u : 2u);
    E = guard_emit(gd);
  }
  constexpr bool kSplitObs = NT >= 128;  // the observation in two halves (write_obs_static)
  const bool split_obs = kSplitObs && p.split_obs && (p.C & 3) == 0 && probe < 4;
  if (split_obs) write_obs_static<NT>(p, e, obs);
  publish_emitters(L, E, n_slot);
  if (probe == 9) return;  // profiling: everything before the raycast barrier
  HEIST_STEP_STAMP(2);
  // 3. visibility (environment.py:257-258); an already-done env recomputes the same plane
  raycast_pass<NT, U, D, COUNT ? 1 : 0>(p, e, smem, L, n_slot, mc, probe);
  if (probe == 7) return;  // profiling: everything up to the raycast
  HEIST_STEP_STAMP(3);

  double reward = 0.0;
  int status = kAlreadyDone;
  if (act) {
    // 1. move (environment.py:239-246): only reward and observation depend on it
    const int a = (a_raw < 0 || a_raw > 4) ? 0 : a_raw;
    // environment.py:52-58: 0 stay, 1 up, 2 down, 3 left, 4 right
    const int nr = s.pos_r + (a == 1 ? -1 : (a == 2 ? 1 : 0)), nc = s.pos_c + (a == 3 ? -1 : (a == 4 ? 1 : 0));
    if (nr >= 0 && nr < p.R && nc >= 0 && nc < p.C && L.grid[nr * p.C + nc] != kWall) {
      s.pos_r = nr;
      s.pos_c = nc;
    }
  }
  if (act) {
    // 4-5. shaping, detection, vault, timeout (environment.py:235, :261-297).  The float64
    // reward is only stored by thread 0, so only wave 0 evaluates it (a wave-uniform branch
    // around each term); every wave needs the integer outcome (done, status) for the
    // auto-reset and the observation.
    const bool rw = (threadIdx.x >> 6) == 0;
    status = kRunning;
    const int curr = iabs_(s.pos_r - p.vr) + iabs_(s.pos_c - p.vc);
    if (rw) {
      reward = p.r_step;
      reward += (double)(s.prev_dist - curr) * 0.1;
      if (curr <= 3 && s.initial_dist > 3) reward += 0.05 * (double)(3 - curr);
    }
    s.prev_dist = curr;
    if (L.vis[L.at(s.pos_r, s.pos_c)] | (cone_vis4(L, p.max_cams, p.max_guards, 0, s.pos_r, s.pos_c) & 1u)) {
      s.detected = 1;
      if (rw) reward += p.r_detect;
      s.done = 1;
      status = kDetected;
    }
    if (s.pos_r == p.vr && s.pos_c == p.vc) {
      s.vault_reached = 1;
      if (rw) reward += p.r_vault;
      s.done = 1;
      status = kVaultReached;
    }
    s.tick += 1;
    if (s.tick >= p.max_steps) {
      s.done = 1;
      status = kTimeout;
      if (rw) {
        double frac = 1.0 - (double)curr / (double)(s.initial_dist > 1 ? s.initial_dist : 1);
        if (frac < 0.0) frac = 0.0;
        reward += frac * 2.0;
      }
    }
  }
  const int done_now = s.done;
  HEIST_STEP_STAMP(4);
  int cset = 0;  // cached guard cones: this tick's
  if (auto_reset && done_now) {  // block-uniform: the barriers inside are safe
    // The reset keeps every heading (environment.py:204-208) and moves only the guards
    // back to patrol point 0, so the camera visibility stays and so does a guard's that
    // stands at its start already.  Cached guards: their reset cones were staged with this
    // tick's (cone set 1, read by write_obs: no barrier, no load); a live-raycast guard off
    // its start forces a full second raycast (rare: guards that do not fit the cone cache).
    const int moved = L.meta[5];  // set by the guard lanes before the raycast barrier
    reset_solver(p, s);
    if (live_guard) {
      const int g = t - mc;
      Guard* gp = eb.guards + (uint32_t)g;
      gp->idx = 0;
      gp->pos = pos0;
      if (gslot != kUncached) gp->nslot = (uint8_t)L.cone[16 * (p.max_guards + g) + 15];  // succ of (0, slot)
    }
    if (moved & 1) {
      __syncthreads();  // every wave's detection read is done
      Emit E2;
      if (t < n_slot) E2 = L.em[t];  // this tick's headings, fov and range stay
      if (live_guard) {
        E2.row = unpack_r(pos0);
        E2.col = unpack_c(pos0);
        if (gslot != kUncached) {
          uint4* dst = reinterpret_cast<uint4*>(L.cone + 16 * (t - mc));
          const uint4* srcr = reinterpret_cast<const uint4*>(L.cone + 16 * (p.max_guards + t - mc));
          dst[0] = srcr[0];
          dst[1] = srcr[1];
        }
      }
      publish_emitters(L, E2, n_slot);
      clear_vis<NT>(p, L);
      raycast_pass<NT, U, D, COUNT ? 1 : 0>(p, e, smem, L, n_slot, mc, probe);
    } else if (moved & 2) {
      cset = 1;
    }
  }
  HEIST_STEP_STAMP(5);
  if (split_obs) write_obs_dynamic<NT>(p, e, s, L, cset, obs);
  else if (probe < 4) write_obs<NT>(p, e, s, L, cset, obs);
  HEIST_STEP_STAMP(6);
  if (t == 0) {
    rew[e] = (float)reward;
    if (rew64) rew64[e] = reward;
    done_out[e] = (uint8_t)done_now;
    status_out[e] = (int8_t)status;
    p.scal[e] = s;
  }
  HEIST_STEP_STAMP(7);
}

// ---------------------------------------------------------------------------
// K ticks per launch (heist_step_multi)
// ---------------------------------------------------------------------------

// The shared camera fan table (FanTick), block k = table entry k: the first camera of the
// first env with a camera (env 0's, in practice) after
// k + 1 rotations from its heading when the filling launch starts (security.py:49-51, every
// tick acting; heist_step_multi fills kFanTicks entries and later launches read them at
// their offset fan_base), its emitter as
// cam_emit forms it, and rays 0 .. num_rays through the same fast-path functions as
// cast_rays (fast_dir, near_tie_key): the near-tie rays, and one ray per run of equal dedup
// keys (a ray is kept when its key differs from the previous ray's, as cast_rays keeps it
// when it differs from the previous lane's).  Runs on the launch's stream before the K-tick
// kernel of a filling launch; a tick without a table (no camera in env 0, range > 6, too
// many rays, exact-only mode) gets n_uniq = -1.
__global__ __launch_bounds__(kFanRays) void fan_kernel(EnvParams p) {
  FanTick* F = p.fan + blockIdx.x;
  const int t = threadIdx.x;
  // the source camera: the first camera of the first env that has one
  __shared__ int src;
  if (t == 0) src = 0x7fffffff;
  __syncthreads();
  for (int b0 = 0; b0 < p.n_envs; b0 += kFanRays) {
    const int e = b0 + t;
    if (e < p.n_envs && p.max_cams > 0 && p.scal[e].n_cams > 0) atomicMin(&src, e);
    __syncthreads();
    if (src != 0x7fffffff) break;
  }
  const bool found = src != 0x7fffffff;
  Cam cm = p.cams[found ? (size_t)src * p.max_cams : 0];
  const bool ok = found && p.ray_mode == 0 && cm.range <= kTieMaxRange && cm.num_rays >= 0 && cm.num_rays < kFanRays;
  if (!ok) {
    if (t == 0) F->n_uniq = -1;
    return;
  }
  double h = cm.heading;
  for (int j = 0; j <= (int)blockIdx.x; ++j) h = py_mod360(h + cm.speed * 1.0);
  cm.heading = h;
  const Emit E = cam_emit(cm);
  const bool active = t <= E.num_rays;
  float cf, sf, xr;
  fast_dir(__builtin_fma((double)t, E.step, E.hmh), &cf, &sf, &xr);
  uint32_t key = 0;
  const bool tie = active && near_tie_key(cf, sf, xr, true, &kTieBuckets_, &key);
  const uint32_t mine = (active && !tie) ? key : 0xFFFFFFFFu;
  __shared__ uint32_t last[kFanRays / 64];
  __shared__ int nf[kFanRays / 64], nt[kFanRays / 64];
  if ((t & 63) == 63) last[t >> 6] = mine;
  uint32_t prev = (uint32_t)__shfl_up((int)mine, 1, 64);
  const unsigned long long bt = __ballot(tie);
  __syncthreads();
  if ((t & 63) == 0 && t > 0) prev = last[(t >> 6) - 1];
  const bool fresh = active && !tie && (t == 0 || prev != mine);
  const unsigned long long bf = __ballot(fresh);
  if ((t & 63) == 0) {
    nf[t >> 6] = __popcll(bf);
    nt[t >> 6] = __popcll(bt);
  }
  __syncthreads();
  int of = 0, ot = 0, tf = 0, tt = 0;
  for (int w = 0; w < kFanRays / 64; ++w) {
    if (w < (t >> 6)) {
      of += nf[w];
      ot += nt[w];
    }
    tf += nf[w];
    tt += nt[w];
  }
  of += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bf >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bf, 0u));
  ot += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bt >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bt, 0u));
  if (fresh) {
    const float dxs = below_one(cf) * 0.5f, dys = -below_one(sf) * 0.5f;  // camera sample stride: half tiles
    F->uniq[2 * of] = dxs;
    F->uniq[2 * of + 1] = dys;
    // the march's tiles relative to the emitter (FanTick::off4/off2): k * d is exact in fp64 and
    // no sample is a .5 tie (the screen), so rint here is the fma's rounding in march_fast
    const int PCf = p.C + 2 * kRing;
    uint32_t w[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      uint32_t pair = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const double kk = (double)(2 * i + h + 1);
        const int dc = (int)__builtin_rint(kk * (double)dxs), dr = (int)__builtin_rint(kk * (double)dys);
        pair |= (uint32_t)((dr + kRing) * PCf + dc + kRing) << (16 * h);
      }
      w[i] = pair;
    }
    F->off4[of] = make_uint4(w[0], w[1], w[2], w[3]);
    F->off2[of] = make_uint2(w[4], w[5]);
  }
  if (tie) F->tie[ot] = (uint16_t)t;
  if (t == 0) {
    F->hmh = E.hmh;
    F->heading = cm.heading;
    F->speed = cm.speed;
    F->fov = E.fov;
    F->num_rays = E.num_rays;
    F->range = E.range;
    F->n_uniq = tf;
    F->n_tie = tt;
  }
}

// Observation lanes: the threads that store a tick's observation row -- waves 1.. when the
// env has two or more waves (wave 0, which updates the emitters and loads the next cone
// entries, then issues no observation stores: vmcnt counts loads and stores together, in
// issue order, so its wait for a load never waits for them), every lane of the one wave
// otherwise.  LB is the first observation lane, PW their count.
template <int NT>
struct ObsLanes {
  static constexpr int LB = NT > 64 ? 64 : 0;
  static constexpr int PW = NT - LB;
};

// Channels 0 and 2 of observation row `o` (the env's [3][R][C] floats of one tick) except
// the solver's quad: the tile grid from LDS, the handle's static position plane from L2
// (one 1.6 KB plane shared by every env; an LDS copy of it per block cost 1.6 KB of the
// block's LDS, which held the K-tick kernel to 14 resident blocks per CU instead of 16).
// Quad q belongs to observation lane q % PW, which stores the solver's quad again in
// write_obs_ch1_tail (program order to one address).
template <int NT>
__device__ __forceinline__ void write_obs_static_lds(const EnvParams& p, const EnvLds& L, const float* plane,
                                                     float* __restrict__ o) {
  constexpr int PW = ObsLanes<NT>::PW;
  const int t = (int)threadIdx.x - ObsLanes<NT>::LB;
  if (t < 0) return;
  const int RC = p.RC, n4 = RC / 4;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(o, (short)0, 12 * RC, 0x00020000);
  const int vault = p.vr * p.C + p.vc, qv = vault >> 2;
  const int pol = p.obs_store;
  for (int q = t; q < n4; q += PW) {
    const uint32_t b = *reinterpret_cast<const uint32_t*>(L.grid + 4 * q);
    float4 v = reinterpret_cast<const float4*>(plane)[q];
    obs_put(rs, pol, 16 * q,
            make_float4((float)(b & 0xff) * 0.2f, (float)((b >> 8) & 0xff) * 0.2f, (float)((b >> 16) & 0xff) * 0.2f,
                        (float)(b >> 24) * 0.2f));
    if (q == qv) patch4(v, vault & 3, p.vault_val);
    obs_put(rs, pol, 16 * (2 * n4 + q), v);
  }
}

// Channel 1 of observation row `o` (ray plane | guard plane) plus the solver's quad of
// channel 2, by the observation lanes.
template <int NT>
__device__ __forceinline__ void write_obs_ch1_tail(const EnvParams& p, const EnvScalars& s, const EnvLds& L,
                                                   const uint8_t* gvis, float* __restrict__ o) {
  constexpr int PW = ObsLanes<NT>::PW;
  const int t = (int)threadIdx.x - ObsLanes<NT>::LB;
  if (t < 0) return;
  const int RC = p.RC, C = p.C, n4 = RC / 4, c4 = C / 4;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(o, (short)0, 12 * RC, 0x00020000);
  const int pol = p.obs_store;
  static_assert((kRing & 1) == 0, "padded vis rows of a C % 4 == 0 grid are 2-byte aligned");
  for (int q = t; q < n4; q += PW) {
    const int r = q / c4, c0 = 4 * (q - r * c4);
    const int a = L.at(r, c0);
    uint32_t v;
    if ((kRing & 3) == 0) {
      v = *reinterpret_cast<const uint32_t*>(L.vis + a) | *reinterpret_cast<const uint32_t*>(gvis + a);
    } else {
      const uint16_t* vp2 = reinterpret_cast<const uint16_t*>(L.vis + a);
      const uint16_t* gp2 = reinterpret_cast<const uint16_t*>(gvis + a);
      v = ((uint32_t)vp2[0] | ((uint32_t)vp2[1] << 16)) | ((uint32_t)gp2[0] | ((uint32_t)gp2[1] << 16));
    }
    obs_put(rs, pol, 16 * (n4 + q),
            make_float4((float)(v & 0xff), (float)((v >> 8) & 0xff), (float)((v >> 16) & 0xff), (float)(v >> 24)));
  }
  const int solver = s.pos_r * C + s.pos_c, qs = solver >> 2;
  if (qs % PW == t) {
    const int vault = p.vr * C + p.vc;
    float4 v = reinterpret_cast<const float4*>(p.plane0)[qs];
    patch4(v, solver & 3, p.plane1[solver]);
    if (qs == (vault >> 2)) patch4(v, vault & 3, p.vault_val);
    obs_put(rs, pol, 16 * (2 * n4 + qs), v);
  }
}

// One-wave K-tick kernel (SOLO): the lane's observation quads q = lane + 64 j (j < kObsQ) keep
// what does not change within a launch in registers -- channel 0 (tile / 5) and channel 2
// (the static plane, vault patched) as float4, and the LDS offset of the quad's 4 visibility
// bytes -- so a tick's observation is 2 stores per quad from registers plus one LDS read and
// 4 conversions for channel 1.  Loading the plane and converting the grid every tick cost
// VALU, and the loop's in-order vmcnt made each iteration wait for the previous stores.
constexpr int kObsQ = 2;  // quads per lane: R * C <= 4 * 64 * kObsQ (20 x 20: 100 quads)
struct ObsRegs {
  float4 ch0[kObsQ], ch2[kObsQ];
  int vis[kObsQ];
};
__device__ __forceinline__ void obs_regs_init(const EnvParams& p, const EnvLds& L, ObsRegs& R) {
  const int lane = threadIdx.x & 63, n4 = p.RC / 4, c4 = p.C / 4;
  const int vault = p.vr * p.C + p.vc, qv = vault >> 2;
#pragma unroll
  for (int j = 0; j < kObsQ; ++j) {
    const int q = lane + 64 * j;
    const int qc = q < n4 ? q : n4 - 1;
    const uint32_t b = *reinterpret_cast<const uint32_t*>(L.grid + 4 * qc);
    R.ch0[j] = make_float4((float)(b & 0xff) * 0.2f, (float)((b >> 8) & 0xff) * 0.2f, (float)((b >> 16) & 0xff) * 0.2f,
                           (float)(b >> 24) * 0.2f);
    float4 v = reinterpret_cast<const float4*>(p.plane0)[qc];
    if (qc == qv) patch4(v, vault & 3, p.vault_val);
    R.ch2[j] = v;
    const int r = qc / c4;
    R.vis[j] = L.at(r, 4 * (qc - r * c4));
  }
}
// The tick's observation row o from ObsRegs: channels 0 and 2 (static part) when STATIC,
// else channel 1 (ray plane | guard plane) and the solver's quad of channel 2.
template <bool STATIC>
__device__ __forceinline__ void write_obs_regs(const EnvParams& p, const EnvScalars& s, const EnvLds& L,
                                               const uint8_t* gvis, const ObsRegs& R, float* __restrict__ o) {
  const int lane = threadIdx.x & 63, n4 = p.RC / 4;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(o, (short)0, 12 * p.RC, 0x00020000);
  auto body = [&](auto pol) {
    constexpr int P = decltype(pol)::value;
#pragma unroll
    for (int j = 0; j < kObsQ; ++j) {
      const int q = lane + 64 * j;
      if (q >= n4) break;
      if constexpr (STATIC) {
        obs_put(rs, P, 16 * q, R.ch0[j]);
        obs_put(rs, P, 16 * (2 * n4 + q), R.ch2[j]);
      } else {
        uint32_t v;
        if ((kRing & 3) == 0) {
          v = *reinterpret_cast<const uint32_t*>(L.vis + R.vis[j]) | *reinterpret_cast<const uint32_t*>(gvis + R.vis[j]);
        } else {
          const uint16_t* vp2 = reinterpret_cast<const uint16_t*>(L.vis + R.vis[j]);
          const uint16_t* gp2 = reinterpret_cast<const uint16_t*>(gvis + R.vis[j]);
          v = ((uint32_t)vp2[0] | ((uint32_t)vp2[1] << 16)) | ((uint32_t)gp2[0] | ((uint32_t)gp2[1] << 16));
        }
        obs_put(rs, P, 16 * (n4 + q),
                make_float4((float)(v & 0xff), (float)((v >> 8) & 0xff), (float)((v >> 16) & 0xff), (float)(v >> 24)));
      }
    }
    if constexpr (!STATIC) {
      const int solver = s.pos_r * p.C + s.pos_c, qs = solver >> 2;
      if ((qs & 63) == lane) {
        const int vault = p.vr * p.C + p.vc;
        float4 v = reinterpret_cast<const float4*>(p.plane0)[qs];
        patch4(v, solver & 3, p.plane1[solver]);
        if (qs == (vault >> 2)) patch4(v, vault & 3, p.vault_val);
        obs_put(rs, P, 16 * (2 * n4 + qs), v);
      }
    }
  };
  // the store policy is a launch constant: one branch here instead of one per store
  switch (p.obs_store) {
    case 1: body(std::integral_constant<int, 1>{}); break;
    case 2: body(std::integral_constant<int, 2>{}); break;
    case 3: body(std::integral_constant<int, 3>{}); break;
    default: body(std::integral_constant<int, 0>{}); break;
  }
}

// The ray plane and the guard plane zeroed by the observation lanes.
template <int NT>
__device__ __forceinline__ void clear_planes(const EnvParams& p, const EnvLds& L, uint8_t* gvis, bool rays) {
  constexpr int PW = ObsLanes<NT>::PW;
  const int t = (int)threadIdx.x - ObsLanes<NT>::LB;
  // 16-byte stores: both planes are 16-byte aligned and D >= the padded size rounded to 16
  uint4* v16 = reinterpret_cast<uint4*>(L.vis);
  uint4* g16 = reinterpret_cast<uint4*>(gvis);
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  for (int i = t; i >= 0 && i < (padded_bytes(p.R, p.C) + 15) / 16; i += PW) {
    if (rays) v16[i] = z;
    g16[i] = z;
  }
}

// The cached guard cones of cone set `set` (the kind-2 emitter slots of meta[6..7]; set 0:
// this tick's poses from the emitter table, set 1: the auto-reset poses, patrol point 0)
// stamped into the guard plane gvis (the vis geometry, cleared each tick) by the
// observation lanes: lane 15 i + j writes row j of cone i (mod the PW / 15 cones per
// pass), one byte per visible tile.  A cone names in-grid tiles only (guard_cone_kernel),
// so every write lands on the grid.
template <int NT>
__device__ __forceinline__ void stamp_guard_cones(const EnvLds& L, uint8_t* gvis, int mc, int mg, int set) {
  constexpr int G = ObsLanes<NT>::PW / 15;  // cones per pass
  const int l = (int)threadIdx.x - ObsLanes<NT>::LB;
  const int grp = l / 15, j = l - 15 * grp;
  if (l < 0 || grp >= G) return;
  uint64_t m = ((uint64_t)(uint32_t)uni(L.meta[7]) << 32) | (uint32_t)uni(L.meta[6]);
  for (int c = 0; m; ++c) {
    const int k = (int)__builtin_ctzll(m);
    m &= m - 1;
    if (c % G != grp) continue;
    const int g = k - mc;
    int gr, gc;
    if (set) {
      const int rp = (int)L.rpos[g];
      gr = unpack_r(rp);
      gc = unpack_c(rp);
    } else {
      gr = L.em[k].row;
      gc = L.em[k].col;
    }
    const uint32_t bits = L.cone[16 * (set * mg + g) + j] & 0x7fffu;
    uint8_t* row = gvis + L.off0 + (gr + j - kConeRange) * L.PC + (gc - kConeRange);
    for (uint32_t b = bits; b; b &= b - 1) row[__builtin_ctz(b)] = 1;
  }
}

// K consecutive heist_step ticks of one env per workgroup (environment.py:216-299 and
// :347-374 K times), with actions[k][env] known up front: what env-only throughput and
// action replay need.  The per-env state stays on chip for the whole launch -- grid, stop
// map, patrol paths, the emitter records and the K actions in LDS (the static position
// plane, one for the handle, is read from L2), the solver scalars in scalar registers -- and is written back once at the end;
// every tick still writes its full observation row (obs[k][env], non-temporal 16-byte
// stores), reward, done and status.  Per tick:
//   A  every thread: the solver's move and the reward terms that precede detection
//      (environment.py:235-269; they need the grid, not the visibility); wave 0: cameras
//      and guards advance (security.py:49-51, :145-159) and the emitter table is
//      published; observation lanes: the tick's static channels 0 and 2, the plane clears;
//   barrier, raycast (all waves), the cached guards' cones stamped into the guard plane
//      by the observation lanes (their raycast share is the smaller one), barrier;
//   C  every thread: detection (ray plane | guard plane), vault, timeout, auto-reset
//      (environment.py:271-297, :183-214); wave 0: the next tick's cone entries are
//      loaded, reward / done / status stored; observation lanes: channel 1.
// The cone entry a cached guard needs at tick k + 1 is loaded at the end of tick k and
// lands in LDS at tick k + 1 (phase A with two or more waves; after the raycast with one,
// where the entry has had the whole raycast to arrive and the wait for it is not held up
// by the observation stores issued since).  A finishing env loads its cached guards'
// reset cones (patrol point 0, same heading) then; a live-raycast guard off its start
// costs a second raycast pass from the reset poses.  A cached guard's heading is the one
// its slot names: read from a cone entry once, at the end.  Results are bit-identical to
// K heist_step launches (tests/test_gpu_env.py).
// PROBE (profiling variant, HEIST_PROBE_MODE at heist_create; results wrong on purpose):
// bit 0 skips the raycast and the cone stamps, bit 1 the observation stores, bit 2 the
// rays' marches (directions and tie screens only).
template <int W, int U, int O, int D, bool STAMP = false, int PROBE = 0>
__device__ __forceinline__ void step_multi_body(
    const EnvParams& p, int K, const int64_t* __restrict__ actions, float* __restrict__ obs, float* __restrict__ rew,
    double* __restrict__ rew64, uint8_t* __restrict__ done_out, int8_t* __restrict__ status_out, int auto_reset,
    unsigned char* smem, int e) {
  constexpr int NT = 64 * W;
  constexpr bool SOLO = W == 1;  // one wave does every role
  const int t = threadIdx.x;
  const bool w0 = (t >> 6) == 0;
  const int RC = p.RC, N = p.n_envs;
  const int mc = p.max_cams, mg = p.max_guards, n_slot = mc + mg;
  const int path_words = mg * p.max_path;
  const EnvLds L = carve<D>(smem, p.R, p.C, n_slot, path_words, W, mg);
  const float* plane = p.plane0;  // static position plane (L2)
  EmitterRaw* rec = reinterpret_cast<EmitterRaw*>(
      smem + align16(env_lds_bytes(p.R, p.C, n_slot, path_words, D, W, mg)));  // [n_slot] records
  uint8_t* act = reinterpret_cast<uint8_t*>(rec + n_slot);
  uint8_t* gvis = act + align16((size_t)K);  // cached guard cones of the tick, vis geometry (stamp_guard_cones)
  const EnvBase eb = env_base(p, e);
  // STAMP (instrumentation, heist_step_stamps): lane 0 of every wave sums the shader clock
  // spent in each of 9 tick segments over the launch into LDS, and writes [segment sums
  // 0..8, lifetime, start clock, HW_ID, XCC_ID] to stamps[env][wave][16]
  TieBuckets* tb = reinterpret_cast<TieBuckets*>(gvis + D);  // the tie screen's tables (868 B)
  float2* uq = reinterpret_cast<float2*>(reinterpret_cast<unsigned char*>(tb) + align16(sizeof(TieBuckets)));
  unsigned long long* st_acc = reinterpret_cast<unsigned long long*>(uq + 128 * W);  // after the unique queues
  unsigned long long st_last = 0, st_start = 0;
  if (STAMP && (t & 63) == 0) {
    st_start = st_last = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < 9; ++j) st_acc[(t >> 6) * 10 + j] = 0;
  }
#define HEIST_MULTI_STAMP(seg)                                                  \
  do {                                                                          \
    if (STAMP && (threadIdx.x & 63) == 0) {                                     \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();             \
      st_acc[(threadIdx.x >> 6) * 10 + (seg)] += now_ - st_last;                \
      st_last = now_;                                                           \
    }                                                                           \
  } while (0)

  // prologue: the env's layout and state, once per launch
  {
    EmitterRaw raw;
    prefetch<NT>(p, e, eb, L, raw);
    if (t < n_slot) rec[t] = raw;
  }
  for (int i = t; i < path_words; i += NT) L.path[i] = eb.paths[i];
  for (int i = t; i < (int)sizeof(TieBuckets) / 4; i += NT)
    reinterpret_cast<uint32_t*>(tb)[i] = reinterpret_cast<const uint32_t*>(&kTieBuckets_)[i];
  for (int k = t; k < K; k += NT) {
    const int64_t a = actions[(size_t)k * N + e];
    act[k] = (uint8_t)((a < 0 || a > 4) ? 0 : a);  // unknown actions do not move (environment.py:239)
  }
  EnvScalars s = p.scal[e];
  const int g = t - mc;
  const bool live_cam = t < s.n_cams, live_guard = g >= 0 && g < s.n_guards;
  bool cached = false;
  // one wave per env: the observation's per-launch constants in registers (ObsRegs)
  const bool reg_obs = SOLO && p.RC <= 256 * kObsQ;
  ObsRegs obr;
  // a cached guard's cone entry for the coming tick, loaded one tick ahead: the pose after
  // its move (idx + step, nslot) if the env acts and the patrol has >= 2 points
  // (security.py:147), else the pose it holds
  uint4 ca = make_uint4(0u, 0u, 0u, 0u), cb = ca;
  auto next_entry = [&](const Guard& gd, bool acts) {
    int idx = gd.idx, slot = gd.hslot;
    if (acts && gd.len >= 2) {
      idx += gd.step;
      if (idx >= gd.len) idx -= gd.len;
      slot = gd.nslot;
    }
    const uint4* src = reinterpret_cast<const uint4*>(eb.cones + cone_off(g, idx, slot));
    ca = src[0];
    cb = src[1];
  };
  // the entry's cone rows into LDS (cone set 0) and the slot after the guard's next move
  auto take_entry = [&]() {
    Guard gd = as_guard(rec[t]);
    gd.nslot = (uint8_t)(cb.w >> 16);  // row 15
    rec[t] = __builtin_bit_cast(EmitterRaw, gd);
    uint4* dst = reinterpret_cast<uint4*>(L.cone + 16 * g);
    dst[0] = ca;
    dst[1] = cb;
  };
  __syncthreads();  // records in LDS
  if (SOLO && reg_obs) obs_regs_init(p, L, obr);
  if (live_guard) {
    const Guard gd = as_guard(rec[t]);
    cached = gd.hslot != kUncached;
    L.rpos[g] = gd.pos0;
    if (cached) next_entry(gd, !s.done);
  }

  // Tick k is one or two raycast passes: pass 0 the tick itself; pass 1 only when the env
  // finishes, auto-resets and a live-raycast guard stood off its patrol start (the reset
  // observation needs the cone from patrol point 0).  One raycast instance in the loop.
  int k = 0;
  bool reset_pass = false;
  double reward = 0.0;
  int status = kAlreadyDone, done_now = 0;
  bool act_now = true;
  int curr = 0;
  FanHdr fhdr{0.0, 0.0, 0, 0, -1, 0, {0.0f, 0.0f}};  // this tick's shared fan (FanTick), -1: none
  while (k < K) {
    __syncthreads();  // the previous pass's readers of vis / em / meta / cones are done
    HEIST_MULTI_STAMP(8);  // 8: end of the previous tick -> through the top barrier
    if (p.fan_on && PROBE == 0 && !reset_pass) fhdr = fan_hdr(p.fan + p.fan_base + k);  // lands during phase A
    Emit E;
    E.kind = -1;
    if (!reset_pass) {
      act_now = !s.done;
      reward = 0.0;
      status = kAlreadyDone;
      if (act_now) {
        // 1. move (environment.py:239-246): needs the grid, not this tick's visibility
        const int a = act[k];
        const int nr = s.pos_r + (a == 1 ? -1 : (a == 2 ? 1 : 0)), nc = s.pos_c + (a == 3 ? -1 : (a == 4 ? 1 : 0));
        if (nr >= 0 && nr < p.R && nc >= 0 && nc < p.C && L.grid[nr * p.C + nc] != kWall) {
          s.pos_r = nr;
          s.pos_c = nc;
        }
        s.pos_r = uni(s.pos_r);
        s.pos_c = uni(s.pos_c);
        // 4. shaping and proximity (environment.py:235, :261-269); the float64 reward on
        // wave 0 only (thread 0 stores it); detection, vault and timeout follow the raycast
        status = kRunning;
        curr = iabs_(s.pos_r - p.vr) + iabs_(s.pos_c - p.vc);
        if (w0) {
          reward = p.r_step;
          reward += (double)(s.prev_dist - curr) * 0.1;
          if (curr <= 3 && s.initial_dist > 3) reward += 0.05 * (double)(3 - curr);
        }
        s.prev_dist = curr;
      }
      HEIST_MULTI_STAMP(0);  // 0: the solver's move, shaping reward
      if (w0) {
        if (t == 0) L.meta[5] = 0;
        // 2. cameras rotate, guards patrol (security.py:49-51, :145-159)
        if (live_cam) {
          Cam cm = as_cam(rec[t]);
          if (act_now) {
            cm.heading = py_mod360(cm.heading + cm.speed * 1.0);
            rec[t] = __builtin_bit_cast(EmitterRaw, cm);
          }
          E = cam_emit(cm);
        } else if (live_guard) {
          Guard gd = as_guard(rec[t]);
          const bool moves = act_now && gd.len >= 2;
          int nidx = gd.idx;
          if (moves) {
            nidx += gd.step;
            if (nidx >= gd.len) nidx -= gd.len;
          }
          const uint16_t np = moves ? L.path[__umul24((uint32_t)g, (uint32_t)p.max_path) + (uint32_t)nidx] : gd.pos;
          if (cached) {
            if (moves) gd.hslot = gd.nslot;  // the slot the entry loaded for this tick was taken with
          } else if (moves) {
            gd.heading = guard_heading_after(p, unpack_r(np) - unpack_r(gd.pos), unpack_c(np) - unpack_c(gd.pos),
                                             gd.heading);
          }
          gd.idx = (int16_t)nidx;
          gd.pos = np;
          if (gd.pos != gd.pos0) atomicOr(reinterpret_cast<unsigned int*>(&L.meta[5]), cached ? 2u : 1u);
          rec[t] = __builtin_bit_cast(EmitterRaw, gd);
          E = guard_emit(gd);
          if (cached && !SOLO) take_entry();  // then nslot := the entry's row 15
        }
        HEIST_MULTI_STAMP(1);  // 1: emitter update
        publish_emitters(L, E, n_slot);
      }
      if (!(PROBE & 2)) {
        if (SOLO && reg_obs)
          write_obs_regs<true>(p, s, L, gvis, obr, obs + ((size_t)k * N + e) * 3 * RC);
        else
          write_obs_static_lds<NT>(p, L, plane, obs + ((size_t)k * N + e) * 3 * RC);
      }
      clear_planes<NT>(p, L, gvis, true);
    } else {  // the emitters with every guard back at patrol point 0, headings kept
      if (w0) {
        if (live_cam) E = cam_emit(as_cam(rec[t]));
        if (live_guard) {
          E = guard_emit(as_guard(rec[t]));
          if (cached) {
            uint4* dst = reinterpret_cast<uint4*>(L.cone + 16 * g);
            const uint4* srcr = reinterpret_cast<const uint4*>(L.cone + 16 * (mg + g));
            dst[0] = srcr[0];
            dst[1] = srcr[1];
          }
        }
        publish_emitters(L, E, n_slot);
      }
      clear_planes<NT>(p, L, gvis, true);
    }
    HEIST_MULTI_STAMP(2);  // 2: publish, static channels, clears
    __syncthreads();  // emitter table, cone rows, cleared planes
    HEIST_MULTI_STAMP(3);  // 3: waiting at the raycast barrier
    // 3. visibility (environment.py:257-258)
    if (live_guard && E.kind == 1) L.vis[L.at(E.row, E.col)] = 1;  // visibility.py:59
    if (!(PROBE & 1))
      cast_rays<NT, U, D, false, true>(smem, L, p.ray_mode, (PROBE & 4) ? 2 : 0, p.half_deg, tb, uq,
                                       p.fan + p.fan_base + k, fhdr);
    if (SOLO && cached && !reset_pass) take_entry();  // loaded a tick ago; the raycast covered its latency
    if (!(PROBE & 1)) stamp_guard_cones<NT>(L, gvis, mc, mg, 0);
    HEIST_MULTI_STAMP(4);  // 4: raycast, cone stamps
    __syncthreads();  // planes complete
    HEIST_MULTI_STAMP(5);  // 5: waiting for the other waves' raycast

    if (!reset_pass) {
      if (act_now) {
        // 5. detection, vault, timeout (environment.py:271-297), in the reference's order
        const int at = L.at(s.pos_r, s.pos_c);
        if (L.vis[at] | gvis[at]) {
          s.detected = 1;
          if (w0) reward += p.r_detect;
          s.done = 1;
          status = kDetected;
        }
        if (s.pos_r == p.vr && s.pos_c == p.vc) {
          s.vault_reached = 1;
          if (w0) reward += p.r_vault;
          s.done = 1;
          status = kVaultReached;
        }
        s.tick += 1;
        if (s.tick >= p.max_steps) {
          s.done = 1;
          status = kTimeout;
          if (w0) {
            double frac = 1.0 - (double)curr / (double)(s.initial_dist > 1 ? s.initial_dist : 1);
            if (frac < 0.0) frac = 0.0;
            reward += frac * 2.0;
          }
        }
      }
      s.done = uni(s.done);  // block-uniform state in scalar registers
      s.detected = uni(s.detected);
      s.vault_reached = uni(s.vault_reached);
      s.tick = uni(s.tick);
      done_now = s.done;
      if (auto_reset && done_now) {  // block-uniform: the barriers inside are safe
        // environment.py:183-214: headings kept, guards back to patrol point 0.  A cached
        // guard's reset cone (point 0, this slot) is loaded now -- only finishing envs pay
        // for it -- for channel 1 (cone set 1) and the slot after its next move (row 15)
        const int moved = L.meta[5];
        reset_solver(p, s);
        if (live_guard) {
          Guard gd = as_guard(rec[t]);
          gd.idx = 0;
          gd.pos = gd.pos0;
          if (cached) {
            const uint4* rsrc = reinterpret_cast<const uint4*>(eb.cones + cone_off(g, 0, gd.hslot));
            const uint4 ra = rsrc[0], rb = rsrc[1];
            uint4* rdst = reinterpret_cast<uint4*>(L.cone + 16 * (mg + g));
            rdst[0] = ra;
            rdst[1] = rb;
            gd.nslot = (uint8_t)(rb.w >> 16);
          }
          rec[t] = __builtin_bit_cast(EmitterRaw, gd);
        }
        if (moved & 1) {  // a live-raycast guard off its start: raycast again from the reset poses
          reset_pass = true;
          continue;
        }
        if (moved & 2) {  // cached guards off their start: the guard plane from the reset cones
          __syncthreads();  // the reset cones in LDS; every wave's detection read is done
          clear_planes<NT>(p, L, gvis, false);
          if constexpr (W > 2) __syncthreads();
          stamp_guard_cones<NT>(L, gvis, mc, mg, 1);
          if constexpr (W > 2) __syncthreads();
        }
      }
    }
    reset_pass = false;
    HEIST_MULTI_STAMP(6);  // 6: detection, vault, timeout, auto-reset
    if (w0) {
      if (live_guard && cached && k + 1 < K) next_entry(as_guard(rec[t]), !s.done);  // lands during the next tick
      if (t == 0) {
        const size_t ko = (size_t)k * N + e;
        rew[ko] = (float)reward;
        if (rew64) rew64[ko] = reward;
        done_out[ko] = (uint8_t)done_now;
        status_out[ko] = (int8_t)status;
      }
    }
    if (!(PROBE & 2)) {
      if (SOLO && reg_obs)
        write_obs_regs<false>(p, s, L, gvis, obr, obs + ((size_t)k * N + e) * 3 * RC);
      else
        write_obs_ch1_tail<NT>(p, s, L, gvis, obs + ((size_t)k * N + e) * 3 * RC);
    }
    HEIST_MULTI_STAMP(7);  // 7: outputs, channel 1 + solver quad
    ++k;
  }
#undef HEIST_MULTI_STAMP
  // epilogue: the state the next launch (or heist_export) starts from
  if (t == 0) p.scal[e] = s;
  if (STAMP && (t & 63) == 0) {
    unsigned long long* q = p.stamps + ((size_t)e * W + (t >> 6)) * 16;
    for (int j = 0; j < 9; ++j) q[j] = st_acc[(t >> 6) * 10 + j];
    q[9] = __builtin_amdgcn_s_memtime() - st_start;
    q[10] = st_start;
    q[11] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    q[12] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  }
  if (live_cam) eb.cams[(uint32_t)t].heading = as_cam(rec[t]).heading;
  if (live_guard) {
    Guard gd = as_guard(rec[t]);
    if (cached) {  // the heading its slot names (u16 16..19 of any entry with that slot)
      const uint4 c2 = reinterpret_cast<const uint4*>(eb.cones + cone_off(g, gd.idx, gd.hslot))[2];
      gd.heading = __builtin_bit_cast(double, ((uint64_t)c2.y << 32) | c2.x);
    }
    Guard* gp = eb.guards + (uint32_t)g;
    gp->heading = gd.heading;
    gp->idx = gd.idx;
    gp->pos = gd.pos;
    gp->hslot = gd.hslot;
    gp->nslot = gd.nslot;
  }
}

template <int W, int U, int O, int D, bool STAMP = false, int PROBE = 0>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(O))) void step_multi_kernel(
    EnvParams p, int K, const int64_t* __restrict__ actions, float* __restrict__ obs, float* __restrict__ rew,
    double* __restrict__ rew64, uint8_t* __restrict__ done_out, int8_t* __restrict__ status_out, int auto_reset) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = block_env(p);
  step_multi_body<W, U, O, D, STAMP, PROBE>(p, K, actions, obs, rew, rew64, done_out, status_out, auto_reset, smem, e);
}

// ---------------------------------------------------------------------------
// Lean K-tick kernel (heist_step_multi, one wave per env, grids up to 20 x 20)
// ---------------------------------------------------------------------------
//
// The same K ticks as step_multi_kernel, bit for bit, laid out for the one-wave case so
// that a tick is a short chain of register and LDS work with no wait on global memory:
//   * every per-launch constant in registers: the lane's camera / guard record, the
//     observation's static channels 0 and 2 and its LDS offsets (two quads per lane), the
//     stop map's rows as bit masks (lane r = row r: the solver's wall test is a readlane);
//   * the data the next tick needs from HBM -- the shared fan's header and its unique
//     directions' sample tiles (FanTick::off4/off2), the cached guards' cone entries -- is
//     loaded at the end of the previous tick, BEFORE that tick's channel-1 stores: vmcnt
//     counts loads and stores in issue order, so waiting for a load issued after the stores
//     would wait for the stores to reach memory;
//   * one visibility plane for cameras and guards (the cached cones ORed in with ds_or_b32);
//     detection reads the solver's byte from the channel-1 quads the observation loads
//     anyway; a finishing env whose guards stood off their start re-casts from the reset
//     poses (rare: the reset observation needs the guards at patrol point 0);
//   * a camera group the shared fan serves (every live camera's emitter equals the tick's
//     table entry, no near-tie ray, range 6) marches the table's unique directions from
//     each camera's tile, one address add per sample: the table holds each sample's tile as
//     an offset from the camera's corner tile;
//   * near-tie rays of the fan (rare) are cast on the exact path from each camera;
//   * an env the lean loop cannot serve for the whole launch -- a camera that is not the fan's
//     (heading, speed, fov, rays, range 6 at the launch's first tick: then every tick's
//     camera equals the table's), a live-raycast guard, exact-only mode, an env already
//     finished at the launch's start -- runs the generic K-tick body (step_multi_body) in the
//     same launch, before any lean register is live;
//   * an env that finished without auto-reset is frozen (environment.py:232-233): its plane
//     is kept and only its outputs are written.

// LDS-DMA of 16 bytes per active lane (global_load_lds_dwordx4: lane i's bytes land at
// lds_dst + 16 i), issued as inline asm so that the compiler's vmcnt bookkeeping does not
// see it: the lean kernel waits for these with its own counted s_waitcnt (kStores).  M0
// (the LDS destination base) is set and restored inside the statement.
__device__ __forceinline__ void lds_dma16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

// The exact path (exact_ray) for a shared fan's near-tie rays (FanTick::tie), from every
// camera of the env (camera m's tile in lane m of cam_rc): a call, so that the glibc sin/cos
// restatement's registers stay out of the lean loop (near-tie rays are rare).
template <int D, int PC>
__device__ __noinline__ void lean_tie_rays(unsigned char* smem, const FanTick* f, int n_tie, uint32_t cam_rc, int n_cams,
                                           const double* hd) {
  const int lane = threadIdx.x;
  for (int b0 = 0; b0 < n_tie; b0 += 64) {
    const int tr = b0 + lane < n_tie ? (int)f->tie[b0 + lane] : -1;
    for (int m = 0; m < n_cams; ++m) {
      Emit E;
      E.hmh = f->hmh;
      E.fov = f->fov;
      E.step = 0.0;
      E.range = f->range;
      E.num_rays = f->num_rays;
      const uint32_t rcm = (uint32_t)__builtin_amdgcn_readlane((int)cam_rc, m);
      E.row = (int)(rcm & 0xffu);
      E.col = (int)(rcm >> 8);
      E.first = 0;
      E.kind = 0;
      E.members = 1;
      if (tr >= 0) exact_ray<4, D>(smem, E, tr, PC, 0, hd);
    }
  }
}

// The exact path for an interval fan's near-cut rays: lane i casts ray `ray` (< 0: none) of
// the camera with emitter (hmh, fov, num_rays) at tile rc (row | col << 8).  A call, as
// lean_tie_rays, so that the exact path's registers stay out of the lean loop.
template <int D, int PC>
__device__ __noinline__ void ivl_tie_rays(unsigned char* smem, int ray, double hmh, double fov, int num_rays,
                                          uint32_t rc, const double* hd) {
  Emit E;
  E.hmh = hmh;
  E.fov = fov;
  E.step = 0.0;
  E.range = kTieMaxRange;
  E.num_rays = num_rays;
  E.row = (int)(rc & 0xffu);
  E.col = (int)(rc >> 8);
  E.first = 0;
  E.kind = 0;
  E.members = 1;
  if (ray >= 0) exact_ray<4, D>(smem, E, ray, PC, 0, hd);
}

// The lean kernel's LDS: the three padded planes (stop map, visibility, sink; the step
// kernels' geometry, so exact_ray works on them), the tile grid, the patrol paths, the
// launch's K actions, the LDS-DMA staging of the next tick's HBM data (LeanStage), the
// cached guards' cone rows [tick parity][rows 0-7 | 8-15][max_guards] x 16 B, and the static
// position plane (channel 2 with the vault patched) -- or step_multi_body's, if larger, for
// the envs that take it.
size_t step_multi_lds(const EnvParams& p, int K);
struct LeanStage {
  uint4 off4[128];  // the fan's unique directions 0 .. 127, samples 1-8 (FanTick::off4)
  uint2 off2[128];  // samples 9-12 (FanTick::off2)
  int hdr[4];       // FanTick num_rays, range, n_uniq, n_tie
};

// Interval fans (heist_fan_intervals.h, tools/gen_fan_intervals.py).  A camera ray's 12
// sample tiles depend on its direction only through which INTERVAL between consecutive
// cuts -- the angles where |cos| or |sin| is a tie point j/k (j odd, k <= 12) or 0 -- the
// direction lies in: inside one, every sample's rint is constant (the fast path's argument,
// cast_rays).  So a camera's fan is the set of intervals its rays land in, and each is
// marched ONCE with its midpoint direction from the camera's tile; a ray within a margin of
// a cut takes the exact path.  Which intervals hold a ray is a few fixed-point comparisons
// per lane (lane = interval), no sin/cos and no dedup: a camera of fov F is ~0.7 F lanes
// instead of 2 F rays.  Angles are in 2^32 units per turn (u32 arithmetic wraps at 360).
// The lean kernel copies the table into LDS (the space the shared fan's staging takes in
// an env the fan serves).
constexpr double kFanUnitsPerDeg = 4294967296.0 / 360.0;
struct IvlTable {
  uint32_t cut[kFanCuts];  // cut angles, ascending
  float2 dir[kFanCuts];    // interval j = [cut j, cut j+1): midpoint (cos / 2, -sin / 2), fp32
  uint8_t idx[368];        // [d] first j with cut j >= d degrees, d = 0 .. 360
};
static_assert(sizeof(IvlTable) % 16 == 0, "copied in 16-byte words");
constexpr IvlTable make_ivl_table() {
  IvlTable t{};
  for (int j = 0; j < kFanCuts; ++j) {
    t.cut[j] = kFanCut[j];
    t.dir[j] = float2{kFanDir[j][0], kFanDir[j][1]};
  }
  for (int d = 0; d < 361; ++d) t.idx[d] = kFanIdx[d];
  return t;
}
__constant__ IvlTable kIvlTable = make_ivl_table();
constexpr size_t kLeanUnion = sizeof(LeanStage) > sizeof(IvlTable) ? sizeof(LeanStage) : sizeof(IvlTable);
struct LeanLds {
  uint8_t* grid;
  uint16_t* path;
  uint8_t* act;
  LeanStage* stg;  // an env the shared fan serves: the next tick's fan entry
  IvlTable* ivl;   // any other env: the interval table (same LDS)
  uint4* icam;     // interval fans, per camera: start angle, first cut, rays | tile << 16
  int32_t* icim;   //   and 2^52 / ray spacing (rounded; < 2^31)
  uint16_t* cone;
  float4* plane2;
};
// The lean kernel's plane gap D: the padded (R + 12) x (C + 12) plane in 1024 (up to 20 x 20)
// or 2048 bytes (up to 33 x 33).
__host__ __device__ constexpr int lean_gap(int R, int C) { return (R + 2 * kRing) * (C + 2 * kRing) <= 1024 ? 1024 : 2048; }
__host__ __device__ inline size_t lean_carve(unsigned char* smem, int R, int C, int mc, int mg, int mp, int K,
                                             LeanLds* L) {
  size_t o = 3 * (size_t)lean_gap(R, C);
  if (L) L->grid = smem + o;
  o += align16((size_t)R * C);
  if (L) L->path = reinterpret_cast<uint16_t*>(smem + o);
  o += align16(2 * (size_t)mg * mp);
  if (L) L->act = smem + o;
  o += align16((size_t)K);
  if (L) L->stg = reinterpret_cast<LeanStage*>(smem + o);
  if (L) L->ivl = reinterpret_cast<IvlTable*>(smem + o);
  o += align16(kLeanUnion);
  if (L) L->icam = reinterpret_cast<uint4*>(smem + o);
  o += 16 * (size_t)(mc > 0 ? mc : 1);
  if (L) L->icim = reinterpret_cast<int32_t*>(smem + o);
  o += align16(8 * (size_t)(mc > 0 ? mc : 1));
  if (L) L->cone = reinterpret_cast<uint16_t*>(smem + o);
  o += 64 * (size_t)(mg > 0 ? mg : 1);
  if (L) L->plane2 = reinterpret_cast<float4*>(smem + o);
  o += 4 * (size_t)R * C;
  return o;
}
static size_t lean_lds_bytes(const EnvParams& p, int K) {
  const size_t lean = align16(lean_carve(nullptr, p.R, p.C, p.max_cams, p.max_guards, p.max_path, K, nullptr)) +
                      (p.stamps ? 80 : 0);  // the STAMP variant's segment sums
  const size_t generic = step_multi_lds(p, K);  // the envs that take step_multi_body
  return lean > generic ? lean : generic;
}

// The lean tick issues its stores every tick after the LDS-DMA of the next tick's data:
// observation channels 0, 1, 2 for Q quads per lane (3 Q), reward, reward64, done, status.
// The next tick's `s_waitcnt vmcnt(3 Q + 4)` (kStores) therefore retires the DMA and never
// waits for a store.

// A cached guard's per-tick state packed in two registers: patrol index | step << 8 | len
// << 16 | heading slot << 24, and position | position 0 << 16 (row | col << 8 each); the slot
// after its next move rides in a third.
struct LeanGuard {
  uint32_t a, b, nslot;
  __device__ int idx() const { return (int)(a & 0xffu); }
  __device__ int step() const { return (int)((a >> 8) & 0xffu); }
  __device__ int len() const { return (int)((a >> 16) & 0xffu); }
  __device__ int hslot() const { return (int)(a >> 24); }
  __device__ uint32_t pos() const { return b & 0xffffu; }
  __device__ uint32_t pos0() const { return b >> 16; }
};

// The generic K-tick body for an env the lean loop does not serve, as a call rather than
// inlined: the lean loop is then scheduled and register-allocated on its own (C2 5.78 ->
// 5.64-5.71 us per tick; with the body removed altogether 5.66-5.69, profiles/r05as_*), at
// the price of a call frame (scratch) on the rare generic path.
template <int D>
__device__ __attribute__((noinline)) void lean_generic_body(EnvParams p, int K, const int64_t* __restrict__ actions,
                                                            float* __restrict__ obs, float* __restrict__ rew,
                                                            double* __restrict__ rew64, uint8_t* __restrict__ done_out,
                                                            int8_t* __restrict__ status_out, int auto_reset,
                                                            unsigned char* smem, int e) {
  step_multi_body<1, 4, 4, D, false, 0>(p, K, actions, obs, rew, rew64, done_out, status_out, auto_reset, smem, e);
}

// STAMP (instrumentation, heist_step_stamps armed): lane 0 sums the shader clock spent in 9
// tick segments over the launch (LEAN_SEGS in tools/probe_lean_stamps.py) in LDS after the
// carve and writes [segment sums 0..8, lifetime, start clock, HW_ID, XCC_ID] to
// stamps[env][0][16] (the generic K-tick body's layout); envs on the generic body record none.
// PROBE (profiling only, HEIST_PROBE_MODE with a library built -DHEIST_LEAN_PROBES,
// tools/build_variant.sh; results wrong): 21 no wait for the previous tick's
// DMA, 22 no visibility cast, 23 no observation stores, 24 / 25 shared-fan marches without
// their visibility stores / stop-byte loads, 26 the observation stores without their LDS reads,
// 27 the stores alone (no move, cast, detection), 28 move + patrol + stores.
template <int R_, int C_, bool STAMP = false, int PROBE = 0, int NW = 1>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(HEIST_LEAN_OCC))) void step_lean_kernel(
    EnvParams p, int K, const int64_t* __restrict__ actions, float* __restrict__ obs, float* __restrict__ rew,
    double* __restrict__ rew64, uint8_t* __restrict__ done_out, int8_t* __restrict__ status_out, int auto_reset) {
  constexpr int D = lean_gap(R_, C_);
  constexpr int PC = C_ + 2 * kRing;
  constexpr int RC = R_ * C_;
  constexpr int N4 = RC / 4;
  constexpr int C4 = C_ / 4;
  constexpr int Q = (N4 + 63) / 64;  // observation quads per lane (20 x 20: 2, 32 x 32: 4)
  constexpr int OFF0 = kRing * PC + kRing;  // padded index of tile (0, 0); also a sample's offset on its own tile
  static_assert((R_ + 2 * kRing) * PC <= D, "the padded planes fit the 1024-byte gap");
  static_assert(C_ % 4 == 0 && R_ <= 64 && C_ <= 32 && (R_ + 2 * kRing) * PC <= 2048, "lean kernel geometry");
  static_assert(NW == 1 || (NW == 2 && !STAMP && PROBE == 0 && Q % 2 == 0), "two waves: the plain form, even Q");
  constexpr int QW = Q / NW;          // observation quads per lane this wave stores
  constexpr int kStores = 3 * QW + 4;  // a wave's stores per tick (see 6. below)
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = block_env(p);
  if (p.prio_mode && p.dispatch_order) {
    const int pr = (int)((uint32_t)p.order[blockIdx.x] >> 24);
    if (pr == 3) __builtin_amdgcn_s_setprio(3);
    else if (pr == 2) __builtin_amdgcn_s_setprio(2);
    else if (pr == 1) __builtin_amdgcn_s_setprio(1);
  }
  // NW = 2 (an interval-fan env of a batch small enough that two waves per env still fit
  // the chip): both waves keep the env's whole state (the same inputs, the same arithmetic),
  // split the cast's pair chunks and the observation quads, and meet at LDS barriers; wave 0
  // alone owns the cached guard cones (their LDS-DMA, staging and stamps) and the write-back
  const int lane = NW == 1 ? (int)threadIdx.x : (int)(threadIdx.x & 63u);
  const int wid = NW == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int tid = threadIdx.x;
  const int N = p.n_envs;
  const int mc = p.max_cams, mg = p.max_guards, n_slot = mc + mg, mp = p.max_path;
  const EnvBase eb = env_base(p, e);
  const FanTick* fan0 = p.fan + p.fan_base;

  // ---- which kernel body serves this env for the launch: the lean loop needs every live
  // camera to BE the shared fan's source camera (same heading after this launch's first
  // rotation, same speed, fov, rays and range 6: then the table's entry k is this camera's
  // fan at tick k, the same functions on the same inputs), every live guard cached, and the
  // env acting at the first tick
  EnvScalars s = p.scal[e];
  const int g = lane - mc;
  double heading = 0.0, speed = 0.0;  // camera lanes
  uint32_t cam_rc = 0;                // camera lanes: row | col << 8
  LeanGuard gd{0u, 0u, 0u};           // guard lanes
  const bool live_cam = lane < s.n_cams, live_guard = g >= 0 && g < s.n_guards;
  bool cached = false;
  // interval fans (camera lanes): fov, the ray spacing in angle units and its reciprocal, rays
  double fovd = 0.0, su = 1.0;
  int32_t im_fx = 0;  // 2^52 / su rounded: the pair bounds as integer products (cast_ivl)
  int cam_n = 0;
  bool ivl = false;  // this env casts its cameras from the interval table (else from the shared fan)
  {
    EmitterRaw rec;
    rec.a = make_uint4(0u, 0u, 0u, 0u);
    rec.b = rec.a;
    if (lane < n_slot) {
      const uint4* rs = lane < mc ? reinterpret_cast<const uint4*>(eb.cams + (uint32_t)lane)
                                  : reinterpret_cast<const uint4*>(eb.guards + (uint32_t)g);
      rec.a = rs[0];
      rec.b = rs[1];
    }
    const Cam cm = as_cam(rec);
    const Guard gr = as_guard(rec);
    heading = cm.heading;
    speed = cm.speed;
    cam_rc = (uint32_t)cm.row | ((uint32_t)cm.col << 8);
    cached = live_guard && gr.hslot != kUncached;
    gd.a = (uint32_t)(uint8_t)gr.idx | ((uint32_t)(uint8_t)gr.step << 8) | ((uint32_t)(uint8_t)gr.len << 16) |
           ((uint32_t)gr.hslot << 24);
    gd.b = (uint32_t)gr.pos | ((uint32_t)gr.pos0 << 16);
    gd.nslot = gr.nslot;
    const double f_heading = fan0->heading, f_speed = fan0->speed, f_fov = fan0->fov;
    const int f_rays = fan0->num_rays, f_range = fan0->range, f_uniq = fan0->n_uniq;
    const bool cam_ok = !live_cam || (py_mod360(cm.heading + cm.speed * 1.0) == f_heading && cm.speed == f_speed &&
                                      cm.fov == f_fov && cm.num_rays == f_rays && cm.range == f_range);
    // patrol index, step and length fit the packed bytes: a cached guard has <= kConePath points
    const bool base_ok = p.ray_mode == 0 && !s.done && __ballot(live_guard && !cached) == 0ull;
    const bool fan_ok = p.fan_on && f_uniq >= 0 && f_range == kTieMaxRange && __ballot(!cam_ok) == 0ull;
    // the interval fans need range 6 (12 samples, the table's), a fan narrower than half a
    // turn (signed angle differences) and rays farther apart than two axis margins (at most
    // one ray near any cut)
    const double su_ = (cm.fov / (double)cm.num_rays) * kFanUnitsPerDeg;
    // (and spacing su >= 2^21 units, ~0.18 degrees, so that 2^52 / su fits an int32; every
    // fov >= 5.3 degrees: security.py:67 spaces rays fov / max(2 fov, 30) apart).  fov < 170:
    // the farthest cut a camera's pairs look at lies at most fov + the widest cut gap (4.8
    // degrees, between an axis and asin(1/12)) past h0, inside the int32 half turn
    const bool ivl_cam = !live_cam || (cm.range == kTieMaxRange && cm.num_rays >= 1 && cm.fov > 0.0 &&
                                       cm.fov < 170.0 && su_ > 2.0 * (double)kFanMarginAxis + 8.0 &&
                                       su_ >= 2097153.0);
    ivl = base_ok && !fan_ok && p.interval_fans && __ballot(!ivl_cam) == 0ull;
    if (!base_ok || (!fan_ok && !ivl)) {
      if (NW == 2 && wid != 0) return;  // the generic body is one wave's (an ended wave leaves the barriers)
      lean_generic_body<D>(p, K, actions, obs, rew, rew64, done_out, status_out, auto_reset, smem, e);
      return;
    }
    if (live_cam) {
      fovd = cm.fov;
      su = su_;
      im_fx = (int32_t)__builtin_rint(4503599627370496.0 / su_);
      cam_n = cm.num_rays;
    }
  }

  // ---- prologue: the env's layout and state, once per launch
  LeanLds L;
  const size_t carved = lean_carve(smem, R_, C_, mc, mg, mp, K, &L);
  unsigned long long* st_acc = reinterpret_cast<unsigned long long*>(smem + align16(carved));
  unsigned long long st_last = 0, st_start = 0;
  if (STAMP && lane == 0) {
    st_start = st_last = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < 9; ++j) st_acc[j] = 0;
  }
#define LEAN_STAMP(seg)                                        \
  do {                                                         \
    if (STAMP && lane == 0) {                                  \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
      st_acc[(seg)] += now_ - st_last;                         \
      st_last = now_;                                          \
    }                                                          \
  } while (0)
  uint8_t* const wall = smem;          // [0, D): the padded stop map
  uint8_t* const vis = smem + D;       // [D, 2D): the visibility plane; [2D, 3D): the sink
  const uint32_t base = (uint32_t)(uintptr_t)smem;  // LDS address of the stop map
  const uint32_t stg_a = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)L.stg);
  const uint32_t stc_a = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)L.cone);
  {
    // grid (static observation channel 0) and the padded stop map, as prefetch does
    const uint32_t* g4 = reinterpret_cast<const uint32_t*>(p.grid + (size_t)e * RC);
    for (int i = tid; i < N4; i += 64 * NW) reinterpret_cast<uint32_t*>(L.grid)[i] = g4[i];
    const uint8_t* ss = p.stop + (size_t)e * p.stop_bytes;
    for (int i = tid; i < p.stop_bytes; i += 64 * NW) expand_stop(wall, i, ss[i]);
    const int vault = p.vr * C_ + p.vc, qv = vault >> 2;
    for (int q = tid; q < N4; q += 64 * NW) {  // channel 2's static plane with the vault patched
      float4 v = reinterpret_cast<const float4*>(p.plane0)[q];
      if (q == qv) patch4(v, vault & 3, p.vault_val);
      L.plane2[q] = v;
    }
  }
  for (int i = tid; i < mg * mp; i += 64 * NW) L.path[i] = eb.paths[i];
  for (int k = tid; k < K; k += 64 * NW) {
    const int64_t a = actions[(size_t)k * N + e];
    L.act[k] = (uint8_t)((a < 0 || a > 4) ? 0 : a);  // unknown actions do not move (environment.py:239)
  }
  __syncthreads();  // LDS filled
  uint32_t vwall = 0;  // lane r < R: bit c = stop byte of tile (r, c) (a wall)
  if (lane < R_)
    for (int c = 0; c < C_; ++c) vwall |= (uint32_t)wall[OFF0 + lane * PC + c] << c;

  // HBM data a tick needs -- its shared fan entry (FanTick: the unique directions' sample
  // tiles, n_uniq, n_tie) and its cached guards' cone entries -- comes by LDS-DMA issued a
  // tick ahead: the fan entry once the tick has marched its own (the staging is then free),
  // a cone entry once the guard's move is known (the pose after the next move; a finishing
  // env re-issues it for its reset pose; double-buffered by tick parity).  The tick's stores
  // go last, so the next tick's counted wait for the DMA (kStores younger operations)
  // never waits for a store to reach memory.
  auto dma_fan = [&](int k, bool wide) {  // k < K
    const FanTick* f = fan0 + k;
    lds_dma16(f->off4 + lane, stg_a + (uint32_t)offsetof(LeanStage, off4));
    if (wide) lds_dma16(f->off4 + 64 + lane, stg_a + (uint32_t)offsetof(LeanStage, off4) + 1024u);
    lds_dma16(f->off2 + 2 * lane, stg_a + (uint32_t)offsetof(LeanStage, off2));
    if (lane == 0) lds_dma16(&f->num_rays, stg_a + (uint32_t)offsetof(LeanStage, hdr));
  };
  // the cone entry (rows 0-15, 32 B) of cached guard g at (idx, slot) into cone staging
  // `par`: lane mc + g writes at the base it is given minus 16 mc
  auto dma_cone = [&](int idx, int slot, int par) {
    if (cached) {
      const uint16_t* src = eb.cones + cone_off((uint32_t)g, (uint32_t)idx, (uint32_t)slot);
      const uint32_t dst = stc_a + (uint32_t)(par * 32 * mg) - 16u * (uint32_t)mc;
      lds_dma16(src, dst);
      lds_dma16(src + 8, dst + 16u * (uint32_t)mg);
    }
  };
  // the entry of the pose after a move from the guard's current one (idx + step, nslot)
  auto dma_next_cone = [&](int par) {
    int idx = gd.idx(), slot = gd.hslot();
    if (gd.len() >= 2) {
      idx += gd.step();
      if (idx >= gd.len()) idx -= gd.len();
      slot = (int)gd.nslot;
    }
    dma_cone(idx, slot, par);
  };
  if (wid == 0) dma_next_cone(0);
  if (ivl) {  // the interval table into the staging space (LDS-DMA, 16 B per lane per pass)
    for (uint32_t o = 1024u * (uint32_t)wid; o < (uint32_t)sizeof(IvlTable); o += 1024u * NW)
      if (o + 16u * (uint32_t)lane < (uint32_t)sizeof(IvlTable))
        lds_dma16(reinterpret_cast<const unsigned char*>(&kIvlTable) + o + 16u * (uint32_t)lane, stg_a + o);
  } else if (wid == 0) {
    dma_fan(0, true);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (NW == 2) __syncthreads();  // both waves' parts of the table in place

  // the cached guards' cone rows (staging parity par) ORed into the plane: lane 15 i + j
  // takes row j of guard slot 4 pass + i; bit dc + 7 of row dr + 7 is tile (gr + dr, gc + dc);
  // the aligned dwords a row spans get its bits as 0/1 bytes (ds_or_b32)
  const uint64_t cmask = __ballot(cached);
  auto stamp_cones = [&](int par) {
    const uint32_t gposv = gd.pos();
    for (int pass = 0; pass * 4 < mg; ++pass) {
      const int i = lane / 15, j = lane - 15 * i;
      const int gs = 4 * pass + i;
      const uint32_t gp = (uint32_t)__shfl((int)gposv, mc + (gs < mg ? gs : 0), 64);
      if (lane < 60 && gs < mg && ((cmask >> (mc + gs)) & 1u)) {
        const uint32_t bits = L.cone[par * 16 * mg + (j >> 3) * 8 * mg + 8 * gs + (j & 7)] & 0x7fffu;
        if (bits) {
          const uint32_t a0 = base + D + OFF0 + (unpack_r((uint16_t)gp) + j - kConeRange) * PC +
                              (unpack_c((uint16_t)gp) - kConeRange);
          const uint32_t m = bits << (a0 & 3u);
          const uint32_t a = a0 & ~3u;
#pragma unroll
          for (int w = 0; w < 5; ++w) {
            const uint32_t nib = (m >> (4 * w)) & 15u;
            if (nib)
              __hip_atomic_fetch_or(reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(a + 4 * w),
                                    __umul24(nib, 0x204081u) & 0x01010101u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
    }
  };
  // one fast-path march: this lane's unique direction from the camera whose corner tile
  // (row - 6, col - 6) is at LDS address `corner`; all 12 stop bytes read before any is used,
  // a running stop flag (and the own tile, only reachable by samples 1 and 2) sends a
  // sample's visibility store to the sink plane (march_fast)
  auto march = [&](uint32_t corner, uint4 o4, uint2 o2) {
    const uint32_t ow[6] = {o4.x, o4.y, o4.z, o4.w, o2.x, o2.y};
    uint32_t a[12], w[12];
#pragma unroll
    for (int u = 0; u < 12; ++u) a[u] = corner + ((u & 1) ? (ow[u >> 1] >> 16) : (ow[u >> 1] & 0xffffu));
#pragma unroll
    for (int u = 0; u < 12; ++u) w[u] = PROBE == 25 ? 0u : lds_ld(a[u]);
    const uint32_t own0 = (ow[0] & 0xffffu) == (uint32_t)OFF0, own1 = (ow[0] >> 16) == (uint32_t)OFF0;
    uint32_t stop = 0;
#pragma unroll
    for (int u = 0; u < 12; ++u) {
      stop = u == 0 ? w[0] : or_b32(stop, w[u]);
      const uint32_t skip = u == 0 ? or_b32(stop, own0) : (u == 1 ? or_b32(stop, own1) : stop);
      if (PROBE != 24) lds_st(__umul24(skip, (uint32_t)D) + a[u] + D, 1);
    }
  };
  // this tick's visibility into the cleared plane: every camera marches the shared fan's
  // unique directions -- from the staging, or (the reset pass, after the next tick's DMA
  // took the staging) from the table -- with the table's near-tie rays on the exact path,
  // then the cached cones
  auto cast_fan = [&](int k, int n_uniq, int n_tie, int par, bool staged, bool staged_wide) {
#pragma unroll
    for (int z = 0; z < D / 1024; ++z)  // 64 x 16 B per pass: the plane
      reinterpret_cast<uint4*>(vis)[lane + 64 * z] = make_uint4(0u, 0u, 0u, 0u);
    const FanTick* f = fan0 + k;
    uint4 o4a = make_uint4(0u, 0u, 0u, 0u), o4b = o4a;
    uint2 o2a = make_uint2(0u, 0u), o2b = o2a;
    if (s.n_cams > 0) {
      const bool want_b = n_uniq > 64;
      if (staged) {
        o4a = L.stg->off4[lane];
        o2a = L.stg->off2[lane];
        if (want_b && staged_wide) {
          o4b = L.stg->off4[64 + lane];
          o2b = L.stg->off2[64 + lane];
        }
      }
      if (!staged || (want_b && !staged_wide)) {  // from the table (rare): waited for here, not after the join
        if (!staged) {
          o4a = f->off4[lane];
          o2a = f->off2[lane];
        }
        if (want_b) {
          o4b = f->off4[64 + lane];
          o2b = f->off2[64 + lane];
        }
        asm volatile("" ::"v"(__builtin_bit_cast(u32x4_t, o4a)), "v"(__builtin_bit_cast(u32x2_t, o2a)),
                     "v"(__builtin_bit_cast(u32x4_t, o4b)), "v"(__builtin_bit_cast(u32x2_t, o2b)));
      }
    }
    // the tick's fan entry is in registers, the staging free: tick k + 1's entry goes out now,
    // a whole cast ahead of the next tick's wait for it (once the staging reads have returned)
    if (staged && k + 1 < K) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(__builtin_bit_cast(u32x4_t, o4a)), "v"(__builtin_bit_cast(u32x2_t, o2a)),
                   "v"(__builtin_bit_cast(u32x4_t, o4b)), "v"(__builtin_bit_cast(u32x2_t, o2b))
                   : "memory");
      dma_fan(k + 1, n_uniq > 64);
    }
    if (s.n_cams > 0) {
      for (int m = 0; m < s.n_cams; ++m) {
        const uint32_t rcm = (uint32_t)__builtin_amdgcn_readlane((int)cam_rc, m);
        const uint32_t corner = base + (rcm & 0xffu) * PC + (rcm >> 8);
        if (lane < n_uniq) march(corner, o4a, o2a);
        if (lane + 64 < n_uniq) march(corner, o4b, o2b);
        for (int c0 = 128; c0 < n_uniq; c0 += 64)  // fans wider than 128 unique directions (fov > ~150)
          if (lane + c0 < n_uniq) march(corner, f->off4[lane + c0], f->off2[lane + c0]);
      }
      if (n_tie > 0) lean_tie_rays<D, PC>(smem, f, n_tie, cam_rc, s.n_cams, p.half_deg);
    }
    LEAN_STAMP(2);
    stamp_cones(par);
  };
  // this tick's visibility from the interval table (an env the shared fan does not serve).
  // Ray i of a camera lies i * su angle units past its fixed-point start h0 (the reference's
  // ray i at hmh + fov * i / n, security.py:70, within 2 units); with rel = cut j - h0 and m
  // its margin, rays B_j = ceil((rel - m) / su) .. A_j - 1 = floor((rel + m) / su) lie within
  // the margin (at most one: su > 2 m) and take the exact path, rays A_j .. B_j+1 - 1 lie
  // inside interval j, which is marched once if there is one.  A and B are pure functions of
  // the cut, the same in whichever lane evaluates them, so the classes partition the rays
  // (tests/test_fan_intervals.py restates this and checks it against the oracle's cones).
  // The env's cameras are packed: camera c needs the cuts jb_c .. je_c - 1 (jb: the last cut
  // before its first ray, je: the first one past its last ray + margin), and the (camera, cut)
  // pairs of all cameras fill the lanes 64 at a time, and each lane whose interval holds a
  // ray marches it in place from its camera's tile -- so a wave's lanes are busy whatever the
  // fan widths, and an env's chain of chunks is as short as its cameras' total cut count
  // allows (about 92 % of the pairs of the synthetic mix hold a ray; packing the marches
  // through an LDS queue, 64 per march, was slower: one more LDS round trip per march).
  // NW = 2: the waves meet with their LDS operations retired (no vector-memory wait: the
  // previous ticks' stores stay in flight)
  auto wave_join = [&]() {
    if constexpr (NW == 2) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  auto cast_ivl = [&](int par) {
    wave_join();  // both waves' reads of the previous plane are done
#pragma unroll
    for (int z = wid; z < D / 1024; z += NW)  // 64 x 16 B per pass: the plane
      reinterpret_cast<uint4*>(vis)[lane + 64 * z] = make_uint4(0u, 0u, 0u, 0u);
    // camera lanes: the start angle, the cut range, the pair count
    const double hmh = heading - fovd / 2.0;  // security.py:64, :70
    const double hu = (hmh < 0.0 ? hmh + 360.0 : hmh) * kFanUnitsPerDeg;
    const uint32_t h0v = hu >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)hu;
    int cnt = 0, jb = 0;
    if (live_cam) {
      jb = (int)L.ivl->idx[__umulhi(h0v, 360u)] - 1;  // -1: cut 251 of the turn before
      const uint64_t e64 = (uint64_t)h0v + (uint64_t)((double)cam_n * su) + (uint64_t)(kFanMarginAxis + 4);
      const int je = (int)L.ivl->idx[__umulhi((uint32_t)e64, 360u) + 1u] + kFanCuts * (int)(e64 >> 32);
      cnt = je - jb;
      L.icam[lane] = make_uint4(h0v, (uint32_t)jb, (uint32_t)cam_n | (cam_rc << 16), 0u);
      L.icim[lane] = im_fx;
    }
    // the pair counts' running sums are scalar: a few cameras, summed where they are needed;
    // camera lane m keeps jo = jb - (pairs of cameras 0 .. m-1), so pair q of camera m has cut
    // jo + q, known before any LDS read (the chunk's loads then go out together)
    // and end_l = pairs of cameras 0 .. m (a chunk looks only at the cameras it overlaps)
    int total = 0, jo_l = 0, end_l = 0;
    for (int m = 0; m < s.n_cams; ++m) {
      if (lane == m) jo_l = jb - total;
      total += __builtin_amdgcn_readlane(cnt, m);
      if (lane == m) end_l = total;
    }
    // one interval's march from the camera tile rc (row | col << 8) along direction d
    auto march_at = [&](uint32_t rc, float2 d) {
      const uint32_t row = rc & 0xffu, col = rc >> 8;
      const uint32_t own = base + (row + kRing) * PC + col + kRing;
      const float mx = __builtin_bit_cast(float, base + col + kRing), my = __builtin_bit_cast(float, row + kRing);
      march_fast<D, 2 * kTieMaxRange, false, false, true>(PC, own, d.x, d.y, mx, my, 2 * kTieMaxRange);
    };
    int mb = 0;  // the first camera whose pairs reach this chunk
    wave_join();  // the plane is clear
    for (int q0 = 64 * wid; q0 < total; q0 += 64 * NW) {
      const int q = q0 + lane;
      while (__builtin_amdgcn_readlane(end_l, mb) <= q0) ++mb;
      // the camera of pair q (those before it end at or below q) and its cut
      int c = mb, jo = __builtin_amdgcn_readlane(jo_l, mb);
      for (int m = mb; m + 1 < s.n_cams; ++m) {
        const int em = __builtin_amdgcn_readlane(end_l, m);
        if (em >= q0 + 64) break;
        const int jo_m = __builtin_amdgcn_readlane(jo_l, m + 1);
        if (q >= em) {
          c = m + 1;
          jo = jo_m;
        }
      }
      int j = jo + q;
      j = j < 0 ? j + kFanCuts : (j >= kFanCuts ? j - kFanCuts : j);
      const uint4 cu = L.icam[c];
      const int im = L.icim[c];
      const int n = (int)(cu.z & 0xffffu);
      const int jn = j + 1 == kFanCuts ? 0 : j + 1;
      const uint32_t cut = L.ivl->cut[j], cutn = L.ivl->cut[jn];
      const float2 dj = L.ivl->dir[j];  // read with the cuts
      const int rel = (int)(cut - cu.x), reln = (int)(cutn - cu.x);
      const int mj = (cut & 0x3FFFFFFFu) ? kFanMarginTie : kFanMarginAxis;
      const int mn = (cutn & 0x3FFFFFFFu) ? kFanMarginTie : kFanMarginAxis;
      // floor(x / su) as the high word of the 64-bit product x * im >> 20 (floor(x im / 2^52));
      // ceil(x / su) = -floor(-x / su).  The product's error is below 2^31 * 2^-53 rays, ~1.4
      // angle units at su = 0.5 degrees, far inside the 64- and 720-unit margins.
      const int A = (__mulhi(rel + mj, im) >> 20) + 1;  // first ray past cut j's margin
      const int B = -(__mulhi(mj - rel, im) >> 20);     // first ray inside it
      const int Bn = -(__mulhi(mn - reln, im) >> 20);   // first ray inside cut j+1's
      const int a0 = A > 0 ? A : 0;
      const bool act = q < total;
      const bool safe = act && a0 <= n && a0 < Bn;
      const bool near = act && B < A && B >= 0 && B <= n;
      if (__ballot(near)) {  // rare: this pair's camera emitter from its lane, the exact path
        const double h_c = __shfl(hmh, c, 64), f_c = __shfl(fovd, c, 64);
        ivl_tie_rays<D, PC>(smem, near ? B : -1, h_c, f_c, n, cu.z >> 16, p.half_deg);
      }
      if (safe) march_at(cu.z >> 16, dj);
    }
    LEAN_STAMP(2);
    if (wid == 0) stamp_cones(par);
    wave_join();  // the plane is complete
  };
  auto cast = [&](int k, int n_uniq, int n_tie, int par, bool staged, bool staged_wide) {
    if (ivl) {
      cast_ivl(par);
    } else {  // the shared fan: wave 0's (its staging and DMA are wave 0's)
      wave_join();
      if (wid == 0) cast_fan(k, n_uniq, n_tie, par, staged, staged_wide);
      wave_join();
    }
  };

  constexpr uint32_t kOOB = 0x40000000u;  // a store offset past every buffer descriptor below
  uint32_t vact = 0;  // lane j: the action of tick 64 c + j (the current 64-tick chunk)
  bool wide = true;   // the DMA staged directions 64 .. 127 for this tick
  for (int k = 0; k < K; ++k) {
    const int par = k & 1;
    if ((k & 63) == 0) vact = k + lane < K ? L.act[k + lane] : 0u;
    // the DMA issued a tick ago (older than the previous tick's kStores stores) has landed
    if (PROBE == 21) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kStores) : "memory");
    int n_uniq = 0, n_tie = 0;
    if (!ivl && wid == 0) {  // one LDS read for both header words
      const int2 h = *reinterpret_cast<const int2*>(&L.stg->hdr[2]);
      n_uniq = __builtin_amdgcn_readfirstlane(h.x);
      n_tie = __builtin_amdgcn_readfirstlane(h.y);
    }
    LEAN_STAMP(0);  // 0: the tick's DMA wait, the fan header
    const bool staged_wide = wide;
    const bool frozen = s.done != 0;  // finished, no auto-reset: environment.py:232-233
    double reward = 0.0;
    int status = kAlreadyDone, curr = 0;
    if (!frozen && PROBE != 27) {
      // 1. move (environment.py:239-246) and the reward terms that precede detection (:235, :261-269)
      const int a = __builtin_amdgcn_readlane((int)vact, k & 63);
      const int nr = s.pos_r + (a == 1 ? -1 : (a == 2 ? 1 : 0)), nc = s.pos_c + (a == 3 ? -1 : (a == 4 ? 1 : 0));
      if (nr >= 0 && nr < R_ && nc >= 0 && nc < C_ && !((__builtin_amdgcn_readlane((int)vwall, nr) >> nc) & 1)) {
        s.pos_r = nr;
        s.pos_c = nc;
      }
      status = kRunning;
      curr = iabs_(s.pos_r - p.vr) + iabs_(s.pos_c - p.vc);
      reward = p.r_step;
      reward += (double)(s.prev_dist - curr) * 0.1;
      if (curr <= 3 && s.initial_dist > 3) reward += 0.05 * (double)(3 - curr);
      s.prev_dist = curr;
      // 2. cameras rotate, guards patrol (security.py:49-51, :145-159; every live guard is
      // cached here: its heading is its slot's)
      if (live_cam) heading = py_mod360(heading + speed * 1.0);
      if (live_guard && gd.len() >= 2) {
        int nidx = gd.idx() + gd.step();
        if (nidx >= gd.len()) nidx -= gd.len();
        const uint32_t np = L.path[__umul24((uint32_t)g, (uint32_t)mp) + (uint32_t)nidx];
        gd.a = (uint32_t)nidx | (gd.a & 0x00ffff00u) | (gd.nslot << 24);
        gd.b = np | (gd.b & 0xffff0000u);
      }
      // the slot after the guard's next move: row 15 of this tick's entry (staged a tick ago)
      if (cached && wid == 0) gd.nslot = L.cone[par * 16 * mg + 8 * mg + 8 * g + 7];
      if (k + 1 < K && wid == 0) dma_next_cone(par ^ 1);  // tick k + 1's entry if the env still acts then
      LEAN_STAMP(1);  // 1: move, rotation, patrol
      // 3. visibility (environment.py:257-258)
      if (PROBE != 22 && PROBE != 28) cast(k, n_uniq, n_tie, par, true, staged_wide);
      LEAN_STAMP(3);  // 3: the cached guard cones (2: the cameras, inside cast)
    }
    // (tick k + 1's fan entry went out inside cast_fan; a frozen env keeps its plane and skips it)
    wide = n_uniq > 64;
    // the plane's channel-1 quads this wave stores (one wave: also the detection test's byte)
    uint32_t v1[QW];
#pragma unroll
    for (int j = 0; j < QW; ++j) {
      const int q = lane + 64 * (wid * QW + j), qc = q < N4 ? q : N4 - 1, r = qc / C4;
      v1[j] = *reinterpret_cast<const uint32_t*>(vis + OFF0 + r * PC + 4 * (qc - r * C4));
    }
    int done_now = s.done;
    LEAN_STAMP(4);  // 4: next fan DMA, the channel-1 quads
    if (!frozen && PROBE != 27 && PROBE != 28) {
      // 4. detection, vault, timeout (environment.py:271-297), in the reference's order
      bool seen;
      if constexpr (NW == 1) {
        const int sol = s.pos_r * C_ + s.pos_c, qs = sol >> 2;
        uint32_t vq = v1[0];  // the quad holding the solver's tile (register qs >> 6, wave-uniform)
#pragma unroll
        for (int j = 1; j < Q; ++j) vq = (qs >> 6) == j ? v1[j] : vq;
        const uint32_t qv = (uint32_t)__builtin_amdgcn_readlane((int)vq, qs & 63);
        seen = ((qv >> (8 * (sol & 3))) & 0xffu) != 0u;
      } else {  // the quad may be the other wave's: the byte itself
        seen = vis[OFF0 + s.pos_r * PC + s.pos_c] != 0;
      }
      if (seen) {
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
      done_now = s.done;
    }
    LEAN_STAMP(5);  // 5: detection, vault, timeout
    if (auto_reset && done_now) {
      // 5. auto-reset (environment.py:183-214): headings kept, guards back to patrol point 0;
      // this row's observation is the next attempt's first one
      const bool moved = __ballot(live_guard && gd.pos() != gd.pos0()) != 0ull;
      reset_solver(p, s);
      if (live_guard) {
        gd.a &= ~0xffu;                        // idx 0
        gd.b = (gd.b & 0xffff0000u) | gd.pos0();  // the patrol start
      }
      if (cached && wid == 0) {  // the cone of (patrol point 0, this slot), loaded now: only finishing envs pay for it
        const uint4* rsrc = reinterpret_cast<const uint4*>(eb.cones + cone_off(g, 0, gd.hslot()));
        const uint4 ra = rsrc[0], rb = rsrc[1];
        if (moved) {
          *reinterpret_cast<uint4*>(L.cone + par * 16 * mg + 8 * g) = ra;
          *reinterpret_cast<uint4*>(L.cone + par * 16 * mg + 8 * mg + 8 * g) = rb;
        }
        gd.nslot = rb.w >> 16;
      }
      if (moved) {  // the plane again from the reset poses (the staging holds tick k + 1's fan now)
        cast(k, n_uniq, n_tie, par, false, false);
#pragma unroll
        for (int j = 0; j < QW; ++j) {
          const int q = lane + 64 * (wid * QW + j), qc = q < N4 ? q : N4 - 1, r = qc / C4;
          v1[j] = *reinterpret_cast<const uint32_t*>(vis + OFF0 + r * PC + 4 * (qc - r * C4));
        }
      }
      if (k + 1 < K && wid == 0) dma_next_cone(par ^ 1);  // tick k + 1's entry from the reset pose
    }
    LEAN_STAMP(6);  // 6: auto-reset
    // 6. tick k's stores (kStores, unconditional; lanes with nothing to store pass an offset
    // past their buffer descriptor, which the hardware drops): observation channels 0, 1, 2
    // (Q quads per lane each), reward, reward64, done, status
    asm volatile("" ::: "memory");
    constexpr int pol = 2;  // nt (policy A/B: profiles/r02ba_probe_obs_store.log; sc1 nt 3 % slower here, r05w)
    float* o = obs + ((size_t)k * N + e) * 3 * RC;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(o, (short)0, 12 * RC, 0x00020000);
    const int sol = s.pos_r * C_ + s.pos_c, qs = sol >> 2;
    const int vault = p.vr * C_ + p.vc;
#pragma unroll
    for (int j = 0; j < QW; ++j) {
      const int q = lane + 64 * (wid * QW + j);
      const bool in = q < N4;
      const int qc = in ? q : N4 - 1;
      const uint32_t b = PROBE == 26 ? 0x01020304u : *reinterpret_cast<const uint32_t*>(L.grid + 4 * qc);
      // float32(tile) / 5 == float32(tile) * 0.2f for every tile type (environment.py:319)
      if (PROBE == 23) continue;
      obs_put(rs, pol, in ? 16 * q : (int)kOOB,
              make_float4((float)(b & 0xff) * 0.2f, (float)((b >> 8) & 0xff) * 0.2f,
                          (float)((b >> 16) & 0xff) * 0.2f, (float)(b >> 24) * 0.2f));
      const uint32_t v = v1[j];
      obs_put(rs, pol, in ? 16 * (N4 + q) : (int)kOOB,
              make_float4((float)(v & 0xff), (float)((v >> 8) & 0xff), (float)((v >> 16) & 0xff), (float)(v >> 24)));
      float4 c2 = PROBE == 26 ? make_float4(0.f, 0.f, 0.f, 0.f) : L.plane2[qc];
      // the solver's cell of channel 2 is fl32(1 + g) for its static value g (heist_create's
      // second plane), unless it is the vault, whose value wins: patched in the register of
      // the lane that stores its quad (one store per quad, no second write of the line)
      const bool pl = q == qs && sol != vault;
      const int m = sol & 3;
      c2.x = pl && m == 0 ? 1.0f + c2.x : c2.x;
      c2.y = pl && m == 1 ? 1.0f + c2.y : c2.y;
      c2.z = pl && m == 2 ? 1.0f + c2.z : c2.z;
      c2.w = pl && m == 3 ? 1.0f + c2.w : c2.w;
      obs_put(rs, pol, in ? 16 * (2 * N4 + q) : (int)kOOB, c2);
    }
    const uint32_t ko = (uint32_t)((size_t)k * N + e);
    const int l0 = lane == 0 && wid == 0 ? 0 : (int)kOOB;
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, (float)reward),
                                          __builtin_amdgcn_make_buffer_rsrc(rew + ko, (short)0, 4, 0x00020000), l0, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, __builtin_bit_cast(uint64_t, reward)),
                                          __builtin_amdgcn_make_buffer_rsrc(rew64 ? rew64 + ko : rew64, (short)0,
                                                                            rew64 ? 8 : 0, 0x00020000),
                                          l0, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)done_now,
                                         __builtin_amdgcn_make_buffer_rsrc(done_out + ko, (short)0, 1, 0x00020000), l0,
                                         0, 0);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(int8_t)status,
                                         __builtin_amdgcn_make_buffer_rsrc(status_out + ko, (short)0, 1, 0x00020000),
                                         l0, 0, 0);
    LEAN_STAMP(7);  // 7: the tick's stores
  }
  // epilogue: the state the next launch (or heist_export) starts from
  if (STAMP && lane == 0) {
    unsigned long long* q = p.stamps + (size_t)e * p.multi_waves * 16;
    for (int j = 0; j < 9; ++j) q[j] = st_acc[j];
    q[9] = __builtin_amdgcn_s_memtime() - st_start;
    q[10] = st_start;
    q[11] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    q[12] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  }
#undef LEAN_STAMP
  if (wid != 0) return;  // (its guards' heading slots are not tracked)
  if (lane == 0) p.scal[e] = s;
  if (live_cam) eb.cams[(uint32_t)lane].heading = heading;
  if (live_guard) {
    // the heading its slot names (u16 16..19 of any entry with that slot)
    const uint4 c2 = reinterpret_cast<const uint4*>(eb.cones + cone_off(g, gd.idx(), gd.hslot()))[2];
    Guard* gp = eb.guards + (uint32_t)g;
    gp->heading = __builtin_bit_cast(double, ((uint64_t)c2.y << 32) | c2.x);
    gp->idx = (int16_t)gd.idx();
    gp->pos = (uint16_t)gd.pos();
    gp->hslot = (uint8_t)gd.hslot();
    gp->nslot = (uint8_t)gd.nslot;
  }
}

template <int W, int U, int O, int D>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(O))) void reset_kernel(EnvParams p, const uint8_t* __restrict__ mask,
                                                        float* __restrict__ obs) {
  constexpr int NT = 64 * W;
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = block_env(p);
  const int t = threadIdx.x;
  if (mask && !mask[e]) return;
  const EnvLds L = carve<D>(smem, p.R, p.C, p.max_cams + p.max_guards, 0, W, p.max_guards);
  const EnvBase eb = env_base(p, e);
  EmitterRaw raw;
  prefetch<NT>(p, e, eb, L, raw);
  EnvScalars s = p.scal[e];
  const int mc = p.max_cams, n_slot = p.max_cams + p.max_guards;
  clear_vis<NT>(p, L);
  __syncthreads();  // grid, stop map in LDS
  reset_solver(p, s);
  Emit E;
  E.kind = -1;
  if (t < s.n_cams) {
    E = cam_emit(as_cam(raw));
  } else if (t >= mc && t - mc < s.n_guards) {
    Guard gd = as_guard(raw);
    gd.idx = 0;
    gd.pos = gd.pos0;
    Guard* gp = eb.guards + (uint32_t)(t - mc);
    gp->idx = 0;
    gp->pos = gd.pos0;
    if (gd.hslot != kUncached) {  // heading kept (environment.py:204-208): cone of (0, hslot)
      stage_guard_cone(p, e, L, t - mc, gd, false);
      gp->nslot = (uint8_t)L.cone[16 * (t - mc) + 15];
    }
    E = guard_emit(gd);
  }
  publish_emitters(L, E, n_slot);
  raycast_pass<NT, U, D>(p, e, smem, L, n_slot, mc);
  write_obs<NT>(p, e, s, L, 0, obs);
  if (t == 0) p.scal[e] = s;
}

// ---------------------------------------------------------------------------
// layout placement + BFS
// ---------------------------------------------------------------------------

// The padded stop map of tile grid g (1 = wall or outside the grid; the layout of
// EnvLds::wall) into p.stop for env e, bit-packed (bit k of byte j = padded cell 8 j + k),
// by threads lane, lane + stride, ...  Built once per layout; step and reset expand it into
// the LDS byte plane with the rest of the prefetch (expand_stop), 1 bit of HBM per cell.
__device__ __forceinline__ void write_stop_map(const EnvParams& p, int e, const uint8_t* g, int lane, int stride) {
  const int R = p.R, C = p.C, PC = C + 2 * kRing, nb = (R + 2 * kRing) * PC;
  uint8_t* stp = p.stop + (size_t)e * p.stop_bytes;
  for (int j = lane; j < p.stop_bytes; j += stride) {
    uint32_t bits = 0;
    for (int k = 0; k < 8; ++k) {
      const int i = 8 * j + k;
      const int pr = i / PC;
      const int r = pr - kRing, c = i - pr * PC - kRing;
      const bool out = i >= nb || (unsigned)r >= (unsigned)R || (unsigned)c >= (unsigned)C;
      if (out || g[r * C + c] == kWall) bits |= 1u << k;
    }
    stp[j] = (uint8_t)bits;
  }
}

// Packed stop map bytes per env: 16-aligned, so its expansion (8 x) ends inside the LDS
// wall plane for every D (a multiple of 128 >= padded_bytes).
int stop_map_bytes(int R, int C) { return (int)align16((size_t)(padded_bytes(R, C) + 7) / 8); }

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

__global__ __launch_bounds__(64) void set_layout_kernel(EnvParams p, int max_walls, const int32_t* __restrict__ wall_rc,
                                                         const int32_t* __restrict__ n_walls,
                                                         const double* __restrict__ cam_params,
                                                         const int32_t* __restrict__ n_cams,
                                                         const int32_t* __restrict__ guard_paths,
                                                         const int32_t* __restrict__ guard_meta,
                                                         const double* __restrict__ guard_fov,
                                                         const int32_t* __restrict__ n_guards,
                                                         const int32_t* __restrict__ budget,
                                                         const uint8_t* __restrict__ mask,
                                                         uint8_t* __restrict__ valid_out) {
  __shared__ uint8_t g[kMaxDim * kMaxDim];
  __shared__ int cnt[4];
  const int e = blockIdx.x;
  if (mask && !mask[e]) return;
  const int lane = threadIdx.x;
  const int R = p.R, C = p.C;
  // _reset_layout + create_empty_grid (environment.py:169-177, utils.py:131-139)
  for (int i = lane; i < p.RC; i += 64) {
    const int r = i / C, c = i - (i / C) * C;
    g[i] = (r == 0 || r == R - 1 || c == 0 || c == C - 1) ? kWall : kEmpty;
  }
  __syncthreads();
  if (lane == 0) {
    g[p.sr * C + p.sc] = kStart;
    g[p.vr * C + p.vc] = kVault;
    const int total = budget[e];
    int spent = 0, nw = 0, nc = 0, ng = 0;
    auto placeable = [&](int r, int c) {  // environment.py:160-167
      return r > 0 && r < R - 1 && c > 0 && c < C - 1 && g[r * C + c] == kEmpty;
    };
    const int wn = min(n_walls[e], max_walls);
    for (int i = 0; i < wn; ++i) {  // :118-121
      const int r = wall_rc[((size_t)e * max_walls + i) * 2], c = wall_rc[((size_t)e * max_walls + i) * 2 + 1];
      if (placeable(r, c) && total - spent >= 1) {
        spent += 1;
        g[r * C + c] = kWall;
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
        g[r * C + c] = kCamera;
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
          dst[k] = (uint16_t)pack_rc(pr, pc);
        }
        Guard gd;
        gd.fov = guard_fov[(size_t)e * p.max_guards + i];
        gd.heading = 0.0;
        gd.idx = 0;
        int st = gm[1] % len;  // Python % (non-negative for len > 0)
        if (st < 0) st += len;
        gd.step = (int16_t)st;
        gd.len = (int16_t)len;
        gd.range = (int16_t)gm[2];
        gd.num_rays = (int16_t)num_rays_for(gd.fov);
        gd.pos = dst[0];
        gd.pos0 = dst[0];
        gd.hslot = kUncached;  // guard_cone_kernel fills the cone cache next
        gd.nslot = kUncached;
        p.guards[(size_t)e * p.max_guards + ng] = gd;
        g[unpack_r(dst[0]) * C + unpack_c(dst[0])] = kGuard;
        ++ng;
      }
    }
    cnt[0] = nw; cnt[1] = nc; cnt[2] = ng; cnt[3] = spent;
  }
  __syncthreads();
  uint64_t m = 0;
  if (lane < R)
    for (int c = 0; c < C; ++c)
      if (g[lane * C + c] != kWall) m |= 1ull << c;
  const bool ok = bfs_wave(m, p.sr, p.sc, p.vr, p.vc);
  uint8_t* dst = p.grid + (size_t)e * p.RC;
  for (int i = lane; i < p.RC; i += 64) dst[i] = g[i];
  write_stop_map(p, e, g, lane, 64);
  if (lane == 0) {
    EnvScalars* s = p.scal + e;
    s->n_walls = cnt[0];
    s->n_cams = cnt[1];
    s->n_guards = cnt[2];
    s->spent = cnt[3];
    valid_out[e] = ok ? 1 : 0;
  }
}

// Guard cone cache (heist_device.h), one wave per (env, guard), run right after
// set_layout_kernel: the guard's distinct headings (the initial one, then the direction of
// every patrol move, as guard_heading_after computes it), the heading slot each patrol
// point is entered with, and the cone of every (patrol index, heading slot) cast on the
// exact fp64 path (security.py:161-192, the same arithmetic as ray_mode 1).  A guard that
// does not fit the cache (patrol > kConePath points, > kConeSlots headings, range >
// kConeRange) keeps hslot = kUncached and is raycast live by step/reset.
template <int D>
__global__ __launch_bounds__(64) void guard_cone_kernel(EnvParams p, const uint8_t* __restrict__ mask) {
  constexpr int U = 4;
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ double heads[kConeSlots];
  __shared__ uint8_t arr[kConePath];  // heading slot on entering patrol point j; kUncached: no move
  __shared__ int n_heads;
  const int e = blockIdx.x, g = blockIdx.y;
  const int lane = threadIdx.x;
  if (mask && !mask[e]) return;
  if (g >= p.scal[e].n_guards) return;
  Guard* gp = p.guards + (size_t)e * p.max_guards + g;
  const Guard gd = *gp;
  const int len = gd.len;
  if (!p.guard_cones || len < 1 || len > kConePath || gd.range < 0 || gd.range > kConeRange) return;
  const int R = p.R, C = p.C;
  const EnvLds L = carve<D>(smem, R, C, 1, kConePath, 1);
  const uint8_t* ss = p.stop + (size_t)e * p.stop_bytes;
  for (int i = lane; i < p.stop_bytes; i += 64) expand_stop(L.wall, i, ss[i]);
  if (lane < len) L.path[lane] = p.paths[((size_t)e * p.max_guards + g) * p.max_path + lane];
  __syncthreads();
  if (lane == 0) {
    int nh = 1;
    heads[0] = gd.heading;  // 0.0 after set_layout (security.py:130)
    for (int j = 0; j < len; ++j) {
      int i0 = j - gd.step;  // the patrol point a move into j starts from (step in [0, len))
      if (i0 < 0) i0 += len;
      const int dr = unpack_r(L.path[j]) - unpack_r(L.path[i0]), dc = unpack_c(L.path[j]) - unpack_c(L.path[i0]);
      if (len < 2 || (dr == 0 && dc == 0)) {  // security.py:147, :158: heading unchanged
        arr[j] = kUncached;
        continue;
      }
      const double h = guard_heading_after(p, dr, dc, 0.0);
      int k = 0;
      while (k < nh && heads[k] != h) ++k;
      if (k == nh) {
        if (nh == kConeSlots) {
          nh = 0;  // too many headings: not cached
          break;
        }
        heads[nh++] = h;
      }
      arr[j] = (uint8_t)k;
    }
    n_heads = nh;
  }
  __syncthreads();
  const int nh = n_heads;
  if (nh == 0) return;
  uint32_t* v4 = reinterpret_cast<uint32_t*>(L.vis);
  for (int st = 0; st < len * nh; ++st) {
    const int i = st / nh, h = st - i * nh;
    for (int q = lane; q < (padded_bytes(R, C) + 3) / 4; q += 64) v4[q] = 0u;
    __syncthreads();
    Emit E;
    E.hmh = heads[h] - gd.fov / 2.0;  // security.py:173-178
    E.fov = gd.fov;
    E.step = 0.0;
    E.row = unpack_r(L.path[i]);
    E.col = unpack_c(L.path[i]);
    E.range = gd.range;
    E.num_rays = gd.num_rays;
    E.first = 0;
    E.kind = 1;
    E.members = 1;
    for (int ray = lane; ray <= E.num_rays; ray += 64) exact_ray<U, D>(smem, E, ray, L.PC, 0, p.half_deg);
    __syncthreads();
    if (lane < kConeEntry) {
      uint32_t bits = 0;
      if (lane >= 16) {  // the pose the entry names: heading of slot h, patrol point i
        const uint64_t hb = __builtin_bit_cast(uint64_t, heads[h]);
        bits = lane < 20 ? (uint32_t)(hb >> (16 * (lane - 16))) & 0xffffu : (lane == 20 ? (uint32_t)L.path[i] : 0u);
      } else if (lane < 2 * kConeRange + 1) {
        const int rr = E.row + lane - kConeRange;
        if ((unsigned)rr < (unsigned)R)
          for (int j = 0; j < 2 * kConeRange + 1; ++j) {
            const int cc = E.col + j - kConeRange;
            if ((unsigned)cc < (unsigned)C && (L.vis[L.at(rr, cc)] || (rr == E.row && cc == E.col))) bits |= 1u << j;
          }
      } else {  // the heading slot after the next move (step_kernel's guard update)
        int i2 = i + gd.step;
        if (i2 >= len) i2 -= len;
        bits = (len >= 2 && arr[i2] != kUncached) ? arr[i2] : (uint32_t)h;
      }
      p.cones[cone_entry(p, e, g, i, h) + lane] = (uint16_t)bits;
    }
    __syncthreads();
  }
  if (lane == 0) {  // state (patrol point 0, initial heading)
    const int i2 = gd.step < len ? gd.step : 0;
    gp->hslot = 0;
    gp->nslot = (len >= 2 && arr[i2] != kUncached) ? arr[i2] : 0;
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

template <int D>
__global__ __launch_bounds__(64) void cones_kernel(int R, int C, const uint8_t* __restrict__ walls,
                                                    const int32_t* __restrict__ meta, const double* __restrict__ params,
                                                    uint8_t* __restrict__ out, int ray_mode) {
  constexpr int U = 4;
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const int RC = R * C;
  const EnvLds L = carve<D>(smem, R, C, 1, 0, 1);
  for (int i = lane; i < RC; i += 64) L.grid[i] = walls[(size_t)e * RC + i] ? kWall : kEmpty;
  for (int i = lane; i < padded_bytes(R, C); i += 64) L.vis[i] = 0;
  if (lane == 0) {
    const int kind = meta[e * 4], row = meta[e * 4 + 1], col = meta[e * 4 + 2], range = meta[e * 4 + 3];
    const double fov = params[e * 2], heading = params[e * 2 + 1];
    Emit E;
    E.hmh = heading - fov / 2.0;
    E.fov = fov;
    E.row = row; E.col = col; E.range = range; E.num_rays = num_rays_for(fov);
    E.step = fov / (double)E.num_rays;
    E.first = 0; E.kind = kind; E.members = 1;
    L.em[0] = E;
    L.meta[0] = 1;
    L.meta[1] = (E.num_rays + 1 + 63) / 64;  // 64-ray chunks (publish_emitters)
  }
  __syncthreads();
  build_wall_map<64>(L.grid, L, R, C);
  __syncthreads();
  cast_rays<64, U, D, false>(smem, L, ray_mode, 0, nullptr);
  __syncthreads();
  for (int i = lane; i < RC; i += 64) {
    const int r = i / C;
    out[(size_t)e * RC + i] = L.vis[L.at(r, i - r * C)];
  }
}

// heist_cone_order: the reference's LIST order of a cone (security.py:53-101 appends a tile
// when a ray first reaches it: rays in index order, samples in distance order).  One
// emitter per block on the exact fp64 path; every reached tile keeps the smallest
// (ray << 12 | sample) key (LDS atomic min), 0xFFFFFFFF where no ray reached it.  Sorting
// the reached tiles by key gives get_vision_cone_tiles' order.
template <int D>
__global__ __launch_bounds__(64) void cone_order_kernel(int R, int C, const uint8_t* __restrict__ walls,
                                                         const int32_t* __restrict__ meta,
                                                         const double* __restrict__ params,
                                                         uint32_t* __restrict__ keys_out) {
  constexpr int U = 4;
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const int RC = R * C;
  const EnvLds L = carve<D>(smem, R, C, 1, 0, 1);
  uint32_t* keys = reinterpret_cast<uint32_t*>(smem + env_lds_bytes(R, C, 1, 0, D, 1));  // [padded] u32
  for (int i = lane; i < RC; i += 64) L.grid[i] = walls[(size_t)e * RC + i] ? kWall : kEmpty;
  for (int i = lane; i < padded_bytes(R, C); i += 64) keys[i] = 0xFFFFFFFFu;
  __syncthreads();
  build_wall_map<64>(L.grid, L, R, C);
  __syncthreads();
  Emit E;
  E.kind = meta[e * 4];
  E.row = meta[e * 4 + 1];
  E.col = meta[e * 4 + 2];
  E.range = meta[e * 4 + 3];
  E.fov = params[e * 2];
  E.hmh = params[e * 2 + 1] - E.fov / 2.0;
  E.num_rays = num_rays_for(E.fov);
  E.step = E.fov / (double)E.num_rays;
  E.first = 0;
  E.members = 1;
  for (int ray = lane; ray <= E.num_rays; ray += 64) exact_ray<U, D, true>(smem, E, ray, L.PC, 0, nullptr, keys);
  __syncthreads();
  for (int i = lane; i < RC; i += 64) {
    const int r = i / C;
    keys_out[(size_t)e * RC + i] = keys[L.at(r, i - r * C)];
  }
}

__global__ void init_kernel(EnvParams p) {  // one thread per env
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.n_envs) return;
  p.order[e] = e;
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
  write_stop_map(p, e, g, 0, 1);
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

__global__ __launch_bounds__(256) void sincos_kernel(const double* __restrict__ x, int64_t n,
                                                     double* __restrict__ so, double* __restrict__ co) {
  __shared__ double tab[kTabDoubles];
  for (int i = threadIdx.x; i < kTabDoubles; i += blockDim.x) tab[i] = kSinCosTab[i];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    heist_trig::sincos(x[i], tab, so + i, co + i);
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------

static size_t env_lds(const EnvParams& p) {
  return env_lds_bytes(p.R, p.C, p.max_cams + p.max_guards, p.max_guards * p.max_path, p.vis_gap, p.step_waves,
                       p.max_guards);
}

// Block -> env dispatch order for step/reset (longest-processing-time first): envs sorted
// by a raycast cost estimate, sum over emitters of (num_rays + 1) * samples per ray, in
// descending 1024-bucket counting-sort order.  The workgroup dispatcher hands out blocks
// in index order, so the heaviest envs start in the first round and the light ones fill
// the tail.  Results do not depend on the order (envs are independent); the order within
// a bucket is whatever the LDS atomics produce.  One workgroup; runs once per set_layout.
__global__ __launch_bounds__(1024) void order_kernel(EnvParams p) {
  __shared__ int bucket[1024];
  const int t = threadIdx.x;
  bucket[t] = 0;
  __syncthreads();
  auto key = [&](int e) {
    const EnvScalars& s = p.scal[e];
    int cost = 0;
    for (int c = 0; c < s.n_cams; ++c) {
      const Cam& cm = p.cams[(size_t)e * p.max_cams + c];
      cost += (cm.num_rays + 1) * 2 * cm.range;
    }
    for (int g = 0; g < s.n_guards; ++g) {
      const Guard& gd = p.guards[(size_t)e * p.max_guards + g];
      if (gd.hslot == kUncached) cost += (gd.num_rays + 1) * gd.range;
    }
    const int b = cost >> 5;
    return 1023 - (b < 1023 ? b : 1023);  // descending cost
  };
  for (int e = t; e < p.n_envs; e += 1024) atomicAdd(&bucket[key(e)], 1);
  __syncthreads();
  if (t == 0) {
    int run = 0;
    for (int b = 0; b < 1024; ++b) {
      const int c = bucket[b];
      bucket[b] = run;
      run += c;
    }
  }
  __syncthreads();
  // rank i (heaviest first) -> block.  dispatch_order 1: block i.  2 (snake draft): the
  // K-tick kernels keep every block of a launch resident (16 per CU), the k-th block a CU
  // receives (block n_cu * k + cu) lands on SIMD k % 4, and a SIMD's time is the sum of its 4
  // envs' ticks -- so ranks are dealt to the 4 n_cu SIMDs round by round in alternating
  // direction (round r = rank / (4 n_cu)), which evens the SIMD sums (heaviest-first alone
  // gives SIMD 0 of every CU the heaviest env of each round); a last partial round keeps its
  // ranks.
  const int S = 4 * p.n_cu, full = p.dispatch_order == 2 && p.n_cu > 0 ? p.n_envs / S * S : 0;
  for (int e = t; e < p.n_envs; e += 1024) {
    const int i = atomicAdd(&bucket[key(e)], 1);
    int b = i;
    if (i < full) {
      const int r = i / S, pos = i - r * S, sl = (r & 1) ? S - 1 - pos : pos;
      const int cu = sl % p.n_cu, simd = sl / p.n_cu;
      b = p.n_cu * (4 * r + simd) + cu;
    }
    // the wave priority (s_setprio) of the env's K-tick lean launch by cost rank i: the
    // heaviest envs get the SIMD first, the light ones fill their latency gaps
    // (prio_mode 1: quartiles 3 / 2 / 1 / 0; 2: top 1/16 -> 3, next 1/16 -> 2, next 1/8 -> 1;
    // 3: top 1/8 -> 1)
    const long long f16 = 16LL * i / (p.n_envs > 0 ? p.n_envs : 1);
    int pr = 0;
    if (p.prio_mode == 1) pr = 3 - (int)(f16 >> 2);
    else if (p.prio_mode == 2) pr = f16 < 1 ? 3 : (f16 < 2 ? 2 : (f16 < 4 ? 1 : 0));
    else if (p.prio_mode == 3) pr = f16 < 2 ? 1 : 0;
    p.order[b] = e | (pr << 24);
  }
}

hipError_t launch_order(const EnvParams& p, hipStream_t st) {
  hipLaunchKernelGGL(order_kernel, dim3(1), dim3(1024), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_init(const EnvParams& p, hipStream_t st) {
  hipLaunchKernelGGL(init_kernel, dim3((p.n_envs + 255) / 256), dim3(256), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_guard_cones(const EnvParams& p, const uint8_t* mask, hipStream_t st) {
  if (p.max_guards == 0 || !p.guard_cones) return hipSuccess;
  const size_t lds = env_lds_bytes(p.R, p.C, 1, kConePath, p.vis_gap, 1);
  if (p.vis_gap == 1024)
    hipLaunchKernelGGL(guard_cone_kernel<1024>, dim3(p.n_envs, p.max_guards), dim3(64), lds, st, p, mask);
  else if (p.vis_gap == 2048)
    hipLaunchKernelGGL(guard_cone_kernel<2048>, dim3(p.n_envs, p.max_guards), dim3(64), lds, st, p, mask);
  else
    hipLaunchKernelGGL(guard_cone_kernel<6144>, dim3(p.n_envs, p.max_guards), dim3(64), lds, st, p, mask);
  return hipGetLastError();
}

hipError_t launch_set_layout(const EnvParams& p, int max_walls, const int32_t* wall_rc, const int32_t* n_walls,
                             const double* cam_params, const int32_t* n_cams, const int32_t* guard_paths,
                             const int32_t* guard_meta, const double* guard_fov, const int32_t* n_guards,
                             const int32_t* budget, const uint8_t* mask, uint8_t* valid_out, hipStream_t st) {
  hipLaunchKernelGGL(set_layout_kernel, dim3(p.n_envs), dim3(64), 0, st, p, max_walls, wall_rc, n_walls, cam_params,
                     n_cams, guard_paths, guard_meta, guard_fov, n_guards, budget, mask, valid_out);
  return hipGetLastError();
}

// (waves per env W, samples per ray chunk U, min waves per SIMD O, stop-map -> vis gap D)
// variants; (2, 4, 8, D) is the default for either D.
#define HEIST_ENV_VARIANTS(X) \
  X(2, 4, 8, 1024) X(2, 4, 8, 2048) X(2, 4, 8, 6144) X(4, 4, 8, 1024) X(4, 4, 8, 2048) X(4, 4, 8, 6144) \
  X(1, 4, 8, 1024)

// the plane gap D: 1024 up to 20 x 20, 2048 up to 33 x 33 (BASELINE C5's 32 x 32), 6144 up to 64 x 64
int vis_gap_for(int R, int C) {
  const int b = padded_bytes(R, C);
  return b <= 1024 ? 1024 : (b <= 2048 ? 2048 : 6144);
}

bool env_variant_exists(int W, int U, int O, int D) {
#define HEIST_HAS_CASE(W_, U_, O_, D_) \
  if (W == W_ && U == U_ && O == O_ && D == D_) return true;
  HEIST_ENV_VARIANTS(HEIST_HAS_CASE)
#undef HEIST_HAS_CASE
  return false;
}

hipError_t launch_reset(const EnvParams& p, const uint8_t* mask, float* obs, hipStream_t st) {
  const size_t lds = env_lds(p);
#define HEIST_RESET_CASE(W, U, O, D)                                                                    \
  if (p.step_waves == W && p.ray_chunk == U && p.step_occ == O && p.vis_gap == D) {                    \
    hipLaunchKernelGGL((reset_kernel<W, U, O, D>), dim3(p.n_envs), dim3(64 * W), lds, st, p, mask, obs); \
    return hipGetLastError();                                                                          \
  }
  HEIST_ENV_VARIANTS(HEIST_RESET_CASE)
#undef HEIST_RESET_CASE
  return hipErrorInvalidValue;
}

// The profiling variant (HEIST_PROBE_MODE != 0) exists for the default 20 x 20 geometry only.
static hipError_t launch_step_probe(const EnvParams& p, const int64_t* actions, float* obs, float* rew, double* rew64,
                                    uint8_t* done_out, int8_t* status_out, int auto_reset, size_t lds, hipStream_t st) {
  if (p.step_waves != 2 || p.ray_chunk != 4 || p.step_occ != 8 || p.vis_gap != 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL((step_kernel<2, 4, 8, 1024, false, false, true>), dim3(p.n_envs), dim3(128), lds, st, p, actions,
                     obs, rew, rew64, done_out, status_out, auto_reset);
  return hipGetLastError();
}

hipError_t launch_step(const EnvParams& p, const int64_t* actions, float* obs, float* rew, double* rew64,
                       uint8_t* done_out, int8_t* status_out, int auto_reset, hipStream_t st) {
  const size_t lds = env_lds(p);
#define HEIST_STEP_CASE(W, U, O, D)                                                                       \
  if (p.step_waves == W && p.ray_chunk == U && p.step_occ == O && p.vis_gap == D) {                      \
    if (p.probe_mode)                                                                                    \
      return launch_step_probe(p, actions, obs, rew, rew64, done_out, status_out, auto_reset, lds, st);  \
    if (p.stamps)                                                                                        \
      hipLaunchKernelGGL((step_kernel<W, U, O, D, true, false>), dim3(p.n_envs), dim3(64 * W), lds, st, p, \
                         actions, obs, rew, rew64, done_out, status_out, auto_reset);                    \
    else if (p.sample_counter || p.redo_counter)                                                         \
      hipLaunchKernelGGL((step_kernel<W, U, O, D, false, true>), dim3(p.n_envs), dim3(64 * W), lds, st, p, \
                         actions, obs, rew, rew64, done_out, status_out, auto_reset);                    \
    else                                                                                                 \
      hipLaunchKernelGGL((step_kernel<W, U, O, D, false, false>), dim3(p.n_envs), dim3(64 * W), lds, st, p, \
                         actions, obs, rew, rew64, done_out, status_out, auto_reset);                    \
    return hipGetLastError();                                                                            \
  }
  HEIST_ENV_VARIANTS(HEIST_STEP_CASE)
#undef HEIST_STEP_CASE
  return hipErrorInvalidValue;
}

// K ticks per launch: the (W, U, O, D) variants below, for grids with C % 4 == 0 (the
// observation rows go out as float4 quads that never cross a grid row); another
// configuration runs K single-tick launches instead (same results).
#define HEIST_MULTI_VARIANTS(X) \
  X(2, 4, 8, 1024) X(2, 4, 8, 2048) X(2, 4, 8, 6144) X(4, 4, 8, 1024) X(4, 4, 8, 2048) X(4, 4, 8, 6144) \
  X(1, 4, 4, 1024) X(1, 4, 4, 2048) X(2, 4, 6, 1024) X(2, 4, 7, 1024) X(1, 4, 5, 1024) X(1, 4, 6, 1024)

bool multi_variant_exists(int W, int U, int O, int D) {
#define HEIST_HAS_MULTI(W_, U_, O_, D_) \
  if (W == W_ && U == U_ && O == O_ && D == D_) return true;
  HEIST_MULTI_VARIANTS(HEIST_HAS_MULTI)
#undef HEIST_HAS_MULTI
  return false;
}

size_t step_multi_lds(const EnvParams& p, int K) {
  const int n_slot = p.max_cams + p.max_guards;
  return align16(env_lds_bytes(p.R, p.C, n_slot, p.max_guards * p.max_path, p.vis_gap, p.multi_waves, p.max_guards)) +
         32 * (size_t)n_slot + align16((size_t)K) + (size_t)p.vis_gap +
         align16(sizeof(TieBuckets)) + 1024 * (size_t)p.multi_waves + (p.stamps ? 80 * (size_t)p.multi_waves : 0);
}

// Two waves per env for the 32 x 32 lean kernel (HEIST_LEAN_WAVES: 0 auto, 1, 2): auto when
// the batch's doubled waves still fit the chip at the kernel's 4 waves per SIMD.
bool lean_two_waves(const EnvParams& p) {
  if (p.lean_waves != 0) return p.lean_waves == 2;
  return 2 * (size_t)p.n_envs <= 16 * (size_t)(p.n_cu > 0 ? p.n_cu : 256);
}

hipError_t launch_step_multi(const EnvParams& p, int K, const int64_t* actions, float* obs,
                             float* rew, double* rew64, uint8_t* done_out, int8_t* status_out, int auto_reset,
                             hipStream_t st) {
  const size_t lds = step_multi_lds(p, K);
  if (p.probe_mode >= 1 && p.probe_mode <= 4 && p.ray_chunk == 4 && p.vis_gap == 1024 &&
      ((p.multi_waves == 2 && p.multi_occ == 8) || (p.multi_waves == 1 && p.multi_occ == 4))) {
    // profiling variants (default 20 x 20 geometry only)
#define HEIST_PROBE_CASE(W_, O_, M)                                                                              \
  if (p.multi_waves == W_ && p.probe_mode == M)                                                                \
    hipLaunchKernelGGL((step_multi_kernel<W_, 4, O_, 1024, false, M>), dim3(p.n_envs), dim3(64 * W_), lds, st, p, K, \
                       actions, obs, rew, rew64, done_out, status_out, auto_reset);
    HEIST_PROBE_CASE(2, 8, 1) HEIST_PROBE_CASE(2, 8, 2) HEIST_PROBE_CASE(2, 8, 3) HEIST_PROBE_CASE(2, 8, 4)
    HEIST_PROBE_CASE(1, 4, 1) HEIST_PROBE_CASE(1, 4, 2) HEIST_PROBE_CASE(1, 4, 3) HEIST_PROBE_CASE(1, 4, 4)
#undef HEIST_PROBE_CASE
    return hipGetLastError();
  }
  // the lean one-wave kernel (step_lean_kernel): the default for 20 x 20 grids at one wave per env
  // (20 x 20 at one wave per env; 32 x 32 at any batch size: its lean form is one wave per env
  // whatever multi_waves says, the envs it cannot serve taking the one-wave generic body)
  const bool lean20 = p.multi_waves == 1 && p.R == 20 && p.C == 20 && p.vis_gap == 1024;
  const bool lean32 = p.R == 32 && p.C == 32 && p.vis_gap == 2048;
#ifdef HEIST_LEAN_PROBES  // profiling variants of the lean kernel (tools/build_variant.sh ... -DHEIST_LEAN_PROBES)
  if (p.lean && lean20 && p.probe_mode >= 21 && p.probe_mode <= 28 && !p.stamps &&
      p.max_cams + p.max_guards <= kMaxEmitters) {
    if (p.fan_on && p.fan_fill) hipLaunchKernelGGL(fan_kernel, dim3(kFanTicks), dim3(kFanRays), 0, st, p);
    const size_t lds_l = lean_lds_bytes(p, K);
#define HEIST_LEAN_PROBE(M)                                                                                       \
  if (p.probe_mode == M)                                                                                          \
    hipLaunchKernelGGL((step_lean_kernel<20, 20, false, M>), dim3(p.n_envs), dim3(64), lds_l, st, p, K, actions, obs, \
                       rew, rew64, done_out, status_out, auto_reset);
    HEIST_LEAN_PROBE(21) HEIST_LEAN_PROBE(22) HEIST_LEAN_PROBE(23) HEIST_LEAN_PROBE(24) HEIST_LEAN_PROBE(25)
    HEIST_LEAN_PROBE(26) HEIST_LEAN_PROBE(27) HEIST_LEAN_PROBE(28)
#undef HEIST_LEAN_PROBE
    return hipGetLastError();
  }
#endif
  if (p.lean && (lean20 || lean32) && p.probe_mode == 0 && !p.sample_counter && !p.redo_counter &&
      p.max_cams + p.max_guards <= kMaxEmitters) {
    if (p.fan_on && p.fan_fill) hipLaunchKernelGGL(fan_kernel, dim3(kFanTicks), dim3(kFanRays), 0, st, p);
    const size_t lds_l = lean_lds_bytes(p, K);
    if (lean20 && p.stamps)
      hipLaunchKernelGGL((step_lean_kernel<20, 20, true>), dim3(p.n_envs), dim3(64), lds_l, st, p, K, actions, obs, rew,
                         rew64, done_out, status_out, auto_reset);
    else if (lean20)
      hipLaunchKernelGGL((step_lean_kernel<20, 20>), dim3(p.n_envs), dim3(64), lds_l, st, p, K, actions, obs, rew, rew64,
                         done_out, status_out, auto_reset);
    else if (p.stamps)
      hipLaunchKernelGGL((step_lean_kernel<32, 32, true>), dim3(p.n_envs), dim3(64), lds_l, st, p, K, actions, obs, rew,
                         rew64, done_out, status_out, auto_reset);
    else if (lean_two_waves(p))
      hipLaunchKernelGGL((step_lean_kernel<32, 32, false, 0, 2>), dim3(p.n_envs), dim3(128), lds_l, st, p, K, actions,
                         obs, rew, rew64, done_out, status_out, auto_reset);
    else
      hipLaunchKernelGGL((step_lean_kernel<32, 32>), dim3(p.n_envs), dim3(64), lds_l, st, p, K, actions, obs, rew,
                         rew64, done_out, status_out, auto_reset);
    return hipGetLastError();
  }
#define HEIST_MULTI_CASE(W, U, O, D)                                                                        \
  if (p.multi_waves == W && p.ray_chunk == U && p.multi_occ == O && p.vis_gap == D && p.probe_mode == 0 && \
      !p.sample_counter && !p.redo_counter && (p.C & 3) == 0) {                                            \
    if (p.fan_on && p.fan_fill) hipLaunchKernelGGL(fan_kernel, dim3(kFanTicks), dim3(kFanRays), 0, st, p);   \
    if (p.stamps)                                                                                            \
      hipLaunchKernelGGL((step_multi_kernel<W, U, O, D, true>), dim3(p.n_envs), dim3(64 * W), lds, st, p, K,  \
                         actions, obs, rew, rew64, done_out, status_out, auto_reset);                         \
    else                                                                                                     \
      hipLaunchKernelGGL((step_multi_kernel<W, U, O, D>), dim3(p.n_envs), dim3(64 * W), lds, st, p, K,        \
                         actions, obs, rew, rew64, done_out, status_out, auto_reset);                         \
    return hipGetLastError();                                                                                \
  }
  HEIST_MULTI_VARIANTS(HEIST_MULTI_CASE)
#undef HEIST_MULTI_CASE
  const size_t n = (size_t)p.n_envs;  // no K-tick variant (or instrumentation armed): K single-tick launches
  for (int k = 0; k < K; ++k) {
    const hipError_t e = launch_step(p, actions + k * n, obs + k * n * 3 * p.RC, rew + k * n, rew64 ? rew64 + k * n : nullptr,
                                     done_out + k * n, status_out + k * n, auto_reset, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
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
                        uint8_t* out, int ray_mode, hipStream_t st) {
  const int D = vis_gap_for(R, C);
  const size_t lds = env_lds_bytes(R, C, 1, 0, D, 1);
  if (D == 1024)
    hipLaunchKernelGGL(cones_kernel<1024>, dim3(n), dim3(64), lds, st, R, C, walls, meta, params, out, ray_mode);
  else if (D == 2048)
    hipLaunchKernelGGL(cones_kernel<2048>, dim3(n), dim3(64), lds, st, R, C, walls, meta, params, out, ray_mode);
  else
    hipLaunchKernelGGL(cones_kernel<6144>, dim3(n), dim3(64), lds, st, R, C, walls, meta, params, out, ray_mode);
  return hipGetLastError();
}

hipError_t launch_cone_order(int n, int R, int C, const uint8_t* walls, const int32_t* meta, const double* params,
                             uint32_t* keys_out, hipStream_t st) {
  const int D = vis_gap_for(R, C);
  const size_t lds = env_lds_bytes(R, C, 1, 0, D, 1) + 4 * (size_t)padded_bytes(R, C);
  if (D == 1024)
    hipLaunchKernelGGL(cone_order_kernel<1024>, dim3(n), dim3(64), lds, st, R, C, walls, meta, params, keys_out);
  else if (D == 2048)
    hipLaunchKernelGGL(cone_order_kernel<2048>, dim3(n), dim3(64), lds, st, R, C, walls, meta, params, keys_out);
  else
    hipLaunchKernelGGL(cone_order_kernel<6144>, dim3(n), dim3(64), lds, st, R, C, walls, meta, params, keys_out);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void fast_dir_kernel(const double* __restrict__ deg, int64_t n,
                                                       float* __restrict__ co, float* __restrict__ so) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
  {
    float xr;
    fast_dir(deg[i], co + i, so + i, &xr);
  }
}

hipError_t launch_fast_dir(const double* deg, int64_t n, float* co, float* so, hipStream_t st) {
  int64_t b = (n + 255) / 256;
  hipLaunchKernelGGL(fast_dir_kernel, dim3((unsigned)(b > 4096 ? 4096 : (b < 1 ? 1 : b))), dim3(256), 0, st, deg, n, co, so);
  return hipGetLastError();
}

hipError_t launch_sincos(const double* x, int64_t n, double* so, double* co, hipStream_t st) {
  int64_t b = (n + 255) / 256;
  hipLaunchKernelGGL(sincos_kernel, dim3((unsigned)(b > 4096 ? 4096 : (b < 1 ? 1 : b))), dim3(256), 0, st, x, n, so, co);
  return hipGetLastError();
}

}  // namespace heist
