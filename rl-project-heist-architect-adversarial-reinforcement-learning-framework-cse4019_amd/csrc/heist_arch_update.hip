// heist_arch_update.hip -- the Architect's per-layout update sequence as ONE persistent launch.
//
// The reference trains the Architect after every layout with a single transition
// (training.py:479-480 / :558-559 -> ArchitectAgent.update, agents/architect.py:91-155).
// With one reward the policy term carries no gradient (its log-prob was recorded under
// no_grad, :75-81) and the value target is the raw reward, so update i is
//     loss_i = value_coeff * (V(s0) - r_i)^2,   V = value_head(relu(fc_global(pool(encoder(s0)))))
// on the constant grid state s0 (networks.py:159-188), then clip_grad_norm_(0.5) and
// torch.optim.Adam (foreach, non-capturable) over the 12 value-path tensors.  The k updates
// of a sequence are strictly sequential; as separate launches each is a chain of ~60 tiny
// kernels (0.38 ms, launch bound).  Here 64 workgroups x 512 threads (one per CU) run all
// k steps in one launch with every parameter and Adam moment on chip, five grid barriers
// per step:
//
//   P1  a1 = relu(conv1(s0)) (all 32 planes, redundantly per WG, sparse in s0's nonzeros)
//       a2[w] = relu(conv2(a1))[w]           (WG w owns conv2/conv3 output channel w)   -> B1
//   P2  a3[w] = relu(conv3(a2))[w]; p[w] = adaptive_avg_pool(a3[w]) (16 cells);
//       gp[w] = fc_global.weight[:, 16w:16w+16] @ p[w]   (WG w owns those 16 columns)   -> B2
//   P3  g = relu(bf + sum_w gp[w]); h, v, dv, dh, dg (value head, redundantly per WG:
//       value_head.0.weight rides in registers); dp[w] = Wf[:, own]^T dg; da3[w];
//       dW3 row w, db3[w]; dWf own columns; dWv1 own slice (rows 2w, 2w+1)            -> B3
//   P4  da2[w] = (conv3^T da3)[w] * (a2[w] > 0); dW2 row w, db2[w]                     -> B4
//   P5  da1[w/2] on half w%2 of the rows; partial dW1, db1; per-tensor sum-of-squares   -> B5
//   P6  clip coefficient from the 12 tensor norms (norm of norms, as clip_grad_norm_);
//       Adam on every owned / redundant tensor; publish W2 / W3 rows and the Wv1 slice.
//
// Hand-offs between workgroups follow MI355X_MICROARCH.md's measured write-through form
// (hand-off table, third row): every handed-off float is stored with a `sc1` store, each
// storing wave drains (`s_waitcnt vmcnt(0)`), a workgroup barrier, one lane's agent-scope
// atomic add to a monotonic counter, a `global_load_dword sc1` poll, a workgroup barrier,
// and every load of handed-off data is an `sc1` load (dword or dwordx4).
//
// Numerics: fp32 throughout, as the eager step.  Sums run in a fixed order that differs
// from MIOpen's / hipBLASLt's, so results match the eager sequence to fp32 rounding (the
// tests bound it), not bit for bit.  The Adam arithmetic mirrors torch's _multi_tensor_adam
// (lerp, mul + addcmul, sqrt / bc2_sqrt + eps, addcdiv with -lr/bc1; bias corrections in
// float64 from the step count) and clip_grad_norm_ (per-tensor norms, their norm,
// max_norm / (total + 1e-6) clamped to 1, grads scaled before Adam).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "heist_device.h"

#pragma clang fp contract(off)

namespace heist {
namespace au {

constexpr int NT = 512;   // threads per workgroup: 8 waves, 2 per SIMD
constexpr int NWG = 64;   // workgroups = conv2 / conv3 output channels
constexpr int C1 = 32, C2 = 64, C3 = 64, HID = 256, VH = 128, NPOOL = C3 * 16;
constexpr int PLANE = 512;  // workspace floats per handed-off channel plane (R*C <= 400, padded to whole lines)
constexpr int REC = 32;     // floats per workgroup partial record (one 128-B line)
constexpr int MAXN = 400;   // R*C
// workspace layout (floats)
constexpr int WS_A2 = 0, WS_GP = WS_A2 + NWG * PLANE, WS_DA3 = WS_GP + NWG * HID, WS_DA2 = WS_DA3 + NWG * PLANE,
              WS_NP = WS_DA2 + NWG * PLANE, WS_CTR = WS_NP + NWG * REC, WS_FLOATS = WS_CTR + 64;

enum { W1, B1, W2, B2, W3, B3, WF, BF, WV1, BV1, WV2, BV2, NTENS };
// NP record slots
enum { NP_W2 = 0, NP_B2 = 1, NP_W3 = 2, NP_B3 = 3, NP_WF = 4, NP_WV1 = 5, NP_DW1 = 8, NP_DB1 = 17 };

struct Args {
  float* p[NTENS];
  float* m[NTENS];
  float* v[NTENS];
  const float* grid;    // [R][C] the constant input plane
  const float* target;  // [k] rewards
  float* vloss;         // [k] value losses
  float* ws;            // WS_FLOATS floats; ws + WS_CTR: barrier counter and timeout flag (zeroed per launch)
  unsigned long long* stamps;  // instrumentation (NULL: off): s_memrealtime per phase point
  int R, C, k;
  double step0, lr, beta1, beta2;
  float lerp_w, beta2f, c2, eps, max_norm, grad_out;
};

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// ---- LDS layout (floats) -------------------------------------------------------------
// BIG holds 64 zero-padded planes: row stride RS = C + 1 (one shared pad column), plane
// stride PS = (R + 1) * RS (one shared pad row); data (y, x) sits at (y + 1) * RS + x + 1.
struct Lds {
  int RS, PS, big, xp, w1, b1, bf, bv1, wv2, bv2, w2r, w3r, wcol, own, own2, red, g, h, dh, dg, p16, dp16, scal,
      nzpos, nzval, ptab, total;
};
__host__ __device__ inline int up4(int x) { return (x + 3) & ~3; }
__host__ __device__ inline Lds lds_layout(int R, int C) {
  Lds L;
  L.RS = C + 1;
  L.PS = (R + 1) * L.RS;
  int o = 0;
  L.big = o;  o += up4(NWG * L.PS + L.RS + 1);
  L.xp = o;   o += up4(L.PS + L.RS + 1);
  L.w1 = o;   o += 3 * C1 * 9;   // param, exp_avg, exp_avg_sq
  L.b1 = o;   o += 3 * C1;
  L.bf = o;   o += 3 * HID;
  L.bv1 = o;  o += 3 * VH;
  L.wv2 = o;  o += 3 * VH;
  L.bv2 = o;  o += 4;
  L.w2r = o;  o += C1 * 9;
  L.w3r = o;  o += C2 * 9;
  L.wcol = o; o += 64 * 9;
  L.own = o;  o += PLANE;
  L.own2 = o; o += PLANE;
  L.red = o;  o += 8 * 576;     // K-split partials (8 x 400), weight-grad partials (8 x 576 / 16 x 288), records
  L.g = o;    o += HID;
  L.h = o;    o += VH;
  L.dh = o;   o += VH;
  L.dg = o;   o += HID;
  L.p16 = o;  o += 16;
  L.dp16 = o; o += 16;
  L.scal = o; o += 64;
  L.nzpos = o; o += MAXN;
  L.nzval = o; o += MAXN;
  L.ptab = o; o += 3 * NTENS * 2;  // 36 tensor pointers (8-byte aligned: o is a multiple of 4)
  L.total = o;
  return L;
}
// scal slots
enum { S_V = 0, S_DV, S_CLIP, S_NS, S_BC2S, S_B2, S_B2M, S_B2V, S_B3, S_B3M, S_B3V, S_NNZ, S_DB3, S_DB2, S_DB1,
       S_NW2, S_NW3, S_NWF, S_NWV1, S_TIMEOUT, S_RED8 = 32 };

// ---- memory helpers ---------------------------------------------------------------------
__device__ __forceinline__ void st_sc1(float* p, float x) {
  __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store_dword ... sc1
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base, int n_floats) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, n_floats * 4, 0x00020000);
}
__device__ __forceinline__ f32x4_t ld4_sc1(__amdgpu_buffer_rsrc_t rs, int float_off) {
  return __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, float_off * 4, 0, 16));  // sc1
}
__device__ __forceinline__ float ld1_sc1(__amdgpu_buffer_rsrc_t rs, int float_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, float_off * 4, 0, 16));
}
// threadIdx.x / blockIdx.x behind an empty asm: address arithmetic derived from them is
// recomputed where it is used instead of being hoisted out of the step loop and kept live
// (or spilled) across every phase.
__device__ __forceinline__ int tid_o() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
__device__ __forceinline__ int wg_o() {
  int w = blockIdx.x;
  asm volatile("" : "+s"(w));
  return w;
}
__device__ __forceinline__ float rdl(float x, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), lane));
}

// Grid barrier number `idx` (0-based over the launch).  Every storing wave drains its sc1
// stores, the workgroup meets, one lane adds to the monotonic counter and polls it with a
// relaxed sc1 load.  The spin is bounded: on a timeout (co-residency lost) the flag is set,
// the host reports it, and later barriers stop waiting so the grid still drains.
__device__ __forceinline__ void grid_barrier(unsigned* ctr, unsigned idx, float* scal) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (idx + 1u) * (unsigned)NWG;
    if (scal[S_TIMEOUT] == 0.f) {
      unsigned spins = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 25)) {
          __hip_atomic_store(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          scal[S_TIMEOUT] = 1.f;
          break;
        }
      }
    }
  }
  __syncthreads();
}

// Deterministic workgroup sums of NV values (the same order in every workgroup): xor
// butterflies inside each wave, lane 0's total per wave, the 8 wave totals in order.
template <int NV>
__device__ __forceinline__ void block_sums(float (&x)[NV], float* scratch /* >= 8*NV */) {
  const int tid_ = tid_o();
  const int wv = tid_ >> 6, lane = tid_ & 63;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x[i] += __shfl_xor(x[i], o);
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) scratch[wv * NV + i] = x[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float s = 0.f;
    for (int w = 0; w < 8; ++w) s += scratch[w * NV + i];
    x[i] = s;
  }
  __syncthreads();
}

// ---- convolution pieces -----------------------------------------------------------------
// One lane's SR x SC output strip: sum over this wave's NCI input planes [ci0, ci0 + NCI) of
// the 3x3 convolution (FLIP: the transposed convolution's flipped taps) of padded LDS planes.
// The window starts at padded offset `base`; the wave's 9 * NCI weights ([ci][tap]) sit in
// wlo / whi (lane j holds weight j / 64 + j) and reach the FMAs as scalars (readlane).
template <int SR, int SC, int NCI, bool FLIP>
__device__ __forceinline__ void strip_conv(const float* __restrict__ big, int PS, int RS, int base, int ci0, float wlo,
                                           float whi, float (&acc)[SR][SC]) {
#pragma unroll 1
  for (int c = 0; c < NCI; ++c) {
    const float* pl = big + (ci0 + c) * PS + base;
    float in[SR + 2][SC + 2];
#pragma unroll
    for (int r = 0; r < SR + 2; ++r)
#pragma unroll
      for (int q = 0; q < SC + 2; ++q) in[r][q] = pl[r * RS + q];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int j = c * 9 + (FLIP ? 8 - (ky * 3 + kx) : ky * 3 + kx);  // wave-uniform
        const float wgt = rdl(j < 64 ? wlo : whi, j & 63);
#pragma unroll
        for (int r = 0; r < SR; ++r)
#pragma unroll
          for (int q = 0; q < SC; ++q) acc[r][q] = fmaf(wgt, in[r + ky][q + kx], acc[r][q]);
      }
  }
}

// Own-channel convolution over 8 * NCI input planes of BIG (8 waves split the planes):
// rows [y0, y0 + nrows) in SR-row strips, 2-column strips; returns, for thread t < the
// strip area's nrows * C, the sum of the 8 waves' partials (in wave order) at position
// (y0 + t / C, t % C); other threads get 0.  wsrc: LDS weights [8 * NCI][9].
template <int SR, int NCI, bool FLIP>
__device__ __forceinline__ float conv_own(const float* big, const Lds& L, int R, int C, int y0, int nrows,
                                          const float* wsrc, float* red) {
  const int tid_ = tid_o();
  const int wv = tid_ >> 6, lane = tid_ & 63;
  constexpr int NWT = 9 * NCI;
  const float wlo = lane < NWT ? wsrc[wv * NWT + lane] : 0.f;
  const float whi = lane + 64 < NWT ? wsrc[wv * NWT + 64 + lane] : 0.f;
  const int nsx = C >> 1, ns = (nrows / SR) * nsx, npos = nrows * C;
  // Every lane runs the strip loop (lanes past the last strip redo strip 0 and store
  // nothing): readlane reads the weights of lanes an exec mask would otherwise switch off.
  const int sl = lane < ns ? lane : 0;
  const int sy = (sl / nsx) * SR, sx = (sl - (sl / nsx) * nsx) * 2;
  float acc[SR][2];
#pragma unroll
  for (int r = 0; r < SR; ++r) acc[r][0] = acc[r][1] = 0.f;
  strip_conv<SR, 2, NCI, FLIP>(big, L.PS, L.RS, (y0 + sy) * L.RS + sx, wv * NCI, wlo, whi, acc);
  if (lane < ns) {
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      red[wv * npos + (sy + r) * C + sx] = acc[r][0];
      red[wv * npos + (sy + r) * C + sx + 1] = acc[r][1];
    }
  }
  __syncthreads();
  float s = 0.f;
  if ((int)tid_ < npos) {
#pragma unroll
    for (int w = 0; w < 8; ++w) s += red[w * npos + tid_];
  }
  __syncthreads();
  return s;
}

// Weight-gradient partial of one input plane `ci`: acc[ky*3+kx] += sum over rows [ya, yb),
// columns [xa, xb) of d[y*C + x] * in_pad[ci][(y + ky) * RS + x + kx], sliding a 3x3 window
// along each row (3 new loads per position).
__device__ __forceinline__ void wgrad(const float* __restrict__ big, const Lds& L, int C, int ci, int ya, int yb,
                                      int xa, int xb, const float* __restrict__ d, float (&acc)[9]) {
  const int RS = L.RS;
  for (int y = ya; y < yb; ++y) {
    const float* pl = big + ci * L.PS + y * RS + xa;
    float a0 = pl[0], a1 = pl[RS], a2 = pl[2 * RS];
    float b0 = pl[1], b1 = pl[RS + 1], b2 = pl[2 * RS + 1];
    const float* drow = d + y * C;
    for (int x = xa; x < xb; ++x) {
      const float* cc = pl + (x - xa) + 2;
      const float c0 = cc[0], c1 = cc[RS], c2 = cc[2 * RS];
      const float dd = drow[x];
      acc[0] = fmaf(dd, a0, acc[0]); acc[1] = fmaf(dd, b0, acc[1]); acc[2] = fmaf(dd, c0, acc[2]);
      acc[3] = fmaf(dd, a1, acc[3]); acc[4] = fmaf(dd, b1, acc[4]); acc[5] = fmaf(dd, c1, acc[5]);
      acc[6] = fmaf(dd, a2, acc[6]); acc[7] = fmaf(dd, b2, acc[7]); acc[8] = fmaf(dd, c2, acc[8]);
      a0 = b0; a1 = b1; a2 = b2;
      b0 = c0; b1 = c1; b2 = c2;
    }
  }
}

// conv1 (1 -> 32) of the constant input plane into BIG planes [0, 32): relu(sum + b1), the
// sum over the input's nonzero pixels inside each 3x3 window in tap order (skipping the
// zero taps changes no bit of the dense sum).  Positions with no nonzero in their window
// hold relu(0 + b1); the few inside a nonzero's 3x3 neighbourhood are then recomputed
// (a position near two nonzeros is written twice with the same value).
__device__ __forceinline__ float conv1_at(const float* sm, const Lds& L, int ci, int y, int x);
__device__ __forceinline__ void conv1_all(float* sm, const Lds& L, int R, int C) {
  const int tid_ = tid_o();
  const int N = R * C, nnz = (int)sm[L.scal + S_NNZ];
  float* big = sm + L.big;
  for (int o = tid_; o < C1 * N; o += NT) {
    const int ci = o / N, pos = o - ci * N, y = pos / C, x = pos - y * C;
    big[ci * L.PS + (y + 1) * L.RS + x + 1] = fmaxf(0.f + sm[L.b1 + ci], 0.f);
  }
  __syncthreads();
  for (int o = tid_; o < C1 * 9 * nnz; o += NT) {
    const int ci = o & (C1 - 1), r = o >> 5, j = r / 9, tap = r - j * 9;
    const int pp = __float_as_int(sm[L.nzpos + j]);
    const int y = (pp >> 8) - tap / 3 + 1, x = (pp & 255) - (tap % 3) + 1;
    if ((unsigned)y < (unsigned)R && (unsigned)x < (unsigned)C)
      big[ci * L.PS + (y + 1) * L.RS + x + 1] = conv1_at(sm, L, ci, y, x);
  }
}

// a1[ci] at (y, x) (one value; same arithmetic as conv1_all)
__device__ __forceinline__ float conv1_at(const float* sm, const Lds& L, int ci, int y, int x) {
  const int nnz = (int)sm[L.scal + S_NNZ];
  float acc = 0.f;
  for (int j = 0; j < nnz; ++j) {
    const int pp = __float_as_int(sm[L.nzpos + j]);
    const int dy = (pp >> 8) - y + 1, dx = (pp & 255) - x + 1;
    if ((unsigned)dy < 3u && (unsigned)dx < 3u) acc = fmaf(sm[L.w1 + ci * 9 + dy * 3 + dx], sm[L.nzval + j], acc);
  }
  return fmaxf(acc + sm[L.b1 + ci], 0.f);
}

// channel planes [0, 64) of a workspace array (stride PLANE, sc1) into BIG's interiors
__device__ __forceinline__ void load_planes(const float* src, float* big, const Lds& L, int R, int C) {
  const int tid_ = tid_o();
  const __amdgpu_buffer_rsrc_t rs = rsrc(src, NWG * PLANE);
  const int nq = (R * C) >> 2, total = NWG * nq;  // C % 4 == 0: a quad stays in one row
  constexpr int MAXQ = (NWG * MAXN / 4 + NT - 1) / NT;
  f32x4_t v[MAXQ];
#pragma unroll
  for (int i = 0; i < MAXQ; ++i) {
    const int q = tid_ + i * NT;
    if (q < total) {
      const int p = q / nq, pos = (q - p * nq) * 4;
      v[i] = ld4_sc1(rs, p * PLANE + pos);
    }
  }
#pragma unroll
  for (int i = 0; i < MAXQ; ++i) {
    const int q = tid_ + i * NT;
    if (q < total) {
      const int p = q / nq, pos = (q - p * nq) * 4;
      const int y = pos / C, x = pos - y * C;
      float* d = big + p * L.PS + (y + 1) * L.RS + x + 1;
      d[0] = v[i].x; d[1] = v[i].y; d[2] = v[i].z; d[3] = v[i].w;
    }
  }
}

// Adam (torch _multi_tensor_adam, non-capturable, amsgrad/weight_decay off) on one element
// whose raw gradient is g; clip = clip_grad_norm_'s clamped coefficient.
__device__ __forceinline__ void adam(float& p, float& m, float& v, float g, float clip, const Args& a, float ns,
                                     float bc2s) {
  g = g * clip;                    // _foreach_mul_(grads, clip_coef_clamped)
  m = fmaf(a.lerp_w, g - m, m);    // _foreach_lerp_(exp_avgs, grads, 1 - beta1)
  v = v * a.beta2f;                // _foreach_mul_(exp_avg_sqs, beta2)
  v = fmaf(a.c2, g * g, v);        // _foreach_addcmul_(exp_avg_sqs, grads, grads, 1 - beta2)
  float d = sqrtf(v) / bc2s;       // _foreach_sqrt, _foreach_div_(bias_correction2_sqrt)
  d = d + a.eps;                   // _foreach_add_(eps)
  p = fmaf(ns, m / d, p);          // _foreach_addcdiv_(params, exp_avgs, denom, -lr / bc1)
}

template <int R, int C>
__global__ void __launch_bounds__(NT, 1) arch_update_kernel(Args a) {
  // STAMP(i): workgroups 0 and 63, steps < 16, 32 points per step (tools/probe_arch_update.py)
#define STAMP(i)                                                                                          \
  if (a.stamps && t == 0 && (w == 0 || w == NWG - 1) && s < 16)                                           \
    a.stamps[((w == 0 ? 0 : 1) * 16 + s) * 32 + (i)] = __builtin_amdgcn_s_memrealtime();
  extern __shared__ float sm[];
  constexpr int N = R * C;
  const int t = threadIdx.x, wv = t >> 6, lane = t & 63, w = blockIdx.x;
  const Lds L = lds_layout(R, C);
  float* big = sm + L.big;
  float* red = sm + L.red;
  float* scal = sm + L.scal;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.ws + WS_CTR);
  const int Npad = (N + 31) & ~31;  // handed-off planes are stored in whole 128-B lines

  // ---- setup: zero BIG + XP (the pads stay zero for the whole launch), load parameters ----
  for (int i = t; i < L.w1; i += NT) sm[i] = 0.f;
  if (t < 64) scal[t] = 0.f;
  if (t < 3 * NTENS) {
    float** tab = reinterpret_cast<float**>(sm + L.ptab);
    tab[t] = t < NTENS ? a.p[t] : t < 2 * NTENS ? a.m[t - NTENS] : a.v[t - 2 * NTENS];
  }
  __syncthreads();
  for (int i = t; i < N; i += NT) {
    const int y = i / C, x = i - y * C;
    sm[L.xp + (y + 1) * L.RS + x + 1] = a.grid[i];
  }
  for (int i = t; i < C1 * 9; i += NT) {
    sm[L.w1 + i] = a.p[W1][i]; sm[L.w1 + 288 + i] = a.m[W1][i]; sm[L.w1 + 576 + i] = a.v[W1][i];
  }
  if (t < C1) { sm[L.b1 + t] = a.p[B1][t]; sm[L.b1 + 32 + t] = a.m[B1][t]; sm[L.b1 + 64 + t] = a.v[B1][t]; }
  if (t < HID) { sm[L.bf + t] = a.p[BF][t]; sm[L.bf + 256 + t] = a.m[BF][t]; sm[L.bf + 512 + t] = a.v[BF][t]; }
  if (t < VH) {
    sm[L.bv1 + t] = a.p[BV1][t]; sm[L.bv1 + 128 + t] = a.m[BV1][t]; sm[L.bv1 + 256 + t] = a.v[BV1][t];
    sm[L.wv2 + t] = a.p[WV2][t]; sm[L.wv2 + 128 + t] = a.m[WV2][t]; sm[L.wv2 + 256 + t] = a.v[WV2][t];
  }
  if (t == 0) {
    sm[L.bv2] = a.p[BV2][0]; sm[L.bv2 + 1] = a.m[BV2][0]; sm[L.bv2 + 2] = a.v[BV2][0];
    scal[S_B2] = a.p[B2][w]; scal[S_B2M] = a.m[B2][w]; scal[S_B2V] = a.v[B2][w];
    scal[S_B3] = a.p[B3][w]; scal[S_B3M] = a.m[B3][w]; scal[S_B3V] = a.v[B3][w];
  }
  // owned: conv2 / conv3 row w (params in LDS, moments in registers)
  float m2 = 0.f, v2 = 0.f, m3a = 0.f, v3a = 0.f, m3b = 0.f, v3b = 0.f;
  if (t < C1 * 9) { sm[L.w2r + t] = a.p[W2][w * 288 + t]; m2 = a.m[W2][w * 288 + t]; v2 = a.v[W2][w * 288 + t]; }
  sm[L.w3r + t] = a.p[W3][w * 576 + t]; m3a = a.m[W3][w * 576 + t]; v3a = a.v[W3][w * 576 + t];
  if (t < 64) {
    sm[L.w3r + 512 + t] = a.p[W3][w * 576 + 512 + t];
    m3b = a.m[W3][w * 576 + 512 + t]; v3b = a.v[W3][w * 576 + 512 + t];
  }
  // owned: fc_global.weight columns 16w + [8*hf, 8*hf + 8) of row i = t >> 1
  const int fi = t >> 1, fhf = t & 1;
  float wf[8], mf[8], vf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int e = fi * NPOOL + 16 * w + 8 * fhf + j;
    wf[j] = a.p[WF][e]; mf[j] = a.m[WF][e]; vf[j] = a.v[WF][e];
  }
  // owned: value_head.0.weight element w * 512 + t (rows 2w, 2w + 1)
  const int ev = w * 512 + t;
  float pv1 = a.p[WV1][ev], mv1 = a.m[WV1][ev], vv1 = a.v[WV1][ev];
  __syncthreads();
  // the input's nonzero pixels in row-major order (wave 0, ballot compaction)
  if (wv == 0) {
    int cnt = 0;
    for (int base = 0; base < N; base += 64) {
      const int i = base + lane;
      float val = 0.f;
      if (i < N) { const int y = i / C, x = i - y * C; val = sm[L.xp + (y + 1) * L.RS + x + 1]; }
      const unsigned long long bal = __ballot(val != 0.f);
      const int before = __popcll(bal & ((1ull << lane) - 1ull));
      if (val != 0.f) {
        const int y = i / C, x = i - y * C;
        sm[L.nzpos + cnt + before] = __int_as_float((y << 8) | x);
        sm[L.nzval + cnt + before] = val;
      }
      cnt += __popcll(bal);
    }
    if (lane == 0) scal[S_NNZ] = (float)cnt;
  }
  __syncthreads();

  float a2keep = 0.f;    // a2[w] at position t (relu mask of P4)
  unsigned bar = 0;
  for (int s = 0; s < a.k; ++s) {
    const int t = tid_o(), wv = t >> 6, lane = t & 63, w = wg_o();
    const int fi = t >> 1, fhf = t & 1, ev = w * 512 + t;
    // ======== P1: conv1 (all planes), conv2 own channel ========
    STAMP(0)
    conv1_all(sm, L, R, C);
    __syncthreads();
    STAMP(15)
    {
      const float z = conv_own<4, 4, false>(big, L, R, C, 0, R, sm + L.w2r, red);
      if (t < N) a2keep = fmaxf(z + scal[S_B2], 0.f);
      if (t < Npad) st_sc1(a.ws + WS_A2 + w * PLANE + t, t < N ? a2keep : 0.f);
    }
    STAMP(16)
    STAMP(1)
    grid_barrier(ctr, bar++, scal);
    STAMP(2)

    // ======== P2: conv3 own channel, pool, fc_global partial ========
    load_planes(a.ws + WS_A2, big, L, R, C);
    __syncthreads();
    STAMP(12)
    // value_head.0.weight as 8x8 blocks (rows 8 * (t >> 5) + r, columns 8 * (t & 31) + c):
    // both h = W g (reduced over the 32 column blocks of a half-wave) and dg = W^T dh
    // (over the 16 row blocks) stay cheap.  In flight during conv3.
    float wb[64];
    {
      const __amdgpu_buffer_rsrc_t rs = rsrc(a.p[WV1], VH * HID);
      const int r0 = 8 * (t >> 5), c0 = 8 * (t & 31);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const f32x4_t q0 = ld4_sc1(rs, (r0 + r) * HID + c0), q1 = ld4_sc1(rs, (r0 + r) * HID + c0 + 4);
        wb[r * 8 + 0] = q0.x; wb[r * 8 + 1] = q0.y; wb[r * 8 + 2] = q0.z; wb[r * 8 + 3] = q0.w;
        wb[r * 8 + 4] = q1.x; wb[r * 8 + 5] = q1.y; wb[r * 8 + 6] = q1.z; wb[r * 8 + 7] = q1.w;
      }
    }
    STAMP(17)
    {
      const float z = conv_own<4, 8, false>(big, L, R, C, 0, R, sm + L.w3r, red);
      if (t < N) sm[L.own + t] = fmaxf(z + scal[S_B3], 0.f);
    }
    __syncthreads();
    STAMP(18)
    if (t < 16) {  // adaptive_avg_pool2d((4, 4)): window sum in row-major order, / kH / kW
      const int oy = t >> 2, ox = t & 3;
      const int ys = (oy * R) / 4, ye = ((oy + 1) * R + 3) / 4, xs = (ox * C) / 4, xe = ((ox + 1) * C + 3) / 4;
      float sum = 0.f;
      for (int y = ys; y < ye; ++y)
        for (int x = xs; x < xe; ++x) sum += sm[L.own + y * C + x];
      sm[L.p16 + t] = sum / (float)(ye - ys) / (float)(xe - xs);
    }
    __syncthreads();
    {
      float gp = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) gp = fmaf(wf[j], sm[L.p16 + 8 * fhf + j], gp);
      const float o = __shfl_xor(gp, 1);
      gp = fhf == 0 ? gp + o : o + gp;
      if (fhf == 0) st_sc1(a.ws + WS_GP + w * HID + fi, gp);
    }
    STAMP(3)
    grid_barrier(ctr, bar++, scal);
    STAMP(4)

    // ======== P3: value head (redundant), dp / da3 / dW3 / dWf / dWv1 (owned) ========
    {  // g = relu(bf + sum over the 64 workgroups' partials, in workgroup order)
      const __amdgpu_buffer_rsrc_t rs = rsrc(a.ws + WS_GP, NWG * HID);
      const int i = t & (HID - 1), h0 = (t >> 8) * (NWG / 2);
      float part[NWG / 2];
#pragma unroll
      for (int j = 0; j < NWG / 2; ++j) part[j] = ld1_sc1(rs, (h0 + j) * HID + i);
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < NWG / 2; ++j) sum += part[j];
      red[t] = sum;
      __syncthreads();
      if (t < HID) sm[L.g + t] = fmaxf(red[t] + red[HID + t] + sm[L.bf + t], 0.f);
    }
    __syncthreads();
    STAMP(20)
    const int vcb = t & 31, vrb = t >> 5;
    {  // h = relu(W g + bv1)
      float gl[8], hp[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) gl[c] = sm[L.g + 8 * vcb + c];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        float x = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) x = fmaf(wb[r * 8 + c], gl[c], x);
        hp[r] = x;
      }
#pragma unroll
      for (int o = 1; o <= 16; o <<= 1)
#pragma unroll
        for (int r = 0; r < 8; ++r) hp[r] += __shfl_xor(hp[r], o);
      if (vcb == 0) {
#pragma unroll
        for (int r = 0; r < 8; ++r) sm[L.h + 8 * vrb + r] = fmaxf(hp[r] + sm[L.bv1 + 8 * vrb + r], 0.f);
      }
    }
    __syncthreads();
    if (wv == 0) {
      float x = fmaf(sm[L.wv2 + lane], sm[L.h + lane], sm[L.wv2 + 64 + lane] * sm[L.h + 64 + lane]);
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
      if (lane == 0) {
        const float v = x + sm[L.bv2];
        const float tg = a.target[s];
        scal[S_V] = v;
        scal[S_DV] = (2.0f * (v - tg)) * a.grad_out;  // mse_loss backward: 2 (v - r) * dL/dmse
        if (w == 0) a.vloss[s] = (v - tg) * (v - tg);
      }
    }
    __syncthreads();
    const float dv = scal[S_DV];
    if (t < VH) {
      const float hv = sm[L.h + t];
      sm[L.dh + t] = hv > 0.f ? dv * sm[L.wv2 + t] : 0.f;
    }
    __syncthreads();
    {  // dg = (W^T dh) * (g > 0): 8 rows per thread, the half-wave pair, the 8 waves in order
      float dl[8], dq[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) dl[r] = sm[L.dh + 8 * vrb + r];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float x = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) x = fmaf(wb[r * 8 + c], dl[r], x);
        dq[c] = x + __shfl_xor(x, 32);
      }
      if (lane < 32) {
#pragma unroll
        for (int c = 0; c < 8; ++c) red[wv * HID + 8 * vcb + c] = dq[c];
      }
      __syncthreads();
      if (t < HID) {
        float x = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) x += red[q * HID + t];
        sm[L.dg + t] = sm[L.g + t] > 0.f ? x : 0.f;
      }
    }
    __syncthreads();
    STAMP(13)
    // dWv1 own slice: dh[row] * g[col]
    const float gv1 = sm[L.dh + (ev >> 8)] * sm[L.g + (ev & 255)];
    // dp own channel: dp[c] = sum_i Wf[i][16w + c] dg[i]; dWf own = dg[i] p[c]
    float gwf[8];
    {
      const float dgi = sm[L.dg + fi];
      float pr[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { pr[j] = wf[j] * dgi; gwf[j] = dgi * sm[L.p16 + 8 * fhf + j]; }
#pragma unroll
      for (int o = 2; o <= 32; o <<= 1)
#pragma unroll
        for (int j = 0; j < 8; ++j) pr[j] += __shfl_xor(pr[j], o);
      if (lane < 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wv * 16 + 8 * lane + j] = pr[j];
      }
      __syncthreads();
      if (t < 16) {
        float sdp = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) sdp += red[q * 16 + t];
        sm[L.dp16 + t] = sdp;
      }
      __syncthreads();
    }
    STAMP(21)
    // da3 own channel: adaptive-pool backward (dp / kH / kW per covering window) * (a3 > 0)
    float da3 = 0.f;
    if (t < N) {
      const int y = t / C, x = t - (t / C) * C;
      const int oys = (y * 4) / R, oye = ((y + 1) * 4 + R - 1) / R, oxs = (x * 4) / C, oxe = ((x + 1) * 4 + C - 1) / C;
      float gsum = 0.f;
      for (int oy = oys; oy < oye; ++oy) {
        const int kh = ((oy + 1) * R + 3) / 4 - (oy * R) / 4;
        for (int ox = oxs; ox < oxe; ++ox) {
          const int kw = ((ox + 1) * C + 3) / 4 - (ox * C) / 4;
          gsum += sm[L.dp16 + oy * 4 + ox] / (float)kh / (float)kw;
        }
      }
      da3 = sm[L.own + t] > 0.f ? gsum : 0.f;
    }
    __syncthreads();
    if (t < N) sm[L.own + t] = da3;
    if (t < Npad) st_sc1(a.ws + WS_DA3 + w * PLANE + t, da3);
    __syncthreads();
    STAMP(22)
    // dW3 row w: lanes = input planes, waves = row groups
    float g3a, g3b = 0.f;
    {
      float acc[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) acc[j] = 0.f;
      wgrad(big, L, C, lane, (wv * R) >> 3, ((wv + 1) * R) >> 3, 0, C, sm + L.own, acc);
#pragma unroll
      for (int j = 0; j < 9; ++j) red[wv * 576 + lane * 9 + j] = acc[j];
      __syncthreads();
      float s0 = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) s0 += red[q * 576 + t];
      g3a = s0;
      if (t < 64) {
        float s1 = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) s1 += red[q * 576 + 512 + t];
        g3b = s1;
      }
      __syncthreads();
    }
    {
      float x[4] = {da3, g3a * g3a + g3b * g3b, 0.f, gv1 * gv1};
#pragma unroll
      for (int j = 0; j < 8; ++j) x[2] = fmaf(gwf[j], gwf[j], x[2]);
      block_sums<4>(x, red);
      if (t == 0) { scal[S_DB3] = x[0]; scal[S_NW3] = x[1]; scal[S_NWF] = x[2]; scal[S_NWV1] = x[3]; }
    }
    STAMP(5)
    grid_barrier(ctr, bar++, scal);
    STAMP(6)

    // ======== P4: da2 own channel (conv3^T), dW2 row w ========
    if (t < C3 * 9) sm[L.wcol + t] = ld_sc1(a.p[W3] + (t / 9) * 576 + w * 9 + (t % 9));
    if (t < 64) sm[L.wcol + 512 + t] = ld_sc1(a.p[W3] + ((512 + t) / 9) * 576 + w * 9 + ((512 + t) % 9));
    load_planes(a.ws + WS_DA3, big, L, R, C);
    __syncthreads();
    STAMP(23)
    float da2 = 0.f;
    {
      const float z = conv_own<4, 8, true>(big, L, R, C, 0, R, sm + L.wcol, red);
      if (t < N) da2 = a2keep > 0.f ? z : 0.f;
      if (t < N) sm[L.own2 + t] = da2;
      if (t < Npad) st_sc1(a.ws + WS_DA2 + w * PLANE + t, da2);
    }
    STAMP(14)
    conv1_all(sm, L, R, C);  // a1 again into planes [0, 32) (da3 no longer needed)
    __syncthreads();
    STAMP(24)
    float g2 = 0.f;
    {
      float acc[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) acc[j] = 0.f;
      const int ci = lane & 31, xh = lane >> 5;
      wgrad(big, L, C, ci, (wv * R) >> 3, ((wv + 1) * R) >> 3, xh * (C >> 1), (xh + 1) * (C >> 1), sm + L.own2, acc);
#pragma unroll
      for (int j = 0; j < 9; ++j) red[(wv * 2 + xh) * 288 + ci * 9 + j] = acc[j];
      __syncthreads();
      if (t < 288) {
#pragma unroll
        for (int q = 0; q < 16; ++q) g2 += red[q * 288 + t];
      }
      __syncthreads();
    }
    {
      float x[2] = {da2, g2 * g2};
      block_sums<2>(x, red);
      if (t == 0) { scal[S_DB2] = x[0]; scal[S_NW2] = x[1]; }
    }
    STAMP(7)
    grid_barrier(ctr, bar++, scal);
    STAMP(8)

    // ======== P5: da1 (channel w/2, half w%2 of the rows), partial dW1 / db1, norm records ========
    {
      const int cj = w >> 1, hh = w & 1, y0 = hh * (R >> 1), nr = R >> 1;
      if (t < 64 * 9) sm[L.wcol + t] = ld_sc1(a.p[W2] + (t / 9) * 288 + cj * 9 + (t % 9));
      if (t < 64) sm[L.wcol + 512 + t] = ld_sc1(a.p[W2] + ((512 + t) / 9) * 288 + cj * 9 + ((512 + t) % 9));
      load_planes(a.ws + WS_DA2, big, L, R, C);
      __syncthreads();
      STAMP(25)
      const float z = conv_own<2, 8, true>(big, L, R, C, y0, nr, sm + L.wcol, red);
      float da1 = 0.f;
      const int np = nr * C;
      if (t < np) {
        const int y = y0 + t / C, x = t - (t / C) * C;
        da1 = conv1_at(sm, L, cj, y, x) > 0.f ? z : 0.f;
        sm[L.own + y * C + x] = da1;
      }
      __syncthreads();
      STAMP(26)
      float x[1] = {da1};
      block_sums<1>(x, red);  // db1 partial (this half)
      float rec = 0.f;
      if (t < 9) {  // dW1 partial: sum over the input's nonzeros of da1[pos] * val, pos = pixel - tap + 1
        const int ky = t / 3, kx = t - (t / 3) * 3, nnz = (int)scal[S_NNZ];
        for (int j = 0; j < nnz; ++j) {
          const int pp = __float_as_int(sm[L.nzpos + j]);
          const int y = (pp >> 8) - ky + 1, xx = (pp & 255) - kx + 1;
          if (y >= y0 && y < y0 + nr && (unsigned)xx < (unsigned)C) rec = fmaf(sm[L.own + y * C + xx], sm[L.nzval + j], rec);
        }
      }
      if (wv == 0) {
        const bool isdw = lane >= NP_DW1 && lane < NP_DW1 + 9;
        const float dw = __shfl(rec, isdw ? lane - NP_DW1 : 0);  // whole wave: lanes 0..8 hold the taps
        float o = 0.f;
        if (isdw) o = dw;
        else if (lane == NP_W2) o = scal[S_NW2];
        else if (lane == NP_B2) o = scal[S_DB2] * scal[S_DB2];
        else if (lane == NP_W3) o = scal[S_NW3];
        else if (lane == NP_B3) o = scal[S_DB3] * scal[S_DB3];
        else if (lane == NP_WF) o = scal[S_NWF];
        else if (lane == NP_WV1) o = scal[S_NWV1];
        else if (lane == NP_DB1) o = x[0];
        if (lane < REC) st_sc1(a.ws + WS_NP + w * REC + lane, o);
      }
    }
    STAMP(9)
    grid_barrier(ctr, bar++, scal);
    STAMP(10)

    // ======== P6: clip coefficient, Adam, publish ========
    {
      const __amdgpu_buffer_rsrc_t rs = rsrc(a.ws + WS_NP, NWG * REC);
      const f32x4_t q = ld4_sc1(rs, 4 * t);  // 512 threads x 4 = the 64 records
      red[4 * t] = q.x; red[4 * t + 1] = q.y; red[4 * t + 2] = q.z; red[4 * t + 3] = q.w;
    }
    __syncthreads();
    STAMP(27)
    float gw1 = 0.f, gb1 = 0.f;
    if (t < 288) {
      const int cj = t / 9, tap = t - (t / 9) * 9;
      gw1 = red[(2 * cj) * REC + NP_DW1 + tap] + red[(2 * cj + 1) * REC + NP_DW1 + tap];
    }
    if (t < C1) gb1 = red[(2 * t) * REC + NP_DB1] + red[(2 * t + 1) * REC + NP_DB1];
    {
      float x[6];
      x[0] = gw1 * gw1;
      x[1] = gb1 * gb1;
      const float dgt = t < HID ? sm[L.dg + t] : 0.f;
      x[2] = dgt * dgt;
      const float dht = t < VH ? sm[L.dh + t] : 0.f;
      x[3] = dht * dht;
      const float gwv2 = t < VH ? dv * sm[L.h + t] : 0.f;
      x[4] = gwv2 * gwv2;
      x[5] = 0.f;
      if (t < 6) {  // owned-tensor sums over the 64 records, in workgroup order
        const int slot = t == 0 ? NP_W2 : t == 1 ? NP_B2 : t == 2 ? NP_W3 : t == 3 ? NP_B3 : t == 4 ? NP_WF : NP_WV1;
        float sacc = 0.f;
        for (int q = 0; q < NWG; ++q) sacc += red[q * REC + slot];
        x[5] = sacc;
      }
      __syncthreads();  // red (records) is reused as the reduction scratch below
      const float own_sum = x[5];
      x[5] = 0.f;
      block_sums<6>(x, red);
      if (t < 6) scal[S_RED8 + t] = own_sum;
      __syncthreads();
      if (t == 0) {
        const float S[NTENS] = {x[0], x[1], scal[S_RED8 + 0], scal[S_RED8 + 1], scal[S_RED8 + 2], scal[S_RED8 + 3],
                                scal[S_RED8 + 4], x[2], scal[S_RED8 + 5], x[3], x[4], dv * dv};
        float tot = 0.f;
        for (int i = 0; i < NTENS; ++i) {
          const float n = sqrtf(S[i]);
          tot = fmaf(n, n, tot);
        }
        const float total = sqrtf(tot);
        const float c = a.max_norm / (total + 1e-6f);
        scal[S_CLIP] = c > 1.0f ? 1.0f : c;
        const double step = a.step0 + (double)(s + 1);
        const double bc1 = 1.0 - pow(a.beta1, step), bc2 = 1.0 - pow(a.beta2, step);
        scal[S_NS] = (float)(-(a.lr / bc1));
        scal[S_BC2S] = (float)sqrt(bc2);
      }
      __syncthreads();
      STAMP(28)
    }
    {
      const float clip = scal[S_CLIP], ns = scal[S_NS], bc2s = scal[S_BC2S];
      if (t < 288) {  // conv1 weight (redundant copy)
        float p = sm[L.w1 + t], m = sm[L.w1 + 288 + t], v = sm[L.w1 + 576 + t];
        adam(p, m, v, gw1, clip, a, ns, bc2s);
        sm[L.w1 + t] = p; sm[L.w1 + 288 + t] = m; sm[L.w1 + 576 + t] = v;
      }
      if (t < C1) {
        float p = sm[L.b1 + t], m = sm[L.b1 + 32 + t], v = sm[L.b1 + 64 + t];
        adam(p, m, v, gb1, clip, a, ns, bc2s);
        sm[L.b1 + t] = p; sm[L.b1 + 32 + t] = m; sm[L.b1 + 64 + t] = v;
      }
      if (t < HID) {
        float p = sm[L.bf + t], m = sm[L.bf + 256 + t], v = sm[L.bf + 512 + t];
        adam(p, m, v, sm[L.dg + t], clip, a, ns, bc2s);
        sm[L.bf + t] = p; sm[L.bf + 256 + t] = m; sm[L.bf + 512 + t] = v;
      }
      if (t < VH) {
        float p = sm[L.bv1 + t], m = sm[L.bv1 + 128 + t], v = sm[L.bv1 + 256 + t];
        adam(p, m, v, sm[L.dh + t], clip, a, ns, bc2s);
        sm[L.bv1 + t] = p; sm[L.bv1 + 128 + t] = m; sm[L.bv1 + 256 + t] = v;
        float q = sm[L.wv2 + t], mq = sm[L.wv2 + 128 + t], vq = sm[L.wv2 + 256 + t];
        adam(q, mq, vq, dv * sm[L.h + t], clip, a, ns, bc2s);
        sm[L.wv2 + t] = q; sm[L.wv2 + 128 + t] = mq; sm[L.wv2 + 256 + t] = vq;
      }
      if (t == 0) {
        float p = sm[L.bv2], m = sm[L.bv2 + 1], v = sm[L.bv2 + 2];
        adam(p, m, v, dv, clip, a, ns, bc2s);
        sm[L.bv2] = p; sm[L.bv2 + 1] = m; sm[L.bv2 + 2] = v;
        float b = scal[S_B2], bm = scal[S_B2M], bv = scal[S_B2V];
        adam(b, bm, bv, scal[S_DB2], clip, a, ns, bc2s);
        scal[S_B2] = b; scal[S_B2M] = bm; scal[S_B2V] = bv;
        float c = scal[S_B3], cm = scal[S_B3M], cv = scal[S_B3V];
        adam(c, cm, cv, scal[S_DB3], clip, a, ns, bc2s);
        scal[S_B3] = c; scal[S_B3M] = cm; scal[S_B3V] = cv;
      }
      if (t < 288) {  // conv2 row w: published for the other workgroups' column reads (P5)
        float p = sm[L.w2r + t];
        adam(p, m2, v2, g2, clip, a, ns, bc2s);
        sm[L.w2r + t] = p;
        st_sc1(a.p[W2] + w * 288 + t, p);
      }
      {  // conv3 row w (P4 column reads)
        float p = sm[L.w3r + t];
        adam(p, m3a, v3a, g3a, clip, a, ns, bc2s);
        sm[L.w3r + t] = p;
        st_sc1(a.p[W3] + w * 576 + t, p);
        if (t < 64) {
          float q = sm[L.w3r + 512 + t];
          adam(q, m3b, v3b, g3b, clip, a, ns, bc2s);
          sm[L.w3r + 512 + t] = q;
          st_sc1(a.p[W3] + w * 576 + 512 + t, q);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) adam(wf[j], mf[j], vf[j], gwf[j], clip, a, ns, bc2s);
      adam(pv1, mv1, vv1, gv1, clip, a, ns, bc2s);
      st_sc1(a.p[WV1] + ev, pv1);  // the next step's P2 reads the whole matrix
    }
    __syncthreads();
    STAMP(11)
  }
#undef STAMP

  // ---- write back what stayed on chip (tensor pointers from the LDS table: the kernel
  // arguments need not stay live in SGPRs across the step loop) ----
  float* const* P = reinterpret_cast<float* const*>(sm + L.ptab);
  float* const* M = P + NTENS;
  float* const* V = P + 2 * NTENS;
  if (t < 288) { M[W2][w * 288 + t] = m2; V[W2][w * 288 + t] = v2; }
  M[W3][w * 576 + t] = m3a; V[W3][w * 576 + t] = v3a;
  if (t < 64) { M[W3][w * 576 + 512 + t] = m3b; V[W3][w * 576 + 512 + t] = v3b; }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int e = fi * NPOOL + 16 * w + 8 * fhf + j;
    P[WF][e] = wf[j]; M[WF][e] = mf[j]; V[WF][e] = vf[j];
  }
  M[WV1][ev] = mv1; V[WV1][ev] = vv1;
  if (t == 0) {
    P[B2][w] = scal[S_B2]; M[B2][w] = scal[S_B2M]; V[B2][w] = scal[S_B2V];
    P[B3][w] = scal[S_B3]; M[B3][w] = scal[S_B3M]; V[B3][w] = scal[S_B3V];
  }
  if (w == 0) {
    for (int i = t; i < C1 * 9; i += NT) {
      P[W1][i] = sm[L.w1 + i]; M[W1][i] = sm[L.w1 + 288 + i]; V[W1][i] = sm[L.w1 + 576 + i];
    }
    if (t < C1) { P[B1][t] = sm[L.b1 + t]; M[B1][t] = sm[L.b1 + 32 + t]; V[B1][t] = sm[L.b1 + 64 + t]; }
    if (t < HID) { P[BF][t] = sm[L.bf + t]; M[BF][t] = sm[L.bf + 256 + t]; V[BF][t] = sm[L.bf + 512 + t]; }
    if (t < VH) {
      P[BV1][t] = sm[L.bv1 + t]; M[BV1][t] = sm[L.bv1 + 128 + t]; V[BV1][t] = sm[L.bv1 + 256 + t];
      P[WV2][t] = sm[L.wv2 + t]; M[WV2][t] = sm[L.wv2 + 128 + t]; V[WV2][t] = sm[L.wv2 + 256 + t];
    }
    if (t == 0) { P[BV2][0] = sm[L.bv2]; M[BV2][0] = sm[L.bv2 + 1]; V[BV2][0] = sm[L.bv2 + 2]; }
  }
}

}  // namespace au

// Compiled grid sizes (the Architect's constant input is R x C): 20x20 (the reference's
// default), 16x16, 12x12, 8x8.
static unsigned long long* g_arch_stamps = nullptr;
void set_arch_stamps(unsigned long long* p) { g_arch_stamps = p; }

bool arch_update_supported(int R, int C) {
  return R == C && (R == 20 || R == 16 || R == 12 || R == 8);
}

int64_t arch_update_workspace_bytes() { return (int64_t)au::WS_FLOATS * 4; }

hipError_t launch_arch_update(float* const* p, float* const* m, float* const* v, const float* grid, int R, int C,
                              const float* target, int k, float* vloss, void* ws, double step0, double lr, double beta1,
                              double beta2, double eps, double max_norm, double value_coeff, hipStream_t st) {
  au::Args a;
  for (int i = 0; i < au::NTENS; ++i) { a.p[i] = p[i]; a.m[i] = m[i]; a.v[i] = v[i]; }
  a.grid = grid; a.target = target; a.vloss = vloss; a.ws = (float*)ws;
  a.stamps = g_arch_stamps;
  a.R = R; a.C = C; a.k = k;
  a.step0 = step0; a.lr = lr; a.beta1 = beta1; a.beta2 = beta2;
  a.lerp_w = (float)(1.0 - beta1);
  a.beta2f = (float)beta2;
  a.c2 = (float)(1.0 - beta2);
  a.eps = (float)eps;
  a.max_norm = (float)max_norm;
  a.grad_out = (float)value_coeff;
  if (!arch_update_supported(R, C)) return hipErrorInvalidValue;
  const size_t lds = (size_t)au::lds_layout(R, C).total * 4;
  const void* fn = R == 20 ? (const void*)au::arch_update_kernel<20, 20>
                 : R == 16 ? (const void*)au::arch_update_kernel<16, 16>
                 : R == 12 ? (const void*)au::arch_update_kernel<12, 12>
                           : (const void*)au::arch_update_kernel<8, 8>;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(a.ws + au::WS_CTR, 0, 64 * sizeof(float), st);
  if (e != hipSuccess) return e;
  if (R == 20) hipLaunchKernelGGL((au::arch_update_kernel<20, 20>), dim3(au::NWG), dim3(au::NT), lds, st, a);
  else if (R == 16) hipLaunchKernelGGL((au::arch_update_kernel<16, 16>), dim3(au::NWG), dim3(au::NT), lds, st, a);
  else if (R == 12) hipLaunchKernelGGL((au::arch_update_kernel<12, 12>), dim3(au::NWG), dim3(au::NT), lds, st, a);
  else hipLaunchKernelGGL((au::arch_update_kernel<8, 8>), dim3(au::NWG), dim3(au::NT), lds, st, a);
  return hipGetLastError();
}

}  // namespace heist
