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
// k steps in one launch with every parameter and Adam moment on chip.
//
// Decomposition: workgroup w = (channel group cg = w % 16, row band b = w / 16).  It owns
// conv2 / conv3 output channels 4cg..4cg+3 on the image rows of pool-cell row b (R/4 rows),
// so every convolution it runs produces 4 channels x one band from all input planes over the
// band plus a one-row halo (its LDS holds 64 planes x (R/4 + 2) rows, and one loaded input
// value feeds 4 output channels).  Five grid barriers per step:
//
//   P1  a1 = relu(conv1(s0)) on band + halo (32 planes, sparse in s0's nonzeros);
//       a2[4 ch][band] = relu(conv2(a1))                                                  -> B1
//   P2  a3[4 ch][band] = relu(conv3(a2)); p = adaptive_avg_pool(a3) (4 ch x 4 cells of cell
//       row b); gp = fc_global.weight[:, own 16 columns] @ p                               -> B2
//   P3  g = relu(bf + sum_w gp[w]); h, v, dv, dh, dg (value head, redundantly per WG:
//       value_head.0.weight rides in registers); dp (own 16 pool cells) = Wf[:, own]^T dg;
//       da3[4 ch][band]; dW3 and db3 partials over the band; dWf own; dWv1 own slice      -> B3
//   P4  da2[4 ch][band] = (conv3^T da3) * (a2 > 0); dW2 / db2 partials over the band      -> B4
//   P4  (also: the own conv3 row's dW3 and the group's db3, sums of their 4 band partials)
//   P5  da1[2 ch][band] = (conv2^T da2) * (a1 > 0); partial dW1 / db1; the group's dW2 /
//       db2 (sum of its 4 bands); per-tensor sums of squares                              -> B5
//   P6  clip coefficient from the 12 tensor norms (norm of norms, as clip_grad_norm_);
//       Adam on every owned / redundant tensor: band b updates and publishes the conv3 row
//       of its group's channel b (the group reloads its 4 rows after the next step's B1);
//       the 4 band workgroups keep identical copies of the group's conv2 rows (needed
//       before B1), and band 0 publishes those.
//
// Hand-offs between workgroups follow MI355X_MICROARCH.md's measured write-through form
// (hand-off table, third row): every handed-off float is stored with a `sc1` store, each
// 128-B line written whole by one store instruction of one wave, each storing wave drains
// (`s_waitcnt vmcnt(0)`), a workgroup barrier, one lane's agent-scope atomic add to a
// monotonic counter, a `global_load_dword sc1` poll, a workgroup barrier, and every load of
// handed-off data is an `sc1` load (dword or dwordx4).
//
// Numerics: fp32 throughout, as the eager step.  Sums run in a fixed order that differs
// from MIOpen's / hipBLASLt's, so results match the eager sequence to fp32 rounding (the
// tests bound it), not bit for bit; the kernel itself is deterministic.  The Adam arithmetic
// mirrors torch's _multi_tensor_adam (lerp, mul + addcmul, sqrt / bc2_sqrt + eps, addcdiv
// with -lr/bc1; bias corrections in float64 from the step count) and clip_grad_norm_
// (per-tensor norms, their norm, max_norm / (total + 1e-6) clamped to 1, grads scaled).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "heist_device.h"

#pragma clang fp contract(off)

#ifndef HEIST_ARCH_XCD_BARRIER
#define HEIST_ARCH_XCD_BARRIER 1  // the two-level grid barrier (A/B: -DHEIST_ARCH_XCD_BARRIER=0, the flat one)
#endif

namespace heist {
namespace au {

constexpr int NT = 512;   // threads per workgroup: 8 waves, 2 per SIMD
constexpr int NWG = 64;   // workgroups: 16 channel groups x 4 row bands
constexpr int CPG = 4;    // conv2 / conv3 channels per group
constexpr int C1 = 32, C2 = 64, C3 = 64, HID = 256, VH = 128, NPOOL = C3 * 16;
constexpr int SEG = 128;             // workspace floats per (channel, band): R/4 * C <= 100, whole 128-B lines
constexpr int PLANE = 4 * SEG;       // per channel
constexpr int REC = 32;              // per-workgroup record (one line)
constexpr int DW3N = CPG * C2 * 9;   // 2304: conv3 weight rows of a group
constexpr int DW2N = CPG * C1 * 9;   // 1152: conv2 weight rows of a group
constexpr int DW3R = DW3N + 32, DW2R = DW2N + 32;  // + the bias partials, whole lines
constexpr int MAXNZ = 64;            // nonzeros of the input plane (the Architect's s0 has 2)
// workspace layout (floats)
constexpr int WS_A2 = 0, WS_GP = WS_A2 + C2 * PLANE, WS_DA3 = WS_GP + NWG * HID, WS_DA2 = WS_DA3 + C3 * PLANE,
              WS_DW3 = WS_DA2 + C2 * PLANE, WS_DW2 = WS_DW3 + NWG * DW3R, WS_NP = WS_DW2 + NWG * DW2R,
              WS_XB = WS_NP + NWG * REC, WS_CTR = WS_XB + 1568, WS_FLOATS = WS_CTR + 64;
// barrier words (unsigned; zeroed per launch).  ws + WS_CTR, the last 64 words: [0] the flat
// barrier's counter, [1] the status word (heist.h: byte offset workspace_bytes - 252).  The
// two-level barrier's words before them, at ws + WS_XB, each on a line of its own (16 XCD
// slots: XCC_ID is 4 bits): [32 x] XCD x's member count, [512 + 32 x] its arrivals,
// [1024 + 32 x] its release generation, [1536] the XCD leaders' counter
constexpr int CW_MEMB = 0, CW_ARR = 512, CW_GEN = 1024, CW_TOP = 1536, CW_WORDS = 1568 + 64;

enum { W1, B1, W2, B2, W3, B3, WF, BF, WV1, BV1, WV2, BV2, NTENS };
// NP record slots
enum { NP_W2 = 0, NP_B2 = 1, NP_W3 = 2, NP_B3 = 3, NP_WF = 4, NP_WV1 = 5, NP_DW1 = 8, NP_DB1 = 26 };

struct Args {
  float* p[NTENS];
  float* m[NTENS];
  float* v[NTENS];
  const float* grid;    // [R][C] the constant input plane
  const float* target;  // [k] rewards
  const float* adam_sc; // [k][2] per step: -lr / bias_correction1, sqrt(bias_correction2) (float32, as torch casts them)
  float* vloss;         // [k] value losses
  float* ws;            // WS_FLOATS floats; ws + WS_CTR: barrier counter and timeout flag (zeroed per launch)
  unsigned long long* stamps;  // instrumentation (NULL: off): s_memrealtime per phase point
  int k;
  unsigned spin_limit;  // polls per grid barrier before it gives up (HEIST_ARCH_SPIN_LIMIT; default 2^25)
  float lerp_w, beta2f, c2, eps, max_norm, grad_out;
};

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// ---- LDS layout (floats) -------------------------------------------------------------
// BIG: 64 zero-padded planes of the band plus its halo rows: row stride RS = C + 2 (pad
// columns 0 and C + 1), BH + 2 rows; data (y, x) of band rows [y0 - 1, y0 + BH] sits at
// (y - y0 + 1) * RS + x + 1.  XP: the whole zero-padded input plane.
template <int R, int C>
struct Lay {
  static constexpr int BH = R / 4, NPB = BH * C, RS = C + 2, PB = (BH + 2) * RS, XRS = C + 2;
  static constexpr int big = 0, xp = big + C2 * PB, w1 = xp + ((R + 2) * XRS + 3) / 4 * 4, b1 = w1 + 3 * C1 * 9,
                       bf = b1 + 3 * C1, bv1 = bf + 3 * HID, wv2 = bv1 + 3 * VH, bv2 = wv2 + 3 * VH, w2r = bv2 + 4,
                       w3r = w2r + 3 * DW2N, w3mv = w3r + DW3N, w2t = w3mv + 2 * 576, b23 = w2t + DW2N, wcol = b23 + 24,
                       gw2 = wcol + DW3N, gw3 = gw2 + DW2N, own = gw3 + 576, own2 = own + 4 * 128, red = own2 + 4 * 128,
                       g = red + 8 * 576, h = g + HID, dh = h + VH, dg = dh + VH, p16 = dg + HID, dp16 = p16 + 16,
                       scal = dp16 + 16, nzpos = scal + 64, nzval = nzpos + MAXNZ, ptab = nzval + MAXNZ,
                       a1b = (ptab + 3 * NTENS * 2 + 3) / 4 * 4, total = a1b + C1 * PB;
};
// scal slots
enum { S_V = 0, S_DV, S_CLIP, S_NS, S_BC2S, S_NNZ, S_TIMEOUT, S_TG, S_DB3 = 8, S_DB2 = 12, S_NWF = 16, S_NWV1,
       S_XC = 56, S_XM, S_XN, S_HB,
       S_NBF, S_NBV1, S_NWV2, S_RED8 = 32 };

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

// Cross-lane sums on DPP / permlane swaps (VALU, no LDS round trip).  Every step pairs
// lanes symmetrically (xor 1, xor 2, the 8-lane and 16-lane mirrors, the 16- and 32-lane
// row swaps), so every lane of a group ends with the same bits: the sum is one fixed
// association, identical in every workgroup.
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float swap16_add(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(x), __float_as_int(x), false, false);
  return __int_as_float(p[0]) + __int_as_float(p[1]);
}
__device__ __forceinline__ float swap32_add(float x) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(x), __float_as_int(x), false, false);
  return __int_as_float(p[0]) + __int_as_float(p[1]);
}
__device__ __forceinline__ float sum16(float x) {  // over each 16-lane row
  x += dpp<0xB1>(x);   // quad_perm [1,0,3,2]: xor 1
  x += dpp<0x4E>(x);   // quad_perm [2,3,0,1]: xor 2
  x += dpp<0x141>(x);  // row_half_mirror: quad pairs
  x += dpp<0x140>(x);  // row_mirror: 8-lane halves
  return x;
}
__device__ __forceinline__ float sum32(float x) { return swap16_add(sum16(x)); }  // over each 32-lane half
__device__ __forceinline__ float sum64(float x) { return swap32_add(sum32(x)); }

// Grid barrier number `idx` (0-based over the launch).  Every storing wave drains its sc1
// stores, the workgroup meets, one lane adds to the monotonic counter and polls it with a
// relaxed sc1 load.  The spin is bounded (spin_limit polls): on a timeout (co-residency
// lost) status word ctr[1] gets bit 0 (heist_arch_update_status; the package restores its
// snapshot and re-runs the steps on another path), and later barriers stop waiting so the
// grid still drains.
__device__ __forceinline__ void grid_barrier(unsigned* ctr, unsigned idx, float* scal, unsigned spin_limit,
                                             unsigned long long* ready = nullptr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (ready) *ready = __builtin_amdgcn_s_memrealtime();  // instrumentation: every wave drained
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (idx + 1u) * (unsigned)NWG;
    if (scal[S_TIMEOUT] == 0.f) {
      // one poll in flight (4 in flight, ~0.2 us apart, measured slower: 51.4 -> 54.4 us per
      // update, the 64 pollers' traffic on the counter's line delays the arrivals, r04y)
      unsigned spins = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > spin_limit) {
          __hip_atomic_fetch_or(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          scal[S_TIMEOUT] = 1.f;
          break;
        }
      }
    }
  }
  __syncthreads();
}

// The two-level form (MI355X_MICROARCH.md barrier-xcd): a workgroup arrives on its XCD's
// counter; the XCD's last arriver arrives on the leaders' counter, waits for every XCD's
// leader and releases its XCD through the XCD's generation word, which only that XCD's
// workgroups poll (8 pollers per line instead of 64 on one).  Membership (m workgroups on
// XCD x, nx XCDs with any) is counted once at the start of the launch.  Data hand-offs are
// unchanged (sc1 stores drained before the arrival, sc1 loads after the release).  Same
// bounded spin and status bit as grid_barrier.
// (Its state -- XCD, member count, XCD count, barrier index -- sits in LDS words read by the
// one polling thread, so it costs the kernel's long-lived registers nothing.)
__device__ __forceinline__ void xcd_barrier(unsigned* ctr, float* scal, unsigned spin_limit,
                                            unsigned long long* ready = nullptr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (ready) *ready = __builtin_amdgcn_s_memrealtime();
    unsigned* xb = ctr - (WS_CTR - WS_XB);
    const unsigned xcc = __float_as_uint(scal[S_XC]), m = __float_as_uint(scal[S_XM]), nx = __float_as_uint(scal[S_XN]);
    const unsigned h = __float_as_uint(scal[S_HB]);
    scal[S_HB] = __uint_as_float(h + 1u);
    unsigned* gen = xb + CW_GEN + 32 * xcc;
    const unsigned old = __hip_atomic_fetch_add(xb + CW_ARR + 32 * xcc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (scal[S_TIMEOUT] == 0.f) {
      unsigned spins = 0;
      bool lost = false;
      if (old == (h + 1u) * m - 1u) {  // the XCD's last: arrive on the leaders' counter, then release the XCD
        __hip_atomic_fetch_add(xb + CW_TOP, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(xb + CW_TOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (h + 1u) * nx) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > spin_limit) { lost = true; break; }
        }
        __hip_atomic_store(gen, h + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < h + 1u) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > spin_limit) { lost = true; break; }
        }
      }
      if (lost) {
        __hip_atomic_fetch_or(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        scal[S_TIMEOUT] = 1.f;
      }
    }
  }
  __syncthreads();
}

// Deterministic workgroup sums of NV values (the same order in every workgroup): the
// wave sums of sum64, the 8 wave totals in order.
template <int NV>
__device__ __forceinline__ void block_sums(float (&x)[NV], float* scratch /* >= 9*NV */) {
  const int tid_ = tid_o();
  const int wv = tid_ >> 6, lane = tid_ & 63;
#pragma unroll
  for (int i = 0; i < NV; ++i) x[i] = sum64(x[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) scratch[wv * NV + i] = x[i];
  }
  __syncthreads();
  if (tid_ < NV) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) s += scratch[w * NV + tid_];
    scratch[8 * NV + tid_] = s;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) x[i] = scratch[8 * NV + i];
  __syncthreads();
}

// ---- convolution pieces -----------------------------------------------------------------
// Plane-major weight layout for the band convolutions: the NCO x 9 weights of input plane c
// are wsrc[c * SPL + q * 9 + tap] (SPL a multiple of 4, 16-byte aligned rows), so one
// plane's weights are 9 (NCO = 4) or 5 (NCO = 2) wave-uniform ds_read_b128 (a broadcast:
// every lane reads the same 16 bytes) straight into VGPRs.  Index of the row-major
// conv weight element (q, ci, tap) of a group's rows (NCI input planes) in that layout:
template <int NCI>
__device__ __forceinline__ int plane_major(int e) {
  const int q = e / (NCI * 9), r = e - q * (NCI * 9), ci = r / 9;
  return ci * 36 + q * 9 + (r - ci * 9);
}

// Band convolution: NCO output channels on the band's BH x C positions from the 8 * NCIW
// input planes of BIG (8 waves split the planes), 1 x 2 output strips per lane as one
// packed pair: per plane and (channel, tap) one v_pk_fma_f32 of the window pair with the
// broadcast weight.  FLIP: the transposed convolution's flipped taps.  Returns, for thread
// t < NCO * NPB, the sum of the 8 waves' partials (in wave order) of channel t / NPB at band
// position t % NPB; other threads get 0.
template <int R, int C, int NCO, int NCIW, bool FLIP>
__device__ __forceinline__ float conv_band(const float* __restrict__ big, const float* __restrict__ wsrc, int SPL,
                                           float* red) {
  using L = Lay<R, C>;
  constexpr int NSX = C / 2, NS = L::BH * NSX, NV4 = (NCO * 9 + 3) / 4;
  const int tid_ = tid_o();
  const int wv = tid_ >> 6, lane = tid_ & 63;
  const int sl = lane < NS ? lane : 0;  // lanes past the last strip redo strip 0 and store nothing
  const int sy = sl / NSX, sx = (sl - (sl / NSX) * NSX) * 2;
  const f32x2_t* pbase = reinterpret_cast<const f32x2_t*>(big + sy * L::RS + sx);
  f32x2_t acc[NCO];
#pragma unroll
  for (int q = 0; q < NCO; ++q) acc[q] = f32x2_t{0.f, 0.f};
#pragma unroll 1
  for (int c = 0; c < NCIW; ++c) {
    const int ci = wv * NCIW + c;
    const f32x4_t* wp = reinterpret_cast<const f32x4_t*>(wsrc + ci * SPL);
    float wt[NV4 * 4];
#pragma unroll
    for (int i = 0; i < NV4; ++i) {
      const f32x4_t x = wp[i];
      wt[4 * i] = x.x; wt[4 * i + 1] = x.y; wt[4 * i + 2] = x.z; wt[4 * i + 3] = x.w;
    }
    const f32x2_t* pl = pbase + ci * (L::PB / 2);
    f32x2_t pr[3][3];  // pr[ky][kx] = (in[ky][kx], in[ky][kx + 1])
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const f32x2_t u0 = pl[r * (L::RS / 2)], u1 = pl[r * (L::RS / 2) + 1];
      pr[r][0] = u0;
      pr[r][1] = f32x2_t{u0.y, u1.x};
      pr[r][2] = u1;
    }
#pragma unroll
    for (int q = 0; q < NCO; ++q)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float w = wt[q * 9 + (FLIP ? 8 - (ky * 3 + kx) : ky * 3 + kx)];
          acc[q] = __builtin_elementwise_fma(f32x2_t{w, w}, pr[ky][kx], acc[q]);
        }
  }
  if (lane < NS) {
#pragma unroll
    for (int q = 0; q < NCO; ++q) {
      red[(wv * NCO + q) * L::NPB + sy * C + sx] = acc[q].x;
      red[(wv * NCO + q) * L::NPB + sy * C + sx + 1] = acc[q].y;
    }
  }
  __syncthreads();
  float s = 0.f;
  if (tid_ < NCO * L::NPB) {
    const int q = tid_ / L::NPB, pos = tid_ - q * L::NPB;
#pragma unroll
    for (int w = 0; w < 8; ++w) s += red[(w * NCO + q) * L::NPB + pos];
  }
  __syncthreads();
  return s;
}

// Weight-gradient partial of one input plane `ci` of BIG: acc[ky*3+kx] += sum over NY band
// rows from ya (band-local) and NX columns from xa of d[y * C + x] * in_pad[ci][(y + ky) *
// RS + x + kx], sliding a 3x3 window along each row (3 new loads per position; unrolled,
// so each row's loads issue together).
template <int R, int C, int NY, int NX>
__device__ __forceinline__ void wgrad(const float* __restrict__ big, int ci, int ya, int xa,
                                      const float* __restrict__ d, float (&acc)[9]) {
  using L = Lay<R, C>;
  constexpr int RS = L::RS;
#pragma unroll 1
  for (int yy = 0; yy < NY; ++yy) {
    const int y = ya + yy;
    const float* pl = big + ci * L::PB + y * RS + xa;
    float col[NX + 2][3];
#pragma unroll
    for (int x = 0; x < NX + 2; ++x) {
      col[x][0] = pl[x]; col[x][1] = pl[RS + x]; col[x][2] = pl[2 * RS + x];
    }
    const float* drow = d + y * C + xa;
#pragma unroll
    for (int x = 0; x < NX; ++x) {
      const float dd = drow[x];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc[ky * 3 + kx] = fmaf(dd, col[x + kx][ky], acc[ky * 3 + kx]);
    }
  }
}

// wgrad for two output channels at once: acc[tap] = (channel-0, channel-1) partials over NY
// band rows from ya and NX columns from xa; one load of the input window feeds both channels
// (a packed FMA of the (d0, d1) pair with the broadcast window value).
template <int R, int C, int NY, int NX>
__device__ __forceinline__ void wgrad2(const float* __restrict__ big, int ci, int ya, int xa,
                                       const float* __restrict__ d0, const float* __restrict__ d1, f32x2_t (&acc)[9]) {
  using L = Lay<R, C>;
  constexpr int RS = L::RS;
#pragma unroll 1
  for (int yy = 0; yy < NY; ++yy) {
    const int y = ya + yy;
    const float* pl = big + ci * L::PB + y * RS + xa;
    float col[NX + 2][3];
#pragma unroll
    for (int x = 0; x < NX + 2; ++x) {
      col[x][0] = pl[x]; col[x][1] = pl[RS + x]; col[x][2] = pl[2 * RS + x];
    }
    f32x2_t dd[NX];
#pragma unroll
    for (int x = 0; x < NX; ++x) dd[x] = f32x2_t{d0[y * C + xa + x], d1[y * C + xa + x]};
#pragma unroll
    for (int x = 0; x < NX; ++x)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float v = col[x + kx][ky];
          acc[ky * 3 + kx] = __builtin_elementwise_fma(dd[x], f32x2_t{v, v}, acc[ky * 3 + kx]);
        }
  }
}

// a1[ci] at (y, x): relu(sum + b1), the sum over the input's nonzero pixels inside the 3x3
// window in tap order (skipping the zero taps changes no bit of the dense sum).
template <int R, int C>
__device__ __forceinline__ float conv1_at(const float* sm, int ci, int y, int x) {
  using L = Lay<R, C>;
  const int nnz = (int)sm[L::scal + S_NNZ];
  float acc = 0.f;
  for (int j = 0; j < nnz; ++j) {
    const int pp = __float_as_int(sm[L::nzpos + j]);
    const int dy = (pp >> 8) - y + 1, dx = (pp & 255) - x + 1;
    if ((unsigned)dy < 3u && (unsigned)dx < 3u) acc = fmaf(sm[L::w1 + ci * 9 + dy * 3 + dx], sm[L::nzval + j], acc);
  }
  return fmaxf(acc + sm[L::b1 + ci], 0.f);
}

// conv1 (1 -> 32) on the band rows and halo rows inside the image, into the A1B planes (the
// step's a1 stays there for conv2, dW2 and da1's mask):
// rows with no nonzero in reach hold relu(0 + b1); the few positions inside a nonzero's 3x3
// neighbourhood are recomputed (a position near two nonzeros is written twice, same value).
template <int R, int C>
__device__ __forceinline__ void conv1_band(float* sm, int y0) {
  using L = Lay<R, C>;
  const int tid_ = tid_o();
  float* big = sm + L::a1b;
  constexpr int NR = L::BH + 2;
  if (tid_ < C1 * NR) {
    const int ci = tid_ / NR, r = tid_ - ci * NR, y = y0 - 1 + r;
    if ((unsigned)y < (unsigned)R) {
      const float val = fmaxf(0.f + sm[L::b1 + ci], 0.f);
      float* row = big + ci * L::PB + r * L::RS + 1;
#pragma unroll
      for (int x = 0; x < C; ++x) row[x] = val;
    }
  }
  __syncthreads();
  const int nnz = (int)sm[L::scal + S_NNZ];
  for (int o = tid_; o < C1 * 9 * nnz; o += NT) {
    const int ci = o & (C1 - 1), rr = o >> 5, j = rr / 9, tap = rr - j * 9;
    const int pp = __float_as_int(sm[L::nzpos + j]);
    const int y = (pp >> 8) - tap / 3 + 1, x = (pp & 255) - (tap % 3) + 1;
    if ((unsigned)y < (unsigned)R && (unsigned)x < (unsigned)C && y >= y0 - 1 && y <= y0 + L::BH)
      big[ci * L::PB + (y - y0 + 1) * L::RS + x + 1] = conv1_at<R, C>(sm, ci, y, x);
  }
}

// the 64 channel planes of a handed-off workspace array ([ch][band][SEG], sc1) on the band
// rows and halo rows inside the image: band_issue loads them into registers (so other loads
// can go out in the same round trip), band_commit writes them into BIG
template <int R, int C>
struct BandQ {
  static constexpr int NR = R / 4 + 2, QR = C / 4, NQ = C2 * NR * QR, MAXQ = (NQ + NT - 1) / NT;
};
template <int R, int C>
__device__ __forceinline__ void band_issue(const float* src, int y0, f32x4_t (&v)[BandQ<R, C>::MAXQ]) {
  using L = Lay<R, C>;
  using Q = BandQ<R, C>;
  const int tid_ = tid_o();
  const __amdgpu_buffer_rsrc_t rs = rsrc(src, C2 * PLANE);
#pragma unroll
  for (int i = 0; i < Q::MAXQ; ++i) {
    const int qd = tid_ + i * NT;
    const int ch = qd / (Q::NR * Q::QR), rem = qd - ch * (Q::NR * Q::QR), r = rem / Q::QR;
    const int x = (rem - r * Q::QR) * 4, y = y0 - 1 + r;
    if (qd < Q::NQ && (unsigned)y < (unsigned)R) {
      const int bb = y / L::BH;
      v[i] = ld4_sc1(rs, ch * PLANE + bb * SEG + (y - bb * L::BH) * C + x);
    }
  }
}
template <int R, int C>
__device__ __forceinline__ void band_commit(float* big, int y0, const f32x4_t (&v)[BandQ<R, C>::MAXQ]) {
  using L = Lay<R, C>;
  using Q = BandQ<R, C>;
  const int tid_ = tid_o();
#pragma unroll
  for (int i = 0; i < Q::MAXQ; ++i) {
    const int qd = tid_ + i * NT;
    const int ch = qd / (Q::NR * Q::QR), rem = qd - ch * (Q::NR * Q::QR), r = rem / Q::QR;
    const int x = (rem - r * Q::QR) * 4, y = y0 - 1 + r;
    if (qd < Q::NQ && (unsigned)y < (unsigned)R) {
      float* d = big + ch * L::PB + r * L::RS + x + 1;
      d[0] = v[i].x; d[1] = v[i].y; d[2] = v[i].z; d[3] = v[i].w;
    }
  }
}
template <int R, int C>
__device__ __forceinline__ void load_band(const float* src, float* big, int y0) {
  f32x4_t v[BandQ<R, C>::MAXQ];
  band_issue<R, C>(src, y0, v);
  band_commit<R, C>(big, y0, v);
}

// store the workgroup's [4][NPB] band values from LDS `src` to its segments of a
// handed-off workspace array (whole lines: segment tails are zero)
template <int R, int C>
__device__ __forceinline__ void store_band(float* dst, const float* src, int cg, int band) {
  using L = Lay<R, C>;
  const int tid_ = tid_o();
  const int q = tid_ >> 7, i = tid_ & (SEG - 1);
  st_sc1(dst + (CPG * cg + q) * PLANE + band * SEG + i, i < L::NPB ? src[q * L::NPB + i] : 0.f);
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
// Adam on LDS-resident (param, exp_avg, exp_avg_sq) triples at base[e], base[n + e],
// base[2n + e] for e = t + j * NT < n (j < K), gradients grad[e] (LDS): every load first,
// then the arithmetic, then the stores (the LDS round trips overlap).  pout[j] = new param.
template <int K>
__device__ __forceinline__ void adam_lds(float* base, int n, int t, const float* grad, float clip, const Args& a,
                                         float ns, float bc2s, float (&pout)[K]) {
  float p[K], m[K], v[K], g[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int e = t + j * NT;
    if (e < n) { p[j] = base[e]; m[j] = base[n + e]; v[j] = base[2 * n + e]; g[j] = grad[e]; }
  }
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (t + j * NT < n) adam(p[j], m[j], v[j], g[j], clip, a, ns, bc2s);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int e = t + j * NT;
    if (e < n) { base[e] = p[j]; base[n + e] = m[j]; base[2 * n + e] = v[j]; pout[j] = p[j]; }
  }
}

// Workgroup w = (channel group w & 15, row band w >> 4): a group's 4 band workgroups are
// w, w + 16, w + 32, w + 48, which dispatch places on one XCD (blockIdx % 8), so the
// group-internal hand-offs (the band partials of dW2 / dW3, read back in P5) stay in that
// XCD's L2 path.
__device__ __forceinline__ int wg_cg(int w) { return w & 15; }
__device__ __forceinline__ int wg_band(int w) { return w >> 4; }
__device__ __forceinline__ int wg_of(int cg, int band) { return band * 16 + cg; }

// fc_global.weight ownership: thread t holds row fc_row(t), local columns 8 * fc_half(t) + [0, 8)
// (the half on lane bit 5, so the row sum over a wave's 32 rows stays inside a half-wave)
__device__ __forceinline__ int fc_row(int t) { return ((t >> 6) << 5) | (t & 31); }
__device__ __forceinline__ int fc_half(int t) { return (t >> 5) & 1; }

template <int R, int C>
__global__ void __launch_bounds__(NT, 1) arch_update_kernel(Args a) {
  using L = Lay<R, C>;
  constexpr int N = R * C, BH = L::BH, NPB = L::NPB;
  static_assert(R % 4 == 0 && C % 4 == 0 && CPG * NPB <= 4 * 128 && NPB <= SEG, "band sizes");
  static_assert(L::total * 4 <= 160 * 1024, "LDS");
  extern __shared__ float sm[];
  float* big = sm + L::big;
  float* red = sm + L::red;
  float* scal = sm + L::scal;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.ws + WS_CTR);
  // STAMP(i): workgroups 0 and 63, steps < 16, 32 points per step (tools/probe_arch_update.py)
#define STAMP(i)                                                                                          \
  if (a.stamps && threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == NWG - 1) && s < 16)               \
    a.stamps[((blockIdx.x == 0 ? 0 : 1) * 16 + s) * 32 + (i)] = __builtin_amdgcn_s_memrealtime();
  // READY(b): every workgroup's time at barrier b of steps < 16, once its waves have drained
  // their stores (after stamp slot 1024: [16 steps][5 barriers][64 workgroups])
#define READY(b) (a.stamps && s < 16 ? a.stamps + 1024 + (s * 5 + (b)) * NWG + blockIdx.x : nullptr)

  // ---- setup: zero BIG + XP (pads and out-of-image halo rows stay zero), load parameters ----
  {
    const int t = threadIdx.x, w = blockIdx.x, cg = wg_cg(w);
    for (int i = t; i < L::w1; i += NT) sm[i] = 0.f;
    for (int i = t; i < C1 * L::PB; i += NT) sm[L::a1b + i] = 0.f;  // a1's pads and out-of-image rows
    if (t < 64) scal[t] = 0.f;
    if (t < 3 * NTENS) {
      float** tab = reinterpret_cast<float**>(sm + L::ptab);
      tab[t] = t < NTENS ? a.p[t] : t < 2 * NTENS ? a.m[t - NTENS] : a.v[t - 2 * NTENS];
    }
    __syncthreads();
    for (int i = t; i < N; i += NT) {
      const int y = i / C, x = i - y * C;
      sm[L::xp + (y + 1) * L::XRS + x + 1] = a.grid[i];
    }
    for (int i = t; i < C1 * 9; i += NT) {
      sm[L::w1 + i] = a.p[W1][i]; sm[L::w1 + 288 + i] = a.m[W1][i]; sm[L::w1 + 576 + i] = a.v[W1][i];
    }
    if (t < C1) { sm[L::b1 + t] = a.p[B1][t]; sm[L::b1 + 32 + t] = a.m[B1][t]; sm[L::b1 + 64 + t] = a.v[B1][t]; }
    if (t < HID) { sm[L::bf + t] = a.p[BF][t]; sm[L::bf + 256 + t] = a.m[BF][t]; sm[L::bf + 512 + t] = a.v[BF][t]; }
    if (t < VH) {
      sm[L::bv1 + t] = a.p[BV1][t]; sm[L::bv1 + 128 + t] = a.m[BV1][t]; sm[L::bv1 + 256 + t] = a.v[BV1][t];
      sm[L::wv2 + t] = a.p[WV2][t]; sm[L::wv2 + 128 + t] = a.m[WV2][t]; sm[L::wv2 + 256 + t] = a.v[WV2][t];
    }
    if (t == 0) { sm[L::bv2] = a.p[BV2][0]; sm[L::bv2 + 1] = a.m[BV2][0]; sm[L::bv2 + 2] = a.v[BV2][0]; }
    if (t < CPG) {  // b2, b3 of the group's channels: [p m v] x 4 each
      const int ch = CPG * cg + t;
      sm[L::b23 + t] = a.p[B2][ch]; sm[L::b23 + 4 + t] = a.m[B2][ch]; sm[L::b23 + 8 + t] = a.v[B2][ch];
      sm[L::b23 + 12 + t] = a.p[B3][ch]; sm[L::b23 + 16 + t] = a.m[B3][ch]; sm[L::b23 + 20 + t] = a.v[B3][ch];
    }
    // the group's conv2 / conv3 rows (contiguous in the tensors): params and moments in LDS
    for (int e = t; e < DW2N; e += NT) {
      const int g = CPG * cg * 288 + e;
      sm[L::w2r + e] = a.p[W2][g]; sm[L::w2r + DW2N + e] = a.m[W2][g]; sm[L::w2r + 2 * DW2N + e] = a.v[W2][g];
      sm[L::w2t + plane_major<C1>(e)] = a.p[W2][g];
    }
    for (int e = t; e < DW3N; e += NT) sm[L::w3r + plane_major<C2>(e)] = a.p[W3][CPG * cg * 576 + e];
    for (int e = t; e < 576; e += NT) {  // the own row's moments (channel 4cg + band)
      const int g = (CPG * cg + wg_band(w)) * 576 + e;
      sm[L::w3mv + e] = a.m[W3][g]; sm[L::w3mv + 576 + e] = a.v[W3][g];
    }
    __syncthreads();
    // the input's nonzero pixels in row-major order (wave 0, ballot compaction)
    if (t < 64) {
      int cnt = 0;
      for (int base = 0; base < N; base += 64) {
        const int i = base + t;
        float val = 0.f;
        if (i < N) { const int y = i / C, x = i - y * C; val = sm[L::xp + (y + 1) * L::XRS + x + 1]; }
        const unsigned long long bal = __ballot(val != 0.f);
        const int before = __popcll(bal & ((1ull << t) - 1ull));
        if (val != 0.f && cnt + before < MAXNZ) {
          const int y = i / C, x = i - y * C;
          sm[L::nzpos + cnt + before] = __int_as_float((y << 8) | x);
          sm[L::nzval + cnt + before] = val;
        }
        cnt += __popcll(bal);
      }
      if (t == 0) scal[S_NNZ] = (float)(cnt < MAXNZ ? cnt : MAXNZ);
      // more than MAXNZ nonzeros: the forward would drop pixels -- status bit 1, results invalid
      if (t == 0 && cnt > MAXNZ && blockIdx.x == 0)
        __hip_atomic_fetch_or(reinterpret_cast<unsigned*>(a.ws + WS_CTR) + 1, 2u, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
  // owned in registers across the whole launch: fc_global.weight columns J(8 hf + j) of row
  // t >> 1 (the group's 4 channels x the band's 4 pool cells) and value_head.0.weight element
  // w * 512 + t (rows 2w, 2w + 1), with their moments
  float wf[8], mf[8], vf[8];
  {
    const int t = threadIdx.x, w = blockIdx.x, cg = wg_cg(w), band = wg_band(w);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int jj = 8 * fc_half(t) + j;  // local column: channel jj >> 2, cell (band, jj & 3)
      const int e = fc_row(t) * NPOOL + (CPG * cg + (jj >> 2)) * 16 + band * 4 + (jj & 3);
      wf[j] = a.p[WF][e]; mf[j] = a.m[WF][e]; vf[j] = a.v[WF][e];
    }
  }
  float pv1 = a.p[WV1][blockIdx.x * 512 + threadIdx.x], mv1 = a.m[WV1][blockIdx.x * 512 + threadIdx.x],
        vv1 = a.v[WV1][blockIdx.x * 512 + threadIdx.x];

  float a2keep = 0.f;  // a2 at (channel t / NPB, band position t % NPB): P4's relu mask
  unsigned bar = 0;
#if HEIST_ARCH_XCD_BARRIER
  unsigned* xb = reinterpret_cast<unsigned*>(a.ws + WS_XB);
  // the two-level barrier's membership: this workgroup's XCD, its workgroup count, the number of
  // XCDs holding any (one flat barrier makes the counts final), in LDS for xcd_barrier
  if (threadIdx.x == 0) {
    const unsigned xcc = __builtin_amdgcn_s_getreg(0x1814) & 15u;  // hwreg(HW_REG_XCC_ID, 0, 4)
    scal[S_XC] = __uint_as_float(xcc);
    scal[S_HB] = __uint_as_float(0u);
    __hip_atomic_fetch_add(xb + CW_MEMB + 32 * xcc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  grid_barrier(ctr, bar++, scal, a.spin_limit);
  if (threadIdx.x == 0) {
    unsigned nx = 0;
    for (int x = 0; x < 16; ++x)
      nx += __hip_atomic_load(xb + CW_MEMB + 32 * x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    const unsigned xcc = __float_as_uint(scal[S_XC]);
    scal[S_XM] = __uint_as_float(__hip_atomic_load(xb + CW_MEMB + 32 * xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    scal[S_XN] = __uint_as_float(nx);
  }
#define BARRIER(i) xcd_barrier(ctr, scal, a.spin_limit, READY(i));
#else
#define BARRIER(i) grid_barrier(ctr, bar++, scal, a.spin_limit, READY(i));
#endif
  for (int s = 0; s < a.k; ++s) {
    const int t = tid_o(), wv = t >> 6, lane = t & 63, w = wg_o();
    const int cg = wg_cg(w), band = wg_band(w), y0 = band * BH;
    const int fi = fc_row(t), fhf = fc_half(t), ev = w * 512 + t;
    // ======== P1: conv1 (band + halo), conv2 own channels ========
    STAMP(0)
    if (t == NT - 1) {  // this step's Adam scalars and target, read well before P3 / P6 need them
      scal[S_NS] = a.adam_sc[2 * s];
      scal[S_BC2S] = a.adam_sc[2 * s + 1];
      scal[S_TG] = a.target[s];
    }
    conv1_band<R, C>(sm, y0);
    __syncthreads();
    STAMP(15)
    {
      const float z = conv_band<R, C, CPG, 4, false>(sm + L::a1b, sm + L::w2t, 36, red);
      if (t < CPG * NPB) {
        a2keep = fmaxf(z + sm[L::b23 + t / NPB], 0.f);
        sm[L::own + t] = a2keep;
      }
      __syncthreads();
      store_band<R, C>(a.ws + WS_A2, sm + L::own, cg, band);
    }
    STAMP(1)
    BARRIER(0)
    STAMP(2)

    // ======== P2: conv3 own channels, pool, fc_global partial ========
    f32x4_t a2v[BandQ<R, C>::MAXQ];
    band_issue<R, C>(a.ws + WS_A2, y0, a2v);
    // the group's conv3 rows as its 4 band workgroups published them: DW3N / 4 = 576 float4,
    // 512 threads -> two loads for threads t < 64
    static_assert(DW3N / 4 > NT && DW3N / 4 <= 2 * NT, "two float4 per thread cover the group's conv3 rows");
    f32x4_t w3q[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    {
      const __amdgpu_buffer_rsrc_t r3 = rsrc(a.p[W3], C3 * 576);
      w3q[0] = ld4_sc1(r3, CPG * cg * 576 + 4 * t);
      if (t + NT < DW3N / 4) w3q[1] = ld4_sc1(r3, CPG * cg * 576 + 4 * (t + NT));
    }
    band_commit<R, C>(big, y0, a2v);
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {  // plane-major for conv_band
      const int e = 4 * (t + h2 * NT);
      if (e < DW3N) {
        sm[L::w3r + plane_major<C2>(e)] = w3q[h2].x; sm[L::w3r + plane_major<C2>(e + 1)] = w3q[h2].y;
        sm[L::w3r + plane_major<C2>(e + 2)] = w3q[h2].z; sm[L::w3r + plane_major<C2>(e + 3)] = w3q[h2].w;
      }
    }
    // value_head.0.weight as 8x8 blocks (rows 8 * (t >> 5) + r, columns 8 * (t & 31) + c):
    // both h = W g (reduced over the 32 column blocks of a half-wave) and dg = W^T dh
    // (over the 16 row blocks) stay cheap.  Issued once the a2 band and the conv3 rows have
    // landed (not beside them: 128 KB per workgroup), in flight during conv3, landed by B2.
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
    __syncthreads();
    STAMP(12)
    STAMP(17)
    {
      const float z = conv_band<R, C, CPG, 8, false>(big, sm + L::w3r, 36, red);
      if (t < CPG * NPB) sm[L::own + t] = fmaxf(z + sm[L::b23 + 12 + t / NPB], 0.f);
    }
    __syncthreads();
    STAMP(18)
    if (t < 16) {  // adaptive_avg_pool2d((4, 4)), cell (band, t & 3) of channel t >> 2: window sum, / kH / kW
      const int q = t >> 2, ox = t & 3;
      constexpr int KW = C / 4;
      const float* src = sm + L::own + q * NPB + ox * KW;
      float vals[BH * KW];
#pragma unroll
      for (int y = 0; y < BH; ++y)
#pragma unroll
        for (int x = 0; x < KW; ++x) vals[y * KW + x] = src[y * C + x];
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < BH * KW; ++i) sum += vals[i];
      sm[L::p16 + t] = sum / (float)BH / (float)KW;
    }
    __syncthreads();
    {
      float gp = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) gp = fmaf(wf[j], sm[L::p16 + 8 * fhf + j], gp);
      gp = swap32_add(gp);  // the two column halves
      if (fhf == 0) st_sc1(a.ws + WS_GP + w * HID + fi, gp);
    }
    STAMP(3)
    BARRIER(1)
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
      if (t < HID) sm[L::g + t] = fmaxf(red[t] + red[HID + t] + sm[L::bf + t], 0.f);
    }
    __syncthreads();
    STAMP(20)
    const int vcb = t & 31, vrb = t >> 5;
    {  // h = relu(W g + bv1)
      float gl[8], hp[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) gl[c] = sm[L::g + 8 * vcb + c];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        float x = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) x = fmaf(wb[r * 8 + c], gl[c], x);
        hp[r] = x;
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) hp[r] = sum32(hp[r]);
      if (vcb == 0) {
#pragma unroll
        for (int r = 0; r < 8; ++r) sm[L::h + 8 * vrb + r] = fmaxf(hp[r] + sm[L::bv1 + 8 * vrb + r], 0.f);
      }
    }
    __syncthreads();
    if (wv == 0) {
      float x = fmaf(sm[L::wv2 + lane], sm[L::h + lane], sm[L::wv2 + 64 + lane] * sm[L::h + 64 + lane]);
      x = sum64(x);
      if (lane == 0) {
        const float v = x + sm[L::bv2];
        const float tg = scal[S_TG];
        scal[S_V] = v;
        scal[S_DV] = (2.0f * (v - tg)) * a.grad_out;  // mse_loss backward: 2 (v - r) * dL/dmse
        if (w == 0) a.vloss[s] = (v - tg) * (v - tg);
      }
    }
    __syncthreads();
    const float dv = scal[S_DV];
    if (t < VH) {
      const float hv = sm[L::h + t];
      sm[L::dh + t] = hv > 0.f ? dv * sm[L::wv2 + t] : 0.f;
    }
    __syncthreads();
    {  // dg = (W^T dh) * (g > 0): 8 rows per thread, the half-wave pair, the 8 waves in order
      float dl[8], dq[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) dl[r] = sm[L::dh + 8 * vrb + r];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float x = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) x = fmaf(wb[r * 8 + c], dl[r], x);
        dq[c] = swap32_add(x);
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
        sm[L::dg + t] = sm[L::g + t] > 0.f ? x : 0.f;
      }
    }
    __syncthreads();
    STAMP(13)
    // dWv1 own slice: dh[row] * g[col]
    const float gv1 = sm[L::dh + (ev >> 8)] * sm[L::g + (ev & 255)];
    // dp own cells: dp[j] = sum_i Wf[i][J(j)] dg[i]; dWf own = dg[i] p[j]
    float gwf[8];
    {
      const float dgi = sm[L::dg + fi];
      float pr[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { pr[j] = wf[j] * dgi; gwf[j] = dgi * sm[L::p16 + 8 * fhf + j]; }
#pragma unroll
      for (int j = 0; j < 8; ++j) pr[j] = sum32(pr[j]);  // the wave's 32 rows, per column half
      if ((lane & 31) == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wv * 16 + 8 * fhf + j] = pr[j];
      }
      __syncthreads();
      if (t < 16) {
        float sdp = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) sdp += red[q * 16 + t];
        sm[L::dp16 + t] = sdp;
      }
      __syncthreads();
    }
    STAMP(21)
    // da3 own channels on the band: adaptive-pool backward (dp / kH / kW) * (a3 > 0)
    float da3 = 0.f;
    if (t < CPG * NPB) {
      const int q = t / NPB, pos = t - q * NPB, x = pos - (pos / C) * C;
      const int ox = (x * 4) / C, kw = ((ox + 1) * C + 3) / 4 - (ox * C) / 4;
      da3 = sm[L::own + t] > 0.f ? sm[L::dp16 + q * 4 + ox] / (float)BH / (float)kw : 0.f;
    }
    __syncthreads();
    if (t < CPG * NPB) sm[L::own + t] = da3;
    __syncthreads();
    store_band<R, C>(a.ws + WS_DA3, sm + L::own, cg, band);
    STAMP(22)
    {  // dW3 partial over the band: lanes = input planes, waves = (channel pair, column quarter);
       // the column quarters are summed (q0 + q2) + (q1 + q3) through red
      f32x2_t acc[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) acc[j] = f32x2_t{0.f, 0.f};
      const int qp = wv & 1, xq = wv >> 1;
      wgrad2<R, C, BH, C / 4>(big, lane, 0, xq * (C / 4), sm + L::own + (2 * qp) * NPB,
                              sm + L::own + (2 * qp + 1) * NPB, acc);
      float* slot = red + (xq & 1) * DW3N + (2 * qp) * 576 + lane * 9;
      if (xq < 2) {
#pragma unroll
        for (int j = 0; j < 9; ++j) { slot[j] = acc[j].x; slot[576 + j] = acc[j].y; }
      }
      __syncthreads();
      if (xq >= 2) {
#pragma unroll
        for (int j = 0; j < 9; ++j) { slot[j] = slot[j] + acc[j].x; slot[576 + j] = slot[576 + j] + acc[j].y; }
      }
      __syncthreads();
      STAMP(16)
      float* dst = a.ws + WS_DW3 + w * DW3R;
#pragma unroll
      for (int k5 = 0; k5 < 5; ++k5) {
        const int e = t + k5 * NT;
        if (e < DW3N) st_sc1(dst + e, red[e] + red[DW3N + e]);
      }
      __syncthreads();
    }
    STAMP(19)
    {  // db3 partials (one per channel) and the value head's sums of squares
      float x[CPG + 6];
#pragma unroll
      for (int q = 0; q < CPG; ++q) x[q] = (t < CPG * NPB && t / NPB == q) ? da3 : 0.f;
      x[CPG] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) x[CPG] = fmaf(gwf[j], gwf[j], x[CPG]);
      x[CPG + 1] = gv1 * gv1;
      const float dgt = t < HID ? sm[L::dg + t] : 0.f, dht = t < VH ? sm[L::dh + t] : 0.f;
      const float gwv2 = t < VH ? dv * sm[L::h + t] : 0.f;
      x[CPG + 2] = dgt * dgt;
      x[CPG + 3] = dht * dht;
      x[CPG + 4] = gwv2 * gwv2;
      x[CPG + 5] = 0.f;
      block_sums<CPG + 6>(x, red);
      if (t < 32) st_sc1(a.ws + WS_DW3 + w * DW3R + DW3N + t, t < CPG ? x[t] : 0.f);
      if (t == 0) {
        scal[S_NWF] = x[CPG]; scal[S_NWV1] = x[CPG + 1]; scal[S_NBF] = x[CPG + 2]; scal[S_NBV1] = x[CPG + 3];
        scal[S_NWV2] = x[CPG + 4];
      }
    }
    STAMP(5)
    BARRIER(2)
    STAMP(6)

    // ======== P4: da2 own channels (conv3^T), dW2 / db2 partials ========
    {  // one round trip: conv3 weight columns of the group's channels (wcol[co * 36 + q * 9 + tap] =
       // W3[co][4cg + q][tap]) and the da3 band
      const __amdgpu_buffer_rsrc_t r3 = rsrc(a.p[W3], C3 * 576);
      float wc[5];
#pragma unroll
      for (int k5 = 0; k5 < 5; ++k5) {
        const int e = t + k5 * NT;
        const int co = e / 36, rem = e - co * 36, q = rem / 9, tap = rem - q * 9;
        wc[k5] = e < DW3N ? ld1_sc1(r3, co * 576 + (CPG * cg + q) * 9 + tap) : 0.f;
      }
      f32x4_t bv[BandQ<R, C>::MAXQ];
      band_issue<R, C>(a.ws + WS_DA3, y0, bv);
      // the own conv3 row's gradient (channel 4cg + band: its 4 band partials, band order) and
      // the group's db3, both complete at B3: read here, beside this phase's other loads
      const __amdgpu_buffer_rsrc_t rd3 = rsrc(a.ws + WS_DW3, NWG * DW3R);
      float pb3[2][4];
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          pb3[k2][b] = t + k2 * NT < 576 ? ld1_sc1(rd3, wg_of(cg, b) * DW3R + band * 576 + t + k2 * NT) : 0.f;
      float pdb[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) pdb[b] = t < CPG ? ld1_sc1(rd3, wg_of(cg, b) * DW3R + DW3N + t) : 0.f;
#pragma unroll
      for (int k5 = 0; k5 < 5; ++k5)
        if (t + k5 * NT < DW3N) sm[L::wcol + t + k5 * NT] = wc[k5];
      band_commit<R, C>(big, y0, bv);
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
        if (t + k2 * NT < 576) sm[L::gw3 + t + k2 * NT] = ((pb3[k2][0] + pb3[k2][1]) + pb3[k2][2]) + pb3[k2][3];
      if (t < CPG) scal[S_DB3 + t] = ((pdb[0] + pdb[1]) + pdb[2]) + pdb[3];
    }
    __syncthreads();
    STAMP(23)
    float da2 = 0.f;
    {
      const float z = conv_band<R, C, CPG, 8, true>(big, sm + L::wcol, 36, red);
      if (t < CPG * NPB) {
        da2 = a2keep > 0.f ? z : 0.f;
        sm[L::own2 + t] = da2;
      }
      __syncthreads();
      store_band<R, C>(a.ws + WS_DA2, sm + L::own2, cg, band);
    }
    STAMP(14)
    STAMP(24)
    {  // dW2 partial over the band, two output channels per lane (one window load feeds both):
       // lanes = (input plane, column quarter bit 0), waves = (channel pair, column quarter
       // bit 1, row half); the lane halves are added by a permlane swap, the 4 wave sets
       // through red (the store loop below)
      f32x2_t acc[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) acc[j] = f32x2_t{0.f, 0.f};
      const int ci = lane & 31, qp = wv & 1, xhi = (wv >> 1) & 1, rh = wv >> 2;
      const int xq = (lane >> 5) | (xhi << 1);
      constexpr int RH0 = (BH + 1) / 2;
      const float* d0 = sm + L::own2 + (2 * qp) * NPB;
      if (rh == 0) wgrad2<R, C, RH0, C / 4>(sm + L::a1b, ci, 0, xq * (C / 4), d0, d0 + NPB, acc);
      else wgrad2<R, C, BH - RH0, C / 4>(sm + L::a1b, ci, RH0, xq * (C / 4), d0, d0 + NPB, acc);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        acc[j].x = swap32_add(acc[j].x);
        acc[j].y = swap32_add(acc[j].y);
      }
      if (lane < 32) {
        float* slot = red + ((xhi * 2 + rh) * CPG + 2 * qp) * 288 + ci * 9;
#pragma unroll
        for (int j = 0; j < 9; ++j) { slot[j] = acc[j].x; slot[288 + j] = acc[j].y; }
      }
      __syncthreads();
      STAMP(31)
      float* dst = a.ws + WS_DW2 + w * DW2R;
#pragma unroll
      for (int k3 = 0; k3 < 3; ++k3) {
        const int e = t + k3 * NT;
        if (e < DW2N) {
          const int q2 = e / 288, r2 = e - q2 * 288;
          float sacc = 0.f;
#pragma unroll
          for (int sset = 0; sset < 4; ++sset) sacc += red[(sset * CPG + q2) * 288 + r2];
          st_sc1(dst + e, sacc);
        }
      }
      __syncthreads();
    }
    {
      float x[CPG];
#pragma unroll
      for (int q = 0; q < CPG; ++q) x[q] = (t < CPG * NPB && t / NPB == q) ? da2 : 0.f;
      block_sums<CPG>(x, red);
      if (t < 32) st_sc1(a.ws + WS_DW2 + w * DW2R + DW2N + t, t < CPG ? x[t] : 0.f);
    }
    STAMP(7)
    BARRIER(3)
    STAMP(8)

    // ======== P5: da1 (2 channels on the band), partial dW1 / db1, the group's weight
    // gradients, norm records ========
    {
      // one round trip: conv2 weight columns (wcol[ci * 20 + j * 9 + tap] = W2[ci][2cg + j][tap]),
      // the group's dW2 / db2 band partials and the da2 band
      const __amdgpu_buffer_rsrc_t rw2 = rsrc(a.p[W2], C2 * 288);
      float wc[3];
#pragma unroll
      for (int k3 = 0; k3 < 3; ++k3) {
        const int e = t + k3 * NT;
        const int ci = e / 18, rem = e - ci * 18, j = rem / 9, tap = rem - j * 9;
        wc[k3] = e < DW2N ? ld1_sc1(rw2, ci * 288 + (2 * cg + j) * 9 + tap) : 0.f;
      }
      f32x4_t bv[BandQ<R, C>::MAXQ];
      band_issue<R, C>(a.ws + WS_DA2, y0, bv);
      // the group's dW2 (sum of its 4 bands' partials, band order) and db2
      const __amdgpu_buffer_rsrc_t r2 = rsrc(a.ws + WS_DW2, NWG * DW2R);
      float g2[3];
#pragma unroll
      for (int k3 = 0; k3 < 3; ++k3) {
        const int e = t + k3 * NT;
        float sacc = 0.f;
        if (e < DW2N) {
          float pb[4];
#pragma unroll
          for (int b = 0; b < 4; ++b) pb[b] = ld1_sc1(r2, wg_of(cg, b) * DW2R + e);
#pragma unroll
          for (int b = 0; b < 4; ++b) sacc += pb[b];
        }
        g2[k3] = sacc;
      }
      if (t < CPG) {  // db2 (db3 was summed in P4)
        float pb[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) pb[b] = ld1_sc1(r2, wg_of(cg, b) * DW2R + DW2N + t);
        scal[S_DB2 + t] = ((pb[0] + pb[1]) + pb[2]) + pb[3];
      }
#pragma unroll
      for (int k3 = 0; k3 < 3; ++k3)
        if (t + k3 * NT < DW2N) {  // planes of 18 weights at a 20-float pitch (16-byte rows)
          const int e = t + k3 * NT;
          sm[L::wcol + e + 2 * (e / 18)] = wc[k3];
        }
      band_commit<R, C>(big, y0, bv);
#pragma unroll
      for (int k3 = 0; k3 < 3; ++k3)
        if (t + k3 * NT < DW2N) sm[L::gw2 + t + k3 * NT] = g2[k3];
      __syncthreads();
      STAMP(25)
      const float z = conv_band<R, C, 2, 8, true>(big, sm + L::wcol, 20, red);
      float da1 = 0.f;
      if (t < 2 * NPB) {
        const int j = t / NPB, pos = t - j * NPB, y = y0 + pos / C, x = pos - (pos / C) * C;
        da1 = sm[L::a1b + (2 * cg + j) * L::PB + (y - y0 + 1) * L::RS + x + 1] > 0.f ? z : 0.f;
        sm[L::own + t] = da1;
      }
      __syncthreads();
      STAMP(26)
      float rec = 0.f;
      if (t < 18) {  // dW1 partial: sum over the input's nonzeros of da1[pos] * val, pos = pixel - tap + 1
        const int j = t / 9, tap = t - j * 9, ky = tap / 3, kx = tap - ky * 3, nnz = (int)scal[S_NNZ];
        for (int jn = 0; jn < nnz; ++jn) {
          const int pp = __float_as_int(sm[L::nzpos + jn]);
          const int y = (pp >> 8) - ky + 1, xx = (pp & 255) - kx + 1;
          if (y >= y0 && y < y0 + BH && (unsigned)xx < (unsigned)C)
            rec = fmaf(sm[L::own + j * NPB + (y - y0) * C + xx], sm[L::nzval + jn], rec);
        }
      }
      float x[6];
      x[0] = (t < NPB) ? da1 : 0.f;           // db1 partial, channel 2cg
      x[1] = (t >= NPB && t < 2 * NPB) ? da1 : 0.f;  // channel 2cg + 1
      x[2] = 0.f; x[3] = 0.f;
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
        if (t + k2 * NT < 576) {
          const float g3 = sm[L::gw3 + t + k2 * NT];
          x[2] = fmaf(g3, g3, x[2]);
        }
#pragma unroll
      for (int k3 = 0; k3 < 3; ++k3) {
        const int e = t + k3 * NT;
        if (e < DW2N) x[3] = fmaf(g2[k3], g2[k3], x[3]);
      }
      x[4] = x[5] = 0.f;
      block_sums<6>(x, red);
      if (wv == 0) {
        const bool isdw = lane >= NP_DW1 && lane < NP_DW1 + 18;
        const float dw = __shfl(rec, isdw ? lane - NP_DW1 : 0);  // whole wave: lanes 0..17 hold the taps
        const bool b0 = band == 0;  // the group's conv2 / bias sums are counted once, by band 0
        float o = 0.f;
        if (isdw) o = dw;
        else if (lane == NP_W2) o = b0 ? x[3] : 0.f;
        else if (lane == NP_B2) {
          float sq = 0.f;
          for (int q = 0; q < CPG; ++q) sq = fmaf(scal[S_DB2 + q], scal[S_DB2 + q], sq);
          o = b0 ? sq : 0.f;
        } else if (lane == NP_W3) o = x[2];  // every band: its own conv3 row
        else if (lane == NP_B3) {
          float sq = 0.f;
          for (int q = 0; q < CPG; ++q) sq = fmaf(scal[S_DB3 + q], scal[S_DB3 + q], sq);
          o = b0 ? sq : 0.f;
        } else if (lane == NP_WF) o = scal[S_NWF];
        else if (lane == NP_WV1) o = scal[S_NWV1];
        else if (lane == NP_DB1) o = x[0];
        else if (lane == NP_DB1 + 1) o = x[1];
        if (lane < REC) st_sc1(a.ws + WS_NP + w * REC + lane, o);
      }
    }
    STAMP(9)
    BARRIER(4)
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
    if (t < 288) {  // conv1 weight gradient: the 4 band records of channel t / 9's group
      const int cj = t / 9, tap = t - cj * 9, g = cj >> 1, o = NP_DW1 + (cj & 1) * 9 + tap;
      gw1 = ((red[wg_of(g, 0) * REC + o] + red[wg_of(g, 1) * REC + o]) + red[wg_of(g, 2) * REC + o]) +
            red[wg_of(g, 3) * REC + o];
    }
    if (t < C1) {
      const int g = t >> 1, o = NP_DB1 + (t & 1);
      gb1 = ((red[wg_of(g, 0) * REC + o] + red[wg_of(g, 1) * REC + o]) + red[wg_of(g, 2) * REC + o]) +
            red[wg_of(g, 3) * REC + o];
    }
    {
      // sums over the 64 records of slots 0..5: wave v sums slot v (lane = record; the same
      // DPP association in every workgroup)
      float own_sum = wv < 6 ? sum64(red[lane * REC + wv]) : 0.f;
      __syncthreads();  // red (records) is reused as the reduction scratch below
      float x[2] = {gw1 * gw1, gb1 * gb1};
      block_sums<2>(x, red);
      if (wv < 6 && lane == 0) scal[S_RED8 + wv] = own_sum;
      __syncthreads();
      if (t == 0) {
        const float S[NTENS] = {x[0], x[1], scal[S_RED8 + NP_W2], scal[S_RED8 + NP_B2], scal[S_RED8 + NP_W3],
                                scal[S_RED8 + NP_B3], scal[S_RED8 + NP_WF], scal[S_NBF], scal[S_RED8 + NP_WV1],
                                scal[S_NBV1], scal[S_NWV2], dv * dv};
        float tot = 0.f;
        for (int i = 0; i < NTENS; ++i) {
          const float n = sqrtf(S[i]);
          tot = fmaf(n, n, tot);
        }
        const float total = sqrtf(tot);
        const float c = a.max_norm / (total + 1e-6f);
        scal[S_CLIP] = c > 1.0f ? 1.0f : c;
      }
      __syncthreads();
    }
    STAMP(28)
    {
      const float clip = scal[S_CLIP], ns = scal[S_NS], bc2s = scal[S_BC2S];
      // redundant small tensors: their gradients go through LDS scratch (red) so the batched
      // form applies: conv1 weight [0, 288), conv1 bias [288, 320), value_head.2.weight
      // [320, 448) (dv * h)
      if (t < 288) red[t] = gw1;
      if (t < C1) red[288 + t] = gb1;
      if (t < VH) red[320 + t] = dv * sm[L::h + t];
      __syncthreads();
      {  // the five as one index space (conv1 w | b, fc_global.bias, value_head.0.bias,
         // value_head.2.weight: 832 elements, two per thread): two LDS round trips instead of five
        constexpr int NSM = C1 * 9 + C1 + HID + VH + VH;
        static_assert(NSM <= 2 * NT, "two small-tensor elements per thread");
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int u = t + j * NT;
          float* bp;
          const float* gp;
          int nn, ee;
          if (u < 288) { bp = sm + L::w1; nn = 288; gp = red; ee = u; }
          else if (u < 320) { bp = sm + L::b1; nn = C1; gp = red + 288; ee = u - 288; }
          else if (u < 576) { bp = sm + L::bf; nn = HID; gp = sm + L::dg; ee = u - 320; }
          else if (u < 704) { bp = sm + L::bv1; nn = VH; gp = sm + L::dh; ee = u - 576; }
          else { bp = sm + L::wv2; nn = VH; gp = red + 320; ee = u - 704; }
          if (u < NSM) {
            float pp = bp[ee], mm = bp[nn + ee], vv = bp[2 * nn + ee];
            adam(pp, mm, vv, gp[ee], clip, a, ns, bc2s);
            bp[ee] = pp; bp[nn + ee] = mm; bp[2 * nn + ee] = vv;
          }
        }
      }
      if (t == 0) {
        float p = sm[L::bv2], m = sm[L::bv2 + 1], v = sm[L::bv2 + 2];
        adam(p, m, v, dv, clip, a, ns, bc2s);
        sm[L::bv2] = p; sm[L::bv2 + 1] = m; sm[L::bv2 + 2] = v;
      }
      if (t < 2 * CPG) {  // b2 (t < 4), b3 (4 <= t < 8) of the group
        const int q = t & 3, which = t >> 2;
        float* base = sm + L::b23 + (which ? 12 : 0);
        float p = base[q], m = base[4 + q], v = base[8 + q];
        adam(p, m, v, scal[(which ? S_DB3 : S_DB2) + q], clip, a, ns, bc2s);
        base[q] = p; base[4 + q] = m; base[8 + q] = v;
      }
      const bool pub = band == 0;  // band 0 publishes the group's rows for the column reads of P4 / P5
      float p2[3];
      STAMP(29)
      adam_lds<3>(sm + L::w2r, DW2N, t, sm + L::gw2, clip, a, ns, bc2s, p2);
#pragma unroll
      for (int k3 = 0; k3 < 3; ++k3)  // the conv copy (read by the next step's conv2 after B5's syncs)
        if (t + k3 * NT < DW2N) sm[L::w2t + plane_major<C1>(t + k3 * NT)] = p2[k3];
      {  // the own conv3 row: params in w3r (row `band`), moments in w3mv
        float p3[2], m3[2], v3[2], g3v[2];
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
          const int e = t + k2 * NT;
          if (e < 576) {
            p3[k2] = sm[L::w3r + plane_major<C2>(band * 576 + e)]; m3[k2] = sm[L::w3mv + e]; v3[k2] = sm[L::w3mv + 576 + e];
            g3v[k2] = sm[L::gw3 + e];
          }
        }
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
          const int e = t + k2 * NT;
          if (e < 576) {
            adam(p3[k2], m3[k2], v3[k2], g3v[k2], clip, a, ns, bc2s);
            sm[L::w3mv + e] = m3[k2]; sm[L::w3mv + 576 + e] = v3[k2];
            st_sc1(a.p[W3] + (CPG * cg + band) * 576 + e, p3[k2]);  // reloaded by the group after B1
          }
        }
      }
      STAMP(30)
      if (pub) {
#pragma unroll
        for (int k3 = 0; k3 < 3; ++k3)
          if (t + k3 * NT < DW2N) st_sc1(a.p[W2] + CPG * cg * 288 + t + k3 * NT, p2[k3]);
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
#undef READY

  // ---- write back what stayed on chip (tensor pointers from the LDS table: the kernel
  // arguments need not stay live in SGPRs across the step loop) ----
  float* const* P = reinterpret_cast<float* const*>(sm + L::ptab);
  float* const* M = P + NTENS;
  float* const* V = P + 2 * NTENS;
  {
    const int t = threadIdx.x, w = blockIdx.x, cg = wg_cg(w), band = wg_band(w);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int jj = 8 * fc_half(t) + j;
      const int e = fc_row(t) * NPOOL + (CPG * cg + (jj >> 2)) * 16 + band * 4 + (jj & 3);
      P[WF][e] = wf[j]; M[WF][e] = mf[j]; V[WF][e] = vf[j];
    }
    M[WV1][w * 512 + t] = mv1; V[WV1][w * 512 + t] = vv1;
    for (int e = t; e < 576; e += NT) {  // the own conv3 row's moments (its params were published)
      M[W3][(CPG * cg + band) * 576 + e] = sm[L::w3mv + e]; V[W3][(CPG * cg + band) * 576 + e] = sm[L::w3mv + 576 + e];
    }
    if (band == 0) {
      for (int e = t; e < DW2N; e += NT) {
        M[W2][CPG * cg * 288 + e] = sm[L::w2r + DW2N + e]; V[W2][CPG * cg * 288 + e] = sm[L::w2r + 2 * DW2N + e];
      }

      if (t < CPG) {
        const int ch = CPG * cg + t;
        P[B2][ch] = sm[L::b23 + t]; M[B2][ch] = sm[L::b23 + 4 + t]; V[B2][ch] = sm[L::b23 + 8 + t];
        P[B3][ch] = sm[L::b23 + 12 + t]; M[B3][ch] = sm[L::b23 + 16 + t]; V[B3][ch] = sm[L::b23 + 20 + t];
      }
    }
    if (w == 0) {
      for (int i = t; i < C1 * 9; i += NT) {
        P[W1][i] = sm[L::w1 + i]; M[W1][i] = sm[L::w1 + 288 + i]; V[W1][i] = sm[L::w1 + 576 + i];
      }
      if (t < C1) { P[B1][t] = sm[L::b1 + t]; M[B1][t] = sm[L::b1 + 32 + t]; V[B1][t] = sm[L::b1 + 64 + t]; }
      if (t < HID) { P[BF][t] = sm[L::bf + t]; M[BF][t] = sm[L::bf + 256 + t]; V[BF][t] = sm[L::bf + 512 + t]; }
      if (t < VH) {
        P[BV1][t] = sm[L::bv1 + t]; M[BV1][t] = sm[L::bv1 + 128 + t]; V[BV1][t] = sm[L::bv1 + 256 + t];
        P[WV2][t] = sm[L::wv2 + t]; M[WV2][t] = sm[L::wv2 + 128 + t]; V[WV2][t] = sm[L::wv2 + 256 + t];
      }
      if (t == 0) { P[BV2][0] = sm[L::bv2]; M[BV2][0] = sm[L::bv2 + 1]; V[BV2][0] = sm[L::bv2 + 2]; }
    }
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

int arch_update_max_nonzeros() { return au::MAXNZ; }

int64_t arch_update_workspace_bytes() { return (int64_t)au::WS_FLOATS * 4; }

template <int R>
static hipError_t launch_sized(const au::Args& a, hipStream_t st) {
  const size_t lds = (size_t)au::Lay<R, R>::total * 4;
  hipError_t e = hipFuncSetAttribute((const void*)au::arch_update_kernel<R, R>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((au::arch_update_kernel<R, R>), dim3(au::NWG), dim3(au::NT), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_arch_update(float* const* p, float* const* m, float* const* v, const float* grid, int R, int C,
                              const float* target, int k, const float* adam_sc, float* vloss, void* ws, double beta1,
                              double beta2, double eps, double max_norm, double value_coeff, hipStream_t st) {
  if (!arch_update_supported(R, C)) return hipErrorInvalidValue;
  au::Args a;
  for (int i = 0; i < au::NTENS; ++i) { a.p[i] = p[i]; a.m[i] = m[i]; a.v[i] = v[i]; }
  a.grid = grid; a.target = target; a.vloss = vloss; a.ws = (float*)ws;
  a.stamps = g_arch_stamps;
  a.k = k;
  a.spin_limit = 1u << 25;
  if (const char* sl = getenv("HEIST_ARCH_SPIN_LIMIT")) a.spin_limit = (unsigned)strtoul(sl, nullptr, 10);
  a.adam_sc = adam_sc;
  a.lerp_w = (float)(1.0 - beta1);
  a.beta2f = (float)beta2;
  a.c2 = (float)(1.0 - beta2);
  a.eps = (float)eps;
  a.max_norm = (float)max_norm;
  a.grad_out = (float)value_coeff;
  hipError_t e = hipMemsetAsync(a.ws + au::WS_XB, 0, au::CW_WORDS * sizeof(float), st);  // through the end
  if (e != hipSuccess) return e;
  switch (R) {
    case 20: return launch_sized<20>(a, st);
    case 16: return launch_sized<16>(a, st);
    case 12: return launch_sized<12>(a, st);
    default: return launch_sized<8>(a, st);
  }
}

}  // namespace heist
