// heist_train_conv.hip -- the Solver backbone's fp32 training convolutions on fp32 MFMA.
//
// The PPO update (agents/solver.py:157-199) runs SolverNetwork.features (networks.py:93-100:
// relu(conv1) -> relu(conv2) -> relu(conv3) -> AdaptiveAvgPool2d(4, 4), 3 -> 32 -> 64 -> 64
// channels, 3 x 3, pad 1) forward and backward on 16,384-sample minibatches: ~2.2 TFLOP per
// optimizer step, all of it in six convolution passes that MIOpen ran at 0.39-0.70 of the
// 157 TF fp32 matrix peak (profiles/r05f_train_kernel_stats.csv).  Here every pass is one
// persistent kernel on v_mfma_f32_16x16x4_f32 -- exact fp32: each MFMA is a k-ordered chain
// of fmaf (cdna_hip_programming.md, 'FP32-input MFMA'), so results differ from MIOpen's or
// the CPU's only by the order of the fp32 sums.
//
// Layout.  Activations are [n][R][C][P] fp32 with P = channels + 4 (channels 0..P-5 are
// data, the 4 pad words are never read): a band of image rows is then one contiguous HBM
// range that LDS-DMA (global_load_lds_dwordx4) copies straight into a padded LDS image whose
// 16-byte reads are bank-conflict free (16 lanes at a 272- or 144-byte position pitch cover
// all 64 banks).  The network input (3 channels) is [n][R][C][4], channel 3 zero.
//
// Work.  A unit is a BAND: 4 output rows of one sample (4C positions = C/4 tiles of 16).  The
// kernels are persistent (one 512-thread workgroup per CU) and draw units from an atomic
// queue, so a kernel that shares the chip with another (the Architect's update kernel holds
// 64 CUs beside the Solver's update, training.py) keeps every CU it gets busy; every output
// element is computed by exactly one wave, so results do not depend on the scheduling.
//
//  conv_a_kernel  (forward and data gradient: a 3 x 3 convolution with register weights)
//    D[co][pos] = sum over (tap, ci) of W[co][tap][ci] * X[pos + tap][ci]: the weights are the
//    MFMA's A operand, held in VGPRs for the whole kernel (144 per lane at 64 -> 64), the
//    activations its B operand, one ds_read_b128 feeding 4 MFMA k-steps.  Wave w owns one
//    16-channel output tile of one band of the unit for all its C/4 position tiles; a lane ends
//    with 4 consecutive channels of one position per tile (one 16-byte store).  (The transposed
//    orientation, D[pos][co] with the activations as A, would let a pool MFMA sum over the
//    positions of D's rows; measured 3-8 % slower on every pass, it was not kept.)  Epilogue:
//    forward  y = relu(D + bias) (torch: conv + b rounded, then max(., 0)), and the ReLU mask bits;
//    backward d = (a > 0) ? D : 0 with a the saved activation of the layer below (threshold_
//             backward on the saved output), the data gradient being the convolution with the
//             transposed, flipped weights (packed by conv_pack_kernel).
//  conv_w_kernel  (weight and bias gradient)
//    dW[co][tap][ci] = sum over samples and positions of dY[pos][co] * X[pos + tap][ci], and
//    db[co] = sum of dY[pos][co] (one more MFMA tile whose B operand is 1.0): positions are
//    the MFMA's k (4 per k-step), each wave accumulates one 16-channel row tile of dW over a
//    CHUNK of 40 bands in registers and writes it as that chunk's partial; conv_w_reduce
//    sums the partials in chunk order (deterministic, no float atomics).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#pragma clang fp contract(off)

#ifndef HEIST_TC_PADW
#define HEIST_TC_PADW 1  // conv1's activation rows written whole, pad words included (A/B: -DHEIST_TC_PADW=0)
#endif

namespace heist {
namespace tc {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 512;  // 8 waves, 2 per SIMD
constexpr int kChunkBands = 40;  // bands per weight-gradient partial (8 samples of 20 rows)

template <int CH>
struct Pitch {
  static constexpr int v = CH == 4 ? 4 : CH + 4;
};

// LDS-DMA of 16 bytes per active lane: lane i's bytes land at lds_dst + 16 i (M0 holds the
// wave-uniform base; set and restored inside the statement).  Waited for with an explicit
// s_waitcnt vmcnt(0) before the barrier that publishes the buffer.
__device__ __forceinline__ void lds_dma16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

__device__ __forceinline__ void wait_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// vmcnt(0) as the builtin, which the compiler's wait insertion sees (an asm wait it does not):
// after the prologue's global loads (weights, bias), so that it does not put a vmcnt(0) at
// their first use INSIDE the unit loop, where it would also wait for the next unit's LDS-DMA
// (issued just before) every iteration.  Encoding: vmcnt 0, expcnt 7, lgkmcnt 15.
__device__ __forceinline__ void settle_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// vmcnt(N): every vector memory op of this wave but the last N issued has completed (they
// complete in issue order): the unit's DMA, issued before the previous unit's N epilogue
// stores, has landed without waiting for those stores.
template <int N>
__device__ __forceinline__ void wait_vm_keep() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// The work queue's next unit, by one lane: the atomic in asm, so the compiler neither waits for
// it where it is issued nor knows its result is pending; queue_value() waits (vmcnt(0): by
// then nothing else is in flight) and hands the value over.
__device__ __forceinline__ int queue_draw(int* queue) {
  int v;
  asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=&v"(v) : "v"(queue), "v"(1) : "memory");
  return v;
}
__device__ __forceinline__ int queue_value(int v) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(v)::"memory");
  return v;
}

typedef __attribute__((address_space(8))) void* rsrc_t;
// a raw buffer resource over `bytes` bytes at p (0 bytes: every store through it is dropped,
// but still issued and counted -- the epilogue's store count is the same in every wave)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_over(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
constexpr int kOOB = 0x7FFFFFF0;  // a buffer offset past any resource: the store is dropped

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)p; }

typedef __attribute__((address_space(3))) float lds_float;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) f4 lds_f4_t;
typedef __attribute__((address_space(3))) f2 lds_f2_t;

// LDS reads through address-space-3 pointers (ds_read_*): a generic pointer that the compiler
// cannot prove is LDS becomes a flat load (both counters, the slower path)
__device__ __forceinline__ const lds_float* as_lds(const float* p) {
  return reinterpret_cast<const lds_float*>((uint32_t)(uintptr_t)p);
}
__device__ __forceinline__ f4 lds_f4(const float* base, int off) { return *reinterpret_cast<const lds_f4_t*>(as_lds(base) + off); }
__device__ __forceinline__ float lds_f1(const float* base, int off) { return as_lds(base)[off]; }
__device__ __forceinline__ f2 lds_f2(const float* base, int off) {
  return *reinterpret_cast<const lds_f2_t*>(as_lds(base) + off);
}

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// Copy `bytes` (a multiple of 16) from global src to LDS dst, wave-instruction pieces of
// 1 KB handed round-robin over the workgroup's waves starting at wave `w0` (wave-uniform).
__device__ __forceinline__ void dma_range(const float* src, float* dst, int bytes, int piece0, int wid, int lane) {
  const int pieces = (bytes + 1023) >> 10;
  for (int k = (wid - piece0 % 8 + 8) % 8; k < pieces; k += 8) {
    const int off = (k << 10) + (lane << 4);
    if (off < bytes)
      lds_dma16(reinterpret_cast<const char*>(src) + off,
                (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds_addr(dst) + (uint32_t)(k << 10))));
  }
}

// The work queue's exit: the last workgroup to leave resets both counters (queue[0] units
// drawn, queue[1] workgroups done), so the next launch on the stream finds them zero.
__device__ __forceinline__ void queue_exit(int* queue) {
  if (threadIdx.x == 0 && atomicAdd(queue + 1, 1) == (int)gridDim.x - 1) {
    atomicExch(queue, 0);
    atomicExch(queue + 1, 0);
  }
}

__device__ __forceinline__ void zero_range(float* dst, int bytes, int wid, int lane) {
  for (int off = (wid * 64 + lane) * 16; off < bytes; off += kThreads * 16)
    *reinterpret_cast<f4*>(reinterpret_cast<char*>(dst) + off) = f4{0.f, 0.f, 0.f, 0.f};
}

// Input band image of band gb (sample gb / NB, output rows 4(gb % NB) .. +3) into LDS
// `img` [6][C + 2][PI]: padded row rr <- image row y0 - 1 + rr, interior columns only (the
// two border columns were zeroed once); rows outside the image are zeroed.
template <int CI, int R, int C>
__device__ __forceinline__ void load_band(const float* x, float* img, int gb, int piece0, int wid, int lane) {
  constexpr int PI = Pitch<CI>::v, RP = C + 2, NB = R / 4, ROWB = C * PI * 4;
  const int smp = gb / NB, y0 = (gb % NB) * 4;
#pragma unroll
  for (int rr = 0; rr < 6; ++rr) {
    const int y = y0 - 1 + rr;
    float* dst = img + (rr * RP + 1) * PI;
    if (y >= 0 && y < R)
      dma_range(x + ((size_t)smp * R + y) * C * PI, dst, ROWB, piece0 + rr * ((ROWB + 1023) >> 10), wid, lane);
    else
      zero_range(dst, ROWB, wid, lane);
  }
}

// ---------------------------------------------------------------------------------------
// conv_a_kernel: y[p][co] = epilogue(sum_{tap, ci} W[co][tap][ci] x[p + tap][ci]).
//   CI, CO input / output channels; S: the k (input channel) range split over S waves whose
//   partial tiles are summed through LDS (S = 2 for 32 output channels, so that 8 waves have
//   work); MODE 0 forward (bias, ReLU), 1 data gradient (mask by the saved activation > 0).
//   ReLU masks travel as bits: [n][R][C][CO / 4] uint8, bit r of byte k = channel 4 k + r > 0
//   (a lane's own 4 channels: no cross-lane gather).  The forward writes its output's
//   (mask_out, optional); the data gradient reads its output channels' (mask_in: the layer
//   below's), DMA'd into LDS with the band, so its epilogue waits for no global load.
struct ConvAArgs {
  const float* x;       // [n][R][C][PI]
  const float* frag;    // packed weights (conv_pack_kernel)
  const float* bias;    // [CO] (MODE 0)
  const uint8_t* mask_in;  // [n][R][C][CO / 4] (MODE 1)
  uint8_t* mask_out;       // [n][R][C][CO / 4] or null (MODE 0)
  float* y;             // [n][R][C][PO]
  int* queue;           // [2]: units drawn, workgroups done (zero between launches: queue_exit)
  int n;
};

template <int CI, int CO, int S, int MODE, int R, int C>
struct ConvAGeom {
  static constexpr int PI = Pitch<CI>::v, PO = Pitch<CO>::v, NCT = CO / 16, BPU = 8 / (NCT * S);
  static constexpr int PT = C / 4, RP = C + 2, NB = R / 4;
  static constexpr int BAND_F = 6 * RP * PI, BUF_F = BPU * BAND_F;
  static constexpr int MASK_B = 4 * C * CO / 4;            // mask bytes per band (MODE 1)
  static constexpr int MASK_F = MODE == 1 ? BPU * MASK_B / 4 : 0;  // floats per buffer
  static constexpr int KBW = CI == 4 ? 1 : (CI / 16) / S;  // 16-channel blocks per tap of a wave
  static constexpr int NWR = CI == 4 ? 9 : 36 * KBW;       // weight registers per lane
  static constexpr int LDS = 2 * (BUF_F + MASK_F) * 4 + 64;
  static_assert(NCT * S * BPU == 8, "8 waves");
  static_assert(MASK_B % 16 == 0, "mask rows are whole DMA lanes");
  static_assert(C % 4 == 0 && R % 4 == 0, "bands of 4 rows, tiles of 16 positions");
  static_assert(S == 1 || (PT * 256 <= C * PI && BPU * NCT <= 6), "a wave's k-split partials fit in a row interior");
};

template <int CI, int CO, int S, int MODE, int R, int C>
__global__ __launch_bounds__(kThreads, 1) void conv_a_kernel(ConvAArgs a) {
  using G = ConvAGeom<CI, CO, S, MODE, R, C>;
  constexpr int PI = G::PI, PO = G::PO, NCT = G::NCT, BPU = G::BPU, PT = G::PT, RP = G::RP, NB = G::NB;
  constexpr int KBW = G::KBW, NWR = G::NWR;
  extern __shared__ f4 smem4[];
  float* smem = reinterpret_cast<float*>(smem4);
  float* buf[2] = {smem, smem + G::BUF_F};
  float* mbuf = smem + 2 * G::BUF_F;  // [2][BPU][MASK_B] uint8 (MODE 1)
  int* slot = reinterpret_cast<int*>(smem + 2 * (G::BUF_F + G::MASK_F));
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = wid % NCT, s = (wid / NCT) % S, bslot = wid / (NCT * S);
  const int j = lane & 15, g = lane >> 4;
  const int nbands = a.n * NB, nunits = (nbands + BPU - 1) / BPU;

  // weights: lane (row i = j, k group g) of output tile c, k range s
  float w[NWR];
  {
    const f4* wf = reinterpret_cast<const f4*>(a.frag) + (size_t)(c * S + s) * (NWR / 4 > 0 ? NWR / 4 : 1) * 64;
    if constexpr (CI == 4) {
#pragma unroll
      for (int t = 0; t < 9; ++t) w[t] = a.frag[(size_t)(c * 9 + t) * 64 + lane];
    } else {
#pragma unroll
      for (int q = 0; q < NWR / 4; ++q) {
        const f4 v = wf[q * 64 + lane];
        w[4 * q] = v[0];
        w[4 * q + 1] = v[1];
        w[4 * q + 2] = v[2];
        w[4 * q + 3] = v[3];
      }
    }
  }
  f4 bias4 = {0.f, 0.f, 0.f, 0.f};  // this lane's output channels 16 c + 4 g + r
  if constexpr (MODE == 0) bias4 = *reinterpret_cast<const f4*>(a.bias + 16 * c + 4 * g);
  settle_vm();

  zero_range(smem, 2 * G::BUF_F * 4, wid, lane);  // border columns stay zero for the whole kernel
  if (tid == 0) {
    slot[0] = atomicAdd(a.queue, 1);
    slot[1] = atomicAdd(a.queue, 1);
  }
  __syncthreads();
  int cur = slot[0], nxt = slot[1];
  auto issue = [&](int u, int par) {
    for (int bb = 0; bb < BPU; ++bb) {
      const int gb = u * BPU + bb;
      if (gb >= nbands) continue;
      load_band<CI, R, C>(a.x, buf[par] + bb * G::BAND_F, gb, bb * 7, wid, lane);
      if constexpr (MODE == 1) {
        const int smp = gb / NB, y0 = (gb % NB) * 4;
        dma_range(reinterpret_cast<const float*>(a.mask_in + ((size_t)smp * R + y0) * C * (CO / 4)),
                  mbuf + (par * BPU + bb) * (G::MASK_B / 4), G::MASK_B, 3 + bb, wid, lane);
      }
    }
  };
  if (cur < nunits) issue(cur, 0);
  // per-lane LDS offsets of the position tiles (tap (0, 0) corner, channel group g)
  int pbase[PT];
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    const int q = 16 * t + j, y = q / C, xx = q % C;
    pbase[t] = (y * RP + xx) * PI + (CI == 4 ? g : 4 * g + 16 * KBW * s);
  }
  // epilogue stores per wave per unit, the same in every wave (dropped ones included)
  constexpr int NST = PT * (1 + (MODE == 0 ? 1 : 0) + (MODE == 0 && CI == 4 && HEIST_TC_PADW ? 1 : 0));
  for (int it = 0; cur < nunits; ++it) {
    float* img = buf[it & 1] + bslot * G::BAND_F;
    // this unit's DMA, not the previous unit's epilogue stores issued after it
    if (it == 0) wait_dma();
    else wait_vm_keep<NST>();
    __syncthreads();  // the unit's images are in LDS; everyone is done with the other buffer
    int drawn = 0;  // the unit after next (tid 0), published after the compute
    if (tid == 0) drawn = queue_draw(a.queue);
    if (nxt < nunits) issue(nxt, (it + 1) & 1);
    const int gb = cur * BPU + bslot;
    f4 acc[PT];
#pragma unroll
    for (int t = 0; t < PT; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
    if (gb < nbands) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = ((tap / 3) * RP + tap % 3) * PI;
        if constexpr (CI == 4) {
          float xv[PT];
#pragma unroll
          for (int t = 0; t < PT; ++t) xv[t] = lds_f1(img, pbase[t] + toff);
#pragma unroll
          for (int t = 0; t < PT; ++t) acc[t] = mfma(w[tap], xv[t], acc[t]);
        }
      }
      if constexpr (CI != 4) {
        // (tap, cb) blocks in order, block b + 1's activations read into the other register
        // set before block b's MFMAs (the compiler reschedules them: it keeps reads 1-4 MFMAs
        // ahead; pinning them a whole block ahead with sched_barrier or sched_group_barrier
        // measured no faster, the SIMD's second wave hides the LDS latency, r06o / r06t)
        constexpr int NBK = 9 * KBW;
        auto boff = [&](int bk) { return ((bk / KBW / 3) * RP + (bk / KBW) % 3) * PI + 16 * (bk % KBW); };
        f4 xv[2][PT];
#pragma unroll
        for (int t = 0; t < PT; ++t) xv[0][t] = lds_f4(img, pbase[t] + boff(0));
#pragma unroll
        for (int bk = 0; bk < NBK; ++bk) {
          if (bk + 1 < NBK) {
#pragma unroll
            for (int t = 0; t < PT; ++t) xv[(bk + 1) & 1][t] = lds_f4(img, pbase[t] + boff(bk + 1));
          }
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int t = 0; t < PT; ++t) acc[t] = mfma(w[bk * 4 + e], xv[bk & 1][t][e], acc[t]);
        }
      }
    }
    if constexpr (S == 2) {  // k halves: wave s = 1 hands its partial tiles to wave s = 0 through LDS
      __syncthreads();       // every wave is done reading this unit's images
      // the partials go to the interior of image row (band slot, c) of this buffer: the two
      // border columns of every row stay zero for the rest of the kernel (the next images are
      // DMA'd / zeroed over the interiors only)
      float* part = buf[it & 1] + ((bslot * NCT + c) * RP + 1) * PI;
      if (s == 1)
#pragma unroll
        for (int t = 0; t < PT; ++t) *reinterpret_cast<f4*>(part + t * 256 + lane * 4) = acc[t];
      __syncthreads();
      if (s == 0)
#pragma unroll
        for (int t = 0; t < PT; ++t) acc[t] += lds_f4(part, t * 256 + lane * 4);
    }
    if (tid == 0) slot[2 + (it & 1)] = queue_value(drawn);
    {
      // D[co][pos]: lane (j, g) holds channels 16 c + 4 g + r of band position 16 t + j; the band's
      // rows are contiguous, so band position q is image position (smp R + y0) C + q.  Every wave
      // issues the same NST buffer stores: a wave with no output (s = 1, or no band) stores
      // through empty resources (dropped), so the next unit's counted wait holds in every wave.
      const bool out = s == 0 && gb < nbands;
      const int smp = gb / NB, y0 = (gb % NB) * 4;
      const size_t bandpos = out ? ((size_t)smp * R + y0) * C : 0;
      const auto ry = rsrc_over(a.y + bandpos * PO, out ? 4 * C * PO * 4 : 0);
      const auto rm = rsrc_over(a.mask_out ? a.mask_out + bandpos * (CO / 4) : nullptr,
                                out && a.mask_out ? 4 * C * (CO / 4) : 0);
      const lds_u8* mk = reinterpret_cast<const lds_u8*>(as_lds(mbuf)) + ((it & 1) * BPU + bslot) * G::MASK_B;
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        const int q = 16 * t + j;
        f4 v = acc[t];
        if constexpr (MODE == 0) {
          v += bias4;  // conv + b rounded once, then ReLU
          uint32_t bits = 0;  // bit r: channel 16 c + 4 g + r of position q > 0
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            bits |= (uint32_t)(v[r] > 0.f) << r;
            v[r] = v[r] > 0.f ? v[r] : 0.f;
          }
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)bits, rm, q * (CO / 4) + 4 * c + g, 0, 0);
        } else {
          const uint32_t bits = (uint32_t)mk[q * (CO / 4) + 4 * c + g];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bits >> r) & 1u ? v[r] : 0.f;
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ry, (q * PO + 16 * c + 4 * g) * 4, 0, 0);
        // conv1's forward (memory-bound) writes the position's 4 pad words as well (zeros, never
        // read): whole 128-B lines, no read-modify-write of a partly written line (0.445 ->
        // 0.346 ms at 16,384 samples); in the MFMA-bound passes the extra store cost 0.3-1.2 %
        if constexpr (MODE == 0 && CI == 4 && HEIST_TC_PADW)
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, ry,
                                                 c == NCT - 1 && g == 3 ? (q * PO + CO) * 4 : kOOB, 0, 0);
      }
    }
    __syncthreads();  // slot written; this buffer free for the unit after next
    cur = nxt;
    nxt = slot[2 + (it & 1)];
  }
  queue_exit(a.queue);
}

// ---------------------------------------------------------------------------------------
// conv_w_kernel: weight and bias gradient partials per chunk of kChunkBands bands.
//   dY [n][R][C][PD] (PD = CO + 4), X [n][R][C][PI]; partial [chunk][WSZ] floats.  An
//   iteration takes BPI bands (one LDS buffer: their X images, then their dY rows), the next
//   iteration's bands DMA'd into the other buffer meanwhile.  The band's k-steps (4 positions
//   each) are unrolled, so every LDS address is a lane base plus an immediate.
//   CI >= 32: wave (m = row tile, h) accumulates the tiles (tap, qq) whose column j holds input
//   channel ci = col_ci(j, h, qq) -- a bank-conflict-free assignment: the 16 lanes of a k group
//   read QW consecutive words each, and the next k group (the next position, 4 banks further)
//   lands on the banks this one leaves free (ds_read_b64: 2 x 32-lane groups; ds_read_b32: 32
//   banks).  CI == 4: wave (m, kg) takes every 4th k-step (k group kg) for both column tiles:
//   columns 0..26 the 27 (tap, ci) pairs of the 3 real input channels, column 27 the bias
//   (B operand 1.0), 28..31 zero; the four k groups' tiles are summed in a fixed order through
//   LDS at the chunk's end.
struct ConvWArgs {
  const float* dy;
  const float* x;
  float* partial;
  int* queue;
  int n;
};

template <int CI, int CO, int R, int C>
struct ConvWGeom {
  static constexpr int PI = Pitch<CI>::v, PD = Pitch<CO>::v, MT = CO / 16, WPM = 8 / MT;
  static constexpr int RP = C + 2, NB = R / 4, KS = C;  // k-steps (4 positions each) per band
  static constexpr int BPI = CI == 4 ? 4 : 1;           // bands per iteration (one LDS buffer)
  static constexpr int XB_F = 6 * RP * PI, DB_F = 4 * C * PD, BUF_F = BPI * (XB_F + DB_F);
  static constexpr int QW = CI == 4 ? 1 : (CI / 16) / WPM;   // input channels per lane per tap
  static constexpr int NTW = CI == 4 ? 2 : 9 * QW;           // column tiles per wave
  static constexpr int NT_ALL = CI == 4 ? 2 : 9 * (CI / 16); // column tiles per row tile
  static constexpr int WSZ = MT * NT_ALL * 256 + CO;         // partial floats per chunk
  static constexpr int LDS = 2 * BUF_F * 4 + 64;
  static_assert(CI == 4 ? WPM == 4 : (CI / 16) % WPM == 0, "wave split");
  static_assert(kChunkBands % BPI == 0, "whole iterations per chunk");
  static_assert(CI != 4 || 8 * 2 * 256 <= BPI * DB_F, "the k groups' partial tiles fit the dY images");
};

// Input channel of column j of the wave's tile qq (CI >= 32, wave half h); for CI == 4 the
// column jj = 16 tile + j < 27 is the pair (tap jj / 3, ci jj % 3), 27 the bias.
template <int CI>
__host__ __device__ constexpr int col_ci(int j, int h, int qq) {
  return CI == 64 ? 8 * (j >> 1) + 2 * (j & 1) + 4 * h + qq : 8 * (j >> 2) + (j & 3) + 4 * h;
}

template <int CI, int CO, int R, int C>
__global__ __launch_bounds__(kThreads, 1) void conv_w_kernel(ConvWArgs a) {
  using G = ConvWGeom<CI, CO, R, C>;
  constexpr int PI = G::PI, PD = G::PD, MT = G::MT, RP = G::RP, NB = G::NB, QW = G::QW, NTW = G::NTW;
  constexpr int BPI = G::BPI, KS = G::KS;
  extern __shared__ f4 smem4[];
  float* smem = reinterpret_cast<float*>(smem4);
  int* slot = reinterpret_cast<int*>(smem + 2 * G::BUF_F);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = wid % MT, h = wid / MT;  // CI == 4: h is the k group
  const int j = lane & 15, g = lane >> 4;
  const int nbands = a.n * NB, nchunks = (nbands + kChunkBands - 1) / kChunkBands;
  const bool has_bias = CI == 4 ? false : h == 0;  // (CI == 4: the bias is column 27)

  // this lane's column offsets within a position (word units)
  int coff[CI == 4 ? 2 : QW];
  bool cval[2] = {true, true};
  float cfix[2] = {0.f, 0.f};  // CI == 4: the B value of a column that is not a (tap, ci) pair
  if constexpr (CI == 4) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int jj = 16 * t + j, tap = jj / 3, ci = jj % 3;
      cval[t] = jj < 27;
      cfix[t] = jj == 27 ? 1.0f : 0.f;
      coff[t] = cval[t] ? ((tap / 3) * RP + tap % 3) * PI + ci : 0;
    }
  } else {
#pragma unroll
    for (int qq = 0; qq < QW; ++qq) coff[qq] = col_ci<CI>(j, h, qq);
  }
  f4 acc[NTW];
  f4 accb = {0.f, 0.f, 0.f, 0.f};

  // iteration `it` of the WG's sequence reads buffer it & 1: BPI bands of chunk `ch` from `ib`
  auto issue = [&](int ch, int ib, int par) {
    float* b0 = smem + par * G::BUF_F;
#pragma unroll
    for (int bb = 0; bb < BPI; ++bb) {
      const int gb = ch * kChunkBands + ib + bb;
      if (gb >= nbands) break;
      load_band<CI, R, C>(a.x, b0 + bb * G::XB_F, gb, bb * 3, wid, lane);
      const int smp = gb / NB, y0 = (gb % NB) * 4;
      dma_range(a.dy + ((size_t)smp * R + y0) * C * PD, b0 + BPI * G::XB_F + bb * G::DB_F, G::DB_F * 4, bb * 3 + 5, wid,
                lane);
    }
  };
  if (tid == 0) {
    slot[0] = atomicAdd(a.queue, 1);
    slot[1] = atomicAdd(a.queue, 1);
  }
  // zero both buffers (the X images' border columns stay zero) before any DMA lands
  zero_range(smem, 2 * G::BUF_F * 4, wid, lane);
  __syncthreads();
  int chunk = slot[0], nchunk = slot[1];
  if (chunk < nchunks) issue(chunk, 0, 0);
  int it = 0;
  while (chunk < nchunks) {
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
    accb = f4{0.f, 0.f, 0.f, 0.f};
    int drawn = 0;  // the chunk after next (tid 0), stored to slot[2] once this chunk's k-steps are done
    for (int i = 0; i < kChunkBands; i += BPI, ++it) {
      const float* xi0 = smem + (it & 1) * G::BUF_F;
      const float* di0 = xi0 + BPI * G::XB_F;
      wait_dma();
      __syncthreads();
      // next iteration: this chunk's next bands, or the first of the next chunk (drawn ahead)
      if (i + BPI < kChunkBands) {
        issue(chunk, i + BPI, (it + 1) & 1);
      } else {
        // drawn before the DMA goes out (the compiler's wait for the atomic, vmcnt(0), would
        // otherwise also wait for the DMA), stored after the k-steps
        if (tid == 0) drawn = atomicAdd(a.queue, 1);
        if (nchunk < nchunks) issue(nchunk, 0, (it + 1) & 1);
      }
#pragma unroll
      for (int bb = 0; bb < BPI; ++bb) {
        if (chunk * kChunkBands + i + bb >= nbands) break;  // (uniform)
        const float* xi = xi0 + bb * G::XB_F;
        const float* di = di0 + bb * G::DB_F;
#pragma unroll
        for (int ks = (CI == 4 ? h : 0); ks < KS; ks += (CI == 4 ? 4 : 1)) {
          // positions 4 ks + g: one image row y (C % 4 == 0), column xx
          const int q = 4 * ks + g, y = (4 * ks) / C, xx = q - y * C;
          const float av = lds_f1(di, q * PD + 16 * m + j);
          const int xb = (y * RP + xx) * PI;
          if constexpr (CI == 4) {
#pragma unroll
            for (int t = 0; t < 2; ++t) acc[t] = mfma(av, cval[t] ? lds_f1(xi, xb + coff[t]) : cfix[t], acc[t]);
          } else {
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
              const int o = xb + ((tap / 3) * RP + tap % 3) * PI;
              if constexpr (QW == 2) {
                const f2 bv = lds_f2(xi, o + coff[0]);
                acc[tap * 2] = mfma(av, bv[0], acc[tap * 2]);
                acc[tap * 2 + 1] = mfma(av, bv[1], acc[tap * 2 + 1]);
              } else {
                acc[tap] = mfma(av, lds_f1(xi, o + coff[0]), acc[tap]);
              }
            }
          }
          // (behind a run-time `if`, so each k-step is its own basic block; compiled once per
          // wave role instead -- one straight block -- conv2's ran 1 % slower and conv3's spilled,
          // profiles/r06w_*)
          if (has_bias) accb = mfma(av, 1.0f, accb);
        }
      }
    }
    if (tid == 0) slot[2] = drawn;
    // this chunk's partial: tiles [m][tile][lane][4], then the bias [CO]
    float* p = a.partial + (size_t)chunk * G::WSZ;
    if constexpr (CI == 4) {
      // the k groups' 2 column tiles summed in k-group order through the dY images of the
      // buffer this iteration read (everyone is done with it after the barrier; the next DMA
      // into it is issued after the next iteration's first barrier)
      __syncthreads();
      float* scr = smem + ((it - 1) & 1) * G::BUF_F + BPI * G::XB_F;
      float* mine = scr + (m * 4 + h) * 2 * 256;
#pragma unroll
      for (int t = 0; t < 2; ++t) *reinterpret_cast<f4*>(mine + t * 256 + lane * 4) = acc[t];
      __syncthreads();
      if (h == 0) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          f4 v = lds_f4(scr, (m * 4 * 2 + t) * 256 + lane * 4);
#pragma unroll
          for (int k = 1; k < 4; ++k) v += lds_f4(scr, ((m * 4 + k) * 2 + t) * 256 + lane * 4);
          *reinterpret_cast<f4*>(p + ((size_t)m * 2 + t) * 256 + lane * 4) = v;
          if (t == 1 && j == 11) *reinterpret_cast<f4*>(p + MT * G::NT_ALL * 256 + 16 * m + 4 * g) = v;  // column 27
        }
      }
    } else {
      __syncthreads();  // slot[2] visible
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int qq = 0; qq < QW; ++qq)
          *reinterpret_cast<f4*>(p + (((size_t)m * 9 + tap) * (CI / 16) + QW * h + qq) * 256 + lane * 4) =
              acc[tap * QW + qq];
      if (has_bias && j == 0) *reinterpret_cast<f4*>(p + MT * G::NT_ALL * 256 + 16 * m + 4 * g) = accb;
    }
    chunk = nchunk;
    nchunk = slot[2];
  }
  queue_exit(a.queue);
}

// dW (torch layout [CO][CI_real][3][3]) and db [CO] = the chunk partials summed in a fixed
// order: workgroup = 64 consecutive partial elements; its 4 waves take the chunks k = 4 i + w,
// each into 8 accumulators by (i mod 8) (8 loads in flight), which are added in order, then the
// 4 waves' sums in order (deterministic; the association is fixed by nchunks alone).
template <int CI, int CO, int R, int C>
__global__ __launch_bounds__(256) void conv_w_reduce_kernel(const float* __restrict__ partial, int nchunks, int ci_real,
                                                            float* __restrict__ dw, float* __restrict__ db) {
  using G = ConvWGeom<CI, CO, R, C>;
  __shared__ float wsum[4][64];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int e = blockIdx.x * 64 + l;
  float acc8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (e < G::WSZ) {
    const float* src = partial + e;
    int i = 0;
    for (; 4 * (i + 7) + w < nchunks; i += 8)
#pragma unroll
      for (int u = 0; u < 8; ++u) acc8[u] += src[(size_t)(4 * (i + u) + w) * G::WSZ];
    for (; 4 * i + w < nchunks; ++i) acc8[i & 7] += src[(size_t)(4 * i + w) * G::WSZ];
  }
  wsum[w][l] = ((acc8[0] + acc8[1]) + (acc8[2] + acc8[3])) + ((acc8[4] + acc8[5]) + (acc8[6] + acc8[7]));
  __syncthreads();
  if (w != 0 || e >= G::WSZ) return;
  const float sum = ((wsum[0][l] + wsum[1][l]) + wsum[2][l]) + wsum[3][l];
  const int tiles = G::MT * G::NT_ALL * 256;
  if (e >= tiles) {
    db[e - tiles] = sum;
    return;
  }
  const int r = e & 3, lane = (e >> 2) & 63, tile = e >> 8, j = lane & 15, g = lane >> 4;
  if constexpr (CI == 4) {
    const int m = tile / 2, t = tile % 2, jj = 16 * t + j, tap = jj / 3, ci = jj % 3;
    if (jj < 27 && ci < ci_real) dw[((size_t)(16 * m + 4 * g + r) * ci_real + ci) * 9 + tap] = sum;
  } else {
    constexpr int NQ = CI / 16, QW = G::QW;
    const int m = tile / (9 * NQ), rest = tile % (9 * NQ), tap = rest / NQ, nq = rest % NQ;
    const int co = 16 * m + 4 * g + r, ci = col_ci<CI>(j, nq / QW, nq % QW);
    dw[((size_t)co * CI + ci) * 9 + tap] = sum;
  }
}

// Weights [CO][CI][3][3] (torch) -> conv_a_kernel fragments.  transpose = 0: the forward
// convolution (out = CO, in = CI); 1: its data gradient (out = CI, in = CO, taps flipped).
// Fragment [c][s][tap][cbw][lane][e] = W'[16c + (lane & 15)][tap][16 (s KBW + cbw) + 4 (lane >> 4) + e];
// for a 3-channel input (padded to 4) [c][tap][lane] = W'[16c + (lane & 15)][tap][lane >> 4].
__global__ __launch_bounds__(256) void conv_pack_kernel(const float* __restrict__ w, int co_t, int ci_t, int transpose,
                                                        int S, float* __restrict__ frag) {
  const int OUT = transpose ? ci_t : co_t, IN = transpose ? co_t : ci_t;
  const int in_pad = IN <= 4 ? 4 : IN;
  const int total = OUT * 9 * in_pad;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  int o, tap, k;
  if (in_pad == 4) {  // [c][tap][lane]
    const int lane = idx & 63, t = (idx >> 6) % 9, c = (idx >> 6) / 9;
    o = 16 * c + (lane & 15);
    tap = t;
    k = lane >> 4;
  } else {
    const int KBW = (IN / 16) / S;
    const int e = idx & 3, lane = (idx >> 2) & 63;
    int rest = idx >> 8;
    const int cbw = rest % KBW;
    rest /= KBW;
    tap = rest % 9;
    rest /= 9;
    const int s = rest % S, c = rest / S;
    o = 16 * c + (lane & 15);
    k = 16 * (s * KBW + cbw) + 4 * (lane >> 4) + e;
  }
  float v = 0.f;
  if (k < IN) {
    if (!transpose) v = w[((size_t)o * ci_t + k) * 9 + tap];
    else v = w[((size_t)k * ci_t + o) * 9 + (8 - tap)];
  }
  frag[idx] = v;
}

// obs [n][3][R][C] (any strides, in elements: the environment's NCHW observation or a
// channels-last copy) -> x4 [n][R][C][4], channel 3 zero.
__global__ __launch_bounds__(256) void obs_nhwc4_kernel(const float* __restrict__ obs, int64_t n_pos, int R, int C,
                                                         int64_t sn, int64_t sc, int64_t sh, int64_t sw,
                                                         float* __restrict__ x4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pos; i += (int64_t)gridDim.x * 256) {
    const int64_t smp = i / (R * C);
    const int p = (int)(i % (R * C)), y = p / C, x = p % C;
    const float* o = obs + smp * sn + y * sh + x * sw;
    reinterpret_cast<f4*>(x4)[i] = f4{o[0], o[sc], o[2 * sc], 0.f};
  }
}

// torch adaptive_avg_pool2d window [start, end) of output cell i (of 4) over n inputs
__device__ __forceinline__ int win_start(int i, int n) { return (i * n) / 4; }
__device__ __forceinline__ int win_end(int i, int n) { return ((i + 1) * n + 3) / 4; }

// feat [n][64 * 16] = adaptive_avg_pool2d(a3, (4, 4)) flattened channel-major; a3 [n][R][C][68].
// Thread = (sample, channel, cell): the window sum in row-major order / the window area.
__global__ __launch_bounds__(256) void pool_kernel(const float* __restrict__ a3, int n, int R, int C,
                                                   float* __restrict__ feat) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)n * 1024) return;
  const int co = e & 63, cell = (e >> 6) & 15;
  const int64_t smp = e >> 10;
  const int cy = cell >> 2, cx = cell & 3;
  const int y0 = win_start(cy, R), y1 = win_end(cy, R), x0 = win_start(cx, C), x1 = win_end(cx, C);
  const float* s = a3 + smp * R * C * 68 + co;
  float sum = 0.f;
  for (int y = y0; y < y1; ++y)
    for (int x = x0; x < x1; ++x) sum += s[(y * C + x) * 68];
  feat[smp * 1024 + co * 16 + cell] = sum / (float)((y1 - y0) * (x1 - x0));
}

// The same for R = C = 20 (windows of 5 x 5): the window's 25 loads unrolled, all in flight
// before the first add (the rolled loop above waits for each load before the next), summed in
// the same row-major order.
__global__ __launch_bounds__(256) void pool20_kernel(const float* __restrict__ a3, int n, float* __restrict__ feat) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)n * 1024) return;
  const int co = e & 63, cell = (e >> 6) & 15;
  const int64_t smp = e >> 10;
  const float* s = a3 + (smp * 400 + (cell >> 2) * 5 * 20 + (cell & 3) * 5) * 68 + co;
  float v[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) v[i] = s[((i / 5) * 20 + i % 5) * 68];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 25; ++i) sum += v[i];
  feat[smp * 1024 + co * 16 + cell] = sum / 25.f;
}

// d3 [n][R][C][68] = (a3 > 0) * (adaptive_avg_pool2d's input gradient of dfeat [n][1024]), the
// mask from conv3's forward bits m3 [n][R][C][16] (uint8 per 4 channels).  One workgroup per
// sample: the sample's 1,024 pooled gradients, each divided by its window's area, go to LDS
// as [cell][channel] (a channel quad = one ds_read_b128), then the workgroup writes the
// sample's positions, thread = (position, channel quad), each position's windows summed in
// (cy, cx) order (the order of torch's adaptive_avg_pool2d backward; one window per position
// when 4 divides R and C).
__global__ __launch_bounds__(256) void pool_bwd_mask_kernel(const float* __restrict__ dfeat, const uint8_t* __restrict__ m3,
                                                            int n, int R, int C, float* __restrict__ d3) {
  __shared__ f4 g[16 * 16];  // [cell][channel quad]
  extern __shared__ uint4 mk[];  // the sample's mask bits, one 16-byte row per position
  const int smp = blockIdx.x, tid = threadIdx.x;
  // the mask rows first, all loads in flight (one per position), so the store loop below
  // waits on no global load
  for (int p = tid; p < R * C; p += 256) mk[p] = reinterpret_cast<const uint4*>(m3)[(int64_t)smp * R * C + p];
  {
    const int cell = tid & 15, qd = tid >> 4;  // reads dfeat[(4 qd + r) * 16 + cell]
    const int cy = cell >> 2, cx = cell & 3;
    const float area = (float)((win_end(cy, R) - win_start(cy, R)) * (win_end(cx, C) - win_start(cx, C)));
    const float* df = dfeat + (int64_t)smp * 1024 + (4 * qd) * 16 + cell;
    f4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = df[r * 16] / area;
    g[cell * 16 + qd] = v;
  }
  __syncthreads();
  const int npos = R * C;
  const int64_t base = (int64_t)smp * npos;
  for (int it = tid; it < npos * 16; it += 256) {
    const int q = it & 15, p = it >> 4;
    const int y = p / C, x = p - (p / C) * C;
    f4 gsum = {0.f, 0.f, 0.f, 0.f};
    for (int cy = 0; cy < 4; ++cy) {
      if (y < win_start(cy, R) || y >= win_end(cy, R)) continue;
      for (int cx = 0; cx < 4; ++cx) {
        if (x < win_start(cx, C) || x >= win_end(cx, C)) continue;
        const f4 t = g[(cy * 4 + cx) * 16 + q];
#pragma unroll
        for (int r = 0; r < 4; ++r) gsum[r] += t[r];
      }
    }
    const uint32_t bits = (uint32_t)reinterpret_cast<const uint8_t*>(mk)[p * 16 + q];
    f4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (bits >> r) & 1u ? gsum[r] : 0.f;
    *reinterpret_cast<f4*>(d3 + (base + p) * 68 + 4 * q) = v;
    // the row's 4 pad words too, so every 128-B line of the rows is written whole (a line
    // left partly unwritten costs the memory system a read-modify-write)
    if (q == 15) *reinterpret_cast<f4*>(d3 + (base + p) * 68 + 64) = f4{0.f, 0.f, 0.f, 0.f};
  }
}

}  // namespace tc

// ---------------------------------------------------------------------------------------
// launchers

namespace {
template <class K>
hipError_t set_lds(K kern, int lds) {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}
}  // namespace

int tc_workgroups() {
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n_cu = 256;
  }
  return n_cu;
}

template <int CI, int CO, int S, int MODE>
static hipError_t launch_a(const tc::ConvAArgs& a, hipStream_t st) {
  using G = tc::ConvAGeom<CI, CO, S, MODE, 20, 20>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = set_lds(&tc::conv_a_kernel<CI, CO, S, MODE, 20, 20>, G::LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((tc::conv_a_kernel<CI, CO, S, MODE, 20, 20>), dim3(tc_workgroups()), dim3(tc::kThreads), G::LDS,
                     st, a);
  return hipGetLastError();
}

// layer: 1 = conv1 (3 -> 32), 2 = conv2 (32 -> 64), 3 = conv3 (64 -> 64); mode 0 forward, 1 data
// gradient (layers 2, 3: input = the gradient at the layer's output, 64 channels)
hipError_t launch_train_conv(int layer, int mode, const float* x, int n, int R, int C, const float* frag,
                             const float* bias, uint8_t* mask_bits, float* y, int* queue, hipStream_t st) {
  if (R != 20 || C != 20) return hipErrorInvalidValue;
  const tc::ConvAArgs a{x, frag, bias, mode == 1 ? mask_bits : nullptr, mode == 0 ? mask_bits : nullptr, y, queue, n};
  if (mode == 0) {
    if (layer == 1) return launch_a<4, 32, 1, 0>(a, st);
    if (layer == 2) return launch_a<32, 64, 1, 0>(a, st);
    if (layer == 3) return launch_a<64, 64, 1, 0>(a, st);
  } else {
    if (layer == 3) return launch_a<64, 64, 1, 1>(a, st);
    if (layer == 2) return launch_a<64, 32, 2, 1>(a, st);
  }
  return hipErrorInvalidValue;
}

int train_conv_frag_floats(int layer, int mode) {
  // forward: CO * 9 * max(CI, 4); gradient: CI * 9 * CO
  if (layer == 1) return mode == 0 ? 32 * 9 * 4 : -1;
  if (layer == 2) return 64 * 9 * 32;
  if (layer == 3) return 64 * 9 * 64;
  return -1;
}

hipError_t launch_train_conv_pack(int layer, int mode, const float* w, float* frag, hipStream_t st) {
  const int total = train_conv_frag_floats(layer, mode);
  if (total < 0) return hipErrorInvalidValue;
  const int co = layer == 1 ? 32 : 64, ci = layer == 1 ? 3 : (layer == 2 ? 32 : 64);
  const int S = (layer == 2 && mode == 1) ? 2 : 1;
  hipLaunchKernelGGL(tc::conv_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w, co, ci, mode, S, frag);
  return hipGetLastError();
}

template <int CI, int CO>
static hipError_t launch_w(const float* dy, const float* x, int n, float* partial, float* dw, float* db, int* queue,
                           int ci_real, hipStream_t st) {
  using G = tc::ConvWGeom<CI, CO, 20, 20>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = set_lds(&tc::conv_w_kernel<CI, CO, 20, 20>, G::LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const tc::ConvWArgs a{dy, x, partial, queue, n};
  hipLaunchKernelGGL((tc::conv_w_kernel<CI, CO, 20, 20>), dim3(tc_workgroups()), dim3(tc::kThreads), G::LDS, st, a);
  const int nchunks = (n * G::NB + tc::kChunkBands - 1) / tc::kChunkBands;
  hipLaunchKernelGGL((tc::conv_w_reduce_kernel<CI, CO, 20, 20>), dim3((G::WSZ + 63) / 64), dim3(256), 0, st, partial,
                     nchunks, ci_real, dw, db);
  return hipGetLastError();
}

int64_t train_conv_partial_floats(int layer, int n, int R, int C) {
  if (R != 20 || C != 20 || n < 0) return -1;
  const int64_t nchunks = ((int64_t)n * 5 + tc::kChunkBands - 1) / tc::kChunkBands;
  int wsz = 0;
  if (layer == 1) wsz = tc::ConvWGeom<4, 32, 20, 20>::WSZ;
  else if (layer == 2) wsz = tc::ConvWGeom<32, 64, 20, 20>::WSZ;
  else if (layer == 3) wsz = tc::ConvWGeom<64, 64, 20, 20>::WSZ;
  else return -1;
  return nchunks * wsz;
}

hipError_t launch_train_conv_wgrad(int layer, const float* dy, const float* x, int n, int R, int C, float* partial,
                                   float* dw, float* db, int* queue, hipStream_t st) {
  if (R != 20 || C != 20) return hipErrorInvalidValue;
  if (layer == 1) return launch_w<4, 32>(dy, x, n, partial, dw, db, queue, 3, st);
  if (layer == 2) return launch_w<32, 64>(dy, x, n, partial, dw, db, queue, 32, st);
  if (layer == 3) return launch_w<64, 64>(dy, x, n, partial, dw, db, queue, 64, st);
  return hipErrorInvalidValue;
}

hipError_t launch_obs_nhwc4(const float* obs, int n, int R, int C, const int64_t* strides, float* x4, hipStream_t st) {
  const int64_t n_pos = (int64_t)n * R * C;
  const int blocks = (int)std::min<int64_t>((n_pos + 255) / 256, 65536);
  hipLaunchKernelGGL(tc::obs_nhwc4_kernel, dim3(blocks), dim3(256), 0, st, obs, n_pos, R, C, strides[0], strides[1],
                     strides[2], strides[3], x4);
  return hipGetLastError();
}

hipError_t launch_train_pool(const float* a3, int n, int R, int C, float* feat, hipStream_t st) {
  const int64_t total = (int64_t)n * 1024;
  if (R == 20 && C == 20) {
    hipLaunchKernelGGL(tc::pool20_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a3, n, feat);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(tc::pool_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a3, n, R, C, feat);
  return hipGetLastError();
}

hipError_t launch_train_pool_bwd(const float* dfeat, const uint8_t* m3, int n, int R, int C, float* d3, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  // the sample's mask rows in LDS: R * C * 16 bytes (64 x 64 at most)
  if (R * C * 16 > 64 * 1024 || (reinterpret_cast<uintptr_t>(m3) & 15)) return hipErrorInvalidValue;
  if (R * C * 16 > 48 * 1024) {
    const hipError_t e = set_lds(&tc::pool_bwd_mask_kernel, R * C * 16);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(tc::pool_bwd_mask_kernel, dim3((unsigned)n), dim3(256), (size_t)R * C * 16, st, dfeat, m3, n, R, C,
                     d3);
  return hipGetLastError();
}

}  // namespace heist
