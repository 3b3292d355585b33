// heist_policy.hip -- fused batched SolverNetwork conv stack on CDNA4 bf16 MFMA.
//
// Replaces the backbone of SolverNetwork.forward (heist_architect/networks.py:93-100):
//   relu(conv1 3->32) -> relu(conv2 32->64) -> relu(conv3 64->64) -> AdaptiveAvgPool(4,4)
//   -> flatten [N, 64*16]
// for a batch of [N,3,R,C] float32 observations, the hot op of every rollout step
// (agents/solver.py:75-99 select_action, batched).  The MLP tail (fc_spatial, LSTM,
// heads) stays on PyTorch-ROCm GEMMs.
//
// Design (one 256-thread workgroup per CU, persistent over envs):
//   * the conv weights stay on chip for the whole kernel as ready-made MFMA fragments
//     (packed once per weight update by heist_solver_pack): conv1 (12) and conv3 (144)
//     in VGPRs, conv2 in LDS (36 KB, read once per k-step and reused over the wave's
//     position tiles), so the loop touches HBM only for the observation (4.8 KB/env) and
//     the pooled features (4 KB/env);
//   * one env at a time sits in LDS as zero-padded NHWC bf16 planes: input [P][4],
//     act1 [P][32+8], act2 [P][64+8] (P = (R+2)(C+2)); the +8 channel pad and a row pitch
//     chosen modulo the 256-byte bank width (ConvGeom::PB1/PB2) make the 16-byte fragment
//     reads of any 16 consecutive output positions bank-conflict free;
//   * each conv is an implicit GEMM on v_mfma_f32_32x32x16_bf16 (fp32 accumulate) whose
//     A/B fragments are single 16-byte LDS reads at compile-time tap offsets;
//     conv1/conv2 compute D[channel][position] so the epilogue writes 4 channels of a
//     position per 8-byte store; conv3 computes D[position][channel] so that the 4x4
//     average pool is one more MFMA, Y[cell][ch] += P[cell][pos] . relu(D)[pos][ch],
//     with the accumulator fed back as the B operand (no LDS round trip, no atomics);
//   * the next env's observation is loaded into registers while conv2/conv3 run.
// Waves: w = 2*mh + nh; conv1 splits position tiles 4 ways, conv2/conv3 split output
// channels by nh (32 each) and position tiles by mh.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

// LDS reads in flight in conv3's A-fragment ring (build-time A/B knob)
#ifndef HEIST_CONV3_PRE
#define HEIST_CONV3_PRE 7
#endif
// act1 reads in flight in conv2's ring (build-time A/B knob)
#ifndef HEIST_CONV2_PRE
#define HEIST_CONV2_PRE 6
#endif

namespace heist {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Packed blob (16-byte units): W1 [3][64], W2 [2][18][64], W3 [2][36][64] MFMA fragments,
// then float biases b1[32], b2[64], b3[64].
constexpr int kW1Steps = 3, kW2Steps = 18, kW3Steps = 36;
constexpr int kOffW1 = 0;
constexpr int kOffW2 = kOffW1 + kW1Steps * 64;
constexpr int kOffW3 = kOffW2 + 2 * kW2Steps * 64;
constexpr int kOffBias = kOffW3 + 2 * kW3Steps * 64;  // in uint4 units
constexpr int kPackedBytes = kOffBias * 16 + (32 + 64 + 64) * 4;

__host__ __device__ constexpr int align16c(int x) { return (x + 15) & ~15; }

template <int R, int C>
struct ConvGeom {
  static constexpr int PC = C + 2, PR = R + 2, NP = PR * PC, RC = R * C, MT = (RC + 31) / 32;
  static constexpr int S0 = 8, S1 = 80, S2 = 144;  // bytes per padded position
  // Row pitch of act1 / act2 in bytes: PB = C*S + 256 j (the smallest such >= PC*S), so
  // stepping from the last position of a row to the first of the next moves the LDS bank
  // group exactly as a step within a row does; 16 consecutive output positions then hit
  // 16 distinct 16-byte bank groups in every ds_read_b128, row breaks included.
  static constexpr int PB1 = C * S1 + 256 * ((2 * S1 + 255) / 256);
  static constexpr int PB2 = C * S2 + 256 * ((2 * S2 + 255) / 256);
  static constexpr int IN = 0;
  static constexpr int A1 = align16c(IN + NP * S0);
  static constexpr int A2 = align16c(A1 + PR * PB1);
  static constexpr int ZERO_END = align16c(A2 + PR * PB2);  // zeroed once (padding borders)
  static constexpr int POOL = ZERO_END;                    // [64][16] f32
  static constexpr int BIAS = POOL + 64 * 16 * 4;          // b1[32] b2[64] b3[64]
  static constexpr int INVA = BIAS + 160 * 4;              // [16] f32 1/area
  static constexpr int NT2 = (MT + 1) / 2;                 // position tiles per wave (conv2/conv3)
  static constexpr int W2 = align16c(INVA + 16 * 4);       // conv2 fragments [2][18][64] x 16 B
  static constexpr int SINK = W2 + 2 * 18 * 64 * 16;       // [64] x 8 B: stores of positions >= RC
  static constexpr int FLAG = SINK + 64 * 8;               // [2] int: conv3 split-tile hand-off (env index)
  static constexpr int LDS = FLAG + 16;
  // conv3's last position tile MT - 1 (mh = 0's) split by k-steps between the two waves of a
  // channel half when MT is odd (the mh = 1 wave's last slot would be pure padding) and the
  // tile holds <= 16 positions (its partial sums: 8 registers per lane)
  static constexpr bool SPLIT3 = (MT & 1) && RC - 32 * (MT - 1) <= 16 && MT >= 5;
  static constexpr int QI = (RC + 255) / 256;              // obs cells per thread
  static_assert(LDS <= 160 * 1024, "one env's planes + conv2 fragments must fit the CU's 160 KiB LDS");
};

// torch adaptive_avg_pool2d window of output index i over n inputs into 4.
__host__ __device__ constexpr int pool_lo(int i, int n) { return (i * n) / 4; }
__host__ __device__ constexpr int pool_hi(int i, int n) { return ((i + 1) * n + 3) / 4; }

__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// Pin a weight fragment in the accumulator register file: MFMA reads A/B operands from
// AGPRs as well (gfx90a+), and with the 144 conv3 + 12 conv1 weight VGPRs moved there the
// VGPR file keeps room for deep LDS read rings.  The empty asm emits nothing; "+a" makes
// the allocator keep the value in an AGPR at every use.
__device__ __forceinline__ bf16x8 in_agpr(bf16x8& w) {
  asm("" : "+a"(w));
  return w;
}

// Byte offset of output position m's padded cell (row pitch PB, S bytes per position).
template <int R, int C, int S, int PB>
__device__ __forceinline__ int pos_off(int m) {
  using G = ConvGeom<R, C>;
  const int mc = m < G::RC ? m : G::RC - 1;
  const int oy = mc / C;
  return (oy + 1) * PB + (mc - oy * C + 1) * S;
}

template <int R, int C>
__device__ __forceinline__ int padded_pos(int m) {  // output position m -> padded index
  using G = ConvGeom<R, C>;
  const int mc = m < G::RC ? m : G::RC - 1;
  const int oy = mc / C;
  return (oy + 1) * G::PC + (mc - oy * C) + 1;
}

// Scheduling pipelines: one MFMA then DS_READS LDS reads, NQ times, after an initial group
// of PRE reads -- keeps the read rings PRE deep (the scheduler otherwise folds them to one
// or two reads in flight).  W = 1 adds the next weight fragment's read at the last tile of
// every k-step (conv2's k-outer stream over NT tiles).
template <int NT, int W, int... Qs>
__device__ __forceinline__ void sched_ring(std::integer_sequence<int, Qs...>) {
  ((__builtin_amdgcn_sched_group_barrier(0x008, 1, 0),
    __builtin_amdgcn_sched_group_barrier(0x100, (W && Qs % NT == NT - 1) ? 2 : 1, 0)),
   ...);
}

// One k-outer pass of conv2 over the wave's position tiles [T0, T1) (tile i = position
// tile mh + 2 i): one LDS weight fragment per k-step feeds every tile of the pass, the
// (k-step, tile) act1 reads run through a ring of kPre2 reads in flight, and the epilogue
// of the previous pass's tiles [P0, P1) (bias, ReLU, bf16, 8-byte stores into act2) is
// spread over this pass's MFMA gaps.  Tiles past MT compute on clamped addresses and store
// to the sink.
template <int R, int C, int T0, int T1, int P0, int P1, int NA, int NP>
__device__ __forceinline__ void conv2_pass(unsigned char* smem, const bf16x8* wl, const float4 (&b2v)[4], int mh,
                                           int nh, int lr, int h, int l, f32x16 (&cur)[NA],
                                           const f32x16 (&prv)[NP]) {
  using G = ConvGeom<R, C>;
  constexpr int NTP = T1 - T0, NQ = kW2Steps * NTP, kPre2 = HEIST_CONV2_PRE;
  constexpr int NPIECE = (P1 - P0) * 16;
  constexpr int PER_Q = NQ > 0 ? (NPIECE + NQ - 1) / (NQ > 0 ? NQ : 1) : NPIECE;
  bf16x4 o;
  auto piece = [&](int k) {  // value k of the previous pass's epilogue
    const int ti = k >> 4, kk = k & 15, g = kk >> 2, jj = kk & 3;
    const float bv = jj == 0 ? b2v[g].x : (jj == 1 ? b2v[g].y : (jj == 2 ? b2v[g].z : b2v[g].w));
    o[jj] = (__bf16)relu(prv[ti][kk] + bv);
    if (jj == 3) {
      const int m = 32 * (mh + 2 * (P0 + ti)) + lr;
      const int off = m < G::RC ? G::A2 + pos_off<R, C, G::S2, G::PB2>(m) + (32 * nh + 8 * g + 4 * h) * 2
                                : G::SINK + 8 * l;
      *reinterpret_cast<bf16x4*>(smem + off) = o;
    }
  };
  if constexpr (NQ > 0) {
    const unsigned char* base[NTP];
#pragma unroll
    for (int i = 0; i < NTP; ++i) {
      base[i] = smem + G::A1 + pos_off<R, C, G::S1, G::PB1>(32 * (mh + 2 * (T0 + i)) + lr) - G::PB1 - G::S1 + 16 * h;
      cur[i] = f32x16{};
    }
    auto rd = [&](int q) {
      const int s = q / NTP, tap = s >> 1;
      return *reinterpret_cast<const bf16x8*>(base[q % NTP] + (tap / 3) * G::PB1 + (tap % 3) * G::S1 + (s & 1) * 32);
    };
    bf16x8 ring[kPre2];
#pragma unroll
    for (int q = 0; q < kPre2; ++q) ring[q] = rd(q < NQ ? q : NQ - 1);
    // weight fragments two k-steps ahead (a 3-slot ring); read one k-step ahead, their LDS
    // latency was exposed at every k-step boundary (only NTP MFMAs after the read)
    bf16x8 wb[3];
    wb[0] = wl[0];
    wb[1] = wl[64];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int s = q / NTP, i = q % NTP;
      if (i == 0 && s + 2 < kW2Steps) wb[(s + 2) % 3] = wl[(s + 2) * 64];
      const bf16x8 f = ring[q % kPre2];
      if (q + kPre2 < NQ) ring[q % kPre2] = rd(q + kPre2);
      cur[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wb[s % 3], f, cur[i], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < PER_Q; ++r)
        if (q * PER_Q + r < NPIECE) piece(q * PER_Q + r);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, kPre2 + 2, 0);
    sched_ring<NTP, 1>(std::make_integer_sequence<int, NQ>{});
  } else {
#pragma unroll
    for (int k = 0; k < NPIECE; ++k) piece(k);
  }
}

template <class G>  // G: ConvGeom or BandGeom
__device__ __forceinline__ void load_obs(const float* __restrict__ obs, int e, float (&v)[G::QI][3]) {
  const float* o = obs + (size_t)e * 3 * G::RC;
#pragma unroll
  for (int i = 0; i < G::QI; ++i) {
    const int q = threadIdx.x + 256 * i;
    if (q < G::RC) {
      v[i][0] = o[q];
      v[i][1] = o[G::RC + q];
      v[i][2] = o[2 * G::RC + q];
    }
  }
}

template <class G>
__device__ __forceinline__ void stage_obs(unsigned char* smem, const float (&v)[G::QI][3]) {
  constexpr int C = G::PC - 2;
#pragma unroll
  for (int i = 0; i < G::QI; ++i) {
    const int q = threadIdx.x + 256 * i;
    if (q < G::RC) {
      const int oy = q / C;
      const int p = (oy + 1) * G::PC + (q - oy * C) + 1;
      bf16x4 b;
      b[0] = (__bf16)v[i][0];
      b[1] = (__bf16)v[i][1];
      b[2] = (__bf16)v[i][2];
      b[3] = (__bf16)0.f;
      *reinterpret_cast<bf16x4*>(smem + G::IN + p * G::S0) = b;
    }
  }
}

// Epilogue of a D[channel][position] tile: lane holds position m = 32t + (l & 31) and, in
// register 4g + i, channel n0 + i with n0 = 8g + 4h; relu(acc + bias) -> 4 bf16 -> 8 bytes.
// bias: the lane's 4 float4 of channels nbase + 8g + 4h (g = 0..3), held in registers (an
// LDS bias read here would be a full lgkmcnt(0) drain per group, serialised per tile).
template <int R, int C, int S, int PB>
__device__ __forceinline__ void store_chan_major(unsigned char* dst, const float4 (&bias)[4], int nbase,
                                                 const f32x16& acc, int m, int h) {
  using G = ConvGeom<R, C>;
  if (m >= G::RC) return;
  const int po = pos_off<R, C, S, PB>(m);
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int n0 = nbase + 8 * g + 4 * h;
    const float4 b = bias[g];
    bf16x4 o;
    o[0] = (__bf16)relu(acc[4 * g + 0] + b.x);
    o[1] = (__bf16)relu(acc[4 * g + 1] + b.y);
    o[2] = (__bf16)relu(acc[4 * g + 2] + b.z);
    o[3] = (__bf16)relu(acc[4 * g + 3] + b.w);
    *reinterpret_cast<bf16x4*>(dst + po + n0 * 2) = o;
  }
}

// In-kernel phase stamps (instrumentation, heist_solver_stamps): lane 0 of every wave
// records s_memtime at kStamps points of its workgroup's second env.
constexpr int kStamps = 10;
#define HEIST_STAMP(k)                                                            \
  do {                                                                            \
    if (stamps && e == (int)blockIdx.x + (int)gridDim.x && l == 0)                \
      stamps[((size_t)blockIdx.x * 4 + w) * kStamps + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// The conv2 fragments global -> LDS (2 x 18 x 64 uint4 = 9 per thread): all 9 loads in
// flight before the first store.  As a rolled loop every store waited for its load
// (vmcnt(0)): nine serial L2 round trips in every launch's prologue.
__device__ __forceinline__ void copy_w2(unsigned char* dst, const uint4* __restrict__ packed, int tid) {
  constexpr int kPer = 2 * kW2Steps * 64 / 256;
  static_assert(kPer * 256 == 2 * kW2Steps * 64, "conv2 fragments split evenly over 256 threads");
  uint4 t[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) t[k] = packed[kOffW2 + tid + 256 * k];
#pragma unroll
  for (int k = 0; k < kPer; ++k) reinterpret_cast<uint4*>(dst)[tid + 256 * k] = t[k];
}

template <int R, int C>
__global__ __launch_bounds__(256, 1) void solver_conv_kernel(const float* __restrict__ obs, int n,
                                                             const uint4* __restrict__ packed,
                                                             float* __restrict__ feat,
                                                             unsigned long long* __restrict__ stamps) {
  using G = ConvGeom<R, C>;
  constexpr int PC = G::PC;
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63, h = l >> 5, lr = l & 31;
  const int nh = w & 1, mh = w >> 1;

  // the first env's observation in flight under the weight loads
  float pre[G::QI][3];
  int e = blockIdx.x;
  if (e < n) load_obs<G>(obs, e, pre);

  // ---- weights -> registers (MFMA fragments), tables -> LDS
  bf16x8 w1[kW1Steps], w3[kW3Steps];
#pragma unroll
  for (int s = 0; s < kW1Steps; ++s) w1[s] = __builtin_bit_cast(bf16x8, packed[kOffW1 + s * 64 + l]);
#pragma unroll
  for (int s = 0; s < kW3Steps; ++s) {
    w3[s] = __builtin_bit_cast(bf16x8, packed[kOffW3 + (nh * kW3Steps + s) * 64 + l]);
    in_agpr(w3[s]);
  }
  copy_w2(smem + G::W2, packed, tid);  // conv2 fragments: LDS, read once per k-step
  const float* gbias = reinterpret_cast<const float*>(packed + kOffBias);
  float* bias = reinterpret_cast<float*>(smem + G::BIAS);
  const float b3v = gbias[96 + 32 * nh + lr];
  if (tid < 160) bias[tid] = gbias[tid];
  if (tid < 2) reinterpret_cast<int*>(smem + G::FLAG)[tid] = -1;
  for (int i = tid; i < G::ZERO_END / 16; i += 256) reinterpret_cast<uint4*>(smem)[i] = make_uint4(0u, 0u, 0u, 0u);
  if (tid < 16) {
    const int ci = tid >> 2, cj = tid & 3;
    const int area = (pool_hi(ci, R) - pool_lo(ci, R)) * (pool_hi(cj, C) - pool_lo(cj, C));
    reinterpret_cast<float*>(smem + G::INVA)[tid] = 1.0f / (float)area;
  }
  // conv1 bias and the pool membership of the lane's P fragments in registers for the whole
  // kernel: an LDS read of either inside the MFMA streams costs a full lgkmcnt(0) drain of
  // the read ring (12 per env in conv3, 16 in conv1's epilogue).  Byte 2 i + s of pbits =
  // P fragment s of the wave's tile i (mh + 2 i): bit j set iff row (cell) lr of the
  // fragment pools position 32 tp + 16 s + 8 (j >> 2) + 4 h + (j & 3).
  float4 b1v[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) b1v[g] = *reinterpret_cast<const float4*>(gbias + 8 * g + 4 * h);
  uint32_t pbits[(2 * G::NT2 + 3) / 4] = {};
  if (lr < 16) {
    const int ci = lr >> 2, cj = lr & 3;
    for (int i = 0; i < G::NT2; ++i) {
      for (int s = 0; s < 2; ++s) {
        unsigned bits = 0;
        for (int j = 0; j < 8; ++j) {
          const int m = 32 * (mh + 2 * i) + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
          if (m < G::RC) {
            const int oy = m / C, ox = m - (m / C) * C;
            if (oy >= pool_lo(ci, R) && oy < pool_hi(ci, R) && ox >= pool_lo(cj, C) && ox < pool_hi(cj, C))
              bits |= 1u << j;
          }
        }
        const int b = 2 * i + s;
#pragma unroll
        for (int d = 0; d < (2 * G::NT2 + 3) / 4; ++d)
          if (d == (b >> 2)) pbits[d] |= bits << (8 * (b & 3));
      }
    }
  }

  // conv1 per-lane tap offsets: k-step s covers taps 4s + 2h, 4s + 2h + 1 (taps >= 9 have
  // zero weights; they read the centre tap)
  int off1a[kW1Steps], off1b[kW1Steps];
#pragma unroll
  for (int s = 0; s < kW1Steps; ++s) {
    int ta = 4 * s + 2 * h, tb = ta + 1;
    ta = ta < 9 ? ta : 4;
    tb = tb < 9 ? tb : 4;
    off1a[s] = ((ta / 3) * PC + (ta % 3)) * G::S0;
    off1b[s] = ((tb / 3) * PC + (tb % 3)) * G::S0;
  }

  __builtin_amdgcn_s_waitcnt(0);  // weights landed: no conservative vmcnt waits inside the loop
  __syncthreads();

  // conv1: D[32 ch][pos] = W1 . im2col(in); wave w owns position tiles w + 4 i (a wave with
  // fewer tiles repeats its last one, result not stored).  Inside the loop it runs for the
  // NEXT env, interleaved with this env's conv3 (see there); the first env's runs here.
  constexpr int NT1 = (G::MT + 3) / 4;
  auto conv1_reads = [&](int i, bf16x8 (&f)[kW1Steps]) {
    const unsigned char* base = smem + G::IN + (padded_pos<R, C>(32 * (w + 4 * i) + lr) - PC - 1) * G::S0;
#pragma unroll
    for (int s = 0; s < kW1Steps; ++s) {
      const uint2 a = *reinterpret_cast<const uint2*>(base + off1a[s]);
      const uint2 b = *reinterpret_cast<const uint2*>(base + off1b[s]);
      f[s] = __builtin_bit_cast(bf16x8, make_uint4(a.x, a.y, b.x, b.y));
    }
  };
  if (e < n) {
    stage_obs<G>(smem, pre);
    __syncthreads();
    bf16x8 f1[NT1][kW1Steps];
#pragma unroll
    for (int i = 0; i < NT1; ++i) conv1_reads(i, f1[i]);
#pragma unroll
    for (int i = 0; i < NT1; ++i) {
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < kW1Steps; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1[s], f1[i][s], acc, 0, 0, 0);
      store_chan_major<R, C, G::S1, G::PB1>(smem + G::A1, b1v, 0, acc, 32 * (w + 4 * i) + lr, h);
    }
  }
  __syncthreads();  // act1 of the first env ready

  for (; e < n; e += gridDim.x) {
    HEIST_STAMP(0);
    const int en = e + gridDim.x;
    const bool has_next = en < n;  // workgroup-uniform
    if (has_next) load_obs<G>(obs, en, pre);  // next env's observation in flight during conv2
    HEIST_STAMP(1);
    HEIST_STAMP(2);
    HEIST_STAMP(3);

    // ---- conv2: D[32 ch of nh][pos] = W2 . im2col(act1) in three k-outer passes over the
    // wave's position tiles; each pass hides the previous pass's epilogue under its MFMAs
    // (conv2_pass), so only the last pass's epilogue is exposed.
    {
      constexpr int NT2 = G::NT2;
#ifdef HEIST_CONV2_SASB  // build-time A/B of the pass boundaries, e.g. -DHEIST_CONV2_SASB=3,6
      constexpr int SASB[2] = {HEIST_CONV2_SASB};  // 20 x 20 (NT2 = 7) only
      constexpr int SA = NT2 == 7 ? SASB[0] : (NT2 * 3 + 6) / 7, SB = NT2 == 7 ? SASB[1] : SA + (NT2 - SA + 1) / 2;
#else
      constexpr int SA = (NT2 * 3 + 6) / 7, SB = SA + (NT2 - SA + 1) / 2;
#endif
      constexpr int NA = SA, NB = SB - SA > 0 ? SB - SA : 1, NC = NT2 - SB > 0 ? NT2 - SB : 1;
      const bf16x8* wl = reinterpret_cast<const bf16x8*>(smem + G::W2) + nh * kW2Steps * 64 + l;
      float4 b2v[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) b2v[g] = *reinterpret_cast<const float4*>(bias + 32 + 32 * nh + 8 * g + 4 * h);
      f32x16 accA[NA], accB[NB], accC[NC];
      conv2_pass<R, C, 0, SA, 0, 0, NA, NA>(smem, wl, b2v, mh, nh, lr, h, l, accA, accA);
      conv2_pass<R, C, SA, SB, 0, SA, NB, NA>(smem, wl, b2v, mh, nh, lr, h, l, accB, accA);
      conv2_pass<R, C, SB, NT2, SA, SB, NC, NB>(smem, wl, b2v, mh, nh, lr, h, l, accC, accB);
      HEIST_STAMP(4);
      conv2_pass<R, C, NT2, NT2, SB, NT2, NC, NC>(smem, wl, b2v, mh, nh, lr, h, l, accC, accC);  // last epilogue
    }
    HEIST_STAMP(5);
    if (has_next) stage_obs<G>(smem, pre);  // in0 is free: this env's conv1 ran an iteration ago
    __syncthreads();  // B3: act2 of env e and the input plane of env en ready; act1 reads done
    HEIST_STAMP(6);

    // ---- conv3: D[pos][32 ch of nh] = im2col(act2) . W3, then Y[cell][ch] += P . relu(D).
    // The wave's (tile, k-step) sequence is one unrolled stream: A fragments run through a
    // ring of kPre LDS reads in flight across tile boundaries, and a tile's pooling (VALU +
    // 2 MFMAs) interleaves with the next tile's chain.  With G::SPLIT3 (20 x 20: 12.5 tiles)
    // the half-empty last tile MT - 1 is split by k-steps: mh = 0 runs its k-steps [0, 18)
    // last, mh = 1 its k-steps [18, 36) first (in place of its all-padding slot MT) and hands
    // the partial sums over through LDS, so both waves run 6.5 tiles instead of 7.  Without
    // it, tiles past MT (the shorter wave's last slot) have all-zero pool membership.
    f32x16 Y = {};
    {
      constexpr int NT2 = G::NT2, kPre = HEIST_CONV3_PRE;
      constexpr bool SP = G::SPLIT3;
      constexpr int KS = kW3Steps / 2;
      // software pipeline: tile i's pooling epilogue (ReLU + bias, bf16 packing, the two
      // pooling MFMAs) is spread over the first k-steps of tile i + 1's MFMA chain, one
      // element per MFMA gap, so it issues under the matrix core instead of stalling it
      f32x16 prev = {};
      bf16x8 x[2], pf[2];
      auto pool_piece = [&](int ti, int s) {  // piece s of the wave's tile ti's epilogue (prev holds its sums)
        if (s < 16) x[s >> 3][s & 7] = (__bf16)relu(prev[s] + b3v);
        if (s == 0 || s == 1) {
          const unsigned bits = (pbits[(2 * ti + s) >> 2] >> (8 * ((2 * ti + s) & 3))) & 0xffu;
#pragma unroll
          for (int j = 0; j < 8; ++j) pf[s][j] = ((bits >> j) & 1u) ? (__bf16)1.0f : (__bf16)0.0f;
        }
        if (s == 16) Y = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf[0], x[0], Y, 0, 0, 0);
        if (s == 17) Y = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf[1], x[1], Y, 0, 0, 0);
      };
      // the split tile's partial sums (rows 0..15 = registers 0..7, 32 B per lane) pass
      // through the act1 cell of position 32 nh + lr: a cell of the mh = 0 reader's own conv1
      // tile, so nothing else writes it (act1's conv2 reads ended at B3) before the reader's
      // next-env conv1 below.  FLAG[nh] = e marks it complete: a wave's LDS operations
      // execute in order, so the volatile stores (kept in program order) suffice.
      // (LDS-typed pointers: a volatile access through a generic one stays a flat access)
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      typedef __attribute__((address_space(3))) f32x2 lds_f32x2;
      typedef __attribute__((address_space(3))) int lds_int;
      lds_f32x2* stash = (lds_f32x2*)(smem + G::A1 + pos_off<R, C, G::S1, G::PB1>(32 * nh + lr) + 8 * h);
      lds_int* flag = (lds_int*)(smem + G::FLAG) + nh;
      auto stream = [&](auto mhc) {
        constexpr int MH = decltype(mhc)::value;
        constexpr bool ST = SP && MH == 1;  // segment 0: the split tile's k-steps [KS, 36), stashed
        constexpr int L0 = ST ? kW3Steps - KS : kW3Steps;
        constexpr int NQ = SP ? (NT2 - 1) * kW3Steps + (MH ? kW3Steps - KS : KS) : NT2 * kW3Steps;
        const unsigned char* base[NT2];  // segment g's tile
#pragma unroll
        for (int g = 0; g < NT2; ++g) {
          const int t = MH == 0 ? 2 * g : (ST ? (g == 0 ? G::MT - 1 : 2 * g - 1) : 2 * g + 1);
          base[g] = smem + G::A2 + pos_off<R, C, G::S2, G::PB2>(32 * t + lr) - G::PB2 - G::S2 + 16 * h;
        }
        auto rd = [&](int q) {
          const int g = q < L0 ? 0 : 1 + (q - L0) / kW3Steps;
          const int s = q < L0 ? (ST ? KS : 0) + q : (q - L0) % kW3Steps, tap = s >> 2;
          return *reinterpret_cast<const bf16x8*>(base[g] + (tap / 3) * G::PB2 + (tap % 3) * G::S2 + (s & 3) * 32);
        };
        auto epi = [&](int g, int j) {  // piece j of segment g's epilogue (prev holds its sums)
          if (ST && g == 0) {
            if (j < 4) *(volatile lds_f32x2*)(stash + 2 * j) = f32x2{prev[2 * j], prev[2 * j + 1]};
            if (j == 4) *(volatile lds_int*)flag = e;
          } else {
            pool_piece(ST ? g - 1 : g, j);
          }
        };
        bf16x8 ring[kPre];
#pragma unroll
        for (int q = 0; q < kPre; ++q) ring[q] = rd(q);
#pragma unroll
        for (int g = 0; g < NT2; ++g) {
          const int k0 = ST && g == 0 ? KS : 0;
          const int k1 = SP && MH == 0 && g == NT2 - 1 ? KS : kW3Steps;
          const int q0 = g == 0 ? 0 : L0 + (g - 1) * kW3Steps;
          f32x16 acc = {};
#pragma unroll
          for (int s = k0; s < k1; ++s) {
            const int q = q0 + s - k0;
            const bf16x8 f = ring[q % kPre];
            if (q + kPre < NQ) ring[q % kPre] = rd(q + kPre);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f, in_agpr(w3[s]), acc, 0, 0, 0);
            if (g > 0 && s - k0 < 18) epi(g - 1, s - k0);
          }
          prev = acc;
        }
        __builtin_amdgcn_sched_group_barrier(0x100, kPre, 0);
        sched_ring<kW3Steps, 0>(std::make_integer_sequence<int, NQ>{});
        if constexpr (SP && MH == 0) {  // the partner's k-steps of the split tile
          while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != e) __builtin_amdgcn_s_sleep(1);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x2 v = stash[2 * j];
            prev[2 * j] += v.x;
            prev[2 * j + 1] += v.y;
          }
        }
#pragma unroll
        for (int s = 0; s < 18; ++s) epi(NT2 - 1, s);  // the last segment's epilogue
      };
      if (mh == 0)
        stream(std::integral_constant<int, 0>{});
      else
        stream(std::integral_constant<int, 1>{});
      // conv1 of the next env (its input plane was staged before B3): all reads first,
      // then tile by tile (also after the last env: harmless)
      {
        bf16x8 g1[NT1][kW1Steps];
#pragma unroll
        for (int j = 0; j < NT1; ++j) conv1_reads(j, g1[j]);
#pragma unroll
        for (int j = 0; j < NT1; ++j) {
          f32x16 a1 = {};
#pragma unroll
          for (int k = 0; k < kW1Steps; ++k) a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1[k], g1[j][k], a1, 0, 0, 0);
          store_chan_major<R, C, G::S1, G::PB1>(smem + G::A1, b1v, 0, a1, 32 * (w + 4 * j) + lr, h);
        }
      }
    }
    HEIST_STAMP(7);
    // Y: lane = channel 32nh + lr, register r < 8 = cell (r & 3) + 8 (r >> 2) + 4h
    float* pool = reinterpret_cast<float*>(smem + G::POOL) + (32 * nh + lr) * 16 + 4 * h;
    if (mh == 1) {
      *reinterpret_cast<float4*>(pool) = make_float4(Y[0], Y[1], Y[2], Y[3]);
      *reinterpret_cast<float4*>(pool + 8) = make_float4(Y[4], Y[5], Y[6], Y[7]);
    }
    __syncthreads();  // B4: partner half of the pool sums in LDS; act1 of env en written
    HEIST_STAMP(8);
    if (mh == 0) {
      const float4 p0 = *reinterpret_cast<const float4*>(pool);
      const float4 p1 = *reinterpret_cast<const float4*>(pool + 8);
      const float* inva = reinterpret_cast<const float*>(smem + G::INVA) + 4 * h;
      const float4 i0 = *reinterpret_cast<const float4*>(inva);
      const float4 i1 = *reinterpret_cast<const float4*>(inva + 8);
      float* out = feat + (size_t)e * 1024 + (32 * nh + lr) * 16 + 4 * h;
      *reinterpret_cast<float4*>(out) =
          make_float4((Y[0] + p0.x) * i0.x, (Y[1] + p0.y) * i0.y, (Y[2] + p0.z) * i0.z, (Y[3] + p0.w) * i0.w);
      *reinterpret_cast<float4*>(out + 8) =
          make_float4((Y[4] + p1.x) * i1.x, (Y[5] + p1.y) * i1.y, (Y[6] + p1.z) * i1.z, (Y[7] + p1.w) * i1.w);
    }
    HEIST_STAMP(9);
  }
}

// ===========================================================================
// 32-column grids (BASELINE C5: 32 x 32) in row bands.
//
// One 32 x 32 env's padded act2 plane alone (34 rows x 34 x 144 B = 166 KB) exceeds the
// CU's 160 KiB LDS, so the env is processed in NB = R / BR bands of BR conv3 output rows.
// Band b (image rows y0 = b BR .. y0 + BR - 1) needs act2 rows y0 - 1 .. y0 + BR (conv2,
// BR + 2 rows) and act1 rows y0 - 2 .. y0 + BR + 1 (conv1, BR + 4 rows); the halo rows are
// recomputed per band (conv1 +50 %, conv2 +25 %, conv3 and the pool exact: 12 % more MFMA
// work in all at BR = 8) and rows outside the image are stored as zeros (the convs' zero
// padding).  With C = 32 an MFMA position tile is exactly one row, so every tile is
// wholly inside or outside the image (a wave-uniform predicate) and the tap offsets are
// plain row / column strides.  The input plane holds the whole env (34 x 34 x 8 B); the
// act planes are band-local.  Per band: conv2 (three k-outer passes as in the full-plane
// kernel) -> B3 -> conv3 + pool, then the NEXT band's conv1 (or the next env's band 0)
// -> B4.  The pooled sums accumulate in registers across the env's bands.
// ===========================================================================

template <int R, int BR>
struct BandGeom {
  static constexpr int C = 32, PC = C + 2, NB = R / BR, RC = R * C;
  static constexpr int S0 = 8, S1 = 80, S2 = 144;  // bytes per padded position (as ConvGeom)
  static constexpr int T1 = BR + 4, T2 = BR + 2, T3 = BR;  // tiles (= rows) of conv1 / conv2 / conv3 per band
  static constexpr int PB0 = PC * S0, PB1 = PC * S1, PB2 = PC * S2;
  // 16 consecutive positions of one row are 80 B (5 bank groups) or 144 B (9 groups)
  // apart: 16 distinct 16-byte bank groups in every ds_read_b128 (5, 9 odd)
  static constexpr int IN = 0;
  static constexpr int A1 = align16c(IN + (R + 2) * PB0);
  static constexpr int A2 = align16c(A1 + T1 * PB1);
  static constexpr int ZERO_END = align16c(A2 + T2 * PB2);  // zeroed once (column pads, input border)
  static constexpr int POOL = ZERO_END;                    // [64][16] f32
  static constexpr int BIAS = POOL + 64 * 16 * 4;          // b1[32] b2[64] b3[64]
  static constexpr int INVA = BIAS + 160 * 4;              // [16] f32 1/area
  static constexpr int PM = INVA + 16 * 4;                 // [R][2][64] pool-membership bytes by image row
  static constexpr int W2 = align16c(PM + R * 128);        // conv2 fragments [2][18][64] x 16 B
  static constexpr int LDS = W2 + 2 * 18 * 64 * 16;
  static constexpr int QI = (RC + 255) / 256;
  static_assert(R % BR == 0 && T1 % 4 == 0 && T2 % 2 == 0 && T3 % 2 == 0, "band tiles split evenly over waves");
  static_assert(LDS <= 160 * 1024, "input plane + band planes + conv2 fragments must fit 160 KiB LDS");
};

// One k-outer pass of a band's conv2 over the wave's tiles [T0, T1) (tile i = band row
// mh + 2 i, image row y0 - 1 + that), hiding the previous pass's epilogue [P0, P1) under
// its MFMAs (see conv2_pass); a tile whose image row is outside the grid stores zeros.
template <int R, int BR, int T0, int T1, int P0, int P1, int NA, int NP>
__device__ __forceinline__ void conv2_band_pass(unsigned char* smem, const bf16x8* wl, const float4 (&b2v)[4], int mh,
                                                int nh, int lr, int h, int y0, f32x16 (&cur)[NA],
                                                const f32x16 (&prv)[NP]) {
  using G = BandGeom<R, BR>;
  constexpr int NTP = T1 - T0, NQ = kW2Steps * NTP, kPre2 = HEIST_CONV2_PRE;
  constexpr int NPIECE = (P1 - P0) * 16;
  constexpr int PER_Q = NQ > 0 ? (NPIECE + NQ - 1) / (NQ > 0 ? NQ : 1) : NPIECE;
  bf16x4 o;
  auto piece = [&](int k) {
    const int ti = k >> 4, kk = k & 15, g = kk >> 2, jj = kk & 3;
    const int row = mh + 2 * (P0 + ti);
    const bool valid = (unsigned)(y0 - 1 + row) < (unsigned)R;
    const float bv = jj == 0 ? b2v[g].x : (jj == 1 ? b2v[g].y : (jj == 2 ? b2v[g].z : b2v[g].w));
    o[jj] = (__bf16)(valid ? relu(prv[ti][kk] + bv) : 0.f);
    if (jj == 3)
      *reinterpret_cast<bf16x4*>(smem + G::A2 + row * G::PB2 + (lr + 1) * G::S2 + (32 * nh + 8 * g + 4 * h) * 2) = o;
  };
  if constexpr (NQ > 0) {
    const unsigned char* base[NTP];
#pragma unroll
    for (int i = 0; i < NTP; ++i) {
      base[i] = smem + G::A1 + (mh + 2 * (T0 + i)) * G::PB1 + lr * G::S1 + 16 * h;
      cur[i] = f32x16{};
    }
    auto rd = [&](int q) {
      const int s = q / NTP, tap = s >> 1;
      return *reinterpret_cast<const bf16x8*>(base[q % NTP] + (tap / 3) * G::PB1 + (tap % 3) * G::S1 + (s & 1) * 32);
    };
    bf16x8 ring[kPre2];
#pragma unroll
    for (int q = 0; q < kPre2; ++q) ring[q] = rd(q < NQ ? q : NQ - 1);
    // weight fragments two k-steps ahead (a 3-slot ring); read one k-step ahead, their LDS
    // latency was exposed at every k-step boundary (only NTP MFMAs after the read)
    bf16x8 wb[3];
    wb[0] = wl[0];
    wb[1] = wl[64];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int s = q / NTP, i = q % NTP;
      if (i == 0 && s + 2 < kW2Steps) wb[(s + 2) % 3] = wl[(s + 2) * 64];
      const bf16x8 f = ring[q % kPre2];
      if (q + kPre2 < NQ) ring[q % kPre2] = rd(q + kPre2);
      cur[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wb[s % 3], f, cur[i], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < PER_Q; ++r)
        if (q * PER_Q + r < NPIECE) piece(q * PER_Q + r);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, kPre2 + 2, 0);
    sched_ring<NTP, 1>(std::make_integer_sequence<int, NQ>{});
  } else {
#pragma unroll
    for (int k = 0; k < NPIECE; ++k) piece(k);
  }
}

template <int R, int BR>
__global__ __launch_bounds__(256, 1) void solver_conv_band_kernel(const float* __restrict__ obs, int n,
                                                                  const uint4* __restrict__ packed,
                                                                  float* __restrict__ feat) {
  using G = BandGeom<R, BR>;
  constexpr int C = G::C, PC = G::PC;
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63, h = l >> 5, lr = l & 31;
  const int nh = w & 1, mh = w >> 1;

  // ---- weights -> registers / LDS, tables -> LDS (as solver_conv_kernel)
  bf16x8 w1[kW1Steps], w3[kW3Steps];
#pragma unroll
  for (int s = 0; s < kW1Steps; ++s) {
    w1[s] = __builtin_bit_cast(bf16x8, packed[kOffW1 + s * 64 + l]);
    in_agpr(w1[s]);
  }
#pragma unroll
  for (int s = 0; s < kW3Steps; ++s) {
    w3[s] = __builtin_bit_cast(bf16x8, packed[kOffW3 + (nh * kW3Steps + s) * 64 + l]);
    in_agpr(w3[s]);
  }
  copy_w2(smem + G::W2, packed, tid);
  const float* gbias = reinterpret_cast<const float*>(packed + kOffBias);
  float* bias = reinterpret_cast<float*>(smem + G::BIAS);
  const float b3v = gbias[96 + 32 * nh + lr];
  if (tid < 160) bias[tid] = gbias[tid];
  for (int i = tid; i < G::ZERO_END / 16; i += 256) reinterpret_cast<uint4*>(smem)[i] = make_uint4(0u, 0u, 0u, 0u);
  if (tid < 16) {
    const int ci = tid >> 2, cj = tid & 3;
    const int area = (pool_hi(ci, R) - pool_lo(ci, R)) * (pool_hi(cj, C) - pool_lo(cj, C));
    reinterpret_cast<float*>(smem + G::INVA)[tid] = 1.0f / (float)area;
  }
  for (int i = tid; i < R * 128; i += 256) {  // pool membership of the P fragment bits, by image row
    const int y = i >> 7, s = (i >> 6) & 1, ll = i & 63;
    const int cell = ll & 31, hh = ll >> 5;
    unsigned bits = 0;
    if (cell < 16) {
      const int ci = cell >> 2, cj = cell & 3;
      for (int j = 0; j < 8; ++j) {
        const int ox = 16 * s + 8 * (j >> 2) + 4 * hh + (j & 3);
        if (y >= pool_lo(ci, R) && y < pool_hi(ci, R) && ox >= pool_lo(cj, C) && ox < pool_hi(cj, C)) bits |= 1u << j;
      }
    }
    smem[G::PM + i] = (unsigned char)bits;
  }
  int off1a[kW1Steps], off1b[kW1Steps];
#pragma unroll
  for (int s = 0; s < kW1Steps; ++s) {
    int ta = 4 * s + 2 * h, tb = ta + 1;
    ta = ta < 9 ? ta : 4;
    tb = tb < 9 ? tb : 4;
    off1a[s] = ((ta / 3) * PC + (ta % 3)) * G::S0;
    off1b[s] = ((tb / 3) * PC + (tb % 3)) * G::S0;
  }

  // conv1 of the band starting at image row y0: band tile j = w + 4 i is image row
  // y0 - 2 + j; rows outside the grid read a clamped row and store zeros
  constexpr int NT1 = G::T1 / 4;
  auto conv1_band = [&](int y0) {
    bf16x8 f1[NT1][kW1Steps];
#pragma unroll
    for (int i = 0; i < NT1; ++i) {
      const int y = y0 - 2 + w + 4 * i;
      const int yc = y < 0 ? 0 : (y >= R ? R - 1 : y);
      const unsigned char* base = smem + G::IN + (yc * PC + lr) * G::S0;  // top-left tap (padded row yc)
#pragma unroll
      for (int s = 0; s < kW1Steps; ++s) {
        const uint2 a = *reinterpret_cast<const uint2*>(base + off1a[s]);
        const uint2 b = *reinterpret_cast<const uint2*>(base + off1b[s]);
        f1[i][s] = __builtin_bit_cast(bf16x8, make_uint4(a.x, a.y, b.x, b.y));
      }
    }
#pragma unroll
    for (int i = 0; i < NT1; ++i) {
      const int j = w + 4 * i;
      const bool valid = (unsigned)(y0 - 2 + j) < (unsigned)R;
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < kW1Steps; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(in_agpr(w1[s]), f1[i][s], acc, 0, 0, 0);
      unsigned char* dst = smem + G::A1 + j * G::PB1 + (lr + 1) * G::S1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n0 = 8 * g + 4 * h;
        const float4 b = *reinterpret_cast<const float4*>(bias + n0);
        bf16x4 o;
        o[0] = (__bf16)(valid ? relu(acc[4 * g + 0] + b.x) : 0.f);
        o[1] = (__bf16)(valid ? relu(acc[4 * g + 1] + b.y) : 0.f);
        o[2] = (__bf16)(valid ? relu(acc[4 * g + 2] + b.z) : 0.f);
        o[3] = (__bf16)(valid ? relu(acc[4 * g + 3] + b.w) : 0.f);
        *reinterpret_cast<bf16x4*>(dst + n0 * 2) = o;
      }
    }
  };

  float pre[G::QI][3];
  int e = blockIdx.x;
  if (e < n) load_obs<G>(obs, e, pre);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (e < n) {
    stage_obs<G>(smem, pre);
    __syncthreads();
    conv1_band(0);
  }
  __syncthreads();  // act1 of the first band ready

  f32x16 Y = {};
  for (; e < n; e += gridDim.x) {
    const int en = e + gridDim.x;
    const bool has_next = en < n;  // workgroup-uniform
    for (int b = 0; b < G::NB; ++b) {
      const int y0 = b * BR;
      const bool last = b == G::NB - 1;
      if (last && has_next) load_obs<G>(obs, en, pre);  // next env's observation in flight during conv2
      // ---- conv2 of the band: D[32 ch of nh][band row] in three k-outer passes
      {
        constexpr int NT2 = G::T2 / 2;
        constexpr int SA = (NT2 * 3 + 6) / 7, SB = SA + (NT2 - SA + 1) / 2;
        constexpr int NA = SA, NB2 = SB - SA > 0 ? SB - SA : 1, NC = NT2 - SB > 0 ? NT2 - SB : 1;
        const bf16x8* wl = reinterpret_cast<const bf16x8*>(smem + G::W2) + nh * kW2Steps * 64 + l;
        float4 b2v[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) b2v[g] = *reinterpret_cast<const float4*>(bias + 32 + 32 * nh + 8 * g + 4 * h);
        f32x16 accA[NA], accB[NB2], accC[NC];
        conv2_band_pass<R, BR, 0, SA, 0, 0, NA, NA>(smem, wl, b2v, mh, nh, lr, h, y0, accA, accA);
        conv2_band_pass<R, BR, SA, SB, 0, SA, NB2, NA>(smem, wl, b2v, mh, nh, lr, h, y0, accB, accA);
        conv2_band_pass<R, BR, SB, NT2, SA, SB, NC, NB2>(smem, wl, b2v, mh, nh, lr, h, y0, accC, accB);
        conv2_band_pass<R, BR, NT2, NT2, SB, NT2, NC, NC>(smem, wl, b2v, mh, nh, lr, h, y0, accC, accC);
      }
      if (last && has_next) stage_obs<G>(smem, pre);  // the input plane's last reader ran a band ago
      __syncthreads();  // B3: act2 of the band (and the next env's input) ready; act1 reads done

      // ---- conv3 of the band + pooling (as solver_conv_kernel), Y accumulates over bands
      {
        constexpr int NT3 = G::T3 / 2, NQ = NT3 * kW3Steps, kPre = 7;
        const unsigned char* base[NT3];
#pragma unroll
        for (int i = 0; i < NT3; ++i) base[i] = smem + G::A2 + (mh + 2 * i) * G::PB2 + lr * G::S2 + 16 * h;
        auto rd = [&](int q) {
          const int s = q % kW3Steps, tap = s >> 2;
          return *reinterpret_cast<const bf16x8*>(base[q / kW3Steps] + (tap / 3) * G::PB2 + (tap % 3) * G::S2 +
                                                  (s & 3) * 32);
        };
        bf16x8 ring[kPre];
#pragma unroll
        for (int q = 0; q < kPre; ++q) ring[q] = rd(q);
        f32x16 prev = {};
        bf16x8 x[2], pf[2];
        auto pool_piece = [&](int row, int s) {  // piece s of band row `row`'s epilogue (prev holds its sums)
          if (s < 16) x[s >> 3][s & 7] = (__bf16)relu(prev[s] + b3v);
          if (s == 0 || s == 1) {
            const unsigned bits = smem[G::PM + ((y0 + row) * 2 + s) * 64 + l];
#pragma unroll
            for (int j = 0; j < 8; ++j) pf[s][j] = ((bits >> j) & 1u) ? (__bf16)1.0f : (__bf16)0.0f;
          }
          if (s == 16) Y = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf[0], x[0], Y, 0, 0, 0);
          if (s == 17) Y = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf[1], x[1], Y, 0, 0, 0);
        };
#pragma unroll
        for (int i = 0; i < NT3; ++i) {
          f32x16 acc = {};
#pragma unroll
          for (int s = 0; s < kW3Steps; ++s) {
            const int q = i * kW3Steps + s;
            const bf16x8 f = ring[q % kPre];
            if (q + kPre < NQ) ring[q % kPre] = rd(q + kPre);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f, in_agpr(w3[s]), acc, 0, 0, 0);
            if (i > 0 && s < 18) pool_piece(mh + 2 * (i - 1), s);
          }
          prev = acc;
        }
        __builtin_amdgcn_sched_group_barrier(0x100, kPre, 0);
        sched_ring<kW3Steps, 0>(std::make_integer_sequence<int, NQ>{});
#pragma unroll
        for (int s = 0; s < 18; ++s) pool_piece(mh + 2 * (NT3 - 1), s);
      }
      // conv1 of the next band (or the next env's first band; after the last env: harmless)
      conv1_band(last ? 0 : y0 + BR);
      float* pool = reinterpret_cast<float*>(smem + G::POOL) + (32 * nh + lr) * 16 + 4 * h;
      if (last && mh == 1) {
        *reinterpret_cast<float4*>(pool) = make_float4(Y[0], Y[1], Y[2], Y[3]);
        *reinterpret_cast<float4*>(pool + 8) = make_float4(Y[4], Y[5], Y[6], Y[7]);
      }
      __syncthreads();  // B4: act1 of the next band written; partner half of the pool sums in LDS
      if (last) {
        if (mh == 0) {
          const float4 p0 = *reinterpret_cast<const float4*>(pool);
          const float4 p1 = *reinterpret_cast<const float4*>(pool + 8);
          const float* inva = reinterpret_cast<const float*>(smem + G::INVA) + 4 * h;
          const float4 i0 = *reinterpret_cast<const float4*>(inva);
          const float4 i1 = *reinterpret_cast<const float4*>(inva + 8);
          float* out = feat + (size_t)e * 1024 + (32 * nh + lr) * 16 + 4 * h;
          *reinterpret_cast<float4*>(out) =
              make_float4((Y[0] + p0.x) * i0.x, (Y[1] + p0.y) * i0.y, (Y[2] + p0.z) * i0.z, (Y[3] + p0.w) * i0.w);
          *reinterpret_cast<float4*>(out + 8) =
              make_float4((Y[4] + p1.x) * i1.x, (Y[5] + p1.y) * i1.y, (Y[6] + p1.z) * i1.z, (Y[7] + p1.w) * i1.w);
        }
        Y = f32x16{};
      }
    }
  }
}

// Weight packing: fragment element j of lane l, k-step s, output tile nt holds
// W[co = 32 nt + (l & 31)][k = 16 s + 8 (l >> 5) + j] with k = tap * CinP + ci,
// tap = 3 ky + kx; zero where ci >= Cin or tap >= 9.  bf16 round-to-nearest-even.
__global__ void solver_pack_kernel(const float* __restrict__ w1, const float* __restrict__ b1,
                                   const float* __restrict__ w2, const float* __restrict__ b2,
                                   const float* __restrict__ w3, const float* __restrict__ b3,
                                   uint4* __restrict__ packed) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // one fragment (8 elements) per thread
  const int nfrag = kOffBias;
  if (i < nfrag) {
    int layer, rem;
    if (i < kOffW2) { layer = 0; rem = i - kOffW1; }
    else if (i < kOffW3) { layer = 1; rem = i - kOffW2; }
    else { layer = 2; rem = i - kOffW3; }
    const int steps = layer == 0 ? kW1Steps : (layer == 1 ? kW2Steps : kW3Steps);
    const int cinp = layer == 0 ? 4 : (layer == 1 ? 32 : 64);
    const int cin = layer == 0 ? 3 : cinp;
    const float* W = layer == 0 ? w1 : (layer == 1 ? w2 : w3);
    const int l = rem & 63, s = (rem >> 6) % steps, nt = (rem >> 6) / steps;
    const int co = 32 * nt + (l & 31);
    bf16x8 f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * s + 8 * (l >> 5) + j;
      const int tap = k / cinp, ci = k % cinp;
      const float v = (tap < 9 && ci < cin) ? W[((size_t)co * cin + ci) * 9 + tap] : 0.0f;
      f[j] = (__bf16)v;
    }
    packed[i] = __builtin_bit_cast(uint4, f);
  } else if (i < nfrag + 160) {
    const int k = i - nfrag;
    const float v = k < 32 ? b1[k] : (k < 96 ? b2[k - 32] : b3[k - 96]);
    reinterpret_cast<float*>(packed + kOffBias)[k] = v;
  }
}

int solver_packed_bytes() { return kPackedBytes; }

hipError_t launch_solver_pack(const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                              const float* b3, void* packed, hipStream_t st) {
  const int total = kOffBias + 160;
  hipLaunchKernelGGL(solver_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w1, b1, w2, b2, w3, b3,
                     reinterpret_cast<uint4*>(packed));
  return hipGetLastError();
}

static unsigned long long* g_conv_stamps = nullptr;
void set_solver_stamps(unsigned long long* p) { g_conv_stamps = p; }

template <int R, int C>
static hipError_t launch_conv_rc(const float* obs, int n, const void* packed, float* feat, int n_cu, hipStream_t st) {
  using G = ConvGeom<R, C>;
  static bool attr_set = false;  // per process; the attribute is per function, not per device
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&solver_conv_kernel<R, C>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int grid = n < n_cu ? n : n_cu;
  hipLaunchKernelGGL((solver_conv_kernel<R, C>), dim3(grid), dim3(256), G::LDS, st, obs, n,
                     reinterpret_cast<const uint4*>(packed), feat, g_conv_stamps);
  return hipGetLastError();
}

// 32 x 32 (BASELINE C5): the row-band kernel, bands of 8 conv3 rows
constexpr int kBandRows = 8;
static hipError_t launch_conv_band32(const float* obs, int n, const void* packed, float* feat, int n_cu,
                                     hipStream_t st) {
  using G = BandGeom<32, kBandRows>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&solver_conv_band_kernel<32, kBandRows>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int grid = n < n_cu ? n : n_cu;
  hipLaunchKernelGGL((solver_conv_band_kernel<32, kBandRows>), dim3(grid), dim3(256), G::LDS, st, obs, n,
                     reinterpret_cast<const uint4*>(packed), feat);
  return hipGetLastError();
}

bool solver_conv_supported(int R, int C) {
  return (R == 20 && C == 20) || (R == 10 && C == 10) || (R == 32 && C == 32);
}

hipError_t launch_solver_conv(const float* obs, int n, int R, int C, const void* packed, float* feat, int n_cu,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (R == 20 && C == 20) return launch_conv_rc<20, 20>(obs, n, packed, feat, n_cu, st);
  if (R == 10 && C == 10) return launch_conv_rc<10, 10>(obs, n, packed, feat, n_cu, st);
  if (R == 32 && C == 32) return launch_conv_band32(obs, n, packed, feat, n_cu, st);
  return hipErrorInvalidValue;
}

// ===========================================================================
// Fused Solver head: fc_spatial + ReLU, one LSTM cell step, policy/value heads,
// softmax, Categorical sample and log-prob (networks.py:102-131, agents/solver.py:75-99)
// for blocks of 32 envs.  GEMMs on v_mfma_f32_32x32x16_bf16 (activations bf16 in LDS,
// weights as packed fragments streamed from L2, fp32 accumulate); the LSTM elementwise
// math, the last head layers (128 -> A, 128 -> 1) and the sampling in fp32.
// ===========================================================================

// Packed head blob, uint4 units: Wfc [8 nt][64 ks][64], Wg = [W_ih | W_hh] [16][24][64],
// Wh1 = [policy_head.0 ; value_head.0] [8][8][64]; then floats.
constexpr int kHFc = 0;
constexpr int kHG = kHFc + 8 * 64 * 64;
constexpr int kHH1 = kHG + 16 * 24 * 64;
constexpr int kHF32 = kHH1 + 8 * 8 * 64;
// float offsets inside the f32 area
constexpr int kFBfc = 0, kFBg = 256, kFBh1 = 768, kFWp2 = 1024, kFBp2 = 1024 + 8 * 128, kFWv2 = kFBp2 + 8,
              kFBv2 = kFWv2 + 128, kFEnd = kFBv2 + 4;
constexpr int kHeadPackedBytes = kHF32 * 16 + kFEnd * 4;
constexpr int kMaxActions = 7;

struct HeadLds {  // byte offsets
  static constexpr int X0S = 1032 * 2, X1S = 264 * 2, HS = 136 * 2, HVS = 260 * 4;
  static constexpr int X0 = 0;
  static constexpr int X1 = X0 + 32 * X0S;
  static constexpr int HP = X1 + 32 * X1S;
  static constexpr int HN = HP + 32 * HS;
  static constexpr int HV = HN + 32 * HS;
  static constexpr int OUT = HV + 32 * HVS;  // [32][8] f32
  static constexpr int LDS = OUT + 32 * 8 * 4;
};

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}

// acc[t] += A(LDS rows, k-steps [ks0, ks0+KS)) . B(fragments of n-tiles nts[t], from global)
template <int NTL, int KS>
__device__ __forceinline__ void head_gemm(f32x16 (&acc)[NTL], const unsigned char* abase, int astride_ks,
                                          const uint4* __restrict__ bfr, const int (&bidx)[NTL], int l) {
  constexpr int kPre = 4;
  bf16x8 ring[kPre][NTL];
#pragma unroll
  for (int q = 0; q < kPre; ++q)
#pragma unroll
    for (int t = 0; t < NTL; ++t) ring[q][t] = __builtin_bit_cast(bf16x8, bfr[bidx[t] + q * 64 + l]);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(abase + ks * astride_ks);
#pragma unroll
    for (int t = 0; t < NTL; ++t) {
      const bf16x8 b = ring[ks % kPre][t];
      if (ks + kPre < KS) ring[ks % kPre][t] = __builtin_bit_cast(bf16x8, bfr[bidx[t] + (ks + kPre) * 64 + l]);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[t], 0, 0, 0);
    }
  }
}

__global__ __launch_bounds__(256, 1) void solver_head_kernel(const float* __restrict__ feat,
                                                             const float* __restrict__ h_in,
                                                             const float* __restrict__ c_in, int n,
                                                             const uint4* __restrict__ packed, int A, uint64_t seed,
                                                             uint64_t counter, float* __restrict__ logits_out,
                                                             float* __restrict__ value_out,
                                                             int64_t* __restrict__ action_out,
                                                             float* __restrict__ logp_out, float* __restrict__ h_out,
                                                             float* __restrict__ c_out) {
  using L = HeadLds;
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, h = l >> 5, lr = l & 31;
  const int e0 = blockIdx.x * 32;
  const float* fp = reinterpret_cast<const float*>(packed + kHF32);

  // ---- stage 0: features and h_prev -> bf16 rows in LDS (rows past n repeat row n-1)
  for (int i = tid; i < 32 * 256; i += 256) {
    const int r = i >> 8, q = i & 255;
    const int e = min(e0 + r, n - 1);
    const float4 v = reinterpret_cast<const float4*>(feat + (size_t)e * 1024)[q];
    bf16x4 b;
    b[0] = (__bf16)v.x; b[1] = (__bf16)v.y; b[2] = (__bf16)v.z; b[3] = (__bf16)v.w;
    *reinterpret_cast<bf16x4*>(smem + L::X0 + r * L::X0S + q * 8) = b;
  }
  for (int i = tid; i < 32 * 32; i += 256) {
    const int r = i >> 5, q = i & 31;
    const int e = min(e0 + r, n - 1);
    const float4 v = h_in ? reinterpret_cast<const float4*>(h_in + (size_t)e * 128)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    bf16x4 b;
    b[0] = (__bf16)v.x; b[1] = (__bf16)v.y; b[2] = (__bf16)v.z; b[3] = (__bf16)v.w;
    *reinterpret_cast<bf16x4*>(smem + L::HP + r * L::HS + q * 8) = b;
  }
  __syncthreads();

  // ---- stage 1: x = relu(feat . Wfc^T + b) [32 x 256]; wave w: n-tiles w, w + 4
  {
    f32x16 acc[2] = {f32x16{}, f32x16{}};
    const int bidx[2] = {(w * 64) * 64, ((w + 4) * 64) * 64};
    head_gemm<2, 64>(acc, smem + L::X0 + lr * L::X0S + 16 * h, 32, packed + kHFc, bidx, l);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int nn = 32 * (w + 4 * t) + lr;
      const float b = fp[kFBfc + nn];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        *reinterpret_cast<__bf16*>(smem + L::X1 + row * L::X1S + nn * 2) = (__bf16)relu(acc[t][r] + b);
      }
    }
  }
  __syncthreads();

  // ---- stage 2: gates = [x | h] . [W_ih | W_hh]^T + b_ih + b_hh; wave w owns hidden units
  // 32w..32w+31 of all four gates (i, f, g, o), so the cell update stays in registers
  {
    f32x16 acc[4] = {f32x16{}, f32x16{}, f32x16{}, f32x16{}};
    const int bidx[4] = {(w * 24) * 64, ((w + 4) * 24) * 64, ((w + 8) * 24) * 64, ((w + 12) * 24) * 64};
    head_gemm<4, 16>(acc, smem + L::X1 + lr * L::X1S + 16 * h, 32, packed + kHG, bidx, l);
    const int bidx2[4] = {bidx[0] + 16 * 64, bidx[1] + 16 * 64, bidx[2] + 16 * 64, bidx[3] + 16 * 64};
    head_gemm<4, 8>(acc, smem + L::HP + lr * L::HS + 16 * h, 32, packed + kHG, bidx2, l);
    const int j = 32 * w + lr;
    const float bi = fp[kFBg + j], bf = fp[kFBg + 128 + j], bg = fp[kFBg + 256 + j], bo = fp[kFBg + 384 + j];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int e = e0 + row;
      const float cprev = (c_in && e < n) ? c_in[(size_t)e * 128 + j] : 0.0f;
      const float c1 = sigmoidf_(acc[1][r] + bf) * cprev + sigmoidf_(acc[0][r] + bi) * tanhf(acc[2][r] + bg);
      const float h1 = sigmoidf_(acc[3][r] + bo) * tanhf(c1);
      if (e < n) {
        c_out[(size_t)e * 128 + j] = c1;
        h_out[(size_t)e * 128 + j] = h1;
      }
      *reinterpret_cast<__bf16*>(smem + L::HN + row * L::HS + j * 2) = (__bf16)h1;
    }
  }
  __syncthreads();

  // ---- stage 3: head hidden layers relu(h' . [Wp1 ; Wv1]^T + b) [32 x 256] (f32 in LDS)
  {
    f32x16 acc[2] = {f32x16{}, f32x16{}};
    const int bidx[2] = {(w * 8) * 64, ((w + 4) * 8) * 64};
    head_gemm<2, 8>(acc, smem + L::HN + lr * L::HS + 16 * h, 32, packed + kHH1, bidx, l);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int nn = 32 * (w + 4 * t) + lr;
      const float b = fp[kFBh1 + nn];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        reinterpret_cast<float*>(smem + L::HV + row * L::HVS)[nn] = relu(acc[t][r] + b);
      }
    }
  }
  __syncthreads();

  // ---- stage 4: logits (128 -> A) and value (128 -> 1) in fp32; thread = (env, output)
  {
    const int row = tid >> 3, o = tid & 7;
    const float* hv = reinterpret_cast<const float*>(smem + L::HV + row * L::HVS);
    float acc = 0.f;
    if (o < A) {
      const float* wr = fp + kFWp2 + o * 128;
      for (int k = 0; k < 128; ++k) acc += hv[k] * wr[k];
      acc += fp[kFBp2 + o];
    } else if (o == 7) {
      const float* wr = fp + kFWv2;
      for (int k = 0; k < 128; ++k) acc += hv[128 + k] * wr[k];
      acc += fp[kFBv2];
    }
    reinterpret_cast<float*>(smem + L::OUT)[row * 8 + o] = acc;
  }
  __syncthreads();

  // ---- stage 5: Categorical(probs = softmax(logits)): sample, log_prob (torch semantics:
  // probs renormalised, log(clamp(p, eps, 1 - eps)))
  if (tid < 32 && e0 + tid < n) {
    const int e = e0 + tid;
    const float* lg = reinterpret_cast<const float*>(smem + L::OUT) + tid * 8;
    float mx = lg[0];
    for (int a = 1; a < A; ++a) mx = fmaxf(mx, lg[a]);
    float p[kMaxActions], s = 0.f;
    for (int a = 0; a < A; ++a) {
      p[a] = __expf(lg[a] - mx);
      s += p[a];
    }
    float ps = 0.f;
    for (int a = 0; a < A; ++a) {
      p[a] = p[a] / s;
      ps += p[a];
    }
    const uint64_t z = mix64(seed ^ (counter * 0xD1B54A32D192ED03ull) ^ ((uint64_t)e * 0x9E3779B97F4A7C15ull));
    const float u = (float)(z >> 40) * 0x1p-24f * ps;
    int act = A - 1;
    float cum = 0.f;
    for (int a = 0; a < A; ++a) {
      cum += p[a];
      if (u < cum) { act = a; break; }
    }
    const float eps = 1.1920928955078125e-07f;
    float pa = p[act] / ps;
    pa = fminf(fmaxf(pa, eps), 1.0f - eps);
    if (logits_out)
      for (int a = 0; a < A; ++a) logits_out[(size_t)e * A + a] = lg[a];
    value_out[e] = lg[7];
    action_out[e] = act;
    logp_out[e] = __logf(pa);
  }
}

// Fragment packing for the head: fragment (nt, ks, lane) element j = W[32 nt + (lane & 31)][k]
// with k = 16 ks + 8 (lane >> 5) + j (bf16 RNE); f32 tail copied (b_ih + b_hh summed).
__global__ void solver_head_pack_kernel(const float* __restrict__ fc_w, const float* __restrict__ fc_b,
                                        const float* __restrict__ w_ih, const float* __restrict__ w_hh,
                                        const float* __restrict__ b_ih, const float* __restrict__ b_hh,
                                        const float* __restrict__ p1_w, const float* __restrict__ p1_b,
                                        const float* __restrict__ v1_w, const float* __restrict__ v1_b,
                                        const float* __restrict__ p2_w, const float* __restrict__ p2_b,
                                        const float* __restrict__ v2_w, const float* __restrict__ v2_b, int A,
                                        uint4* __restrict__ packed) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < kHF32) {
    const int l = i & 63, f = i >> 6;
    const int r = l & 31, hh = l >> 5;
    const float* src;
    int ld, nn, k0;
    if (i < kHG) {
      const int nt = f / 64, ks = f % 64;
      src = fc_w; ld = 1024; nn = 32 * nt + r; k0 = 16 * ks + 8 * hh;
    } else if (i < kHH1) {
      const int g = f - kHG / 64, nt = g / 24, ks = g % 24;
      nn = 32 * nt + r;
      if (ks < 16) { src = w_ih; ld = 256; k0 = 16 * ks + 8 * hh; }
      else { src = w_hh; ld = 128; k0 = 16 * (ks - 16) + 8 * hh; }
    } else {
      const int g = f - kHH1 / 64, nt = g / 8, ks = g % 8;
      nn = 32 * nt + r;
      ld = 128; k0 = 16 * ks + 8 * hh;
      src = nn < 128 ? p1_w : v1_w;
      if (nn >= 128) nn -= 128;
    }
    bf16x8 fr;
#pragma unroll
    for (int j = 0; j < 8; ++j) fr[j] = (__bf16)src[(size_t)nn * ld + k0 + j];
    packed[i] = __builtin_bit_cast(uint4, fr);
  } else if (i < kHF32 + kFEnd) {
    const int k = i - kHF32;
    float v = 0.f;
    if (k < kFBg) v = fc_b[k];
    else if (k < kFBh1) v = b_ih[k - kFBg] + b_hh[k - kFBg];
    else if (k < kFWp2) v = (k - kFBh1) < 128 ? p1_b[k - kFBh1] : v1_b[k - kFBh1 - 128];
    else if (k < kFBp2) { const int o = (k - kFWp2) / 128; v = o < A ? p2_w[(k - kFWp2)] : 0.f; }
    else if (k < kFWv2) v = (k - kFBp2) < A ? p2_b[k - kFBp2] : 0.f;
    else if (k < kFBv2) v = v2_w[k - kFWv2];
    else v = k == kFBv2 ? v2_b[0] : 0.f;
    reinterpret_cast<float*>(packed + kHF32)[k] = v;
  }
}

int solver_head_packed_bytes() { return kHeadPackedBytes; }

hipError_t launch_solver_head_pack(const float* const* w, int A, void* packed, hipStream_t st) {
  const int total = kHF32 + kFEnd;
  hipLaunchKernelGGL(solver_head_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w[0], w[1], w[2], w[3],
                     w[4], w[5], w[6], w[7], w[8], w[9], w[10], w[11], w[12], w[13], A,
                     reinterpret_cast<uint4*>(packed));
  return hipGetLastError();
}

hipError_t launch_solver_head(const float* feat, const float* h_in, const float* c_in, int n, const void* packed,
                              int A, uint64_t seed, uint64_t counter, float* logits_out, float* value_out,
                              int64_t* action_out, float* logp_out, float* h_out, float* c_out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&solver_head_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, HeadLds::LDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(solver_head_kernel, dim3((n + 31) / 32), dim3(256), HeadLds::LDS, st, feat, h_in, c_in, n,
                     reinterpret_cast<const uint4*>(packed), A, seed, counter, logits_out, value_out, action_out,
                     logp_out, h_out, c_out);
  return hipGetLastError();
}

}  // namespace heist
