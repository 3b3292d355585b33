// Store-stream microbenchmark for the lean K-tick kernel's observation writes: 4096 waves
// (16 per CU), each writing one env's [3][20][20] f32 row (4,800 B) per tick for K = 20 ticks
// into a [K][4096][4800 B] buffer, in several instruction shapes and cache policies.  Prints
// TB/s per variant (HIP events around 20 launches after 5 warm-up).  Not part of the product;
// build: hipcc --offload-arch=gfx950 -O3 tools/store_bench.hip -o /tmp/store_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
constexpr int N = 4096, K = 20, Q4 = 100;  // quads per channel (400 floats / 4)

template <int AUX>
__device__ __forceinline__ void put(__amdgpu_buffer_rsrc_t rs, int off, u32x4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, AUX);
}

// SHAPE 0: the lean kernel's (per channel: quads lane and 64 + lane < 100, i.e. 1,024 B + 576 B;
//          order ch0 a, ch1 a, ch2 a, ch0 b, ch1 b, ch2 b)
// SHAPE 1: the row as 300 flat quads: 5 instructions (4 x 1,024 B + 704 B)
// SHAPE 2: as 0, rows padded to a 4,864-B stride (every row line-aligned)
template <int SHAPE, int AUX>
__global__ __launch_bounds__(64) void store_kernel(unsigned char* out, int stride, int spin) {
  const int e = blockIdx.x, lane = threadIdx.x;
  const u32x4_t v = {(unsigned)lane, (unsigned)e, 1u, 2u};
  for (int k = 0; k < K; ++k) {
    unsigned char* row = out + ((size_t)k * N + e) * stride;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row, (short)0, 4800, 0x00020000);
    if (SHAPE == 0 || SHAPE == 2) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q = lane + 64 * j;
        const int off = q < Q4 ? 16 * q : 0x40000000;
#pragma unroll
        for (int c = 0; c < 3; ++c) put<AUX>(rs, off == 0x40000000 ? off : off + 1600 * c, v);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const int q = lane + 64 * j;
        put<AUX>(rs, q < 3 * Q4 ? 16 * q : 0x40000000, v);
      }
    }
    for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(1);  // a stand-in for the tick's compute
  }
}

template <int SHAPE, int AUX>
static float run(unsigned char* buf, int spin) {
  const int stride = SHAPE == 2 ? 4864 : 4800;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((store_kernel<SHAPE, AUX>), dim3(N), dim3(64), 0, 0, buf, stride, spin);
  hipEventRecord(a, 0);
  const int iters = 20;
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((store_kernel<SHAPE, AUX>), dim3(N), dim3(64), 0, 0, buf, stride, spin);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = (double)iters * K * N * 4800.0;
  const double tbs = bytes / (ms * 1e-3) / 1e12;
  printf("{\"shape\": %d, \"aux\": %d, \"spin\": %d, \"us_per_tick\": %.3f, \"TB_s\": %.3f}\n", SHAPE, AUX, spin,
         ms * 1e3 / (iters * K), tbs);
  fflush(stdout);
  return (float)tbs;
}

int main() {
  unsigned char* buf = nullptr;
  if (hipMalloc(&buf, (size_t)K * N * 4864) != hipSuccess) return 1;
  hipMemset(buf, 0, (size_t)K * N * 4864);
  for (int spin : {0, 8}) {
    run<0, 2>(buf, spin);
    run<0, 0>(buf, spin);
    run<1, 2>(buf, spin);
    run<1, 0>(buf, spin);
    run<2, 2>(buf, spin);
    run<2, 0>(buf, spin);
  }
  hipFree(buf);
  return 0;
}
