// heist_train.hip -- the elementwise tail of the Solver backbone's fp32 training step, fused.
//
// The PPO update (agents/solver.py:157-199) runs SolverNetwork.features (networks.py:93-100:
// relu(conv1) -> relu(conv2) -> relu(conv3) -> AdaptiveAvgPool2d(4, 4)) forward and backward
// on 16,384-sample minibatches.  The convolutions stay on MIOpen (fp32 implicit GEMM on MFMA,
// ~90 TFLOP/s); what PyTorch runs around them -- the bias add, ReLU, the NHWC adaptive pool
// and its backward, ReLU's backward and the bias-gradient reductions -- is one full pass over
// a [B, 20, 20, C] fp32 activation each (1.7 GB at C = 64), ~30 % of the update
// (profiles/r05f_train_kernel_stats.csv).  Here each layer's tail is ONE pass:
//   forward   y = relu(conv_nobias(x) + b) in place; for conv3 also the pooled features
//   backward  d = (y > 0) ? g : 0 in place (conv3: g from the pooled gradient / window
//             area), and per-sample bias-gradient partials, summed over samples in a fixed
//             order by a second small kernel (deterministic, no float atomics).
// Activations are NHWC (channels_last) fp32, the network's memory format.  The arithmetic is
// torch's: x + b rounded once, then max(., 0); the pool is the window sum in row-major order
// divided by the window area (torch's adaptive_avg_pool2d windows); ReLU's backward uses the
// saved output as torch's threshold_backward does.  Sums (pool, bias gradients) run in a fixed
// order that differs from torch's, so results match torch to fp32 rounding
// (tests/test_gpu_train_backbone.py), not bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace heist {
namespace tr {

// torch adaptive_avg_pool2d window [start, end) of output cell i (of 4) over n inputs
__device__ __forceinline__ int win_start(int i, int n) { return (i * n) / 4; }
__device__ __forceinline__ int win_end(int i, int n) { return ((i + 1) * n + 3) / 4; }

// y = relu(x + b) in place over n_pos positions of C channels (C % 4 == 0).
__global__ __launch_bounds__(256) void bias_relu_kernel(float* __restrict__ x, const float* __restrict__ b,
                                                         int64_t n4, int c4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 v = reinterpret_cast<float4*>(x)[i];
    const float4 bb = reinterpret_cast<const float4*>(b)[i % c4];
    v.x = fmaxf(v.x + bb.x, 0.f);
    v.y = fmaxf(v.y + bb.y, 0.f);
    v.z = fmaxf(v.z + bb.z, 0.f);
    v.w = fmaxf(v.w + bb.w, 0.f);
    reinterpret_cast<float4*>(x)[i] = v;
  }
}

// One block per sample (256 threads = 16 channel quads x 16 pool cells; C = 64): y = relu(x +
// b) in place over the sample's R x W positions, and feat[s][c * 16 + cell] = the cell's
// window sum / its area (the flatten order of [C][4][4]).
template <int C>
__global__ __launch_bounds__(256) void bias_relu_pool_kernel(float* __restrict__ x, const float* __restrict__ b,
                                                              int R, int W, float* __restrict__ feat) {
  static_assert(C == 64, "16 channel quads x 16 cells");
  const int s = blockIdx.x, t = threadIdx.x, q = t & 15, cell = t >> 4, cy = cell >> 2, cx = cell & 3;
  const int y0 = win_start(cy, R), y1 = win_end(cy, R), x0 = win_start(cx, W), x1 = win_end(cx, W);
  const float4 bb = reinterpret_cast<const float4*>(b)[q];
  float4* xs = reinterpret_cast<float4*>(x + (size_t)s * R * W * C);
  float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
  if ((R & 3) == 0 && (W & 3) == 0) {  // disjoint windows: each position's one cell transforms and sums it
    for (int y = y0; y < y1; ++y)
      for (int xx = x0; xx < x1; ++xx) {
        const int i = (y * W + xx) * (C / 4) + q;
        float4 v = xs[i];
        v.x = fmaxf(v.x + bb.x, 0.f);
        v.y = fmaxf(v.y + bb.y, 0.f);
        v.z = fmaxf(v.z + bb.z, 0.f);
        v.w = fmaxf(v.w + bb.w, 0.f);
        xs[i] = v;
        sum.x += v.x;
        sum.y += v.y;
        sum.z += v.z;
        sum.w += v.w;
      }
  } else {  // overlapping windows (R % 4 != 0): transform every position once, then sum the windows
    for (int p = t >> 4; p < R * W; p += 16) {
      float4 v = xs[p * (C / 4) + q];
      v.x = fmaxf(v.x + bb.x, 0.f);
      v.y = fmaxf(v.y + bb.y, 0.f);
      v.z = fmaxf(v.z + bb.z, 0.f);
      v.w = fmaxf(v.w + bb.w, 0.f);
      xs[p * (C / 4) + q] = v;
    }
    __syncthreads();  // the block's global stores are visible to the block after the barrier
    for (int y = y0; y < y1; ++y)
      for (int xx = x0; xx < x1; ++xx) {
        const float4 v = xs[(y * W + xx) * (C / 4) + q];
        sum.x += v.x;
        sum.y += v.y;
        sum.z += v.z;
        sum.w += v.w;
      }
  }
  const float area = (float)((y1 - y0) * (x1 - x0));
  float* f = feat + (size_t)s * C * 16 + (4 * q) * 16 + cell;
  f[0] = sum.x / area;
  f[16] = sum.y / area;
  f[32] = sum.z / area;
  f[48] = sum.w / area;
}

// Backward of relu(conv3 + b3) -> pool for one sample per block (the same thread mapping):
// d[pos][c] = (y > 0) ? dfeat[c * 16 + cell] / area : 0, summed over every cell holding pos
// (overlapping windows, R % 4 != 0); written to d (a separate tensor: it becomes conv3's
// grad_output), and the sample's bias-gradient partial part[s][c] = sum over positions of d.
// R, W multiples of 4: thread (quad q, cell) owns the cell's positions; otherwise thread
// (quad q, lane l) owns positions l, l + 16, ... and a position's gradient adds its cells in
// cell order.
template <int C>
__global__ __launch_bounds__(256) void pool_relu_bwd_kernel(const float* __restrict__ dfeat,
                                                             const float* __restrict__ y, int R, int W,
                                                             float* __restrict__ d, float* __restrict__ part) {
  static_assert(C == 64, "16 channel quads x 16 cells");
  __shared__ float4 red[256];
  const int s = blockIdx.x, t = threadIdx.x, q = t & 15;
  const float4* ys = reinterpret_cast<const float4*>(y + (size_t)s * R * W * C);
  float4* ds = reinterpret_cast<float4*>(d + (size_t)s * R * W * C);
  const float* fg = dfeat + (size_t)s * C * 16;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if ((R & 3) == 0 && (W & 3) == 0) {
    // disjoint windows: thread (quad q, cell) owns its cell's positions, whose gradient is the
    // cell's pooled gradient / area (torch's adaptive_avg_pool2d backward)
    const int cell = t >> 4, cy = cell >> 2, cx = cell & 3, kh = R >> 2, kw = W >> 2;
    const float area = (float)(kh * kw);
    const float4 g = make_float4(fg[(4 * q) * 16 + cell] / area, fg[(4 * q + 1) * 16 + cell] / area,
                                 fg[(4 * q + 2) * 16 + cell] / area, fg[(4 * q + 3) * 16 + cell] / area);
    for (int y = cy * kh; y < (cy + 1) * kh; ++y)
      for (int x = cx * kw; x < (cx + 1) * kw; ++x) {
        const int i = (y * W + x) * (C / 4) + q;
        const float4 v = ys[i];
        const float4 o = make_float4(v.x > 0.f ? g.x : 0.f, v.y > 0.f ? g.y : 0.f, v.z > 0.f ? g.z : 0.f,
                                     v.w > 0.f ? g.w : 0.f);
        ds[i] = o;
        acc.x += o.x;
        acc.y += o.y;
        acc.z += o.z;
        acc.w += o.w;
      }
  } else
  // overlapping windows: positions p = t >> 4, + 16, ...: every position once, its gradient
  // the sum of the cells whose windows hold it
  for (int p = t >> 4; p < R * W; p += 16) {
    const int py = p / W, px = p - py * W;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int cy = 0; cy < 4; ++cy) {
      const int y0 = win_start(cy, R), y1 = win_end(cy, R);
      if (py < y0 || py >= y1) continue;
      for (int cx = 0; cx < 4; ++cx) {
        const int x0 = win_start(cx, W), x1 = win_end(cx, W);
        if (px < x0 || px >= x1) continue;
        const float area = (float)((y1 - y0) * (x1 - x0));
        const int cell = cy * 4 + cx;
        g.x += fg[(4 * q) * 16 + cell] / area;
        g.y += fg[(4 * q + 1) * 16 + cell] / area;
        g.z += fg[(4 * q + 2) * 16 + cell] / area;
        g.w += fg[(4 * q + 3) * 16 + cell] / area;
      }
    }
    const float4 v = ys[p * (C / 4) + q];
    const float4 o = make_float4(v.x > 0.f ? g.x : 0.f, v.y > 0.f ? g.y : 0.f, v.z > 0.f ? g.z : 0.f,
                                 v.w > 0.f ? g.w : 0.f);
    ds[p * (C / 4) + q] = o;
    acc.x += o.x;
    acc.y += o.y;
    acc.z += o.z;
    acc.w += o.w;
  }
  red[t] = acc;
  __syncthreads();
  if (t < 16) {  // the 16 position lanes of quad t, in order
    float4 a = red[t];
    for (int k = 1; k < 16; ++k) {
      const float4 r = red[t + 16 * k];
      a.x += r.x;
      a.y += r.y;
      a.z += r.z;
      a.w += r.w;
    }
    reinterpret_cast<float4*>(part + (size_t)s * C)[t] = a;
  }
}

// ReLU backward in place, g = (y > 0) ? g : 0 over one sample per block (256 threads = C/4
// channel quads x 256/(C/4) position lanes), and the sample's bias-gradient partial.
template <int C>
__global__ __launch_bounds__(256) void relu_bwd_kernel(float* __restrict__ g, const float* __restrict__ y, int P,
                                                        float* __restrict__ part) {
  constexpr int NQ = C / 4, NL = 256 / NQ;
  __shared__ float4 red[256];
  const int s = blockIdx.x, t = threadIdx.x, q = t % NQ, l = t / NQ;
  float4* gs = reinterpret_cast<float4*>(g + (size_t)s * P * C);
  const float4* ys = reinterpret_cast<const float4*>(y + (size_t)s * P * C);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int p = l; p < P; p += NL) {
    const float4 v = ys[p * NQ + q];
    float4 o = gs[p * NQ + q];
    o.x = v.x > 0.f ? o.x : 0.f;
    o.y = v.y > 0.f ? o.y : 0.f;
    o.z = v.z > 0.f ? o.z : 0.f;
    o.w = v.w > 0.f ? o.w : 0.f;
    gs[p * NQ + q] = o;
    acc.x += o.x;
    acc.y += o.y;
    acc.z += o.z;
    acc.w += o.w;
  }
  red[t] = acc;
  __syncthreads();
  if (t < NQ) {
    float4 a = red[t];
    for (int k = 1; k < NL; ++k) {
      const float4 r = red[t + NQ * k];
      a.x += r.x;
      a.y += r.y;
      a.z += r.z;
      a.w += r.w;
    }
    reinterpret_cast<float4*>(part + (size_t)s * C)[t] = a;
  }
}

// db[c] = sum over samples of part[s][c], one block per channel: thread t sums samples t,
// t + 256, ... in order, then a fixed tree over the 256 threads.
__global__ __launch_bounds__(256) void bias_grad_reduce_kernel(const float* __restrict__ part, int n, int C,
                                                                float* __restrict__ db) {
  __shared__ float red[256];
  const int c = blockIdx.x, t = threadIdx.x;
  float a = 0.f;
  for (int s = t; s < n; s += 256) a += part[(size_t)s * C + c];
  red[t] = a;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (t == 0) db[c] = red[0];
}

}  // namespace tr

hipError_t launch_bias_relu(float* x, const float* b, int64_t n_pos, int C, hipStream_t st) {
  const int64_t n4 = n_pos * C / 4;
  const int64_t blocks = (n4 + 255) / 256;
  hipLaunchKernelGGL(tr::bias_relu_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, st, x, b,
                     n4, C / 4);
  return hipGetLastError();
}

hipError_t launch_bias_relu_pool(float* x, const float* b, int n, int R, int W, int C, float* feat, hipStream_t st) {
  if (C != 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tr::bias_relu_pool_kernel<64>, dim3(n), dim3(256), 0, st, x, b, R, W, feat);
  return hipGetLastError();
}

hipError_t launch_pool_relu_bwd(const float* dfeat, const float* y, int n, int R, int W, int C, float* d, float* part,
                                float* db, hipStream_t st) {
  if (C != 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tr::pool_relu_bwd_kernel<64>, dim3(n), dim3(256), 0, st, dfeat, y, R, W, d, part);
  hipLaunchKernelGGL(tr::bias_grad_reduce_kernel, dim3(C), dim3(256), 0, st, part, n, C, db);
  return hipGetLastError();
}

hipError_t launch_relu_bwd(float* g, const float* y, int n, int P, int C, float* part, float* db, hipStream_t st) {
  if (C == 64)
    hipLaunchKernelGGL(tr::relu_bwd_kernel<64>, dim3(n), dim3(256), 0, st, g, y, P, part);
  else if (C == 32)
    hipLaunchKernelGGL(tr::relu_bwd_kernel<32>, dim3(n), dim3(256), 0, st, g, y, P, part);
  else
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(tr::bias_grad_reduce_kernel, dim3(C), dim3(256), 0, st, part, n, C, db);
  return hipGetLastError();
}

}  // namespace heist
