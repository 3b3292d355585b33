// heist_ppo.hip -- GAE scan, advantage normalisation and the fused clipped-PPO loss.
//
// All three are HBM-bound elementwise/reduction work (no contraction): one thread per
// env column for the reverse GAE scan ([T][N] layout, coalesced over N), grid-stride
// float64 reductions for the advantage moments, and one thread per sample row for the
// loss with per-block float64 partials reduced in a fixed order (deterministic).
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace heist {

constexpr int kMaxActions = 16;

// SolverAgent._compute_gae (agents/solver.py:228-244) per column, with torch's float32
// op order: delta = (r + (g*nv)*(1-d)) - v;  A = delta + (gl*(1-d))*A.
__global__ __launch_bounds__(256) void gae_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                   const uint8_t* __restrict__ d, const float* __restrict__ last_value,
                                                   int T, int N, float g, float gl, float* __restrict__ adv,
                                                   float* __restrict__ ret) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float nv = last_value ? last_value[n] : 0.0f;
  float A = 0.0f;
  constexpr int U = 4;  // keep U timesteps of loads in flight ahead of the dependent scan
  int t = T - 1;
  for (; t >= U - 1; t -= U) {
    float rr[U], vv[U], nd[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = (size_t)(t - u) * N + n;
      rr[u] = r[i];
      vv[u] = v[i];
      nd[u] = 1.0f - (float)d[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = (size_t)(t - u) * N + n;
      const float delta = (rr[u] + (g * nv) * nd[u]) - vv[u];
      A = delta + (gl * nd[u]) * A;
      adv[i] = A;
      ret[i] = A + vv[u];
      nv = vv[u];
    }
  }
  for (; t >= 0; --t) {
    const size_t i = (size_t)t * N + n;
    const float vt = v[i];
    const float ndt = 1.0f - (float)d[i];
    const float delta = (r[i] + (g * nv) * ndt) - vt;
    A = delta + (gl * ndt) * A;
    adv[i] = A;
    ret[i] = A + vt;
    nv = vt;
  }
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}

// Block-level sum of `x` into lane 0 of wave 0 (blockDim.x == 256).
__device__ __forceinline__ double block_sum(double x, double* sh) {
  x = wave_sum(x);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = x;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += sh[k];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(256) void adv_moments_kernel(const float* __restrict__ x, int64_t n, int phase,
                                                           double* __restrict__ acc) {
  __shared__ double sh[4];
  const double mean = phase == 0 ? 0.0 : acc[0] / acc[1];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = (double)x[i];
    s += phase == 0 ? v : (v - mean) * (v - mean);
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    if (phase == 0) {
      atomicAdd(acc + 0, s);
      if (blockIdx.x == 0) atomicAdd(acc + 1, (double)n);
    } else {
      atomicAdd(acc + 2, s);
    }
  }
}

// (x - mean) / (std + eps) in float32 (agents/solver.py:146-147); count <= 1 -> unchanged.
__global__ __launch_bounds__(256) void adv_apply_kernel(float* __restrict__ x, int64_t n, const double* __restrict__ acc,
                                                         float eps) {
  const double cnt = acc[1];
  if (cnt <= 1.0) return;
  const float mean = (float)(acc[0] / cnt);
  const float stdv = (float)sqrt(acc[2] / (cnt - 1.0));
  const float den = stdv + eps;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = (x[i] - mean) / den;
}

// Fused clipped-PPO loss forward + backward (agents/solver.py:172-193), one row per thread.
// Categorical(probs=softmax(logits)): probs are renormalised, log-probs are
// log(clamp(p, eps, 1-eps)), entropy = -sum p * logp; torch.min splits tie gradients.
__global__ __launch_bounds__(256) void ppo_loss_kernel(const float* __restrict__ logits, const float* __restrict__ values,
                                                        const int64_t* __restrict__ actions,
                                                        const float* __restrict__ old_logp, const float* __restrict__ adv,
                                                        const float* __restrict__ ret, int M, int A, float lo, float hi,
                                                        float vcoef_over_m2, float ecoef_over_m, float inv_m,
                                                        float* __restrict__ dlogits, float* __restrict__ dvalues,
                                                        double* __restrict__ partials) {
  __shared__ double sh[4];
  const float eps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  double pg = 0.0, vl = 0.0, ent_acc = 0.0;
  if (i < M) {
    float x[kMaxActions], p[kMaxActions], lc[kMaxActions];
    const float* row = logits + (size_t)i * A;
    float mx = row[0];
    for (int j = 0; j < A; ++j) {
      x[j] = row[j];
      mx = fmaxf(mx, x[j]);
    }
    float s = 0.0f;
    for (int j = 0; j < A; ++j) {
      p[j] = expf(x[j] - mx);
      s += p[j];
    }
    for (int j = 0; j < A; ++j) p[j] = p[j] / s;  // F.softmax
    float S = 0.0f;
    for (int j = 0; j < A; ++j) S += p[j];
    float ent = 0.0f;
    float pn[kMaxActions];
    for (int j = 0; j < A; ++j) {
      pn[j] = p[j] / S;  // Categorical(probs) normalisation
      const float c = fminf(fmaxf(pn[j], eps), 1.0f - eps);
      lc[j] = logf(c);
      ent -= pn[j] * lc[j];
    }
    const int a = min(max((int)actions[i], 0), A - 1);
    const float av = adv[i];
    const float ratio = expf(lc[a] - old_logp[i]);
    const float s1 = ratio * av;
    const float rc = fminf(fmaxf(ratio, lo), hi);
    const float s2 = rc * av;
    pg = (double)fminf(s1, s2);
    const float dv = values[i] - ret[i];
    vl = (double)dv * (double)dv;
    ent_acc = (double)ent;
    // backward
    const bool in_clip = ratio >= lo && ratio <= hi;
    const float clip_grad = in_clip ? av : 0.0f;
    const float dmin = s1 < s2 ? av : (s2 < s1 ? clip_grad : 0.5f * av + 0.5f * clip_grad);
    const float g_logp = -(dmin * ratio) * inv_m;
    float gpn_dot_p = 0.0f;
    float gpn[kMaxActions];
    for (int j = 0; j < A; ++j) {
      const bool unclamped = pn[j] >= eps && pn[j] <= 1.0f - eps;
      float gj = ecoef_over_m * (lc[j] + (unclamped ? 1.0f : 0.0f));
      if (j == a && unclamped) gj += g_logp / pn[j];
      gpn[j] = gj;
      gpn_dot_p += gj * p[j];
    }
    float gp_dot = 0.0f;
    for (int j = 0; j < A; ++j) {
      gpn[j] = gpn[j] / S - gpn_dot_p / (S * S);  // through p / sum(p)
      gp_dot += gpn[j] * p[j];
    }
    float* drow = dlogits + (size_t)i * A;
    for (int j = 0; j < A; ++j) drow[j] = p[j] * (gpn[j] - gp_dot);  // through softmax
    dvalues[i] = vcoef_over_m2 * dv;
  }
  pg = block_sum(pg, sh);
  vl = block_sum(vl, sh);
  ent_acc = block_sum(ent_acc, sh);
  if (threadIdx.x == 0) {
    partials[blockIdx.x * 3 + 0] = pg;
    partials[blockIdx.x * 3 + 1] = vl;
    partials[blockIdx.x * 3 + 2] = ent_acc;
  }
}

__global__ void ppo_finalize_kernel(const double* __restrict__ partials, int nblocks, int M, float vcoef, float ecoef,
                                    float* __restrict__ parts) {
  if (threadIdx.x != 0) return;
  double pg = 0.0, vl = 0.0, en = 0.0;
  for (int b = 0; b < nblocks; ++b) {
    pg += partials[b * 3];
    vl += partials[b * 3 + 1];
    en += partials[b * 3 + 2];
  }
  const float fpg = (float)(-pg / M), fvl = (float)(vl / M), fen = (float)(en / M);
  parts[0] = fpg + vcoef * fvl - ecoef * fen;
  parts[1] = fpg;
  parts[2] = fvl;
  parts[3] = fen;
}

// ---------------------------------------------------------------------------

// The rollout's per-tick attempt bookkeeping (training.py:515-544: steps and reward of the
// running attempt, its outcome when it ends, the fresh LSTM state of the next one), one thread
// per (env, hidden slot): slot 0 also does the env's counters.  The same arithmetic as the
// torch expressions it replaces (heist_amd/training.py _rollout): counting = valid and
// attempts < A; reward += (counting ? r : 0.0) in float64; an ended attempt counts by status;
// h, c *= (done ? 0 : 1) as float multiplies (negative values become -0.0, as torch's do).
__global__ __launch_bounds__(256) void rollout_tally_kernel(const uint8_t* __restrict__ valid, int32_t* __restrict__ attempts,
                                                            int A, const uint8_t* __restrict__ done,
                                                            const int8_t* __restrict__ status,
                                                            const double* __restrict__ reward64, int32_t* __restrict__ steps,
                                                            double* __restrict__ reward_sum, int32_t* __restrict__ solve,
                                                            int32_t* __restrict__ detect, int32_t* __restrict__ timeout,
                                                            float* __restrict__ h, float* __restrict__ c, int hidden, int n,
                                                            int vault, int det) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)n * hidden) return;
  const int e = (int)(i / hidden), k = (int)(i - (int64_t)e * hidden);
  const bool d = done[e] != 0;
  const float keep = d ? 0.f : 1.f;
  h[(int64_t)e * hidden + k] = h[(int64_t)e * hidden + k] * keep;
  c[(int64_t)e * hidden + k] = c[(int64_t)e * hidden + k] * keep;
  if (k != 0) return;
  const bool counting = valid[e] != 0 && attempts[e] < A;
  steps[e] += counting ? 1 : 0;
  reward_sum[e] = reward_sum[e] + (counting ? reward64[e] : 0.0);
  const bool fin = counting && d;
  const int st = (int)status[e];
  solve[e] += (fin && st == vault) ? 1 : 0;
  detect[e] += (fin && st == det) ? 1 : 0;
  timeout[e] += (fin && st != vault && st != det) ? 1 : 0;
  attempts[e] += fin ? 1 : 0;
}

hipError_t launch_rollout_tally(const uint8_t* valid, int32_t* attempts, int A, const uint8_t* done, const int8_t* status,
                                const double* reward64, int32_t* steps, double* reward_sum, int32_t* solve,
                                int32_t* detect, int32_t* timeout, float* h, float* c, int hidden, int n, int vault,
                                int det, hipStream_t st) {
  const int64_t total = (int64_t)n * hidden;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(rollout_tally_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, valid, attempts, A,
                     done, status, reward64, steps, reward_sum, solve, detect, timeout, h, c, hidden, n, vault, det);
  return hipGetLastError();
}

// The Solver's LSTM cell after its two gate GEMMs (networks.py:90-100 nn.LSTM, one time step,
// gate order i, f, g, o), one thread per (row, hidden unit): gates = gx + gh, then
// c1 = sigmoid(f) c + sigmoid(i) tanh(g), h1 = sigmoid(o) tanh(c1) -- each product and sum
// rounded to fp32 as the ten torch kernels it replaces round them (sigmoid as 1 / (1 + exp(-x)),
// torch's form), so the result is theirs bit for bit.
__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }
__global__ __launch_bounds__(256) void lstm_cell_kernel(const float* __restrict__ gx, const float* __restrict__ gh,
                                                        const float* __restrict__ c, float* __restrict__ h1,
                                                        float* __restrict__ c1, int H, int n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)n * H) return;
  const int64_t b = i / H;
  const int j = (int)(i - b * H);
  const float* x = gx + b * 4 * H;
  const float* y = gh + b * 4 * H;
  const float gi = x[j] + y[j], gf = x[H + j] + y[H + j], gg = x[2 * H + j] + y[2 * H + j],
              go = x[3 * H + j] + y[3 * H + j];
  const float t1 = sigmoid_f(gf) * c[i];
  const float t2 = sigmoid_f(gi) * tanhf(gg);
  const float cc = t1 + t2;
  c1[i] = cc;
  h1[i] = sigmoid_f(go) * tanhf(cc);
}

hipError_t launch_lstm_cell(const float* gx, const float* gh, const float* c, float* h1, float* c1, int H, int n,
                            hipStream_t st) {
  const int64_t total = (int64_t)n * H;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(lstm_cell_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, gx, gh, c, h1, c1, H, n);
  return hipGetLastError();
}

hipError_t launch_gae(const float* r, const float* v, const uint8_t* d, const float* last_value, int T, int N,
                      double gamma, double lam, float* adv, float* ret, hipStream_t st) {
  const float g = (float)gamma, gl = (float)(gamma * lam);
  hipLaunchKernelGGL(gae_kernel, dim3((N + 255) / 256), dim3(256), 0, st, r, v, d, last_value, T, N, g, gl, adv, ret);
  return hipGetLastError();
}

static int reduce_blocks(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

hipError_t launch_adv_moments(const float* x, int64_t n, int phase, double* acc, hipStream_t st) {
  hipLaunchKernelGGL(adv_moments_kernel, dim3(reduce_blocks(n)), dim3(256), 0, st, x, n, phase, acc);
  return hipGetLastError();
}

hipError_t launch_adv_apply(float* x, int64_t n, const double* acc, float eps, hipStream_t st) {
  hipLaunchKernelGGL(adv_apply_kernel, dim3(reduce_blocks(n)), dim3(256), 0, st, x, n, acc, eps);
  return hipGetLastError();
}

hipError_t launch_ppo_loss(const float* logits, const float* values, const int64_t* actions, const float* old_logp,
                           const float* adv, const float* ret, int M, int A, double clip, double vcoef, double ecoef,
                           float* parts, float* dlogits, float* dvalues, double* scratch, hipStream_t st) {
  const int nb = (M + 255) / 256;
  const float lo = (float)(1.0 - clip), hi = (float)(1.0 + clip);
  hipLaunchKernelGGL(ppo_loss_kernel, dim3(nb), dim3(256), 0, st, logits, values, actions, old_logp, adv, ret, M, A,
                     lo, hi, (float)(vcoef * 2.0 / M), (float)(ecoef / M), 1.0f / (float)M, dlogits, dvalues, scratch);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(ppo_finalize_kernel, dim3(1), dim3(64), 0, st, scratch, nb, M, (float)vcoef, (float)ecoef, parts);
  return hipGetLastError();
}

}  // namespace heist
