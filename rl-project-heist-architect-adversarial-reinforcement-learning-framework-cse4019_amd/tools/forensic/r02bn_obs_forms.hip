#include <hip/hip_runtime.h>
#include <stdint.h>
// Forensic reconstruction of the round-2 "batched-load" split observation write
// (both passes' loads issued before either store), NT = 256 threads (4 waves), PW = 192.
struct P { const uint8_t* grid; const float* plane0; int RC; float vault_val; int qv; };
__device__ __forceinline__ void put(float* o, int off, float4 v) { *reinterpret_cast<float4*>(o + off) = v; }
template <int NT, int FORM>
__global__ __launch_bounds__(NT) void obs_static(P p, float* __restrict__ obs) {
  constexpr int PW = NT - 64;
  const int t = (int)threadIdx.x - 64;
  if (t < 0) return;
  const int e = blockIdx.x, RC = p.RC, n4 = RC / 4;
  const uint32_t* s4 = reinterpret_cast<const uint32_t*>(p.grid + (size_t)e * RC);
  const float4* pl = reinterpret_cast<const float4*>(p.plane0);
  float* o = obs + (size_t)e * 3 * RC;
  for (int q = t; q < n4; q += 2 * PW) {
    const int q1 = q + PW;
    uint32_t b0 = s4[q], b1 = 0;
    float4 v0 = pl[q], v1 = make_float4(0, 0, 0, 0);
    if (FORM == 0) {            // guarded second pass
      if (q1 < n4) { b1 = s4[q1]; v1 = pl[q1]; }
    } else {                    // unguarded second-pass loads (stores guarded)
      b1 = s4[q1]; v1 = pl[q1];
    }
    put(o, 4 * q, make_float4((float)(b0 & 0xff), (float)(b0 >> 24), 0, 0));
    put(o, 4 * (2 * n4 + q), v0);
    if (q1 < n4) {
      put(o, 4 * q1, make_float4((float)(b1 & 0xff), (float)(b1 >> 24), 0, 0));
      put(o, 4 * (2 * n4 + q1), v1);
    }
  }
}
template __global__ void obs_static<256, 0>(P, float*);
template __global__ void obs_static<256, 1>(P, float*);
