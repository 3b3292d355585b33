// heist_arch.hip -- Architect layout decode on the GPU (networks.py:283-335).
//
// Turns per-cell sampled asset classes {0 none, 1 wall, 2 camera, 3 guard} into the
// heist_set_layout input arrays, so a batch of Architect samples reaches the
// environment without a host round trip.  The decode is a greedy row-major scan with
// a running budget -- inherently sequential per layout -- so one lane owns one layout;
// the interior of a layout row is read as a contiguous run (the map is [N][R][C]).
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace heist {

__global__ __launch_bounds__(64) void arch_decode_kernel(
    const int64_t* __restrict__ amap, int n, int R, int C, const float* __restrict__ cam, int cam_stride,
    const int32_t* __restrict__ budget, int allow_cams, int allow_guards, int max_walls, int max_cams, int max_guards,
    int max_path, int32_t* __restrict__ wall_rc, int32_t* __restrict__ n_walls, double* __restrict__ cam_out,
    int32_t* __restrict__ n_cams, int32_t* __restrict__ guard_paths, int32_t* __restrict__ guard_meta,
    double* __restrict__ guard_fov, int32_t* __restrict__ n_guards) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int64_t* m = amap + (size_t)e * R * C;
  const float* cp = cam + (size_t)e * cam_stride;
  // cam_params["fov"/"speed"/"heading"].item(): float32 values seen as Python floats
  const double fov = (double)cp[0], speed = (double)cp[1], heading = (double)cp[2];
  int remaining = budget[e];
  int nw = 0, nc = 0, ng = 0;
  for (int r = 1; r < R - 1 && remaining > 0; ++r) {
    for (int c = 1; c < C - 1; ++c) {
      const int64_t t = m[r * C + c];
      if (t == 0) continue;
      if (t == 1 && remaining >= 1) {  // BUDGET_COSTS["wall"]
        if (nw < max_walls) {
          wall_rc[((size_t)e * max_walls + nw) * 2] = r;
          wall_rc[((size_t)e * max_walls + nw) * 2 + 1] = c;
        }
        ++nw;
        remaining -= 1;
      } else if (t == 2 && remaining >= 3) {  // camera, vision_range 6
        if (nc < max_cams) {
          double* o = cam_out + ((size_t)e * max_cams + nc) * 6;
          o[0] = r; o[1] = c; o[2] = fov; o[3] = heading; o[4] = speed; o[5] = 6.0;
        }
        ++nc;
        remaining -= 3;
      } else if (t == 3 && remaining >= 5) {  // guard: 8-point rectangle patrol (networks.py:324-335)
        if (ng < max_guards) {
          int32_t* pth = guard_paths + ((size_t)e * max_guards + ng) * max_path * 2;
          const int offs[8][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 2}, {2, 2}, {2, 1}, {2, 0}, {1, 0}};
          for (int k = 0; k < 8 && k < max_path; ++k) {
            pth[2 * k] = max(1, min(R - 2, r + offs[k][0] - 1));
            pth[2 * k + 1] = max(1, min(C - 2, c + offs[k][1] - 1));
          }
          int32_t* gm = guard_meta + ((size_t)e * max_guards + ng) * 3;
          gm[0] = 8 < max_path ? 8 : max_path;
          gm[1] = 1;  // speed
          gm[2] = 4;  // vision_range
          guard_fov[(size_t)e * max_guards + ng] = 90.0;
        }
        ++ng;
        remaining -= 5;
      }
      if (remaining <= 0) break;  // networks.py:315-318
    }
  }
  n_walls[e] = nw < max_walls ? nw : max_walls;
  n_cams[e] = allow_cams ? (nc < max_cams ? nc : max_cams) : 0;     // training.py:464-467 curriculum filter
  n_guards[e] = allow_guards ? (ng < max_guards ? ng : max_guards) : 0;
}

hipError_t launch_arch_decode(const int64_t* amap, int n, int R, int C, const float* cam, int cam_stride,
                              const int32_t* budget, int allow_cams, int allow_guards, int max_walls, int max_cams,
                              int max_guards, int max_path, int32_t* wall_rc, int32_t* n_walls, double* cam_out,
                              int32_t* n_cams, int32_t* guard_paths, int32_t* guard_meta, double* guard_fov,
                              int32_t* n_guards, hipStream_t st) {
  hipLaunchKernelGGL(arch_decode_kernel, dim3((n + 63) / 64), dim3(64), 0, st, amap, n, R, C, cam, cam_stride, budget,
                     allow_cams, allow_guards, max_walls, max_cams, max_guards, max_path, wall_rc, n_walls, cam_out,
                     n_cams, guard_paths, guard_meta, guard_fov, n_guards);
  return hipGetLastError();
}

}  // namespace heist
