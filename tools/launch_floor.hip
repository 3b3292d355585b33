// Launch / dispatch floor of the step kernel's grid shape on MI355X: an empty kernel (or
// one that reads one global int per block, as step_kernel reads order[b]) at various
// block counts, block sizes and dynamic LDS sizes, timed with HIP events over 200
// launches.  Build: hipcc -O3 --offload-arch=gfx950 tools/launch_floor.hip -o /tmp/lf
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void empty_kernel(int* out) {
  extern __shared__ int smem[];
  if (threadIdx.x == 1023) out[0] = smem[0];  // never true for <= 256 threads
}

__global__ void read_kernel(const int* __restrict__ order, int* out) {
  const int e = order[blockIdx.x];
  if (e < 0) out[0] = e;  // never
}

// persistent: each block walks k envs, reading order[] per env
__global__ void persist_kernel(const int* __restrict__ order, int n, int* out) {
  int acc = 0;
  for (int b = blockIdx.x; b < n; b += gridDim.x) acc += order[b];
  if (acc < 0) out[0] = acc;
}

int main() {
  int* order;
  int* out;
  hipMalloc(&order, 1 << 20);
  hipMalloc(&out, 64);
  hipMemset(order, 0, 1 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks[] = {1024, 2048, 4096, 8192};
  const int threads[] = {64, 128, 256};
  const int lds[] = {0, 9216, 16384};
  for (int kind = 0; kind < 2; ++kind)
    for (int nb : blocks)
      for (int nt : threads)
        for (int l : lds) {
          for (int it = 0; it < 20; ++it) {
            if (kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(nb), dim3(nt), l, 0, out);
            else hipLaunchKernelGGL(read_kernel, dim3(nb), dim3(nt), l, 0, order, out);
          }
          hipEventRecord(a, 0);
          for (int it = 0; it < 200; ++it) {
            if (kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(nb), dim3(nt), l, 0, out);
            else hipLaunchKernelGGL(read_kernel, dim3(nb), dim3(nt), l, 0, order, out);
          }
          hipEventRecord(b, 0);
          hipEventSynchronize(b);
          float ms;
          hipEventElapsedTime(&ms, a, b);
          printf("{\"kernel\": \"%s\", \"blocks\": %d, \"threads\": %d, \"lds\": %d, \"us\": %.2f}\n",
                 kind ? "read_order" : "empty", nb, nt, l, ms * 1000.0f / 200.0f);
        }
  for (int nb : {256, 512, 1024, 2048}) {
    hipEventRecord(a, 0);
    for (int it = 0; it < 200; ++it) hipLaunchKernelGGL(persist_kernel, dim3(nb), dim3(256), 9216, 0, order, 4096, out);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"kernel\": \"persist_4096\", \"blocks\": %d, \"threads\": 256, \"lds\": 9216, \"us\": %.2f}\n", nb,
           ms * 1000.0f / 200.0f);
  }
  return 0;
}
