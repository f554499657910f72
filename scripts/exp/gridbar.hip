// Experiment (not product code): cost of a device-wide barrier inside a persistent kernel on MI355X, with the
// cross-XCD visibility a decoder megakernel would need (each block writes a slot, after the barrier reads a
// slot written by a block on another XCD).
//   hipcc --offload-arch=gfx950 -O3 scripts/exp/gridbar.hip -o scripts/exp/gridbar && ./scripts/exp/gridbar
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ inline void grid_barrier(unsigned* counter, unsigned nblocks, unsigned& target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    target += nblocks;
    __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    while (__hip_atomic_load(counter, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
}

__global__ void k_bar(unsigned* counter, int* slots, int iters, int* errors) {
  unsigned target = 0;
  const int nb = gridDim.x, b = blockIdx.x;
  for (int it = 0; it < iters; ++it) {
    if (threadIdx.x == 0) slots[(it & 1) * nb + b] = it * 1000 + b;
    grid_barrier(counter, nb, target);
    if (threadIdx.x == 0) {
      const int o = (b + 37) % nb;
      if (slots[(it & 1) * nb + o] != it * 1000 + o) atomicAdd(errors, 1);
    }
  }
}

__global__ void k_empty(int* x) {
  if (threadIdx.x == 0 && x[blockIdx.x] == 12345) x[blockIdx.x] = 0;
}

int main() {
  unsigned* counter;
  int *slots, *errors;
  hipMalloc(&counter, 4);
  hipMalloc(&slots, 4096 * 4);
  hipMalloc(&errors, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int nb : {64, 128, 256}) {
    for (int threads : {256, 512}) {
      const int iters = 2000;
      hipMemset(counter, 0, 4);
      hipMemset(errors, 0, 4);
      hipLaunchKernelGGL(k_bar, dim3(nb), dim3(threads), 0, 0, counter, slots, 10, errors);  // warm
      hipDeviceSynchronize();
      hipMemset(counter, 0, 4);
      hipEventRecord(a);
      hipLaunchKernelGGL(k_bar, dim3(nb), dim3(threads), 0, 0, counter, slots, iters, errors);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      int err;
      hipMemcpy(&err, errors, 4, hipMemcpyDeviceToHost);
      printf("blocks %3d x %3d threads: %.2f us per barrier, %d visibility errors\n", nb, threads, ms * 1000 / iters, err);
    }
  }
  // kernel-boundary cost for comparison: back-to-back empty kernels in a graph
  hipStream_t s;
  hipStreamCreate(&s);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, slots);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEventRecord(a, s);
  hipGraphLaunch(ge, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("graph of empty 256-block kernels: %.2f us per kernel\n", ms * 1000 / 200);
  return 0;
}
