// Probe (not product code): does streaming a large buffer evict a smaller table from the 256 MiB Infinity Cache,
// by the buffer's allocation flavour (default / hipDeviceMallocUncached / fine-grained) and load policy (plain / nt)?
// And at what rate does each flavour stream? Prints one line per case.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mall_probe scripts/exp/mall_probe.hip && /tmp/mall_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const f32x4* __restrict__ p, long n, float* out) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * 4) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long j = i + u * stride;
      if (j < n) v[u] = NT ? __builtin_nontemporal_load(p + j) : p[j];
      else v[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u];
  }
  const float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 12345.678f) out[0] = s;  // keeps the loads
}

static float time_read(const void* p, size_t bytes, bool nt, float* out, hipEvent_t a, hipEvent_t b) {
  const long n = (long)(bytes / 16);
  CK(hipEventRecord(a));
  if (nt) hipLaunchKernelGGL(k_read<true>, dim3(2048), dim3(256), 0, 0, (const f32x4*)p, n, out);
  else hipLaunchKernelGGL(k_read<false>, dim3(2048), dim3(256), 0, 0, (const f32x4*)p, n, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f;  // us
}

int main() {
  const size_t TBL = 150ull << 20, STR = 800ull << 20;
  float* out;
  CK(hipMalloc(&out, 64));
  void* tbl;
  CK(hipMalloc(&tbl, TBL));
  CK(hipMemset(tbl, 0, TBL));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[3] = {"default", "uncached", "finegrained"};
  const unsigned flags[3] = {hipDeviceMallocDefault, hipDeviceMallocUncached, hipDeviceMallocFinegrained};
  for (int f = 0; f < 3; ++f) {
    void* str;
    CK(hipExtMallocWithFlags(&str, STR, flags[f]));
    CK(hipMemset(str, 0, STR));
    CK(hipDeviceSynchronize());
    for (int nt = 0; nt < 2; ++nt) {
      for (int rep = 0; rep < 2; ++rep) {
        time_read(tbl, TBL, false, out, a, b);
        const float t_warm = time_read(tbl, TBL, false, out, a, b);  // table re-read right away
        const float t_str = time_read(str, STR, nt, out, a, b);       // the stream
        const float t_after = time_read(tbl, TBL, false, out, a, b);  // table after the stream
        printf("%-12s nt=%d  stream %.1f us = %.2f TB/s | table warm %.1f us (%.2f TB/s), after stream %.1f us "
               "(%.2f TB/s)\n",
               names[f], nt, t_str, STR / t_str / 1e6, t_warm, TBL / t_warm / 1e6, t_after, TBL / t_after / 1e6);
      }
    }
    CK(hipFree(str));
  }
  return 0;
}
