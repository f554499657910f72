// Synthetic encoder-like neighbours for scripts/exp/interference.py: what in an encoder GEMM workgroup slows the
// decoder kernels running beside it? Both kernels hold one 512-thread workgroup per CU with 136 KiB of LDS (as
// k_gemm_big), one issuing back-to-back MFMAs only, one streaming HBM -> LDS with LDS-DMA only.
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared scripts/exp/neighbors.hip -o scripts/exp/libneighbors.so
#include <hip/hip_runtime.h>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((address_space(3))) void lds_void_t;

__global__ __launch_bounds__(512, 1) void k_mfma_spin(float* out, int iters) {
  __shared__ float pad[34816];  // 136 KiB: one workgroup per CU, as the encoder GEMM
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(0.001f * (threadIdx.x + j));
    b[j] = (__bf16)(0.002f * j);
  }
  f32x4 c[8];
  for (int i = 0; i < 8; ++i) c[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[i], 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  if (s == 12345.f) {
    pad[threadIdx.x] = s;
    __syncthreads();
    out[blockIdx.x] = pad[(threadIdx.x + 1) & 511];
  }
}

__global__ __launch_bounds__(512, 1) void k_mem_stream(const uint4* src, size_t n16, float* out, int iters) {
  __shared__ __attribute__((aligned(16))) unsigned pad[34816];
  const int tid = threadIdx.x, wid = tid >> 6;
  size_t base = (size_t)blockIdx.x * 8192 + tid;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const size_t k = (base + (size_t)i * 512 + (size_t)it * gridDim.x * 8192) % n16;
      __builtin_amdgcn_global_load_lds((const void*)(src + k), (lds_void_t*)(pad + (wid * 8 + i) * 256), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (pad[tid] == 0x12345678u) out[blockIdx.x] = 1.f;
}

extern "C" int nb_mfma_spin(float* out, int grid, int iters, void* stream) {
  hipLaunchKernelGGL(k_mfma_spin, dim3(grid), dim3(512), 0, (hipStream_t)stream, out, iters);
  return hipGetLastError() != hipSuccess;
}

extern "C" int nb_mem_stream(const void* src, size_t bytes, float* out, int grid, int iters, void* stream) {
  hipLaunchKernelGGL(k_mem_stream, dim3(grid), dim3(512), 0, (hipStream_t)stream, (const uint4*)src, bytes / 16, out,
                     iters);
  return hipGetLastError() != hipSuccess;
}
