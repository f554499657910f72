// Experiment: semantics of ds_read_b64_tr_b16 on gfx950 (not product code)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((address_space(3))) short4_t lds_short4_t;
__global__ void k(short* out, int mode) {
  __shared__ __attribute__((aligned(16))) short lds[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i] = i;  // value = row*64 + col
  __syncthreads();
  const int lane = threadIdx.x;
  const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
  int addr;
  if (mode == 0) addr = (q + 4 * g) * 64 + 4 * p;          // group g: rows 4g..4g+3, cols 0..15
  else addr = q * 64 + 16 * g + 4 * p;                     // group g: rows 0..3, cols 16g..16g+15
  short4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4_t*)(lds + addr));
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  short h[256];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    printf("mode %d\n", mode);
    for (int l = 0; l < 64; l += 1) {
      printf("lane %2d:", l);
      for (int e = 0; e < 4; ++e) printf(" (r%d,c%d)", h[l * 4 + e] / 64, h[l * 4 + e] % 64);
      printf("%s", (l % 2) ? "\n" : "   ");
    }
  }
  return 0;
}
