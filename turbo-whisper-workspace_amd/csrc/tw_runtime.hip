// C-ABI runtime plumbing: error strings, version, synthetic weight generator.
//
// The synthetic generator is the single definition of the seeded weights used by the engine,
// by the oracle (oracle/whisper_oracle.py: synth_uniform) and by the golden-vector script
// (tests/golden/make_golden.py), so all three see bit-identical, bf16-exact parameters.
#include <stdarg.h>
#include <stdio.h>
#include "tw_common.h"
#include "../../include/tw_whisper.h"

static thread_local char g_err[512] = {0};

void tw_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int tw_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    tw_set_error("%s: %s", what, hipGetErrorString(e));
    return TW_ERR_LAUNCH;
  }
  return TW_OK;
}

extern "C" const char* tw_last_error(void) { return g_err; }
extern "C" int tw_version(void) { return TW_ABI_VERSION; }

// splitmix64-style counter hash -> 24-bit signed integer -> exact f32 in (-1, 1).
__host__ __device__ inline float tw_synth_unit(uint64_t seed, uint32_t tensor_id, uint64_t idx) {
  uint64_t z = (seed * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(tensor_id + 1u) * 0xD1B54A32D192ED03ull);
  z += idx * 0x9E3779B97F4A7C15ull;
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27; z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  int32_t s = (int32_t)(z >> 40) - 8388608;                  // [-2^23, 2^23)
  return (float)(2 * s + 1) * (1.0f / 16777216.0f);          // exact
}

__global__ void k_fill_synth(void* out, long n, uint64_t seed, uint32_t tid, float scale, float offset,
                             int as_f32) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    float u = tw_synth_unit(seed, tid, (uint64_t)i);
    float v = __fadd_rn(__fmul_rn(u, scale), offset);           // no fma contraction: matches numpy
    bf16_t h = f32_to_bf16(v);
    if (as_f32) ((float*)out)[i] = bf16_to_f32(h);
    else ((bf16_t*)out)[i] = h;
  }
}

extern "C" int tw_fill_synth(void* out, long n, uint64_t seed, uint32_t tensor_id, float scale, float offset,
                             int as_f32, void* stream) {
  TW_REQUIRE(out != nullptr && n >= 0, "tw_fill_synth: bad args");
  if (n == 0) return TW_OK;
  unsigned grid = tw_cdiv(n, 256);
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(k_fill_synth, dim3(grid), dim3(256), 0, (hipStream_t)stream, out, n, seed, tensor_id, scale,
                     offset, as_f32);
  return tw_check_launch("tw_fill_synth");
}

__global__ void k_f32_to_bf16(const float* in, bf16_t* out, long n, float scale) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = f32_to_bf16(in[i] * scale);
}

extern "C" int tw_f32_to_bf16(const float* in, bf16_t* out, long n, float scale, void* stream) {
  TW_REQUIRE(in && out && n >= 0, "tw_f32_to_bf16: bad args");
  if (n == 0) return TW_OK;
  unsigned grid = tw_cdiv(n, 256);
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(k_f32_to_bf16, dim3(grid), dim3(256), 0, (hipStream_t)stream, in, out, n, scale);
  return tw_check_launch("tw_f32_to_bf16");
}
