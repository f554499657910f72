// Shared device/host helpers for the MI355X (gfx950) Whisper hot path.
// Storage conventions: bf16 tensors are raw uint16 (no HIP bf16 class types cross the C-ABI),
// f32 everywhere else. Every C-ABI entry returns 0 on success or a nonzero tw error code;
// tw_last_error() gives the message (see include/tw_whisper.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;  // MFMA bf16 operand fragment (8 elems, 4 VGPRs)
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

#define TW_WAVE 64

#ifndef TW_DEBUG
#define TW_DEBUG 0  // -DTW_DEBUG=1 (make debug): contract checks on the C-ABI (tw_attn_decode_self_tab's table)
#endif

// ---- bf16 <-> f32 (round-to-nearest-even; NaN kept NaN) --------------------------------------
__host__ __device__ inline float bf16_to_f32(bf16_t h) {
  union { uint32_t u; float f; } v; v.u = ((uint32_t)h) << 16; return v.f;
}
__host__ __device__ inline bf16_t f32_to_bf16(float f) {
  union { uint32_t u; float f; } v; v.f = f;
  uint32_t u = v.u;
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (bf16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}
__device__ inline uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

// ---- erf GELU (ACT2FN["gelu"] = nn.GELU() = 0.5 x (1 + erf(x/sqrt2))) ---------------------------
// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, below the f32 resolution of GELU outputs that are then
// rounded to bf16): one v_rcp, one v_exp and five FMAs, branch-free. The ocml erff costs ~3x the instructions and
// the fc1 / conv-stem epilogues evaluate it for every one of B*1500*5120 outputs.
__device__ inline float erf_fast(float x) {
  const float z = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);
  return copysignf(fmaf(-p, e, 1.0f), x);
}
__device__ inline float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

// The same GELU on two values with packed f32 VALU (v_pk_fma_f32 / v_pk_mul_f32: two results per issue, the f32
// vector peak): the GEMM epilogues evaluate it with no MFMA beside them (one workgroup per CU), so their cost is
// pure VALU issue. Same operations and rounding order as gelu_erf (bit-identical results).
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ inline f32x2 gelu_erf2(f32x2 x) {
  const f32x2 u = x * 0.70710678118654752f;
  const f32x2 z = __builtin_elementwise_abs(u);
  const f32x2 d = z * 0.3275911f + 1.0f;
  f32x2 t;
  t.x = __builtin_amdgcn_rcpf(d.x);
  t.y = __builtin_amdgcn_rcpf(d.y);
  f32x2 p = t * 1.061405429f + -1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t + -0.284496736f;
  p = p * t + 0.254829592f;
  p = p * t;
  const f32x2 q = (-z * z) * 1.4426950408889634f;
  f32x2 e;
  e.x = __builtin_amdgcn_exp2f(q.x);
  e.y = __builtin_amdgcn_exp2f(q.y);
  const f32x2 a = 1.0f - p * e;
  f32x2 erf;
  erf.x = copysignf(a.x, u.x);
  erf.y = copysignf(a.y, u.y);
  const f32x2 hx = x * 0.5f;
  return hx * (erf + 1.0f);  // (0.5x)(1+erf) exactly as gelu_erf rounds it
}
__device__ inline float4 gelu_erf4(float4 v) {
  const f32x2 a = gelu_erf2((f32x2){v.x, v.y}), b = gelu_erf2((f32x2){v.z, v.w});
  return make_float4(a.x, a.y, b.x, b.y);
}

// ---- wave reductions (64 lanes) ----------------------------------------------------------------
// Sum over each aligned group of 8 lanes, in every lane of the group: DPP quad_perm xor 1, xor 2, then the half-row
// mirror (lane i with 7 - i, the other quad). Bit-identical to `d += __shfl_xor(d, 1); ... 2; ... 4` (after the two
// quad steps every lane of a quad holds the same bits, and a + b == b + a), without the three ds_bpermute round trips
// through the LDS crossbar per dot product (the decoder attentions' key loops issue one per key per row).
__device__ __forceinline__ float lane8_sum(float d) {
  d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0xB1, 0xF, 0xF, false));
  d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x4E, 0xF, 0xF, false));
  d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x141, 0xF, 0xF, false));
  return d;
}

__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- MX fp8 (BASELINE config 5: fp8 MFMA encoder) -----------------------------------------------
// OCP MX block format for the encoder GEMM operands: e4m3fn elements, one e8m0 scale per 32 consecutive K
// elements of a row (the block v_mfma_scale_f32_16x16x128_f8f6f4 consumes). Scale byte s = E - 8, plus one
// when the absmax mantissa exceeds 1.75 (E = biased f32 exponent of the block's absmax; s = 1 for E < 9): the
// OCP shared exponent floor(log2 amax) - emax(e4m3), raised by one where it would push the block's largest
// elements past 448 = 1.75 * 2^8, so no element saturates; element = e4m3_rne(clamp(x * 2^(127 - s), +-448)).
// oracle/whisper_oracle.py mx_quant restates this bit for bit.
// Scale layout in HBM: [K/128][rows_pad][4] bytes (one dword per row per 128-deep K-step: a GEMM tile's scales
// of one K-step are one contiguous 1 KiB run), byte (k/32) % 4.
__host__ __device__ inline size_t tw_mx_sidx(int m, int kb, int rows_pad) {
  return ((size_t)(kb >> 2) * rows_pad + m) * 4 + (kb & 3);
}
__device__ inline uint32_t mx_scale_byte(float amax) {
  const uint32_t u = __float_as_uint(amax), e = (u >> 23) & 0xffu;
  return e < 9u ? 1u : e - 8u + ((u & 0x7fffffu) > 0x600000u ? 1u : 0u);
}
__device__ inline float mx_inv_scale(uint32_t s) { return __uint_as_float((254u - s) << 23); }  // 2^(127 - s)
__device__ inline uint32_t mx_pack4(float a, float b, float c, float d, float inv) {
  a = fminf(fmaxf(a * inv, -448.f), 448.f);
  b = fminf(fmaxf(b * inv, -448.f), 448.f);
  c = fminf(fmaxf(c * inv, -448.f), 448.f);
  d = fminf(fmaxf(d * inv, -448.f), 448.f);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}
// absmax over the 8 consecutive lanes (xor 1, 2, 4) that hold one 32-element block as 4 values each
__device__ inline float mx_group8_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  v = fmaxf(v, __shfl_xor(v, 4, 64));
  return v;
}
// the same by DPP lane moves (VALU instructions instead of ds_bpermute round trips on the LDS pipeline): xor 1 and
// xor 2 as quad permutes, then the half-row mirror (lane i <-> 7 - i) once every quad holds its own maximum
__device__ inline float mx_dpp_max(float v, int v2) { return fmaxf(v, __builtin_bit_cast(float, v2)); }
__device__ inline float mx_group4_max_dpp(float v) {  // over the 4 lanes of a quad (xor 1, 2)
  v = mx_dpp_max(v, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
  v = mx_dpp_max(v, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  return v;
}
__device__ inline float mx_group8_max_dpp(float v) {
  v = mx_dpp_max(v, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
  v = mx_dpp_max(v, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  v = mx_dpp_max(v, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));  // half mirror
  return v;
}
__device__ inline float abs4max(float a, float b, float c, float d) {
  return fmaxf(fmaxf(fabsf(a), fabsf(b)), fmaxf(fabsf(c), fabsf(d)));
}

// ---- order-preserving float <-> uint key (for atomicMax over signed floats) ----------------------
__device__ inline uint32_t f32_order_key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float f32_from_order_key(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// Decoder kernels raise their waves' issue priority so that, sharing CUs with the encoder GEMM of the next
// window batch, their (latency-bound) instructions are picked first. Compile-time knob for A/B builds.
// Encoder-side bulk outputs stored with the non-temporal hint, by producer (TW_ENC_NT bit mask): they are far larger
// than the L2s, and streaming them keeps the L2s free of dirty lines, which every kernel boundary of the concurrently
// running decoder step otherwise has to write back. Bits: 0 GEMM bf16 (q/k/v), 1 GEMM GELU (fc1), 2 GEMM residual
// update (out_proj, fc2), 3 other GEMM epilogues (conv stem, cross K/V), 4 attention output, 5 LayerNorm output,
// 6 conv2 im2col. Measured in the bench (10 steps, two interleaved rounds per build, MI355X): GEMM epilogues except
// the residual update (0x0B) 92.9 ms vs 93.8 ms with none; all GEMM epilogues (0x0F) 93.1; adding the attention,
// LayerNorm and im2col outputs (0x7F) 94.6 vs 93.4 (the next GEMM re-reads those as its A operand). In situ (scripts/
// exp/insitu_breakdown.py) the decode step beside the fc1 GEMM went 849 -> 772 us with the GEMM bits set.
// Write-through (device-scope sc1) stores instead were slower for every producer set tried (94.6-99.0 vs 93.0 ms).
#define TW_NT_GEMM_BF16 1
#define TW_NT_GEMM_GELU 2
#define TW_NT_GEMM_RESID 4
#define TW_NT_GEMM_OTHER 8
#define TW_NT_ATTN 16
#define TW_NT_LN 32
#define TW_NT_IM2COL 64
#ifndef TW_ENC_NT
#define TW_ENC_NT (TW_NT_GEMM_BF16 | TW_NT_GEMM_GELU | TW_NT_GEMM_OTHER)
#endif
typedef unsigned int tw_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int tw_u32x4 __attribute__((ext_vector_type(4)));
typedef float tw_f32x4 __attribute__((ext_vector_type(4)));
template <int BIT>
__device__ inline void tw_st_enc(void* p, uint2 w) {
  if (TW_ENC_NT & BIT) __builtin_nontemporal_store((tw_u32x2){w.x, w.y}, (tw_u32x2*)p);
  else *(uint2*)p = w;
}
template <int BIT>
__device__ inline void tw_st_enc(void* p, uint4 w) {
  if (TW_ENC_NT & BIT) __builtin_nontemporal_store((tw_u32x4){w.x, w.y, w.z, w.w}, (tw_u32x4*)p);
  else *(uint4*)p = w;
}
template <int BIT>
__device__ inline void tw_st_enc(void* p, float4 v) {
  if (TW_ENC_NT & BIT) __builtin_nontemporal_store((tw_f32x4){v.x, v.y, v.z, v.w}, (tw_f32x4*)p);
  else *(float4*)p = v;
}

// Minimum waves per SIMD the decoder-step kernels are compiled for (0: each kernel's own default). Experiment builds
// (-DTW_DEC_WPE=6: <= 80 VGPRs) test decoder co-residency beside a fatter encoder GEMM (k_gemm_8p: 2 x 216 VGPRs).
#ifndef TW_DEC_WPE
#define TW_DEC_WPE 0
#endif
#define TW_DEC_LB(threads, wpe) __launch_bounds__(threads, TW_DEC_WPE ? TW_DEC_WPE : (wpe))
#ifndef TW_DEC_PRIORITY
#define TW_DEC_PRIORITY 3
#endif
#define TW_DEC_PRIO()                                        \
  do {                                                       \
    if (TW_DEC_PRIORITY) __builtin_amdgcn_s_setprio(TW_DEC_PRIORITY); \
  } while (0)

// Register cap of the decoder kernels (VGPRs per wave; 0 = the compiler's choice). A decoder wave can only start on a
// SIMD whose register file has room beside the encoder workgroup running there: k_gemm_big (184 VGPRs x 2 waves)
// leaves 128 of 512, k_gemm_8p (211 x 2) 80, the encoder attention at one workgroup per CU 272. Decoder kernels
// that need more wait for an encoder tile to retire (scripts/exp/interference.py: 2-9x slower launches).
#ifndef TW_DEC_VGPR
#define TW_DEC_VGPR 0
#endif
#if TW_DEC_VGPR
#define TW_DEC_REGS __attribute__((amdgpu_num_vgpr(TW_DEC_VGPR)))
#else
#define TW_DEC_REGS
#endif

// Decoder fragment layouts (include/tw_whisper.h "packed" formats), M <= 64 activation rows:
//   activation [M/32][K/32][2][64][8] bf16: element (m, k) at 32 K (m/32) + ((k/32 * 2 + (m/16)%2) * 64 + (m%16) +
//     16*((k/8)%4)) * 8 + k%8, i.e. rows 0..31 and 32..63 are two 32-row blocks; in a block step s = k/32, m-tile
//     t = (m/16)%2 is the 16x32 A fragment of v_mfma_f32_16x16x32_bf16 (1 KiB contiguous)
//   weight     [N/16][K/32][64][8] bf16: element (n, k) at ((n/16 * K/32 + k/32) * 64 + (n%16) + 16*((k/8)%4)) * 8 + k%8
__host__ __device__ inline size_t tw_pack_act_idx(int m, int k, int K) {
  return (m >= 32 ? (size_t)32 * K : (size_t)0) +
         ((size_t)((k >> 5) * 2 + ((m >> 4) & 1)) * 64 + (m & 15) + 16 * ((k >> 3) & 3)) * 8 + (k & 7);
}
__host__ __device__ inline size_t tw_pack_w_idx(int n, int k, int K) {
  return ((size_t)((n >> 4) * (K >> 5) + (k >> 5)) * 64 + (n & 15) + 16 * ((k >> 3) & 3)) * 8 + (k & 7);
}

// ---- decoder row LayerNorm (one 256-thread block per row) ----------------------------------------
// The row's d_model values sit as float4 chunks c = tid + 256 i in v[i] (valid for c < D/4), s = this thread's
// partial sum of them. Writes bf16(LayerNorm(row) * g + bta) row-major (out + row * D) or in the packed
// activation layout. red: 8 floats of LDS. Shared by k_resid_ln and the fused select/embed/LN tail.
template <bool PACKED, int NV>
__device__ inline void tw_row_ln_store(const float4 (&v)[NV], float s, int row, int D, float eps,
                                       const float* __restrict__ g, const float* __restrict__ bta,
                                       bf16_t* __restrict__ out, float* red) {
  const int tid = threadIdx.x, nc = D >> 2;
  s = wave_sum(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  const float mean = (red[0] + red[1] + red[2] + red[3]) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (tid + 256 * i < nc) {
      const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
      q += (a * a + b * b) + (c * c + d * d);
    }
  }
  q = wave_sum(q);
  if ((tid & 63) == 0) red[4 + (tid >> 6)] = q;
  __syncthreads();
  const float rstd = rsqrtf((red[4] + red[5] + red[6] + red[7]) / (float)D + eps);
  bf16_t* orow = out + (size_t)row * D;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + 256 * i;
    if (c < nc) {
      const float4 gg = ((const float4*)g)[c], bb = ((const float4*)bta)[c];
      uint2 w;
      w.x = pack_bf16x2((v[i].x - mean) * rstd * gg.x + bb.x, (v[i].y - mean) * rstd * gg.y + bb.y);
      w.y = pack_bf16x2((v[i].z - mean) * rstd * gg.z + bb.z, (v[i].w - mean) * rstd * gg.w + bb.w);
      if constexpr (PACKED) {
        *(uint2*)(out + tw_pack_act_idx(row, 4 * c, D)) = w;  // 4 columns = half a 16-byte fragment chunk
      } else {
        ((uint2*)orow)[c] = w;
      }
    }
  }
}

// ---- error plumbing -------------------------------------------------------------------------------
enum {
  TW_OK = 0,
  TW_ERR_ARG = 1,     // bad shape / null pointer / unsupported size
  TW_ERR_LAUNCH = 2,  // hipGetLastError after launch
};
void tw_set_error(const char* fmt, ...);
int tw_check_launch(const char* what);

#define TW_REQUIRE(cond, ...)            \
  do {                                   \
    if (!(cond)) {                       \
      tw_set_error(__VA_ARGS__);         \
      return TW_ERR_ARG;                 \
    }                                    \
  } while (0)

static inline unsigned tw_cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }
