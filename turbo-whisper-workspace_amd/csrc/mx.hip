// MX-fp8 producers of the fp8 encoder (BASELINE config 5: "fp8 MFMA encoder + bf16 decoder"): the encoder
// projections of $TF/models/whisper/modeling_whisper.py:279-282,309 (q/k/v/o) and :375-376 (fc1/fc2) take
// e4m3 operands with one e8m0 scale per 32 K elements (format: tw_common.h "MX fp8").
//   k_quant_mx       bf16 rows -> MX fp8 (encoder weights once at load; the attention output before o-proj)
//   k_layernorm_mx   nn.LayerNorm (:371,377) with the MX quantisation fused into its store (the qkv / fc1 operand)
// The fc1 -> fc2 operand is quantised in the fc1 GEMM epilogue (gemm.hip, TW_EPI_GELU_MX).
#include "tw_common.h"
#include "../../include/tw_whisper.h"

// 8 elements per thread (one 16-byte bf16 load, one 8-byte fp8 store); the 4 threads of one 32-element block
// are consecutive lanes, so the block absmax is two xor shuffles.
__global__ __launch_bounds__(256) void k_quant_mx(const bf16_t* __restrict__ src, int rows, int K, int ld,
                                                  uint8_t* __restrict__ dst, uint8_t* __restrict__ scales,
                                                  int rows_pad) {
  const int per_row = K >> 3;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = t < (long)rows * per_row;
  const long tt = live ? t : 0;
  const int m = (int)(tt / per_row), c = (int)(tt - (long)m * per_row);
  const uint4 raw = *(const uint4*)(src + (size_t)m * ld + c * 8);
  float v[8];
  const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
  float a = fmaxf(abs4max(v[0], v[1], v[2], v[3]), abs4max(v[4], v[5], v[6], v[7]));
  a = fmaxf(a, __shfl_xor(a, 1, 64));
  a = fmaxf(a, __shfl_xor(a, 2, 64));
  const uint32_t s = mx_scale_byte(a);
  const float inv = mx_inv_scale(s);
  uint2 q;
  q.x = mx_pack4(v[0], v[1], v[2], v[3], inv);
  q.y = mx_pack4(v[4], v[5], v[6], v[7], inv);
  if (!live) return;
  *(uint2*)(dst + (size_t)m * K + c * 8) = q;
  if ((c & 3) == 0) scales[tw_mx_sidx(m, c >> 2, rows_pad)] = (uint8_t)s;
}

extern "C" int tw_quant_mx(const bf16_t* src, int rows, int K, int ld, uint8_t* dst, uint8_t* scales, int rows_pad,
                           void* stream) {
  TW_REQUIRE(src && dst && scales && rows > 0, "tw_quant_mx: bad args");
  TW_REQUIRE(K % 128 == 0 && ld % 8 == 0 && ld >= K, "tw_quant_mx: K=%d must be a multiple of 128 (ld=%d)", K, ld);
  TW_REQUIRE(rows_pad >= rows, "tw_quant_mx: rows_pad %d < rows %d", rows_pad, rows);
  const long n = (long)rows * (K / 8);
  hipLaunchKernelGGL(k_quant_mx, dim3(tw_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, src, rows, K, ld, dst,
                     scales, rows_pad);
  return tw_check_launch("tw_quant_mx");
}

// LayerNorm as k_layernorm (one wave per row, the row kept in registers, sized to it by NC = ceil(D / 256) float4
// chunks per lane; gamma / beta loaded with the row), storing MX fp8: lane l holds columns 4(l + 64 i) .. +3, so the 8
// consecutive lanes of a group cover one 32-column block, whose absmax is three DPP lane moves on the VALU
// (mx_group8_max_dpp) instead of three ds_bpermute round trips.
#define LNQ_MAXC 16
template <int NC>
__global__ __launch_bounds__(256) void k_layernorm_mx(const float* __restrict__ x, const float* __restrict__ g,
                                                      const float* __restrict__ bta, int M, int D, float eps,
                                                      uint8_t* __restrict__ out, uint8_t* __restrict__ scales,
                                                      int rows_pad) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;  // wave-uniform
  const int nc = D >> 2;
  const float4* xr = (const float4*)(x + (size_t)row * D);
  float4 v[NC], gg[NC], bb[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    if (64 * i < nc) {  // wave-uniform trip bound; the lane index is clamped, not branched on
      const int cc = min(lane + 64 * i, nc - 1);
      v[i] = xr[cc];
      gg[i] = ((const float4*)g)[cc];
      bb[i] = ((const float4*)bta)[cc];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i)
    if (64 * i < nc && lane + 64 * i < nc) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    if (64 * i < nc && lane + 64 * i < nc) {
      const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, d = v[i].w - mean;
      q += (a * a + b * b) + (cc * cc + d * d);
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
  uint32_t* orow = (uint32_t*)(out + (size_t)row * D);
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + 64 * i;
    if (64 * i < nc) {  // wave-uniform: every lane of a group takes part in the lane moves (D % 32 == 0)
      const float y0 = (v[i].x - mean) * rstd * gg[i].x + bb[i].x, y1 = (v[i].y - mean) * rstd * gg[i].y + bb[i].y;
      const float y2 = (v[i].z - mean) * rstd * gg[i].z + bb[i].z, y3 = (v[i].w - mean) * rstd * gg[i].w + bb[i].w;
      const uint32_t sb = mx_scale_byte(mx_group8_max_dpp(abs4max(y0, y1, y2, y3)));
      const uint32_t w = mx_pack4(y0, y1, y2, y3, mx_inv_scale(sb));
      if (c < nc) {
        orow[c] = w;
#ifndef TW_LNQ_PROBE_NOSCALE  // (probe build only: what the scattered scale-byte stores cost)
        if ((c & 7) == 0) scales[tw_mx_sidx(row, c >> 3, rows_pad)] = (uint8_t)sb;
#endif
      }
    }
  }
}

size_t tw_layernorm_lds_pad_bytes();  // elementwise.hip: tw_layernorm_set_lds_pad's cap, beside a decode

extern "C" int tw_layernorm_mx(const float* x, const float* gamma, const float* beta, int M, int D, float eps,
                               uint8_t* out, uint8_t* scales, int rows_pad, void* stream) {
  TW_REQUIRE(x && gamma && beta && out && scales && M > 0, "tw_layernorm_mx: bad args");
  TW_REQUIRE(D % 128 == 0 && D <= 256 * LNQ_MAXC, "tw_layernorm_mx: D=%d must be a multiple of 128 and <= %d", D,
             256 * LNQ_MAXC);
  TW_REQUIRE(rows_pad >= M, "tw_layernorm_mx: rows_pad %d < M %d", rows_pad, M);
  const dim3 grid(tw_cdiv(M, 4)), blk(256);
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = tw_layernorm_lds_pad_bytes();
#define TW_LNQ(nc) hipLaunchKernelGGL(k_layernorm_mx<nc>, grid, blk, lds, st, x, gamma, beta, M, D, eps, out, scales, rows_pad)
  switch (tw_cdiv(D, 256)) {
    case 1: TW_LNQ(1); break;
    case 2: TW_LNQ(2); break;
    case 3: TW_LNQ(3); break;
    case 4: TW_LNQ(4); break;
    case 5: TW_LNQ(5); break;
    case 6: TW_LNQ(6); break;
    case 7: case 8: TW_LNQ(8); break;
    default: TW_LNQ(LNQ_MAXC); break;
  }
#undef TW_LNQ
  return tw_check_launch("tw_layernorm_mx");
}
