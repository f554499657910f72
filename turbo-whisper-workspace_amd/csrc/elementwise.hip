// Row-wise and data-movement kernels of the Whisper hot path:
//   LayerNorm (nn.LayerNorm eps 1e-5, $TF/models/whisper/modeling_whisper.py:371,377,434,443,446,573,682)
//   conv-stem im2col (Conv1d k3 p1 / k3 s2 p1, :566-567) incl. the seek-window slice + zero pad of
//     WhisperGenerationMixin._get_input_segment ($TF/models/whisper/generation_whisper.py:1831-1850)
//   decoder token + learned-position embedding (:737,753-762)
#include "tw_common.h"
#include "../../include/tw_whisper.h"

// One wave per row, f32 in -> bf16 out (the GEMM A operand). The row is read once with 16-byte loads and
// kept in registers (D <= 64 * 4 * LN_MAXC); mean and variance are two wave reductions over it.
#define LN_MAXC 16
template <int NC>  // float4 chunks per lane: ceil(D / 256) (registers sized to the row, not to LN_MAXC)
__global__ __launch_bounds__(256) void k_layernorm(const float* __restrict__ x, const float* __restrict__ g,
                                                   const float* __restrict__ bta, int M, int D, float eps,
                                                   bf16_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nc = D >> 2;
  const float4* xr = (const float4*)(x + (size_t)row * D);
  float4 v[NC], gg[NC], bb[NC];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + 64 * i;
    if (64 * i < nc) {  // wave-uniform trip bound; the lane index is clamped, not branched on
      v[i] = xr[min(c, nc - 1)];
      // gamma / beta fly with the row instead of after both reductions (one dependent round trip less)
      gg[i] = ((const float4*)g)[min(c, nc - 1)];
      bb[i] = ((const float4*)bta)[min(c, nc - 1)];
    }
  }
#pragma unroll
  for (int i = 0; i < NC; ++i)
    if (64 * i < nc && lane + 64 * i < nc) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + 64 * i;
    if (64 * i < nc && c < nc) {
      const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, d = v[i].w - mean;
      q += (a * a + b * b) + (cc * cc + d * d);
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
  uint2* orow = (uint2*)(out + (size_t)row * D);
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + 64 * i;
    if (64 * i < nc && c < nc) {
      uint2 w;
      w.x = pack_bf16x2((v[i].x - mean) * rstd * gg[i].x + bb[i].x, (v[i].y - mean) * rstd * gg[i].y + bb[i].y);
      w.y = pack_bf16x2((v[i].z - mean) * rstd * gg[i].z + bb[i].z, (v[i].w - mean) * rstd * gg[i].w + bb[i].w);
      tw_st_enc<TW_NT_LN>(orow + c, w);
    }
  }
}

// Dynamic LDS requested per LayerNorm workgroup (KiB; tw_layernorm_set_lds_pad): none alone; beside a decode it caps
// the LayerNorm's workgroups per CU so that their waves leave registers and LDS for a decoder wave on every SIMD
// (uncapped, ~6 LayerNorm waves of 78 registers fill a SIMD) — the encoder attention's cap (tw_attn_set_lds_pad), here.
static int tw_ln_lds_pad_kib = 0;
size_t tw_layernorm_lds_pad_bytes() { return (size_t)tw_ln_lds_pad_kib * 1024; }  // (also tw_layernorm_mx's cap)
extern "C" int tw_layernorm_set_lds_pad(int kib) {
  TW_REQUIRE(kib >= 0 && kib <= 64, "tw_layernorm_set_lds_pad: %d KiB (0..64)", kib);
  tw_ln_lds_pad_kib = kib;
  return 0;
}

extern "C" int tw_layernorm(const float* x, const float* gamma, const float* beta, int M, int D, float eps, bf16_t* out,
                            void* stream) {
  TW_REQUIRE(x && gamma && beta && out && M > 0, "tw_layernorm: bad args");
  TW_REQUIRE(D % 4 == 0 && D <= 256 * LN_MAXC, "tw_layernorm: D=%d must be a multiple of 4 and <= %d", D, 256 * LN_MAXC);
  const dim3 grid(tw_cdiv(M, 4)), blk(256);
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = (size_t)tw_ln_lds_pad_kib * 1024;
  switch (tw_cdiv(D, 256)) {
    case 1: hipLaunchKernelGGL(k_layernorm<1>, grid, blk, lds, st, x, gamma, beta, M, D, eps, out); break;
    case 2: hipLaunchKernelGGL(k_layernorm<2>, grid, blk, lds, st, x, gamma, beta, M, D, eps, out); break;
    case 3: hipLaunchKernelGGL(k_layernorm<3>, grid, blk, lds, st, x, gamma, beta, M, D, eps, out); break;
    case 4: hipLaunchKernelGGL(k_layernorm<4>, grid, blk, lds, st, x, gamma, beta, M, D, eps, out); break;
    case 5: hipLaunchKernelGGL(k_layernorm<5>, grid, blk, lds, st, x, gamma, beta, M, D, eps, out); break;
    case 6: hipLaunchKernelGGL(k_layernorm<6>, grid, blk, lds, st, x, gamma, beta, M, D, eps, out); break;
    case 7: case 8: hipLaunchKernelGGL(k_layernorm<8>, grid, blk, lds, st, x, gamma, beta, M, D, eps, out); break;
    default: hipLaunchKernelGGL(k_layernorm<LN_MAXC>, grid, blk, lds, st, x, gamma, beta, M, D, eps, out); break;
  }
  return tw_check_launch("tw_layernorm");
}

// conv1 im2col: A[r*3000 + t][k], k = j*n_mels + c (kw-major, weights reordered to match),
// value = seg[c][t + j - 1] where seg = feats[row_map[r]][:, seek[r]:] zero-padded to 3000 frames.
// (feats rows of ld frames; maxf: per-row feature length — the seek window is feats[seek : min(seek + 3000, maxf)],
// _get_input_segment's seek_num_frames; NULL = 3000, the 30-s windows)
__global__ void k_im2col_conv1(const float* __restrict__ feats, int n_mels, const int* __restrict__ row_map,
                               const int* __restrict__ seek, int R, int kpad, bf16_t* __restrict__ out, long ld,
                               const int* __restrict__ maxf) {
  const long total = (long)R * 3000 * kpad;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  for (; i < total; i += stride) {
    const int k = (int)(i % kpad);
    const long m = i / kpad;
    const int r = (int)(m / 3000), t = (int)(m - (long)r * 3000);
    float v = 0.f;
    if (k < 3 * n_mels) {
      const int j = k / n_mels, c = k - j * n_mels;
      const int sk = seek ? seek[r] : 0;
      const int u = t + j - 1;
      const int chunk = row_map ? row_map[r] : r;
      if (u >= 0 && u < min(3000, (maxf ? maxf[chunk] : 3000) - sk)) v = feats[((size_t)chunk * n_mels + c) * ld + sk + u];
    }
    out[i] = f32_to_bf16(v);
  }
}

extern "C" int tw_im2col_conv1(const float* feats, int n_mels, const int* row_map, const int* seek, int R, int kpad,
                               bf16_t* out, void* stream) {
  TW_REQUIRE(feats && out && R > 0 && kpad >= 3 * n_mels && kpad % 64 == 0, "tw_im2col_conv1: bad args");
  long total = (long)R * 3000 * kpad;
  unsigned grid = tw_cdiv(total, 256);
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(k_im2col_conv1, dim3(grid), dim3(256), 0, (hipStream_t)stream, feats, n_mels, row_map, seek, R,
                     kpad, out, 3000L, (const int*)nullptr);
  return tw_check_launch("tw_im2col_conv1");
}

extern "C" int tw_im2col_conv1_long(const float* feats, int n_mels, long ld, const int* max_frames, const int* row_map,
                                    const int* seek, int R, int kpad, bf16_t* out, void* stream) {
  TW_REQUIRE(feats && max_frames && seek && out && R > 0 && kpad >= 3 * n_mels && kpad % 64 == 0 && ld >= 3000,
             "tw_im2col_conv1_long: bad args");
  long total = (long)R * 3000 * kpad;
  unsigned grid = tw_cdiv(total, 256);
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(k_im2col_conv1, dim3(grid), dim3(256), 0, (hipStream_t)stream, feats, n_mels, row_map, seek, R,
                     kpad, out, ld, max_frames);
  return tw_check_launch("tw_im2col_conv1_long");
}

// conv2 im2col (stride 2): A[r*1500 + t][j*D + c] = h1[r*3000 + 2t + j - 1][c], zero outside [0, 3000).
__global__ void k_im2col_conv2(const bf16_t* __restrict__ h1, int R, int D, bf16_t* __restrict__ out) {
  const int cpr = 3 * D / 8;  // 16-byte chunks per output row
  const long total = (long)R * 1500 * cpr;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  for (; i < total; i += stride) {
    const int ch = (int)(i % cpr);
    const long m = i / cpr;
    const int r = (int)(m / 1500), t = (int)(m - (long)r * 1500);
    const int k = ch * 8, j = k / D, c = k - j * D;
    const int u = 2 * t + j - 1;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (u >= 0 && u < 3000) v = *(const uint4*)(h1 + ((size_t)r * 3000 + u) * D + c);
    tw_st_enc<TW_NT_IM2COL>(out + (size_t)m * 3 * D + k, v);
  }
}

extern "C" int tw_im2col_conv2(const bf16_t* h1, int R, int D, bf16_t* out, void* stream) {
  TW_REQUIRE(h1 && out && R > 0 && D % 8 == 0, "tw_im2col_conv2: bad args");
  long total = (long)R * 1500 * (3 * D / 8);
  unsigned grid = tw_cdiv(total, 256);
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(k_im2col_conv2, dim3(grid), dim3(256), 0, (hipStream_t)stream, h1, R, D, out);
  return tw_check_launch("tw_im2col_conv2");
}

// x[b][:] = embed_tokens[ids[b]] + embed_positions[pos[b]]  (f32 residual stream)
__global__ void k_embed_decoder(const bf16_t* __restrict__ tok_emb, const bf16_t* __restrict__ pos_emb,
                                const int* __restrict__ ids, const int* __restrict__ pos, int D,
                                float* __restrict__ x) {
  TW_DEC_PRIO();
  const int b = blockIdx.x;
  const bf16_t* te = tok_emb + (size_t)ids[b] * D;
  const bf16_t* pe = pos_emb + (size_t)pos[b] * D;
  for (int c = threadIdx.x; c < D; c += blockDim.x) x[(size_t)b * D + c] = bf16_to_f32(te[c]) + bf16_to_f32(pe[c]);
}

extern "C" int tw_embed_decoder(const bf16_t* tok_emb, const bf16_t* pos_emb, const int* ids, const int* pos, int B,
                                int D, float* x, void* stream) {
  TW_REQUIRE(tok_emb && pos_emb && ids && pos && x && B > 0 && D > 0, "tw_embed_decoder: bad args");
  hipLaunchKernelGGL(k_embed_decoder, dim3(B), dim3(256), 0, (hipStream_t)stream, tok_emb, pos_emb, ids, pos, D, x);
  return tw_check_launch("tw_embed_decoder");
}

// Decoder residual update + LayerNorm, one block per row:
//   x[row] += bias + sum_p parts[p][row]   (the split-K partial sums of the previous projection,
//                                           tw_gemm_bf16_partial; nparts = 0 and bias = NULL: no update)
//   out[row] = bf16(LayerNorm(x[row]))      (gamma = NULL: residual update only)
// Restates the residual adds of WhisperDecoderLayer.forward ($TF/models/whisper/modeling_whisper.py:
// 468-505) fused with the next pre-LayerNorm (:434,443,446,682).
#define RLN_MAXV 4  // float4 chunks per thread: D <= 4096
// All loads are unconditional (index clamped into the row, result discarded): a guarded load per
// element makes hipcc wait vmcnt(0) per element, a chain of L2 round trips.
// (x_out: where the updated row goes; x itself for the in-place form)
template <bool PACKED>
__global__ __launch_bounds__(256) void k_resid_ln(const float* x, const float* __restrict__ parts, int nparts,
                                                  long part_stride, const float* __restrict__ bias,
                                                  const float* __restrict__ g, const float* __restrict__ bta, int D,
                                                  float eps, bf16_t* __restrict__ out, float* x_out) {
  TW_DEC_PRIO();
  __shared__ float red[8];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int nc = D >> 2;
  const float* xr = x + (size_t)row * D;
  float* xo = x_out + (size_t)row * D;
  const float* pr = parts ? parts + (size_t)row * D : nullptr;
  float4 v[RLN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < RLN_MAXV; ++i) {
    const int c = min(tid + 256 * i, nc - 1);
    float4 a = ((const float4*)xr)[c];
    if (bias) {
      const float4 bb = ((const float4*)bias)[c];
      a.x += bb.x; a.y += bb.y; a.z += bb.z; a.w += bb.w;
    }
    if (nparts > 0) {
      float4 q[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) q[p] = ((const float4*)(pr + min(p, nparts - 1) * part_stride))[c];
#pragma unroll
      for (int p = 0; p < 4; ++p)
        if (p < nparts) { a.x += q[p].x; a.y += q[p].y; a.z += q[p].z; a.w += q[p].w; }
      for (int p = 4; p < nparts; ++p) {
        const float4 qq = ((const float4*)(pr + p * part_stride))[c];
        a.x += qq.x; a.y += qq.y; a.z += qq.z; a.w += qq.w;
      }
    }
    v[i] = a;
    if (tid + 256 * i < nc) s += (a.x + a.y) + (a.z + a.w);
  }
  if (nparts > 0 || bias || x_out != x) {
#pragma unroll
    for (int i = 0; i < RLN_MAXV; ++i)
      if (tid + 256 * i < nc) ((float4*)xo)[tid + 256 * i] = v[i];
  }
  if (!g) return;
  tw_row_ln_store<PACKED>(v, s, row, D, eps, g, bta, out, red);
}

// k_resid_ln for D = 256 * NV with ONE wave per row: every lane holds NV float4 chunks (c = lane + 64 i), both
// LayerNorm reductions are wave shuffles, no LDS round trip or block barrier. A decode step runs 13 of these on 24
// rows; the 4-wave form (k_resid_ln, the fallback for other D) spends most of its ~6.8 us in its two
// barrier-separated reductions.
// (min 4 waves per SIMD: <= 128 VGPRs, so a wave fits beside an encoder GEMM workgroup's two ~190-VGPR waves)
template <bool PACKED, int NV>
__global__ TW_DEC_LB(64, 4) void k_resid_ln_w(const float* x, const float* __restrict__ parts, int nparts,
                                                   long part_stride, const float* __restrict__ bias,
                                                   const float* __restrict__ g, const float* __restrict__ bta, int D,
                                                   float eps, bf16_t* __restrict__ out, float* x_out) {
  TW_DEC_PRIO();
  const int row = blockIdx.x, lane = threadIdx.x;
  const float* xr = x + (size_t)row * D;
  float* xo = x_out + (size_t)row * D;
  const float* pr = parts ? parts + (size_t)row * D : nullptr;
  float4 gg[NV], bb[NV];
  // the row, the bias and up to four partials: every load in flight before the first add (one memory round trip;
  // the sched_barrier keeps hipcc from interleaving them with the adds, which serialises them). Summation order as
  // before: ((x + bias) + p0) + p1 + ...
  float4 v[NV], bv[NV], q[4][NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = ((const float4*)xr)[lane + 64 * i];
  if (bias) {
#pragma unroll
    for (int i = 0; i < NV; ++i) bv[i] = ((const float4*)bias)[lane + 64 * i];
  }
  if (nparts > 0) {
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int i = 0; i < NV; ++i) q[p][i] = ((const float4*)(pr + min(p, nparts - 1) * part_stride))[lane + 64 * i];
  }
  __builtin_amdgcn_sched_barrier(0);
  if (bias) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      v[i].x += bv[i].x; v[i].y += bv[i].y; v[i].z += bv[i].z; v[i].w += bv[i].w;
    }
  }
  if (nparts > 0) {
#pragma unroll
    for (int p = 0; p < 4; ++p)
      if (p < nparts)
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          v[i].x += q[p][i].x; v[i].y += q[p][i].y; v[i].z += q[p][i].z; v[i].w += q[p][i].w;
        }
    for (int p = 4; p < nparts; ++p)
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const float4 qq = ((const float4*)(pr + p * part_stride))[lane + 64 * i];
        v[i].x += qq.x; v[i].y += qq.y; v[i].z += qq.z; v[i].w += qq.w;
      }
  }
  // gamma / beta issued before the two reductions, so their latency hides behind them (loading them with the row
  // measured +2.5 ms per bench step)
  if (g) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      gg[i] = ((const float4*)g)[lane + 64 * i];
      bb[i] = ((const float4*)bta)[lane + 64 * i];
    }
  }
  if (nparts > 0 || bias || x_out != x) {
#pragma unroll
    for (int i = 0; i < NV; ++i) ((float4*)xo)[lane + 64 * i] = v[i];
  }
  if (!g) return;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = wave_sum(s) / (float)D;
  float q2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
    q2 += (a * a + b * b) + (c * c + d * d);
  }
  const float rstd = rsqrtf(wave_sum(q2) / (float)D + eps);
  bf16_t* orow = out + (size_t)row * D;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    uint2 w;
    w.x = pack_bf16x2((v[i].x - mean) * rstd * gg[i].x + bb[i].x, (v[i].y - mean) * rstd * gg[i].y + bb[i].y);
    w.y = pack_bf16x2((v[i].z - mean) * rstd * gg[i].z + bb[i].z, (v[i].w - mean) * rstd * gg[i].w + bb[i].w);
    if constexpr (PACKED) {
      *(uint2*)(out + tw_pack_act_idx(row, 4 * c, D)) = w;
    } else {
      ((uint2*)orow)[c] = w;
    }
  }
}

extern "C" int tw_resid_layernorm(float* x, const float* parts, int nparts, const float* bias, const float* gamma,
                                  const float* beta, int M, int D, float eps, uint16_t* out, void* stream) {
  TW_REQUIRE(x && M > 0 && D > 0 && D % 4 == 0 && D <= 1024 * RLN_MAXV, "tw_resid_layernorm: bad args (D %% 4, D <= %d)",
             1024 * RLN_MAXV);
  TW_REQUIRE(nparts >= 0 && (nparts == 0 || parts), "tw_resid_layernorm: parts");
  TW_REQUIRE(!gamma || (beta && out), "tw_resid_layernorm: gamma without beta/out");
  if (D == 1280)
    hipLaunchKernelGGL((k_resid_ln_w<false, 5>), dim3(M), dim3(64), 0, (hipStream_t)stream, x, parts, nparts,
                       (long)M * D, bias, gamma, beta, D, eps, out, x);
  else
    hipLaunchKernelGGL(k_resid_ln<false>, dim3(M), dim3(256), 0, (hipStream_t)stream, x, parts, nparts, (long)M * D,
                       bias, gamma, beta, D, eps, out, x);
  return tw_check_launch("tw_resid_layernorm");
}

static int resid_ln_packed(const float* x, float* x_out, const float* parts, int nparts, const float* bias,
                           const float* gamma, const float* beta, int M, int D, float eps, uint16_t* out,
                           void* stream) {
  TW_REQUIRE(x && x_out && gamma && beta && out && M > 0 && M <= 64 && D > 0 && D % 32 == 0 && D <= 1024 * RLN_MAXV,
             "tw_resid_layernorm_packed: bad args (M <= 64, D %% 32, gamma/beta/out required)");
  TW_REQUIRE(nparts >= 0 && (nparts == 0 || parts), "tw_resid_layernorm_packed: parts");
  if (D == 1280)
    hipLaunchKernelGGL((k_resid_ln_w<true, 5>), dim3(M), dim3(64), 0, (hipStream_t)stream, x, parts, nparts,
                       (long)M * D, bias, gamma, beta, D, eps, out, x_out);
  else
    hipLaunchKernelGGL(k_resid_ln<true>, dim3(M), dim3(256), 0, (hipStream_t)stream, x, parts, nparts, (long)M * D,
                       bias, gamma, beta, D, eps, out, x_out);
  return tw_check_launch("tw_resid_layernorm_packed");
}

extern "C" int tw_resid_layernorm_packed(float* x, const float* parts, int nparts, const float* bias,
                                         const float* gamma, const float* beta, int M, int D, float eps, uint16_t* out,
                                         void* stream) {
  return resid_ln_packed(x, x, parts, nparts, bias, gamma, beta, M, D, eps, out, stream);
}

extern "C" int tw_resid_layernorm_packed_to(const float* x, float* x_out, const float* parts, int nparts,
                                            const float* bias, const float* gamma, const float* beta, int M, int D,
                                            float eps, uint16_t* out, void* stream) {
  return resid_ln_packed(x, x_out, parts, nparts, bias, gamma, beta, M, D, eps, out, stream);
}
