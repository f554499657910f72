// fp32 arithmetic path of the Whisper hot path (BASELINE configs[0]: whisper-tiny.en fp32, the reference's CPU
// load `pipeline(..., torch_dtype=torch.float32)`, /root/reference/vocalis/core/audio_pipeline.py:195-200).
// Every operand, activation, cache and accumulator is f32; matrices run on the f32 matrix cores
// (v_mfma_f32_16x16x4_f32), the attention cores on f32 VALU with wave-shuffle reductions. The kernels restate the same
// modules as the bf16 path ($TF/models/whisper/modeling_whisper.py: nn.Linear / Conv1d :279-282, :375-376, :566-567,
// :970; LayerNorm :371,377,434,443,446,573,682; encoder self-attention :312-335; decoder self / cross attention with the
// KV cache :448-505; token + position embedding :737,753-762) at the precision the configuration names.
#include <math.h>

#include "tw_common.h"
#include "../../include/tw_whisper.h"

// ------------------------------------------------------------------------------------------------
// GEMM: C[M][N] = A[M][K] . W[N][K]^T, f32 operands, 64 x 64 tiles, 4 waves (2 x 2, 32 x 32 each as 2 x 2 blocks of
// v_mfma_f32_16x16x4_f32), K-steps of 16 staged through LDS (register double buffer: tile t+1's loads fly during
// tile t's MFMAs). Operand fragments: A lane l = A[row l & 15][k l >> 4], B lane l = W[col l & 15][k l >> 4];
// accumulator lane l, register r = C[4 (l >> 4) + r][l & 15].
// ------------------------------------------------------------------------------------------------
#define GF_BM 64
#define GF_BN 64
#define GF_BK 16
#define GF_LD (GF_BK + 1)

struct EpiF32 {
  float* out;
  int ldo;
  const float* bias;  // [N] or null
  const float* aux;   // TW_EPI_GELU_POS_F32: positional table [aux_rows][ldo]
  int aux_rows;
  int kv_S, kv_B, kv_D, kv_H;  // TW_EPI_CROSSKV scatter geometry
};

__device__ inline float gelu_f32(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

template <int EPI>
__device__ inline void f32_store(const EpiF32& ea, int m, int n, float v) {
  if (ea.bias) v += ea.bias[n];
  if constexpr (EPI == TW_EPI_F32) {
    ea.out[(size_t)m * ea.ldo + n] = v;
  } else if constexpr (EPI == TW_EPI_GELU_F32) {
    ea.out[(size_t)m * ea.ldo + n] = gelu_f32(v);
  } else if constexpr (EPI == TW_EPI_RESID_F32) {
    float* o = ea.out + (size_t)m * ea.ldo + n;
    *o = *o + v;
  } else if constexpr (EPI == TW_EPI_GELU_POS_F32) {
    ea.out[(size_t)m * ea.ldo + n] = gelu_f32(v) + ea.aux[(size_t)(m % ea.aux_rows) * ea.ldo + n];
  } else if constexpr (EPI == TW_EPI_CROSSKV) {  // n spans [layer][k|v][D], m spans [b][s] -> [layer][kv][b][h][s][64]
    const int D = ea.kv_D, S = ea.kv_S;
    const int l = n / (2 * D), rem = n - l * 2 * D;
    const int kv = rem / D, hd = rem - kv * D;
    const int b = m / S, s = m - b * S;
    ea.out[((((size_t)(l * 2 + kv) * ea.kv_B + b) * ea.kv_H + (hd >> 6)) * S + s) * 64 + (hd & 63)] = v;
  }
}

template <int EPI>
__global__ __launch_bounds__(256) void k_gemm_f32(const float* __restrict__ A, const float* __restrict__ W, int M,
                                                  int N, int K, int lda, int ldw, EpiF32 ea) {
  __shared__ float As[2][GF_BM][GF_LD];
  __shared__ float Ws[2][GF_BN][GF_LD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.y * GF_BM, n0 = blockIdx.x * GF_BN;
  // loader: row tid / 4 of each tile, 4 consecutive k (one float4) at (tid % 4) * 4; rows past M / N load zeros
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  const bool av = m0 + lr < M, wv = n0 + lr < N;
  const float* ap = A + (size_t)min(m0 + lr, M - 1) * lda + lk;
  const float* wp = W + (size_t)min(n0 + lr, N - 1) * ldw + lk;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 ra = av ? *(const float4*)ap : z4;
  float4 rw = wv ? *(const float4*)wp : z4;
  auto put = [&](int buf) {
    As[buf][lr][lk] = ra.x; As[buf][lr][lk + 1] = ra.y; As[buf][lr][lk + 2] = ra.z; As[buf][lr][lk + 3] = ra.w;
    Ws[buf][lr][lk] = rw.x; Ws[buf][lr][lk + 1] = rw.y; Ws[buf][lr][lk + 2] = rw.z; Ws[buf][lr][lk + 3] = rw.w;
  };
  put(0);
  __syncthreads();
  const int wr = wid >> 1, wc = wid & 1, fr = lane & 15, fk = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int nk = K / GF_BK;
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) {
      ra = av ? *(const float4*)(ap + (size_t)(t + 1) * GF_BK) : z4;
      rw = wv ? *(const float4*)(wp + (size_t)(t + 1) * GF_BK) : z4;
    }
#pragma unroll
    for (int kk = 0; kk < GF_BK / 4; ++kk) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[cur][32 * wr + 16 * i + fr][4 * kk + fk];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Ws[cur][32 * wc + 16 * j + fr][4 * kk + fk];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nk) put(cur ^ 1);  // (buffer cur ^ 1 was last read before the previous barrier)
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 32 * wc + 16 * j + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 32 * wr + 16 * i + 4 * fk + r;
        if (m < M && n < N) f32_store<EPI>(ea, m, n, acc[i][j][r]);
      }
    }
}

extern "C" int tw_gemm_f32(const float* A, const float* W, int M, int N, int K, int lda, int ldw, int epi, float* out,
                           int ldo, const float* bias, const float* aux, int aux_rows, const int* kv_geom,
                           void* stream) {
  TW_REQUIRE(A && W && out, "tw_gemm_f32: null pointer");
  TW_REQUIRE(M > 0 && N > 0 && K > 0 && K % GF_BK == 0, "tw_gemm_f32: M=%d N=%d K=%d (K %% 16 required)", M, N, K);
  TW_REQUIRE(lda % 4 == 0 && ldw % 4 == 0 && lda >= K && ldw >= K && ((uintptr_t)A & 15) == 0 &&
                 ((uintptr_t)W & 15) == 0,
             "tw_gemm_f32: lda=%d ldw=%d (multiples of 4, >= K, 16-byte aligned operands)", lda, ldw);
  EpiF32 ea{out, ldo, bias, aux, aux_rows, 0, 0, 0, 0};
  const dim3 grid(tw_cdiv(N, GF_BN), tw_cdiv(M, GF_BM)), blk(256);
  hipStream_t s = (hipStream_t)stream;
  switch (epi) {
    case TW_EPI_F32: hipLaunchKernelGGL(k_gemm_f32<TW_EPI_F32>, grid, blk, 0, s, A, W, M, N, K, lda, ldw, ea); break;
    case TW_EPI_GELU_F32:
      hipLaunchKernelGGL(k_gemm_f32<TW_EPI_GELU_F32>, grid, blk, 0, s, A, W, M, N, K, lda, ldw, ea);
      break;
    case TW_EPI_RESID_F32:
      hipLaunchKernelGGL(k_gemm_f32<TW_EPI_RESID_F32>, grid, blk, 0, s, A, W, M, N, K, lda, ldw, ea);
      break;
    case TW_EPI_GELU_POS_F32:
      TW_REQUIRE(aux && aux_rows > 0, "tw_gemm_f32: GELU_POS needs the positional table");
      hipLaunchKernelGGL(k_gemm_f32<TW_EPI_GELU_POS_F32>, grid, blk, 0, s, A, W, M, N, K, lda, ldw, ea);
      break;
    case TW_EPI_CROSSKV:
      TW_REQUIRE(kv_geom, "tw_gemm_f32: CROSSKV needs kv_geom");
      ea.kv_S = kv_geom[0];
      ea.kv_B = kv_geom[1];
      ea.kv_D = kv_geom[2];
      ea.kv_H = kv_geom[3];
      TW_REQUIRE(ea.kv_D == 64 * ea.kv_H && N % (2 * ea.kv_D) == 0 && M == ea.kv_S * ea.kv_B,
                 "tw_gemm_f32: CROSSKV geometry S=%d B=%d D=%d H=%d vs M=%d N=%d", ea.kv_S, ea.kv_B, ea.kv_D, ea.kv_H,
                 M, N);
      hipLaunchKernelGGL(k_gemm_f32<TW_EPI_CROSSKV>, grid, blk, 0, s, A, W, M, N, K, lda, ldw, ea);
      break;
    default: TW_REQUIRE(false, "tw_gemm_f32: epilogue %d not on the f32 path", epi);
  }
  return tw_check_launch("tw_gemm_f32");
}

// ------------------------------------------------------------------------------------------------
// LayerNorm f32 -> f32, one wave per row (two wave reductions: mean, then the centred variance, as nn.LayerNorm)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_layernorm_f32(const float* __restrict__ x, const float* __restrict__ g,
                                                       const float* __restrict__ bta, int M, int D, float eps,
                                                       float* __restrict__ out) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + (size_t)row * D;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += xr[c];
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float d = xr[c] - mean;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
  float* o = out + (size_t)row * D;
  for (int c = lane; c < D; c += 64) o[c] = (xr[c] - mean) * rstd * g[c] + bta[c];
}

extern "C" int tw_layernorm_f32(const float* x, const float* gamma, const float* beta, int M, int D, float eps,
                                float* out, void* stream) {
  TW_REQUIRE(x && gamma && beta && out && M > 0 && D > 0 && x != out, "tw_layernorm_f32: bad args");
  hipLaunchKernelGGL(k_layernorm_f32, dim3(tw_cdiv(M, 4)), dim3(256), 0, (hipStream_t)stream, x, gamma, beta, M, D,
                     eps, out);
  return tw_check_launch("tw_layernorm_f32");
}

// ------------------------------------------------------------------------------------------------
// Conv stem im2col, f32 (the layout and seek-window semantics of tw_im2col_conv1 / tw_im2col_conv2)
// ------------------------------------------------------------------------------------------------
__global__ void k_im2col_conv1_f32(const float* __restrict__ feats, int n_mels, const int* __restrict__ row_map,
                                   const int* __restrict__ seek, int R, int kpad, float* __restrict__ out, long ld,
                                   const int* __restrict__ maxf) {
  const long total = (long)R * 3000 * kpad;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int k = (int)(i % kpad);
    const long m = i / kpad;
    const int r = (int)(m / 3000), t = (int)(m - (long)r * 3000);
    float v = 0.f;
    if (k < 3 * n_mels) {
      const int j = k / n_mels, c = k - j * n_mels;
      const int sk = seek ? seek[r] : 0, u = t + j - 1, chunk = row_map ? row_map[r] : r;
      if (u >= 0 && u < min(3000, (maxf ? maxf[chunk] : 3000) - sk)) v = feats[((size_t)chunk * n_mels + c) * ld + sk + u];
    }
    out[i] = v;
  }
}

extern "C" int tw_im2col_conv1_f32(const float* feats, int n_mels, long ld, const int* max_frames, const int* row_map,
                                   const int* seek, int R, int kpad, float* out, void* stream) {
  TW_REQUIRE(feats && out && R > 0 && kpad >= 3 * n_mels && kpad % 16 == 0 && ld >= 3000 &&
                 (ld == 3000 || (max_frames && seek)),
             "tw_im2col_conv1_f32: bad args");
  unsigned grid = tw_cdiv((long)R * 3000 * kpad, 256);
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(k_im2col_conv1_f32, dim3(grid), dim3(256), 0, (hipStream_t)stream, feats, n_mels, row_map, seek,
                     R, kpad, out, ld, max_frames);
  return tw_check_launch("tw_im2col_conv1_f32");
}

__global__ void k_im2col_conv2_f32(const float* __restrict__ h1, int R, int D, float* __restrict__ out) {
  const int cpr = 3 * D / 4;  // float4 chunks per output row
  const long total = (long)R * 1500 * cpr;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int ch = (int)(i % cpr);
    const long m = i / cpr;
    const int r = (int)(m / 1500), t = (int)(m - (long)r * 1500);
    const int k = ch * 4, j = k / D, c = k - j * D, u = 2 * t + j - 1;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (u >= 0 && u < 3000) v = *(const float4*)(h1 + ((size_t)r * 3000 + u) * D + c);
    *(float4*)(out + (size_t)m * 3 * D + k) = v;
  }
}

extern "C" int tw_im2col_conv2_f32(const float* h1, int R, int D, float* out, void* stream) {
  TW_REQUIRE(h1 && out && R > 0 && D % 4 == 0, "tw_im2col_conv2_f32: bad args");
  unsigned grid = tw_cdiv((long)R * 1500 * (3 * D / 4), 256);
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(k_im2col_conv2_f32, dim3(grid), dim3(256), 0, (hipStream_t)stream, h1, R, D, out);
  return tw_check_launch("tw_im2col_conv2_f32");
}

// x[b] = embed_tokens[ids[b]] + embed_positions[pos[b]]
__global__ void k_embed_decoder_f32(const float* __restrict__ tok_emb, const float* __restrict__ pos_emb,
                                    const int* __restrict__ ids, const int* __restrict__ pos, int D,
                                    float* __restrict__ x) {
  const int b = blockIdx.x;
  const float* te = tok_emb + (size_t)ids[b] * D;
  const float* pe = pos_emb + (size_t)pos[b] * D;
  for (int c = threadIdx.x; c < D; c += blockDim.x) x[(size_t)b * D + c] = te[c] + pe[c];
}

extern "C" int tw_embed_decoder_f32(const float* tok_emb, const float* pos_emb, const int* ids, const int* pos, int B,
                                    int D, float* x, void* stream) {
  TW_REQUIRE(tok_emb && pos_emb && ids && pos && x && B > 0 && D > 0, "tw_embed_decoder_f32: bad args");
  hipLaunchKernelGGL(k_embed_decoder_f32, dim3(B), dim3(256), 0, (hipStream_t)stream, tok_emb, pos_emb, ids, pos, D, x);
  return tw_check_launch("tw_embed_decoder_f32");
}

// ------------------------------------------------------------------------------------------------
// Encoder self-attention, f32: softmax(q k^T) v per (window, head) over S keys (q carries the 1/8 scale, as the packed
// q projection does). One query per thread (its q and output rows in registers), 64 queries per workgroup; key / value
// tiles of 32 rows staged in LDS and read as broadcasts; online softmax per tile (one rescale per 32 keys).
// ------------------------------------------------------------------------------------------------
#define AE_KT 32
__global__ __launch_bounds__(64) void k_attn_encoder_f32(const float* __restrict__ qkv, int S, int H,
                                                         float* __restrict__ out) {
  __shared__ float4 Ks[AE_KT][16];
  __shared__ float4 Vs[AE_KT][16];
  const int lane = threadIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int D = H * 64, i = blockIdx.x * 64 + lane;
  const float* base = qkv + (size_t)b * S * 3 * D;
  float4 q[16], acc[16];
  const float4* qr = (const float4*)(base + (size_t)min(i, S - 1) * 3 * D + h * 64);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    q[c] = qr[c];
    acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < S; k0 += AE_KT) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < AE_KT * 16 / 64; ++u) {  // 8 float4 of K and of V per lane
      const int e = u * 64 + lane, r = e >> 4, c = e & 15, key = min(k0 + r, S - 1);
      const float* kr = base + (size_t)key * 3 * D + D + h * 64;
      Ks[r][c] = ((const float4*)kr)[c];
      Vs[r][c] = ((const float4*)(kr + D))[c];
    }
    __syncthreads();
    const int n = min(AE_KT, S - k0);
    float sc[AE_KT];
    float mx = m;
#pragma unroll
    for (int j = 0; j < AE_KT; ++j) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int c = 0; c < 16; c += 2) {
        const float4 k0v = Ks[j][c], k1v = Ks[j][c + 1];
        s0 = fmaf(q[c].x, k0v.x, s0); s0 = fmaf(q[c].y, k0v.y, s0); s0 = fmaf(q[c].z, k0v.z, s0); s0 = fmaf(q[c].w, k0v.w, s0);
        s1 = fmaf(q[c + 1].x, k1v.x, s1); s1 = fmaf(q[c + 1].y, k1v.y, s1);
        s1 = fmaf(q[c + 1].z, k1v.z, s1); s1 = fmaf(q[c + 1].w, k1v.w, s1);
      }
      sc[j] = j < n ? s0 + s1 : -INFINITY;
      mx = fmaxf(mx, sc[j]);
    }
    const float corr = __expf(m - mx);  // (m = -inf on the first tile: 0)
    l *= corr;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      acc[c].x *= corr; acc[c].y *= corr; acc[c].z *= corr; acc[c].w *= corr;
    }
#pragma unroll
    for (int j = 0; j < AE_KT; ++j) {
      const float p = __expf(sc[j] - mx);
      l += p;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const float4 v = Vs[j][c];
        acc[c].x = fmaf(p, v.x, acc[c].x); acc[c].y = fmaf(p, v.y, acc[c].y);
        acc[c].z = fmaf(p, v.z, acc[c].z); acc[c].w = fmaf(p, v.w, acc[c].w);
      }
    }
    m = mx;
  }
  if (i < S) {
    const float inv = 1.0f / l;
    float4* o = (float4*)(out + ((size_t)b * S + i) * D + h * 64);
#pragma unroll
    for (int c = 0; c < 16; ++c) o[c] = make_float4(acc[c].x * inv, acc[c].y * inv, acc[c].z * inv, acc[c].w * inv);
  }
}

extern "C" int tw_attn_encoder_f32(const float* qkv, int B, int S, int H, float* out, void* stream) {
  TW_REQUIRE(qkv && out && B > 0 && S > 0 && H > 0 && ((uintptr_t)qkv & 15) == 0 && ((uintptr_t)out & 15) == 0,
             "tw_attn_encoder_f32: bad args");
  hipLaunchKernelGGL(k_attn_encoder_f32, dim3(tw_cdiv(S, 64), H, B), dim3(64), 0, (hipStream_t)stream, qkv, S, H, out);
  return tw_check_launch("tw_attn_encoder_f32");
}

// ------------------------------------------------------------------------------------------------
// Decoder attention for one query per (row, head), f32: 256 threads; scores by groups of 16 lanes (one key per group,
// a float4 of q per lane, 16-lane shuffle reduction: coalesced 256-byte key rows), softmax over the block, then
// p . V by 4 key phases x 64 dims (coalesced value rows) and an LDS reduction.
//   self  (kc != null): keys ks .. pos[b] of the row's cache (history through kv_tab when given, the step's own key
//         from qkv), the step's k / v written to the cache at pos[b]; q = qkv[b][h*64..], k / v at +D / +2D
//   cross (kc == null): keys 0 .. S-1 of cross_kv [2][Bt][H][S][64], row b reading slot row_map[b]; q = q[b][h*64..]
// ------------------------------------------------------------------------------------------------
#define DF_MAXK 2048
struct DecAttnF32 {
  const float* q;  // self: qkv [B][3D]; cross: q [B][D]
  int q_ld;
  int H, S, max_pos, Bt;
  const int* pos;
  float* kc;
  float* vc;
  const int* kv_tab;
  int row0;
  const int* kv_start;
  const float* cross_kv;
  const int* row_map;
  float* out;
  // alignment heads (cross only): probs [B][n_steps][n_slots][S]
  float* probs;
  unsigned head_mask;
  int slot0, n_slots, pos0, n_steps;
};

__global__ __launch_bounds__(256) void k_attn_decode_f32(DecAttnF32 p) {
  __shared__ float sc[DF_MAXK];
  __shared__ float part[4][64];
  __shared__ float red[8];
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int H = p.H, D = H * 64;
  const bool self = p.kc != nullptr;
  const float* qrow = p.q + (size_t)b * p.q_ld + h * 64;
  int k_lo = 0, n_keys;
  const float *K = nullptr, *V = nullptr, *knew = nullptr, *vnew = nullptr;
  long row_stride = 0;
  int t = 0;
  if (self) {
    t = p.pos[b];
    n_keys = t + 1;
    if (p.kv_start) {
      const int ks = p.kv_start[b];
      k_lo = t >= ks ? ks : 0;
    }
    K = p.kc + ((size_t)b * H + h) * p.max_pos * 64;
    V = p.vc + ((size_t)b * H + h) * p.max_pos * 64;
    row_stride = (long)H * p.max_pos * 64;
    knew = qrow + D;
    vnew = qrow + 2 * D;
  } else {
    n_keys = p.S;
    const int slot = p.row_map ? p.row_map[b] : b;
    K = p.cross_kv + ((size_t)slot * H + h) * p.S * 64;
    V = p.cross_kv + (((size_t)p.Bt + slot) * H + h) * p.S * 64;
  }
  auto key_row = [&](const float* base, const float* cur, int j) -> const float* {
    if (self && j == t) return cur;
    if (self && p.kv_tab) return base + (long)(p.kv_tab[(size_t)(p.row0 + b) * p.max_pos + j] - (p.row0 + b)) * row_stride + (size_t)j * 64;
    return base + (size_t)j * 64;
  };
  // scores: group g of 16 lanes takes keys k_lo + g, + 16, ...
  const int g = tid >> 4, gl = tid & 15;
  const float4 qv = ((const float4*)qrow)[gl];
  float mx = -INFINITY;
  for (int j = k_lo + g; j < n_keys; j += 16) {
    const float4 kv = ((const float4*)key_row(K, knew, j))[gl];
    float s = qv.x * kv.x + qv.y * kv.y + qv.z * kv.z + qv.w * kv.w;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
    if (gl == 0) sc[j - k_lo] = s;
    mx = fmaxf(mx, s);
  }
  if (self && tid < 64) {  // the step's own key / value into the cache (read above from qkv, never from the cache)
    const size_t cell = (((size_t)b * H + h) * p.max_pos + t) * 64 + tid;
    p.kc[cell] = knew[tid];
    p.vc[cell] = vnew[tid];
  }
  mx = wave_max(mx);
  if (lane == 0) red[wid] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int n = n_keys - k_lo;
  float sum = 0.f;
  for (int j = tid; j < n; j += 256) {
    const float e = __expf(sc[j] - mx);
    sc[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  if (lane == 0) red[4 + wid] = sum;
  __syncthreads();
  const float inv = 1.0f / ((red[4] + red[5]) + (red[6] + red[7]));
  // p . V: wave w takes keys w, w + 4, ...; lane = dim
  float a = 0.f;
  for (int j = wid; j < n; j += 4) a = fmaf(sc[j], key_row(V, vnew, k_lo + j)[lane], a);
  part[wid][lane] = a;
  __syncthreads();
  if (tid < 64) p.out[(size_t)b * D + h * 64 + tid] = ((part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid])) * inv;
  if (p.probs && ((p.head_mask >> h) & 1u)) {
    const int step = p.pos[b] - p.pos0;
    if (step >= 0 && step < p.n_steps) {
      const int sl = p.slot0 + __popc(p.head_mask & ((1u << h) - 1u));
      float* dst = p.probs + (((size_t)b * p.n_steps + step) * p.n_slots + sl) * p.S;
      for (int j = tid; j < n; j += 256) dst[j] = sc[j] * inv;
    }
  }
}

extern "C" int tw_attn_decode_self_f32(const float* qkv, int B, int H, int max_pos, const int* pos, float* k_cache,
                                       float* v_cache, const int* kv_tab, int row0, const int* kv_start, float* out,
                                       void* stream) {
  TW_REQUIRE(qkv && pos && k_cache && v_cache && out && B > 0 && H > 0 && H <= 32 && max_pos > 0 &&
                 max_pos <= DF_MAXK && row0 >= 0,
             "tw_attn_decode_self_f32: bad args (max_pos <= %d)", DF_MAXK);
  DecAttnF32 p{};
  p.q = qkv;
  p.q_ld = 3 * H * 64;
  p.H = H;
  p.max_pos = max_pos;
  p.pos = pos;
  p.kc = k_cache;
  p.vc = v_cache;
  p.kv_tab = kv_tab;
  p.row0 = row0;
  p.kv_start = kv_start;
  p.out = out;
  hipLaunchKernelGGL(k_attn_decode_f32, dim3(H, B), dim3(256), 0, (hipStream_t)stream, p);
  return tw_check_launch("tw_attn_decode_self_f32");
}

extern "C" int tw_attn_decode_cross_f32(const float* q, int B, int H, int S, int Bt, const int* row_map,
                                        const float* cross_kv, float* out, float* probs, unsigned head_mask, int slot0,
                                        int n_slots, const int* pos, int pos0, int n_steps, void* stream) {
  TW_REQUIRE(q && cross_kv && out && B > 0 && H > 0 && H <= 32 && S > 0 && S <= DF_MAXK && Bt > 0 &&
                 (row_map || B <= Bt),
             "tw_attn_decode_cross_f32: bad args (S <= %d)", DF_MAXK);
  TW_REQUIRE(!probs || (pos && n_steps > 0 && slot0 >= 0 && slot0 + __builtin_popcount(head_mask) <= n_slots),
             "tw_attn_decode_cross_f32: bad alignment-head arguments");
  DecAttnF32 p{};
  p.q = q;
  p.q_ld = H * 64;
  p.H = H;
  p.S = S;
  p.Bt = Bt;
  p.cross_kv = cross_kv;
  p.row_map = row_map;
  p.out = out;
  p.probs = probs;
  p.head_mask = head_mask;
  p.slot0 = slot0;
  p.n_slots = n_slots;
  p.pos = pos;
  p.pos0 = pos0;
  p.n_steps = n_steps;
  hipLaunchKernelGGL(k_attn_decode_f32, dim3(H, B), dim3(256), 0, (hipStream_t)stream, p);
  return tw_check_launch("tw_attn_decode_cross_f32");
}
