// bf16 "NT" GEMM on MFMA: C[M][N] = A[M][K] . W[N][K]^T with fused Whisper epilogues.
//
// Replaces every nn.Linear / Conv1d-as-GEMM of the Whisper encoder and decoder
// ($TF/models/whisper/modeling_whisper.py:279-282 q/k/v/o, :375-376 fc1/fc2, :566-567 conv stem,
// :970 proj_out) with one CDNA4 kernel family. W keeps PyTorch's Linear layout [out][in] so both
// operands are K-contiguous: each MFMA lane fragment is one 16-byte run of a row.
//
// Large-M path (encoder, cross-KV projection, conv stem): 128x128x64 tile, 4 waves (2x2), each wave
// a 64x64 sub-tile = 2x2 v_mfma_f32_32x32x16_bf16 accumulators. Register-staged double-buffered LDS
// (issue the next tile's global loads before the MFMAs, write them after), XOR-swizzled 16-B chunks
// (chunk ^ (row & 7)) so ds_read_b128 fragment reads spread over the bank row, XCD-aware block remap
// so the blocks of one A row-panel share an XCD's L2.
//
// Skinny path (decoder, M <= 32 rows): one wave owns 16 output columns and a K-slice; the 4 waves of a
// block split K and reduce through LDS; weights are streamed straight to VGPRs (each weight byte is
// read exactly once per step) with v_mfma_f32_16x16x32_bf16.
#include "tw_common.h"
#include "../../include/tw_whisper.h"

struct EpiArgs {
  void* out;
  int ldo;
  const float* bias;  // [N] or null
  const float* aux;   // EPI_GELU_POS_F32: positional table [aux_rows][N]
  int aux_rows;
  int kv_S, kv_B, kv_D, kv_H;  // EPI_CROSSKV scatter geometry
};

template <int EPI>
__device__ inline void epi_store(const EpiArgs& ea, int m, int n, float v) {
  if (ea.bias) v += ea.bias[n];
  if constexpr (EPI == TW_EPI_BF16) {
    ((bf16_t*)ea.out)[(size_t)m * ea.ldo + n] = f32_to_bf16(v);
  } else if constexpr (EPI == TW_EPI_GELU_BF16) {
    ((bf16_t*)ea.out)[(size_t)m * ea.ldo + n] = f32_to_bf16(gelu_erf(v));
  } else if constexpr (EPI == TW_EPI_RESID_F32) {
    float* o = (float*)ea.out + (size_t)m * ea.ldo + n;
    *o = *o + v;
  } else if constexpr (EPI == TW_EPI_GELU_POS_F32) {
    ((float*)ea.out)[(size_t)m * ea.ldo + n] = gelu_erf(v) + ea.aux[(size_t)(m % ea.aux_rows) * ea.ldo + n];
  } else if constexpr (EPI == TW_EPI_F32) {
    ((float*)ea.out)[(size_t)m * ea.ldo + n] = v;
  } else if constexpr (EPI == TW_EPI_CROSSKV) {
    // n spans [layer][k|v][D]; m spans [b][s]. Output layout [layer][kv][b][head][s][64].
    const int D = ea.kv_D, S = ea.kv_S;
    int l = n / (2 * D), rem = n - l * 2 * D;
    int kv = rem / D, hd = rem - kv * D;
    int h = hd >> 6, d = hd & 63;
    int b = m / S, s = m - b * S;
    size_t idx = ((((size_t)(l * 2 + kv) * ea.kv_B + b) * ea.kv_H + h) * S + s) * 64 + d;
    ((bf16_t*)ea.out)[idx] = f32_to_bf16(v);
  }
}

// ------------------------------------------------------------------------------------------------
// Large-M tile kernel
// ------------------------------------------------------------------------------------------------
#define G_BM 128
#define G_BN 128
#define G_BK 64

__device__ inline int lds_off(int row, int kc) { return row * G_BK + ((kc ^ (row & 7)) << 3); }

template <int EPI>
__global__ __launch_bounds__(256, 2) void k_gemm_tile(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                      int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * 2 * G_BM * G_BK];  // [buf][A|W][128*64]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + G_BM - 1) / G_BM, ntn = (N + G_BN - 1) / G_BN;
  const int nwg = ntm * ntn;
  // XCD-aware bijective remap: blocks b, b+8, ... (one XCD under round-robin dispatch) get
  // consecutive tile ids, so the tiles of one A row-panel are served by one L2.
  const int orig = blockIdx.x;
  const int q = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
  const int tm = wgid / ntn, tn = wgid - tm * ntn;
  const int m0 = tm * G_BM, n0 = tn * G_BN;

  // staging assignment: 4 chunks of A + 4 chunks of W per thread (16 B each)
  const bf16_t* ga[4];
  const bf16_t* gw[4];
  int so[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int c = tid + 256 * i;
    int row = c >> 3, kc = c & 7;
    int am = min(m0 + row, M - 1), wn = min(n0 + row, N - 1);
    ga[i] = A + (size_t)am * lda + kc * 8;
    gw[i] = W + (size_t)wn * ldw + kc * 8;
    so[i] = lds_off(row, kc);
  }
  uint4 ra[4], rw[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = *(const uint4*)(ga[i] + k0);
      rw[i] = *(const uint4*)(gw[i] + k0);
    }
  };
  auto sstore = [&](int buf) {
    bf16_t* As = smem + buf * 2 * G_BM * G_BK;
    bf16_t* Ws = As + G_BM * G_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *(uint4*)(As + so[i]) = ra[i];
      *(uint4*)(Ws + so[i]) = rw[i];
    }
  };

  const int wr = wid >> 1, wc = wid & 1;
  const int lr = lane & 31, lh = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0};

  const int nk = K / G_BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * G_BK);
    const bf16_t* As = smem + cur * 2 * G_BM * G_BK;
    const bf16_t* Ws = As + G_BM * G_BK;
#pragma unroll
    for (int s = 0; s < G_BK / 16; ++s) {
      const int kc = 2 * s + lh;
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        int row = wr * 64 + i * 32 + lr;
        af[i] = *(const bf16x8*)(As + lds_off(row, kc));
        int col = wc * 64 + i * 32 + lr;
        bfr[i] = *(const bf16x8*)(Ws + lds_off(col, kc));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wc * 64 + j * 32 + lr;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) epi_store<EPI>(ea, m, n, acc[i][j][r]);
      }
    }
}

// ------------------------------------------------------------------------------------------------
// Skinny kernel (M <= 32): weight streaming GEMV-like MFMA
// ------------------------------------------------------------------------------------------------
// Block = 4 waves = 16 output columns. Wave w handles the K range [w*K/4, (w+1)*K/4) for two
// 16-row M tiles (rows 0..15 and 16..31) with v_mfma_f32_16x16x32_bf16:
//   A lane l: A[row = l&15][k = 8(l>>4)+j]   B lane l: W[col = l&15][k = 8(l>>4)+j]
//   C lane l: col = l&15, row = (l>>4)*4 + reg
template <int EPI>
__global__ __launch_bounds__(256) void k_gemm_skinny(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                     int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  __shared__ float red[4][32][17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n0 = blockIdx.x * 16;
  const int kq = K / 4;               // K % 128 == 0 guaranteed by host
  const int kb = wid * kq;
  const int col = min(n0 + (lane & 15), N - 1);
  const int ksub = 8 * (lane >> 4);
  const int ar0 = min(lane & 15, M - 1), ar1 = min(16 + (lane & 15), M - 1);
  const bf16_t* wp = W + (size_t)col * ldw + kb + ksub;
  const bf16_t* ap0 = A + (size_t)ar0 * lda + kb + ksub;
  const bf16_t* ap1 = A + (size_t)ar1 * lda + kb + ksub;
  f32x4 c0 = {0}, c1 = {0};
  const bool two = M > 16;
#pragma unroll 4
  for (int k = 0; k < kq; k += 32) {
    bf16x8 bw = *(const bf16x8*)(wp + k);
    bf16x8 a0 = *(const bf16x8*)(ap0 + k);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw, c0, 0, 0, 0);
    if (two) {
      bf16x8 a1 = *(const bf16x8*)(ap1 + k);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw, c1, 0, 0, 0);
    }
  }
  const int cc = lane & 15, rb = (lane >> 4) * 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[wid][rb + r][cc] = c0[r];
    red[wid][16 + rb + r][cc] = c1[r];
  }
  __syncthreads();
  for (int e = tid; e < 32 * 16; e += 256) {
    int m = e >> 4, c = e & 15;
    int n = n0 + c;
    if (m < M && n < N) {
      float v = red[0][m][c] + red[1][m][c] + red[2][m][c] + red[3][m][c];
      epi_store<EPI>(ea, m, n, v);
    }
  }
}

template <int EPI>
static int launch_gemm(const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldw, const EpiArgs& ea,
                       hipStream_t s) {
  if (M <= 32 && K % 128 == 0) {
    hipLaunchKernelGGL(k_gemm_skinny<EPI>, dim3(tw_cdiv(N, 16)), dim3(256), 0, s, A, W, M, N, K, lda, ldw, ea);
  } else {
    unsigned nwg = tw_cdiv(M, G_BM) * tw_cdiv(N, G_BN);
    hipLaunchKernelGGL(k_gemm_tile<EPI>, dim3(nwg), dim3(256), 0, s, A, W, M, N, K, lda, ldw, ea);
  }
  return tw_check_launch("tw_gemm_bf16");
}

extern "C" int tw_gemm_bf16(const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldw, int epi,
                            void* out, int ldo, const float* bias, const float* aux, int aux_rows,
                            const int* kv_geom, void* stream) {
  TW_REQUIRE(A && W && out, "tw_gemm_bf16: null pointer");
  TW_REQUIRE(M > 0 && N > 0 && K > 0 && K % G_BK == 0, "tw_gemm_bf16: M=%d N=%d K=%d (K %% 64 required)", M, N, K);
  TW_REQUIRE(lda % 8 == 0 && ldw % 8 == 0 && lda >= K && ldw >= K, "tw_gemm_bf16: lda=%d ldw=%d", lda, ldw);
  EpiArgs ea{out, ldo, bias, aux, aux_rows, 0, 0, 0, 0};
  hipStream_t s = (hipStream_t)stream;
  switch (epi) {
    case TW_EPI_BF16: return launch_gemm<TW_EPI_BF16>(A, W, M, N, K, lda, ldw, ea, s);
    case TW_EPI_GELU_BF16: return launch_gemm<TW_EPI_GELU_BF16>(A, W, M, N, K, lda, ldw, ea, s);
    case TW_EPI_RESID_F32: return launch_gemm<TW_EPI_RESID_F32>(A, W, M, N, K, lda, ldw, ea, s);
    case TW_EPI_GELU_POS_F32:
      TW_REQUIRE(aux && aux_rows > 0, "tw_gemm_bf16: GELU_POS needs aux table");
      return launch_gemm<TW_EPI_GELU_POS_F32>(A, W, M, N, K, lda, ldw, ea, s);
    case TW_EPI_F32: return launch_gemm<TW_EPI_F32>(A, W, M, N, K, lda, ldw, ea, s);
    case TW_EPI_CROSSKV:
      TW_REQUIRE(kv_geom != nullptr, "tw_gemm_bf16: CROSSKV needs kv_geom {S,B,D,H}");
      ea.kv_S = kv_geom[0]; ea.kv_B = kv_geom[1]; ea.kv_D = kv_geom[2]; ea.kv_H = kv_geom[3];
      TW_REQUIRE(ea.kv_S * ea.kv_B == M && N % (2 * ea.kv_D) == 0 && ea.kv_H * 64 == ea.kv_D,
                 "tw_gemm_bf16: CROSSKV geometry mismatch");
      return launch_gemm<TW_EPI_CROSSKV>(A, W, M, N, K, lda, ldw, ea, s);
    default: tw_set_error("tw_gemm_bf16: unknown epilogue %d", epi); return TW_ERR_ARG;
  }
}
