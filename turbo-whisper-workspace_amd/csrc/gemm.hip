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
#include <algorithm>
#include <type_traits>

#include "tw_common.h"
#include "../../include/tw_whisper.h"

struct EpiArgs {
  void* out;
  int ldo;
  const float* bias;  // [N] or null
  const float* aux;   // EPI_GELU_POS_F32: positional table [aux_rows][N]
  int aux_rows;
  int kv_S, kv_B, kv_D, kv_H;  // EPI_CROSSKV scatter geometry
  uint8_t* sout;      // EPI_GELU_MX: e8m0 scales of the fp8 output, [N/128][s_rows][4]
  int s_rows;
  int group_m;        // large-M kernels: tile rows per group of the tile order (tw_tile_grouped); <= 1 row-major
  float* stats;       // TW_EPI_RESID_STATS: per-16-column-group row statistics of the updated rows (tw_gemv_packed_stats)
};

// Tile (tm, tn) of tile id `wgid` (after the XCD remap, which hands each XCD a contiguous id range) in grouped
// order: groups of gm tile rows, walked down the group's rows first. The ~32 tiles one XCD runs at once then span
// gm A row panels x 32/gm W column panels instead of 1 x 32, so each K-step's operand slices are shared by more
// of the XCD's CUs through its L2 (row-major order re-streams every W panel once per A row panel).
__device__ inline void tw_tile_grouped(int wgid, int ntm, int ntn, int gm, int& tm, int& tn) {
  if (gm <= 1) {
    tm = wgid / ntn;
    tn = wgid - tm * ntn;
    return;
  }
  const int per = gm * ntn, g = wgid / per, first = g * gm;
  const int rows = min(ntm - first, gm), l = wgid - g * per;
  tm = first + l % rows;
  tn = l / rows;
}

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
  int tm, tn;
  tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
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

// Large-M kernel selection (tw_gemm_set_variant, for A/B measurement): 1 = k_gemm_big (256x256, 2-stage BK=64
// LDS-DMA; default), 0 = k_gemm_tile (128x128 register-staged), 3 = k_gemm_ns<256, 2 stages> (counted vmcnt,
// raw barrier, setprio), 4 = k_gemm_ns<BN=128, 3 stages>. Measured on the encoder shapes (scripts/gemm_bench.py,
// random operands): 1 ~ 3 (641-1079 TF/s), 4 is 12-18% slower, a 4-stage BK=32 ring was 6% slower.
static int tw_gemm_big_enabled = 1;
// tw_tile_grouped rows per group for the large-M kernels (tw_gemm_set_group; 0 = by shape). Measured
// (scripts/gemm_bench.py, M = 36000, groups 1/4/8/16): 8 gains 2-7 % on the wide-N shapes (q/k/v, fc1, cross-K/V:
// >= 15 column tiles), while the 5-column-tile shapes (o_proj, fc2, conv2) are best row-major.
static int tw_gemm_group_m = 0;
extern "C" int tw_gemm_set_group(int gm) {
  tw_gemm_group_m = gm < 0 ? 0 : (gm > 64 ? 64 : gm);
  return 0;
}
static inline int tw_group_for(int N) {
  if (tw_gemm_group_m > 0) return tw_gemm_group_m;
  return (N + 255) / 256 >= 10 ? 8 : 1;
}
// packed GEMVs with N >= this (proj_out) read their weights non-temporally: bench step -1 ms (109.2 vs 110.3)
static int tw_gemv_nt_min_n = 16384;
#ifndef TW_PROJ_PAIRS_DEFAULT
#define TW_PROJ_PAIRS_DEFAULT 0
#endif
#ifndef TW_PROJ_KW_DEFAULT
#define TW_PROJ_KW_DEFAULT 1
#endif
static int tw_tune_skinny_nw = 0;  // 0 = heuristic; 4 / 8 / 16 force the skinny kernel's waves per block
static int tw_tune_gemv_kw = 0;    // 0 = heuristic; 1 / 2 / 4 / 8 force the packed GEMV's K-slices per column group
static int tw_proj_kw = TW_PROJ_KW_DEFAULT;  // K-slices per column group of the vocabulary-wide proj_out (1 / 2 / 4)
// the decoder's layer GEMVs as k_gemv_pc (two column groups per wave). Measured in the bench (three interleaved pairs,
// 10 steps): 91.8 vs 92.4 ms, the encoder GEMM beside the decode 785 vs 781 TF/s (fewer decoder vector-memory
// instructions in its CUs); per launch in situ equal (11.6 vs 11.3 us). tw_gemm_set_variant bit 28: k_gemv_p (A/B).
static int tw_gemv_pairs = 1;
static int tw_proj_pairs = TW_PROJ_PAIRS_DEFAULT;  // proj_out as k_gemv_pc with one K-slice (tw_gemm_set_variant bit 29)
// Largest K-slice count the packed-GEMV heuristic picks. 4 = at most 256-thread workgroups: one decoder wave per SIMD
// then co-resides with an encoder GEMM workgroup (2 waves of ~190 VGPRs on every SIMD), where a 512-thread decoder
// workgroup waits for GEMM workgroups to retire (scripts/exp/interference.py, q/k/v GEMV beside k_gemm_8p: 33.6 us per
// launch at KW = 8, 11.5 at KW = 4; alone 3.3 vs 3.6 us). With the batched GEMV loads (k_gemv_p) the bench step went
// 104.3 -> 99.9 ms (two interleaved pairs; scripts/exp/insitu_breakdown.py: the GEMVs of a decode step beside an encoder
// GEMM +239 us at KW = 8, +128 us at KW = 4). 8 = the round-1 heuristic (A/B).
static int tw_gemv_max_kw = 4;
extern "C" int tw_gemv_set_max_kw(int kw) {
  tw_gemv_max_kw = (kw == 1 || kw == 2 || kw == 4 || kw == 8) ? kw : 4;
  return 0;
}
extern "C" int tw_gemm_set_variant(int big) {
  tw_gemm_big_enabled = big & 15;
  const int nw = (big >> 8) & 0xff;
  tw_tune_skinny_nw = (nw == 4 || nw == 8 || nw == 16) ? nw : 0;
  tw_gemv_nt_min_n = (big & 0x1000000) ? (1 << 30) : 16384;  // bit 24: proj_out weights through the caches (A/B)
  tw_gemv_pairs = ((big >> 28) & 1) ? 0 : 1;
  tw_proj_pairs = ((big >> 29) & 1) ? !TW_PROJ_PAIRS_DEFAULT : TW_PROJ_PAIRS_DEFAULT;  // bit 29: the other proj_out form
  {  // bits 26-27: proj_out K-slices (0: the default, 1: 1, 2: 2, 3: 4)
    const int pk = (big >> 26) & 3;
    tw_proj_kw = pk == 0 ? TW_PROJ_KW_DEFAULT : (pk == 1 ? 1 : (pk == 2 ? 2 : 4));
  }
  const int kw = (big >> 16) & 0xff;
  tw_tune_gemv_kw = (kw == 1 || kw == 2 || kw == 4 || kw == 8) ? kw : 0;
  return 0;
}

// ------------------------------------------------------------------------------------------------
// Large-M kernel, 256 x 256 x 64 tiles (encoder projections, FFN, conv stem, cross-K/V)
// ------------------------------------------------------------------------------------------------
// 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128 x 64 sub-tile = 8 x 4 accumulators of
// v_mfma_f32_16x16x32_bf16 (128 accumulator registers). One workgroup per CU (128 KiB LDS: two
// buffers of the A and W tiles). Tiles are staged HBM/L2 -> LDS by global_load_lds_dwordx4 (LDS-DMA,
// no VGPR round trip): one wave-instruction moves 8 rows x 128 B; the LDS image is lane-linear, so the
// bank swizzle is applied on the SOURCE chunk (chunk ^ swz(row)) and undone on the ds_read_b128
// address (same involution). swz(r) = (r >> 1) & 7 makes every 16x16x32 fragment read conflict-free.
// K loop: issue tile t+1's DMA, run tile t's 64 MFMAs per wave, then one vmcnt(0) + barrier.
// Epilogue: accumulators go through LDS (64-row halves, padded rows) so every global load/store of the
// fused epilogue (bias, GELU, residual f32 read-modify-write, positional add, cross-K/V scatter) is a
// 16-byte (f32) or 8-byte (bf16) access of 4 consecutive columns.
#define GB_BM 256
#define GB_BN 256
#define GB_BK 64
#ifndef GB_XKV_NT
#define GB_XKV_NT 0  // 1: the cross-K/V epilogue stores non-temporally (experiment build)
#endif
#ifndef GB_A_POL
#define GB_A_POL 0  // cache policy of k_gemm_big's activation-operand DMA (experiment builds: 2 = nt)
#endif
#ifndef GB_BIG_PADV
#define GB_BIG_PADV 0
#endif
#define GB_EPI_LD 68  // f32 row stride of the epilogue staging image (64 + 4: conflict-free writes)

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ inline int gb_swz(int r) { return (r >> 1) & 7; }

// epilogue of 4 consecutive columns n..n+3 of row m (v already includes the bias)
// TW_ENC_NT producer bit of a large-M GEMM epilogue
constexpr int gb_nt_bit(int epi) {
  return epi == TW_EPI_BF16 ? TW_NT_GEMM_BF16 : epi == TW_EPI_GELU_BF16 ? TW_NT_GEMM_GELU
         : epi == TW_EPI_RESID_F32 ? TW_NT_GEMM_RESID : TW_NT_GEMM_OTHER;
}

template <int EPI>
__device__ inline void epi_store4(const EpiArgs& ea, int m, int n, int N, float4 v) {
  if (n + 3 >= N) {  // ragged right edge (tests only: the model's N are multiples of 256)
    const float t[4] = {v.x, v.y, v.z, v.w};
    EpiArgs e2 = ea;
    e2.bias = nullptr;
    for (int q = 0; q < 4; ++q)
      if (n + q < N) epi_store<EPI>(e2, m, n + q, t[q]);
    return;
  }
  if constexpr (EPI == TW_EPI_BF16 || EPI == TW_EPI_GELU_BF16) {
    if constexpr (EPI == TW_EPI_GELU_BF16) v = gelu_erf4(v);
    uint2 w;
    w.x = pack_bf16x2(v.x, v.y);
    w.y = pack_bf16x2(v.z, v.w);
    tw_st_enc<gb_nt_bit(EPI)>((bf16_t*)ea.out + (size_t)m * ea.ldo + n, w);
  } else if constexpr (EPI == TW_EPI_RESID_F32) {
    float4* o = (float4*)((float*)ea.out + (size_t)m * ea.ldo + n);
    float4 x = *o;
    x.x += v.x; x.y += v.y; x.z += v.z; x.w += v.w;
    tw_st_enc<gb_nt_bit(EPI)>(o, x);
  } else if constexpr (EPI == TW_EPI_GELU_POS_F32) {
    const float4 a = *(const float4*)(ea.aux + (size_t)(m % ea.aux_rows) * ea.ldo + n);
    float4 o = gelu_erf4(v);
    o.x += a.x; o.y += a.y; o.z += a.z; o.w += a.w;
    tw_st_enc<gb_nt_bit(EPI)>((float*)ea.out + (size_t)m * ea.ldo + n, o);
  } else if constexpr (EPI == TW_EPI_F32) {
    tw_st_enc<gb_nt_bit(EPI)>((float*)ea.out + (size_t)m * ea.ldo + n, v);
  } else if constexpr (EPI == TW_EPI_CROSSKV) {
    const int D = ea.kv_D, S = ea.kv_S;
    int l = n / (2 * D), rem = n - l * 2 * D;
    int kv = rem / D, hd = rem - kv * D;
    int h = hd >> 6, d = hd & 63;
    int b = m / S, s = m - b * S;
    size_t idx = ((((size_t)(l * 2 + kv) * ea.kv_B + b) * ea.kv_H + h) * S + s) * 64 + d;
    uint2 w;
    w.x = pack_bf16x2(v.x, v.y);
    w.y = pack_bf16x2(v.z, v.w);
    tw_st_enc<gb_nt_bit(EPI)>((bf16_t*)ea.out + idx, w);
  }
}

// the second f32 operand of a RESID / GELU_POS epilogue for 4 columns n..n+3 of row m (zeros when the group is
// ragged: that path re-reads it element-wise in epi_store4)
template <int EPI>
__device__ inline float4 epi_addend(const EpiArgs& ea, int m, int n, bool full) {
  if (!full) return make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (EPI == TW_EPI_RESID_F32) return *(const float4*)((const float*)ea.out + (size_t)m * ea.ldo + n);
  else return *(const float4*)(ea.aux + (size_t)(m % ea.aux_rows) * ea.ldo + n);
}
// epi_store4 for a full group whose second operand `a` was loaded ahead
template <int EPI>
__device__ inline void epi_store4_pre(const EpiArgs& ea, int m, int n, float4 v, float4 a) {
  if constexpr (EPI == TW_EPI_GELU_POS_F32) v = gelu_erf4(v);
  v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
  tw_st_enc<gb_nt_bit(EPI)>((float*)ea.out + (size_t)m * ea.ldo + n, v);
}

// epilogue of 8 consecutive columns n..n+7 of row m (v already includes the bias): one 16-byte store for the bf16
// outputs (a wave's epilogue is store-issue bound: half the instructions of two 8-byte stores)
template <int EPI>
__device__ inline void epi_store8(const EpiArgs& ea, int m, int n, int N, float4 v0, float4 v1) {
  if constexpr (EPI == TW_EPI_BF16 || EPI == TW_EPI_GELU_BF16 || EPI == TW_EPI_CROSSKV) {
    if (n + 7 < N) {
      if constexpr (EPI == TW_EPI_GELU_BF16) {
        v0 = gelu_erf4(v0);
        v1 = gelu_erf4(v1);
      }
      uint4 w;
      w.x = pack_bf16x2(v0.x, v0.y);
      w.y = pack_bf16x2(v0.z, v0.w);
      w.z = pack_bf16x2(v1.x, v1.y);
      w.w = pack_bf16x2(v1.z, v1.w);
      size_t idx;
      if constexpr (EPI == TW_EPI_CROSSKV) {  // 8 | 64: the group stays inside one head's 64 contiguous dims
        const int D = ea.kv_D, S = ea.kv_S;
        int l = n / (2 * D), rem = n - l * 2 * D;
        int kv = rem / D, hd = rem - kv * D;
        int h = hd >> 6, d = hd & 63;
        int b = m / S, s2 = m - b * S;
        idx = ((((size_t)(l * 2 + kv) * ea.kv_B + b) * ea.kv_H + h) * S + s2) * 64 + d;
#if GB_XKV_NT
        // the cross K/V cache is read back only by the decoder's non-temporal loads: write it past the caches too
        typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
        const u32x4_nt wv = {w.x, w.y, w.z, w.w};
        __builtin_nontemporal_store(wv, (u32x4_nt*)((bf16_t*)ea.out + idx));
        return;
#endif
      } else {
        idx = (size_t)m * ea.ldo + n;
      }
      tw_st_enc<gb_nt_bit(EPI)>((bf16_t*)ea.out + idx, w);
      return;
    }
  }
  epi_store4<EPI>(ea, m, n, N, v0);
  if (n + 4 < N) epi_store4<EPI>(ea, m, n + 4, N, v1);
}

#ifndef GB_EPI_BLOCKSYNC
#define GB_EPI_BLOCKSYNC 0  // 1: block barriers around the epilogue staging (the round-1 form; A/B builds)
#endif
// Ordering between a wave's own epilogue-image writes and reads: every wave stages through its own LDS region, and
// LDS instructions of one wave execute in issue order, so a compiler fence (plus the LDS count) is enough; block
// barriers here only made the 8 waves of a tile wait for each other (and, beside a running decode step, for the
// wave the decoder's waves slow down most).
#ifndef GB_EPI_WIDE
#define GB_EPI_WIDE 1  // k_gemm_big's bf16 epilogues read back 8 columns per lane (16-byte stores); 0: 4 (A/B)
#endif
__device__ inline void gb_epi_sync() {
  if (GB_EPI_BLOCKSYNC) {
    __syncthreads();
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

// Epilogue of one wave's 128 x 64 sub-tile (rows mw0.., columns ncol0..) held as 8 x 4 16x16 MFMA accumulators,
// through the wave's own [64][GB_EPI_LD] f32 LDS image `wimg` (shared by k_gemm_big and k_gemm_h; every wave of the
// block calls it: it holds block barriers). The caller's K loop must have ended on a barrier.
// stage(half, wimg) writes rows 64 half .. 64 half + 63 of the wave's sub-tile into its [64][GB_EPI_LD] f32 image
template <int EPI, class Stage>
__device__ inline void gemm_epi_128x64_st(Stage stage, float* wimg, int lane, int mw0, int ncol0, int M, int N,
                                          const EpiArgs& ea) {
  // ---- epilogue through LDS: each wave stages 64 of its 128 rows at a time in its own
  // [64][GB_EPI_LD] f32 image (k_gemm_big: 8 images = 136 KiB, the K loop's LDS plus 8 KiB), then reads
  // back 4 consecutive columns per lane (16 lanes x 16 B per row) for vectorised global I/O.
  const int rc = (lane & 15) * 4;  // this lane's 4 columns in the read-back phase
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ea.bias) {
    const int n = ncol0 + rc;
    bias4.x = ea.bias[min(n, N - 1)];
    bias4.y = ea.bias[min(n + 1, N - 1)];
    bias4.z = ea.bias[min(n + 2, N - 1)];
    bias4.w = ea.bias[min(n + 3, N - 1)];
  }
  // epilogues that read a second f32 operand (RESID: the residual stream it updates in place; GELU_POS: the
  // positional table) load it ahead: rows rr and rr + 8 of a half share a register slot, so a half costs two
  // dependent HBM round trips instead of sixteen (the compiler cannot hoist a load above the previous row's store
  // to the same buffer), and the first eight loads fly while the accumulators are staged through LDS.
  constexpr bool PRE = EPI == TW_EPI_RESID_F32 || EPI == TW_EPI_GELU_POS_F32;
  const bool full = ncol0 + rc + 3 < N;
  float b8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // (the 8-column read-back's bias)
  if (GB_EPI_WIDE && !PRE && ea.bias) {
#pragma unroll
    for (int q = 0; q < 8; ++q) b8[q] = ea.bias[min(ncol0 + (lane & 7) * 8 + q, N - 1)];
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int ib = 4 * half;
    const int mrow0 = mw0 + ib * 16;
    float4 ad[8];
    if constexpr (PRE) {
#pragma unroll
      for (int q = 0; q < 8; ++q) ad[q] = epi_addend<EPI>(ea, min(mrow0 + q * 4 + (lane >> 4), M - 1), ncol0 + rc, full);
    }
    if (half) gb_epi_sync();  // (first pass: the K loop ended on a barrier)
    stage(half, wimg);
    gb_epi_sync();
    if constexpr (PRE) {
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int lr = rr * 4 + (lane >> 4);  // 4 rows per wave-instruction
        const int m = mrow0 + lr;
        float4 v = *(const float4*)(wimg + lr * GB_EPI_LD + rc);
        v.x += bias4.x; v.y += bias4.y; v.z += bias4.z; v.w += bias4.w;
        if (full) {
          if (m < M) epi_store4_pre<EPI>(ea, m, ncol0 + rc, v, ad[rr & 7]);
        } else if (m < M && ncol0 + rc < N) {
          epi_store4<EPI>(ea, m, ncol0 + rc, N, v);
        }
        if (rr < 8) ad[rr] = epi_addend<EPI>(ea, min(m + 32, M - 1), ncol0 + rc, full);
      }
    } else if constexpr (GB_EPI_WIDE && (EPI == TW_EPI_BF16 || EPI == TW_EPI_GELU_BF16 || EPI == TW_EPI_CROSSKV)) {
      // bf16 outputs: 8 consecutive columns per lane (8 lanes x 32 B per row, 8 rows per wave-instruction), one
      // 16-byte store each: half the store instructions of the 4-column form, and whole 128-byte row segments per
      // 8 lanes for the non-temporal stores (no partial-line write-backs)
      const int rc8 = (lane & 7) * 8;
#pragma unroll 4
      for (int rr = 0; rr < 8; ++rr) {
        const int lr = rr * 8 + (lane >> 3);
        const int m = mrow0 + lr;
        float4 v0 = *(const float4*)(wimg + lr * GB_EPI_LD + rc8);
        float4 v1 = *(const float4*)(wimg + lr * GB_EPI_LD + rc8 + 4);
        v0.x += b8[0]; v0.y += b8[1]; v0.z += b8[2]; v0.w += b8[3];
        v1.x += b8[4]; v1.y += b8[5]; v1.z += b8[6]; v1.w += b8[7];
        if (m < M && ncol0 + rc8 < N) epi_store8<EPI>(ea, m, ncol0 + rc8, N, v0, v1);
      }
    } else {
#pragma unroll 4
      for (int rr = 0; rr < 16; ++rr) {
        const int lr = rr * 4 + (lane >> 4);
        const int m = mrow0 + lr;
        float4 v = *(const float4*)(wimg + lr * GB_EPI_LD + rc);
        v.x += bias4.x; v.y += bias4.y; v.z += bias4.z; v.w += bias4.w;
        if (m < M && ncol0 + rc < N) epi_store4<EPI>(ea, m, ncol0 + rc, N, v);
      }
    }
  }
}

// the 16x16x32 MFMA layout (8 x 4 accumulators of 16 x 16: lane (fr, fq) holds rows 4 fq + r of column fr)
template <int EPI>
__device__ inline void gemm_epi_128x64(const f32x4 (&acc)[8][4], float* wimg, int lane, int mw0, int ncol0, int M,
                                       int N, const EpiArgs& ea) {
  const int fr = lane & 15, fq = lane >> 4;
  auto stage = [&](int half, float* w) {
    const int ib = 4 * half;
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) w[(ii * 16 + fq * 4 + r) * GB_EPI_LD + j * 16 + fr] = acc[ib + ii][j][r];
  };
  gemm_epi_128x64_st<EPI>(stage, wimg, lane, mw0, ncol0, M, N, ea);
}
// the 32x32x16 MFMA layout (4 x 2 accumulators of 32 x 32: lane l holds column l % 32, rows 8 (r / 4) + 4 (l / 32)
// + r % 4 for its 16 registers r)
template <int EPI>
__device__ inline void gemm_epi_128x64_m32(const f32x16 (&acc)[4][2], float* wimg, int lane, int mw0, int ncol0,
                                           int M, int N, const EpiArgs& ea) {
  const int c = lane & 31, h4 = (lane >> 5) * 4;
  auto stage = [&](int half, float* w) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          w[(i2 * 32 + (r >> 2) * 8 + h4 + (r & 3)) * GB_EPI_LD + j * 32 + c] = acc[2 * half + i2][j][r];
  };
  gemm_epi_128x64_st<EPI>(stage, wimg, lane, mw0, ncol0, M, N, ea);
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm_big(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                     int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  // [buf][A | W][256 rows x 64 k] bf16 = 128 KiB for the K loop; 8 x [64][68] f32 = 136 KiB after it
  __shared__ __attribute__((aligned(16))) bf16_t smem[8 * 64 * GB_EPI_LD * 2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + GB_BM - 1) / GB_BM, ntn = (N + GB_BN - 1) / GB_BN;
  const int nwg = ntm * ntn;
  // XCD-aware bijective remap: blocks b, b+8, ... (one XCD under round-robin dispatch) take consecutive
  // tile ids, so the N-tiles of one A row-panel are computed out of one L2.
  const int orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int tm, tn;
  tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
  const int m0 = tm * GB_BM, n0 = tn * GB_BN;

  // DMA assignment: wave w issues instructions i = 0..3 for A and for W; instruction (w, i) fills tile
  // rows 8(4w+i) .. 8(4w+i)+7. Lane l: row 8(4w+i) + (l>>3), LDS chunk slot l&7 <- global chunk
  // (l&7) ^ swz(row).
  const bf16_t* ga[4];
  const bf16_t* gw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wid + i) + (lane >> 3);
    const int ch = (lane & 7) ^ gb_swz(row);
    ga[i] = A + (size_t)min(m0 + row, M - 1) * lda + ch * 8;
    gw[i] = W + (size_t)min(n0 + row, N - 1) * ldw + ch * 8;
  }
  auto stage = [&](int buf, int k0) {
    bf16_t* As = smem + buf * 2 * GB_BM * GB_BK;
    bf16_t* Ws = As + GB_BM * GB_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rb = 8 * (4 * wid + i) * GB_BK;  // wave-uniform LDS base of this instruction
      __builtin_amdgcn_global_load_lds((const void*)(ga[i] + k0), (lds_void_t*)(As + rb), 16, 0, GB_A_POL);
      __builtin_amdgcn_global_load_lds((const void*)(gw[i] + k0), (lds_void_t*)(Ws + rb), 16, 0, 0);
    }
  };

  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / GB_BK;
#if GB_BIG_PADV
  // diagnostic builds only: GB_BIG_PADV dummy registers live across the K loop (co-residency experiments)
  float padv[GB_BIG_PADV];
#pragma unroll
  for (int i = 0; i < GB_BIG_PADV; ++i) padv[i] = (float)(lane * (i + 1));
#pragma unroll
  for (int i = 0; i < GB_BIG_PADV; ++i) asm volatile("" : "+v"(padv[i]));
#endif
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * GB_BK);
    const bf16_t* As = smem + cur * 2 * GB_BM * GB_BK;
    const bf16_t* Ws = As + GB_BM * GB_BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kc = 4 * kk + fq;
      bf16x8 bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wc * 64 + j * 16 + fr;
        bfr[j] = *(const bf16x8*)(Ws + col * GB_BK + ((kc ^ gb_swz(col)) << 3));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = wr * 128 + i * 16 + fr;
        const bf16x8 af = *(const bf16x8*)(As + row * GB_BK + ((kc ^ gb_swz(row)) << 3));
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();  // vmcnt(0) (tile kt+1 landed) + lgkmcnt(0) + barrier
  }
#if GB_BIG_PADV
#pragma unroll
  for (int i = 0; i < GB_BIG_PADV; ++i) asm volatile("" : "+v"(padv[i]));
#endif

  gemm_epi_128x64<EPI>(acc, (float*)smem + wid * (64 * GB_EPI_LD), lane, m0 + wr * 128, n0 + wc * 64, M, N, ea);
}

// k_gemm_big32: k_gemm_big with v_mfma_f32_32x32x16_bf16 (MI355X_MICROARCH / cdna_hip_programming §5.4 rule 28:
// the chip can hold a different clock on the other bf16 MFMA shape; same wave tile, half the MFMA instructions).
// Same LDS image, swizzle, DMA and one barrier per K-step; per 16-deep K substep a wave reads 4 A and 2 B fragments
// (32 rows x 16 k: lane l row l % 32, k chunk 2 kk + l / 32) into 4 x 2 accumulators of 32 x 32.
template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm_big32(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                       int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[8 * 64 * GB_EPI_LD * 2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + GB_BM - 1) / GB_BM, ntn = (N + GB_BN - 1) / GB_BN;
  const int nwg = ntm * ntn;
  const int orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int tm, tn;
  tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
  const int m0 = tm * GB_BM, n0 = tn * GB_BN;
  const bf16_t* ga[4];
  const bf16_t* gw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wid + i) + (lane >> 3);
    const int ch = (lane & 7) ^ gb_swz(row);
    ga[i] = A + (size_t)min(m0 + row, M - 1) * lda + ch * 8;
    gw[i] = W + (size_t)min(n0 + row, N - 1) * ldw + ch * 8;
  }
  auto stage = [&](int buf, int k0) {
    bf16_t* As = smem + buf * 2 * GB_BM * GB_BK;
    bf16_t* Ws = As + GB_BM * GB_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rb = 8 * (4 * wid + i) * GB_BK;
      __builtin_amdgcn_global_load_lds((const void*)(ga[i] + k0), (lds_void_t*)(As + rb), 16, 0, GB_A_POL);
      __builtin_amdgcn_global_load_lds((const void*)(gw[i] + k0), (lds_void_t*)(Ws + rb), 16, 0, 0);
    }
  };
  const int wr = wid >> 2, wc = wid & 3;
  const int lr = lane & 31, lh = lane >> 5;
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0.f};
  const int nk = K / GB_BK;
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * GB_BK);
    const bf16_t* As = smem + cur * 2 * GB_BM * GB_BK;
    const bf16_t* Ws = As + GB_BM * GB_BK;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kc = 2 * kk + lh;
      bf16x8 bfr[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wc * 64 + j * 32 + lr;
        bfr[j] = *(const bf16x8*)(Ws + col * GB_BK + ((kc ^ gb_swz(col)) << 3));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wr * 128 + i * 32 + lr;
        const bf16x8 af = *(const bf16x8*)(As + row * GB_BK + ((kc ^ gb_swz(row)) << 3));
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  gemm_epi_128x64_m32<EPI>(acc, (float*)smem + wid * (64 * GB_EPI_LD), lane, m0 + wr * 128, n0 + wc * 64, M, N, ea);
}

// ------------------------------------------------------------------------------------------------
// k_gemm_kh: k_gemm_big's tile, waves, fragments and epilogue (so the same ~184 VGPRs: beside a running decode step
// every SIMD keeps room for one decoder wave, DESIGN §4 "Round 2") with a deeper DMA pipeline. The LDS image is split
// by K-half: slot (buffer, half) holds the A and W rows of one 32-deep half of a 64-deep K-tile as [256 rows][64 B]
// (chunk swizzle c ^ ((row >> 2) & 3): a ds_read_b128 fragment's 16 rows hit 16 distinct bank groups). The loop runs
// over half-steps u = 2t + h: wait for half u's DMA (counted vmcnt, 2 halves left in flight), one raw barrier, issue
// the DMA of half u + 3 into the slot half u - 1 just released, then 32 MFMAs per wave on half u. A half is issued
// 1.5 K-tiles before it is read (k_gemm_big: one K-tile), at two barriers per K-tile instead of one; no ordinary
// global load sits in the loop, so hipcc's waits stay the counted ones.
// ------------------------------------------------------------------------------------------------
// Buffer descriptor from values the compiler can prove wave-uniform (readfirstlane'd base halves and size): the
// descriptor then lives in SGPRs and every buffer op through it is one instruction, not a waterfall loop.
__device__ inline __amdgpu_buffer_rsrc_t tw_uniform_rsrc(const void* p, int bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ inline int gk_swz(int r) { return (r >> 2) & 3; }

template <int N>
__device__ inline void gk_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm_kh(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  // 4 slots x [A | W][256 rows x 32 k] bf16 = 128 KiB for the K loop; 8 x [64][68] f32 = 136 KiB after it (one array)
  __shared__ __attribute__((aligned(16))) bf16_t smem[8 * 64 * GB_EPI_LD * 2];
  constexpr int SLOT = 2 * GB_BM * 32;  // bf16 elements per slot (A rows, then W rows)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + GB_BM - 1) / GB_BM, ntn = (N + GB_BN - 1) / GB_BN;
  const int nwg = ntm * ntn;
  const int orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int tm, tn;
  tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
  const int m0 = tm * GB_BM, n0 = tn * GB_BN;

  // DMA: per half, wave w issues instructions i = 0, 1 for A and for W; instruction (w, i) fills rows
  // 16 (2w + i) .. + 15 (16 rows x 64 B = 1 KiB). Lane l: row 16 (2w + i) + (l >> 2), LDS chunk slot l & 3 <- global
  // chunk (l & 3) ^ gk_swz(row). Buffer descriptors (rows past M / N read as zeros; never stored) keep the per-lane
  // part a 32-bit offset.
  const __amdgpu_buffer_rsrc_t rsA = tw_uniform_rsrc(A + (size_t)m0 * lda, max(0, min(GB_BM, M - m0)) * lda * 2);
  const __amdgpu_buffer_rsrc_t rsW = tw_uniform_rsrc(W + (size_t)n0 * ldw, max(0, min(GB_BN, N - n0)) * ldw * 2);
  unsigned va[2], vw[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * (2 * wid + i) + (lane >> 2);
    const int ch = (lane & 3) ^ gk_swz(row);
    va[i] = (unsigned)(row * lda + ch * 8) * 2u;
    vw[i] = (unsigned)(row * ldw + ch * 8) * 2u;
  }
  auto issue = [&](int u) {  // DMA of half-step u (K-tile u >> 1, half u & 1) into slot u & 3
    bf16_t* As = smem + (u & 3) * SLOT;
    bf16_t* Ws = As + GB_BM * 32;
    const unsigned ko = (unsigned)(u * 32) * 2u;  // K offset (bytes) of this half
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rb = 16 * (2 * wid + i) * 32;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void_t*)(As + rb), 16, va[i], ko, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (lds_void_t*)(Ws + rb), 16, vw[i], ko, 0, 0);
    }
  };

  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int u) {
    const bf16_t* As = smem + (u & 3) * SLOT;
    const bf16_t* Ws = As + GB_BM * 32;
    bf16x8 bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wc * 64 + j * 16 + fr;
      bfr[j] = *(const bf16x8*)(Ws + col * 32 + ((fq ^ gk_swz(col)) << 3));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr * 128 + i * 16 + fr;
      const bf16x8 af = *(const bf16x8*)(As + row * 32 + ((fq ^ gk_swz(row)) << 3));
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  const int nh = 2 * (K / GB_BK);  // half-steps (the launcher guarantees nh >= 4)
  issue(0);
  issue(1);
  issue(2);
  // one half-step per iteration: half u landed (this wave's DMA by the count, every wave's by the barrier), then the
  // slot of half u - 1 is free for half u + 3. One copy of the body (a peeled tail makes the register allocator copy
  // the accumulators: 244 instead of ~184 VGPRs); the count drops to 4 / 0 on the last two halves (scalar branches).
  for (int u = 0; u < nh; ++u) {
    if (u < nh - 2) gk_vmcnt<8>();
    else if (u == nh - 2) gk_vmcnt<4>();
    else gk_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (u + 3 < nh) issue(u + 3);
    compute(u);
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();  // every wave done with the K-loop slots before the epilogue images reuse them

  gemm_epi_128x64<EPI>(acc, (float*)smem + wid * (64 * GB_EPI_LD), lane, m0 + wr * 128, n0 + wc * 64, M, N, ea);
}

// ------------------------------------------------------------------------------------------------
// k_gemm_h: 256 x 128 x 32 tiles, 256 threads = 4 waves (2 M x 2 N, each a 128 x 64 sub-tile exactly as a
// k_gemm_big wave), a 3-stage LDS-DMA ring of 24 KiB stages (two K-steps of DMA in flight behind the one being
// computed), and TWO workgroups per CU (72 KiB LDS each). The point is the epilogue: with one 256 x 256 block per
// CU every CU reaches its epilogue at the same moment (the grid runs in lock-step rounds), so the output stores
// (and the residual reads) of all 256 CUs contend for HBM while the MFMAs idle, and then the K loops contend for L2
// while HBM idles. Two resident blocks per CU drift apart after the first round: one block's epilogue runs beside
// the other's K loop. BK = 32: a row is 64 B (4 16-byte chunks), swizzle chunk ^ ((row >> 2) & 3) makes the
// 16-lane groups of a ds_read_b128 fragment read hit 16 distinct 16-byte bank groups.
// ------------------------------------------------------------------------------------------------
#define GH_BN 128
#define GH_BK 32
#define GH_ST 3
#define GH_STAGE ((GB_BM + GH_BN) * GH_BK)  // bf16 elements per stage (A rows then W rows)
__device__ inline int gh_swz(int r) { return (r >> 2) & 3; }

template <int EPI>
__global__ __launch_bounds__(256, 2) void k_gemm_h(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                   int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  // 3 x 24 KiB ring; after the K loop 4 x [64][68] f32 epilogue images (69.6 KB) reuse it
  __shared__ __attribute__((aligned(16))) bf16_t smem[GH_ST * GH_STAGE];
  static_assert(4 * 64 * GB_EPI_LD * 4 <= GH_ST * GH_STAGE * 2, "epilogue images exceed the ring");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + GB_BM - 1) / GB_BM, ntn = (N + GH_BN - 1) / GH_BN;
  const int nwg = ntm * ntn;
  const int orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int tm, tn;
  tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
  const int m0 = tm * GB_BM, n0 = tn * GH_BN;

  // DMA: a stage is 384 rows x 64 B (A rows 0..255, W rows 256..383) = 24 wave-instructions of 16 rows; wave w
  // issues instructions t = 6w .. 6w+5. Lane l: row 16t + (l >> 2), LDS chunk slot l & 3 <- global chunk
  // (l & 3) ^ swz(row) (rows past M / N are clamped: their outputs are never stored).
  const bf16_t* src[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int t = wid * 6 + i, r = 16 * t + (lane >> 2);
    const int ch = (lane & 3) ^ gh_swz(r);
    src[i] = r < GB_BM ? A + (size_t)min(m0 + r, M - 1) * lda + ch * 8
                       : W + (size_t)min(n0 + r - GB_BM, N - 1) * ldw + ch * 8;
  }
  auto stage = [&](int buf, int k0) {
#pragma unroll
    for (int i = 0; i < 6; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + k0),
                                       (lds_void_t*)(smem + buf * GH_STAGE + (wid * 6 + i) * 16 * GH_BK), 16, 0, 0);
  };

  const int wr = wid >> 1, wc = wid & 1;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / GH_BK;
  stage(0, 0);
  if (nk > 1) stage(1, GH_BK);
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // K-step kt landed (this wave's DMA: all but the newest stage; everyone's: the barrier), and every wave is
    // past K-step kt-1, whose buffer the DMA below refills
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + 2 < nk) stage(cur == 0 ? 2 : cur - 1, (kt + 2) * GH_BK);
    const bf16_t* As = smem + cur * GH_STAGE;
    const bf16_t* Ws = As + GB_BM * GH_BK;
    bf16x8 bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wc * 64 + j * 16 + fr;
      bfr[j] = *(const bf16x8*)(Ws + col * GH_BK + ((fq ^ gh_swz(col)) << 3));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr * 128 + i * 16 + fr;
      const bf16x8 af = *(const bf16x8*)(As + row * GH_BK + ((fq ^ gh_swz(row)) << 3));
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
    }
    cur = cur == 2 ? 0 : cur + 1;
  }
  __syncthreads();  // every wave's last ds_reads are done before the ring becomes epilogue images
  gemm_epi_128x64<EPI>(acc, (float*)smem + wid * (64 * GB_EPI_LD), lane, m0 + wr * 128, n0 + wc * 64, M, N, ea);
}

// ------------------------------------------------------------------------------------------------
// k_gemm_ns: 256 x BN tiles, BK = 64, an NST-stage LDS-DMA ring (NST - 1 K-steps in flight), counted vmcnt +
// one raw barrier per K-step, optional s_setprio(1) around the MFMA cluster. BN = 128 makes a 3-stage ring fit
// (3 x 48 KiB) so the DMA of a K-step has two K-steps of MFMAs to land instead of one.
// ------------------------------------------------------------------------------------------------
template <int N_AFTER, int PER_STEP>
__device__ inline void ns_wait_barrier() {
  // this wave's DMA of the K-step about to be read is complete when at most N_AFTER * PER_STEP newer
  // instructions are outstanding
  if constexpr (N_AFTER * PER_STEP == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N_AFTER * PER_STEP == 5) asm volatile("s_waitcnt vmcnt(5)\n\ts_barrier" ::: "memory");
  else if constexpr (N_AFTER * PER_STEP == 6) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
  else if constexpr (N_AFTER * PER_STEP == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  else if constexpr (N_AFTER * PER_STEP == 10) asm volatile("s_waitcnt vmcnt(10)\n\ts_barrier" ::: "memory");
  else if constexpr (N_AFTER * PER_STEP == 12) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
  else if constexpr (N_AFTER * PER_STEP == 16) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  else static_assert(N_AFTER * PER_STEP == 0, "unsupported vmcnt");
}

template <int EPI, int BN, int NST, bool PRIO>
__global__ __launch_bounds__(512, 1) void k_gemm_ns(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  constexpr int WN = BN / 4, NT = WN / 16;                    // per-wave columns, 16-wide n-tiles
  constexpr int STAGE = (GB_BM + BN) * GB_BK;                   // bf16 elements per stage
  constexpr int IA = GB_BM * GB_BK / (8 * 512), IB = BN * GB_BK / (8 * 512);  // DMA instructions per wave
  constexpr int EPI_LD = WN + 4;
  constexpr int SMEM = (NST * STAGE * 2 > 8 * 64 * EPI_LD * 4) ? NST * STAGE * 2 : 8 * 64 * EPI_LD * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[SMEM];
  bf16_t* smem = (bf16_t*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + GB_BM - 1) / GB_BM, ntn = (N + BN - 1) / BN;
  const int nwg = ntm * ntn;
  const int orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int tm, tn;
  tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
  const int m0 = tm * GB_BM, n0 = tn * BN;

  const bf16_t* ga[IA];
  const bf16_t* gw[IB];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int row = 8 * (IA * wid + i) + (lane >> 3);
    ga[i] = A + (size_t)min(m0 + row, M - 1) * lda + ((lane & 7) ^ gb_swz(row)) * 8;
  }
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int row = 8 * (IB * wid + i) + (lane >> 3);
    gw[i] = W + (size_t)min(n0 + row, N - 1) * ldw + ((lane & 7) ^ gb_swz(row)) * 8;
  }
  auto stage = [&](int st, int k0) {
    bf16_t* As = smem + st * STAGE;
    bf16_t* Ws = As + GB_BM * GB_BK;
#pragma unroll
    for (int i = 0; i < IA; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(ga[i] + k0), (lds_void_t*)(As + 8 * (IA * wid + i) * GB_BK), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < IB; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(gw[i] + k0), (lds_void_t*)(Ws + 8 * (IB * wid + i) * GB_BK), 16, 0, 0);
  };

  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[8][NT];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / GB_BK;
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nk) stage(t, t * GB_BK);
  for (int kt = 0; kt < nk; ++kt) {
    const int after = min(NST - 2, nk - 1 - kt);
    if constexpr (NST == 3) {
      if (after == 1) ns_wait_barrier<1, IA + IB>();
      else ns_wait_barrier<0, IA + IB>();
    } else {
      ns_wait_barrier<0, IA + IB>();
    }
    if (kt + NST - 1 < nk) stage((kt + NST - 1) % NST, (kt + NST - 1) * GB_BK);
    const bf16_t* As = smem + (kt % NST) * STAGE;
    const bf16_t* Ws = As + GB_BM * GB_BK;
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kc = 4 * kk + fq;
      bf16x8 bfr[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = wc * WN + j * 16 + fr;
        bfr[j] = *(const bf16x8*)(Ws + col * GB_BK + ((kc ^ gb_swz(col)) << 3));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = wr * 128 + i * 16 + fr;
        const bf16x8 af = *(const bf16x8*)(As + row * GB_BK + ((kc ^ gb_swz(row)) << 3));
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");  // LDS is reused by the epilogue

  // epilogue through LDS (as k_gemm_big): per wave 64 rows x WN cols at a time, read back 4 cols per lane
  constexpr int LPR = WN / 4;           // lanes per row in the read-back
  constexpr int RPI = 64 / LPR;         // rows per wave-instruction
  const int ncol0 = n0 + wc * WN;
  const int rc = (lane % LPR) * 4;
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ea.bias) {
    const int n = ncol0 + rc;
    bias4.x = ea.bias[min(n, N - 1)];
    bias4.y = ea.bias[min(n + 1, N - 1)];
    bias4.z = ea.bias[min(n + 2, N - 1)];
    bias4.w = ea.bias[min(n + 3, N - 1)];
  }
  float* wimg = (float*)smem + wid * (64 * EPI_LD);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int ib = 4 * half;
    if (half) __syncthreads();
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) wimg[(ii * 16 + fq * 4 + r) * EPI_LD + j * 16 + fr] = acc[ib + ii][j][r];
    __syncthreads();
    const int mrow0 = m0 + wr * 128 + ib * 16;
#pragma unroll 4
    for (int rr = 0; rr < 64 / RPI; ++rr) {
      const int lr = rr * RPI + lane / LPR;
      const int m = mrow0 + lr;
      float4 v = *(const float4*)(wimg + lr * EPI_LD + rc);
      v.x += bias4.x; v.y += bias4.y; v.z += bias4.z; v.w += bias4.w;
      if (m < M && ncol0 + rc < N) epi_store4<EPI>(ea, m, ncol0 + rc, N, v);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// k_gemm_8p: 256 x 256 x 64 tiles, 8 waves in two ping-pong groups, 4 phases per K-tile
// (cdna_hip_programming.md §5 "The 256² 8-phase template": the structure, not its code).
// LDS holds two K-tiles, each as four 16 KiB half-tiles A0 | A1 | B0 | B1 (rows 0-127 / 128-255 of the A and W
// tiles). Phase p of K-tile t computes one C-quadrant (A half, B half) = (0,0), (0,1), (1,1), (1,0): every wave
// owns a 64 x 32 piece of each quadrant (rows 64*wr + 128*mh, cols 32*wc + 128*nh), i.e. 16 MFMAs per phase, and
// re-reads only the operand half that changed. Each phase also stages one half-tile of K-tile t+1 (A0, B0, B1,
// A1 — the order K-tile t+1 first needs them), so two phases of MFMAs cover every DMA. Waits are counted
// (vmcnt never 0 inside the loop), barriers raw; waves 4-7 run one barrier behind waves 0-3, so on each SIMD
// one wave's MFMA cluster (at raised priority) overlaps the other wave's ds_reads and DMA issue.
//   RAW: a half-tile is waited for (vmcnt) before the first barrier of the phase before the one that reads it.
//   WAR: a half-tile is restaged >= 2 phases after its last ds_read (A0 4, B0 2, B1 4, A1 4).
// ------------------------------------------------------------------------------------------------
template <int N>
__device__ inline void p8_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm_8p(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  // K loop: 2 buffers x 4 half-tiles x 16 KiB = 128 KiB; epilogue: 8 x [64][68] f32 = 136 KiB (one array: a
  // second __shared__ object makes hipcc drain vmcnt before every ds_read)
  __shared__ __attribute__((aligned(16))) bf16_t smem[8 * 64 * GB_EPI_LD * 2];
  constexpr int HT = 128 * GB_BK;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + GB_BM - 1) / GB_BM, ntn = (N + GB_BN - 1) / GB_BN;
  const int nwg = ntm * ntn;
  const int orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int tm, tn;
  tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
  const int m0 = tm * GB_BM, n0 = tn * GB_BN;
  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;

  // DMA: half-tile h (0 A0, 1 A1, 2 B0, 3 B1), wave instruction i = 0,1 fills rows 8(2*wid+i) .. +7.
  // buffer_load ... lds through one descriptor per half-tile (wave-uniform base = the half-tile's first row,
  // num_records = its rows inside M / N): the per-lane part is a 32-bit row/chunk offset (4 VGPRs instead of 8
  // 64-bit pointers, so the kernel stays under 196 VGPRs and a decoder wave can co-reside on every SIMD), the
  // K offset rides in soffset, and rows past M / N read as zeros (their outputs are never stored).
  __amdgpu_buffer_rsrc_t rs[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int r0 = (h < 2 ? m0 : n0) + 128 * (h & 1), lim = h < 2 ? M : N, ld = h < 2 ? lda : ldw;
    const int rows = max(0, min(128, lim - r0));
    rs[h] = tw_uniform_rsrc((h < 2 ? A : W) + (size_t)r0 * ld, rows * ld * 2);
  }
  unsigned voff[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 8 * (2 * wid + i) + (lane >> 3);
    const int ch = (lane & 7) ^ gb_swz(row);
    voff[0][i] = (unsigned)(row * lda + ch * 8) * 2u;
    voff[1][i] = (unsigned)(row * ldw + ch * 8) * 2u;
  }
  auto stage = [&](int buf, int h, int k0) {
    bf16_t* dst = smem + (buf * 4 + h) * HT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs[h], (lds_void_t*)(dst + 8 * (2 * wid + i) * GB_BK), 16,
                                               voff[h >> 1][i], (unsigned)k0 * 2u, 0, 0);
  };

  bf16x8 af[4][2], bfr[2][2];
  auto readA = [&](int buf, int mh) {
    const bf16_t* As = smem + (buf * 4 + mh) * HT;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int row = 64 * wr + 16 * i + fr, kc = 4 * kk + fq;
        af[i][kk] = *(const bf16x8*)(As + row * GB_BK + ((kc ^ gb_swz(row)) << 3));
      }
  };
  auto readB = [&](int buf, int nh) {
    const bf16_t* Bs = smem + (buf * 4 + 2 + nh) * HT;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int row = 32 * wc + 16 * j + fr, kc = 4 * kk + fq;
        bfr[j][kk] = *(const bf16x8*)(Bs + row * GB_BK + ((kc ^ gb_swz(row)) << 3));
      }
  };
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto mfma_q = [&](auto MH, auto NH) {
    constexpr int mh = decltype(MH)::value, nh = decltype(NH)::value;
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mh][nh][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bfr[j][kk], acc[mh][nh][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  const int nk = K / GB_BK;
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // ping-pong: group 1 one barrier behind
  // one K-tile = 4 phases; NXT: stage K-tile t+1 (compile-time, so the steady-state loop has no branches)
  auto ktile = [&](int t, auto NXT) {
    constexpr bool nxt = decltype(NXT)::value;
    const int buf = t & 1, nb = buf ^ 1, kn = (t + 1) * GB_BK;
    // phase 1: quadrant (A0, B0)
    readB(buf, 0);
    __builtin_amdgcn_sched_barrier(0);
    readA(buf, 0);
    if constexpr (nxt) {
      stage(nb, 0, kn);
      p8_vmcnt<4>();  // B1 of tile t (staged in phase 3 of t-1)
    } else {
      p8_vmcnt<2>();
    }
    mfma_q(I0{}, I0{});
    // phase 2: (A0, B1)
    readB(buf, 1);
    if constexpr (nxt) {
      stage(nb, 2, kn);
      p8_vmcnt<4>();  // A1 of tile t (phase 4 of t-1)
    } else {
      p8_vmcnt<0>();
    }
    mfma_q(I0{}, I1{});
    // phase 3: (A1, B1)
    readA(buf, 1);
    if constexpr (nxt) stage(nb, 3, kn);
    mfma_q(I1{}, I1{});
    // phase 4: (A1, B0)
    readB(buf, 0);
    if constexpr (nxt) {
      stage(nb, 1, kn);
      p8_vmcnt<4>();  // A0, B0 of tile t+1 (phases 1, 2 of t)
    }
    mfma_q(I1{}, I0{});
  };
  using BT = std::integral_constant<bool, true>;
  using BF = std::integral_constant<bool, false>;
  for (int t = 0; t + 1 < nk; ++t) ktile(t, BT{});
  ktile(nk - 1, BF{});
  if (wr == 0) __builtin_amdgcn_s_barrier();  // realign the groups
  __syncthreads();

  // epilogue through LDS: per wave two 64-row halves (mh) of [64][64] f32 (cols = its two 32-col chunks), read
  // back 8 consecutive columns per lane (8 lanes per row) for 16-byte global stores
  const int rc = (lane & 7) * 8;
  const int ncol = n0 + (rc < 32 ? 32 * wc + rc : 128 + 32 * wc + rc - 32);
  float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
  if (ea.bias) {
    b0.x = ea.bias[min(ncol, N - 1)];
    b0.y = ea.bias[min(ncol + 1, N - 1)];
    b0.z = ea.bias[min(ncol + 2, N - 1)];
    b0.w = ea.bias[min(ncol + 3, N - 1)];
    b1.x = ea.bias[min(ncol + 4, N - 1)];
    b1.y = ea.bias[min(ncol + 5, N - 1)];
    b1.z = ea.bias[min(ncol + 6, N - 1)];
    b1.w = ea.bias[min(ncol + 7, N - 1)];
  }
  float* wimg = (float*)smem + wid * (64 * GB_EPI_LD);
  // RESID / GELU_POS: second operand loaded ahead, rows rr and rr + 4 sharing a slot (see k_gemm_big)
  constexpr bool PRE = EPI == TW_EPI_RESID_F32 || EPI == TW_EPI_GELU_POS_F32;
  const bool full = ncol + 7 < N;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
    const int mrow0 = m0 + 128 * mh + 64 * wr;
    float4 ad[4][2];
    if constexpr (PRE) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int mq = min(mrow0 + q * 8 + (lane >> 3), M - 1);
        ad[q][0] = epi_addend<EPI>(ea, mq, ncol, full);
        ad[q][1] = epi_addend<EPI>(ea, mq, ncol + 4, full);
      }
    }
    if (mh) gb_epi_sync();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            wimg[(i * 16 + fq * 4 + r) * GB_EPI_LD + nh * 32 + j * 16 + fr] = acc[mh][nh][i][j][r];
    gb_epi_sync();
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      const int lr = rr * 8 + (lane >> 3);
      const int m = mrow0 + lr;
      float4 v0 = *(const float4*)(wimg + lr * GB_EPI_LD + rc);
      float4 v1 = *(const float4*)(wimg + lr * GB_EPI_LD + rc + 4);
      v0.x += b0.x; v0.y += b0.y; v0.z += b0.z; v0.w += b0.w;
      v1.x += b1.x; v1.y += b1.y; v1.z += b1.z; v1.w += b1.w;
      if constexpr (PRE) {
        if (full) {
          if (m < M) {
            epi_store4_pre<EPI>(ea, m, ncol, v0, ad[rr & 3][0]);
            epi_store4_pre<EPI>(ea, m, ncol + 4, v1, ad[rr & 3][1]);
          }
        } else if (m < M && ncol < N) {
          epi_store8<EPI>(ea, m, ncol, N, v0, v1);
        }
        if (rr < 4) {
          const int mq = min(m + 32, M - 1);
          ad[rr][0] = epi_addend<EPI>(ea, mq, ncol, full);
          ad[rr][1] = epi_addend<EPI>(ea, mq, ncol + 4, full);
        }
      } else {
        if (m < M && ncol < N) epi_store8<EPI>(ea, m, ncol, N, v0, v1);
      }
    }
  }
}

// k_gemm_8pp: k_gemm_8p made persistent — one block per CU loops over tiles (virtual ids b, b + G, ...; G % 8 == 0
// keeps a block on one XCD's share of the bijective remap). The whole grid is resident after one dispatch round,
// so the command processor is free to dispatch other queues' kernels (the decoder step beside the encoder) instead
// of feeding this kernel's thousands of workgroups. The next tile's K-tile 0 lands in buffer 0 during the epilogue;
// the epilogue images move to [64 KiB, 132 KiB) and run in four 32-row passes.
template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm_8pp(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                     int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[8 * 64 * GB_EPI_LD * 2];
  constexpr int HT = 128 * GB_BK;
  constexpr int EPI_BASE = 64 * 1024 / 4;  // f32 offset of the epilogue images
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + GB_BM - 1) / GB_BM, ntn = (N + GB_BN - 1) / GB_BN;
  const int nwg = ntm * ntn;
  const int q8 = nwg / 8, r8 = nwg % 8;
  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  auto tile_origin = [&](int vid, int& m0, int& n0) {
    const int xcd = vid % 8;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + vid / 8;
    int tm, tn;
    tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
    m0 = tm * GB_BM;
    n0 = tn * GB_BN;
  };
  const bf16_t* gsrc[4][2];
  auto set_src = [&](int m0, int n0) {
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = 8 * (2 * wid + i) + (lane >> 3);
        const int ch = (lane & 7) ^ gb_swz(row);
        gsrc[h][i] = h < 2 ? A + (size_t)min(m0 + 128 * h + row, M - 1) * lda + ch * 8
                           : W + (size_t)min(n0 + 128 * (h - 2) + row, N - 1) * ldw + ch * 8;
      }
  };
  auto stage = [&](int buf, int h, int k0) {
    bf16_t* dst = smem + (buf * 4 + h) * HT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(gsrc[h][i] + k0), (lds_void_t*)(dst + 8 * (2 * wid + i) * GB_BK),
                                       16, 0, 0);
  };
  bf16x8 af[4][2], bfr[2][2];
  auto readA = [&](int buf, int mh) {
    const bf16_t* As = smem + (buf * 4 + mh) * HT;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int row = 64 * wr + 16 * i + fr, kc = 4 * kk + fq;
        af[i][kk] = *(const bf16x8*)(As + row * GB_BK + ((kc ^ gb_swz(row)) << 3));
      }
  };
  auto readB = [&](int buf, int nh) {
    const bf16_t* Bs = smem + (buf * 4 + 2 + nh) * HT;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int row = 32 * wc + 16 * j + fr, kc = 4 * kk + fq;
        bfr[j][kk] = *(const bf16x8*)(Bs + row * GB_BK + ((kc ^ gb_swz(row)) << 3));
      }
  };
  f32x4 acc[2][2][4][2];
  auto mfma_q = [&](auto MH, auto NH) {
    constexpr int mh = decltype(MH)::value, nh = decltype(NH)::value;
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mh][nh][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bfr[j][kk], acc[mh][nh][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto ktile = [&](int t, auto NXT) {
    constexpr bool nxt = decltype(NXT)::value;
    const int buf = t & 1, nb = buf ^ 1, kn = (t + 1) * GB_BK;
    readB(buf, 0);
    __builtin_amdgcn_sched_barrier(0);
    readA(buf, 0);
    if constexpr (nxt) {
      stage(nb, 0, kn);
      p8_vmcnt<4>();
    } else {
      p8_vmcnt<2>();
    }
    mfma_q(I0{}, I0{});
    readB(buf, 1);
    if constexpr (nxt) {
      stage(nb, 2, kn);
      p8_vmcnt<4>();
    } else {
      p8_vmcnt<0>();
    }
    mfma_q(I0{}, I1{});
    readA(buf, 1);
    if constexpr (nxt) stage(nb, 3, kn);
    mfma_q(I1{}, I1{});
    readB(buf, 0);
    if constexpr (nxt) {
      stage(nb, 1, kn);
      p8_vmcnt<4>();
    }
    mfma_q(I1{}, I0{});
  };
  using BT = std::integral_constant<bool, true>;
  using BF = std::integral_constant<bool, false>;
  const int nk = K / GB_BK;
  const int rc = (lane & 7) * 8;
  float* wimg = (float*)smem + EPI_BASE + wid * (32 * GB_EPI_LD);

  int vid = blockIdx.x, m0, n0;
  tile_origin(vid, m0, n0);
  set_src(m0, n0);
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, 0);
  while (true) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // K-tile 0 (and the previous tile's stores)
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();
    for (int t = 0; t + 1 < nk; ++t) ktile(t, BT{});
    ktile(nk - 1, BF{});
    if (wr == 0) __builtin_amdgcn_s_barrier();
    __syncthreads();
    const int cm0 = m0, cn0 = n0;
    const int nvid = vid + gridDim.x;
    const bool more = nvid < nwg;
    if (more) {
      tile_origin(nvid, m0, n0);
      set_src(m0, n0);
#pragma unroll
      for (int h = 0; h < 4; ++h) stage(0, h, 0);
    }
    const int ncol = cn0 + (rc < 32 ? 32 * wc + rc : 128 + 32 * wc + rc - 32);
    float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
    if (ea.bias) {
      b0.x = ea.bias[min(ncol, N - 1)];
      b0.y = ea.bias[min(ncol + 1, N - 1)];
      b0.z = ea.bias[min(ncol + 2, N - 1)];
      b0.w = ea.bias[min(ncol + 3, N - 1)];
      b1.x = ea.bias[min(ncol + 4, N - 1)];
      b1.y = ea.bias[min(ncol + 5, N - 1)];
      b1.z = ea.bias[min(ncol + 6, N - 1)];
      b1.w = ea.bias[min(ncol + 7, N - 1)];
    }
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int ih = 0; ih < 2; ++ih) {
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
          for (int nh = 0; nh < 2; ++nh)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                wimg[(i2 * 16 + fq * 4 + r) * GB_EPI_LD + nh * 32 + j * 16 + fr] = acc[mh][nh][2 * ih + i2][j][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int mrow0 = cm0 + 128 * mh + 64 * wr + 32 * ih;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int lr = rr * 8 + (lane >> 3);
          const int m = mrow0 + lr;
          float4 v0 = *(const float4*)(wimg + lr * GB_EPI_LD + rc);
          float4 v1 = *(const float4*)(wimg + lr * GB_EPI_LD + rc + 4);
          v0.x += b0.x; v0.y += b0.y; v0.z += b0.z; v0.w += b0.w;
          v1.x += b1.x; v1.y += b1.y; v1.z += b1.z; v1.w += b1.w;
          if (m < M && ncol < N) epi_store8<EPI>(ea, m, ncol, N, v0, v1);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    if (!more) break;
    vid = nvid;
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// k_gemm_4w: 256 x 256 x 64 tiles on FOUR waves (256 threads, one wave per SIMD), each wave a 128 x 128 sub-tile =
// 8 x 8 accumulators of v_mfma_f32_16x16x32_bf16 (256 accumulator registers; the unified register file holds them
// beside the operand fragments at one wave per SIMD). Against the 8-wave kernels (128 x 64 per wave) a wave reads
// 32 KiB of LDS per K-step for 2 MFLOP instead of 24 KiB for 1 MFLOP, and the CU issues half the LDS reads per FLOP;
// it is the decomposition hipBLASLt picks on these shapes (MT256x256x64, MI16x16, 256 threads). Staging as
// k_gemm_8p: buffer_load ... lds (LDS-DMA) through one wave-uniform descriptor per operand tile (rows past M / N
// read as zeros), source-side chunk swizzle chunk ^ ((row >> 1) & 7) undone on the ds_read_b128 address; the
// per-instruction row block rides in soffset, so the per-lane part is two 32-bit offsets per operand. K loop: DMA of
// K-tile t+1 issued first, then the two 32-deep k-substeps of tile t (16 fragment reads + 64 MFMAs each), one
// vmcnt(0) + barrier per K-tile. Epilogue: each wave stages 32-row slabs of its 128 x 128 f32 results in its own
// LDS image (row stride 132 floats: conflict-free writes) and stores 8 consecutive columns per lane.
// MEASURED SLOWER than k_gemm_8p and kept only as an A/B variant (tw_gemm_set_variant(8), scripts/gemm_bench.py,
// MI355X): qkv 792 vs 1048, fc2 820 vs 1119 TF/s; with the K-loop DMA removed (timing only) fc2 reaches 1226, so
// at one wave per SIMD this hipcc-scheduled loop (92 AGPR<->VGPR moves per K-tile, exposed fragment-read latency)
// is the limit before the staging is; hipBLASLt's hand-scheduled kernel of this shape reaches 1318.
// ------------------------------------------------------------------------------------------------
#define G4_LD 132  // f32 row stride of a wave's epilogue image (128 + 4)
template <int EPI>
__global__ __launch_bounds__(256, 1) void k_gemm_4w(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  // K loop: 2 buffers x (A | W) x 256 rows x 64 bf16 = 128 KiB; epilogue: 4 waves x 32 rows x 132 f32 = 66 KiB
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * 2 * 256 * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform: soffset / LDS bases in SGPRs
  const int ntm = (M + 255) / 256, ntn = (N + 255) / 256;
  const int nwg = ntm * ntn;
  const int orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int tm, tn;
  tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int wr = wid >> 1, wc = wid & 1;
  const int fr = lane & 15, fq = lane >> 4;

  // DMA: wave w fills rows [64w, 64w + 64) of the A tile and of the W tile with 8 instructions each; instruction i
  // moves rows 64w + 8i + (lane >> 3), 16-byte chunk (lane & 7) ^ swz(row). swz(row) depends on i only through its
  // parity, so two voffsets per operand; the row block (64w + 8i) * ld goes into soffset with the K offset.
  const int ra = M - m0, rw = N - n0;
  const __amdgpu_buffer_rsrc_t rsA = tw_uniform_rsrc(A + (size_t)m0 * lda, max(0, min(256, ra)) * lda * 2);
  const __amdgpu_buffer_rsrc_t rsW = tw_uniform_rsrc(W + (size_t)n0 * ldw, max(0, min(256, rw)) * ldw * 2);
  unsigned va[2], vw[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int r = 8 * par + (lane >> 3);  // row within an aligned 16-row block: swz = (r >> 1) & 7
    const int ch = (lane & 7) ^ ((r >> 1) & 7);
    va[par] = (unsigned)((lane >> 3) * lda + ch * 8) * 2u;
    vw[par] = (unsigned)((lane >> 3) * ldw + ch * 8) * 2u;
  }
  auto stage = [&](int buf, int k0) {
    bf16_t* As = smem + buf * (2 * 256 * 64);
    bf16_t* Ws = As + 256 * 64;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rb = 64 * wid + 8 * i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void_t*)(As + rb * 64), 16, va[i & 1],
                                               (unsigned)(rb * lda + k0) * 2u, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (lds_void_t*)(Ws + rb * 64), 16, vw[i & 1],
                                               (unsigned)(rb * ldw + k0) * 2u, 0, 0);
    }
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // Software pipeline, one barrier per K-tile placed mid-tile (two LDS buffers; tile t lives in buffer t & 1):
  //   phase A of tile t: 64 MFMAs on the k-substep-0 fragments F0(t) || ds_read of F1(t)
  //   mid barrier:       vmcnt(0) (this wave's DMA of tile t+1 landed) + lgkmcnt(0) + s_barrier
  //   phase B of tile t: 64 MFMAs on F1(t) || ds_read of F0(t+1) || DMA of tile t+2 into buffer t & 1
  // RAW: F0(t+1) is read after the mid barrier of t, which follows every wave's wait for its DMA of tile t+1.
  // WAR: the DMA of t+2 overwrites buffer t & 1 after the mid barrier of t, by which every wave's reads of F0(t)
  // (phase B of t-1) and F1(t) (phase A of t, lgkmcnt(0) before the barrier) have completed.
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  auto rdfr = [&](int buf, int kk, bf16x8 (&af)[8], bf16x8 (&bw)[8]) {
    const bf16_t* As = smem + buf * (2 * 256 * 64);
    const bf16_t* Ws = As + 256 * 64;
    const int kc = 4 * kk + fq;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = 128 * wc + 16 * j + fr;
      bw[j] = *(const bf16x8*)(Ws + col * 64 + ((kc ^ gb_swz(col)) << 3));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = 128 * wr + 16 * i + fr;
      af[i] = *(const bf16x8*)(As + row * 64 + ((kc ^ gb_swz(row)) << 3));
    }
  };
  auto mma = [&](const bf16x8 (&af)[8], const bf16x8 (&bw)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bw[j], acc[i][j], 0, 0, 0);
  };
  const int nk = K / GB_BK;
  stage(0, 0);
  if (nk > 1) stage(1, GB_BK);
  if (nk > 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 (its 16 instructions were issued first)
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  rdfr(0, 0, fa0, fb0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // phase A
    rdfr(cur, 1, fa1, fb1);
    mma(fa0, fb0);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 ds_read
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // phase B
    if (kt + 1 < nk) rdfr(cur ^ 1, 0, fa0, fb0);
    if (kt + 2 < nk) stage(cur, (kt + 2) * GB_BK);
    mma(fa1, fb1);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 ds_read
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // 1 LDS-DMA (VMEM read)
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the staging LDS

  // epilogue: four 32-row slabs per wave through its [32][G4_LD] f32 image; 16 lanes per row, 8 columns per lane
  float* img = (float*)smem + wid * (32 * G4_LD);
  const int rc = (lane & 15) * 8;  // this lane's 8 columns in the read-back
  const int ncol = n0 + 128 * wc + rc;
  float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
  if (ea.bias) {
    b0.x = ea.bias[min(ncol, N - 1)];
    b0.y = ea.bias[min(ncol + 1, N - 1)];
    b0.z = ea.bias[min(ncol + 2, N - 1)];
    b0.w = ea.bias[min(ncol + 3, N - 1)];
    b1.x = ea.bias[min(ncol + 4, N - 1)];
    b1.y = ea.bias[min(ncol + 5, N - 1)];
    b1.z = ea.bias[min(ncol + 6, N - 1)];
    b1.w = ea.bias[min(ncol + 7, N - 1)];
  }
  constexpr bool PRE = EPI == TW_EPI_RESID_F32 || EPI == TW_EPI_GELU_POS_F32;
  const bool full = ncol + 7 < N;
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) {  // slab sl = accumulator rows i = 2 sl, 2 sl + 1 (32 rows)
    const int mrow0 = m0 + 128 * wr + 32 * sl;
    float4 ad[8][2];
    if constexpr (PRE) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int mq = min(mrow0 + q * 4 + (lane >> 4), M - 1);
        ad[q][0] = epi_addend<EPI>(ea, mq, ncol, full);
        ad[q][1] = epi_addend<EPI>(ea, mq, ncol + 4, full);
      }
    }
    if (sl) __syncthreads();  // (first slab: the K loop ended on a barrier)
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) img[(16 * ii + 4 * fq + r) * G4_LD + 16 * j + fr] = acc[2 * sl + ii][j][r];
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      const int lr = rr * 4 + (lane >> 4);
      const int m = mrow0 + lr;
      float4 v0 = *(const float4*)(img + lr * G4_LD + rc);
      float4 v1 = *(const float4*)(img + lr * G4_LD + rc + 4);
      v0.x += b0.x; v0.y += b0.y; v0.z += b0.z; v0.w += b0.w;
      v1.x += b1.x; v1.y += b1.y; v1.z += b1.z; v1.w += b1.w;
      if constexpr (PRE) {
        if (full) {
          if (m < M) {
            epi_store4_pre<EPI>(ea, m, ncol, v0, ad[rr][0]);
            epi_store4_pre<EPI>(ea, m, ncol + 4, v1, ad[rr][1]);
          }
        } else if (m < M && ncol < N) {
          epi_store8<EPI>(ea, m, ncol, N, v0, v1);
        }
      } else {
        if (m < M && ncol < N) epi_store8<EPI>(ea, m, ncol, N, v0, v1);
      }
    }
  }
}

static int tw_num_cus() {
  static int cus = 0;  // one device per process (the engine's)
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 8) cus = 256;
  }
  return cus;
}

// ------------------------------------------------------------------------------------------------
// Skinny kernel (M <= 32): weight-streaming MFMA GEMV for the decoder step
// ------------------------------------------------------------------------------------------------
// Block = NW waves = 16 output columns; the K range is cut into NW * gridDim.y slices of 32-deep
// steps (wave w of block row y takes slice y*NW + w). Each wave streams its slice of the 16 weight
// rows straight to VGPRs (every weight byte is read exactly once per step: this path is HBM-bound)
// with 8 steps of loads in flight, and runs v_mfma_f32_16x16x32_bf16 on two 16-row M tiles:
//   A lane l: A[row = l&15][k = 8(l>>4)+j]   B lane l: W[col = l&15][k = 8(l>>4)+j]
//   C lane l: col = l&15, row = (l>>4)*4 + reg
// The NW partial sums meet in LDS. gridDim.y > 1 (split-K over blocks, used for the N = d_model
// projections whose 80 column groups alone cannot fill 256 CUs): each block row writes its f32 partial
// to part[y][M][ldo] and the consumer (tw_resid_layernorm) adds the partials, bias and residual.
#define TW_EPI_PARTIAL 100
// The decoder's residual update with LayerNorm statistics (tw_gemv_packed_stats): x[m][n] += acc + bias as
// TW_EPI_RESID_F32, and for every 16-column group g the updated row slice's (mean, M2 = sum of squared deviations
// from that mean) into stats[(g * 32 + m) * 2 ..]. The consuming GEMV (tw_gemv_packed_lnst) combines the K/16 groups
// into the row's mean and variance (Chan, Golub & LeVeque's pairwise update, as exact as a two-pass LayerNorm),
// so the LayerNorm between the two projections needs no launch of its own.
#define TW_EPI_RESID_STATS 102

template <int EPI, int NW, bool TWO>
__global__ __launch_bounds__(NW * 64) void k_gemm_skinny(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                         int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  TW_DEC_PRIO();
  __shared__ float red[NW][32][17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n0 = blockIdx.x * 16;
  const int nsl = NW * gridDim.y, gw = blockIdx.y * NW + wid;
  const int ns = K >> 5;
  const int s0 = (int)((long)gw * ns / nsl), s1 = (int)((long)(gw + 1) * ns / nsl);
  const int col = min(n0 + (lane & 15), N - 1);
  const int ksub = 8 * (lane >> 4);
  const int ar0 = min(lane & 15, M - 1), ar1 = min(16 + (lane & 15), M - 1);
  const bf16_t* wp = W + (size_t)col * ldw + ksub;
  const bf16_t* ap0 = A + (size_t)ar0 * lda + ksub;
  const bf16_t* ap1 = A + (size_t)ar1 * lda + ksub;
  f32x4 c0 = {0}, c1 = {0};
  int s = s0;
  for (; s + 8 <= s1; s += 8) {
    bf16x8 bw[8], a0[8], a1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      bw[u] = *(const bf16x8*)(wp + 32 * (s + u));
      a0[u] = *(const bf16x8*)(ap0 + 32 * (s + u));
      if (TWO) a1[u] = *(const bf16x8*)(ap1 + 32 * (s + u));
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], bw[u], c0, 0, 0, 0);
      if (TWO) c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], bw[u], c1, 0, 0, 0);
    }
  }
  for (; s < s1; ++s) {
    bf16x8 bw = *(const bf16x8*)(wp + 32 * s);
    bf16x8 a0 = *(const bf16x8*)(ap0 + 32 * s);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw, c0, 0, 0, 0);
    if (TWO) {
      bf16x8 a1 = *(const bf16x8*)(ap1 + 32 * s);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw, c1, 0, 0, 0);
    }
  }
  const int cc = lane & 15, rb = (lane >> 4) * 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[wid][rb + r][cc] = c0[r];
    if (TWO) red[wid][16 + rb + r][cc] = c1[r];
  }
  __syncthreads();
  const int rows = TWO ? 32 : 16;
  for (int e = tid; e < rows * 16; e += NW * 64) {
    int m = e >> 4, c = e & 15;
    int n = n0 + c;
    if (m < M && n < N) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += red[w][m][c];
      if constexpr (EPI == TW_EPI_PARTIAL) {
        ((float*)ea.out)[((size_t)blockIdx.y * M + m) * ea.ldo + n] = v;
      } else {
        epi_store<EPI>(ea, m, n, v);
      }
    }
  }
}

template <int EPI, int NW>
static void launch_skinny_nw(const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldw,
                             const EpiArgs& ea, int splits, hipStream_t s) {
  dim3 grid(tw_cdiv(N, 16), splits);
  if (M > 16)
    hipLaunchKernelGGL((k_gemm_skinny<EPI, NW, true>), grid, dim3(NW * 64), 0, s, A, W, M, N, K, lda, ldw, ea);
  else
    hipLaunchKernelGGL((k_gemm_skinny<EPI, NW, false>), grid, dim3(NW * 64), 0, s, A, W, M, N, K, lda, ldw, ea);
}

// Waves per block: enough column-group x K-slice waves to put ~4 waves on every CU, while every wave keeps
// at least two 32-deep steps.
template <int EPI>
static void launch_skinny(const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldw,
                          const EpiArgs& ea, int splits, hipStream_t s) {
  const long nb = tw_cdiv(N, 16) * (long)splits;
  const int ns = K / 32;
  int nw = 4;
  // at most 8 waves (17 KiB LDS): a 16-wave block (35 KiB) cannot co-reside with a k_gemm_big workgroup
  while (nb * nw < 1024 && nw < 8 && ns >= 2 * 2 * nw * splits) nw *= 2;
  if (tw_tune_skinny_nw) nw = tw_tune_skinny_nw;
  if (nw == 4) launch_skinny_nw<EPI, 4>(A, W, M, N, K, lda, ldw, ea, splits, s);
  else if (nw == 8) launch_skinny_nw<EPI, 8>(A, W, M, N, K, lda, ldw, ea, splits, s);
  else launch_skinny_nw<EPI, 16>(A, W, M, N, K, lda, ldw, ea, splits, s);
}

// ------------------------------------------------------------------------------------------------
// Packed decoder GEMV (M <= 32): weights pre-arranged in MFMA fragment order (tw_pack_weight), activations either
// in the packed activation layout (written by tw_resid_layernorm_packed / the GELU_PACKED epilogue) or row-major.
// Every wave-load is one contiguous 1 KiB fragment (weights: the whole read is one HBM stream per wave), instead
// of 16 rows x 64 B. Block = 4 (or KW = 8: 8) waves = GPB column groups x KW K-slices; gridDim.y = split-K over
// blocks for the PARTIAL epilogue (partials summed by the consumer, tw_resid_layernorm*).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pack_weight(const bf16_t* __restrict__ W, int N, int K, int ldw,
                                                     bf16_t* __restrict__ Wp, long nchunks) {
  const long c = (long)blockIdx.x * 256 + threadIdx.x;
  if (c >= nchunks) return;
  const int lane = (int)(c & 63);
  const long rest = c >> 6;
  const int ns = K >> 5;
  const int st = (int)(rest % ns), g = (int)(rest / ns);
  const int n = g * 16 + (lane & 15), k = st * 32 + 8 * (lane >> 4);
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (n < N) v = *(const uint4*)(W + (size_t)n * ldw + k);
  *(uint4*)(Wp + c * 8) = v;
}

// ALN (tw_gemv_packed_ln): the A operand is LayerNorm(x) of the f32 residual stream x [M][K] (row-major), computed
// inside the GEMV instead of by a separate decoder LayerNorm launch: the prologue computes every row's mean and
// 1/std (two-pass, as k_resid_ln_w, one wave per row in turn) into LDS, and each A fragment is normalised from x,
// gamma and beta as it is loaded. The residual stream is then updated in place by the producing GEMVs' RESID
// epilogue (x += A.W^T + bias, no split-K partials), so a decoder layer is 8 launches instead of 11.
struct LnArgs {
  const float* x;
  const float* g;
  const float* b;
  float eps;
  const float* stats;  // non-null: the rows' statistics come from the producing GEMV (TW_EPI_RESID_STATS)
};
#define GEMV_LN_MAXV 8  // float4 chunks per lane of one row in the LN prologue: K <= 2048

// NTW: weight fragments read with non-temporal loads (proj_out: 133 MB streamed once per step, kept out of the
// caches so that the layer weights can stay in them).
template <int EPI, int KW, int U, bool APACK, bool TWO, bool NTW = false, bool ALN = false>
__global__ TW_DEC_LB(KW > 4 ? 512 : 256, 1) void k_gemv_p(const bf16_t* __restrict__ A, int lda,
                                                               const bf16_t* __restrict__ Wp, int M, int N, int K,
                                                               EpiArgs ea, LnArgs la = LnArgs{}) {
  TW_DEC_PRIO();
  constexpr int NW = KW > 4 ? KW : 4, GPB = NW / KW;
  // (KW = 1: no cross-wave sum, no LDS — see the epilogue)
  __shared__ float red[KW > 1 ? NW : 1][KW > 1 ? 32 : 1][17];
  __shared__ float lnst[ALN ? 32 : 1][2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int gl = wid / KW, kw = wid - gl * KW;
  const int g = blockIdx.x * GPB + gl;
  const int ngroups = (N + 15) >> 4, ns = K >> 5;
  const int nsl = KW * gridDim.y, sl = blockIdx.y * KW + kw;
  const int s0 = (int)((long)sl * ns / nsl), s1 = (int)((long)(sl + 1) * ns / nsl);
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
  if constexpr (ALN) {
    if (la.stats) {
      // statistics from the producer (TW_EPI_RESID_STATS): 8 lanes per row, each combining every 8th of the K/16
      // groups' (mean, M2); one round of loads for all rows
      const int G = K >> 4;
      for (int r0 = 0; r0 < M; r0 += NW * 8) {
        const int r = r0 + (tid >> 3), j0 = tid & 7;
        float mg[GEMV_LN_MAXV * 2], s = 0.f, q = 0.f;
#pragma unroll
        for (int i = 0; i < GEMV_LN_MAXV * 2; ++i) {
          const int j = j0 + 8 * i;
          mg[i] = 0.f;
          if (j < G && r < M) {
            const float2 st = *(const float2*)(la.stats + ((size_t)j * 32 + r) * 2);
            mg[i] = st.x;
            s += st.x;
            q += st.y;
          }
        }
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
          s += __shfl_xor(s, o, 64);
          q += __shfl_xor(q, o, 64);
        }
        const float mean = s / (float)G;
        float d2 = 0.f;
#pragma unroll
        for (int i = 0; i < GEMV_LN_MAXV * 2; ++i)
          if (j0 + 8 * i < G) {
            const float d = mg[i] - mean;
            d2 += d * d;
          }
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) d2 += __shfl_xor(d2, o, 64);
        if (j0 == 0 && r < M) {
          lnst[r][0] = mean;
          lnst[r][1] = rsqrtf((q + 16.f * d2) / (float)K + la.eps);
        }
      }
      __syncthreads();
    }
    const int nc = la.stats ? 0 : K >> 2;  // (the row statistics computed here when no producer wrote them)
    for (int r = wid; nc && r < M; r += NW) {
      const float4* xr = (const float4*)(la.x + (size_t)r * K);
      float4 v[GEMV_LN_MAXV];
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < GEMV_LN_MAXV; ++i) {
        if (64 * i < nc) {  // wave-uniform bound; the chunk index is clamped, not branched on
          v[i] = xr[min(lane + 64 * i, nc - 1)];
          if (lane + 64 * i < nc) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
        }
      }
      const float mean = wave_sum(s) / (float)K;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < GEMV_LN_MAXV; ++i) {
        if (64 * i < nc && lane + 64 * i < nc) {
          const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
          q += (a * a + b * b) + (c * c + d * d);
        }
      }
      const float rstd = rsqrtf(wave_sum(q) / (float)K + la.eps);
      if (lane == 0) {
        lnst[r][0] = mean;
        lnst[r][1] = rstd;
      }
    }
    __syncthreads();
  }
  if (g < ngroups) {
    const bf16_t* wp = Wp + (size_t)g * ns * 512 + lane * 8;
    const bf16_t* ap;
    const bf16_t* ap1 = nullptr;
    if constexpr (APACK) {
      ap = A + lane * 8;  // step s, m-tile t at + s*1024 + t*512
    } else {
      ap = A + (size_t)min(lane & 15, M - 1) * lda + 8 * (lane >> 4);
      ap1 = A + (size_t)min(16 + (lane & 15), M - 1) * lda + 8 * (lane >> 4);
    }
    // ALN: fragment (m-tile t, step st) of LayerNorm(x): lane = row 16t + (lane & 15), k = 32st + 8(lane >> 4) + j
    auto ldA_ln = [&](int st, int t) -> bf16x8 {
      const int m = min(16 * t + (lane & 15), M - 1);
      const int k = 32 * st + 8 * (lane >> 4);
      const float* xp = la.x + (size_t)m * K + k;
      const float4 x0 = *(const float4*)xp, x1 = *(const float4*)(xp + 4);
      const float4 g0 = *(const float4*)(la.g + k), g1 = *(const float4*)(la.g + k + 4);
      const float4 b0 = *(const float4*)(la.b + k), b1 = *(const float4*)(la.b + k + 4);
      const float mean = lnst[m][0], rstd = lnst[m][1];
      bf16x8 r;
      r[0] = (__bf16)((x0.x - mean) * rstd * g0.x + b0.x);
      r[1] = (__bf16)((x0.y - mean) * rstd * g0.y + b0.y);
      r[2] = (__bf16)((x0.z - mean) * rstd * g0.z + b0.z);
      r[3] = (__bf16)((x0.w - mean) * rstd * g0.w + b0.w);
      r[4] = (__bf16)((x1.x - mean) * rstd * g1.x + b1.x);
      r[5] = (__bf16)((x1.y - mean) * rstd * g1.y + b1.y);
      r[6] = (__bf16)((x1.z - mean) * rstd * g1.z + b1.z);
      r[7] = (__bf16)((x1.w - mean) * rstd * g1.w + b1.w);
      return r;
    };
    auto ldA0 = [&](int st) -> bf16x8 {
      if constexpr (ALN) return ldA_ln(st, 0);
      return APACK ? *(const bf16x8*)(ap + (size_t)st * 1024) : *(const bf16x8*)(ap + 32 * st);
    };
    auto ldA1 = [&](int st) -> bf16x8 {
      if constexpr (ALN) return ldA_ln(st, 1);
      return APACK ? *(const bf16x8*)(ap + (size_t)st * 1024 + 512) : *(const bf16x8*)(ap1 + 32 * st);
    };
    auto ldW = [&](int st) -> bf16x8 {
      if constexpr (NTW) {
        typedef short s16x8_nt __attribute__((ext_vector_type(8)));
        const s16x8_nt t = __builtin_nontemporal_load((const s16x8_nt*)(wp + (size_t)st * 512));
        return __builtin_bit_cast(bf16x8, t);
      } else {
        return *(const bf16x8*)(wp + (size_t)st * 512);
      }
    };
    // One batch of NB steps: every load of the batch issued before the first MFMA (the sched_barrier keeps hipcc
    // from interleaving the loads with the MFMAs, which it otherwise does to save registers: 2-3 loads in flight
    // and a dependent memory round trip per step, the latency that dominates these launches, worse still beside an
    // encoder GEMM). n <= NB valid steps: past s1 the loads are clamped to the last step and their MFMAs skipped.
    auto batch = [&](auto NBc, int st0, int n) {
      constexpr int NB = decltype(NBc)::value;
      bf16x8 bw[NB], a0[NB], a1[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int st = min(st0 + u, s1 - 1);
        bw[u] = ldW(st);
        a0[u] = ldA0(st);
        if (TWO) a1[u] = ldA1(st);
      }
      // (not on the bandwidth-bound vocabulary-wide proj_out, NTW: its 3242 waves hide the latency, and 48 live
      // fragments cost it occupancy: 26.2 -> 30.8 us per launch alone)
      if constexpr (!ALN && !NTW) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        if (u < n) {
          c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], bw[u], c0, 0, 0, 0);
          if (TWO) c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], bw[u], c1, 0, 0, 0);
        }
      }
    };
    using IU = std::integral_constant<int, U>;
    int st = s0;
    for (; st + U <= s1; st += U) batch(IU{}, st, U);
    const int rem = s1 - st;  // 0 .. U-1: one predicated batch of the next size up (not a step-by-step loop)
    if (rem > U / 2) batch(IU{}, st, rem);
    else if (rem > U / 4) batch(std::integral_constant<int, (U / 2 > 0 ? U / 2 : 1)>{}, st, rem);
    else if (rem > 0) batch(std::integral_constant<int, (U / 4 > 0 ? U / 4 : 1)>{}, st, rem);
  }
  const int cc = lane & 15, rb = (lane >> 4) * 4;
  auto store = [&](int m, int n, float v) {
    if constexpr (EPI == TW_EPI_PARTIAL) {
      ((float*)ea.out)[((size_t)blockIdx.y * M + m) * ea.ldo + n] = v;
    } else if constexpr (EPI == TW_EPI_GELU_PACKED) {
      if (ea.bias) v += ea.bias[n];
      ((bf16_t*)ea.out)[tw_pack_act_idx(m, n)] = f32_to_bf16(gelu_erf(v));
    } else {
      epi_store<EPI>(ea, m, n, v);
    }
  };
  // TW_EPI_RESID_STATS: the 16 lanes holding one row's 16 columns of group gs reduce the updated values to the
  // group's (mean, M2); xn is this lane's updated element (0 for rows past M: the segment is then skipped whole)
  auto group_stats = [&](int m, int gs, float xn, bool ok) {
    float sm = xn;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sm += __shfl_xor(sm, o, 64);
    const float mg = sm * (1.f / 16.f);
    const float d = ok ? xn - mg : 0.f;
    float q = d * d;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) q += __shfl_xor(q, o, 64);
    if (ok && (lane & 15) == 0) *(float2*)(ea.stats + ((size_t)gs * 32 + m) * 2) = make_float2(mg, q);
  };
  if constexpr (KW == 1) {
    // one wave per column group: its accumulators are the results. Stored straight from registers (16 lanes per
    // row = 16 consecutive columns), so the kernel holds no LDS: the vocabulary-wide proj_out's 811 workgroups then
    // co-reside with an encoder GEMM workgroup (136 KiB of the CU's 160 KiB LDS) several per CU, in one round.
    const int n = g * 16 + cc;
    if constexpr (EPI == TW_EPI_RESID_STATS) {  // (N % 16 == 0: a group's 16 columns are all valid or all not)
      if (g < ngroups) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
          for (int t = 0; t < (TWO ? 2 : 1); ++t) {
            const int m = 16 * t + rb + r;
            const bool ok = m < M;
            float xn = 0.f;
            if (ok) {
              float* o = (float*)ea.out + (size_t)m * ea.ldo + n;
              xn = *o + ((t ? c1[r] : c0[r]) + (ea.bias ? ea.bias[n] : 0.f));
              *o = xn;
            }
            group_stats(m, g, xn, ok);
          }
        }
      }
      return;
    }
    if (g < ngroups && n < N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (rb + r < M) store(rb + r, n, c0[r]);
        if (TWO && 16 + rb + r < M) store(16 + rb + r, n, c1[r]);
      }
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[wid][rb + r][cc] = c0[r];
    if (TWO) red[wid][16 + rb + r][cc] = c1[r];
  }
  __syncthreads();
  constexpr int ROWS = TWO ? 32 : 16;
  for (int e = tid; e < GPB * ROWS * 16; e += NW * 64) {
    const int gg = e / (ROWS * 16), rem = e - gg * ROWS * 16;
    const int m = rem >> 4, c = rem & 15;
    const int n = (blockIdx.x * GPB + gg) * 16 + c;
    if constexpr (EPI == TW_EPI_RESID_STATS) {  // whole waves run each iteration: the 16-lane shuffles are safe
      const int gs = blockIdx.x * GPB + gg;
      const bool ok = m < M && gs < ngroups;
      float xn = 0.f;
      if (ok) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < KW; ++w) v += red[gg * KW + w][m][c];
        float* o = (float*)ea.out + (size_t)m * ea.ldo + n;
        xn = *o + (v + (ea.bias ? ea.bias[n] : 0.f));
        *o = xn;
      }
      group_stats(m, gs, xn, ok);
      continue;
    }
    if (m < M && n < N) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < KW; ++w) v += red[gg * KW + w][m][c];
      store(m, n, v);
    }
  }
}

// k_gemv_pc: k_gemv_p with TWO column groups per wave (32 output columns) sharing each A fragment. At M = 17..32 rows
// a step of k_gemv_p loads one W fragment and two A fragments (the activations, L2-resident and identical for every
// column group); here a step loads two W fragments and the same two A fragments: a third fewer vector-memory
// instructions and VGPRs per weight byte. Every decoder-step kernel shares its CU with an encoder GEMM workgroup
// (run_batches' overlap), whose LDS-DMA keeps the same vector-memory path busy. KW >= 2 K-slices
// per column-group pair, reduced through LDS; epilogues BF16, PARTIAL (split-K) and GELU_PACKED.
template <int EPI, int KW, int U, bool APACK, bool TWO, bool NTW = false>
__global__ TW_DEC_LB(256, 1) void k_gemv_pc(const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ Wp,
                                            int M, int N, int K, EpiArgs ea) {
  TW_DEC_PRIO();
  static_assert(KW == 1 || KW == 2 || KW == 4, "k_gemv_pc: 1, 2 or 4 K-slices");
  constexpr int NW = 4, GPB = NW / KW;  // pairs per workgroup
  __shared__ float red[KW > 1 ? NW : 1][2][KW > 1 ? 32 : 1][17];  // (KW = 1: stored from registers, no LDS)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int gl = wid / KW, kw = wid - gl * KW;
  const int g0 = (blockIdx.x * GPB + gl) * 2;  // this wave's column groups g0, g0 + 1
  const int ngroups = (N + 15) >> 4, ns = K >> 5;
  const int nsl = KW * gridDim.y, sl = blockIdx.y * KW + kw;
  const int s0 = (int)((long)sl * ns / nsl), s1 = (int)((long)(sl + 1) * ns / nsl);
  f32x4 c00 = {0.f, 0.f, 0.f, 0.f}, c01 = c00, c10 = c00, c11 = c00;  // c<group><m-tile>
  if (g0 < ngroups) {
    const bool has1 = g0 + 1 < ngroups;
    const bf16_t* wp0 = Wp + (size_t)g0 * ns * 512 + lane * 8;
    const bf16_t* wp1 = has1 ? wp0 + (size_t)ns * 512 : wp0;  // (an odd last group: its twin re-reads group g0)
    const bf16_t* ap;
    const bf16_t* ap1 = nullptr;
    if constexpr (APACK) {
      ap = A + lane * 8;
    } else {
      ap = A + (size_t)min(lane & 15, M - 1) * lda + 8 * (lane >> 4);
      ap1 = A + (size_t)min(16 + (lane & 15), M - 1) * lda + 8 * (lane >> 4);
    }
    auto ldA0 = [&](int st) -> bf16x8 {
      return APACK ? *(const bf16x8*)(ap + (size_t)st * 1024) : *(const bf16x8*)(ap + 32 * st);
    };
    auto ldA1 = [&](int st) -> bf16x8 {
      return APACK ? *(const bf16x8*)(ap + (size_t)st * 1024 + 512) : *(const bf16x8*)(ap1 + 32 * st);
    };
    // one batch of NB steps, every load issued before the first MFMA (see k_gemv_p)
    auto batch = [&](auto NBc, int st0, int n) {
      constexpr int NB = decltype(NBc)::value;
      bf16x8 b0[NB], b1[NB], a0[NB], a1[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int st = min(st0 + u, s1 - 1);
        if constexpr (NTW) {  // (proj_out: 133 MB streamed once per step, kept out of the caches)
          typedef short s16x8_nt __attribute__((ext_vector_type(8)));
          b0[u] = __builtin_bit_cast(bf16x8, __builtin_nontemporal_load((const s16x8_nt*)(wp0 + (size_t)st * 512)));
          b1[u] = __builtin_bit_cast(bf16x8, __builtin_nontemporal_load((const s16x8_nt*)(wp1 + (size_t)st * 512)));
        } else {
          b0[u] = *(const bf16x8*)(wp0 + (size_t)st * 512);
          b1[u] = *(const bf16x8*)(wp1 + (size_t)st * 512);
        }
        a0[u] = ldA0(st);
        if (TWO) a1[u] = ldA1(st);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        if (u < n) {
          c00 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], b0[u], c00, 0, 0, 0);
          c10 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], b1[u], c10, 0, 0, 0);
          if (TWO) {
            c01 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], b0[u], c01, 0, 0, 0);
            c11 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], b1[u], c11, 0, 0, 0);
          }
        }
      }
    };
    using IU = std::integral_constant<int, U>;
    int st = s0;
    for (; st + U <= s1; st += U) batch(IU{}, st, U);
    const int rem = s1 - st;
    if (rem > U / 2) batch(IU{}, st, rem);
    else if (rem > 0) batch(std::integral_constant<int, (U / 2 > 0 ? U / 2 : 1)>{}, st, rem);
  }
  const int cc = lane & 15, rb = (lane >> 4) * 4;
  if constexpr (KW == 1) {  // the accumulators are the results: 16 lanes per row store 16 consecutive columns
    auto st1 = [&](int m, int n, float v) {
      if constexpr (EPI == TW_EPI_PARTIAL) ((float*)ea.out)[((size_t)blockIdx.y * M + m) * ea.ldo + n] = v;
      else if constexpr (EPI == TW_EPI_GELU_PACKED)
        ((bf16_t*)ea.out)[tw_pack_act_idx(m, n)] = f32_to_bf16(gelu_erf(v + (ea.bias ? ea.bias[n] : 0.f)));
      else epi_store<EPI>(ea, m, n, v);
    };
    const int n0 = g0 * 16 + cc, n1 = n0 + 16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = rb + r;
      if (m < M && n0 < N) st1(m, n0, c00[r]);
      if (m < M && n1 < N) st1(m, n1, c10[r]);
      if (TWO && 16 + m < M && n0 < N) st1(16 + m, n0, c01[r]);
      if (TWO && 16 + m < M && n1 < N) st1(16 + m, n1, c11[r]);
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[wid][0][rb + r][cc] = c00[r];
    red[wid][1][rb + r][cc] = c10[r];
    if (TWO) {
      red[wid][0][16 + rb + r][cc] = c01[r];
      red[wid][1][16 + rb + r][cc] = c11[r];
    }
  }
  __syncthreads();
  constexpr int ROWS = TWO ? 32 : 16;
  for (int e = tid; e < GPB * 2 * ROWS * 16; e += NW * 64) {
    const int pg = e / (2 * ROWS * 16), rem = e - pg * 2 * ROWS * 16;  // pair in the block, then group, row, column
    const int h = rem / (ROWS * 16), r2 = rem - h * ROWS * 16;
    const int m = r2 >> 4, c = r2 & 15;
    const int n = ((blockIdx.x * GPB + pg) * 2 + h) * 16 + c;
    if (m < M && n < N) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < KW; ++w) v += red[pg * KW + w][h][m][c];
      if constexpr (EPI == TW_EPI_PARTIAL) {
        ((float*)ea.out)[((size_t)blockIdx.y * M + m) * ea.ldo + n] = v;
      } else if constexpr (EPI == TW_EPI_GELU_PACKED) {
        if (ea.bias) v += ea.bias[n];
        ((bf16_t*)ea.out)[tw_pack_act_idx(m, n)] = f32_to_bf16(gelu_erf(v));
      } else {
        epi_store<EPI>(ea, m, n, v);
      }
    }
  }
}

template <int EPI, int KW, bool APACK, int U = 5, bool NTW = false>
static void launch_gemv_pc(const bf16_t* A, int lda, const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea,
                           int splits, hipStream_t s) {
  constexpr int GPB = 4 / KW;
  dim3 grid(tw_cdiv(tw_cdiv(tw_cdiv(N, 16), 2), GPB), splits);
  if (M > 16)
    hipLaunchKernelGGL((k_gemv_pc<EPI, KW, U, APACK, true, NTW>), grid, dim3(256), 0, s, A, lda, Wp, M, N, K, ea);
  else
    hipLaunchKernelGGL((k_gemv_pc<EPI, KW, U, APACK, false, NTW>), grid, dim3(256), 0, s, A, lda, Wp, M, N, K, ea);
}

template <int EPI, int KW, int U, bool APACK, bool NTW = false>
static void launch_gemv_p3(const bf16_t* A, int lda, const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea, int splits,
                           hipStream_t s) {
  constexpr int NW = KW > 4 ? KW : 4, GPB = NW / KW;
  dim3 grid(tw_cdiv(tw_cdiv(N, 16), GPB), splits);
  if (M > 16)
    hipLaunchKernelGGL((k_gemv_p<EPI, KW, U, APACK, true, NTW>), grid, dim3(NW * 64), 0, s, A, lda, Wp, M, N, K, ea,
                       LnArgs{});
  else
    hipLaunchKernelGGL((k_gemv_p<EPI, KW, U, APACK, false, NTW>), grid, dim3(NW * 64), 0, s, A, lda, Wp, M, N, K, ea,
                       LnArgs{});
}

// LayerNorm-fused GEMV (ALN): fewer steps per batch (U = 4: a step's A fragments are 4 x 16-byte x loads + gamma /
// beta instead of one 16-byte packed load) and the launcher's K-slice heuristic
template <int EPI, int KW>
static void launch_gemv_ln3(const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea, const LnArgs& la, hipStream_t s) {
  constexpr int NW = KW > 4 ? KW : 4, GPB = NW / KW;
  dim3 grid(tw_cdiv(tw_cdiv(N, 16), GPB), 1);
  if (M > 16)
    hipLaunchKernelGGL((k_gemv_p<EPI, KW, 4, true, true, false, true>), grid, dim3(NW * 64), 0, s, nullptr, 0, Wp, M, N,
                       K, ea, la);
  else
    hipLaunchKernelGGL((k_gemv_p<EPI, KW, 4, true, false, false, true>), grid, dim3(NW * 64), 0, s, nullptr, 0, Wp, M,
                       N, K, ea, la);
}

template <int EPI>
static void launch_gemv_ln(const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea, const LnArgs& la, hipStream_t s) {
  const long groups = tw_cdiv(N, 16);
  const int steps = K / 32;
  int kw = 1;
  while (groups * kw < 1024 && kw < tw_gemv_max_kw && steps >= 8 * kw) kw *= 2;
  if (tw_tune_gemv_kw) kw = tw_tune_gemv_kw;
  if (kw == 1) launch_gemv_ln3<EPI, 1>(Wp, M, N, K, ea, la, s);
  else if (kw == 2) launch_gemv_ln3<EPI, 2>(Wp, M, N, K, ea, la, s);
  else if (kw == 4) launch_gemv_ln3<EPI, 4>(Wp, M, N, K, ea, la, s);
  else launch_gemv_ln3<EPI, 8>(Wp, M, N, K, ea, la, s);
}


#ifndef TW_PROJ_KW4
#define TW_PROJ_KW4 0  // 1: proj_out with 4 K-slices per group: 25 vs 33 us alone, neutral in the bench (A/B)
#endif
template <int EPI, bool APACK>
static void launch_gemv_p2(const bf16_t* A, int lda, const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea, int splits,
                           hipStream_t s) {
  // K-slices per column group: enough waves to put ~4 on every CU while each keeps >= 4 steps
  const long groups = tw_cdiv(N, 16) * (long)splits;
  const int steps = K / 32 / splits;
  int kw = 1;
  while (groups * kw < 1024 && kw < tw_gemv_max_kw && steps >= 8 * kw) kw *= 2;
  // the vocabulary-wide proj_out (3242 column groups): 4 K-slices per group, 25.0 vs 32.8 us per launch with one
  // (scripts/gemv_bench.py, B = 24): more waves in flight per CU for the one launch that streams 133 MB
  const bool wide = N >= tw_gemv_nt_min_n;
  if (TW_PROJ_KW4 && wide && steps >= 16) kw = 4;
  if (wide && steps >= 8 * tw_proj_kw) kw = tw_proj_kw;
  if (tw_tune_gemv_kw) kw = tw_tune_gemv_kw;
  if constexpr (EPI == TW_EPI_BF16 || EPI == TW_EPI_PARTIAL || EPI == TW_EPI_GELU_PACKED) {
    if (tw_gemv_pairs && !wide && !tw_tune_gemv_kw) {  // column-group pairs (a forced K-slice count: k_gemv_p)
      const long pairs = tw_cdiv(tw_cdiv(N, 16), 2) * (long)splits;
      int kp = 2;
      if (pairs * kp < 1024 && steps >= 8 * 4) kp = 4;
      if (kp == 2) launch_gemv_pc<EPI, 2, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
      else launch_gemv_pc<EPI, 4, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
      return;
    }
  }
  if constexpr (EPI == TW_EPI_F32) {
    if (tw_proj_pairs && wide && kw == 1 && splits == 1) {  // proj_out in column-group pairs (variant bit 29: off)
      launch_gemv_pc<EPI, 1, APACK, 6, true>(A, lda, Wp, M, N, K, ea, splits, s);
      return;
    }
  }
  if (kw == 4 && wide) launch_gemv_p3<EPI, 4, 8, APACK, true>(A, lda, Wp, M, N, K, ea, splits, s);
  else if (kw == 2 && wide) launch_gemv_p3<EPI, 2, 8, APACK, true>(A, lda, Wp, M, N, K, ea, splits, s);
  else if (kw == 1 && wide) launch_gemv_p3<EPI, 1, 16, APACK, true>(A, lda, Wp, M, N, K, ea, splits, s);
  else if (kw == 1) launch_gemv_p3<EPI, 1, 16, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
  else if (kw == 2) launch_gemv_p3<EPI, 2, 8, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
  else if (kw == 4) launch_gemv_p3<EPI, 4, 8, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
  else launch_gemv_p3<EPI, 8, 8, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
}

template <int EPI>
static void launch_gemv_p(const bf16_t* A, int a_packed, int lda, const bf16_t* Wp, int M, int N, int K,
                          const EpiArgs& ea, int splits, hipStream_t s) {
  if (a_packed) launch_gemv_p2<EPI, true>(A, lda, Wp, M, N, K, ea, splits, s);
  else launch_gemv_p2<EPI, false>(A, lda, Wp, M, N, K, ea, splits, s);
}

template <int EPI>
static int launch_gemm(const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldw, const EpiArgs& ea,
                       hipStream_t s) {
  if (M <= 32) {
    launch_skinny<EPI>(A, W, M, N, K, lda, ldw, ea, 1, s);
  } else {
    if (tw_gemm_big_enabled == 7) {
      unsigned nwg = tw_cdiv(M, GB_BM) * tw_cdiv(N, GH_BN);
      hipLaunchKernelGGL(k_gemm_h<EPI>, dim3(nwg), dim3(256), 0, s, A, W, M, N, K, lda, ldw, ea);
    } else if (tw_gemm_big_enabled == 5) {
      unsigned nwg = tw_cdiv(M, GB_BM) * tw_cdiv(N, GB_BN);
      hipLaunchKernelGGL(k_gemm_8p<EPI>, dim3(nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
    } else if (tw_gemm_big_enabled == 10) {
      unsigned nwg = tw_cdiv(M, GB_BM) * tw_cdiv(N, GB_BN);
      hipLaunchKernelGGL(k_gemm_big32<EPI>, dim3(nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
    } else if (tw_gemm_big_enabled == 9 && K >= 2 * GB_BK) {
      unsigned nwg = tw_cdiv(M, GB_BM) * tw_cdiv(N, GB_BN);
      hipLaunchKernelGGL(k_gemm_kh<EPI>, dim3(nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
    } else if (tw_gemm_big_enabled == 8) {
      unsigned nwg = tw_cdiv(M, 256) * tw_cdiv(N, 256);
      hipLaunchKernelGGL(k_gemm_4w<EPI>, dim3(nwg), dim3(256), 0, s, A, W, M, N, K, lda, ldw, ea);
    } else if (tw_gemm_big_enabled == 6) {
      unsigned nwg = tw_cdiv(M, GB_BM) * tw_cdiv(N, GB_BN);
      const unsigned grid = std::min<unsigned>(nwg, (unsigned)(tw_num_cus() & ~7));
      hipLaunchKernelGGL(k_gemm_8pp<EPI>, dim3(grid), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
    } else if (tw_gemm_big_enabled >= 3) {
      const int v = tw_gemm_big_enabled;
      if (v == 3) {  // 256x256, 2 stages, counted-vmcnt loop, setprio
        unsigned nwg = tw_cdiv(M, GB_BM) * tw_cdiv(N, 256);
        hipLaunchKernelGGL((k_gemm_ns<EPI, 256, 2, true>), dim3(nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
      } else {  // 256x128, 3 stages
        unsigned nwg = tw_cdiv(M, GB_BM) * tw_cdiv(N, 128);
        hipLaunchKernelGGL((k_gemm_ns<EPI, 128, 3, false>), dim3(nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
      }
    } else if (tw_gemm_big_enabled) {
      unsigned nwg = tw_cdiv(M, GB_BM) * tw_cdiv(N, GB_BN);
      hipLaunchKernelGGL(k_gemm_big<EPI>, dim3(nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
    } else {
      unsigned nwg = tw_cdiv(M, G_BM) * tw_cdiv(N, G_BN);
      hipLaunchKernelGGL(k_gemm_tile<EPI>, dim3(nwg), dim3(256), 0, s, A, W, M, N, K, lda, ldw, ea);
    }
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
  ea.group_m = tw_group_for(N);
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

extern "C" int tw_gemm_bf16_partial(const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldw,
                                    int splits, float* part, int ldp, void* stream) {
  TW_REQUIRE(A && W && part, "tw_gemm_bf16_partial: null pointer");
  TW_REQUIRE(M > 0 && M <= 32 && N > 0 && K > 0 && K % 32 == 0, "tw_gemm_bf16_partial: M=%d N=%d K=%d (M <= 32, K %% 32)",
             M, N, K);
  TW_REQUIRE(splits >= 1 && splits <= 16 && splits <= K / 32, "tw_gemm_bf16_partial: splits=%d", splits);
  TW_REQUIRE(lda % 8 == 0 && ldw % 8 == 0 && lda >= K && ldw >= K && ldp >= N, "tw_gemm_bf16_partial: lda=%d ldw=%d ldp=%d",
             lda, ldw, ldp);
  EpiArgs ea{part, ldp, nullptr, nullptr, 0, 0, 0, 0, 0};
  launch_skinny<TW_EPI_PARTIAL>(A, W, M, N, K, lda, ldw, ea, splits, (hipStream_t)stream);
  return tw_check_launch("tw_gemm_bf16_partial");
}

extern "C" int tw_pack_weight(const bf16_t* W, int N, int K, int ldw, bf16_t* Wp, void* stream) {
  TW_REQUIRE(W && Wp && N > 0 && K > 0 && K % 32 == 0 && ldw >= K && ldw % 8 == 0,
             "tw_pack_weight: N=%d K=%d ldw=%d (K %% 32, ldw %% 8)", N, K, ldw);
  const long nchunks = (long)tw_cdiv(N, 16) * (K / 32) * 64;
  hipLaunchKernelGGL(k_pack_weight, dim3(tw_cdiv(nchunks, 256)), dim3(256), 0, (hipStream_t)stream, W, N, K, ldw, Wp,
                     nchunks);
  return tw_check_launch("tw_pack_weight");
}

extern "C" int tw_gemv_packed(const bf16_t* A, int a_packed, int lda, const bf16_t* Wp, int M, int N, int K, int epi,
                              void* out, int ldo, const float* bias, int splits, void* stream) {
  TW_REQUIRE(A && Wp && out, "tw_gemv_packed: null pointer");
  TW_REQUIRE(M > 0 && M <= 32 && N > 0 && K > 0 && K % 32 == 0, "tw_gemv_packed: M=%d N=%d K=%d (M <= 32, K %% 32)", M,
             N, K);
  TW_REQUIRE(a_packed || (lda >= K && lda % 8 == 0), "tw_gemv_packed: lda=%d", lda);
  TW_REQUIRE(splits >= 1 && splits <= 16 && splits <= K / 32, "tw_gemv_packed: splits=%d", splits);
  TW_REQUIRE(splits == 1 || epi == TW_EPI_PARTIAL_F32, "tw_gemv_packed: split-K needs the PARTIAL epilogue");
  EpiArgs ea{out, ldo, bias, nullptr, 0, 0, 0, 0, 0};
  hipStream_t s = (hipStream_t)stream;
  switch (epi) {
    case TW_EPI_BF16: launch_gemv_p<TW_EPI_BF16>(A, a_packed, lda, Wp, M, N, K, ea, splits, s); break;
    case TW_EPI_F32: launch_gemv_p<TW_EPI_F32>(A, a_packed, lda, Wp, M, N, K, ea, splits, s); break;
    case TW_EPI_GELU_PACKED:
      TW_REQUIRE(N % 32 == 0, "tw_gemv_packed: GELU_PACKED needs N %% 32 (it is the next GEMV's K)");
      launch_gemv_p<TW_EPI_GELU_PACKED>(A, a_packed, lda, Wp, M, N, K, ea, splits, s);
      break;
    case TW_EPI_PARTIAL_F32:
      TW_REQUIRE(ldo >= N, "tw_gemv_packed: ldo=%d < N", ldo);
      ea.bias = nullptr;
      launch_gemv_p<TW_EPI_PARTIAL>(A, a_packed, lda, Wp, M, N, K, ea, splits, s);
      break;
    case TW_EPI_RESID_F32:  // out[m][n] += A.W^T + bias: the decoder's residual update, one writer per element
      TW_REQUIRE(ldo >= N, "tw_gemv_packed: ldo=%d < N", ldo);
      launch_gemv_p<TW_EPI_RESID_F32>(A, a_packed, lda, Wp, M, N, K, ea, splits, s);
      break;
    default: tw_set_error("tw_gemv_packed: unsupported epilogue %d", epi); return TW_ERR_ARG;
  }
  return tw_check_launch("tw_gemv_packed");
}

extern "C" int tw_gemv_packed_ln(const float* x, const float* gamma, const float* beta, float eps, const bf16_t* Wp,
                                 int M, int N, int K, int epi, void* out, int ldo, const float* bias, void* stream) {
  TW_REQUIRE(x && gamma && beta && Wp && out, "tw_gemv_packed_ln: null pointer");
  TW_REQUIRE(M > 0 && M <= 32 && N > 0 && K > 0 && K % 32 == 0 && K <= 256 * GEMV_LN_MAXV,
             "tw_gemv_packed_ln: M=%d N=%d K=%d (M <= 32, K %% 32, K <= %d)", M, N, K, 256 * GEMV_LN_MAXV);
  EpiArgs ea{out, ldo, bias, nullptr, 0, 0, 0, 0, 0};
  const LnArgs la{x, gamma, beta, eps, nullptr};
  hipStream_t s = (hipStream_t)stream;
  switch (epi) {
    case TW_EPI_BF16: launch_gemv_ln<TW_EPI_BF16>(Wp, M, N, K, ea, la, s); break;
    case TW_EPI_F32: launch_gemv_ln<TW_EPI_F32>(Wp, M, N, K, ea, la, s); break;
    case TW_EPI_GELU_PACKED:
      TW_REQUIRE(N % 32 == 0, "tw_gemv_packed_ln: GELU_PACKED needs N %% 32 (it is the next GEMV's K)");
      launch_gemv_ln<TW_EPI_GELU_PACKED>(Wp, M, N, K, ea, la, s);
      break;
    default: tw_set_error("tw_gemv_packed_ln: unsupported epilogue %d", epi); return TW_ERR_ARG;
  }
  return tw_check_launch("tw_gemv_packed_ln");
}

extern "C" int tw_gemv_packed_stats(const bf16_t* A, int a_packed, int lda, const bf16_t* Wp, int M, int N, int K,
                                    float* x, int ldx, const float* bias, float* stats, void* stream) {
  TW_REQUIRE(A && Wp && x && stats, "tw_gemv_packed_stats: null pointer");
  TW_REQUIRE(M > 0 && M <= 32 && N > 0 && N % 16 == 0 && K > 0 && K % 32 == 0 && ldx >= N,
             "tw_gemv_packed_stats: M=%d N=%d K=%d ldx=%d (M <= 32, N %% 16, K %% 32)", M, N, K, ldx);
  TW_REQUIRE(a_packed || (lda >= K && lda % 8 == 0), "tw_gemv_packed_stats: lda=%d", lda);
  EpiArgs ea{x, ldx, bias, nullptr, 0, 0, 0, 0, 0};
  ea.stats = stats;
  launch_gemv_p<TW_EPI_RESID_STATS>(A, a_packed, lda, Wp, M, N, K, ea, 1, (hipStream_t)stream);
  return tw_check_launch("tw_gemv_packed_stats");
}

extern "C" int tw_gemv_packed_lnst(const float* x, const float* stats, const float* gamma, const float* beta, float eps,
                                   const bf16_t* Wp, int M, int N, int K, int epi, void* out, int ldo,
                                   const float* bias, void* stream) {
  TW_REQUIRE(x && stats && gamma && beta && Wp && out, "tw_gemv_packed_lnst: null pointer");
  TW_REQUIRE(M > 0 && M <= 32 && N > 0 && K > 0 && K % 32 == 0 && K <= 256 * GEMV_LN_MAXV,
             "tw_gemv_packed_lnst: M=%d N=%d K=%d (M <= 32, K %% 32, K <= %d)", M, N, K, 256 * GEMV_LN_MAXV);
  EpiArgs ea{out, ldo, bias, nullptr, 0, 0, 0, 0, 0};
  const LnArgs la{x, gamma, beta, eps, stats};
  hipStream_t s = (hipStream_t)stream;
  switch (epi) {
    case TW_EPI_BF16: launch_gemv_ln<TW_EPI_BF16>(Wp, M, N, K, ea, la, s); break;
    case TW_EPI_F32: launch_gemv_ln<TW_EPI_F32>(Wp, M, N, K, ea, la, s); break;
    case TW_EPI_GELU_PACKED:
      TW_REQUIRE(N % 32 == 0, "tw_gemv_packed_lnst: GELU_PACKED needs N %% 32 (it is the next GEMV's K)");
      launch_gemv_ln<TW_EPI_GELU_PACKED>(Wp, M, N, K, ea, la, s);
      break;
    default: tw_set_error("tw_gemv_packed_lnst: unsupported epilogue %d", epi); return TW_ERR_ARG;
  }
  return tw_check_launch("tw_gemv_packed_lnst");
}

// ------------------------------------------------------------------------------------------------
// k_gemm_mx: the encoder projections in MX fp8 (BASELINE config 5). C[M][N] = A[M][K] . W[N][K]^T with e4m3
// operands and one e8m0 scale per 32 K elements of every A row and W row (tw_common.h "MX fp8"), on
// v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate per clock: MI355X_MICROARCH.md § Matrix cores).
// The structure is k_gemm_big's with BK = 128 elements: a K-step row is still 128 bytes, so the LDS-DMA staging,
// the bank swizzle and the 24 ds_read_b128 per wave per K-step are unchanged, while one K-step now covers twice
// the K (32 MFMAs of 16x16x128 per wave instead of 64 of 16x16x32). The K-step's scales (one dword per tile row:
// 1 KiB for A, 1 KiB for W, contiguous in HBM) ride along by LDS-DMA from waves 0 and 1. Lane map of the
// 16x16x128 f8 operand, measured by scripts/exp/mx_probe.hip: lane l (row l % 16, group g = l / 16) holds K bytes
// [16g, 16g+16) in its first 16 bytes and [64+16g, 64+16g+16) in its last 16, while its scale VGPR scales K block
// g = [32g, 32g+32) of row l % 16 (the hardware pairs them up: block g's bytes sit in lane groups 2(g%2), 2(g%2)+1).
// So a lane reads 16-byte chunks g and g+4 of the K-step row, and its own scale byte with one ds_read_u8.
// ------------------------------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(8))) int i32x8;
#define MX_BK 128                                  // K elements (= bytes) per K-step
#define MX_TILE (GB_BM * MX_BK)                    // 32 KiB: one operand tile of one K-step
#define MX_STAGE (2 * MX_TILE + 2 * GB_BM * 4)     // A | W | A scales | W scales = 66 KiB

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm_mx(const uint8_t* __restrict__ A, const uint8_t* __restrict__ W,
                                                    const uint8_t* __restrict__ Sa, const uint8_t* __restrict__ Sw,
                                                    int M, int N, int K, int lda, int ldw, int Mp, int Np,
                                                    EpiArgs ea) {
  // K loop: 2 x 66 KiB; epilogue: 8 x [64][68] f32 = 136 KiB (one array: see cdna_hip_programming.md §5 trap (a))
  __shared__ __attribute__((aligned(16))) uint8_t smem[8 * 64 * GB_EPI_LD * 4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + GB_BM - 1) / GB_BM, ntn = (N + GB_BN - 1) / GB_BN;
  const int nwg = ntm * ntn;
  const int orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int tm, tn;
  tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
  const int m0 = tm * GB_BM, n0 = tn * GB_BN;

  const uint8_t* ga[4];
  const uint8_t* gw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wid + i) + (lane >> 3);
    const int ch = (lane & 7) ^ gb_swz(row);
    ga[i] = A + (size_t)min(m0 + row, M - 1) * lda + ch * 16;
    gw[i] = W + (size_t)min(n0 + row, N - 1) * ldw + ch * 16;
  }
  // scales of K-step kt: rows m0..m0+255 of [K/128][Mp][4] are 1 KiB contiguous (Mp, Np: multiples of 256)
  const uint8_t* gs = wid == 0 ? Sa + (size_t)m0 * 4 + lane * 16 : Sw + (size_t)n0 * 4 + lane * 16;
  const size_t gs_step = (size_t)(wid == 0 ? Mp : Np) * 4;
  auto stage = [&](int buf, int kt) {
    uint8_t* As = smem + buf * MX_STAGE;
    uint8_t* Ws = As + MX_TILE;
    const int k0 = kt * MX_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rb = 8 * (4 * wid + i) * MX_BK;
      __builtin_amdgcn_global_load_lds((const void*)(ga[i] + k0), (lds_void_t*)(As + rb), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(gw[i] + k0), (lds_void_t*)(Ws + rb), 16, 0, 0);
    }
    if (wid < 2)
      __builtin_amdgcn_global_load_lds((const void*)(gs + kt * gs_step), (lds_void_t*)(As + 2 * MX_TILE + wid * 1024),
                                       16, 0, 0);
  };

  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / MX_BK;
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
    const uint8_t* As = smem + cur * MX_STAGE;
    const uint8_t* Ws = As + MX_TILE;
    const uint8_t* SAs = As + 2 * MX_TILE;
    const uint8_t* SWs = SAs + 1024;
    i32x8 bfr[4];
    int sb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wc * 64 + j * 16 + fr;
      const uint8_t* p = Ws + col * MX_BK;
      const int4 lo = *(const int4*)(p + ((fq ^ gb_swz(col)) << 4));
      const int4 hi = *(const int4*)(p + (((fq + 4) ^ gb_swz(col)) << 4));
      bfr[j] = (i32x8){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      sb[j] = SWs[col * 4 + fq];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr * 128 + i * 16 + fr;
      const uint8_t* p = As + row * MX_BK;
      const int4 lo = *(const int4*)(p + ((fq ^ gb_swz(row)) << 4));
      const int4 hi = *(const int4*)(p + (((fq + 4) ^ gb_swz(row)) << 4));
      const i32x8 af = (i32x8){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      const int sa = SAs[row * 4 + fq];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[j], acc[i][j], 0, 0, 0, sa, 0, sb[j]);
    }
    __syncthreads();
  }

  // ---- epilogue through LDS, as k_gemm_big (4 consecutive columns per lane in the read-back)
  const int ncol0 = n0 + wc * 64;
  const int rc = (lane & 15) * 4;
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ea.bias) {
    const int n = ncol0 + rc;
    bias4.x = ea.bias[min(n, N - 1)];
    bias4.y = ea.bias[min(n + 1, N - 1)];
    bias4.z = ea.bias[min(n + 2, N - 1)];
    bias4.w = ea.bias[min(n + 3, N - 1)];
  }
  float* wimg = (float*)smem + wid * (64 * GB_EPI_LD);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int ib = 4 * half;
    if (half) __syncthreads();
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) wimg[(ii * 16 + fq * 4 + r) * GB_EPI_LD + j * 16 + fr] = acc[ib + ii][j][r];
    __syncthreads();
    const int mrow0 = m0 + wr * 128 + ib * 16;
#pragma unroll 4
    for (int rr = 0; rr < 16; ++rr) {
      const int lr = rr * 4 + (lane >> 4);
      const int m = mrow0 + lr;
      float4 v = *(const float4*)(wimg + lr * GB_EPI_LD + rc);
      v.x += bias4.x; v.y += bias4.y; v.z += bias4.z; v.w += bias4.w;
      if constexpr (EPI == TW_EPI_GELU_MX) {
        // fc1 -> fc2 operand: GELU, then MX-quantise; the 8 lanes of a 32-column block share one scale
        // (N % 256 == 0 is checked on the host, so every lane of the group is inside N)
        v = gelu_erf4(v);
        const uint32_t sbyte = mx_scale_byte(mx_group8_max(abs4max(v.x, v.y, v.z, v.w)));
        const uint32_t w = mx_pack4(v.x, v.y, v.z, v.w, mx_inv_scale(sbyte));
        if (m < M) {
          *(uint32_t*)((uint8_t*)ea.out + (size_t)m * ea.ldo + ncol0 + rc) = w;
          if ((lane & 7) == 0) ea.sout[tw_mx_sidx(m, (ncol0 + rc) >> 5, ea.s_rows)] = (uint8_t)sbyte;
        }
      } else {
        if (m < M && ncol0 + rc < N) epi_store4<EPI>(ea, m, ncol0 + rc, N, v);
      }
    }
  }
}

// k_gemm_8p_mx: k_gemm_8p's 8-phase ping-pong schedule on MX fp8 operands (tw_gemm_mx's FFN-shape kernel).
// A K-tile is 128 fp8 elements = 128 bytes per row, so the four half-tiles are the same 16 KiB and the per-phase
// ds_reads the same count (a 16x16x128 fragment is 32 bytes = two ds_read_b128), while each phase issues 8
// v_mfma_scale_f32_16x16x128_f8f6f4 (32 cycles) where the bf16 kernel issued 16 16x16x32 (16 cycles): the same
// MFMA time per phase for twice the K. Scales: per K-tile 1 KiB of A and 1 KiB of W scale dwords, one 4-byte
// LDS-DMA per wave (waves 0-3: A rows 64w..64w+63, waves 4-7: W rows), staged with half-tile A0 in phase 1 and read
// into registers (12 bytes per lane) in phase 1 of the K-tile that uses them: WAR distance 4 phases; the vmcnt
// counts of phases 1 and 2 grow by that one DMA (5 instead of 4).
#define MX8_SC (8 * 128 * MX_BK)  // byte offset of the scale area: after 2 buffers x 4 half-tiles of 16 KiB
template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm_8p_mx(const uint8_t* __restrict__ A, const uint8_t* __restrict__ W,
                                                       const uint8_t* __restrict__ Sa, const uint8_t* __restrict__ Sw,
                                                       int M, int N, int K, int lda, int ldw, int Mp, int Np,
                                                       EpiArgs ea) {
  // K loop: 128 KiB of half-tiles + 2 x 2 KiB scales; epilogue: 8 x [64][68] f32 = 136 KiB (one array)
  __shared__ __attribute__((aligned(16))) uint8_t smem[8 * 64 * GB_EPI_LD * 4];
  constexpr int HT = 128 * MX_BK;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + GB_BM - 1) / GB_BM, ntn = (N + GB_BN - 1) / GB_BN;
  const int nwg = ntm * ntn;
  const int orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int tm, tn;
  tw_tile_grouped(wgid, ntm, ntn, ea.group_m, tm, tn);
  const int m0 = tm * GB_BM, n0 = tn * GB_BN;
  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;

  const uint8_t* gsrc[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 8 * (2 * wid + i) + (lane >> 3);
      const int ch = (lane & 7) ^ gb_swz(row);
      gsrc[h][i] = h < 2 ? A + (size_t)min(m0 + 128 * h + row, M - 1) * lda + ch * 16
                         : W + (size_t)min(n0 + 128 * (h - 2) + row, N - 1) * ldw + ch * 16;
    }
  // scale DMA: wave w < 4 -> A scale dwords of rows 64w + lane, w >= 4 -> W rows 64(w-4) + lane
  const uint8_t* gsc = wid < 4 ? Sa + (size_t)(m0 + 64 * wid + lane) * 4 : Sw + (size_t)(n0 + 64 * (wid - 4) + lane) * 4;
  const size_t gsc_step = (size_t)(wid < 4 ? Mp : Np) * 4;
  auto stage = [&](int buf, int h, int kt) {
    uint8_t* dst = smem + (buf * 4 + h) * HT;
    const int k0 = kt * MX_BK;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(gsrc[h][i] + k0), (lds_void_t*)(dst + 8 * (2 * wid + i) * MX_BK),
                                       16, 0, 0);
  };
  auto stage_sc = [&](int buf, int kt) {
    __builtin_amdgcn_global_load_lds((const void*)(gsc + kt * gsc_step),
                                     (lds_void_t*)(smem + MX8_SC + buf * 2048 + wid * 256), 4, 0, 0);
  };

  i32x8 af[4], bfr[2];
  int sa[2][4], sb[2][2];
  auto frag = [&](const uint8_t* base, int row) {
    const uint8_t* p = base + row * MX_BK;
    const int4 lo = *(const int4*)(p + ((fq ^ gb_swz(row)) << 4));
    const int4 hi = *(const int4*)(p + (((fq + 4) ^ gb_swz(row)) << 4));
    return (i32x8){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  };
  auto readA = [&](int buf, int mh) {
    const uint8_t* As = smem + (buf * 4 + mh) * HT;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(As, 64 * wr + 16 * i + fr);
  };
  auto readB = [&](int buf, int nh) {
    const uint8_t* Bs = smem + (buf * 4 + 2 + nh) * HT;
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[j] = frag(Bs, 32 * wc + 16 * j + fr);
  };
  auto readS = [&](int buf) {  // this lane's scale bytes: (tile row, K block fq) of every fragment of the K-tile
    const uint8_t* S = smem + MX8_SC + buf * 2048;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int i = 0; i < 4; ++i) sa[mh][i] = S[(128 * mh + 64 * wr + 16 * i + fr) * 4 + fq];
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int j = 0; j < 2; ++j) sb[nh][j] = S[1024 + (128 * nh + 32 * wc + 16 * j + fr) * 4 + fq];
  };
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto mfma_q = [&](auto MH, auto NH) {
    constexpr int mh = decltype(MH)::value, nh = decltype(NH)::value;
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[mh][nh][i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[mh][nh][i][j], 0, 0, 0,
                                                                             sa[mh][i], 0, sb[nh][j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  const int nk = K / MX_BK;
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, 0);
  stage_sc(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();
  auto ktile = [&](int t, auto NXT) {
    constexpr bool nxt = decltype(NXT)::value;
    const int buf = t & 1, nb = buf ^ 1;
    // phase 1: quadrant (A0, B0); this K-tile's scales into registers
    readB(buf, 0);
    __builtin_amdgcn_sched_barrier(0);
    readA(buf, 0);
    readS(buf);
    if constexpr (nxt) {
      stage(nb, 0, t + 1);
      stage_sc(nb, t + 1);
      p8_vmcnt<5>();  // B1 of tile t (phase 3 of t-1)
    } else {
      p8_vmcnt<2>();
    }
    mfma_q(I0{}, I0{});
    // phase 2: (A0, B1)
    readB(buf, 1);
    if constexpr (nxt) {
      stage(nb, 2, t + 1);
      p8_vmcnt<5>();  // A1 of tile t (phase 4 of t-1)
    } else {
      p8_vmcnt<0>();
    }
    mfma_q(I0{}, I1{});
    // phase 3: (A1, B1)
    readA(buf, 1);
    if constexpr (nxt) stage(nb, 3, t + 1);
    mfma_q(I1{}, I1{});
    // phase 4: (A1, B0)
    readB(buf, 0);
    if constexpr (nxt) {
      stage(nb, 1, t + 1);
      p8_vmcnt<4>();  // A0 + scales, B0 of tile t+1 (phases 1, 2 of t)
    }
    mfma_q(I1{}, I0{});
  };
  using BT = std::integral_constant<bool, true>;
  using BF = std::integral_constant<bool, false>;
  for (int t = 0; t + 1 < nk; ++t) ktile(t, BT{});
  ktile(nk - 1, BF{});
  if (wr == 0) __builtin_amdgcn_s_barrier();
  __syncthreads();

  // epilogue as k_gemm_8p: 8 consecutive columns per lane, 8 lanes per 64-column row
  const int rc = (lane & 7) * 8;
  const int ncol = n0 + (rc < 32 ? 32 * wc + rc : 128 + 32 * wc + rc - 32);
  float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
  if (ea.bias) {
    b0.x = ea.bias[min(ncol, N - 1)];
    b0.y = ea.bias[min(ncol + 1, N - 1)];
    b0.z = ea.bias[min(ncol + 2, N - 1)];
    b0.w = ea.bias[min(ncol + 3, N - 1)];
    b1.x = ea.bias[min(ncol + 4, N - 1)];
    b1.y = ea.bias[min(ncol + 5, N - 1)];
    b1.z = ea.bias[min(ncol + 6, N - 1)];
    b1.w = ea.bias[min(ncol + 7, N - 1)];
  }
  float* wimg = (float*)smem + wid * (64 * GB_EPI_LD);
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
    if (mh) __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            wimg[(i * 16 + fq * 4 + r) * GB_EPI_LD + nh * 32 + j * 16 + fr] = acc[mh][nh][i][j][r];
    __syncthreads();
    const int mrow0 = m0 + 128 * mh + 64 * wr;
#pragma unroll 4
    for (int rr = 0; rr < 8; ++rr) {
      const int lr = rr * 8 + (lane >> 3);
      const int m = mrow0 + lr;
      float4 v0 = *(const float4*)(wimg + lr * GB_EPI_LD + rc);
      float4 v1 = *(const float4*)(wimg + lr * GB_EPI_LD + rc + 4);
      v0.x += b0.x; v0.y += b0.y; v0.z += b0.z; v0.w += b0.w;
      v1.x += b1.x; v1.y += b1.y; v1.z += b1.z; v1.w += b1.w;
      if constexpr (EPI == TW_EPI_GELU_MX) {
        // a 32-column block is 4 lanes x 8 columns (lanes 0-3 / 4-7 of the row's 8): absmax over xor 1, 2
        v0 = gelu_erf4(v0);
        v1 = gelu_erf4(v1);
        float a = fmaxf(abs4max(v0.x, v0.y, v0.z, v0.w), abs4max(v1.x, v1.y, v1.z, v1.w));
        a = fmaxf(a, __shfl_xor(a, 1, 64));
        a = fmaxf(a, __shfl_xor(a, 2, 64));
        const uint32_t sbyte = mx_scale_byte(a);
        const float inv = mx_inv_scale(sbyte);
        uint2 w;
        w.x = mx_pack4(v0.x, v0.y, v0.z, v0.w, inv);
        w.y = mx_pack4(v1.x, v1.y, v1.z, v1.w, inv);
        if (m < M) {
          *(uint2*)((uint8_t*)ea.out + (size_t)m * ea.ldo + ncol) = w;
          if ((lane & 3) == 0) ea.sout[tw_mx_sidx(m, ncol >> 5, ea.s_rows)] = (uint8_t)sbyte;
        }
      } else {
        if (m < M && ncol < N) epi_store8<EPI>(ea, m, ncol, N, v0, v1);
      }
    }
  }
}

// tw_gemm_mx kernel choice: 0 = by shape (default), 1 = k_gemm_mx, 8 = k_gemm_8p_mx (tw_gemm_mx_set_variant, A/B).
// Measured (scripts/gemm_bench.py, B = 24 and 64 windows): the 8-phase kernel wins on the long-K / wide-N FFN
// shapes (fc1 +10-14 %, fc2 +14-18 %) and on o_proj at M = 96000 (+11 %); the 2-stage kernel on qkv (+3-5 %) and
// on o_proj at M = 36000 (+2 %).
static int tw_gemm_mx_variant = 0;
extern "C" int tw_gemm_mx_set_variant(int v) {
  tw_gemm_mx_variant = (v == 1 || v == 8) ? v : 0;
  return 0;
}
static inline bool mx_use_8p(int M, int N, int K) {
  if (tw_gemm_mx_variant) return tw_gemm_mx_variant == 8;
  return N >= 4096 || K >= 4096 || (N <= 1280 && M >= 65536);
}

template <int EPI>
static void launch_gemm_mx(const uint8_t* A, const uint8_t* Sa, const uint8_t* W, const uint8_t* Sw, int M, int N,
                           int K, int lda, int ldw, int Mp, int Np, const EpiArgs& ea, hipStream_t s) {
  const unsigned nwg = tw_cdiv(M, GB_BM) * tw_cdiv(N, GB_BN);
  if (!mx_use_8p(M, N, K))
    hipLaunchKernelGGL(k_gemm_mx<EPI>, dim3(nwg), dim3(512), 0, s, A, W, Sa, Sw, M, N, K, lda, ldw, Mp, Np, ea);
  else
    hipLaunchKernelGGL(k_gemm_8p_mx<EPI>, dim3(nwg), dim3(512), 0, s, A, W, Sa, Sw, M, N, K, lda, ldw, Mp, Np, ea);
}

extern "C" int tw_gemm_mx(const uint8_t* A, const uint8_t* Sa, const uint8_t* W, const uint8_t* Sw, int M, int N,
                          int K, int lda, int ldw, int Mp, int Np, int epi, void* out, int ldo, const float* bias,
                          uint8_t* sout, int sout_rows, void* stream) {
  TW_REQUIRE(A && Sa && W && Sw && out, "tw_gemm_mx: null pointer");
  TW_REQUIRE(M > 0 && N > 0 && K > 0 && K % MX_BK == 0, "tw_gemm_mx: M=%d N=%d K=%d (K %% 128 required)", M, N, K);
  TW_REQUIRE(lda % 16 == 0 && ldw % 16 == 0 && lda >= K && ldw >= K, "tw_gemm_mx: lda=%d ldw=%d", lda, ldw);
  TW_REQUIRE(Mp % GB_BM == 0 && Mp >= M && Np % GB_BN == 0 && Np >= N,
             "tw_gemm_mx: scale row pads Mp=%d Np=%d must be multiples of 256 covering M=%d N=%d", Mp, Np, M, N);
  EpiArgs ea{out, ldo, bias, nullptr, 0, 0, 0, 0, 0, nullptr, 0};
  ea.group_m = tw_group_for(N);
  hipStream_t s = (hipStream_t)stream;
  switch (epi) {
    case TW_EPI_BF16: launch_gemm_mx<TW_EPI_BF16>(A, Sa, W, Sw, M, N, K, lda, ldw, Mp, Np, ea, s); break;
    case TW_EPI_RESID_F32: launch_gemm_mx<TW_EPI_RESID_F32>(A, Sa, W, Sw, M, N, K, lda, ldw, Mp, Np, ea, s); break;
    case TW_EPI_F32: launch_gemm_mx<TW_EPI_F32>(A, Sa, W, Sw, M, N, K, lda, ldw, Mp, Np, ea, s); break;
    case TW_EPI_GELU_MX:
      TW_REQUIRE(sout && sout_rows >= M && N % GB_BN == 0 && ldo >= N && ldo % 4 == 0,
                 "tw_gemm_mx: GELU_MX needs scale output (sout_rows %d >= M), N %% 256 (N=%d), ldo %% 4", sout_rows, N);
      ea.sout = sout;
      ea.s_rows = sout_rows;
      launch_gemm_mx<TW_EPI_GELU_MX>(A, Sa, W, Sw, M, N, K, lda, ldw, Mp, Np, ea, s);
      break;
    default: tw_set_error("tw_gemm_mx: unsupported epilogue %d", epi); return TW_ERR_ARG;
  }
  return tw_check_launch("tw_gemm_mx");
}
