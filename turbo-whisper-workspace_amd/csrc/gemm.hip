// bf16 "NT" GEMM on MFMA: C[M][N] = A[M][K] . W[N][K]^T with fused Whisper epilogues.
//
// Replaces every nn.Linear / Conv1d-as-GEMM of the Whisper encoder and decoder
// ($TF/models/whisper/modeling_whisper.py:279-282 q/k/v/o, :375-376 fc1/fc2, :566-567 conv stem,
// :970 proj_out) with one CDNA4 kernel family. W keeps PyTorch's Linear layout [out][in] so both
// operands are K-contiguous: each MFMA lane fragment is one 16-byte run of a row.
//
// Large-M path (encoder, cross-KV projection, conv stem): 256x256x64 tiles, 8 waves, LDS-DMA staging, XCD-aware
// block remap. Two kernels of that tile, chosen per context by the engine (tw_gemm_set_variant): k_gemm_8p (8-phase
// ping-pong, fastest alone) and k_gemm_big (one barrier per K-tile, 184 VGPRs: a decoder wave co-resides on every
// SIMD, so it is the kernel queued beside a running decode step). Earlier variants measured slower are archived in
// scripts/exp/archive/ (not built).
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

// Large-M kernel per context (tw_gemm_set_variant): 5 = k_gemm_8p (alone), 1 = k_gemm_big (beside a decode).
static int tw_gemm_kernel = 1;
// Epilogue form of the large-M kernels (tw_gemm_set_epilogue): 0 = the f32 LDS image of the row-major accumulators
// (gemm_epi_128x64 / k_gemm_8p's own), 1 = transposed accumulators (gemm_epi_tr). 0: the transposed form measured
// 0.94-0.99x on the encoder shapes (1.06x on cross-K/V only; profiles/r05s_gemm_epi_ab.txt) — the epilogue's time is
// neither its LDS staging nor its instruction count (scripts/exp/gemm_probe.py)
static int tw_gemm_tr = 0;
extern "C" int tw_gemm_set_epilogue(int tr) {
  TW_REQUIRE(tr == 0 || tr == 1, "tw_gemm_set_epilogue: %d (0 or 1)", tr);
  tw_gemm_tr = tr;
  return 0;
}
// tw_tile_grouped rows per group: 8 for the wide-N shapes (>= 10 column tiles: q/k/v, fc1, cross-K/V; 2-7 % measured),
// row-major for the 5-column-tile ones (o_proj, fc2, conv2), scripts/gemm_bench.py, M = 36000
static inline int tw_group_for(int N) { return (N + 255) / 256 >= 10 ? 8 : 1; }
// packed GEMVs with N >= this (proj_out) read their weights non-temporally: bench step -1 ms (109.2 vs 110.3)
static constexpr int tw_gemv_nt_min_n = 16384;
// K-slices per column group of the vocabulary-wide proj_out (tw_gemv_set_wide_slices): 1 beside an encoder GEMM (its
// MALL residency is what the other decoder weights lose: bench 93.1 vs 92.5 ms with 2 / 4), 4 for a decode pass with the
// GPU to itself (22.7 vs 33 us per launch alone at 24 rows)
static int tw_gemv_wide_kw = 1;
extern "C" int tw_gemv_set_wide_slices(int kw) {
  TW_REQUIRE(kw == 1 || kw == 2 || kw == 4, "tw_gemv_set_wide_slices: kw=%d (1, 2 or 4)", kw);
  tw_gemv_wide_kw = kw;
  return 0;
}
// Largest K-slice count the packed-GEMV heuristic picks: 4 = at most 256-thread workgroups, so one decoder wave per
// SIMD co-resides with an encoder GEMM workgroup (2 waves of ~190 VGPRs on every SIMD), where a 512-thread decoder
// workgroup waits for GEMM workgroups to retire (q/k/v GEMV beside k_gemm_8p: 33.6 us per launch at 8, 11.5 at 4).
static constexpr int tw_gemv_max_kw = 4;
// The decoder layer GEMVs' kernel (tw_gemv_set_variant): 0 = k_gemv_pc (two column groups per wave, batches of 5
// steps), 1 = k_gemv_q (one column group per wave, its whole K-slice in flight) for 17..32 rows; k_gemv_pc at <= 16
// rows and at 64 (config 5's decode passes alone: 198.8-198.9 vs 201.7-202.5 ms per step with k_gemv_q, three
// interleaved pairs, profiles/r05aa_c5_gemv_ab.txt)
static int tw_gemv_kernel = 0;
extern "C" int tw_gemv_set_variant(int v) {
  TW_REQUIRE(v == 0 || v == 1, "tw_gemv_set_variant: v=%d (0 or 1)", v);
  tw_gemv_kernel = v;
  return 0;
}
extern "C" int tw_gemm_set_variant(int v) {
  tw_gemm_kernel = (v & 15) == 5 ? 5 : (v & 15) == 6 ? 6 : 1;
  return 0;
}
// persistent grid of k_gemm_8pp: the device's CUs, a multiple of the 8 XCDs (blocks b, b + 8, ... share one XCD), or
// fewer (tw_gemm_set_persistent_grid: a GEMM queued beside a decode that leaves CUs to the decoder's kernels)
static int tw_pgrid_override = 0;
extern "C" int tw_gemm_set_persistent_grid(int n) {
  TW_REQUIRE(n == 0 || (n >= 8 && n % 8 == 0), "tw_gemm_set_persistent_grid: %d (0 = all CUs, else a multiple of 8)", n);
  tw_pgrid_override = n;
  return 0;
}
static int tw_persistent_grid() {
  static int g = 0;
  if (tw_pgrid_override) return tw_pgrid_override;
  if (!g) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 8)
      cus = 256;
    g = cus / 8 * 8;
  }
  return g;
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

// Ordering between a wave's own epilogue-image writes and reads: every wave stages through its own LDS region, and
// LDS instructions of one wave execute in issue order, so a compiler fence (plus the LDS count) is enough; block
// barriers here only made the 8 waves of a tile wait for each other (and, beside a running decode step, for the
// wave the decoder's waves slow down most).
__device__ inline void gb_epi_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Epilogue of one wave's 128 x 64 sub-tile (rows mw0.., columns ncol0..) held as 8 x 4 16x16 MFMA accumulators,
// through the wave's own [64][GB_EPI_LD] f32 LDS image `wimg` (k_gemm_big; every wave of the
// block calls it: it holds block barriers). The caller's K loop must have ended on a barrier.
// stage(half, wimg) writes rows 64 half .. 64 half + 63 of the wave's sub-tile into its [64][GB_EPI_LD] f32 image
template <int EPI, class Stage>
__device__ inline void gemm_epi_128x64_st(Stage stage, float* wimg, int lane, int mw0, int ncol0, int M, int N,
                                          const EpiArgs& ea, bool interior = false) {
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
  if (!PRE && ea.bias) {
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
      if (interior) {
        // every row and column of the tile in range: straight-line code, so hipcc counts the addend waits instead
        // of draining vmcnt to 0 at each use (which retired every row's stores before the next row's math)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int lr = rr * 4 + (lane >> 4);
          const int m = mrow0 + lr;
          float4 v = *(const float4*)(wimg + lr * GB_EPI_LD + rc);
          v.x += bias4.x; v.y += bias4.y; v.z += bias4.z; v.w += bias4.w;
          epi_store4_pre<EPI>(ea, m, ncol0 + rc, v, ad[rr & 7]);
          if (rr < 8) ad[rr] = epi_addend<EPI>(ea, m + 32, ncol0 + rc, true);
        }
        continue;
      }
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
    } else if constexpr (EPI == TW_EPI_BF16 || EPI == TW_EPI_GELU_BF16 || EPI == TW_EPI_CROSSKV) {
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
                                       int N, const EpiArgs& ea, bool interior = false) {
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
  gemm_epi_128x64_st<EPI>(stage, wimg, lane, mw0, ncol0, M, N, ea, interior);
}
// ------------------------------------------------------------------------------------------------
// Transposed-accumulator epilogue (TR). The K loop runs the MFMA as W . A^T (operands swapped: the fragment reads
// are unchanged), so lane (fr, fq) of accumulator block (i, j) holds sub-tile row 16 i + fr, columns 16 j + 4 fq ..
// + 3 — four consecutive output columns in registers. The fused bias (+ GELU) then applies before any staging, bf16
// outputs pack to 8-byte bf16x4 units, and f32 outputs leave straight from registers:
//   bf16 (BF16 / GELU_BF16 / CROSSKV): units staged in the wave's own [128][64] bf16 LDS image (16 KiB; unit
//     index XOR row & 15: conflict-free ds_write_b64 and ds_read_b128, scripts/exp/tr_swizzle_check.py), read
//     back as 8 consecutive columns per lane (one 16-byte store, 8 lanes per 128-byte row): per wave 32 ds_write_b64
//     + 16 ds_read_b128 instead of 128 ds_write_b32 + 16 ds_read_b128 of the f32 image, and half the LDS bytes.
//   f32 (RESID / GELU_POS / F32): 16-byte accesses of 4 columns, 4 lanes per 64-byte row run; the residual / table
//     operand of block row i + 1 is loaded while block row i is stored.
// The tile's bias sits in LDS (bias_s, tile-local columns, staged with the first K-tile).
// acc(i, j): the accumulator of block (i, j) of the wave's 128 x 64 sub-tile; rowmap(lr) its global row for sub-tile
// row lr (0..127); tcol(lc) the tile-local column of sub-tile column lc (0..63; runs of 8 stay contiguous).
// ------------------------------------------------------------------------------------------------
template <int EPI, class Acc, class RowMap, class TCol>
__device__ inline void gemm_epi_tr(Acc acc, bf16_t* img, const float* bias_s, int lane, RowMap rowmap, TCol tcol, int n0,
                                   int M, int N, const EpiArgs& ea) {
  const int fr = lane & 15, fq = lane >> 4;
  float4 b4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    b4[j] = ea.bias ? *(const float4*)(bias_s + tcol(16 * j + 4 * fq)) : make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (EPI == TW_EPI_BF16 || EPI == TW_EPI_GELU_BF16 || EPI == TW_EPI_CROSSKV) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = 16 * i + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 a = acc(i, j);
        float4 v = make_float4(a[0] + b4[j].x, a[1] + b4[j].y, a[2] + b4[j].z, a[3] + b4[j].w);
        if constexpr (EPI == TW_EPI_GELU_BF16) v = gelu_erf4(v);
        uint2 w;
        w.x = pack_bf16x2(v.x, v.y);
        w.y = pack_bf16x2(v.z, v.w);
        *(uint2*)(img + row * 64 + (((4 * j + fq) ^ (row & 15)) << 2)) = w;
      }
    }
    gb_epi_sync();
#pragma unroll 4
    for (int rr = 0; rr < 16; ++rr) {
      const int row = rr * 8 + (lane >> 3), p = lane & 7, g = row & 15;
      uint4 d = *(const uint4*)(img + row * 64 + ((p ^ (g >> 1)) << 3));
      if (g & 1) d = make_uint4(d.z, d.w, d.x, d.y);  // (the XOR swapped the two 8-byte units)
      const int m = rowmap(row), n = n0 + tcol(8 * p);
      if (m >= M || n >= N) continue;
      if (n + 7 < N) {
        size_t idx;
        if constexpr (EPI == TW_EPI_CROSSKV) {  // 8 | 64: the group stays inside one head's 64 contiguous dims
          const int D = ea.kv_D, S = ea.kv_S;
          const int l = n / (2 * D), rem = n - l * 2 * D;
          const int kv = rem / D, hd = rem - kv * D;
          const int b = m / S, s2 = m - b * S;
          idx = ((((size_t)(l * 2 + kv) * ea.kv_B + b) * ea.kv_H + (hd >> 6)) * S + s2) * 64 + (hd & 63);
        } else {
          idx = (size_t)m * ea.ldo + n;
        }
        tw_st_enc<gb_nt_bit(EPI)>((bf16_t*)ea.out + idx, d);
      } else {  // ragged right edge (tests only)
        const uint32_t u[4] = {d.x, d.y, d.z, d.w};
        EpiArgs e2 = ea;
        e2.bias = nullptr;
        for (int e = 0; e < 8 && n + e < N; ++e) {
          const bf16_t h = (bf16_t)((u[e >> 1] >> (16 * (e & 1))) & 0xffffu);
          if constexpr (EPI == TW_EPI_CROSSKV) {
            epi_store<EPI>(e2, m, n + e, bf16_to_f32(h));
          } else {
            ((bf16_t*)ea.out)[(size_t)m * ea.ldo + n + e] = h;
          }
        }
      }
    }
  } else {
    constexpr bool PRE = EPI == TW_EPI_RESID_F32 || EPI == TW_EPI_GELU_POS_F32;
    float4 ad[2][4];
    auto load_ad = [&](int i, float4 (&dst)[4]) {
      const int m = min(rowmap(16 * i + fr), M - 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + tcol(16 * j + 4 * fq);
        dst[j] = epi_addend<EPI>(ea, m, n, n + 3 < N);
      }
    };
    if constexpr (PRE) load_ad(0, ad[0]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (PRE) {
        if (i + 1 < 8) load_ad(i + 1, ad[(i + 1) & 1]);
      }
      const int m = rowmap(16 * i + fr);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 a = acc(i, j);
        const float4 v = make_float4(a[0] + b4[j].x, a[1] + b4[j].y, a[2] + b4[j].z, a[3] + b4[j].w);
        const int n = n0 + tcol(16 * j + 4 * fq);
        if (m >= M || n >= N) continue;
        if (n + 3 < N) {
          if constexpr (PRE) epi_store4_pre<EPI>(ea, m, n, v, ad[i & 1][j]);
          else epi_store4<EPI>(ea, m, n, N, v);
        } else {
          epi_store4<EPI>(ea, m, n, N, v);
        }
      }
    }
  }
}

// The tile's bias into LDS (tile-local columns 0..255, clamped at N - 1): wave 0 issues the loads beside the first
// K-tile's DMA, writes them after that wait, and the barrier that publishes the K-tile publishes them too.
__device__ inline void gemm_bias_load(const EpiArgs& ea, int n0, int N, float4& b) {
  const int c = n0 + 4 * (threadIdx.x & 63);
  if (ea.bias)
    b = make_float4(ea.bias[min(c, N - 1)], ea.bias[min(c + 1, N - 1)], ea.bias[min(c + 2, N - 1)],
                    ea.bias[min(c + 3, N - 1)]);
}

template <int EPI, bool TR>
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
      __builtin_amdgcn_global_load_lds((const void*)(ga[i] + k0), (lds_void_t*)(As + rb), 16, 0, 0);
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
  // (TR: the tile's bias in the LDS spare beyond the K loop's 128 KiB, staged with the first K-tile)
  float* bias_s = (float*)(smem + 4 * GB_BM * GB_BK);
  float4 bl = make_float4(0.f, 0.f, 0.f, 0.f);
  stage(0, 0);
  if (TR && wid == 0) gemm_bias_load(ea, n0, N, bl);
  if (TR && wid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *(float4*)(bias_s + 4 * lane) = bl;
  }
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
        for (int j = 0; j < 4; ++j) {
          if constexpr (TR) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af, acc[i][j], 0, 0, 0);
          else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // vmcnt(0) (tile kt+1 landed) + lgkmcnt(0) + barrier
  }

  if constexpr (TR) {
    gemm_epi_tr<EPI>([&](int i, int j) { return acc[i][j]; }, smem + wid * (128 * 64), bias_s, lane,
                     [&](int lr) { return m0 + wr * 128 + lr; }, [&](int lc) { return wc * 64 + lc; }, n0, M, N, ea);
  } else {
    gemm_epi_128x64<EPI>(acc, (float*)smem + wid * (64 * GB_EPI_LD), lane, m0 + wr * 128, n0 + wc * 64, M, N, ea,
                         m0 + GB_BM <= M && n0 + GB_BN <= N);
  }
}

// Buffer descriptor from values the compiler can prove wave-uniform (readfirstlane'd base halves and size): the
// descriptor then lives in SGPRs and every buffer op through it is one instruction, not a waterfall loop.
__device__ inline __amdgpu_buffer_rsrc_t tw_uniform_rsrc(const void* p, int bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
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
#ifdef TW_GEMM_PROBE
// Measurement build only (make probe -> scripts/exp/libtwhip_probe.so, scripts/exp/gemm_probe.py; never shipped):
// per-workgroup timestamps of the large-M kernels' phases. Slots: 0 start, 1 first K-tile landed, 2 K loop done,
// 3 epilogue stores retired (100 MHz s_memrealtime); 4, 5 core-clock s_memtime at start / K loop done; 6 HW_ID, 7 XCC_ID;
// 8.. epilogue sub-phases of wave 0 (TW_PROBE_W: a vmcnt(0) first, so each names the data it waited for).
#define TW_PROBE_SLOTS 16
__device__ unsigned long long tw_probe_ts[32768 * TW_PROBE_SLOTS];
#define TW_PROBE(slot)                                                                                     \
  do {                                                                                                     \
    if (threadIdx.x == 0) tw_probe_ts[blockIdx.x * TW_PROBE_SLOTS + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define TW_PROBE_CLK(slot)                                                                                 \
  do {                                                                                                     \
    if (threadIdx.x == 0) tw_probe_ts[blockIdx.x * TW_PROBE_SLOTS + (slot)] = __builtin_amdgcn_s_memtime();  \
  } while (0)
__device__ inline void tw_probe_ids() {
  if (threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    tw_probe_ts[blockIdx.x * TW_PROBE_SLOTS + 6] = hw;
    tw_probe_ts[blockIdx.x * TW_PROBE_SLOTS + 7] = xcc;
  }
}
extern "C" int tw_gemm_probe_read(unsigned long long* host, int nwg) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(tw_probe_ts), (size_t)nwg * TW_PROBE_SLOTS * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#define TW_PROBE_W(slot)                              \
  do {                                                \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
    TW_PROBE(slot);                                   \
  } while (0)
#define TW_PROBE_END()                                \
  do {                                                \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
    __syncthreads();                                  \
    TW_PROBE(3);                                      \
  } while (0)
#else
#define TW_PROBE(slot) do {} while (0)
#define TW_PROBE_CLK(slot) do {} while (0)
#define TW_PROBE_END() do {} while (0)
#define TW_PROBE_W(slot) do {} while (0)
__device__ inline void tw_probe_ids() {}
#endif

template <int N>
__device__ inline void p8_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

template <int EPI, bool TR>
__global__ __launch_bounds__(512, 1) void k_gemm_8p(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  // K loop: 2 buffers x 4 half-tiles x 16 KiB = 128 KiB; epilogue: 8 x [64][68] f32 = 136 KiB (one array: a
  // second __shared__ object makes hipcc drain vmcnt before every ds_read)
  __shared__ __attribute__((aligned(16))) bf16_t smem[8 * 64 * GB_EPI_LD * 2];
  constexpr int HT = 128 * GB_BK;
  TW_PROBE(0);
  TW_PROBE_CLK(4);
  tw_probe_ids();
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
    // (the last row's K elements: an operand whose rows overlap, ld < K, tw_conv2_gemm's implicit im2col)
    rs[h] = tw_uniform_rsrc((h < 2 ? A : W) + (size_t)r0 * ld, rows ? ((rows - 1) * ld + K) * 2 : 0);
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
          acc[mh][nh][i][j] = TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], af[i][kk], acc[mh][nh][i][j], 0, 0, 0)
                                 : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bfr[j][kk], acc[mh][nh][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  const int nk = K / GB_BK;
  // (TR: the tile's bias in the LDS spare beyond the K loop's 128 KiB, loaded beside the first K-tile's DMA)
  float* bias_s = (float*)(smem + 8 * HT);
  float4 bl = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, 0);
  if (TR && wid == 0) gemm_bias_load(ea, n0, N, bl);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (TR && wid == 0) *(float4*)(bias_s + 4 * lane) = bl;
  if (TR) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  TW_PROBE(1);
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
  TW_PROBE(2);
  TW_PROBE_CLK(5);
  if constexpr (TR) {
    TW_PROBE_W(8);
    gemm_epi_tr<EPI>([&](int i, int j) { return acc[i >> 2][j >> 1][i & 3][j & 1]; }, smem + wid * (128 * 64), bias_s,
                     lane, [&](int lr) { return m0 + 128 * (lr >> 6) + 64 * wr + (lr & 63); },
                     [&](int lc) { return 128 * (lc >> 5) + 32 * wc + (lc & 31); }, n0, M, N, ea);
    TW_PROBE_END();
    return;
  }

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
  TW_PROBE_W(8);
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
    TW_PROBE_W(9 + 2 * mh);
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
    TW_PROBE_W(10 + 2 * mh);
  }
  TW_PROBE_END();
}

// ------------------------------------------------------------------------------------------------
// k_gemm_8pp: k_gemm_8p made persistent — one workgroup per CU walks tiles slot, slot + S, ... of its XCD's contiguous
// range (the same XCD split and grouped order as k_gemm_8p's remap). The epilogue of a 256 x 256 tile costs ~7 us of a
// ~40-us tile with no MFMA beside it (scripts/exp/gemm_probe.py, profiles/r05t_*): bias loads 0.8, LDS staging 0.6,
// store issue and write-ack ~2.6 per half, with a fresh workgroup's first K-tile DMA (1.5) after it. Here, per tile:
//   * the NEXT tile's first K-tile (and its bias) is DMA'd into buffer 0 before this tile's epilogue stores issue;
//   * the epilogue stages through buffer 1 + the spare, in 32-row quarters (8 x [32][68] f32 = 68 KiB);
//   * an interior bf16 tile (16 stores per wave) then waits vmcnt(16) only: vector memory operations retire in issue
//     order, so the DMA ahead of the stores has landed while the stores may still drain — into the next tile's first
//     K-tile, whose phases 1-3 need no wait (its four halves are in) and whose phase 4 waits for K-tile 1.
// LDS: [0, 64K) buffer 0 | [64K, 128K) buffer 1 | staging [64K, 132K) between K loops | bias slots 2 x 1 KiB at 132K.
// ------------------------------------------------------------------------------------------------
// The read-back of 4 rows x 8 columns of an epilogue image as one asm block (8 ds_read_b128, then lgkmcnt(0)): while
// the next tile's LDS DMA is in flight, hipcc would otherwise put a vmcnt(0) before every ds_read of the same
// __shared__ array (it cannot tell the image from the DMA's buffer), draining the epilogue's own stores each time.
__device__ inline void gb_read_rows4(const float* img, float4 (&v)[4][2]) {
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)img;
  asm volatile(
      "ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:16\n\t"
      "ds_read_b128 %2, %8 offset:%9\n\tds_read_b128 %3, %8 offset:%10\n\t"
      "ds_read_b128 %4, %8 offset:%11\n\tds_read_b128 %5, %8 offset:%12\n\t"
      "ds_read_b128 %6, %8 offset:%13\n\tds_read_b128 %7, %8 offset:%14\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=v"(v[0][0]), "=v"(v[0][1]), "=v"(v[1][0]), "=v"(v[1][1]), "=v"(v[2][0]), "=v"(v[2][1]), "=v"(v[3][0]),
        "=v"(v[3][1])
      : "v"(a), "i"(8 * GB_EPI_LD * 4), "i"(8 * GB_EPI_LD * 4 + 16), "i"(16 * GB_EPI_LD * 4),
        "i"(16 * GB_EPI_LD * 4 + 16), "i"(24 * GB_EPI_LD * 4), "i"(24 * GB_EPI_LD * 4 + 16)
      : "memory");
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm_8pp(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                     int M, int N, int K, int lda, int ldw, EpiArgs ea) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[8 * 64 * GB_EPI_LD * 2];
  constexpr int HT = 128 * GB_BK;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (M + GB_BM - 1) / GB_BM, ntn = (N + GB_BN - 1) / GB_BN;
  const int nwg = ntm * ntn;
  const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8, S = gridDim.x / 8;
  const int q8 = nwg / 8, r8 = nwg % 8;
  const int cnt = q8 + (xcd < r8 ? 1 : 0);
  const int base = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  if (slot >= cnt) return;  // (workgroup-uniform, before any barrier)
  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  float* const bias_sl = (float*)(smem + 4 * HT) + 8 * 32 * GB_EPI_LD;  // 2 x 256 f32

  __amdgpu_buffer_rsrc_t rs[4];
  auto set_tile = [&](int tile, int& m0, int& n0) {
    int tm, tn;
    tw_tile_grouped(tile, ntm, ntn, ea.group_m, tm, tn);
    m0 = tm * GB_BM;
    n0 = tn * GB_BN;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int r0 = (h < 2 ? m0 : n0) + 128 * (h & 1), lim = h < 2 ? M : N, ld = h < 2 ? lda : ldw;
      const int rows = max(0, min(128, lim - r0));
      rs[h] = tw_uniform_rsrc((h < 2 ? A : W) + (size_t)r0 * ld, rows ? ((rows - 1) * ld + K) * 2 : 0);
    }
  };
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
  // the tile's 256 bias values (columns clamped into [0, N - 4]; host: N % 4 == 0, bias 16-byte aligned) by wave 0
  auto stage_bias = [&](int sl, int n0) {
    if (ea.bias && wid == 0)
      __builtin_amdgcn_global_load_lds((const void*)(ea.bias + min(n0 + 4 * lane, N - 4)),
                                       (lds_void_t*)(bias_sl + 256 * sl), 16, 0, 0);
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
  // one K-tile = 4 phases (k_gemm_8p's); NXT: stage K-tile t+1; FIRST: K-tile 0, all four halves already waited for
  // (no phase 1 / 2 waits: they would also drain the previous tile's epilogue stores)
  auto ktile = [&](int t, auto NXT, auto FIRST) {
    constexpr bool nxt = decltype(NXT)::value, first = decltype(FIRST)::value;
    const int buf = t & 1, nb = buf ^ 1, kn = (t + 1) * GB_BK;
    readB(buf, 0);
    __builtin_amdgcn_sched_barrier(0);
    readA(buf, 0);
    if constexpr (nxt) {
      stage(nb, 0, kn);
      if constexpr (!first) p8_vmcnt<4>();
    } else if constexpr (!first) {
      p8_vmcnt<2>();
    }
    mfma_q(I0{}, I0{});
    readB(buf, 1);
    if constexpr (nxt) {
      stage(nb, 2, kn);
      if constexpr (!first) p8_vmcnt<4>();
    } else if constexpr (!first) {
      p8_vmcnt<0>();
    }
    mfma_q(I0{}, I1{});
    readA(buf, 1);
    if constexpr (nxt) stage(nb, 3, kn);
    mfma_q(I1{}, I1{});
    readB(buf, 0);
    if constexpr (nxt) {
      stage(nb, 1, kn);
      p8_vmcnt<4>();  // A0, B0 of K-tile t+1 (and, for K-tile 0, the previous tile's stores ahead of them)
    }
    mfma_q(I1{}, I0{});
  };
  using BT = std::integral_constant<bool, true>;
  using BF = std::integral_constant<bool, false>;

  constexpr bool PRE = EPI == TW_EPI_RESID_F32 || EPI == TW_EPI_GELU_POS_F32;
  constexpr bool BF16OUT = EPI == TW_EPI_BF16 || EPI == TW_EPI_GELU_BF16 || EPI == TW_EPI_CROSSKV;
  // epilogue through LDS in 32-row quarters (mh, ih) of the wave's 128 x 64 piece, 8 consecutive columns per lane in
  // the read-back (8 lanes per row) for 16-byte global stores; bias from the tile's LDS slot
  auto epilogue = [&](int m0, int n0, const float* bias_s) {
    const int rc = (lane & 7) * 8;
    const int lcol = rc < 32 ? 32 * wc + rc : 128 + 32 * wc + rc - 32;
    const int ncol = n0 + lcol;
    float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
    if (ea.bias) {
      b0 = *(const float4*)(bias_s + lcol);
      b1 = *(const float4*)(bias_s + lcol + 4);
    }
    float* wimg = (float*)(smem + 4 * HT) + wid * (32 * GB_EPI_LD);
    const bool full = ncol + 7 < N;
    auto stage_q = [&](int q, float4 (&vv)[4][2]) {  // quarter q of the wave's piece -> rows (lane >> 3) + 8 rr
      const int mh = q >> 1, ih = q & 1;
      if (q) gb_epi_sync();
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              wimg[(ii * 16 + fq * 4 + r) * GB_EPI_LD + nh * 32 + j * 16 + fr] = acc[mh][nh][2 * ih + ii][j][r];
      gb_epi_sync();
      gb_read_rows4(wimg + (lane >> 3) * GB_EPI_LD + rc, vv);
    };
    if constexpr (PRE) {
      if (m0 + GB_BM <= M && n0 + GB_BN <= N) {
        // interior tile: straight-line code (no lane conditions), so hipcc counts its waits instead of draining vmcnt
        // to 0 before every addend use — which made each row group's stores retire before the next group's math
        // (one drain per quarter remains: the quarter's addend loads are issued after the previous quarter's stores)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int mr = m0 + 128 * (q >> 1) + 64 * wr + 32 * (q & 1) + (lane >> 3);
          float4 ad[4][2];
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            ad[rr][0] = epi_addend<EPI>(ea, mr + rr * 8, ncol, true);
            ad[rr][1] = epi_addend<EPI>(ea, mr + rr * 8, ncol + 4, true);
          }
          float4 vv[4][2];
          stage_q(q, vv);
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            float4 v0 = vv[rr][0], v1 = vv[rr][1];
            v0.x += b0.x; v0.y += b0.y; v0.z += b0.z; v0.w += b0.w;
            v1.x += b1.x; v1.y += b1.y; v1.z += b1.z; v1.w += b1.w;
            epi_store4_pre<EPI>(ea, mr + rr * 8, ncol, v0, ad[rr][0]);
            epi_store4_pre<EPI>(ea, mr + rr * 8, ncol + 4, v1, ad[rr][1]);
          }
        }
        return;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mh = q >> 1, ih = q & 1;
      const int mrow0 = m0 + 128 * mh + 64 * wr + 32 * ih;
      float4 ad[4][2];
      if constexpr (PRE) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int mq = min(mrow0 + rr * 8 + (lane >> 3), M - 1);
          ad[rr][0] = epi_addend<EPI>(ea, mq, ncol, full);
          ad[rr][1] = epi_addend<EPI>(ea, mq, ncol + 4, full);
        }
      }
      float4 vv[4][2];  // rows rr * 8 + (lane >> 3), rr = 0..3 (8 rows = 8 * GB_EPI_LD floats apart)
      stage_q(q, vv);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int lr = rr * 8 + (lane >> 3);
        const int m = mrow0 + lr;
        float4 v0 = vv[rr][0], v1 = vv[rr][1];
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
  };

  const int nk = K / GB_BK;
  int local = slot, m0, n0;
  set_tile(base + local, m0, n0);
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, 0);
  stage_bias(0, n0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // ping-pong: group 1 one barrier behind
  for (int it = 0;; ++it) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (nk == 1) {
      ktile(0, BF{}, BT{});
    } else {
      ktile(0, BT{}, BT{});
      for (int t = 1; t + 1 < nk; ++t) ktile(t, BT{}, BF{});
      ktile(nk - 1, BF{}, BF{});
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // realign the groups
    __syncthreads();
    const int nlocal = local + S;
    const bool has_next = nlocal < cnt;
    const int cm0 = m0, cn0 = n0;
    if (has_next) {  // the next tile's first K-tile + bias, ahead of this tile's stores
      set_tile(base + nlocal, m0, n0);
#pragma unroll
      for (int h = 0; h < 4; ++h) stage(0, h, 0);
      stage_bias((it + 1) & 1, n0);
    }
    epilogue(cm0, cn0, bias_sl + 256 * (it & 1));
    if (!has_next) break;
    if (BF16OUT && cm0 + GB_BM <= M && cn0 + GB_BN <= N)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // exactly 16 stores per wave follow the DMA
    else if (PRE && cm0 + GB_BM <= M && cn0 + GB_BN <= N)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // the last quarter's 8 stores end the interior epilogue
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();
    local = nlocal;
  }
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
  if (nw == 4) launch_skinny_nw<EPI, 4>(A, W, M, N, K, lda, ldw, ea, splits, s);
  else if (nw == 8) launch_skinny_nw<EPI, 8>(A, W, M, N, K, lda, ldw, ea, splits, s);
  else launch_skinny_nw<EPI, 16>(A, W, M, N, K, lda, ldw, ea, splits, s);
}

// ------------------------------------------------------------------------------------------------
// Packed decoder GEMV (M <= 64): weights pre-arranged in MFMA fragment order (tw_pack_weight), activations either
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


// NTW: weight fragments read with non-temporal loads (proj_out: 133 MB streamed once per step, kept out of the
// caches so that the layer weights can stay in them).
// MT: 16-row m-tiles of the activation (1: M <= 16, 2: M <= 32, 4: M <= 64). Packed activations hold rows 32..63 as a
// second 32-row block 32 K elements on (tw_pack_act_idx), so m-tile t of step s sits at
// (t / 2) * 32 K + s * 1024 + (t % 2) * 512; row-major activations read rows 16 t + lane % 16.
template <int MT, bool APACK>
__device__ inline const bf16_t* gemv_a_base(const bf16_t* A, int lda, int M, int K, int t, int lane) {
  if constexpr (APACK) return A + (size_t)(t >> 1) * 32 * K + (t & 1) * 512 + lane * 8;
  else return A + (size_t)min(16 * t + (lane & 15), M - 1) * lda + 8 * (lane >> 4);
}
template <bool APACK>
__device__ inline bf16x8 gemv_a_load(const bf16_t* ap, int st) {
  return APACK ? *(const bf16x8*)(ap + (size_t)st * 1024) : *(const bf16x8*)(ap + 32 * st);
}

// (NTW, the vocabulary-wide proj_out: at most 128 registers, like every other kernel of the decoder step, so that
// its waves fit beside an encoder GEMM workgroup's two waves on a SIMD; uncapped it took 134 at MT = 2)
template <int EPI, int KW, int U, bool APACK, int MT, bool NTW = false>
__global__ TW_DEC_LB(KW > 4 ? 512 : 256, NTW ? 4 : 1) void k_gemv_p(const bf16_t* __restrict__ A, int lda,
                                                               const bf16_t* __restrict__ Wp, int M, int N, int K,
                                                               EpiArgs ea) {
  TW_DEC_PRIO();
  constexpr int NW = KW > 4 ? KW : 4, GPB = NW / KW;
  // (KW = 1: no cross-wave sum, no LDS — see the epilogue)
  __shared__ float red[KW > 1 ? NW : 1][KW > 1 ? MT * 16 : 1][17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int gl = wid / KW, kw = wid - gl * KW;
  const int g = blockIdx.x * GPB + gl;
  const int ngroups = (N + 15) >> 4, ns = K >> 5;
  const int nsl = KW * gridDim.y, sl = blockIdx.y * KW + kw;
  const int s0 = (int)((long)sl * ns / nsl), s1 = (int)((long)(sl + 1) * ns / nsl);
  f32x4 c[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) c[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (g < ngroups) {
    const bf16_t* wp = Wp + (size_t)g * ns * 512 + lane * 8;
    const bf16_t* ap[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) ap[t] = gemv_a_base<MT, APACK>(A, lda, M, K, t, lane);
    auto ldW = [&](int st) -> bf16x8 {
      if constexpr (NTW) {
        typedef short s16x8_nt __attribute__((ext_vector_type(8)));
        const s16x8_nt v = __builtin_nontemporal_load((const s16x8_nt*)(wp + (size_t)st * 512));
        return __builtin_bit_cast(bf16x8, v);
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
      bf16x8 bw[NB], a[NB][MT];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int st = min(st0 + u, s1 - 1);
        bw[u] = ldW(st);
#pragma unroll
        for (int t = 0; t < MT; ++t) a[u][t] = gemv_a_load<APACK>(ap[t], st);
      }
      // (not on the bandwidth-bound vocabulary-wide proj_out, NTW: its 3242 waves hide the latency, and 48 live
      // fragments cost it occupancy: 26.2 -> 30.8 us per launch alone)
      if constexpr (!NTW) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        if (u < n) {
#pragma unroll
          for (int t = 0; t < MT; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][t], bw[u], c[t], 0, 0, 0);
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
      ((bf16_t*)ea.out)[tw_pack_act_idx(m, n, N)] = f32_to_bf16(gelu_erf(v));
    } else {
      epi_store<EPI>(ea, m, n, v);
    }
  };
  if constexpr (KW == 1) {
    // one wave per column group: its accumulators are the results. Stored straight from registers (16 lanes per
    // row = 16 consecutive columns), so the kernel holds no LDS: the vocabulary-wide proj_out's 811 workgroups then
    // co-reside with an encoder GEMM workgroup (136 KiB of the CU's 160 KiB LDS) several per CU, in one round.
    const int n = g * 16 + cc;
    if (g < ngroups && n < N) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * t + rb + r < M) store(16 * t + rb + r, n, c[t][r]);
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wid][16 * t + rb + r][cc] = c[t][r];
  __syncthreads();
  constexpr int ROWS = MT * 16;
  for (int e = tid; e < GPB * ROWS * 16; e += NW * 64) {
    const int gg = e / (ROWS * 16), rem = e - gg * ROWS * 16;
    const int m = rem >> 4, cl = rem & 15;
    const int n = (blockIdx.x * GPB + gg) * 16 + cl;
    if (m < M && n < N) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < KW; ++w) v += red[gg * KW + w][m][cl];
      store(m, n, v);
    }
  }
}

// k_gemv_pc: k_gemv_p with TWO column groups per wave (32 output columns) sharing each A fragment. At M = 17..32 rows
// a step of k_gemv_p loads one W fragment and two A fragments (the activations, L2-resident and identical for every
// column group); here a step loads two W fragments and the same two A fragments: a third fewer vector-memory
// instructions and VGPRs per weight byte. Every decoder-step kernel shares its CU with an encoder GEMM workgroup
// (run_batches' overlap), whose LDS-DMA keeps the same vector-memory path busy. KW >= 2 K-slices
// per column-group pair, reduced through LDS; epilogues BF16, PARTIAL (split-K) and GELU_PACKED. MT = 4 (M = 33..64:
// beam rows, config 5's 64 windows) streams every weight byte once for all 64 rows; its cross-wave sum runs in two
// 32-row passes over the same 17 KiB of LDS as MT = 2.
template <int EPI, int KW, int U, bool APACK, int MT, bool NTW = false>
__global__ TW_DEC_LB(256, 1) void k_gemv_pc(const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ Wp,
                                            int M, int N, int K, EpiArgs ea) {
  TW_DEC_PRIO();
  static_assert(KW == 1 || KW == 2 || KW == 4, "k_gemv_pc: 1, 2 or 4 K-slices");
  constexpr int NW = 4, GPB = NW / KW;  // pairs per workgroup
  constexpr int RT = MT > 2 ? 2 : MT;   // m-tiles per LDS reduction pass
  __shared__ float red[KW > 1 ? NW : 1][2][KW > 1 ? RT * 16 : 1][17];  // (KW = 1: stored from registers, no LDS)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int gl = wid / KW, kw = wid - gl * KW;
  const int g0 = (blockIdx.x * GPB + gl) * 2;  // this wave's column groups g0, g0 + 1
  const int ngroups = (N + 15) >> 4, ns = K >> 5;
  const int nsl = KW * gridDim.y, sl = blockIdx.y * KW + kw;
  const int s0 = (int)((long)sl * ns / nsl), s1 = (int)((long)(sl + 1) * ns / nsl);
  f32x4 c[2][MT];  // [group][m-tile]
#pragma unroll
  for (int t = 0; t < MT; ++t) c[0][t] = c[1][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (g0 < ngroups) {
    const bool has1 = g0 + 1 < ngroups;
    const bf16_t* wp0 = Wp + (size_t)g0 * ns * 512 + lane * 8;
    const bf16_t* wp1 = has1 ? wp0 + (size_t)ns * 512 : wp0;  // (an odd last group: its twin re-reads group g0)
    const bf16_t* ap[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) ap[t] = gemv_a_base<MT, APACK>(A, lda, M, K, t, lane);
    // one batch of NB steps, every load issued before the first MFMA (see k_gemv_p)
    // MT = 4 runs the batch in two halves of two m-tiles over the same weight registers: the second half's
    // activation fragments (L2-resident) load after the first half's MFMAs into the same VGPRs, so a batch keeps
    // U = 5 steps of weights in flight within the 128-VGPR budget (four m-tiles at once allowed only U = 3: twice the
    // HBM round trips per weight byte)
    constexpr int TH = MT > 2 ? 2 : MT;
    auto batch = [&](auto NBc, int st0, int n) {
      constexpr int NB = decltype(NBc)::value;
      bf16x8 b0[NB], b1[NB], a[NB][TH];
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
#pragma unroll
        for (int t = 0; t < TH; ++t) a[u][t] = gemv_a_load<APACK>(ap[t], st);
      }
#pragma unroll
      for (int h = 0; h < MT / TH; ++h) {
        if (h) {
#pragma unroll
          for (int u = 0; u < NB; ++u) {
            const int st = min(st0 + u, s1 - 1);
#pragma unroll
            for (int t = 0; t < TH; ++t) a[u][t] = gemv_a_load<APACK>(ap[h * TH + t], st);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          if (u < n) {
#pragma unroll
            for (int t = 0; t < TH; ++t) {
              c[0][h * TH + t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][t], b0[u], c[0][h * TH + t], 0, 0, 0);
              c[1][h * TH + t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][t], b1[u], c[1][h * TH + t], 0, 0, 0);
            }
          }
        }
        // (between the halves only: at MT <= 2 a barrier here makes hipcc keep 8 more registers live into the next
        // batch, 134 instead of 128, and the step beside an encoder GEMM slower, profiles/r04q_*)
        if constexpr (MT > TH) __builtin_amdgcn_sched_barrier(0);
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
  auto store = [&](int m, int n, float v) {
    if constexpr (EPI == TW_EPI_PARTIAL) {
      ((float*)ea.out)[((size_t)blockIdx.y * M + m) * ea.ldo + n] = v;
    } else if constexpr (EPI == TW_EPI_GELU_PACKED) {
      if (ea.bias) v += ea.bias[n];
      ((bf16_t*)ea.out)[tw_pack_act_idx(m, n, N)] = f32_to_bf16(gelu_erf(v));
    } else {
      epi_store<EPI>(ea, m, n, v);
    }
  };
  if constexpr (KW == 1) {  // the accumulators are the results: 16 lanes per row store 16 consecutive columns
    const int n0 = g0 * 16 + cc, n1 = n0 + 16;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * t + rb + r;
        if (m < M && n0 < N) store(m, n0, c[0][t][r]);
        if (m < M && n1 < N) store(m, n1, c[1][t][r]);
      }
    return;
  }
  constexpr int ROWS = RT * 16;
#pragma unroll
  for (int pass = 0; pass < MT / RT; ++pass) {
    if (pass) __syncthreads();  // (the previous pass's reads of red are done)
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[wid][0][16 * t + rb + r][cc] = c[0][pass * RT + t][r];
        red[wid][1][16 * t + rb + r][cc] = c[1][pass * RT + t][r];
      }
    __syncthreads();
    for (int e = tid; e < GPB * 2 * ROWS * 16; e += NW * 64) {
      const int pg = e / (2 * ROWS * 16), rem = e - pg * 2 * ROWS * 16;  // pair in the block, then group, row, column
      const int h = rem / (ROWS * 16), r2 = rem - h * ROWS * 16;
      const int m = pass * ROWS + (r2 >> 4), cl = r2 & 15;
      const int n = ((blockIdx.x * GPB + pg) * 2 + h) * 16 + cl;
      if (m < M && n < N) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < KW; ++w) v += red[pg * KW + w][h][r2 >> 4][cl];
        store(m, n, v);
      }
    }
  }
}

template <int EPI, int KW, bool APACK, int U = 5, bool NTW = false>
static void launch_gemv_pc(const bf16_t* A, int lda, const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea,
                           int splits, hipStream_t s) {
  constexpr int GPB = 4 / KW;
  dim3 grid(tw_cdiv(tw_cdiv(tw_cdiv(N, 16), 2), GPB), splits);
  if (M > 32)  // (four m-tiles per step, run as two halves: see k_gemv_pc)
    hipLaunchKernelGGL((k_gemv_pc<EPI, KW, U, APACK, 4, NTW>), grid, dim3(256), 0, s, A, lda, Wp, M, N, K, ea);
  else if (M > 16)
    hipLaunchKernelGGL((k_gemv_pc<EPI, KW, U, APACK, 2, NTW>), grid, dim3(256), 0, s, A, lda, Wp, M, N, K, ea);
  else
    hipLaunchKernelGGL((k_gemv_pc<EPI, KW, U, APACK, 1, NTW>), grid, dim3(256), 0, s, A, lda, Wp, M, N, K, ea);
}

// k_gemv_q: ONE column group per wave and every weight fragment of the wave's K-slice in flight at once (n <= U
// steps, one HBM round trip per wave), spread over >= 256 workgroups where the shape allows; the activation fragments
// (L2-resident, shared by every column group) stream two steps behind through a double buffer, so they cost no
// long-lived registers. k_gemv_pc's waves instead hold two column groups and run their K-slice in batches of 5 steps
// (two dependent HBM round trips per wave for the 40-step slices of q/k/v, cross-q, fc1, fc2) on 40-160 workgroups.
// Block = 4 waves = GPB column groups x KW K-slices (reduced through LDS); gridDim.y = split-K slices over blocks
// (PARTIAL only). n = this wave's step count, wave-uniform (the guards are scalar branches, not clamped re-loads).
template <int EPI, int KW, int U, bool APACK, int MT>
__global__ TW_DEC_LB(256, 1) void k_gemv_q(const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ Wp,
                                           int M, int N, int K, EpiArgs ea) {
  TW_DEC_PRIO();
  static_assert(KW == 1 || KW == 2 || KW == 4, "k_gemv_q: 1, 2 or 4 K-slices");
  constexpr int NW = 4, GPB = NW / KW;
  __shared__ float red[KW > 1 ? NW : 1][KW > 1 ? MT * 16 : 1][17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int gl = wid / KW, kw = wid - gl * KW;
  const int g = blockIdx.x * GPB + gl;
  const int ngroups = (N + 15) >> 4, ns = K >> 5;
  const int nsl = KW * gridDim.y, sl = blockIdx.y * KW + kw;
  const int s0 = (int)((long)sl * ns / nsl), s1 = (int)((long)(sl + 1) * ns / nsl);
  const int n = s1 - s0;
  f32x4 c[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) c[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (g < ngroups) {
    const bf16_t* wp = Wp + ((size_t)g * ns + s0) * 512 + lane * 8;
    const bf16_t* ap[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) ap[t] = gemv_a_base<MT, APACK>(A, lda, M, K, t, lane);
    bf16x8 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < n) w[u] = *(const bf16x8*)(wp + (size_t)u * 512);
    bf16x8 a[2][MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) a[0][t] = gemv_a_load<APACK>(ap[t], s0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < n) {
        if (u + 1 < n) {
#pragma unroll
          for (int t = 0; t < MT; ++t) a[(u + 1) & 1][t] = gemv_a_load<APACK>(ap[t], s0 + u + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < MT; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u & 1][t], w[u], c[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  const int cc = lane & 15, rb = (lane >> 4) * 4;
  auto store = [&](int m, int col, float v) {
    if constexpr (EPI == TW_EPI_PARTIAL) {
      ((float*)ea.out)[((size_t)blockIdx.y * M + m) * ea.ldo + col] = v;
    } else if constexpr (EPI == TW_EPI_GELU_PACKED) {
      if (ea.bias) v += ea.bias[col];
      ((bf16_t*)ea.out)[tw_pack_act_idx(m, col, N)] = f32_to_bf16(gelu_erf(v));
    } else {
      epi_store<EPI>(ea, m, col, v);
    }
  };
  if constexpr (KW == 1) {
    const int col = g * 16 + cc;
    if (g < ngroups && col < N) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * t + rb + r < M) store(16 * t + rb + r, col, c[t][r]);
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wid][16 * t + rb + r][cc] = c[t][r];
  __syncthreads();
  constexpr int ROWS = MT * 16;
  for (int e = tid; e < GPB * ROWS * 16; e += NW * 64) {
    const int gg = e / (ROWS * 16), rem = e - gg * ROWS * 16;
    const int m = rem >> 4, cl = rem & 15;
    const int col = (blockIdx.x * GPB + gg) * 16 + cl;
    if (m < M && col < N) {
      float v = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < KW; ++w2) v += red[gg * KW + w2][m][cl];
      store(m, col, v);
    }
  }
}

// k_gemv_q's geometry: the fewest K-slices per block that bring every wave to <= 10 steps. Returns false when the
// shape needs more (the caller falls back to k_gemv_pc).
template <int EPI, bool APACK, int KW, int MT>
static void launch_gemv_q_mt(const bf16_t* A, int lda, const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea,
                             int splits, hipStream_t s) {
  dim3 grid(tw_cdiv(tw_cdiv(N, 16), 4 / KW), splits);
  hipLaunchKernelGGL((k_gemv_q<EPI, KW, 10, APACK, MT>), grid, dim3(256), 0, s, A, lda, Wp, M, N, K, ea);
}
template <int EPI, bool APACK, int KW>
static void launch_gemv_q_kw(const bf16_t* A, int lda, const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea,
                             int splits, hipStream_t s) {
  if (M > 32) launch_gemv_q_mt<EPI, APACK, KW, 4>(A, lda, Wp, M, N, K, ea, splits, s);
  else if (M > 16) launch_gemv_q_mt<EPI, APACK, KW, 2>(A, lda, Wp, M, N, K, ea, splits, s);
  else launch_gemv_q_mt<EPI, APACK, KW, 1>(A, lda, Wp, M, N, K, ea, splits, s);
}
template <int EPI, bool APACK>
static bool launch_gemv_q(const bf16_t* A, int lda, const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea,
                          int splits, hipStream_t s) {
  const int ns = K / 32;  // MFMA steps over K
  const int ngroups = tw_cdiv(N, 16);
  // the longest wave slice at kw K-slices per block: the kernel cuts ns into kw * splits slices of floor / ceil size,
  // and a wave holds at most U = 10 steps in flight (a longer slice would drop its tail)
  auto longest = [&](int kw) { return tw_cdiv(ns, kw * splits); };
  // K-slices per block: the fewest that bring a wave to <= 10 steps; one more halving while the grid stays below
  // 256 workgroups and the waves keep >= 5 steps (o_proj: 80 groups x 4 splits of 10 steps -> KW = 2, 160 blocks)
  int kw = 1;
  while (kw < 4 && longest(kw) > 10) kw *= 2;
  if (longest(kw) > 10) return false;
  while (kw < 4 && (long)tw_cdiv(ngroups, 4 / kw) * splits < 256 && longest(2 * kw) >= 5) kw *= 2;
  if (kw == 1) launch_gemv_q_kw<EPI, APACK, 1>(A, lda, Wp, M, N, K, ea, splits, s);
  else if (kw == 2) launch_gemv_q_kw<EPI, APACK, 2>(A, lda, Wp, M, N, K, ea, splits, s);
  else launch_gemv_q_kw<EPI, APACK, 4>(A, lda, Wp, M, N, K, ea, splits, s);
  return true;
}

template <int EPI, int KW, int U, bool APACK, bool NTW = false>
static void launch_gemv_p3(const bf16_t* A, int lda, const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea, int splits,
                           hipStream_t s) {
  constexpr int NW = KW > 4 ? KW : 4, GPB = NW / KW;
  constexpr int U4 = U > 4 ? U / 2 : U;  // M > 32: four A fragments per step
  dim3 grid(tw_cdiv(tw_cdiv(N, 16), GPB), splits);
  if (M > 32)
    hipLaunchKernelGGL((k_gemv_p<EPI, KW, U4, APACK, 4, NTW>), grid, dim3(NW * 64), 0, s, A, lda, Wp, M, N, K, ea);
  else if (M > 16)
    hipLaunchKernelGGL((k_gemv_p<EPI, KW, U, APACK, 2, NTW>), grid, dim3(NW * 64), 0, s, A, lda, Wp, M, N, K, ea);
  else
    hipLaunchKernelGGL((k_gemv_p<EPI, KW, U, APACK, 1, NTW>), grid, dim3(NW * 64), 0, s, A, lda, Wp, M, N, K, ea);
}

template <int EPI, bool APACK>
static void launch_gemv_p2(const bf16_t* A, int lda, const bf16_t* Wp, int M, int N, int K, const EpiArgs& ea, int splits,
                           hipStream_t s) {
  // K-slices per column group: enough waves to put ~4 on every CU while each keeps >= 4 steps
  const long groups = tw_cdiv(N, 16) * (long)splits;
  const int steps = K / 32 / splits;
  int kw = 1;
  while (groups * kw < 1024 && kw < tw_gemv_max_kw && steps >= 8 * kw) kw *= 2;
  // the vocabulary-wide proj_out (3242 column groups, 133 MB streamed once per step): one K-slice per group,
  // non-temporal weight loads (its MALL residency is what the decoder's layer weights would lose)
  const bool wide = N >= tw_gemv_nt_min_n;
  if (wide) {
    if constexpr (EPI == TW_EPI_F32) {
      // 33..64 rows (beam-5 passes, config 5's windows): two column groups per wave (k_gemv_pc) halve the activation
      // fragments each weight byte costs — at four m-tiles k_gemv_p's waves read 4 KiB of L2-resident activations per
      // 1 KiB weight fragment; one K-slice per group, the MFMA order per output unchanged (bit-identical logits).
      // As-shipped beam-5 call 0.518 -> 0.513 s (profiles/r06pc_proj_out_pc_ab.txt)
      if (M > 32 && tw_gemv_wide_kw == 1) {
        launch_gemv_pc<EPI, 1, APACK, 5, true>(A, lda, Wp, M, N, K, ea, splits, s);
        return;
      }
    }
    if (tw_gemv_wide_kw == 4 && steps >= 8 * 4) launch_gemv_p3<EPI, 4, 8, APACK, true>(A, lda, Wp, M, N, K, ea, splits, s);
    else if (tw_gemv_wide_kw >= 2 && steps >= 8 * 2) launch_gemv_p3<EPI, 2, 8, APACK, true>(A, lda, Wp, M, N, K, ea, splits, s);
    else launch_gemv_p3<EPI, 1, 16, APACK, true>(A, lda, Wp, M, N, K, ea, splits, s);
    return;
  }
  if constexpr (EPI == TW_EPI_BF16 || EPI == TW_EPI_PARTIAL || EPI == TW_EPI_GELU_PACKED) {
    // the layer GEMVs as column-group pairs (k_gemv_pc): a third fewer vector-memory instructions per weight byte
    // (k_gemv_q from 17 rows: at <= 16 one m-tile leaves its waves too little work, step 328 vs 323 us at 15 rows)
    if (tw_gemv_kernel == 1 && M > 16 && M <= 32 && launch_gemv_q<EPI, APACK>(A, lda, Wp, M, N, K, ea, splits, s)) return;
    const long pairs = tw_cdiv(tw_cdiv(N, 16), 2) * (long)splits;
    if (pairs * 2 < 1024 && steps >= 8 * 4) launch_gemv_pc<EPI, 4, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
    else launch_gemv_pc<EPI, 2, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
    return;
  }
  if (kw == 1) launch_gemv_p3<EPI, 1, 16, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
  else if (kw == 2) launch_gemv_p3<EPI, 2, 8, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
  else launch_gemv_p3<EPI, 4, 8, APACK>(A, lda, Wp, M, N, K, ea, splits, s);
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
    const unsigned nwg = tw_cdiv(M, GB_BM) * tw_cdiv(N, GB_BN);
    // k_gemm_8pp stages the bias by 16-byte DMA: N % 4 == 0 and a 16-byte aligned bias (else k_gemm_8p)
    if (tw_gemm_kernel == 6 && N % 4 == 0 && N >= 4 && ((uintptr_t)ea.bias & 15) == 0)
      hipLaunchKernelGGL(k_gemm_8pp<EPI>, dim3(std::min<unsigned>(tw_persistent_grid(), (nwg + 7) / 8 * 8)), dim3(512),
                         0, s, A, W, M, N, K, lda, ldw, ea);
    else if (tw_gemm_kernel >= 5 && tw_gemm_tr)
      hipLaunchKernelGGL((k_gemm_8p<EPI, true>), dim3(nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
    else if (tw_gemm_kernel >= 5)
      hipLaunchKernelGGL((k_gemm_8p<EPI, false>), dim3(nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
    else if (tw_gemm_tr)
      hipLaunchKernelGGL((k_gemm_big<EPI, true>), dim3(nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
    else
      hipLaunchKernelGGL((k_gemm_big<EPI, false>), dim3(nwg), dim3(512), 0, s, A, W, M, N, K, lda, ldw, ea);
  }
  return tw_check_launch("tw_gemm_bf16");
}

extern "C" int tw_gemm_bf16(const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldw, int epi,
                            void* out, int ldo, const float* bias, const float* aux, int aux_rows,
                            const int* kv_geom, void* stream) {
  TW_REQUIRE(A && W && out, "tw_gemm_bf16: null pointer");
  TW_REQUIRE(M > 0 && N > 0 && K > 0 && K % GB_BK == 0, "tw_gemm_bf16: M=%d N=%d K=%d (K %% 64 required)", M, N, K);
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

// Encoder conv2 + GELU + positional add as an implicit GEMM (modeling_whisper.py:566-568: Conv1d(D, D, 3, stride 2,
// padding 1)). Output frame t of window r reads input frames 2t-1, 2t, 2t+1; in the time-major h1 [R][3000][D]
// those are 3 D contiguous elements starting at frame 2t-1, so the A operand is h1 itself read at a row stride of
// 2 D (rows overlapping by D) — no im2col copy. Frame -1 is the zero padding, which that view does not see: the
// t = 0 row of window r takes its first tap from window r-1's last frame (window 0: from the row in front of h1), so
// those R rows are recomputed afterwards from taps 1-2 alone (K = 2 D, A rows one window apart).
extern "C" int tw_conv2_gemm(const bf16_t* h1, int R, int D, const bf16_t* W, const float* bias, const float* pos,
                             float* out, void* stream) {
  TW_REQUIRE(h1 && W && bias && pos && out, "tw_conv2_gemm: null pointer");
  TW_REQUIRE(R > 0 && D > 0 && D % 32 == 0, "tw_conv2_gemm: R=%d D=%d (D %% 32 required)", R, D);
  hipStream_t s = (hipStream_t)stream;
  EpiArgs ea{out, D, bias, pos, 1500, 0, 0, 0, 0};
  ea.group_m = tw_group_for(D);
  int rc = launch_gemm<TW_EPI_GELU_POS_F32>(h1 - D, W, R * 1500, D, 3 * D, 2 * D, 3 * D, ea, s);
  if (rc) return rc;
  // fixup rows in chunks of <= 32 windows: always the skinny kernel, whose per-row sums do not depend on the row
  // count, so a window's encoder output is the same in a batch of 8 as in a batch of 64
  for (int r0 = 0; r0 < R && !rc; r0 += 32) {
    EpiArgs e0{out + (size_t)r0 * 1500 * D, 1500 * D, bias, pos, 1, 0, 0, 0, 0};  // row r -> output row 1500 r
    e0.group_m = 1;
    rc = launch_gemm<TW_EPI_GELU_POS_F32>(h1 + (size_t)r0 * 3000 * D, W + D, std::min(32, R - r0), D, 2 * D,
                                          3000 * D, 3 * D, e0, s);
  }
  return rc;
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
  TW_REQUIRE(M > 0 && M <= 64 && N > 0 && K > 0 && K % 32 == 0, "tw_gemv_packed: M=%d N=%d K=%d (M <= 64, K %% 32)", M,
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

  // operands through one buffer descriptor per operand tile (32-bit per-lane offsets instead of eight 64-bit
  // pointers: the registers that keep this kernel beside a decode; rows past M / N read as zeros, never stored)
  const int rows_a = max(0, min(GB_BM, M - m0)), rows_w = max(0, min(GB_BN, N - n0));
  const __amdgpu_buffer_rsrc_t ra = tw_uniform_rsrc(A + (size_t)m0 * lda, rows_a ? (rows_a - 1) * lda + K : 0);
  const __amdgpu_buffer_rsrc_t rw = tw_uniform_rsrc(W + (size_t)n0 * ldw, rows_w ? (rows_w - 1) * ldw + K : 0);
  unsigned va[4], vw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wid + i) + (lane >> 3);
    const int ch = (lane & 7) ^ gb_swz(row);
    va[i] = (unsigned)(row * lda + ch * 16);
    vw[i] = (unsigned)(row * ldw + ch * 16);
  }
  // scales of K-step kt: rows m0..m0+255 of [K/128][Mp][4] are 1 KiB contiguous (Mp, Np: multiples of 256)
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const unsigned gs_step = (unsigned)(wu == 0 ? Mp : Np) * 4u;
  const __amdgpu_buffer_rsrc_t rsc =
      tw_uniform_rsrc(wu == 0 ? Sa + (size_t)m0 * 4 : Sw + (size_t)n0 * 4, (int)((K / MX_BK - 1) * gs_step + 1024u));
  auto stage = [&](int buf, int kt) {
    uint8_t* As = smem + buf * MX_STAGE;
    uint8_t* Ws = As + MX_TILE;
    const unsigned k0 = (unsigned)(kt * MX_BK);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rb = 8 * (4 * wid + i) * MX_BK;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)(As + rb), 16, va[i], k0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_void_t*)(Ws + rb), 16, vw[i], k0, 0, 0);
    }
    if (wu < 2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsc, (lds_void_t*)(As + 2 * MX_TILE + wu * 1024), 16,
                                               (unsigned)lane * 16u, (unsigned)kt * gs_step, 0, 0);
  };

  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int lane_lo = fr * MX_BK + ((fq ^ ((fr >> 1) & 7)) << 4), lane_hi = fr * MX_BK + (((fq + 4) ^ ((fr >> 1) & 7)) << 4);
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
    // (fragments loaded as bf16x8 values and bit-cast, as k_gemm_8p_mx: int4 loads make hipcc drain vmcnt before
    // them; the four W scale bytes packed into one register, picked by the MFMA's op_sel)
    // (every fragment row of this lane is 16 k + fr: the chunk swizzle gb_swz(row) = (fr >> 1) & 7 is the same for
    // all of them, so a fragment's address is one lane offset plus a compile-time row offset — no per-fragment
    // address registers held across the loop)
    auto frag = [&](const uint8_t* p, int r) {
      (void)r;
      const bf16x8 lo8 = *(const bf16x8*)(p + lane_lo);
      const bf16x8 hi8 = *(const bf16x8*)(p + lane_hi);
      const int4 lo = __builtin_bit_cast(int4, lo8), hi = __builtin_bit_cast(int4, hi8);
      return (i32x8){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    };
    uint32_t sbp = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) sbp |= (uint32_t)SWs[(wc * 64 + j * 16 + fr) * 4 + fq] << (8 * j);
    // two passes over the A fragments, two W fragments each: 16 instead of 32 W-fragment registers (the
    // co-residency budget: <= 192 VGPRs leaves every SIMD a decoder wave of <= 128 beside two GEMM waves), at twice
    // the A-fragment LDS reads (~60 % of the LDS bandwidth at full MFMA rate)
    auto pass = [&](auto JH) {
      constexpr int jh = decltype(JH)::value;
      i32x8 bfr[2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        bfr[jj] = frag(Ws + (wc * 64 + (2 * jh + jj) * 16) * MX_BK, 0);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const i32x8 af = frag(As + (wr * 128 + i * 16) * MX_BK, 0);
        const int sa = SAs[(wr * 128 + i * 16 + fr) * 4 + fq];
        acc[i][2 * jh] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[0], acc[i][2 * jh], 0, 0, 0, sa,
                                                                          2 * jh, (int)sbp);
        acc[i][2 * jh + 1] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[1], acc[i][2 * jh + 1], 0, 0, 0,
                                                                              sa, 2 * jh + 1, (int)sbp);
        __builtin_amdgcn_sched_barrier(0);  // (one A fragment live at a time)
      }
    };
    pass(std::integral_constant<int, 0>{});
    pass(std::integral_constant<int, 1>{});
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

  // operands through one buffer descriptor per half-tile (as k_gemm_8p: 32-bit per-lane offsets instead of eight 64-bit
  // pointers — the registers this kernel's spill margin needs; rows past M / N read as zeros, never stored)
  __amdgpu_buffer_rsrc_t rs[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int r0 = (h < 2 ? m0 : n0) + 128 * (h & 1), lim = h < 2 ? M : N, ld = h < 2 ? lda : ldw;
    const int rows = max(0, min(128, lim - r0));
    rs[h] = tw_uniform_rsrc((h < 2 ? A : W) + (size_t)r0 * ld, rows ? (rows - 1) * ld + K : 0);
  }
  unsigned voff[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 8 * (2 * wid + i) + (lane >> 3);
    const int ch = (lane & 7) ^ gb_swz(row);
    voff[0][i] = (unsigned)(row * lda + ch * 16);
    voff[1][i] = (unsigned)(row * ldw + ch * 16);
  }
  // scale DMA: wave w < 4 -> A scale dwords of rows 64w + lane, w >= 4 -> W rows 64(w-4) + lane, through one buffer
  // descriptor per wave. (It was a global_load_lds: hipcc then drained vmcnt to 0 before every ds_read of the K loop —
  // four full drains per K-tile, the next K-tile's DMA latency exposed in every phase — which it does not do for
  // buffer_load ... lds.)
  const int nk = K / MX_BK;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const unsigned gsc_step = (unsigned)(wu < 4 ? Mp : Np) * 4u;
  const __amdgpu_buffer_rsrc_t rsc = tw_uniform_rsrc(
      wu < 4 ? Sa + (size_t)(m0 + 64 * wu) * 4 : Sw + (size_t)(n0 + 64 * (wu - 4)) * 4, (int)((nk - 1) * gsc_step + 256u));
  auto stage = [&](int buf, int h, int kt) {
    uint8_t* dst = smem + (buf * 4 + h) * HT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs[h], (lds_void_t*)(dst + 8 * (2 * wid + i) * MX_BK), 16,
                                               voff[h >> 1][i], (unsigned)(kt * MX_BK), 0, 0);
  };
  auto stage_sc = [&](int buf, int kt) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsc, (lds_void_t*)(smem + MX8_SC + buf * 2048 + wu * 256), 4,
                                             (unsigned)lane * 4u, (unsigned)kt * gsc_step, 0, 0);
  };

  i32x8 af[4], bfr[2];
  int sap[2], sbp;
  auto frag = [&](const uint8_t* base, int row) {
    const uint8_t* p = base + row * MX_BK;
    // (loaded as bf16x8 values, as k_gemm_8p's fragments, and only then bit-cast: with int4 loads — also what
    // __builtin_bit_cast of the dereference itself emits — hipcc drained vmcnt to 0 before the fragment reads of every
    // phase, exposing the next K-tile's DMA latency four times per K-tile; with bf16x8 loads it relies on the kernel's
    // own counted waits, as in k_gemm_8p)
    const bf16x8 lo8 = *(const bf16x8*)(p + ((fq ^ gb_swz(row)) << 4));
    const bf16x8 hi8 = *(const bf16x8*)(p + (((fq + 4) ^ gb_swz(row)) << 4));
    const int4 lo = __builtin_bit_cast(int4, lo8), hi = __builtin_bit_cast(int4, hi8);
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
  auto readS = [&](int buf) {  // this lane's scale bytes: (tile row, K block fq) of every fragment of the K-tile,
    // packed four to a register (the MFMA's op_sel picks the byte): 3 VGPRs instead of 12, the kernel's spill margin
    const uint8_t* S = smem + MX8_SC + buf * 2048;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh) {
      uint32_t p = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) p |= (uint32_t)S[(128 * mh + 64 * wr + 16 * i + fr) * 4 + fq] << (8 * i);
      sap[mh] = (int)p;
    }
    uint32_t q = 0;
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int j = 0; j < 2; ++j) q |= (uint32_t)S[1024 + (128 * nh + 32 * wc + 16 * j + fr) * 4 + fq] << (8 * (2 * nh + j));
    sbp = (int)q;
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
#define TW_MXS(i, j)                                                                                          \
  acc[mh][nh][i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[mh][nh][i][j], 0, 0, i, \
                                                                       sap[mh], 2 * nh + j, sbp)
    TW_MXS(0, 0); TW_MXS(0, 1); TW_MXS(1, 0); TW_MXS(1, 1); TW_MXS(2, 0); TW_MXS(2, 1); TW_MXS(3, 0); TW_MXS(3, 1);
#undef TW_MXS
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

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
        a = mx_group4_max_dpp(a);  // (quad permutes on the VALU, not two ds_bpermute round trips)
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

// tw_gemm_mx kernel choice: 0 = default, by shape — k_gemm_mx for the q/k/v shape (N = 3 K), k_gemm_8p_mx for the
// rest; 1 = k_gemm_mx, 8 = k_gemm_8p_mx (tw_gemm_mx_set_variant, forced forms for A/B and tests). Since k_gemm_8p_mx
// packs its scale bytes four to a register (op_sel) and streams through buffer descriptors (spills 136 -> 84 bytes)
// it won every encoder shape (profiles/r05y_gemm_mx_ab.txt); since k_gemm_mx did the same and took 182 VGPRs it wins
// q/k/v again (573 vs 596 us at M = 96000, profiles/r05ba_mx_beside_ab.txt): config 5 183.2 -> 180.7 ms per step with
// the shape rule (profiles/r05bb_mx_shape_rule_ab.txt).
static int tw_gemm_mx_variant = 0;
extern "C" int tw_gemm_mx_set_variant(int v) {
  tw_gemm_mx_variant = (v == 1 || v == 8) ? v : 0;
  return 0;
}
static inline bool mx_use_8p(int M, int N, int K) {
  (void)M;
  if (tw_gemm_mx_variant == 0) return N != 3 * K;
  return tw_gemm_mx_variant == 8;
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
