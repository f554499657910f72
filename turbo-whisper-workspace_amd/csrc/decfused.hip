// decfused.hip — the decoder's layers for one token as ONE persistent launch (k_dec_fused).
//
// Replaces, for a decode pass that has the GPU to itself, the 45 launches of WhisperEngine.decoder_step between the
// token embedding and proj_out (per layer: residual + LayerNorm, q/k/v GEMV, self-attention, out_proj, residual +
// LayerNorm, cross-q GEMV, cross-attention, out_proj, residual + LayerNorm, fc1 + GELU, fc2; then the final
// LayerNorm): WhisperDecoderLayer.forward ($TF/models/whisper/modeling_whisper.py:448-505) and the decoder's final
// layer_norm (:682, :795). In the launch chain every one of those kernels pays a dispatch-to-completion floor of
// 4-6 us for ~5 us of work; here one workgroup per CU walks the step's phases and hands each phase's
// output to the next through write-through stores and per-XCD-sharded completion counters
// (cdna_hip_programming.md §6 Guideline 16, recipe R1: sc1 payload stores, every storing wave drained, one counter
// add behind a workgroup barrier; consumer: one relaxed poll of the counter's eight shards, then sc1 loads of every
// handed-off byte — the table row under which the agent-scope acquire may go; tw_dec_fused_set_acquire(1) keeps it
// for an A/B, with bit-identical results). A workgroup
// issues the weight loads of its next GEMV item BEFORE it waits for that phase's inputs, so the weight stream of a
// phase overlaps the previous phase's tail and the hand-off itself.
//
// Phases per layer (items i of a phase go to workgroups (off + i) mod G, G = grid size = resident workgroups):
//   LN1   R rows: self_attn_layer_norm -> hp (packed bf16, the GEMV operand; one wave per row)
//   QKV   240 column groups of 16 (K = 1280) of hp, + bias; q -> qb, k / v -> the self-attention cache at pos
//   SELF  R x 20 (row, head), 1, 2 or 4 heads per item: online softmax over keys 0..pos (the cache) -> ab
//   O     80 groups: x += ab . Wo + bo (the owner of a column group updates the residual in place)
//   LN2   R rows -> hp;  QX  80 groups: cross q -> qb
//   CROSS R x 20 x XS key slices: online softmax over the encoder keys (non-temporal K/V); the (row, head)'s last
//         slice (arrival ticket) merges the slice states -> ab
//   OX    80 groups: x += ab . Wo_x + bo_x;  LN3  R rows -> hp
//   FC1   160 items of two column groups: GELU(hp . W1 + b1) -> fb (packed, K = 5120)
//   FC2   160 items = 40 column-group pairs x 4 K-quarters: f32 partial slabs; the last of a pair's four arrivals
//         (arrival ticket) adds x + b2 + the four slabs in quarter order and writes x
//   then FIN: R rows, the final LayerNorm -> hp (proj_out's operand)
// Per-phase timestamps from the kernel itself (tw_dec_fused_set_probe, scripts/fused_probe.py) put a phase at 1.5-4 us
// of work plus a 0.6-2.5 us hand-off, against the 4-6 us dispatch-to-completion floor of each launch it replaces.
// A phase waits only for its predecessor's counter to reach (layer + 1) x its item count (monotonic within the
// launch; the counters are zeroed by a memset node in front of every launch). Every spin is bounded: on timeout the
// workgroup sets the sticky error word and every later wait falls through, so the grid always drains; the host
// checks the word after the pass.
//
// Residency: one 256-thread workgroup per CU (its registers admit no second) and G <= the CU count, so every
// workgroup is resident once whatever else shares the device has retired; no wait depends on a workgroup that is
// not yet running for longer than that. The engine uses the launch for decode passes with nothing queued beside.
#include "tw_common.h"
#include "../../include/tw_whisper.h"

namespace {

constexpr int FD = 1280, FH = 20, FF = 5120;
constexpr int FNS = FD / 32;      // 40 MFMA steps of K = 32 per d_model-deep item
constexpr int FNS2 = FF / 32;     // 160 (fc2)
constexpr int NWAVE = 4, NTHR = NWAVE * 64;  // waves per workgroup (one workgroup per CU, one wave per SIMD)
constexpr int US = FNS / NWAVE;   // K-steps per wave per item (4 waves x 10 = 40)
constexpr int G_QKV = 3 * FD / 16, G_D = FD / 16, G_FP = FF / 32;  // 240, 80, 160 (fc1 column-group pairs)
constexpr int N_FC2 = (G_D / 2) * 4;                                 // 160: 40 pairs x 4 K-quarters
enum { K_LN1, K_QKV, K_SELF, K_O, K_LN2, K_QX, K_CROSS, K_OX, K_LN3, K_FC1, K_FC2, K_FIN, NKIND };
constexpr int SHARDS = 8, CSTRIDE = 32;                  // one 128-B line per counter shard
// Arrival tickets, spread over cache lines: atomics on one 128-B line serialise (~12 ns each, MI355X_MICROARCH.md
// fanin), so a line takes at most 8 pair / (row, head) tickets and a row ticket (80 arrivals per layer) has its own.
constexpr int TSTRIDE = 4;                               // words between pair / (row, head) tickets
constexpr int TICKET_OFF = NKIND * SHARDS * CSTRIDE;     // words: 40 fc2 pair tickets
constexpr int XTICKET_OFF = TICKET_OFF + 40 * TSTRIDE;   // 20 R cross-attention (row, head) tickets
constexpr int RTICKET_OFF = XTICKET_OFF + 640 * TSTRIDE; // 3 x 32 row tickets (rows of x completed by O, OX, FC2)
constexpr int SYNC_WORDS = RTICKET_OFF + 3 * 32 * CSTRIDE;
constexpr int XS_MAX = 12;                               // key slices of a cross-attention (row, head)
constexpr int XUNR = 16;                                 // cross-attention key rows in flight per 8-lane group
// The phases' first workgroups (item i -> workgroup (off + i) mod G): the LayerNorm rows and the phases that follow a
// narrow phase start on workgroups that sat the previous phase out, so their weight loads are in flight during it.
constexpr int OFF_LN1 = 224, OFF_LN = 96, OFF_QX = 128, OFF_FC1 = 128;
constexpr unsigned SPIN_MAX = 1u << 20;                  // polls (each >= one L2 round trip + s_sleep 1)

// LDS: [0, 2.5 KiB) attention scratch; [2.5 KiB, +17 KiB) cross-wave GEMV reduction; then flag words. (One
// 256-thread workgroup per CU: one wave per SIMD with up to 512 registers; the grid is what the occupancy query admits.)
constexpr int SM_A = 0, SM_RED = 2560, SM_FLAG = SM_RED + NWAVE * 2 * 32 * 17 * 4, SM_BYTES = SM_FLAG + 64;

struct FusedArgs {
  const TwDecLayerW* layers;
  int n_layers, R, T, S;
  const int* pos;
  float* x;
  bf16_t *kc, *vc;
  long kv_layer_stride;
  const bf16_t* xkv;
  long xkv_layer_stride, xkv_v_off;
  bf16_t *qb, *ab, *fb;
  float* slab;
  const float *lnf_g, *lnf_b;
  bf16_t* hp;
  float eps;
  unsigned* sync;
  unsigned* err;
  int acq;  // 1: an agent-scope acquire after every poll (redundant with the sc1 loads; A/B)
  int hp_self;  // heads per self-attention item (1, 2 or 4: items <= grid)
  int xs;       // key slices per cross-attention (row, head) (1 .. XS_MAX)
  float* xpart; // [R x 20][xs][66] slice states
  unsigned long long* probe;  // NULL, or [n_layers + 1][NKIND][grid][2] timestamps
};

// Measurement (tw_dec_fused_set_probe): per (layer, phase, workgroup) the 100-MHz real-time clock when the workgroup
// started the phase's first item (after its wait) and finished its last; slot (n_layers, 0) = the workgroup's start.
__device__ __forceinline__ void probe(const FusedArgs& a, int l, int kind, int which) {
  if (a.probe != nullptr && threadIdx.x == 0)
    a.probe[(((size_t)l * NKIND + kind) * gridDim.x + blockIdx.x) * 2 + which] = __builtin_amdgcn_s_memrealtime();
}

// Global-memory loads through pointers the compiler cannot place (fields of the layer table): without the address
// space they compile to flat loads, which also count against lgkmcnt and make every LDS wait conservative.
// (HIP's float4 / float2 / uint4 are structs, for which the address space is lost: loaded as ext vectors)
template <class T>
__device__ inline T gld(const void* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}
template <>
__device__ inline float4 gld<float4>(const void* p) {
  const f32x4 v = gld<f32x4>(p);
  return make_float4(v[0], v[1], v[2], v[3]);
}
template <>
__device__ inline float2 gld<float2>(const void* p) {
  const f32x2 v = gld<f32x2>(p);
  return make_float2(v[0], v[1]);
}
template <>
__device__ inline uint4 gld<uint4>(const void* p) {
  const tw_u32x4 v = gld<tw_u32x4>(p);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// Loads of bytes another workgroup of this launch wrote (all stored write-through, st_sc1): sc1 buffer loads, which
// bypass this CU's L1, the only cache that can hold a stale copy (the XCD L2s are kept coherent for device memory).
// With every such load sc1 the agent-scope acquire after a poll is redundant (cdna_hip_programming.md §6 Guideline 16,
// Valid forms, table row 1); FusedArgs::acq keeps it for an A/B (tw_dec_fused_set_acquire).
__device__ inline __amdgpu_buffer_rsrc_t hrs(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
}
__device__ inline f32x4 hld4(const void* base, size_t off) {  // 16 B at base + off bytes
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(hrs(base), (int)off, 0, 16));
}
__device__ inline f32x2 hld2(const void* base, size_t off) {  // 8 B
  return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(hrs(base), (int)off, 0, 16));
}

__device__ inline unsigned* ctr(unsigned* s, int kind, int shard) { return s + (kind * SHARDS + shard) * CSTRIDE; }

__device__ inline void st_sc1(void* p, unsigned v) {
  __hip_atomic_store((unsigned*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_sc1(void* p, float a, float b) {
  const unsigned long long v =
      (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32);
  __hip_atomic_store((unsigned long long*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0: poll the kind's eight shards (lanes 0..7, relaxed agent loads = global_load sc1) until their sum reaches
// target; false on timeout or when another workgroup has already failed.
__device__ __forceinline__ bool poll_ge(unsigned* s, int kind, unsigned target, unsigned* err, int lane) {
  unsigned* p = ctr(s, kind, lane & 7);
  for (unsigned it = 0;; ++it) {
    unsigned v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v = lane < 8 ? v : 0u;
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v = __shfl(v, 0, 64);
    if (v >= target) return true;
    if ((it & 255u) == 255u) {
      const unsigned e = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (e != 0u || it >= SPIN_MAX) {
        if (lane == 0 && e == 0u) __hip_atomic_store(err, 0x100u + (unsigned)kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// The consumer side of a hand-off: one poll, (optionally) one acquire (this CU's L1 dropped) and its wait, then the
// barrier that releases every wave's sc1 loads of the handed-off bytes. Returns false when the wait failed (the outputs of the step are then void).
__device__ __forceinline__ bool wg_wait(const FusedArgs& a, int kind, unsigned target, int* flag) {
  if (threadIdx.x < 64) {
    const bool ok = poll_ge(a.sync, kind, target, a.err, threadIdx.x);
    if (a.acq) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the poll)
    }
    if (threadIdx.x == 0) *flag = ok ? 1 : 0;
  }
  __syncthreads();
  return *flag != 0;
}

// The producer side: every wave drains its write-through stores, then one lane counts the item.
__device__ __forceinline__ void wg_signal(const FusedArgs& a, int kind) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr(a.sync, kind, blockIdx.x & 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Weight fragments of one item for this wave: NG column groups from g0, steps [s0, s0 + US) of a K of ns steps.
template <int NG>
__device__ inline void load_w(bf16x8 (&w)[NG][US], const bf16_t* Wp, int ns, int g0, int s0, int lane) {
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const bf16_t* p = Wp + ((size_t)(g0 + g) * ns + s0) * 512 + lane * 8;
#pragma unroll
    for (int u = 0; u < US; ++u) w[g][u] = gld<bf16x8>(p + (size_t)u * 512);
  }
}

// A operand sources: 0 = LDS packed (K = 1280), 1 = global row-major [R][1280], 2 = global packed (K = 5120).
template <int ASRC, int MT>
__device__ inline bf16x8 load_a(const bf16_t* A, int R, int s, int t, int lane) {
  if constexpr (ASRC == 1) {
    const int row = min(16 * t + (lane & 15), R - 1);
    return __builtin_bit_cast(bf16x8, hld4(A, ((size_t)row * FD + s * 32 + 8 * (lane >> 4)) * 2));
  } else if constexpr (ASRC == 2) {
    return __builtin_bit_cast(bf16x8, hld4(A, ((size_t)(s * 2 + t) * 64 + lane) * 16));
  } else {
    return *(const bf16x8*)(A + ((size_t)(s * 2 + t) * 64 + lane) * 8);
  }
}

// This wave's US steps from s0 of NG column groups: every A fragment loaded before the first MFMA.
template <int NG, int MT, int ASRC>
__device__ inline void gemv_mma(f32x4 (&c)[NG][MT], const bf16x8 (&w)[NG][US], const bf16_t* A, int R, int s0,
                                int lane) {
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int t = 0; t < MT; ++t) c[g][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 af[US][MT];
#pragma unroll
  for (int u = 0; u < US; ++u)
#pragma unroll
    for (int t = 0; t < MT; ++t) af[u][t] = load_a<ASRC, MT>(A, R, s0 + u, t, lane);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int u = 0; u < US; ++u)
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int t = 0; t < MT; ++t) c[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u][t], w[g][u], c[g][t], 0, 0, 0);
}

// Cross-wave sum through LDS: red[w][g][row][17]; after it, sum4(g, m, col) is the item's output (waves in order).
template <int NG, int MT>
__device__ inline void red_store(float* red, const f32x4 (&c)[NG][MT]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, cc = lane & 15, rb = (lane >> 4) * 4;
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((wid * 2 + g) * 32 + 16 * t + rb + r) * 17 + cc] = c[g][t][r];
}
__device__ inline float red_sum(const float* red, int g, int m, int col) {
  float v = 0.f;
#pragma unroll
  for (int w = 0; w < NWAVE; ++w) v += red[((w * 2 + g) * 32 + m) * 17 + col];
  return v;
}

// One (row, head) attention over keys [k0, k1) by the NWV waves of sub-group wid / NWV of the workgroup (8 / NWV heads
// at once): online softmax per 8-lane key group (NWV x 8 groups; keys k0 + g, k0 + g + NG, ...), the groups merged by
// shuffles and through LDS (the arithmetic of k_attn_decode_cross_lean<32> at NWV = 4, UNR = 8). q (64 bf16, pre-scaled) at
// qb + q_off elements, written in this launch (sc1 loads); K / V rows [key][64] at Kb / Vb + kv_off: NT (the encoder's
// cross K/V) non-temporal plain loads, else (the self-attention cache, appended in this launch) sc1 loads. Result:
// out != NULL: the 64 normalised outputs (bf16, sc1 stores); else the unnormalised state {max, sum, 64 sums} at st.
template <bool NT, int NWV, int UNR>
__device__ __forceinline__ void attend(const bf16_t* qb, size_t q_off, const bf16_t* Kb, const bf16_t* Vb,
                                       size_t kv_off, int k0, int k1, bf16_t* out, float* st, float* wpart,
                                       float* wml) {
  constexpr int NG = NWV * 8;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, sub = wid / NWV;
  const int lt = tid - sub * NWV * 64, g = lt >> 3, gl = lt & 7;
  float qv[8];
  {
    const uint4 qr = __builtin_bit_cast(uint4, hld4(qb, (q_off + gl * 8) * 2));
    const bf16_t* qe = (const bf16_t*)&qr;
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[e] = bf16_to_f32(qe[e]);
  }
  const int nk = k1 - k0;
  float m = -INFINITY, l = 0.f;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int nit = (nk + NG - 1) / NG;
  for (int it0 = 0; it0 < nit; it0 += UNR) {
    uint4 kk[UNR], vv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int key = k0 + min((it0 + u) * NG + g, nk - 1);
      const size_t e = kv_off + (size_t)key * 64 + gl * 8;
      if constexpr (NT) {
        typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
        typedef const __attribute__((address_space(1))) u32x4_nt* gp;
        const u32x4_nt a4 = __builtin_nontemporal_load((gp)(Kb + e));
        const u32x4_nt c4 = __builtin_nontemporal_load((gp)(Vb + e));
        kk[u] = make_uint4(a4.x, a4.y, a4.z, a4.w);
        vv[u] = make_uint4(c4.x, c4.y, c4.z, c4.w);
      } else {
        kk[u] = __builtin_bit_cast(uint4, hld4(Kb, e * 2));
        vv[u] = __builtin_bit_cast(uint4, hld4(Vb, e * 2));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    float sv[UNR];
    float bm = m;
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      float d = 0.f;
      const bf16_t* ke = (const bf16_t*)&kk[u];
#pragma unroll
      for (int e = 0; e < 8; ++e) d += qv[e] * bf16_to_f32(ke[e]);
      d = lane8_sum(d);
      sv[u] = (it0 + u) * NG + g < nk ? d : -INFINITY;
      bm = fmaxf(bm, sv[u]);
    }
    if (bm == -INFINITY) continue;
    const float sc = __expf(m - bm);
    l *= sc;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= sc;
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const float p = __expf(sv[u] - bm);
      l += p;
      const bf16_t* ve = (const bf16_t*)&vv[u];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += p * bf16_to_f32(ve[e]);
    }
    m = bm;
  }
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) {
    const float m2 = __shfl_xor(m, o, 64), l2 = __shfl_xor(l, o, 64);
    const float M = fmaxf(m, m2);
    const float s1 = m == -INFINITY ? 0.f : __expf(m - M), s2 = m2 == -INFINITY ? 0.f : __expf(m2 - M);
    l = l * s1 + l2 * s2;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = acc[e] * s1 + __shfl_xor(acc[e], o, 64) * s2;
    m = M;
  }
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) wpart[wid * 64 + lane * 8 + e] = acc[e];
    if (lane == 0) {
      wml[wid * 2] = m;
      wml[wid * 2 + 1] = l;
    }
  }
  __syncthreads();
  if (lt < 32) {
    const int w1 = sub * NWV;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NWV; ++w) M = fmaxf(M, wml[(w1 + w) * 2]);
    float v0 = 0.f, v1 = 0.f, tot = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      const float mg = wml[(w1 + w) * 2];
      const float wt = mg == -INFINITY ? 0.f : __expf(mg - M);
      tot += wt * wml[(w1 + w) * 2 + 1];
      v0 += wt * wpart[(w1 + w) * 64 + 2 * lt];
      v1 += wt * wpart[(w1 + w) * 64 + 2 * lt + 1];
    }
    if (out != nullptr) {
      st_sc1(out + 2 * lt, pack_bf16x2(v0 / tot, v1 / tot));
    } else {
      st_sc1(st + 2 + 2 * lt, v0, v1);
      if (lt == 0) st_sc1(st, M, tot);
    }
  }
  __syncthreads();  // (wpart / wml reused by the next item)
}

// LayerNorm of one row held by one wave (lane: float4 chunks lane + 64 i; the arithmetic of k_resid_ln_w) -> row r of
// the packed activation hp (sc1 stores).
__device__ __forceinline__ void ln_vals(const float4 (&v)[5], const float4 (&gg)[5], const float4 (&bb)[5], int r,
                                        float eps, bf16_t* hp, int lane) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 5; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = wave_sum(s) / (float)FD;
  float q2 = 0.f;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const float p = v[i].x - mean, q = v[i].y - mean, rr = v[i].z - mean, t = v[i].w - mean;
    q2 += (p * p + q * q) + (rr * rr + t * t);
  }
  const float rstd = rsqrtf(wave_sum(q2) / (float)FD + eps);
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int c = lane + 64 * i;
    const unsigned lo = pack_bf16x2((v[i].x - mean) * rstd * gg[i].x + bb[i].x, (v[i].y - mean) * rstd * gg[i].y + bb[i].y);
    const unsigned hi = pack_bf16x2((v[i].z - mean) * rstd * gg[i].z + bb[i].z, (v[i].w - mean) * rstd * gg[i].w + bb[i].w);
    st_sc1(hp + tw_pack_act_idx(r, 4 * c, FD), __uint_as_float(lo), __uint_as_float(hi));
  }
}

// LayerNorm of row r of x by one wave -> hp.
__device__ __forceinline__ void ln_row(const float* x, int r, const float* g, const float* b, float eps, bf16_t* hp,
                                       int lane) {
  float4 v[5], gg[5], bb[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const f32x4 t = hld4(x, ((size_t)r * FD + 4 * (lane + 64 * i)) * 4);
    v[i] = make_float4(t[0], t[1], t[2], t[3]);
    gg[i] = gld<float4>(g + 4 * (lane + 64 * i));
    bb[i] = gld<float4>(b + 4 * (lane + 64 * i));
  }
  ln_vals(v, gg, bb, r, eps, hp, lane);
}

// Items i of a phase of n items go to workgroup (off + i) mod G: this workgroup's first item, or n if none.
__device__ inline int first_item(int off, int G) { return (int)(((long)blockIdx.x - off % G + G) % G); }

template <int MT>
__global__ __launch_bounds__(NTHR, 1) void k_dec_fused(FusedArgs a) {
  TW_DEC_PRIO();
  __shared__ __attribute__((aligned(16))) char smem[SM_BYTES];
  float* red = (float*)(smem + SM_RED);
  int* flag = (int*)(smem + SM_FLAG);
  float* wpart = (float*)(smem + SM_A);
  float* wml = wpart + NWAVE * 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, G = gridDim.x;
  const int R = a.R, nrh = R * FH, HP = a.hp_self, XS = a.xs;
  const int n_self = nrh / HP, n_cross = nrh * XS;
  bool ok = true;
  probe(a, a.n_layers, 0, 0);  // (the workgroup's start)
  for (int l = 0; l < a.n_layers; ++l) {
    const TwDecLayerW L = a.layers[l];
    bf16_t* kc = a.kc + (size_t)l * a.kv_layer_stride;
    bf16_t* vc = a.vc + (size_t)l * a.kv_layer_stride;
    const unsigned lp1 = (unsigned)(l + 1);
    // ---- LN1: self_attn_layer_norm of row it -> hp (one wave)
    for (int it = first_item(OFF_LN1, G); it < R; it += G) {
      if (it == first_item(OFF_LN1, G) && l > 0) ok = wg_wait(a, K_FC2, (unsigned)l * (G_D / 2), flag) && ok;
      if (it == first_item(OFF_LN1, G)) probe(a, l, K_LN1, 0);
      if (wid == 0) ln_row(a.x, it, L.ln1_g, L.ln1_b, a.eps, a.hp, lane);
      wg_signal(a, K_LN1);
      probe(a, l, K_LN1, 1);
    }
    // ---- QKV: q/k/v projection of hp; q -> qb, k / v appended to the cache at pos
    for (int it = first_item(0, G); it < G_QKV; it += G) {
      bf16x8 w[1][US];
      load_w<1>(w, (const bf16_t*)L.wqkv, FNS, it, wid * US, lane);
      if (it == first_item(0, G)) ok = wg_wait(a, K_LN1, lp1 * R, flag) && ok;
      if (it == first_item(0, G)) probe(a, l, K_QKV, 0);
      f32x4 c[1][MT];
      gemv_mma<1, MT, 2>(c, w, a.hp, R, wid * US, lane);
      red_store<1, MT>(red, c);
      __syncthreads();
      for (int e = tid; e < R * 8; e += NTHR) {
        const int m = e >> 3, cl = (e & 7) * 2, col = it * 16 + cl;
        const unsigned pk = pack_bf16x2(red_sum(red, 0, m, cl) + gld<float>(L.bqkv + col),
                                        red_sum(red, 0, m, cl + 1) + gld<float>(L.bqkv + col + 1));
        if (col < FD) {
          st_sc1(a.qb + (size_t)m * FD + col, pk);
        } else {
          const int cc = col < 2 * FD ? col - FD : col - 2 * FD, h = cc >> 6, d = cc & 63;
          bf16_t* cache = col < 2 * FD ? kc : vc;
          st_sc1(cache + (((size_t)m * FH + h) * a.T + a.pos[m]) * 64 + d, pk);
        }
      }
      wg_signal(a, K_QKV);
      probe(a, l, K_QKV, 1);
    }
    // ---- SELF: attention over the cache, keys 0..pos; HP heads of one row per item (8 / HP waves per head)
    for (int it = first_item(0, G); it < n_self; it += G) {
      if (it == first_item(0, G)) ok = wg_wait(a, K_QKV, lp1 * G_QKV, flag) && ok;
      if (it == first_item(0, G)) probe(a, l, K_SELF, 0);
      const int f = it * HP + wid / (NWAVE / HP), r = f / FH, h = f - r * FH;
      const size_t off = ((size_t)r * FH + h) * a.T * 64, qo = (size_t)r * FD + h * 64;
      bf16_t* o = a.ab + qo;
      const int nk = a.pos[r] + 1;
      if (HP == 1) attend<false, NWAVE, 8>(a.qb, qo, kc, vc, off, 0, nk, o, nullptr, wpart, wml);
      else if (HP == 2) attend<false, NWAVE / 2, 8>(a.qb, qo, kc, vc, off, 0, nk, o, nullptr, wpart, wml);
      else attend<false, NWAVE / 4, 8>(a.qb, qo, kc, vc, off, 0, nk, o, nullptr, wpart, wml);
      wg_signal(a, K_SELF);
      probe(a, l, K_SELF, 1);
    }
    // ---- O: x += ab . Wo + bo (the owner of column group it)
    for (int it = first_item(0, G); it < G_D; it += G) {
      bf16x8 w[1][US];
      load_w<1>(w, (const bf16_t*)L.wo, FNS, it, wid * US, lane);
      if (it == first_item(0, G)) ok = wg_wait(a, K_SELF, lp1 * n_self, flag) && ok;
      if (it == first_item(0, G)) probe(a, l, K_O, 0);
      f32x4 c[1][MT];
      gemv_mma<1, MT, 1>(c, w, a.ab, R, wid * US, lane);
      red_store<1, MT>(red, c);
      __syncthreads();
      for (int e = tid; e < R * 8; e += NTHR) {
        const int m = e >> 3, cl = (e & 7) * 2, col = it * 16 + cl;
        const f32x2 xo = hld2(a.x, ((size_t)m * FD + col) * 4);
        st_sc1(a.x + (size_t)m * FD + col, (xo[0] + gld<float>(L.bo + col)) + red_sum(red, 0, m, cl),
               (xo[1] + gld<float>(L.bo + col + 1)) + red_sum(red, 0, m, cl + 1));
      }
      wg_signal(a, K_O);
      probe(a, l, K_O, 1);
    }
    // ---- LN2: encoder_attn_layer_norm -> hp
    for (int it = first_item(OFF_LN, G); it < R; it += G) {
      if (it == first_item(OFF_LN, G)) ok = wg_wait(a, K_O, lp1 * G_D, flag) && ok;
      if (it == first_item(OFF_LN, G)) probe(a, l, K_LN2, 0);
      if (wid == 0) ln_row(a.x, it, L.ln2_g, L.ln2_b, a.eps, a.hp, lane);
      wg_signal(a, K_LN2);
      probe(a, l, K_LN2, 1);
    }
    // ---- QX: cross-attention query of hp -> qb
    for (int it = first_item(OFF_QX, G); it < G_D; it += G) {
      bf16x8 w[1][US];
      load_w<1>(w, (const bf16_t*)L.wq_x, FNS, it, wid * US, lane);
      if (it == first_item(OFF_QX, G)) ok = wg_wait(a, K_LN2, lp1 * R, flag) && ok;
      if (it == first_item(OFF_QX, G)) probe(a, l, K_QX, 0);
      f32x4 c[1][MT];
      gemv_mma<1, MT, 2>(c, w, a.hp, R, wid * US, lane);
      red_store<1, MT>(red, c);
      __syncthreads();
      for (int e = tid; e < R * 8; e += NTHR) {
        const int m = e >> 3, cl = (e & 7) * 2, col = it * 16 + cl;
        st_sc1(a.qb + (size_t)m * FD + col, pack_bf16x2(red_sum(red, 0, m, cl) + gld<float>(L.bq_x + col),
                                                        red_sum(red, 0, m, cl + 1) + gld<float>(L.bq_x + col + 1)));
      }
      wg_signal(a, K_QX);
      probe(a, l, K_QX, 1);
    }
    // ---- CROSS: (row, head) over the encoder keys in XS key slices; a slice's unnormalised state goes to xpart. After
    //      its last slice a workgroup drains once and takes one arrival ticket per slice (a lane each); the (row,
    //      head)s its tickets complete it merges (XS states in slice order -> ab), eight at a time (32 lanes each)
    {
      const bf16_t* xk = a.xkv + (size_t)l * a.xkv_layer_stride;
      const int i0 = first_item(0, G);
      for (int it = i0; it < n_cross; it += G) {
        if (it == i0) ok = wg_wait(a, K_QX, lp1 * G_D, flag) && ok;
        if (it == i0) probe(a, l, K_CROSS, 0);
        const int rh = it / XS, z = it - rh * XS, r = rh / FH, h = rh - r * FH;
        const int k0 = (int)((long)z * a.S / XS), k1 = (int)((long)(z + 1) * a.S / XS);
        const size_t off = ((size_t)r * FH + h) * a.S * 64, qo = (size_t)r * FD + h * 64;
        if (XS == 1) {
          attend<true, NWAVE, XUNR>(a.qb, qo, xk, xk + a.xkv_v_off, off, k0, k1, a.ab + qo, nullptr, wpart, wml);
          wg_signal(a, K_CROSS);
        } else {
          attend<true, NWAVE, XUNR>(a.qb, qo, xk, xk + a.xkv_v_off, off, k0, k1, nullptr,
                                    a.xpart + ((size_t)rh * XS + z) * 66, wpart, wml);
        }
      }
      if (XS > 1 && i0 < n_cross) {
        const int nmine = (n_cross - i0 + G - 1) / G;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int done = 0;
        for (int c0 = 0; c0 < nmine; c0 += 64) {  // this workgroup's slices, 64 tickets at a time
          if (tid < 64) {
            bool last = false;
            if (c0 + tid < nmine) {
              const int rh = (i0 + (c0 + tid) * G) / XS;
              const unsigned old = __hip_atomic_fetch_add(a.sync + XTICKET_OFF + rh * TSTRIDE, 1u, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
              last = old % (unsigned)XS == (unsigned)XS - 1u;
            }
            const unsigned long long mk = __ballot(last);
            if (tid == 0) {
              flag[2] = (int)(unsigned)mk;
              flag[3] = (int)(unsigned)(mk >> 32);
              if (mk != 0ull && a.acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
          }
          __syncthreads();
          unsigned long long mk = (unsigned long long)(unsigned)flag[2] | ((unsigned long long)(unsigned)flag[3] << 32);
          done += __popcll(mk);
          for (int k = 0; mk != 0ull; ++k, mk &= mk - 1ull) {  // the completed (row, head)s, eight at a time
            if ((k & 7) != (tid >> 5)) continue;
            const int rh = (i0 + (c0 + __ffsll((long long)mk) - 1) * G) / XS, r = rh / FH, h = rh - r * FH;
            const int lt = tid & 31;
            const float* s0 = a.xpart + (size_t)rh * XS * 66;
            float M = -INFINITY;
            for (int zz = 0; zz < XS; ++zz) M = fmaxf(M, hld2(s0, (size_t)zz * 66 * 4)[0]);
            float v0 = 0.f, v1 = 0.f, tot = 0.f;
            for (int zz = 0; zz < XS; ++zz) {
              const f32x2 ml = hld2(s0, (size_t)zz * 66 * 4);
              const f32x2 vv = hld2(s0, ((size_t)zz * 66 + 2 + 2 * lt) * 4);
              const float wt = ml[0] == -INFINITY ? 0.f : __expf(ml[0] - M);
              tot += wt * ml[1];
              v0 += wt * vv[0];
              v1 += wt * vv[1];
            }
            st_sc1(a.ab + (size_t)r * FD + h * 64 + 2 * lt, pack_bf16x2(v0 / tot, v1 / tot));
          }
          __syncthreads();  // (flag words reused by the next chunk)
        }
        if (done > 0) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid == 0)
            __hip_atomic_fetch_add(ctr(a.sync, K_CROSS, blockIdx.x & 7), (unsigned)done, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (i0 < n_cross) probe(a, l, K_CROSS, 1);
    }
    // ---- OX: x += ab . Wo_x + bo_x
    for (int it = first_item(0, G); it < G_D; it += G) {
      bf16x8 w[1][US];
      load_w<1>(w, (const bf16_t*)L.wo_x, FNS, it, wid * US, lane);
      if (it == first_item(0, G)) ok = wg_wait(a, K_CROSS, lp1 * nrh, flag) && ok;
      if (it == first_item(0, G)) probe(a, l, K_OX, 0);
      f32x4 c[1][MT];
      gemv_mma<1, MT, 1>(c, w, a.ab, R, wid * US, lane);
      red_store<1, MT>(red, c);
      __syncthreads();
      for (int e = tid; e < R * 8; e += NTHR) {
        const int m = e >> 3, cl = (e & 7) * 2, col = it * 16 + cl;
        const f32x2 xo = hld2(a.x, ((size_t)m * FD + col) * 4);
        st_sc1(a.x + (size_t)m * FD + col, (xo[0] + gld<float>(L.bo_x + col)) + red_sum(red, 0, m, cl),
               (xo[1] + gld<float>(L.bo_x + col + 1)) + red_sum(red, 0, m, cl + 1));
      }
      wg_signal(a, K_OX);
      probe(a, l, K_OX, 1);
    }
    // ---- LN3: final_layer_norm -> hp
    for (int it = first_item(OFF_LN, G); it < R; it += G) {
      if (it == first_item(OFF_LN, G)) ok = wg_wait(a, K_OX, lp1 * G_D, flag) && ok;
      if (it == first_item(OFF_LN, G)) probe(a, l, K_LN3, 0);
      if (wid == 0) ln_row(a.x, it, L.ln3_g, L.ln3_b, a.eps, a.hp, lane);
      wg_signal(a, K_LN3);
      probe(a, l, K_LN3, 1);
    }
    // ---- FC1: fc1 + GELU of hp, two column groups per item -> fb (packed, K = 5120)
    for (int it = first_item(OFF_FC1, G); it < G_FP; it += G) {
      bf16x8 w[2][US];
      load_w<2>(w, (const bf16_t*)L.w1, FNS, 2 * it, wid * US, lane);
      if (it == first_item(OFF_FC1, G)) ok = wg_wait(a, K_LN3, lp1 * R, flag) && ok;
      if (it == first_item(OFF_FC1, G)) probe(a, l, K_FC1, 0);
      f32x4 c[2][MT];
      gemv_mma<2, MT, 2>(c, w, a.hp, R, wid * US, lane);
      red_store<2, MT>(red, c);
      __syncthreads();
      for (int e = tid; e < R * 16; e += NTHR) {
        const int m = e >> 4, g = (e >> 3) & 1, cl = (e & 7) * 2, col = (2 * it + g) * 16 + cl;
        const float v0 = gelu_erf(red_sum(red, g, m, cl) + gld<float>(L.b1 + col));
        const float v1 = gelu_erf(red_sum(red, g, m, cl + 1) + gld<float>(L.b1 + col + 1));
        st_sc1(a.fb + tw_pack_act_idx(m, col, FF), pack_bf16x2(v0, v1));
      }
      wg_signal(a, K_FC1);
      probe(a, l, K_FC1, 1);
    }
    // ---- FC2: column-group pair p, K-quarter q: f32 slab; the pair's last arrival adds them into x
    for (int it = first_item(0, G); it < N_FC2; it += G) {
      const int p = it >> 2, q = it & 3;
      bf16x8 w[2][US];
      load_w<2>(w, (const bf16_t*)L.w2, FNS2, 2 * p, q * FNS + wid * US, lane);
      if (it == first_item(0, G)) ok = wg_wait(a, K_FC1, lp1 * G_FP, flag) && ok;
      if (it == first_item(0, G)) probe(a, l, K_FC2, 0);
      f32x4 c[2][MT];
      gemv_mma<2, MT, 2>(c, w, a.fb, R, q * FNS + wid * US, lane);
      red_store<2, MT>(red, c);
      __syncthreads();
      float* sl = a.slab + (size_t)q * R * FD;
      for (int e = tid; e < R * 16; e += NTHR) {
        const int m = e >> 4, g = (e >> 3) & 1, cl = (e & 7) * 2, col = (2 * p + g) * 16 + cl;
        st_sc1(sl + (size_t)m * FD + col, red_sum(red, g, m, cl), red_sum(red, g, m, cl + 1));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add(a.sync + TICKET_OFF + p * TSTRIDE, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        flag[1] = (old & 3u) == 3u;
        if (flag[1] && a.acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      if (flag[1]) {  // the pair's last arrival: x = (((x + b2) + s0) + s1) + s2) + s3 over its 32 columns
        for (int e = tid; e < R * 16; e += NTHR) {
          const int m = e >> 4, col = 32 * p + (e & 15) * 2;
          f32x2 v = hld2(a.x, ((size_t)m * FD + col) * 4);
          v[0] += gld<float>(L.b2 + col);
          v[1] += gld<float>(L.b2 + col + 1);
#pragma unroll
          for (int s = 0; s < 4; ++s) v += hld2(a.slab, (((size_t)s * R + m) * FD + col) * 4);
          st_sc1(a.x + (size_t)m * FD + col, v[0], v[1]);
        }
        wg_signal(a, K_FC2);
      }
      probe(a, l, K_FC2, 1);
    }
  }
  // ---- FIN: the decoder's final layer_norm of row it -> hp (proj_out's operand, read by the next launch)
  for (int it = first_item(OFF_LN1, G); it < R; it += G) {
    if (it == first_item(OFF_LN1, G)) ok = wg_wait(a, K_FC2, (unsigned)a.n_layers * (G_D / 2), flag) && ok;
    if (it == first_item(OFF_LN1, G)) probe(a, a.n_layers, K_FIN, 0);
    if (wid == 0) ln_row(a.x, it, a.lnf_g, a.lnf_b, a.eps, a.hp, lane);
    probe(a, a.n_layers, K_FIN, 1);
  }
  (void)ok;
}

int g_fused_grid = 0;  // workgroups per launch (0: the resident maximum, g_fused_max)
int g_fused_max = 0;   // the CU count x the workgroups the occupancy query admits per CU (at most 2)

// Queries g_fused_max once. Every workgroup of a launch must be resident at the same time (static item assignment:
// a workgroup never started would leave its items undone until the waits time out), so no grid may exceed it.
int fused_max_grid() {
  if (g_fused_max > 0) return TW_OK;
  int dev = 0, cus = 0, occ1 = 0, occ2 = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
    tw_set_error("tw_dec_fused: cannot query the CU count");
    return TW_ERR_LAUNCH;
  }
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ1, k_dec_fused<1>, NTHR, 0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ2, k_dec_fused<2>, NTHR, 0) != hipSuccess ||
      min(occ1, occ2) < 1) {
    tw_set_error("tw_dec_fused: occupancy query failed (%d, %d)", occ1, occ2);
    return TW_ERR_LAUNCH;
  }
  g_fused_max = cus * min(2, min(occ1, occ2));
  return TW_OK;
}
int g_fused_acq = 0;   // FusedArgs::acq
unsigned long long* g_fused_probe = nullptr;

}  // namespace

extern "C" size_t tw_dec_fused_sync_bytes(void) { return (size_t)SYNC_WORDS * 4; }

extern "C" int tw_dec_fused_supported(int d_model, int heads, int ffn, int rows) {
  return d_model == FD && heads == FH && ffn == FF && rows >= 1 && rows <= 32 ? 1 : 0;
}

extern "C" int tw_dec_fused_set_grid(int n) {
  if (int rc = fused_max_grid()) return rc;
  TW_REQUIRE(n >= 0 && n <= g_fused_max, "tw_dec_fused_set_grid: %d workgroups (0 .. %d resident)", n, g_fused_max);
  g_fused_grid = n;
  return TW_OK;
}

extern "C" int tw_dec_fused_set_probe(void* buf) {
  g_fused_probe = (unsigned long long*)buf;
  return TW_OK;
}

extern "C" int tw_dec_fused_grid(void) { return g_fused_grid; }

extern "C" int tw_dec_fused_set_acquire(int on) {
  g_fused_acq = on ? 1 : 0;
  return TW_OK;
}

// Key slices per cross-attention (row, head): the fewest dependent load round trips on the busiest workgroup (items
// per workgroup x batches of NWAVE x 8 groups x XUNR keys per item), a slice merge charged a quarter of one.
static int cross_slices(int R, int S, int G) {
  const int n = R * FH;
  int best = 1;
  double best_cost = 1e30;
  for (int xs = 1; xs <= XS_MAX; ++xs) {
    const int keys = (S + xs - 1) / xs, trips = (keys + NWAVE * 8 * XUNR - 1) / (NWAVE * 8 * XUNR);
    const double cost = (double)((n * xs + G - 1) / G) * (trips + (xs > 1 ? 0.25 : 0.0));
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = xs;
    }
  }
  return best;
}

extern "C" size_t tw_dec_fused_xpart_bytes(int rows) { return (size_t)rows * FH * XS_MAX * 66 * sizeof(float); }

extern "C" int tw_dec_fused(const TwDecLayerW* layers, int n_layers, int R, const int* pos, float* x, uint16_t* kc,
                            uint16_t* vc, long kv_layer_stride, int max_pos, const uint16_t* xkv,
                            long xkv_layer_stride, long xkv_v_off, int S, uint16_t* qb, uint16_t* ab, uint16_t* fb,
                            float* slab, float* xpart, const float* lnf_g, const float* lnf_b, uint16_t* hp, float eps,
                            unsigned* sync, unsigned* err, void* stream) {
  TW_REQUIRE(layers && pos && x && kc && vc && xkv && qb && ab && fb && slab && xpart && lnf_g && lnf_b && hp &&
                 sync && err,
             "tw_dec_fused: null pointer");
  TW_REQUIRE(n_layers >= 1 && n_layers <= 64 && R >= 1 && R <= 32, "tw_dec_fused: n_layers %d (1..64), rows %d (1..32)",
             n_layers, R);
  TW_REQUIRE(max_pos >= 1 && S >= 1 && kv_layer_stride > 0 && xkv_layer_stride > 0 && xkv_v_off > 0,
             "tw_dec_fused: bad cache geometry");
  TW_REQUIRE(((uintptr_t)sync & 15) == 0, "tw_dec_fused: sync words not 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  if (int rc = fused_max_grid()) return rc;
  if (g_fused_grid == 0) g_fused_grid = g_fused_max;
  if (hipMemsetAsync(sync, 0, (size_t)SYNC_WORDS * 4, s) != hipSuccess) {  // (a memset node when captured)
    tw_set_error("tw_dec_fused: memset of the sync words failed");
    return TW_ERR_LAUNCH;
  }
  FusedArgs fa{layers, n_layers, R, max_pos, S, pos, x, (bf16_t*)kc, (bf16_t*)vc, kv_layer_stride, (const bf16_t*)xkv,
               xkv_layer_stride, xkv_v_off, (bf16_t*)qb, (bf16_t*)ab, (bf16_t*)fb, slab, lnf_g, lnf_b, (bf16_t*)hp,
               eps, sync, err, g_fused_acq, 1, cross_slices(R, S, g_fused_grid), xpart, g_fused_probe};
  // heads per self-attention item: 1, 2 or 4 (divisors of the 20 heads, so no item straddles a row end)
  while (fa.hp_self < 4 && R * FH / fa.hp_self > g_fused_grid) fa.hp_self *= 2;
  if (R > 16)
    hipLaunchKernelGGL(k_dec_fused<2>, dim3(g_fused_grid), dim3(NTHR), 0, s, fa);
  else
    hipLaunchKernelGGL(k_dec_fused<1>, dim3(g_fused_grid), dim3(NTHR), 0, s, fa);
  return tw_check_launch("tw_dec_fused");
}
