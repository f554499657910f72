// Fused Whisper logits processing + greedy selection, one workgroup per batch row, no host sync.
//
// Restates, for num_beams = 1, the per-step work of GenerationMixin._sample
// ($TF/generation/utils.py:2876-2941: f32 logits, processors, argmax = first max, pad after EOS,
// EOS / max_length stopping) with the Whisper processor chain in the order
// WhisperGenerationMixin._retrieve_logit_processors builds it
// ($TF/models/whisper/generation_whisper.py:1774-1812):
//   SuppressTokensAtBeginLogitsProcessor  ($TF/generation/logits_process.py:1816-1866)
//   SuppressTokensLogitsProcessor         (:1869-1906)
//   WhisperTimeStampLogitsProcessor        (:1909-2047)
// The reference loops over rows in Python with .tolist() (a device->host sync per row per step);
// here the processor state (#generated, last two tokens, last timestamp) lives in a device array and
// the masks, the timestamp log-prob rule and the argmax are evaluated in one pass over the vocab.
// Language detection (generation_whisper.py:1610-1673: argmax over the language ids of the first
// decoder step) is mode 1 of the same kernel.
#include "tw_common.h"
#include "../../include/tw_whisper.h"

struct Best {
  float v;
  int i;
};
__device__ inline Best best_of(Best a, Best b) {
  // larger value wins; ties -> smaller index (torch.argmax returns the first maximal index)
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}
__device__ inline void lse_merge(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) { m = m2; s = s2; return; }
  if (m2 > m) { s = s * __expf(m - m2) + s2; m = m2; }
  else s = s + s2 * __expf(m2 - m);
}

// lse_merge(m, s, x, 1) without branches (per logit in the beam partials): d = x - m; x above m rescales s by
// exp(m - x) = exp(-|d|) and adds 1, otherwise s gains exp(d) = exp(-|d|) — the same exp argument and the same
// arithmetic as lse_merge in every case (an -inf x adds exp(-inf) = 0; a first finite x over m = -inf gives
// s * 0 + 1), so the result is bit-identical
__device__ inline void lse_add1(float& m, float& s, float x) {
  const float d = x - m;
  const float e = (x == -INFINITY) ? 0.f : __expf(-fabsf(d));
  s = (d > 0.f) ? s * e + 1.f : s + e;
  m = fmaxf(m, x);
}

// Partial record of one vocab chunk of one row (8 words).
struct SelPart {
  float bt_v; int bt_i;   // best text (or mode-1) candidate
  float bs_v; int bs_i;   // best timestamp candidate
  float m_ts, s_ts;       // logsumexp state over the timestamp logits
  float pad0, pad1;
};

// Row-constant masks of WhisperTimeStampLogitsProcessor.__call__ for this step.
struct RowMask {
  int init_step, mask_ts_all, mask_text_lt_eos, ts_hi_block;
};
__device__ inline RowMask row_mask(const int* st, const TwSelectParams& p) {
  const int n_gen = st[TW_ST_NGEN], last = st[TW_ST_LAST], penult = st[TW_ST_PENULT], last_ts = st[TW_ST_LASTTS];
  const int tsb = p.ts_begin;
  RowMask r{n_gen == 0, 0, 0, tsb};
  if (p.mode == 0 && p.use_timestamps) {
    const bool last_was_ts = n_gen >= 1 && last >= tsb;
    const bool penult_was_ts = n_gen < 2 || penult >= tsb;
    if (last_was_ts) {
      if (penult_was_ts) r.mask_ts_all = 1;
      else r.mask_text_lt_eos = 1;
    }
    if (last_ts >= 0) r.ts_hi_block = (last_was_ts && !penult_was_ts) ? last_ts : last_ts + 1;
  }
  return r;
}

// One vocab chunk [v0, v1) of one row with a 256-thread block (4 waves): the processed (masked) logits' best text and
// best timestamp candidates and the timestamp logsumexp state, reduced to one record in `out` (valid in thread 0).
// TX: also accumulate (per thread, unreduced) the logsumexp state of the unmasked TEXT logits into m_tx / s_tx
// (k_select_full's log_softmax denominator); off, the arithmetic is k_select_partial's exactly.
template <bool TX>
__device__ inline void sel_chunk(const float* __restrict__ row, const uint32_t* __restrict__ suppress_bits,
                                 const TwSelectParams& p, const RowMask& rm, int v0, int v1, SelPart* sp,
                                 SelPart& out, float& m_tx, float& s_tx) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tsb = p.ts_begin;
  Best bt{-INFINITY, 0x7fffffff}, bs{-INFINITY, 0x7fffffff};
  float m_ts = -INFINITY, s_ts = 0.f;
  // 4 loads in flight per thread; indices clamped into the chunk (duplicates are dropped by `ok`)
  for (int base = v0 + tid; base < v1; base += 4 * 256) {
    float xs[4];
    uint32_t sb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int v = min(base + 256 * u, v1 - 1);
      xs[u] = row[v];
      sb[u] = suppress_bits ? suppress_bits[v >> 5] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int v = base + 256 * u;
      const bool ok = v < v1;
      float x = xs[u];
      bool masked;
      if (p.mode == 1) {
        masked = (v < p.lo || v >= p.hi);
      } else {
        masked = (sb[u] >> (v & 31)) & 1u;
        if (rm.init_step)
          for (int i = 0; i < p.n_begin_suppress; ++i) masked |= (v == p.begin_suppress[i]);
        if (p.use_timestamps) {
          masked |= (v == p.no_timestamps);
          if (v >= tsb) {
            masked |= rm.mask_ts_all || (v < rm.ts_hi_block);
            if (rm.init_step && p.max_initial_ts >= 0) masked |= (v > tsb + p.max_initial_ts);
          } else {
            masked |= (rm.mask_text_lt_eos && v < p.eos) || rm.init_step;
          }
        }
      }
      if (masked) x = -INFINITY;
      if (!ok) continue;
      if (v < tsb || !p.use_timestamps || p.mode == 1) {
        bt = best_of(bt, Best{x, v});
        if (TX && x != -INFINITY) lse_merge(m_tx, s_tx, x, 1.f);
      } else {
        bs = best_of(bs, Best{x, v});
        if (x != -INFINITY) lse_merge(m_ts, s_ts, x, 1.f);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Best ot{__shfl_xor(bt.v, o, 64), __shfl_xor(bt.i, o, 64)};
    Best os{__shfl_xor(bs.v, o, 64), __shfl_xor(bs.i, o, 64)};
    bt = best_of(bt, ot);
    bs = best_of(bs, os);
    float m2 = __shfl_xor(m_ts, o, 64), s2 = __shfl_xor(s_ts, o, 64);
    lse_merge(m_ts, s_ts, m2, s2);
  }
  if (lane == 0) sp[wid] = SelPart{bt.v, bt.i, bs.v, bs.i, m_ts, s_ts, 0.f, 0.f};
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w) {
      bt = best_of(bt, Best{sp[w].bt_v, sp[w].bt_i});
      bs = best_of(bs, Best{sp[w].bs_v, sp[w].bs_i});
      lse_merge(m_ts, s_ts, sp[w].m_ts, sp[w].s_ts);
    }
    out = SelPart{bt.v, bt.i, bs.v, bs.i, m_ts, s_ts, 0.f, 0.f};
  }
}

// grid (B, TW_SELECT_CHUNKS): chunk c of row b scans vocab [c*V/NC, (c+1)*V/NC) with float4 loads where aligned.
__global__ TW_DEC_LB(256, 1) void k_select_partial(const float* __restrict__ logits, int ld_logits,
                                                        const uint32_t* __restrict__ suppress_bits, TwSelectParams p,
                                                        const int* __restrict__ state, SelPart* __restrict__ ws) {
  TW_DEC_PRIO();
  __shared__ SelPart sp[4];
  const int b = blockIdx.x, c = blockIdx.y, NC = gridDim.y;
  const RowMask rm = row_mask(state + b * TW_STATE_STRIDE, p);
  const int V = p.V;
  const int v0 = (int)((long)c * V / NC), v1 = (int)((long)(c + 1) * V / NC);
  SelPart out;
  float m_tx = -INFINITY, s_tx = 0.f;
  sel_chunk<false>(logits + (size_t)b * ld_logits, suppress_bits, p, rm, v0, v1, sp, out, m_tx, s_tx);
  if (threadIdx.x == 0) ws[b * NC + c] = out;
}

// Merge of a row's chunk records (in chunk order: ties keep the first index): every lane ends with the row's best
// text / best timestamp candidates and its timestamp logsumexp state.
__device__ inline void sel_merge(const SelPart* __restrict__ ws, int NC, int b, int lane, Best& bt, Best& bs,
                                 float& m_ts, float& s_ts) {
  bt = Best{-INFINITY, 0x7fffffff};
  bs = Best{-INFINITY, 0x7fffffff};
  m_ts = -INFINITY;
  s_ts = 0.f;
  for (int c = lane; c < NC; c += 64) {
    const SelPart r = ws[b * NC + c];
    bt = best_of(bt, Best{r.bt_v, r.bt_i});
    bs = best_of(bs, Best{r.bs_v, r.bs_i});
    lse_merge(m_ts, s_ts, r.m_ts, r.s_ts);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Best ot{__shfl_xor(bt.v, o, 64), __shfl_xor(bt.i, o, 64)};
    Best os{__shfl_xor(bs.v, o, 64), __shfl_xor(bs.i, o, 64)};
    bt = best_of(bt, ot);
    bs = best_of(bs, os);
    float m2 = __shfl_xor(m_ts, o, 64), s2 = __shfl_xor(s_ts, o, 64);
    lse_merge(m_ts, s_ts, m2, s2);
  }
}
// The timestamp processor's rule ("if sum of probability over timestamps is above any other token, sample timestamp":
// the text logits are masked when the timestamps' logsumexp beats the best text logit) and the greedy choice.
__device__ inline bool sel_rule_fires(const TwSelectParams& p, Best bt, float m_ts, float s_ts) {
  if (!p.use_timestamps) return false;
  const float lse_ts = (m_ts == -INFINITY) ? -INFINITY : m_ts + __logf(s_ts);
  return lse_ts > bt.v;
}
__device__ inline int sel_greedy(const TwSelectParams& p, Best bt, Best bs, float m_ts, float s_ts) {
  if (!p.use_timestamps) return bt.i;
  return sel_rule_fires(p, bt, m_ts, s_ts) ? bs.i : best_of(bt, bs).i;
}
// _sample's pad-after-EOS / stopping rule and the processor state update for the chosen `sel`; returns the token fed
// to the next step.
__device__ inline int sel_commit(const TwSelectParams& p, int* __restrict__ st, int sel, int* __restrict__ tokens_out,
                                 int ld_tokens, int* __restrict__ next_ids, int b) {
  const int n_gen = st[TW_ST_NGEN], last = st[TW_ST_LAST];
  const int finished = st[TW_ST_FINISHED];
  const int tok = finished ? p.pad : sel;
  if (tokens_out) tokens_out[(size_t)b * ld_tokens + n_gen] = tok;
  if (next_ids) next_ids[b] = tok;
  st[TW_ST_PENULT] = last;
  st[TW_ST_LAST] = tok;
  if (tok >= p.ts_begin && p.use_timestamps) st[TW_ST_LASTTS] = tok;
  st[TW_ST_NGEN] = n_gen + 1;
  if (!finished && (tok == p.eos || n_gen + 1 >= p.max_new)) st[TW_ST_FINISHED] = 1;
  return tok;
}

// One wave per row: merge the row's chunk records, then the selection rule of the timestamp processor, the
// pad-after-EOS / stopping rule of _sample, and the processor state update. Lane 0 returns the token fed to the next
// step (tok) and the row's next position (npos).
__device__ inline void select_final_row(const SelPart* __restrict__ ws, int NC, const TwSelectParams& p,
                                        int* __restrict__ state, int* __restrict__ tokens_out, int ld_tokens,
                                        int* __restrict__ next_ids, int* __restrict__ pos, int b, int lane,
                                        int& tok_out, int& npos) {
  Best bt, bs;
  float m_ts, s_ts;
  sel_merge(ws, NC, b, lane, bt, bs, m_ts, s_ts);
  if (lane != 0) return;
  int* st = state + b * TW_STATE_STRIDE;
  npos = 0;
  if (pos) npos = pos[b] += 1;  // the next decoder step writes its K/V one position later
  if (p.mode == 1) {
    const int sel = bt.i;
    st[TW_ST_LANG] = sel;
    if (next_ids) next_ids[b] = sel;
    tok_out = sel;
    return;
  }
  tok_out = sel_commit(p, st, sel_greedy(p, bt, bs, m_ts, s_ts), tokens_out, ld_tokens, next_ids, b);
}

// grid B, one wave per row
__global__ __launch_bounds__(64) void k_select_final(const SelPart* __restrict__ ws, int NC, TwSelectParams p,
                                                     int* __restrict__ state, int* __restrict__ tokens_out,
                                                     int ld_tokens, int* __restrict__ next_ids,
                                                     int* __restrict__ pos) {
  TW_DEC_PRIO();
  int tok, npos;
  select_final_row(ws, NC, p, state, tokens_out, ld_tokens, next_ids, pos, blockIdx.x, threadIdx.x, tok, npos);
}

// k_select_final fused with the head of the NEXT decoder step (grid B, 256 threads per row): wave 0 selects the
// token, then the block embeds it at the row's next position (embed_tokens + embed_positions, f32 residual
// stream x, as k_embed_decoder) and writes the first layer's self_attn_layer_norm output (as k_resid_ln with no
// partials). Replaces three launches per generated token with one; the results are those of the three.
#define SFE_MAXV 4  // float4 chunks per thread: D <= 4096
template <bool PACKED>
__global__ TW_DEC_LB(256, 1) void k_select_final_embed(const SelPart* __restrict__ ws, int NC, TwSelectParams p,
                                                            int* __restrict__ state, int* __restrict__ tokens_out,
                                                            int ld_tokens, int* __restrict__ next_ids,
                                                            int* __restrict__ pos, const bf16_t* __restrict__ tok_emb,
                                                            const bf16_t* __restrict__ pos_emb, int D, int max_pos,
                                                            float* __restrict__ x, const float* __restrict__ g,
                                                            const float* __restrict__ bta, float eps,
                                                            bf16_t* __restrict__ out) {
  TW_DEC_PRIO();
  __shared__ float red[8];
  __shared__ int sh[2];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid < 64) {
    int tok = 0, npos = 0;
    select_final_row(ws, NC, p, state, tokens_out, ld_tokens, next_ids, pos, b, tid, tok, npos);
    if (tid == 0) {
      sh[0] = tok;
      sh[1] = min(npos, max_pos - 1);  // (past the last step: the embedding is never consumed)
    }
  }
  __syncthreads();
  const bf16_t* te = tok_emb + (size_t)sh[0] * D;
  const bf16_t* pe = pos_emb + (size_t)sh[1] * D;
  float* xr = x + (size_t)b * D;
  const int nc = D >> 2;
  float4 v[SFE_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < SFE_MAXV; ++i) {
    const int c = min(tid + 256 * i, nc - 1);
    const uint2 t = ((const uint2*)te)[c], q = ((const uint2*)pe)[c];
    float4 a;
    a.x = bf16_to_f32((bf16_t)(t.x & 0xffff)) + bf16_to_f32((bf16_t)(q.x & 0xffff));
    a.y = bf16_to_f32((bf16_t)(t.x >> 16)) + bf16_to_f32((bf16_t)(q.x >> 16));
    a.z = bf16_to_f32((bf16_t)(t.y & 0xffff)) + bf16_to_f32((bf16_t)(q.y & 0xffff));
    a.w = bf16_to_f32((bf16_t)(t.y >> 16)) + bf16_to_f32((bf16_t)(q.y >> 16));
    v[i] = a;
    if (tid + 256 * i < nc) {
      ((float4*)xr)[tid + 256 * i] = a;
      s += (a.x + a.y) + (a.z + a.w);
    }
  }
  tw_row_ln_store<PACKED>(v, s, b, D, eps, g, bta, out, red);
}

extern "C" int tw_logits_select(const float* logits, int B, int ld_logits, const uint32_t* suppress_bits,
                                const TwSelectParams* params, int* state, int* tokens_out, int ld_tokens,
                                int* next_ids, int* pos, float* workspace, void* stream) {
  TW_REQUIRE(logits && params && state && workspace && B > 0, "tw_logits_select: bad args");
  TW_REQUIRE(params->V > 0 && params->V <= ld_logits, "tw_logits_select: V=%d ld=%d", params->V, ld_logits);
  TW_REQUIRE(params->n_begin_suppress >= 0 && params->n_begin_suppress <= 8, "tw_logits_select: begin_suppress");
  static_assert(sizeof(SelPart) * TW_SELECT_CHUNKS == sizeof(float) * TW_SELECT_WS_PER_ROW, "workspace size");
  hipStream_t s = (hipStream_t)stream;
  SelPart* ws = (SelPart*)workspace;
  hipLaunchKernelGGL(k_select_partial, dim3(B, TW_SELECT_CHUNKS), dim3(256), 0, s, logits, ld_logits, suppress_bits,
                     *params, state, ws);
  hipLaunchKernelGGL(k_select_final, dim3(B), dim3(64), 0, s, ws, TW_SELECT_CHUNKS, *params, state, tokens_out,
                     ld_tokens, next_ids, pos);
  return tw_check_launch("tw_logits_select");
}

extern "C" int tw_logits_select_embed(const float* logits, int B, int ld_logits, const uint32_t* suppress_bits,
                                      const TwSelectParams* params, int* state, int* tokens_out, int ld_tokens,
                                      int* next_ids, int* pos, float* workspace, const uint16_t* tok_emb,
                                      const uint16_t* pos_emb, int D, int max_pos, float* x, const float* gamma,
                                      const float* beta, float eps, uint16_t* out, int packed, void* stream) {
  TW_REQUIRE(logits && params && state && workspace && next_ids && pos && B > 0, "tw_logits_select_embed: bad args");
  TW_REQUIRE(params->mode == 0, "tw_logits_select_embed: greedy token selection (mode 0) only");
  TW_REQUIRE(params->V > 0 && params->V <= ld_logits, "tw_logits_select_embed: V=%d ld=%d", params->V, ld_logits);
  TW_REQUIRE(params->n_begin_suppress >= 0 && params->n_begin_suppress <= 8, "tw_logits_select_embed: begin_suppress");
  TW_REQUIRE(tok_emb && pos_emb && x && gamma && beta && out && max_pos > 0, "tw_logits_select_embed: embed/LN args");
  TW_REQUIRE(D > 0 && D % 4 == 0 && D <= 1024 * SFE_MAXV && (!packed || (B <= 64 && D % 32 == 0)),
             "tw_logits_select_embed: D=%d B=%d packed=%d", D, B, packed);
  hipStream_t s = (hipStream_t)stream;
  SelPart* ws = (SelPart*)workspace;
  hipLaunchKernelGGL(k_select_partial, dim3(B, TW_SELECT_CHUNKS), dim3(256), 0, s, logits, ld_logits, suppress_bits,
                     *params, state, ws);
  if (packed)
    hipLaunchKernelGGL(k_select_final_embed<true>, dim3(B), dim3(256), 0, s, ws, TW_SELECT_CHUNKS, *params, state,
                       tokens_out, ld_tokens, next_ids, pos, tok_emb, pos_emb, D, max_pos, x, gamma, beta, eps, out);
  else
    hipLaunchKernelGGL(k_select_final_embed<false>, dim3(B), dim3(256), 0, s, ws, TW_SELECT_CHUNKS, *params, state,
                       tokens_out, ld_tokens, next_ids, pos, tok_emb, pos_emb, D, max_pos, x, gamma, beta, eps, out);
  return tw_check_launch("tw_logits_select_embed");
}

// =================================================================================================
// Temperature fallback (WhisperGenerationMixin.generate_with_fallback, $TF/models/whisper/generation_whisper.py:
// 970-1116): one workgroup per row does the whole selection of a decode step, because the fallback criteria need the
// step's log-probability and sampling needs the row's top-k.
//   * the processors and the chosen greedy token are tw_logits_select's, bit for bit: the row is scanned as the same
//     TW_SELECT_CHUNKS chunks with the same per-thread mapping (sel_chunk) and merged in the same order (sel_merge);
//   * temperature > 0 (do_sample): TemperatureLogitsWarper then TopKLogitsWarper (GenerationConfig's default top_k 50,
//     ties at the k-th value kept: logits_process.py TopKLogitsWarper) and a draw from the softmax of what is left
//     ($TF/generation/utils.py _sample: multinomial) by the Gumbel-max trick — argmax of s/T + G, G = -log(-log U) with
//     U from a counter-based hash of (seed, row key, token index in the pass, vocabulary id): the same distribution as
//     torch.multinomial, not its random stream (sampled tokens are therefore not comparable token for token);
//   * the log-probability of the chosen token under the step's scores as generate() returns them (output_scores: the
//     processed scores, after the warpers when sampling) at temperature 1 — _retrieve_avg_logprobs
//     (generation_whisper.py:1958-1975) — is added to the row's state slot TW_ST_SUMLP (f32 bits) while the row is
//     unfinished (EOS included, pads not).
// =================================================================================================
__device__ inline uint64_t tw_mix64(uint64_t z) {  // splitmix64 finaliser
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ inline float tw_gumbel(uint64_t seed, uint32_t key, uint32_t step, uint32_t v) {
  const uint64_t h = tw_mix64(seed ^ tw_mix64(((uint64_t)key << 32) ^ ((uint64_t)step << 20) ^ (uint64_t)v));
  const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1), 24 bits
  return -logf(-logf(u));
}
// the processed value of vocabulary entry v (the masks of sel_chunk, mode 0)
__device__ inline float sel_processed(const float* __restrict__ row, const uint32_t* __restrict__ suppress_bits,
                                      const TwSelectParams& p, const RowMask& rm, int v) {
  const int tsb = p.ts_begin;
  bool masked = suppress_bits ? (suppress_bits[v >> 5] >> (v & 31)) & 1u : false;
  if (rm.init_step)
    for (int i = 0; i < p.n_begin_suppress; ++i) masked |= (v == p.begin_suppress[i]);
  if (p.use_timestamps) {
    masked |= (v == p.no_timestamps);
    if (v >= tsb) {
      masked |= rm.mask_ts_all || (v < rm.ts_hi_block);
      if (rm.init_step && p.max_initial_ts >= 0) masked |= (v > tsb + p.max_initial_ts);
    } else {
      masked |= (rm.mask_text_lt_eos && v < p.eos) || rm.init_step;
    }
  }
  return masked ? -INFINITY : row[v];
}
__device__ inline float block_sum256(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}
__device__ inline void block_lse256(float& m, float& s, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lse_merge(m, s, __shfl_xor(m, o, 64), __shfl_xor(s, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[2 * (threadIdx.x >> 6)] = m;
    red[2 * (threadIdx.x >> 6) + 1] = s;
  }
  __syncthreads();
  m = red[0];
  s = red[1];
  for (int w = 1; w < 4; ++w) lse_merge(m, s, red[2 * w], red[2 * w + 1]);
}

// grid B, 256 threads (mode 0)
__global__ __launch_bounds__(256) void k_select_full(const float* __restrict__ logits, int ld_logits,
                                                     const uint32_t* __restrict__ suppress_bits, TwSelectParams p,
                                                     float temperature, int top_k, uint64_t seed,
                                                     const int* __restrict__ row_key, int* __restrict__ state,
                                                     int* __restrict__ tokens_out, int ld_tokens,
                                                     int* __restrict__ next_ids, int* __restrict__ pos) {
  __shared__ SelPart sp[4];
  __shared__ SelPart parts[TW_SELECT_CHUNKS];
  __shared__ float red[8];
  __shared__ uint32_t hist[256];
  __shared__ int bcast[4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  int* st = state + b * TW_STATE_STRIDE;
  const RowMask rm = row_mask(st, p);
  const float* row = logits + (size_t)b * ld_logits;
  const int V = p.V, NC = TW_SELECT_CHUNKS, tsb = p.ts_begin;
  float m_tx = -INFINITY, s_tx = 0.f;
  for (int c = 0; c < NC; ++c) {
    SelPart out;
    sel_chunk<true>(row, suppress_bits, p, rm, (int)((long)c * V / NC), (int)((long)(c + 1) * V / NC), sp, out, m_tx,
                    s_tx);
    if (tid == 0) parts[c] = out;
    __syncthreads();
  }
  block_lse256(m_tx, s_tx, red);  // every thread: the unmasked text logits' logsumexp state
  Best bt, bs;
  float m_ts, s_ts;
  sel_merge(parts, NC, 0, lane, bt, bs, m_ts, s_ts);  // (every wave merges the same records: identical results)
  const bool fire = sel_rule_fires(p, bt, m_ts, s_ts);
  int sel;
  float lse;  // log_softmax denominator of the scores generate() reports for this step
  if (temperature <= 0.f) {
    sel = sel_greedy(p, bt, bs, m_ts, s_ts);
    float m = fire ? -INFINITY : m_tx, sm = fire ? 0.f : s_tx;
    if (p.use_timestamps) lse_merge(m, sm, m_ts, s_ts);
    lse = m + __logf(sm);
  } else {
    // eligible: unmasked after the processors (the rule masks every text logit when it fires)
    const float invT = 1.f / temperature;
    auto elig = [&](int v, float x) { return x != -INFINITY && !(fire && v < tsb); };
    // k-th largest eligible key (f32_order_key of the value: order-preserving), MSB-first radix select
    uint32_t prefix = 0u, mask = 0u;
    int n_el = 0;
    for (int v = tid; v < V; v += 256) n_el += elig(v, sel_processed(row, suppress_bits, p, rm, v)) ? 1 : 0;
    n_el = (int)block_sum256((float)n_el, red);
    const bool restrict_k = top_k > 0 && n_el > top_k;
    if (restrict_k) {
      int k_rem = top_k;
      for (int shift = 24; shift >= 0; shift -= 8) {
        hist[tid] = 0u;
        __syncthreads();
        for (int v = tid; v < V; v += 256) {
          const float x = sel_processed(row, suppress_bits, p, rm, v);
          if (!elig(v, x)) continue;
          const uint32_t key = f32_order_key(x);
          if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid == 0) {
          int cum = 0, d = 255;
          for (; d > 0; --d) {
            if (cum + (int)hist[d] >= k_rem) break;
            cum += (int)hist[d];
          }
          bcast[0] = d;
          bcast[1] = k_rem - cum;
        }
        __syncthreads();
        prefix |= (uint32_t)bcast[0] << shift;
        mask |= 255u << shift;
        k_rem = bcast[1];
        __syncthreads();
      }
    }
    // Gumbel-max over the kept set (key >= the k-th largest), and the kept set's logsumexp (scores * T = x)
    const uint32_t rkey = row_key ? (uint32_t)row_key[b] : (uint32_t)b;
    const uint32_t step = (uint32_t)st[TW_ST_NGEN];
    Best g{-INFINITY, 0x7fffffff};
    float m = -INFINITY, sm = 0.f;
    for (int v = tid; v < V; v += 256) {
      const float x = sel_processed(row, suppress_bits, p, rm, v);
      if (!elig(v, x) || (restrict_k && f32_order_key(x) < prefix)) continue;
      lse_merge(m, sm, x, 1.f);
      g = best_of(g, Best{x * invT + tw_gumbel(seed, rkey, step, (uint32_t)v), v});
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) g = best_of(g, Best{__shfl_xor(g.v, o, 64), __shfl_xor(g.i, o, 64)});
    __syncthreads();
    if (lane == 0) {
      red[tid >> 6] = g.v;
      bcast[tid >> 6] = g.i;
    }
    __syncthreads();
    g = Best{red[0], bcast[0]};
    for (int w = 1; w < 4; ++w) g = best_of(g, Best{red[w], bcast[w]});
    sel = g.i;
    block_lse256(m, sm, red);
    lse = m + __logf(sm);
  }
  if (tid != 0) return;
  if (pos) pos[b] += 1;
  const int was_finished = st[TW_ST_FINISHED];
  const int tok = sel_commit(p, st, sel, tokens_out, ld_tokens, next_ids, b);
  if (!was_finished) {
    const float lp = row[tok] - lse;
    st[TW_ST_SUMLP] = __float_as_int(__int_as_float(st[TW_ST_SUMLP]) + lp);
  }
}

// grid B, 256 threads: softmax(raw logits)[token] into the state slot TW_ST_NOSPEECH (f32 bits)
__global__ __launch_bounds__(256) void k_token_prob(const float* __restrict__ logits, int ld_logits, int V, int token,
                                                    int* __restrict__ state) {
  __shared__ float red[8];
  const float* row = logits + (size_t)blockIdx.x * ld_logits;
  float m = -INFINITY, s = 0.f;
  for (int v = threadIdx.x; v < V; v += 256) lse_merge(m, s, row[v], 1.f);
  block_lse256(m, s, red);
  if (threadIdx.x == 0)
    state[blockIdx.x * TW_STATE_STRIDE + TW_ST_NOSPEECH] = __float_as_int(__expf(row[token] - (m + __logf(s))));
}

extern "C" int tw_logits_sample(const float* logits, int B, int ld_logits, const uint32_t* suppress_bits,
                                const TwSelectParams* params, float temperature, int top_k, uint64_t seed,
                                const int* row_key, int* state, int* tokens_out, int ld_tokens, int* next_ids,
                                int* pos, void* stream) {
  TW_REQUIRE(logits && params && state && B > 0, "tw_logits_sample: bad args");
  TW_REQUIRE(params->mode == 0, "tw_logits_sample: generation steps (mode 0) only");
  TW_REQUIRE(params->V > 0 && params->V <= ld_logits, "tw_logits_sample: V=%d ld=%d", params->V, ld_logits);
  TW_REQUIRE(params->n_begin_suppress >= 0 && params->n_begin_suppress <= 8, "tw_logits_sample: begin_suppress");
  TW_REQUIRE(temperature >= 0.f && temperature == temperature, "tw_logits_sample: temperature %f", temperature);
  hipLaunchKernelGGL(k_select_full, dim3(B), dim3(256), 0, (hipStream_t)stream, logits, ld_logits, suppress_bits,
                     *params, temperature, top_k, seed, row_key, state, tokens_out, ld_tokens, next_ids, pos);
  return tw_check_launch("tw_logits_sample");
}

extern "C" int tw_token_prob(const float* logits, int B, int ld_logits, int V, int token, int* state, void* stream) {
  TW_REQUIRE(logits && state && B > 0 && V > 0 && V <= ld_logits && token >= 0 && token < V,
             "tw_token_prob: B=%d V=%d token=%d", B, V, token);
  hipLaunchKernelGGL(k_token_prob, dim3(B), dim3(256), 0, (hipStream_t)stream, logits, ld_logits, V, token, state);
  return tw_check_launch("tw_token_prob");
}

// =================================================================================================
// Beam search (num_beams > 1): GenerationMixin._beam_search ($TF/generation/utils.py:3208-3512) with the same Whisper
// processor chain, early_stopping=False, one EOS id. Rows are window-major: row = w * nb + j.
//   k_beam_partial  grid (R, NC): per vocab chunk of a row, the log-sum-exp of the raw logits (log_softmax), the
//                   timestamp-rule statistics of k_select_partial, and the top-K masked text and timestamp
//                   candidates (K = 2 nb continuations per window, :3277-3282)
//   k_beam_step     grid W: per window, the row candidates (the timestamp rule removes the text ones when it fires),
//                   the window's top-K by accumulated log-prob (:3316-3349), running beams for the next step
//                   (:3131-3151), finished beams (:3153-3206), the early-stop heuristic (:3008-3073); then it
//                   reorders the running token histories, the processor state, ids/pos, and writes the row each
//                   new running beam continues (for the self-attention K/V reorder, tw_kv_reorder)
// =================================================================================================
struct Cand {
  float v;
  int i;
};
// (bitwise, not short-circuit: the || / && form compiled to exec-mask branches around every compare, which set the
// beam kernels' time)
__device__ inline bool cand_better(float v, int i, const Cand& c) { return (v > c.v) | ((v == c.v) & (i < c.i)); }

// Sorted insert as a compare-swap chain: every index is static, so the list stays in VGPRs (the shifting form with
// an early return was lowered to scratch: 80-272 B/lane, k_beam_partial 139 us per step at 60 rows).
template <int K>
__device__ inline void cand_insert(Cand (&L)[K], float v, int i) {
  if (!cand_better(v, i, L[K - 1])) return;
  Cand c{v, i};
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const bool better = cand_better(c.v, c.i, L[j]);
    const Cand o = L[j];
    L[j] = better ? c : o;
    c = better ? o : c;
  }
}

// The wave's best (v, i, l) under the strict order "v higher, then i lower, then lane l lower", in every lane. DPP
// within each 16-lane row (quad xor 1, xor 2, half-row mirror, row mirror: every lane of a row meets every other),
// then the four rows' winners by readlane: ~4x shorter than a 6-level ds_bpermute butterfly (__shfl_xor), whose
// latency chain set most of the beam kernels' time (K dependent rounds per list; k_beam_step 22 of 34 us). The order
// is total, so the winner (and every later round) is the one the butterfly found.
__device__ inline void wave_best(float& bv, int& bi, int& bl) {
  auto step = [&](auto ctrl_tag) {
    constexpr int ctrl = decltype(ctrl_tag)::value;
    const float ov = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(bv), ctrl, 0xF, 0xF, false));
    const int oi = __builtin_amdgcn_update_dpp(0, bi, ctrl, 0xF, 0xF, false);
    const int ol = __builtin_amdgcn_update_dpp(0, bl, ctrl, 0xF, 0xF, false);
    const bool b = (ov > bv) | ((ov == bv) & ((oi < bi) | ((oi == bi) & (ol < bl))));
    bv = b ? ov : bv;
    bi = b ? oi : bi;
    bl = b ? ol : bl;
  };
  step(std::integral_constant<int, 0xB1>{});   // quad_perm [1, 0, 3, 2]
  step(std::integral_constant<int, 0x4E>{});   // quad_perm [2, 3, 0, 1]
  step(std::integral_constant<int, 0x141>{});  // row_half_mirror
  step(std::integral_constant<int, 0x140>{});  // row_mirror
  float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bv), 0));
  int i = __builtin_amdgcn_readlane(bi, 0), l = __builtin_amdgcn_readlane(bl, 0);
#pragma unroll
  for (int r = 16; r < 64; r += 16) {
    const float ov = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bv), r));
    const int oi = __builtin_amdgcn_readlane(bi, r), ol = __builtin_amdgcn_readlane(bl, r);
    const bool b = (ov > v) | ((ov == v) & ((oi < i) | ((oi == i) & (ol < l))));
    v = b ? ov : v;
    i = b ? oi : i;
    l = b ? ol : l;
  }
  bv = v;
  bi = i;
  bl = l;
}

// K rounds of wave argmax over the lanes' sorted lists: out (LDS, K entries) = the wave's top-K, descending.
template <int K>
__device__ inline void wave_topk(Cand (&L)[K], Cand* out, int lane) {
  for (int r = 0; r < K; ++r) {
    float bv = L[0].v;
    int bi = L[0].i, bl = lane;
    wave_best(bv, bi, bl);
    if (lane == 0) out[r] = Cand{bv, bi};
    const bool pop = lane == bl;  // pop the head (selects, not a branch around register moves)
#pragma unroll
    for (int j = 0; j < K - 1; ++j) L[j] = pop ? L[j + 1] : L[j];
    L[K - 1] = pop ? Cand{-INFINITY, 0x7fffffff} : L[K - 1];
  }
}

template <int K>
struct BeamPart {
  Cand t[K];  // top-K masked text candidates (logit value)
  Cand s[K];  // top-K masked timestamp candidates
  float m_all, s_all, m_ts, s_ts;
  float m_tx, s_tx;  // (renorm) log-sum-exp of the allowed text tokens
};

// -DTW_BEAM_PROBE (measurement builds only, never the product library): per-phase timestamps of block 0 of the two
// beam kernels (100 MHz s_memrealtime, thread 0), read back with tw_beam_probe_read
#ifdef TW_BEAM_PROBE
__device__ unsigned long long tw_beam_probe_ts[2][16];
#define BPROBE(k, slot) \
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) tw_beam_probe_ts[k][slot] = __builtin_amdgcn_s_memrealtime()
extern "C" int tw_beam_probe_read(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(tw_beam_probe_ts), sizeof(tw_beam_probe_ts)) == hipSuccess ? 0 : 1;
}
#else
#define BPROBE(k, slot)
#endif

template <int K>
__global__ __launch_bounds__(256) void k_beam_partial(const float* __restrict__ logits, int ld_logits,
                                                      const uint32_t* __restrict__ suppress_bits, TwSelectParams p,
                                                      const int* __restrict__ state, BeamPart<K>* __restrict__ ws,
                                                      int renorm) {
  TW_DEC_PRIO();
  BPROBE(0, 0);
  __shared__ Cand wl[2][4][K];
  __shared__ float wst[4][6];
  const int b = blockIdx.x, c = blockIdx.y, NC = gridDim.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const RowMask rm = row_mask(state + b * TW_STATE_STRIDE, p);
  const float* row = logits + (size_t)b * ld_logits;
  const int V = p.V, tsb = p.ts_begin;
  // with timestamps the last chunk is exactly the timestamp tokens and the others split the text tokens, so no block
  // holds both kinds: each reduces one candidate list (the block holding both set the launch's duration)
  const bool split_ts = p.use_timestamps && tsb > 0 && tsb < V && NC > 1;
  const int v0 = split_ts ? (c == NC - 1 ? tsb : (int)((long)c * tsb / (NC - 1))) : (int)((long)c * V / NC);
  const int v1 = split_ts ? (c == NC - 1 ? V : (int)((long)(c + 1) * tsb / (NC - 1))) : (int)((long)(c + 1) * V / NC);
  Cand T[K], S[K];
#pragma unroll
  for (int j = 0; j < K; ++j) T[j] = S[j] = Cand{-INFINITY, 0x7fffffff};
  float m_all = -INFINITY, s_all = 0.f, m_ts = -INFINITY, s_ts = 0.f, m_tx = -INFINITY, s_tx = 0.f;
  auto visit = [&](int v, float x, uint32_t sbw) {
    lse_add1(m_all, s_all, x);
    bool masked = (sbw >> (v & 31)) & 1u;
    if (rm.init_step)
      for (int i = 0; i < p.n_begin_suppress; ++i) masked |= (v == p.begin_suppress[i]);
    if (p.use_timestamps) {
      masked |= (v == p.no_timestamps);
      if (v >= tsb) {
        masked |= rm.mask_ts_all || (v < rm.ts_hi_block);
        if (rm.init_step && p.max_initial_ts >= 0) masked |= (v > tsb + p.max_initial_ts);
      } else {
        masked |= (rm.mask_text_lt_eos && v < p.eos) || rm.init_step;
      }
    }
    if (masked) return;
    if (v < tsb || !p.use_timestamps) {
      cand_insert<K>(T, x, v);
      if (renorm) lse_add1(m_tx, s_tx, x);
    } else {
      cand_insert<K>(S, x, v);
      lse_add1(m_ts, s_ts, x);
    }
  };
  // every logit (and suppress word) of this thread's share in flight at once: one load per loop trip serialised ~13
  // memory round trips (57 us per launch at 60 rows); a share past BP_MAXE per thread (V > 65536) takes the tail loop
  constexpr int BP_MAXE = 16;
  float xs[BP_MAXE];
  uint32_t sb[BP_MAXE];
#pragma unroll
  for (int u = 0; u < BP_MAXE; ++u) {
    const int v = min(v0 + tid + 256 * u, v1 - 1);
    xs[u] = row[v];
    sb[u] = suppress_bits ? suppress_bits[v >> 5] : 0u;
  }
#pragma unroll
  for (int u = 0; u < BP_MAXE; ++u) {
    const int v = v0 + tid + 256 * u;
    if (v < v1) visit(v, xs[u], sb[u]);
  }
  for (int v = v0 + tid + 256 * BP_MAXE; v < v1; v += 256) visit(v, row[v], suppress_bits ? suppress_bits[v >> 5] : 0u);
  BPROBE(0, 1);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float m2 = __shfl_xor(m_all, o, 64), s2 = __shfl_xor(s_all, o, 64);
    lse_merge(m_all, s_all, m2, s2);
    m2 = __shfl_xor(m_ts, o, 64);
    s2 = __shfl_xor(s_ts, o, 64);
    lse_merge(m_ts, s_ts, m2, s2);
    if (renorm) {
      m2 = __shfl_xor(m_tx, o, 64);
      s2 = __shfl_xor(s_tx, o, 64);
      lse_merge(m_tx, s_tx, m2, s2);
    }
  }
  // a chunk wholly below the timestamps has no timestamp candidate (14 of the 16 chunks at large-v3 sizes), one
  // wholly inside them no text candidate: that list's K dependent argmax rounds (here and in the merge below) are
  // skipped, uniformly per block (each round is a 6-level shuffle chain: the reductions were ~20 us of 55)
  const bool any_ts = p.use_timestamps && v1 > tsb, any_tx = !p.use_timestamps || v0 < tsb;
  BPROBE(0, 2);
  if (any_tx) wave_topk<K>(T, wl[0][wid], lane);
  if (any_ts) wave_topk<K>(S, wl[1][wid], lane);
  BPROBE(0, 3);
  if (lane == 0) {
    wst[wid][0] = m_all;
    wst[wid][1] = s_all;
    wst[wid][2] = m_ts;
    wst[wid][3] = s_ts;
    wst[wid][4] = m_tx;
    wst[wid][5] = s_tx;
  }
  __syncthreads();
  if (wid != 0) return;
  BeamPart<K>* out = ws + (size_t)b * NC + c;
  for (int l = 0; l < 2; ++l) {  // merge the 4 wave lists: lane q holds entry q (4K <= 64), K rounds of argmax
    if (!(l == 0 ? any_tx : any_ts)) {  // an empty list
      if (lane < K) {
        if (l == 0) out->t[lane] = Cand{-INFINITY, 0x7fffffff};
        else out->s[lane] = Cand{-INFINITY, 0x7fffffff};
      }
      continue;
    }
    // the block's top-K of the 4 waves' lists by rank (each of the 4K entries counts the entries ahead of it under
    // the rounds' order, position breaking ties): one pass over 4K LDS broadcasts instead of K argmax rounds
    if (lane < 4 * K) {
      const Cand* all = &wl[l][0][0];
      const Cand mine = all[lane];
      int rank = 0;
      for (int e = 0; e < 4 * K; ++e) {
        const Cand o = all[e];
        rank += (o.v > mine.v) | ((o.v == mine.v) & ((o.i < mine.i) | ((o.i == mine.i) & (e < lane))));
      }
      if (rank < K) {
        if (l == 0) out->t[rank] = mine;
        else out->s[rank] = mine;
      }
    }
  }
  if (lane == 0) {
    float ma = wst[0][0], sa = wst[0][1], mt = wst[0][2], st2 = wst[0][3], mx = wst[0][4], sx = wst[0][5];
    for (int w = 1; w < 4; ++w) {
      lse_merge(ma, sa, wst[w][0], wst[w][1]);
      lse_merge(mt, st2, wst[w][2], wst[w][3]);
      lse_merge(mx, sx, wst[w][4], wst[w][5]);
    }
    out->m_all = ma;
    out->s_all = sa;
    out->m_ts = mt;
    out->s_ts = st2;
    out->m_tx = mx;
    out->s_tx = sx;
  }
  BPROBE(0, 4);
}

#define TW_BEAM_MAXNB 8
#define TW_BEAM_MAXT 448

template <int K>
__global__ __launch_bounds__(512) void k_beam_step(const BeamPart<K>* __restrict__ ws, int NC, TwSelectParams p,
                                                   TwBeamParams bp, TwBeamState bs, int* __restrict__ state,
                                                   int* __restrict__ tokens, int* __restrict__ ids,
                                                   int* __restrict__ pos) {
  TW_DEC_PRIO();
  BPROBE(1, 0);
  __shared__ Cand rc[TW_BEAM_MAXNB][K];  // row candidates: accumulated log-prob, token
  __shared__ int old_tok[TW_BEAM_MAXNB][TW_BEAM_MAXT];
  __shared__ int old_fin[TW_BEAM_MAXNB][TW_BEAM_MAXT];
  __shared__ int old_st[TW_BEAM_MAXNB][TW_STATE_STRIDE];
  __shared__ int old_tab[TW_BEAM_MAXNB][TW_BEAM_MAXT];  // the K/V position table rows (bs.kv_tab)
  __shared__ int old_ftab[TW_BEAM_MAXNB][TW_BEAM_MAXT];  // the finished hypotheses' tables (bs.fin_tab)
  __shared__ int old_pos[TW_BEAM_MAXNB];
  __shared__ int old_flen[TW_BEAM_MAXNB];
  __shared__ int s_src[TW_BEAM_MAXNB], s_tok[TW_BEAM_MAXNB], f_from[TW_BEAM_MAXNB], f_flag[TW_BEAM_MAXNB];
  __shared__ float s_score[TW_BEAM_MAXNB], f_score[TW_BEAM_MAXNB];
  // (bs.run_lp: every candidate's running sum of log-probabilities renormalised over the allowed tokens — what
  // _retrieve_avg_logprobs takes from the processed beam scores — carried beside the beam scores)
  __shared__ float rc_lp[TW_BEAM_MAXNB][K], c_lp[2 * K], s_lp[TW_BEAM_MAXNB], f_lp[TW_BEAM_MAXNB];
  __shared__ int c_beam[2 * K], c_tok[2 * K];
  // per-row sorted lists and the one-thread bookkeeping arrays live in LDS: as per-thread arrays with runtime
  // indices they were lowered to scratch (224-768 B/lane) and the serial section ran at scratch latency
  __shared__ Cand tops[TW_BEAM_MAXNB][2][K];
  __shared__ float csc[2 * K], rsc[2 * K], merged[TW_BEAM_MAXNB + 2 * K];
  __shared__ bool hits[2 * K];
  const int w = blockIdx.x, nb = bp.num_beams, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ldt = bp.ld_tokens;
  const bool lpt = bs.run_lp != nullptr && bs.fin_lp != nullptr;
  int* win = bs.win + 4 * w;
  const int t = win[2];
  const float NEG = -1.0e9f;
  // the window's running and finished histories and processor states, loaded now so their latency hides behind
  // step 1 (as a load-then-LDS-store loop after it, each trip waited for its own loads); positions past a history's
  // length are staged too (any value: they are never read back)
  constexpr int STG = (TW_BEAM_MAXNB * TW_BEAM_MAXT + 511) / 512;
  int rt[STG], rf[STG], rk[STG], rft[STG];
  const bool tab = bs.kv_tab != nullptr;
  const bool ftab = tab && bs.fin_tab != nullptr;
#pragma unroll
  for (int u = 0; u < STG; ++u) {
    const int e = tid + 512 * u, j = e / TW_BEAM_MAXT, q = e % TW_BEAM_MAXT;
    const bool ok = j < nb && q < ldt;
    const size_t off = (size_t)(w * nb + (ok ? j : 0)) * ldt + (ok ? q : 0);
    rt[u] = ok ? tokens[off] : 0;
    rf[u] = ok ? bs.fin_tokens[off] : 0;
    rk[u] = ok && tab ? bs.kv_tab[off] : 0;
    rft[u] = ok && ftab ? bs.fin_tab[off] : 0;
  }
  const int st_v = tid < nb * TW_STATE_STRIDE ? state[(w * nb) * TW_STATE_STRIDE + tid] : 0;
  const int fl_v = tid < nb ? bs.fin_len[w * nb + tid] : 0;
  const int ps_v = tid < nb ? pos[w * nb + tid] : 0;
  BPROBE(1, 1);

  // 1. per row (one wave each): merge the chunk records, apply the timestamp rule, score the candidates
  if (wid < nb) {
    const int row = w * nb + wid;
    const BeamPart<K>* parts = ws + (size_t)row * NC;
    float m_all = -INFINITY, s_all = 0.f, m_ts = -INFINITY, s_ts = 0.f, m_tx = -INFINITY, s_tx = 0.f;
    for (int c = lane; c < NC; c += 64) {
      lse_merge(m_all, s_all, parts[c].m_all, parts[c].s_all);
      lse_merge(m_ts, s_ts, parts[c].m_ts, parts[c].s_ts);
      if (lpt) lse_merge(m_tx, s_tx, parts[c].m_tx, parts[c].s_tx);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float m2 = __shfl_xor(m_all, o, 64), s2 = __shfl_xor(s_all, o, 64);
      lse_merge(m_all, s_all, m2, s2);
      m2 = __shfl_xor(m_ts, o, 64);
      s2 = __shfl_xor(s_ts, o, 64);
      lse_merge(m_ts, s_ts, m2, s2);
      if (lpt) {
        m2 = __shfl_xor(m_tx, o, 64);
        s2 = __shfl_xor(s_tx, o, 64);
        lse_merge(m_tx, s_tx, m2, s2);
      }
    }
    BPROBE(1, 8);
    // top-K of the text list and of the timestamp list over the NC chunk lists (<= 4 entries per lane). With the
    // timestamp split of k_beam_partial every timestamp candidate sits in the last chunk's (sorted) list and every
    // other chunk's list is empty: that list is the merge's result as it stands
    Cand(*top)[K] = tops[wid];
    const bool split_ts = p.use_timestamps && p.ts_begin > 0 && p.ts_begin < p.V && NC > 1;
    if (split_ts && lane < K) top[1][lane] = parts[NC - 1].s[lane];
    for (int l = 0; l < (split_ts ? 1 : 2); ++l) {
      Cand mine[4];
      bool used[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = lane + 64 * q;
        mine[q] = e < NC * K ? (l == 0 ? parts[e / K].t[e % K] : parts[e / K].s[e % K]) : Cand{-INFINITY, 0x7fffffff};
        used[q] = false;
      }
      for (int r = 0; r < K; ++r) {
        float bv = -INFINITY;
        int bi = 0x7fffffff, bq = -1;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool b = !used[q] & cand_better(mine[q].v, mine[q].i, Cand{bv, bi});
          bv = b ? mine[q].v : bv;
          bi = b ? mine[q].i : bi;
          bq = b ? q : bq;
        }
        int bl = lane;
        wave_best(bv, bi, bl);
#pragma unroll
        for (int q = 0; q < 4; ++q) used[q] = used[q] || (lane == bl && bq == q);
        if (lane == 0) top[l][r] = Cand{bv, bi};
      }
      BPROBE(1, 9 + l);
    }
    if (lane == 0) {  // lane 0 wrote top
      const float lse_all = m_all + __logf(s_all);
      const float lse_ts = (m_ts == -INFINITY) ? -INFINITY : m_ts + __logf(s_ts);
      // WhisperTimeStampLogitsProcessor: timestamp mass above every text token -> text tokens -inf
      const bool fires = p.use_timestamps && lse_ts > top[0][0].v;
      const float run = bs.run_score[row];
      // the allowed set log_softmax renormalises over: the allowed timestamps alone when the rule fires
      float lse_ok = 0.f, run_lp = 0.f;
      if (lpt) {
        const float lse_tx = (m_tx == -INFINITY) ? -INFINITY : m_tx + __logf(s_tx);
        lse_ok = fires ? lse_ts : (lse_tx == -INFINITY ? lse_ts : lse_ts == -INFINITY ? lse_tx
                                   : fmaxf(lse_tx, lse_ts) + log1pf(__expf(-fabsf(lse_tx - lse_ts))));
        run_lp = bs.run_lp[row];
      }
      int a = 0, bb = 0;
      for (int k = 0; k < K; ++k) {
        Cand pick;
        if (fires) {
          pick = top[1][bb++];
        } else if (cand_better(top[0][a].v, top[0][a].i, top[1][bb])) {
          pick = top[0][a++];
        } else {
          pick = top[1][bb++];
        }
        rc[wid][k] = Cand{pick.v == -INFINITY ? -INFINITY : run + (pick.v - lse_all), pick.i};
        if (lpt) rc_lp[wid][k] = pick.v == -INFINITY ? -INFINITY : run_lp + (pick.v - lse_ok);
      }
    }
  }
  BPROBE(1, 11);
  // stage the old running histories, finished histories and processor states of the window
#pragma unroll
  for (int u = 0; u < STG; ++u) {
    const int e = tid + 512 * u, j = e / TW_BEAM_MAXT, q = e % TW_BEAM_MAXT;
    if (j < nb) {
      old_tok[j][q] = rt[u];
      old_fin[j][q] = rf[u];
      old_tab[j][q] = rk[u];
      old_ftab[j][q] = rft[u];
    }
  }
  if (tid < nb * TW_STATE_STRIDE) old_st[tid / TW_STATE_STRIDE][tid % TW_STATE_STRIDE] = st_v;
  if (tid < nb) {
    old_flen[tid] = fl_v;
    old_pos[tid] = ps_v;
  }
  BPROBE(1, 2);
  __syncthreads();
  BPROBE(1, 3);

  // 2. the window's beam bookkeeping. Each selection below is a stable top-n; it is computed as ranks, every
  // candidate counting the candidates ahead of it (LDS broadcast reads), instead of n sequential argmax rounds in
  // one thread (that serial section was ~25 of the kernel's 52 us at 12 windows x 5 beams).
  // a. top-K over all beams' candidates by accumulated log-prob; ties -> lower flat index beam * V + token (rows
  //    hold distinct tokens; a row's repeated empty entries keep their list order)
  if (tid < nb * K) {
    const int j = tid / K, k = tid - j * K;
    const float v = rc[j][k].v;
    const long f = (long)j * p.V + rc[j][k].i;
    int rank = 0;
    for (int e = 0; e < nb * K; ++e) {
      const int j2 = e / K, k2 = e - j2 * K;
      const float v2 = rc[j2][k2].v;
      const long f2 = (long)j2 * p.V + rc[j2][k2].i;
      rank += (v2 > v) | ((v2 == v) & ((f2 < f) | ((f2 == f) & (e < tid))));  // (bitwise: no branches)
    }
    if (rank < K) {
      c_beam[rank] = j;
      c_tok[rank] = rc[j][k].i;
      csc[rank] = v;
      if (lpt) c_lp[rank] = rc_lp[j][k];
    }
  }
  __syncthreads();
  BPROBE(1, 4);
  const int unsat_prev = win[0];
  const float lp_div = __powf((float)(t + 1), bp.length_penalty);
  if (tid < K) {
    const int c = tid;
    hits[c] = c_tok[c] == p.eos || t + 1 >= bp.max_new;
    rsc[c] = csc[c] + (hits[c] ? NEG : 0.f);
  }
  // f. the finished candidates: previous best nb, then the just-finished top-nb continuations
  if (tid < nb + K) {
    const int e = tid;
    if (e < nb) {
      merged[e] = bs.fin_score[w * nb + e];
    } else {
      const int c = e - nb;
      float v = csc[c] / lp_div;
      if (!unsat_prev) v += NEG;
      const bool just = (c_tok[c] == p.eos || t + 1 >= bp.max_new) && c < nb;
      if (!just) v += NEG;
      merged[e] = v;
    }
  }
  __syncthreads();
  // e. running beams for the next step: best nb of the continuations by rsc (ties -> lower c)
  if (tid < K) {
    const int c = tid;
    int rank = 0;
    for (int c2 = 0; c2 < K; ++c2) rank += (rsc[c2] > rsc[c]) | ((rsc[c2] == rsc[c]) & (c2 < c));
    if (rank < nb) {
      s_src[rank] = c_beam[c];
      s_tok[rank] = c_tok[c];
      s_score[rank] = rsc[c];
      if (lpt) s_lp[rank] = c_lp[c];
    }
  }
  // f. finished beams: best nb of the nb + K merged scores (ties -> lower e)
  if (tid >= 64 && tid < 64 + nb + K) {
    const int e = tid - 64;
    int rank = 0;
    for (int e2 = 0; e2 < nb + K; ++e2) rank += (merged[e2] > merged[e]) | ((merged[e2] == merged[e]) & (e2 < e));
    if (rank < nb) {
      f_from[rank] = e;
      f_score[rank] = merged[e];
      f_flag[rank] = e < nb ? bs.fin_flag[w * nb + e] : (hits[e - nb] && e - nb < nb);
      if (lpt) f_lp[rank] = e < nb ? bs.fin_lp[w * nb + e] : c_lp[e - nb];
    }
  }
  __syncthreads();
  // g. early-stop heuristic (early_stopping=False: best running score at the current length)
  if (tid == 0) {
    bool all_hit = true;
    for (int c = 0; c < K; ++c) all_hit = all_hit && hits[c];
    float min_fin = INFINITY;
    for (int q = 0; q < nb; ++q) min_fin = fminf(min_fin, f_score[q]);
    const float best_possible = s_score[0] / __powf((float)(t + 1), bp.length_penalty);
    bool any_better = false;
    for (int q = 0; q < nb; ++q) any_better = any_better || best_possible > (f_flag[q] ? min_fin : NEG);
    const int unsat = unsat_prev && any_better;
    win[0] = unsat;
    win[1] = (!unsat || all_hit) ? 1 : 0;
    win[2] = t + 1;
  }
  __syncthreads();
  BPROBE(1, 5);

  // 3. apply: running histories, state, ids, pos, the K/V source rows; finished histories
  for (int e = tid; e < nb * (t + 1); e += blockDim.x) {
    const int j = e / (t + 1), q = e % (t + 1);
    tokens[(size_t)(w * nb + j) * ldt + q] = q < t ? old_tok[s_src[j]][q] : s_tok[j];
  }
  // K/V position table: the new beam j reads its source's history, positions [0, pos + 1) (this step's position
  // included: the source wrote it); later positions keep j's own row (kv_tab[r][*] = r from the pass start)
  if (tab) {
    for (int e = tid; e < nb * TW_BEAM_MAXT; e += blockDim.x) {
      const int j = e / TW_BEAM_MAXT, q = e % TW_BEAM_MAXT;
      if (q <= old_pos[j] && q < ldt && s_src[j] != j) bs.kv_tab[(size_t)(w * nb + j) * ldt + q] = old_tab[s_src[j]][q];
    }
  }
  for (int e = tid; e < nb * TW_BEAM_MAXT; e += blockDim.x) {
    const int qs = e / TW_BEAM_MAXT, q = e % TW_BEAM_MAXT;
    const int from = f_from[qs];
    int len, v;
    if (from < nb) {
      len = old_flen[from];
      v = q < len ? old_fin[from][q] : 0;
    } else {
      const int c = from - nb;
      len = t + 1;
      v = q < t ? old_tok[c_beam[c]][q] : c_tok[c];
    }
    if (q < len) bs.fin_tokens[(size_t)(w * nb + qs) * ldt + q] = v;
    // the rows that fed the history's positions: a kept slot's own table, or (just finished) its source beam's
    // table up to the position the source fed this step
    if (ftab && q < ldt) {
      int r;
      if (from < nb) {
        r = old_ftab[from][q];
      } else {
        const int src = c_beam[from - nb];
        r = q <= old_pos[src] ? old_tab[src][q] : 0;
      }
      bs.fin_tab[(size_t)(w * nb + qs) * ldt + q] = r;
    }
  }
  if (tid < nb) {
    const int j = tid, row = w * nb + j, src = s_src[j], tok = s_tok[j];
    int* st = state + row * TW_STATE_STRIDE;
    st[TW_ST_NGEN] = t + 1;
    st[TW_ST_PENULT] = old_st[src][TW_ST_LAST];
    st[TW_ST_LAST] = tok;
    st[TW_ST_LASTTS] = (p.use_timestamps && tok >= p.ts_begin) ? tok : old_st[src][TW_ST_LASTTS];
    st[TW_ST_FINISHED] = 0;
    ids[row] = tok;
    pos[row] += 1;
    bs.src_rows[row] = w * nb + src;
    bs.run_score[row] = s_score[j];
    const int from = f_from[j];
    bs.fin_score[row] = f_score[j];
    bs.fin_flag[row] = f_flag[j];
    bs.fin_len[row] = from < nb ? old_flen[from] : t + 1;
    if (lpt) {
      bs.run_lp[row] = s_lp[j];
      bs.fin_lp[row] = f_lp[j];
    }
  }
  BPROBE(1, 6);
}

template <int K>
static int launch_beam(const float* logits, int W, int ld_logits, const uint32_t* suppress_bits,
                       const TwSelectParams* p, const TwBeamParams* bp, TwBeamState bs, int* state, int* tokens,
                       int* ids, int* pos, void* workspace, hipStream_t s) {
  const int R = W * bp->num_beams;
  BeamPart<K>* ws = (BeamPart<K>*)workspace;
  hipLaunchKernelGGL(k_beam_partial<K>, dim3(R, TW_SELECT_CHUNKS), dim3(256), 0, s, logits, ld_logits, suppress_bits,
                     *p, state, ws, (int)(bs.run_lp != nullptr && bs.fin_lp != nullptr));
  hipLaunchKernelGGL(k_beam_step<K>, dim3(W), dim3(512), 0, s, ws, TW_SELECT_CHUNKS, *p, *bp, bs, state, tokens, ids,
                     pos);
  return tw_check_launch("tw_beam_step");
}

extern "C" size_t tw_beam_workspace_bytes(int rows) {
  return (size_t)rows * TW_SELECT_CHUNKS * sizeof(BeamPart<2 * TW_BEAM_MAXNB>);
}

extern "C" int tw_beam_step(const float* logits, int W, int ld_logits, const uint32_t* suppress_bits,
                            const TwSelectParams* params, const TwBeamParams* bp, const TwBeamState* bs, int* state,
                            int* tokens, int* ids, int* pos, void* workspace, void* stream) {
  TW_REQUIRE(logits && params && bp && bs && state && tokens && ids && pos && workspace && W > 0,
             "tw_beam_step: null argument");
  TW_REQUIRE(bp->num_beams >= 2 && bp->num_beams <= TW_BEAM_MAXNB, "tw_beam_step: num_beams=%d (2..%d)",
             bp->num_beams, TW_BEAM_MAXNB);
  TW_REQUIRE(bp->ld_tokens <= TW_BEAM_MAXT && bp->max_new >= 1 && bp->max_new <= bp->ld_tokens,
             "tw_beam_step: ld_tokens=%d max_new=%d", bp->ld_tokens, bp->max_new);
  TW_REQUIRE(params->mode == 0 && params->V <= ld_logits, "tw_beam_step: params");
  hipStream_t s = (hipStream_t)stream;
  switch (bp->num_beams) {
    case 2: return launch_beam<4>(logits, W, ld_logits, suppress_bits, params, bp, *bs, state, tokens, ids, pos, workspace, s);
    case 3: return launch_beam<6>(logits, W, ld_logits, suppress_bits, params, bp, *bs, state, tokens, ids, pos, workspace, s);
    case 4: return launch_beam<8>(logits, W, ld_logits, suppress_bits, params, bp, *bs, state, tokens, ids, pos, workspace, s);
    case 5: return launch_beam<10>(logits, W, ld_logits, suppress_bits, params, bp, *bs, state, tokens, ids, pos, workspace, s);
    case 6: return launch_beam<12>(logits, W, ld_logits, suppress_bits, params, bp, *bs, state, tokens, ids, pos, workspace, s);
    case 7: return launch_beam<14>(logits, W, ld_logits, suppress_bits, params, bp, *bs, state, tokens, ids, pos, workspace, s);
    default: return launch_beam<16>(logits, W, ld_logits, suppress_bits, params, bp, *bs, state, tokens, ids, pos, workspace, s);
  }
}

// Self-attention K/V reorder after a beam step: row r continues row src_rows[r]; positions [0, pos[r]) move.
// In place, one launch for K and V: block (layer*head, position tile, K|V) stages the tile of every moved row's
// source in LDS, then writes the destinations. Tiles are disjoint across blocks and a block reads all its sources
// before it writes, so any permutation is safe; HBM traffic is one read + one write per moved (row, position)
// (the earlier two-phase copy through a cache-sized scratch moved every byte twice, in four launches).
#define TW_KVR_LDS 57344
__global__ __launch_bounds__(256) void k_kv_reorder(bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
                                                    const int* __restrict__ src_rows, const int* __restrict__ pos,
                                                    int rows_cap, int H, int T, int R, int TT) {
  extern __shared__ uint4 kvr_tile[];  // [R][TT * 8] uint4 (a position of one head = 64 bf16 = 8 uint4)
  __shared__ int s_src[512], s_n[512];
  __shared__ int s_any;
  const int lh = blockIdx.x, l = lh / H, h = lh - l * H, t0 = blockIdx.y * TT;
  bf16_t* cache = blockIdx.z == 0 ? k_cache : v_cache;
  if (threadIdx.x == 0) s_any = 0;
  __syncthreads();
  for (int r = threadIdx.x; r < R; r += 256) {
    const int s = src_rows[r];
    // positions of this tile row r takes from s (an out-of-range source or position moves nothing: never a fault)
    const bool ok = s != r && s >= 0 && s < rows_cap;
    const int n = ok ? min(max(min(pos[r], T) - t0, 0), TT) : 0;
    s_src[r] = s;
    s_n[r] = n;
    if (n > 0) s_any = 1;
  }
  __syncthreads();
  if (!s_any) return;
  const int per_row = TT * 8;
  const size_t head = (size_t)T * 8;  // uint4 per (layer, row, head)
  const uint4* c4 = (const uint4*)cache;
  for (int e = threadIdx.x; e < R * per_row; e += 256) {
    const int r = e / per_row, q = e - r * per_row;
    if (q < s_n[r] * 8)
      kvr_tile[e] = c4[(((size_t)l * rows_cap + s_src[r]) * H + h) * head + (size_t)t0 * 8 + q];
  }
  __syncthreads();
  uint4* w4 = (uint4*)cache;
  for (int e = threadIdx.x; e < R * per_row; e += 256) {
    const int r = e / per_row, q = e - r * per_row;
    if (q < s_n[r] * 8) w4[(((size_t)l * rows_cap + r) * H + h) * head + (size_t)t0 * 8 + q] = kvr_tile[e];
  }
}

extern "C" int tw_kv_reorder(uint16_t* k_cache, uint16_t* v_cache, uint16_t* k_scratch, uint16_t* v_scratch, int layers,
                             int rows_cap, int H, int T, int R, const int* src_rows, const int* pos, void* stream) {
  (void)k_scratch;
  (void)v_scratch;
  // one position per tile at least: R * 128 B of dynamic LDS within TW_KVR_LDS (R <= 448)
  TW_REQUIRE(k_cache && v_cache && src_rows && pos && R > 0 && R <= rows_cap && R <= TW_KVR_LDS / 128 && T > 0,
             "tw_kv_reorder: bad args (R=%d rows_cap=%d T=%d; R <= %d)", R, rows_cap, T, TW_KVR_LDS / 128);
  int TT = 16;  // positions per tile: R * TT * 128 B of LDS
  while (TT > 1 && (size_t)R * TT * 128 > TW_KVR_LDS) TT >>= 1;
  const dim3 grid(layers * H, (T + TT - 1) / TT, 2);
  hipLaunchKernelGGL(k_kv_reorder, grid, dim3(256), (size_t)R * TT * 128, (hipStream_t)stream, (bf16_t*)k_cache,
                     (bf16_t*)v_cache, src_rows, pos, rows_cap, H, T, R, TT);
  return tw_check_launch("tw_kv_reorder");
}
