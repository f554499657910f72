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

// grid (B, TW_SELECT_CHUNKS): chunk c of row b scans vocab [c*V/NC, (c+1)*V/NC) with float4 loads where aligned.
__global__ __launch_bounds__(256) void k_select_partial(const float* __restrict__ logits, int ld_logits,
                                                        const uint32_t* __restrict__ suppress_bits, TwSelectParams p,
                                                        const int* __restrict__ state, SelPart* __restrict__ ws) {
  TW_DEC_PRIO();
  __shared__ SelPart sp[4];
  const int b = blockIdx.x, c = blockIdx.y, NC = gridDim.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const RowMask rm = row_mask(state + b * TW_STATE_STRIDE, p);
  const float* row = logits + (size_t)b * ld_logits;
  const int V = p.V, tsb = p.ts_begin;
  const int v0 = (int)((long)c * V / NC), v1 = (int)((long)(c + 1) * V / NC);
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
    ws[b * NC + c] = SelPart{bt.v, bt.i, bs.v, bs.i, m_ts, s_ts, 0.f, 0.f};
  }
}

// grid B, one wave: merge the row's chunk records (in chunk order: ties keep the first index), then
// the selection rule of the timestamp processor, the pad-after-EOS / stopping rule of _sample, and
// the processor state update.
__global__ __launch_bounds__(64) void k_select_final(const SelPart* __restrict__ ws, int NC, TwSelectParams p,
                                                     int* __restrict__ state, int* __restrict__ tokens_out,
                                                     int ld_tokens, int* __restrict__ next_ids,
                                                     int* __restrict__ pos) {
  TW_DEC_PRIO();
  const int b = blockIdx.x, lane = threadIdx.x;
  Best bt{-INFINITY, 0x7fffffff}, bs{-INFINITY, 0x7fffffff};
  float m_ts = -INFINITY, s_ts = 0.f;
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
  if (lane != 0) return;
  int* st = state + b * TW_STATE_STRIDE;
  const int n_gen = st[TW_ST_NGEN], last = st[TW_ST_LAST];
  if (pos) pos[b] += 1;  // the next decoder step writes its K/V one position later
  int sel;
  if (p.mode == 1) {
    sel = bt.i;
    st[TW_ST_LANG] = sel;
    if (next_ids) next_ids[b] = sel;
    return;
  }
  if (p.use_timestamps) {
    // "if sum of probability over timestamps is above any other token, sample timestamp"
    const float lse_ts = (m_ts == -INFINITY) ? -INFINITY : m_ts + __logf(s_ts);
    if (lse_ts > bt.v) sel = bs.i;
    else sel = best_of(bt, bs).i;
  } else {
    sel = bt.i;
  }
  const int finished = st[TW_ST_FINISHED];
  const int tok = finished ? p.pad : sel;
  if (tokens_out) tokens_out[(size_t)b * ld_tokens + n_gen] = tok;
  if (next_ids) next_ids[b] = tok;
  st[TW_ST_PENULT] = last;
  st[TW_ST_LAST] = tok;
  if (tok >= p.ts_begin && p.use_timestamps) st[TW_ST_LASTTS] = tok;
  st[TW_ST_NGEN] = n_gen + 1;
  if (!finished && (tok == p.eos || n_gen + 1 >= p.max_new)) st[TW_ST_FINISHED] = 1;
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
