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

__global__ __launch_bounds__(256) void k_logits_select(const float* __restrict__ logits, int ld_logits,
                                                       const uint32_t* __restrict__ suppress_bits, TwSelectParams p,
                                                       int* __restrict__ state, int* __restrict__ tokens_out,
                                                       int ld_tokens, int* __restrict__ next_ids,
                                                       int* __restrict__ pos) {
  __shared__ Best sb_text[4], sb_ts[4];
  __shared__ float sm_ts[4], ss_ts[4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int* st = state + b * TW_STATE_STRIDE;
  const float* row = logits + (size_t)b * ld_logits;
  const int n_gen = st[TW_ST_NGEN], last = st[TW_ST_LAST], penult = st[TW_ST_PENULT], last_ts = st[TW_ST_LASTTS];
  const int V = p.V, tsb = p.ts_begin;

  // ---- per-row mask parameters (WhisperTimeStampLogitsProcessor.__call__) ----
  int mask_ts_all = 0, mask_text_lt_eos = 0, ts_lo_block = tsb, ts_hi_block = tsb;  // masked [tsb, ts_hi_block)
  int init_step = (n_gen == 0);
  if (p.mode == 0 && p.use_timestamps) {
    const bool last_was_ts = n_gen >= 1 && last >= tsb;
    const bool penult_was_ts = n_gen < 2 || penult >= tsb;
    if (last_was_ts) {
      if (penult_was_ts) mask_ts_all = 1;
      else mask_text_lt_eos = 1;
    }
    if (last_ts >= 0) ts_hi_block = (last_was_ts && !penult_was_ts) ? last_ts : last_ts + 1;
  }

  Best bt{-INFINITY, 0x7fffffff}, bs{-INFINITY, 0x7fffffff};
  float m_ts = -INFINITY, s_ts = 0.f;
  for (int v = tid; v < V; v += 256) {
    float x = row[v];
    bool masked = false;
    if (p.mode == 1) {
      masked = (v < p.lo || v >= p.hi);
    } else {
      if (init_step)
        for (int i = 0; i < p.n_begin_suppress; ++i) masked |= (v == p.begin_suppress[i]);
      if (suppress_bits) masked |= (suppress_bits[v >> 5] >> (v & 31)) & 1u;
      if (p.use_timestamps) {
        masked |= (v == p.no_timestamps);
        if (v >= tsb) {
          masked |= mask_ts_all;
          masked |= (v >= ts_lo_block && v < ts_hi_block);
          if (init_step && p.max_initial_ts >= 0) masked |= (v > tsb + p.max_initial_ts);
        } else {
          masked |= mask_text_lt_eos && (v < p.eos);
          masked |= init_step;
        }
      }
    }
    if (masked) x = -INFINITY;
    if (v < tsb || !p.use_timestamps || p.mode == 1) {
      bt = best_of(bt, Best{x, v});
    } else {
      bs = best_of(bs, Best{x, v});
      if (x != -INFINITY) lse_merge(m_ts, s_ts, x, 1.f);
    }
  }
  // wave + block reductions
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Best ot{__shfl_xor(bt.v, o, 64), __shfl_xor(bt.i, o, 64)};
    Best os{__shfl_xor(bs.v, o, 64), __shfl_xor(bs.i, o, 64)};
    bt = best_of(bt, ot);
    bs = best_of(bs, os);
    float m2 = __shfl_xor(m_ts, o, 64), s2 = __shfl_xor(s_ts, o, 64);
    lse_merge(m_ts, s_ts, m2, s2);
  }
  if (lane == 0) { sb_text[wid] = bt; sb_ts[wid] = bs; sm_ts[wid] = m_ts; ss_ts[wid] = s_ts; }
  __syncthreads();
  if (tid != 0) return;
  if (pos) pos[b] += 1;  // the next decoder step writes its K/V one position later
  for (int w = 1; w < 4; ++w) {
    bt = best_of(bt, sb_text[w]);
    bs = best_of(bs, sb_ts[w]);
    lse_merge(m_ts, s_ts, sm_ts[w], ss_ts[w]);
  }
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
  if (tok >= tsb && p.use_timestamps) st[TW_ST_LASTTS] = tok;
  st[TW_ST_NGEN] = n_gen + 1;
  if (!finished && (tok == p.eos || n_gen + 1 >= p.max_new)) st[TW_ST_FINISHED] = 1;
}

extern "C" int tw_logits_select(const float* logits, int B, int ld_logits, const uint32_t* suppress_bits,
                                const TwSelectParams* params, int* state, int* tokens_out, int ld_tokens,
                                int* next_ids, int* pos, void* stream) {
  TW_REQUIRE(logits && params && state && B > 0, "tw_logits_select: bad args");
  TW_REQUIRE(params->V > 0 && params->V <= ld_logits, "tw_logits_select: V=%d ld=%d", params->V, ld_logits);
  TW_REQUIRE(params->n_begin_suppress >= 0 && params->n_begin_suppress <= 8, "tw_logits_select: begin_suppress");
  hipLaunchKernelGGL(k_logits_select, dim3(B), dim3(256), 0, (hipStream_t)stream, logits, ld_logits, suppress_bits,
                     *params, state, tokens_out, ld_tokens, next_ids, pos);
  return tw_check_launch("tw_logits_select");
}
