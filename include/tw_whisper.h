/*
 * tw_whisper.h — C-ABI of the MI355X (gfx950) Whisper batch-transcription hot path.
 *
 * The reference (crmorton/Turbo-Whisper-Workspace) has no native code: its hot path is the
 * Hugging Face ASR pipeline it builds in AudioProcessingPipeline.load_transcription_model
 * (/root/reference/vocalis/core/audio_pipeline.py:171-208) and calls at exactly one site
 * (:351-358). The arithmetic it executes lives in transformers ($TF =
 * site-packages/transformers, 5.15.0 here; reference pins 4.54.1). Each entry point below
 * replaces one stage of that executed path and cites it. The Python host layer
 * (turbo-whisper-workspace_amd/twamd) binds these symbols with ctypes and mirrors the reference's
 * callable / AudioProcessingPipeline interface on top of them.
 *
 * Conventions: plain pointers to DEVICE memory (HBM) unless noted, sizes in elements, bf16 passed
 * as raw uint16_t, `stream` is a hipStream_t (NULL = legacy default stream). Every function
 * returns 0 on success, nonzero on failure; tw_last_error() describes the failure (thread-local).
 * No function allocates, frees or synchronises: all are hipGraph-capturable.
 */
#ifndef TW_WHISPER_H
#define TW_WHISPER_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TW_ABI_VERSION 1

/* GEMM epilogues (tw_gemm_bf16). out/ldo are interpreted per epilogue. */
#define TW_EPI_BF16 0         /* out bf16[M][ldo] = acc + bias                                  */
#define TW_EPI_GELU_BF16 1    /* out bf16 = gelu_erf(acc + bias)             (fc1, conv1)       */
#define TW_EPI_RESID_F32 2    /* out f32[M][ldo] += acc + bias               (o-proj, fc2)      */
#define TW_EPI_GELU_POS_F32 3 /* out f32 = gelu(acc+bias) + aux[m % aux_rows][n] (conv2 + pos)  */
#define TW_EPI_F32 4          /* out f32 = acc + bias                        (proj_out logits)  */
#define TW_EPI_CROSSKV 5      /* out bf16 scattered to [layer][k|v][b][head][s][64]             */
#define TW_EPI_GELU_PACKED 6  /* tw_gemv_packed: out = packed activation (below) of gelu(acc+bias) (fc1 -> fc2) */
#define TW_EPI_GELU_MX 7      /* tw_gemm_mx: out fp8 e4m3[M][ldo] + e8m0 scales of gelu(acc+bias) (fc1 -> fc2) */
#define TW_EPI_GELU_F32 8     /* tw_gemm_f32: out f32 = gelu_erf(acc + bias)         (fc1, conv1 of the f32 path) */
#define TW_EPI_PARTIAL_F32 100 /* tw_gemv_packed: out f32[splits][M][ldo] split-K partials (no bias)          */

/* Decoder per-row state (tw_logits_select), int32[TW_STATE_STRIDE] per batch row. */
#define TW_STATE_STRIDE 8
#define TW_ST_NGEN 0     /* tokens generated so far in this decode pass                         */
#define TW_ST_LAST 1     /* last generated token                                                */
#define TW_ST_PENULT 2   /* penultimate generated token                                         */
#define TW_ST_LASTTS 3   /* last generated timestamp token id, -1 if none                       */
#define TW_ST_FINISHED 4 /* 1 once EOS was produced or max length reached                       */
#define TW_ST_LANG 5     /* language id chosen by mode-1 selection                              */
#define TW_ST_SUMLP 6    /* f32 bits: sum of the chosen tokens' log-probabilities (tw_logits_sample) */
#define TW_ST_NOSPEECH 7 /* f32 bits: no-speech probability (tw_token_prob)                      */

/* tw_logits_select workspace: f32[B][TW_SELECT_WS_PER_ROW] (TW_SELECT_CHUNKS vocab chunks per row). */
#define TW_SELECT_CHUNKS 16
#define TW_SELECT_WS_PER_ROW 128

typedef struct TwSelectParams {
  int32_t V;                  /* vocabulary size                                                 */
  int32_t eos;                /* eos_token_id (50257 multilingual)                               */
  int32_t pad;                /* pad_token_id (== eos for Whisper)                               */
  int32_t ts_begin;           /* no_timestamps_token_id + 1                                      */
  int32_t no_timestamps;      /* <|notimestamps|>                                               */
  int32_t max_initial_ts;     /* max_initial_timestamp_index, -1 = None                         */
  int32_t use_timestamps;     /* WhisperTimeStampLogitsProcessor active (return_timestamps)     */
  int32_t max_new;            /* finish after this many generated tokens (max_length - begin)   */
  int32_t mode;               /* 0 = generation step, 1 = language detection argmax in [lo,hi)  */
  int32_t lo, hi;             /* mode 1 range (language token ids)                              */
  int32_t n_begin_suppress;   /* <= 8                                                            */
  int32_t begin_suppress[8];  /* begin_suppress_tokens (e.g. 220, eos)                          */
} TwSelectParams;

/* ---- runtime ------------------------------------------------------------------------------- */
int tw_version(void);
const char* tw_last_error(void);

/* Seeded synthetic parameters (bf16-exact values). as_f32: write f32 instead of bf16.
 * Replaces: loading `openai/whisper-*` weights through transformers.pipeline
 * (/root/reference/vocalis/core/audio_pipeline.py:195-200) when no checkpoint is on disk. */
int tw_fill_synth(void* out, long n, uint64_t seed, uint32_t tensor_id, float scale, float offset, int as_f32,
                  void* stream);
/* out[i] = bf16(in[i] * scale) (checkpoint conversion; q-projection 0.125 fold). */
int tw_f32_to_bf16(const float* in, uint16_t* out, long n, float scale, void* stream);

/* ---- front end ------------------------------------------------------------------------------ */
/* Log-mel of n_chunks 30-s windows: wave f32[n_chunks][480000] -> feats f32[n_chunks][n_mels][3000].
 * basis_cos/basis_sin: the [400][224] periodic-Hann-windowed DFT basis (cols >= 201 zero) and
 * mel_fb: the [224][ceil32(n_mels)] slaney filterbank (rows >= 201, cols >= n_mels zero), both f32 in "k8" order:
 * element [k][c] of a [K][C] table at ((k/8 * C + c) * 2 + k%2) * 4 + (k%8)/2 (twamd.frontend.pack_k8);
 * maxkeys: u32[n_chunks] workspace. Replaces WhisperFeatureExtractor._torch_extract_fbank_features
 * ($TF/models/whisper/feature_extraction_whisper.py:135-168), run on the host CPU by the reference. */
int tw_logmel(const float* wave, int n_chunks, const float* basis_cos, const float* basis_sin, const float* mel_fb,
              int n_mels, float* feats, uint32_t* maxkeys, void* stream);

/* Log-mel of ONE input of any length > 200 samples (long-form generate(), > 30 s without chunking; the ASR pipeline's
 * feature extractor with truncation=False, padding="longest"): wave f32[n_samples] -> feats f32[n_mels][feats_ld],
 * frames 0 .. n_samples/160 - 1 written (reflect padding at the input's two ends only), the clamp at max - 8 over
 * the whole input; columns >= n_samples/160 are left untouched (the caller zeroes them: _get_input_segment's pad).
 * maxkey: u32[1] workspace. Basis / filterbank as tw_logmel. */
int tw_logmel_long(const float* wave, long n_samples, const float* basis_cos, const float* basis_sin,
                   const float* mel_fb, int n_mels, float* feats, long feats_ld, uint32_t* maxkey, void* stream);

/* conv1 im2col with the seek-window slice: out bf16[R*3000][kpad], k = j*n_mels + c, value
 * feats[row_map[r]][c][seek[r] + t + j - 1] inside [0, 3000 - seek[r]), else 0. row_map/seek may
 * be NULL (identity / 0). Replaces _get_input_segment ($TF/models/whisper/generation_whisper.py:
 * 1831-1850) + the Conv1d(k3,p1) input of WhisperEncoder.forward ($TF/.../modeling_whisper.py:618). */
int tw_im2col_conv1(const float* feats, int n_mels, const int* row_map, const int* seek, int R, int kpad,
                    uint16_t* out, void* stream);
/* tw_im2col_conv1 over feature rows of ld >= 3000 frames (long-form inputs): row r reads feature row row_map[r]
 * (NULL: r) from frame seek[r], valid frames u < min(3000, max_frames[row] - seek[r]) (generate()'s seek_num_frames;
 * max_frames[row] <= ld), zero beyond. */
int tw_im2col_conv1_long(const float* feats, int n_mels, long ld, const int* max_frames, const int* row_map,
                         const int* seek, int R, int kpad, uint16_t* out, void* stream);
/* conv2 im2col (k3, stride 2, pad 1): h1 bf16[R*3000][D] -> out bf16[R*1500][3D], k = j*D + c.
 * Replaces the Conv1d(k3,s2,p1) input of modeling_whisper.py:619. */
int tw_im2col_conv2(const uint16_t* h1, int R, int D, uint16_t* out, void* stream);
/* conv2 + GELU + positional add without the im2col copy (the engine's path): out f32[R*1500][D] =
 * gelu(Conv1d(k3,s2,p1)(h1)[r][t] + bias) + pos[t], h1 bf16[R][3000][D] read in place as an operand of row stride
 * 2D. D % 32 == 0. The D elements in front of h1 must be readable memory (the caller allocates one row before the
 * first frame; its contents do not matter). Replaces modeling_whisper.py:566-568 (conv2, GELU, embed_positions). */
int tw_conv2_gemm(const uint16_t* h1, int R, int D, const uint16_t* W, const float* bias, const float* pos, float* out,
                  void* stream);

/* ---- dense ops ------------------------------------------------------------------------------ */
/* C = A[M][K] . W[N][K]^T (bf16, f32 accumulate) with epilogue `epi` (TW_EPI_*). K % 64 == 0.
 * kv_geom = {S, B, D, H} for TW_EPI_CROSSKV, else NULL. Replaces nn.Linear / Conv1d of
 * $TF/models/whisper/modeling_whisper.py:279-282,309 (q,k,v,o), :375-376,444-445 (fc1, fc2),
 * :566-567 (conv stem), :970,1080 (tied proj_out) and the cross-attention K/V projections
 * cached by EncoderDecoderCache (:312-335). */
int tw_gemm_bf16(const uint16_t* A, const uint16_t* W, int M, int N, int K, int lda, int ldw, int epi, void* out,
                 int ldo, const float* bias, const float* aux, int aux_rows, const int* kv_geom, void* stream);
/* Process-wide kernel choice for the large-M path of tw_gemm_bf16 (returns 0): 1 = k_gemm_big (default: one
 * barrier per K-tile, 184 VGPRs, the kernel the engine queues beside a running decode step), 5 = k_gemm_8p (8-phase
 * ping-pong, faster when the encoder has the GPU to itself). Same results either way. */
int tw_gemm_set_variant(int v);
/* Split-K partial product for the decoder step (M <= 32 rows, K % 32 == 0): part f32[splits][M][ldp]
 * receives the `splits` partial sums of A . W^T over consecutive K ranges (no bias). Used for the
 * d_model-wide projections (self/cross out_proj, fc2) whose residual add is done by
 * tw_resid_layernorm, which sums the partials. Replaces the same nn.Linear calls as tw_gemm_bf16. */
int tw_gemm_bf16_partial(const uint16_t* A, const uint16_t* W, int M, int N, int K, int lda, int ldw, int splits,
                         float* part, int ldp, void* stream);
/* Decoder residual update + LayerNorm, one row per block: x f32[M][D] += bias + sum_p parts[p] (parts
 * f32[nparts][M][D]); then, if gamma != NULL, out bf16[M][D] = LayerNorm(x). Replaces the residual adds
 * of WhisperDecoderLayer.forward (modeling_whisper.py:468-505) + the following pre-LayerNorm. */
int tw_resid_layernorm(float* x, const float* parts, int nparts, const float* bias, const float* gamma,
                       const float* beta, int M, int D, float eps, uint16_t* out, void* stream);
/* out bf16[M][D] = LayerNorm(x f32[M][D]) (eps, affine). Replaces nn.LayerNorm (modeling_whisper.py
 * :371,377,434,443,446,573,682). */
int tw_layernorm(const float* x, const float* gamma, const float* beta, int M, int D, float eps, uint16_t* out,
                 void* stream);
/* Dynamic LDS (KiB, 0..64) requested by every later tw_layernorm workgroup: a cap on its workgroups per CU, set by the
 * caller beside a decode so that each SIMD keeps room for a decoder wave (as tw_attn_set_lds_pad); 0 (default) alone. */
int tw_layernorm_set_lds_pad(int kib);

/* ---- MX fp8 encoder (BASELINE config 5: fp8 MFMA encoder + bf16 decoder) --------------------- */
/* MX block format: e4m3fn elements [rows][K] (row-major bytes), e8m0 scales [K/128][rows_pad][4] bytes (byte
 * (k/32)%4 of row r's dword for K-step k/128; rows_pad >= rows, a multiple of 256 for GEMM operands). Scale
 * s = E - 8 + (absmax mantissa > 1.75) (E = biased f32 exponent of the 32-block's absmax; s = 1 for E < 9),
 * element = e4m3_rne(clamp(x * 2^(127-s), +-448)). The arithmetic they replace is the same nn.Linear of the encoder as tw_gemm_bf16
 * (modeling_whisper.py:279-282,309 q/k/v/o, :375-376 fc1/fc2), at reduced operand precision. */
/* C = A . W^T on v_mfma_scale_f32_16x16x128_f8f6f4, f32 accumulate. K % 128 == 0, lda/ldw in bytes (% 16),
 * Mp / Np the scale row pads of A / W (multiples of 256). epi: TW_EPI_BF16, TW_EPI_RESID_F32, TW_EPI_F32, or
 * TW_EPI_GELU_MX (out fp8[M][ldo] + sout scales [N/128][sout_rows][4]; N % 256 == 0). */
int tw_gemm_mx(const uint8_t* A, const uint8_t* Sa, const uint8_t* W, const uint8_t* Sw, int M, int N, int K, int lda,
               int ldw, int Mp, int Np, int epi, void* out, int ldo, const float* bias, uint8_t* sout, int sout_rows,
               void* stream);
/* Process-wide (returns 0): tw_gemm_mx's kernel, 0 = default (by shape: k_gemm_mx for q/k/v, N = 3 K; k_gemm_8p_mx
 * otherwise), 1 = k_gemm_mx (2-stage), 8 = k_gemm_8p_mx (8-phase ping-pong); the forced forms exist so that tests
 * cover both kernels on every shape. */
int tw_gemm_mx_set_variant(int v);
/* bf16 src[rows][ld] -> MX fp8 dst[rows][K] + scales (K % 128 == 0). Encoder weights once at load; the
 * attention output before out_proj (modeling_whisper.py:350-356). */
int tw_quant_mx(const uint16_t* src, int rows, int K, int ld, uint8_t* dst, uint8_t* scales, int rows_pad,
                void* stream);
/* LayerNorm (as tw_layernorm) with the MX quantisation of its output fused into the store (D % 128 == 0). */
int tw_layernorm_mx(const float* x, const float* gamma, const float* beta, int M, int D, float eps, uint8_t* out,
                    uint8_t* scales, int rows_pad, void* stream);

/* ---- attention ------------------------------------------------------------------------------ */
/* Encoder self-attention. qkv bf16[B*S][3*H*64] (q pre-scaled by 64^-0.5) -> out bf16[B*S][H*64].
 * Replaces WhisperAttention + eager_attention_forward/SDPA for the encoder
 * (modeling_whisper.py:215-238, 241-356). */
int tw_attn_encoder(const uint16_t* qkv, int B, int S, int H, uint16_t* out, void* stream);
/* tw_attn_encoder with the output stored as MX fp8 (out e4m3[B*S][H*64], scales [H*64/128][rows_pad][4]; format:
 * "MX fp8 encoder" above), the out_proj operand of the config-5 encoder (modeling_whisper.py:350-356). H even. */
int tw_attn_encoder_mx(const uint16_t* qkv, int B, int S, int H, uint8_t* out, uint8_t* scales, int rows_pad,
                       void* stream);
/* Measurement knob (process-wide, returns 0 or TW_ERR_ARG): encoder attention kernel of tw_attn_encoder and
 * tw_attn_encoder_mx. 32 (default) = k_attn_enc5 (64 queries per wave, log2-unit scores, guarded unshifted exp2),
 * 16 = k_attn_enc4 (bit-identical to k_attn_enc2), 8 = k_attn_enc2 (32 queries per wave, running-max softmax; the
 * MX-output kernel for 8 and 16). */
int tw_attn_set_variant(int variant);
/* Process-wide: reserve units x 16 KiB (0..8) of extra LDS per tw_attn_encoder workgroup, capping its workgroups per CU
 * so that decoder kernels launched beside it on another stream find free wave slots (the engine sets 4 for encoder
 * chunks queued beside a decode, 0 otherwise). Returns 0, or TW_ERR_ARG. */
int tw_attn_set_lds_pad(int units);

/* ---- beam search ------------------------------------------------------------------------------ */
/* GenerationMixin._beam_search ($TF/generation/utils.py:3208-3512) with the Whisper processor chain, for W windows
 * of num_beams rows each (row = w * num_beams + j), early_stopping=False, one EOS id. One call per generated token:
 * per row the log_softmax of the f32 logits, the processors (as tw_logits_select) and the top 2*num_beams
 * continuations; per window the running beams, the finished beams (score / len**length_penalty) and the
 * early-stop heuristic. It rewrites the running token histories (tokens), the processor state, ids and pos of
 * every row, and src_rows (the row whose self-attention K/V each new running beam continues: tw_kv_reorder).
 * TwBeamState holds DEVICE arrays; win[w] = {improvement possible, done, tokens generated, unused}. Initialise
 * run_score to {0, -1e9, ...} per window, fin_score to -1e9, fin_flag/fin_len to 0, win to {1, 0, 0, 0}.
 * The best hypothesis of window w is finished slot 0: fin_tokens[w*nb][0 .. fin_len[w*nb]). */
typedef struct TwBeamParams {
  int32_t num_beams;     /* 2 .. 8                                                      */
  int32_t max_new;       /* max_length - prompt length                                   */
  float length_penalty;  /* generation_config.length_penalty (1.0)                       */
  int32_t ld_tokens;     /* row stride of tokens / fin_tokens (<= 448)                   */
} TwBeamParams;
typedef struct TwBeamState {
  float* run_score;      /* f32[R]   running beam scores (descending within a window)    */
  float* fin_score;      /* f32[R]                                                        */
  int32_t* fin_flag;     /* i32[R]                                                        */
  int32_t* fin_len;      /* i32[R]                                                        */
  int32_t* fin_tokens;   /* i32[R][ld_tokens]                                             */
  int32_t* win;          /* i32[W][4]                                                     */
  int32_t* src_rows;     /* i32[R]   out                                                  */
  int32_t* kv_tab;       /* i32[R][ld_tokens] or NULL: the self-attention K/V position table
                          * (tw_attn_decode_self_tab): row r's positions [0, pos[r]) take row src_rows[r]'s
                          * entries, in place of a tw_kv_reorder copy. Initialise kv_tab[r][*] = r; its row
                          * stride ld_tokens must equal the caches' max_pos.                                 */
  int32_t* fin_tab;      /* i32[R][ld_tokens] or NULL (needs kv_tab): finished slot s of window w gets the row
                          * that fed each position of its history (kv_tab of its source at the step it finished,
                          * positions 0 .. its last fed one) — the beam_indices of token-level timestamps
                          * (generation_whisper.py:265-300): position p's cross-attention is that row's.       */
  float* run_lp;         /* f32[R] or NULL (with fin_lp): per running beam the sum of its tokens' log-probabilities
                          * renormalised over the allowed tokens (log_softmax of the processed beam scores:
                          * _retrieve_avg_logprobs, generation_whisper.py:1958-1975); initialise 0                  */
  float* fin_lp;         /* f32[R] or NULL: the same sum of each finished slot's hypothesis                       */
} TwBeamState;
/* workspace: tw_beam_workspace_bytes(R) bytes of device memory. */
size_t tw_beam_workspace_bytes(int rows);
int tw_beam_step(const float* logits, int W, int ld_logits, const uint32_t* suppress_bits,
                 const TwSelectParams* params, const TwBeamParams* beam, const TwBeamState* bstate, int* state,
                 int* tokens, int* ids, int* pos, void* workspace, void* stream);
/* caches bf16[layers][rows_cap][H][T][64]: rows 0..R-1 take positions [0, pos[r]) of row src_rows[r] (any
 * permutation, R <= 448 = the 56 KiB LDS tile at one position), in place. k_scratch / v_scratch are unused (may be NULL; kept for ABI stability). */
int tw_kv_reorder(uint16_t* k_cache, uint16_t* v_cache, uint16_t* k_scratch, uint16_t* v_scratch, int layers,
                  int rows_cap, int H, int T, int R, const int* src_rows, const int* pos, void* stream);

/* ---- packed decoder GEMV ------------------------------------------------------------------------- */
/* The decoder step's projections (M <= 32 rows: $TF/models/whisper/modeling_whisper.py:279-282, 375-376, and the
 * tied proj_out :970) read every weight byte once per token, so their layout is chosen for the HBM stream:
 *   packed weight      bf16 [ceil(N/16)][K/32][64][8]: (n, k) at ((n/16*K/32 + k/32)*64 + n%16 + 16*(k/8%4))*8 + k%8
 *   packed activation  bf16 [K/32][2][64][8]:          (m, k) at ((k/32*2 + m/16)*64 + m%16 + 16*(k/8%4))*8 + k%8
 * i.e. each (16 columns or rows) x (32-deep step) MFMA operand fragment is 1 KiB contiguous; pad columns are zero,
 * activation rows M..31 are never written (keep them finite, e.g. zeroed once).
 * tw_pack_weight: W bf16[N][ldw] -> Wp packed weight (setup time).
 * tw_gemv_packed: out = epi(A . W^T); A packed activation (a_packed = 1) or row-major [M][lda]; epi TW_EPI_BF16,
 *   TW_EPI_F32 (row-major [M][ldo]), TW_EPI_GELU_PACKED (packed activation, N % 32 == 0), TW_EPI_RESID_F32
 *   (f32 [M][ldo] += A.W^T + bias: the decoder's residual update; splits = 1) or TW_EPI_PARTIAL_F32 (splits > 1
 *   allowed; bias ignored). */
int tw_pack_weight(const uint16_t* W, int N, int K, int ldw, uint16_t* Wp, void* stream);
int tw_gemv_packed(const uint16_t* A, int a_packed, int lda, const uint16_t* Wp, int M, int N, int K, int epi,
                   void* out, int ldo, const float* bias, int splits, void* stream);
/* Process-wide K-slice count (1, 2 or 4; default 1) of tw_gemv_packed's vocabulary-wide case (N >= 16384: proj_out):
 * 1 beside a running encoder GEMM, 4 when the decode has the GPU to itself. Same results up to the f32 order of the
 * K-slice sum. Returns 0. */
int tw_gemv_set_wide_slices(int kw);
/* Process-wide kernel of tw_gemv_packed's decoder-layer shapes (N < 16384, epilogues BF16 / GELU_PACKED / PARTIAL):
 * 0 = two column groups per wave in batches of 5 K-steps, 1 = one column group per wave with its whole K-slice of
 * weight fragments in flight (<= 10 steps). Same results up to the f32 order of the K-slice sum. Returns 0. */
int tw_gemv_set_variant(int v);
/* Epilogue form of tw_gemm_bf16's large-M kernels: 0 (default) = the f32 LDS image of row-major accumulators, 1 =
 * transposed accumulators (the MFMA as W . A^T: bias / GELU in registers, bf16 outputs staged as packed bf16, f32
 * outputs stored from registers). The same sums either way (A/B switch; results agree to the output rounding). */
int tw_gemm_set_epilogue(int tr);
/* Workgroups of the persistent large-M GEMM (tw_gemm_set_variant(6)): 0 = one per CU, else n (a multiple of 8, one per
 * CU on n / 8 CUs of every XCD) — the rest of the CUs stay free for other queues' kernels. */
int tw_gemm_set_persistent_grid(int n);
/* ---- the decoder's layers as one persistent launch ------------------------------------------------- */
/* One decoder layer's parameters (device memory, an array of n_layers): packed weights (tw_pack_weight of the
 * [N][K] projections, q pre-scaled as for the launch chain), f32 biases and LayerNorm parameters. */
typedef struct TwDecLayerW {
  const uint16_t *wqkv, *wo, *wq_x, *wo_x, *w1, *w2;
  const float *bqkv, *bo, *bq_x, *bo_x, *b1, *b2;
  const float *ln1_g, *ln1_b, *ln2_g, *ln2_b, *ln3_g, *ln3_b;
} TwDecLayerW;
/* tw_dec_fused: WhisperDecoder's layers for one token of R <= 32 rows ($TF/models/whisper/modeling_whisper.py:
 * 448-505 per layer, then the final layer_norm :682) — what the launch chain of residual + LayerNorm, q/k/v, self-
 * attention, out_proj, cross-q, cross-attention, out_proj, fc1 and fc2 kernels computes — as ONE persistent launch
 * of one workgroup per CU whose phases hand off through device-memory counters (d_model 1280, 20 heads, ffn 5120:
 * tw_dec_fused_supported). In: x f32 [R][1280] = the token + position embedding (tw_embed_decoder); the self K/V
 * caches kc / vc ([rows][20][max_pos][64] per layer, layer l at + l * kv_layer_stride elements) hold positions
 * < pos[r]; the cross K/V of layer l at xkv + l * xkv_layer_stride (K) and + xkv_v_off (V), [rows][20][S][64].
 * Out: x = the last layer's output, the caches appended at pos, hp = the final LayerNorm as a packed activation
 * (proj_out's tw_gemv_packed operand; also the launch's LayerNorm scratch). Scratch: qb, ab bf16 [R][1280], fb packed
 * [32][5120], slab f32 [4][R][1280], xpart f32 tw_dec_fused_xpart_bytes(R),
 * sync: tw_dec_fused_sync_bytes() bytes, 16-byte aligned (zeroed by the call, on the stream). err: a sticky word the
 * caller zeroes once; a phase wait that times out sets it (0x100 + phase) and the launch's outputs are void. The
 * caller must not run other work on the device that waits for this launch's completion from inside a kernel. */
size_t tw_dec_fused_sync_bytes(void);
int tw_dec_fused_supported(int d_model, int heads, int ffn, int rows);
/* Workgroups per launch (0 = the device's CU count, the default; n <= the CU count keeps every workgroup resident). */
int tw_dec_fused_set_grid(int n);
/* 1: an agent-scope acquire fence after every phase wait in addition to the sc1 (L1-bypassing) loads of every
 * handed-off byte; 0 (default): the loads alone. The same results either way (A/B switch). Returns 0. */
int tw_dec_fused_set_acquire(int on);
/* Measurement: buf (device, u64 [n_layers + 1][12][grid][2], zeroed by the caller) receives per (layer, phase,
 * workgroup) the 100-MHz real-time clock at the start of the workgroup's first item of the phase (after its wait) and
 * at the end of its last; slot (n_layers, 0) = each workgroup's start, (n_layers, 11) = the final LayerNorm. NULL (the
 * default) turns it off. tw_dec_fused_grid: the grid of the last launch (0 before the first). */
int tw_dec_fused_set_probe(void* buf);
int tw_dec_fused_grid(void);
int tw_dec_fused(const TwDecLayerW* layers, int n_layers, int R, const int* pos, float* x, uint16_t* kc,
                 uint16_t* vc, long kv_layer_stride, int max_pos, const uint16_t* xkv, long xkv_layer_stride,
                 long xkv_v_off, int S, uint16_t* qb, uint16_t* ab, uint16_t* fb, float* slab, float* xpart,
                 const float* lnf_g, const float* lnf_b, uint16_t* hp, float eps, unsigned* sync, unsigned* err,
                 void* stream);
/* Bytes of tw_dec_fused's cross-attention slice scratch (xpart) for R rows. */
size_t tw_dec_fused_xpart_bytes(int rows);
/* tw_resid_layernorm with the normalised rows written as a packed activation (M <= 64, D % 32 == 0). */
int tw_resid_layernorm_packed(float* x, const float* parts, int nparts, const float* bias, const float* gamma,
                              const float* beta, int M, int D, float eps, uint16_t* out, void* stream);
/* The same with the updated residual rows written to x_out instead of in place (x is only read; x_out may equal x). */
int tw_resid_layernorm_packed_to(const float* x, float* x_out, const float* parts, int nparts, const float* bias,
                                 const float* gamma, const float* beta, int M, int D, float eps, uint16_t* out,
                                 void* stream);

/* Decoder self-attention for one new token per row: appends k,v of qkv bf16[B][3D] at pos[b] into
 * k_cache/v_cache bf16[B][H][max_pos][64] (this layer) and attends over 0..pos[b].
 * Replaces the causal self-attention + DynamicCache.update of modeling_whisper.py:312-335,448-505. */
int tw_attn_decode_self(const uint16_t* qkv, int B, int H, int max_pos, const int* pos, uint16_t* k_cache,
                        uint16_t* v_cache, uint16_t* out, void* stream);
/* The same with beam search's copy-free K/V history: position q < pos[b] of row b is read from cache row
 * kv_tab[(row0 + b) * max_pos + q] (a global row: k_cache / v_cache point at row row0 of the layer's caches, which
 * hold rows_cap rows); the step's own K/V is written to row b at pos[b], and kv_tab[(row0 + b) * max_pos + pos[b]]
 * must equal row0 + b (tw_beam_step keeps it so). Each physical (row, position) is written once per pass, so no
 * history is ever overwritten while another beam still reads it. Caller contract: no history entry q < pos[b] may
 * name a row b2 of this launch with q == pos[b2] (that cell is written by the same launch; the read would race).
 * Beam tables keep it: a window's beams share one position. A library built with -DTW_DEBUG=1 (`make debug`,
 * libtwhip_dbg.so) checks the contract with tw_kv_tab_check before every launch outside a graph capture and returns
 * TW_ERR_ARG naming the row instead of racing. */
int tw_attn_decode_self_tab(const uint16_t* qkv, int B, int H, int max_pos, const int* pos, uint16_t* k_cache,
                            uint16_t* v_cache, const int* kv_tab, int row0, uint16_t* out, void* stream);
/* tw_attn_decode_self / _tab with left-padded prompts (condition_on_prev_tokens over a batch: generate()'s
 * decoder_attention_mask, generation_whisper.py:1893-1908): kv_start int32[B] (device) = row b's pad count; a query at
 * pos[b] >= kv_start[b] attends keys kv_start[b] .. pos[b] only (the pad positions still take their positions). */
int tw_attn_decode_self_masked(const uint16_t* qkv, int B, int H, int max_pos, const int* pos, uint16_t* k_cache,
                               uint16_t* v_cache, const int* kv_start, uint16_t* out, void* stream);
int tw_attn_decode_self_tab_masked(const uint16_t* qkv, int B, int H, int max_pos, const int* pos, uint16_t* k_cache,
                                   uint16_t* v_cache, const int* kv_tab, int row0, const int* kv_start, uint16_t* out,
                                   void* stream);
/* The contract of tw_attn_decode_self_tab as a check: bad int32[B] (device) receives, per row b of a launch with the
 * same (kv_tab, pos, row0, B, max_pos), the number of history entries that name a (row, position) that launch
 * writes (0 everywhere = the launch is race-free). Asynchronous on `stream`. */
int tw_kv_tab_check(const int* kv_tab, const int* pos, int row0, int B, int max_pos, int* bad, void* stream);
/* 1 if the library was built with -DTW_DEBUG=1 (the guarded tw_attn_decode_self_tab), else 0. */
int tw_debug_build(void);
/* Decoder cross-attention for one query per row over the cached encoder K/V of this layer,
 * cross_kv bf16[2][Bt][H][S][64]; row b reads slot row_map[b] (NULL = b). */
int tw_attn_decode_cross(const uint16_t* q, int B, int H, int S, int Bt, const int* row_map, const uint16_t* cross_kv,
                         uint16_t* out, void* stream);
/* The same for rows that share an encoder slot in groups (the beams of one window, rows w * num_beams + j): the first
 * `first` rows (0 <= first < group, the tail of a group that began before this view) form one group, then every
 * `group` rows (2..8) one group; all rows of a group must hold the same row_map entry (required, not checked). Each
 * K/V row is read once per group; the keys are split in slices whose states ws (device memory of
 * tw_attn_decode_cross_grouped_ws_bytes(B, H) bytes) holds until a second launch combines them. Agrees with
 * tw_attn_decode_cross to bf16 rounding (another softmax merge order). */
size_t tw_attn_decode_cross_grouped_ws_bytes(int B, int H);
int tw_attn_decode_cross_grouped(const uint16_t* q, int B, int H, int S, int Bt, const int* row_map, int group,
                                 int first, const uint16_t* cross_kv, float* ws, uint16_t* out, void* stream);
/* The same plus the attention probabilities of selected heads (token-level timestamps, the cross_attentions of
 * WhisperGenerationMixin._extract_token_timestamps, $TF/models/whisper/generation_whisper.py:241-380):
 * probs f32[B][n_steps][n_slots][S] receives, for every head h with bit h of head_mask set (H <= 32), row b's
 * probabilities at step pos[b] - pos0 into slot slot0 + (set bits of head_mask below h), when 0 <= step < n_steps. */
int tw_attn_decode_cross_probs(const uint16_t* q, int B, int H, int S, int Bt, const int* row_map,
                               const uint16_t* cross_kv, uint16_t* out, float* probs, uint32_t head_mask, int slot0,
                               int n_slots, const int* pos, int pos0, int n_steps, void* stream);
/* Host memory: dynamic time warping of matrix f64[n][m] (the cost, i.e. minus the smoothed attention) as
 * _dynamic_time_warping (generation_whisper.py:64-114); text_idx / time_idx int32[n + m] receive the path,
 * *path_len its length. */
int tw_dtw(const double* matrix, int n, int m, int* text_idx, int* time_idx, int* path_len);

/* ---- fp32 path (BASELINE configs[0]: whisper-tiny.en fp32) --------------------------------------------------
 * The same modules as the bf16 entries above at f32 operand / activation / cache precision, for the reference's
 * fp32 load (/root/reference/vocalis/core/audio_pipeline.py:195-200, torch_dtype=torch.float32; csrc/f32path.hip).
 * tw_gemm_f32: C = A[M][K] . W[N][K]^T on v_mfma_f32_16x16x4_f32, K % 16 == 0, lda / ldw multiples of 4, epi
 *   TW_EPI_F32, TW_EPI_GELU_F32, TW_EPI_RESID_F32, TW_EPI_GELU_POS_F32 or TW_EPI_CROSSKV (f32 out, kv_geom as
 *   tw_gemm_bf16). Replaces nn.Linear / Conv1d-as-GEMM (modeling_whisper.py:279-282,375-376,566-567,970). */
int tw_gemm_f32(const float* A, const float* W, int M, int N, int K, int lda, int ldw, int epi, float* out, int ldo,
                const float* bias, const float* aux, int aux_rows, const int* kv_geom, void* stream);
/* out f32[M][D] = LayerNorm(x f32[M][D]) (out != x). */
int tw_layernorm_f32(const float* x, const float* gamma, const float* beta, int M, int D, float eps, float* out,
                     void* stream);
/* tw_im2col_conv1 / tw_im2col_conv1_long with f32 output: feature rows of ld frames (3000: the 30-s windows, then
 * max_frames and seek may be NULL; ld > 3000: long-form rows, both required). */
int tw_im2col_conv1_f32(const float* feats, int n_mels, long ld, const int* max_frames, const int* row_map,
                        const int* seek, int R, int kpad, float* out, void* stream);
/* tw_im2col_conv2 with f32 operands (D % 4 == 0). */
int tw_im2col_conv2_f32(const float* h1, int R, int D, float* out, void* stream);
/* x f32[B][D] = tok_emb f32[ids[b]] + pos_emb f32[pos[b]]. */
int tw_embed_decoder_f32(const float* tok_emb, const float* pos_emb, const int* ids, const int* pos, int B, int D,
                         float* x, void* stream);
/* Encoder self-attention over qkv f32[B*S][3*H*64] (q pre-scaled) -> out f32[B*S][H*64]. */
int tw_attn_encoder_f32(const float* qkv, int B, int S, int H, float* out, void* stream);
/* tw_attn_decode_self[_tab][_masked] in one entry, f32 caches [B][H][max_pos][64]: kv_tab (NULL: none) with row0 as
 * tw_attn_decode_self_tab, kv_start (NULL: none) as tw_attn_decode_self_masked. max_pos <= 2048. */
int tw_attn_decode_self_f32(const float* qkv, int B, int H, int max_pos, const int* pos, float* k_cache,
                            float* v_cache, const int* kv_tab, int row0, const int* kv_start, float* out,
                            void* stream);
/* tw_attn_decode_cross[_probs] in one entry, cross_kv f32[2][Bt][H][S][64] (S <= 2048); probs NULL: no alignment
 * heads, else as tw_attn_decode_cross_probs. */
int tw_attn_decode_cross_f32(const float* q, int B, int H, int S, int Bt, const int* row_map, const float* cross_kv,
                             float* out, float* probs, unsigned head_mask, int slot0, int n_slots, const int* pos,
                             int pos0, int n_steps, void* stream);

/* ---- decoder glue --------------------------------------------------------------------------- */
/* x f32[B][D] = embed_tokens[ids[b]] + embed_positions[pos[b]] (modeling_whisper.py:737,753-762). */
int tw_embed_decoder(const uint16_t* tok_emb, const uint16_t* pos_emb, const int* ids, const int* pos, int B, int D,
                     float* x, void* stream);
/* Whisper logits processors + greedy argmax for B rows of f32 logits (see TwSelectParams; state
 * int32[B][TW_STATE_STRIDE]; tokens_out int32[B][ld_tokens] receives token n_gen; next_ids int32[B];
 * pos int32[B] (may be NULL) is incremented so a captured decode step can be replayed unchanged;
 * workspace f32[B][TW_SELECT_WS_PER_ROW]).
 * `params` is a HOST pointer (passed by value to the kernel). suppress_bits: u32[ceil(V/32)] or NULL.
 * Replaces GenerationMixin._sample's selection step ($TF/generation/utils.py:2876-2941) with
 * SuppressTokensAtBegin / SuppressTokens / WhisperTimeStamp processors
 * ($TF/generation/logits_process.py:1816-2047) and detect_language's argmax
 * ($TF/models/whisper/generation_whisper.py:1664-1671). */
int tw_logits_select(const float* logits, int B, int ld_logits, const uint32_t* suppress_bits,
                     const TwSelectParams* params, int* state, int* tokens_out, int ld_tokens, int* next_ids,
                     int* pos, float* workspace, void* stream);
/* tw_logits_select (mode 0, next_ids and pos required) fused with the head of the next decoder step: the chosen
 * token is embedded at the row's incremented position into x f32[B][D] (as tw_embed_decoder) and the first decoder
 * layer's self_attn_layer_norm (gamma, beta, eps) is written to out bf16 — row-major [B][D], or the packed
 * activation layout when packed != 0 (B <= 32, D % 32 == 0; as tw_resid_layernorm_packed). max_pos = rows of
 * pos_emb (a position past it, after the last step, reads the last row; that embedding is never consumed).
 * Same results as tw_logits_select + tw_embed_decoder + tw_resid_layernorm[_packed](nparts 0) in two launches
 * instead of four (the step's graph starts at the first layer's q/k/v projection). */
int tw_logits_select_embed(const float* logits, int B, int ld_logits, const uint32_t* suppress_bits,
                           const TwSelectParams* params, int* state, int* tokens_out, int ld_tokens, int* next_ids,
                           int* pos, float* workspace, const uint16_t* tok_emb, const uint16_t* pos_emb, int D,
                           int max_pos, float* x, const float* gamma, const float* beta, float eps, uint16_t* out,
                           int packed, void* stream);

/* Temperature-fallback decode step (WhisperGenerationMixin.generate_with_fallback,
 * $TF/models/whisper/generation_whisper.py:970-1116), one workgroup per row, same arguments as tw_logits_select minus
 * the workspace. temperature == 0: the greedy token, bit-identical to tw_logits_select. temperature > 0 (do_sample):
 * TemperatureLogitsWarper + TopKLogitsWarper(top_k; <= 0 = off; ties at the k-th value kept) and a draw from the
 * softmax of the kept scores by the Gumbel-max trick with a counter-based hash of (seed, row_key[b] (NULL: b), token
 * index in the pass, vocabulary id): the distribution of _sample's torch.multinomial, not its random stream.
 * Every row unfinished before the step adds log_softmax(scores)[token] (the scores generate() returns with
 * output_scores, at temperature 1: _retrieve_avg_logprobs, :1958-1975) to state[TW_ST_SUMLP] (f32 bits). */
int tw_logits_sample(const float* logits, int B, int ld_logits, const uint32_t* suppress_bits,
                     const TwSelectParams* params, float temperature, int top_k, uint64_t seed, const int* row_key,
                     int* state, int* tokens_out, int ld_tokens, int* next_ids, int* pos, void* stream);
/* state[b][TW_ST_NOSPEECH] (f32 bits) = softmax(logits[b][0:V])[token]: WhisperNoSpeechDetection's no_speech_prob
 * ($TF/generation/logits_process.py:2050-2112) from the logits at the <|startoftranscript|> position. */
int tw_token_prob(const float* logits, int B, int ld_logits, int V, int token, int* state, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TW_WHISPER_H */
