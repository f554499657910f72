// PyTorch-ROCm custom operators over the C-ABI (libtwhip.so): the `tw::` op namespace (torch.ops.tw.*).
//
// Each op checks its tensors (device, dtype, contiguity of the inner dimension, shapes), launches the hand-written
// HIP kernel through the C-ABI entry point on the CURRENT HIP stream (so it orders with torch work, is captured by
// torch.cuda.graph, and shows up as an op in the profiler), and raises with tw_last_error() on a failed call. The ops
// are registered for device tensors (the dispatcher's GPU key; on ROCm builds of torch that key holds HIP tensors)
// and for Meta tensors (shape functions: FakeTensor / torch.compile tracing). Functional forms allocate their
// output; `_out` forms write caller-owned buffers (allocation-free: the engine's graph-captured paths use those).
//
// Kept out of libtwhip.so itself so that the C-ABI library stays free of torch (a C caller links
// it alone); this library links libtwhip.so and libtorch and is loaded with torch.ops.load_library
// (twamd/_ops.py). SURVEY §8b; BASELINE north_star ("Python host code calling hand-written HIP through PyTorch-ROCm
// custom ops").
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <vector>

#include "tw_whisper.h"

namespace {

using at::Tensor;

// Every op runs on the device of its first tensor: a device guard for the launch (TW_OP_DEVICE) and that device's
// current stream (not the current device's, which may differ)
#define TW_OP_DEVICE(t)                                                                                  \
  c10::hip::OptionalHIPGuard tw_guard_((t).is_cuda() ? std::optional<c10::DeviceIndex>((t).device().index()) \
                                                     : std::nullopt)
void* cur_stream(const Tensor& t) { return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void ok(int rc, const char* what) { TORCH_CHECK(rc == 0, "tw::", what, " failed (", rc, "): ", tw_last_error()); }

void dev(const Tensor& t, at::ScalarType st, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
  TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
}

void rows(const Tensor& t, const char* name) {  // 2-D, unit stride along the inner dimension
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, name, " must be 2-D with a contiguous inner dimension");
}

void same_device(const Tensor& a, const Tensor& b, const char* name) {
  TORCH_CHECK(a.device() == b.device(), name, " is on ", b.device(), ", the op's operands on ", a.device());
}

// a contiguous device tensor of dtype st holding at least n elements, on the op's device
void holds(const Tensor& first, const Tensor& t, at::ScalarType st, int64_t n, const char* name) {
  dev(t, st, name);
  same_device(first, t, name);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.numel() >= n, name, " holds ", t.numel(), " elements, the call needs ", n);
}

void opt_holds(const Tensor& first, const c10::optional<Tensor>& t, at::ScalarType st, int64_t n, const char* name) {
  if (t.has_value() && t->defined()) holds(first, *t, st, n, name);
}

template <class T>
T* ptr(const Tensor& t) { return (T*)t.data_ptr(); }

template <class T>
T* optr(const c10::optional<Tensor>& t) { return t.has_value() && t->defined() ? (T*)t->data_ptr() : nullptr; }

constexpr int64_t kFrames = 3000, kSamples = 480000;

// ---- log-mel (WhisperFeatureExtractor._torch_extract_fbank_features, $TF/.../feature_extraction_whisper.py:135-168)
void logmel_out(const Tensor& wave, const Tensor& basis_cos, const Tensor& basis_sin, const Tensor& mel_fb,
                int64_t n_mels, Tensor& out, Tensor& maxkeys) {
  TW_OP_DEVICE(wave);
  dev(wave, at::kFloat, "wave");
  TORCH_CHECK(wave.dim() == 2 && wave.size(1) == kSamples && wave.is_contiguous(), "wave must be [B][480000]");
  dev(out, at::kFloat, "out");
  const int64_t B = wave.size(0);
  TORCH_CHECK(out.is_contiguous() && out.numel() >= B * n_mels * kFrames, "out must hold [B][n_mels][3000]");
  dev(maxkeys, at::kInt, "maxkeys");
  TORCH_CHECK(maxkeys.numel() >= B, "maxkeys must hold B entries");
  for (auto* t : {&basis_cos, &basis_sin, &mel_fb}) dev(*t, at::kFloat, "basis / filterbank");
  ok(tw_logmel(ptr<float>(wave), (int)B, ptr<float>(basis_cos), ptr<float>(basis_sin), ptr<float>(mel_fb),
               (int)n_mels, ptr<float>(out), ptr<uint32_t>(maxkeys), cur_stream(wave)),
     "logmel");
}

Tensor logmel(const Tensor& wave, const Tensor& basis_cos, const Tensor& basis_sin, const Tensor& mel_fb,
              int64_t n_mels) {
  Tensor out = at::empty({wave.size(0), n_mels, kFrames}, wave.options());
  Tensor mk = at::empty({wave.size(0)}, wave.options().dtype(at::kInt));
  logmel_out(wave, basis_cos, basis_sin, mel_fb, n_mels, out, mk);
  return out;
}

Tensor logmel_meta(const Tensor& wave, const Tensor&, const Tensor&, const Tensor&, int64_t n_mels) {
  return at::empty({wave.size(0), n_mels, kFrames}, wave.options());
}

// ---- large-M / skinny bf16 GEMM with the fused epilogues (modeling_whisper.py projections, FFN, conv stem) --------
void gemm_bf16_out(const Tensor& A, const Tensor& W, int64_t epi, Tensor& out, const c10::optional<Tensor>& bias,
                   const c10::optional<Tensor>& aux, int64_t aux_rows, at::OptionalIntArrayRef kv_geom) {
  TW_OP_DEVICE(A);
  dev(A, at::kBFloat16, "A");
  dev(W, at::kBFloat16, "W");
  rows(A, "A");
  rows(W, "W");
  TORCH_CHECK(A.size(1) == W.size(1), "A and W disagree on K");
  const bool bf_out = epi == TW_EPI_BF16 || epi == TW_EPI_GELU_BF16 || epi == TW_EPI_CROSSKV;
  dev(out, bf_out ? at::kBFloat16 : at::kFloat, "out");
  same_device(A, W, "W");
  same_device(A, out, "out");
  const int M = (int)A.size(0), N = (int)W.size(0), K = (int)A.size(1);
  opt_holds(A, bias, at::kFloat, N, "bias");
  int geom[4] = {0, 0, 0, 0};
  int ldo = N;
  if (epi == TW_EPI_CROSSKV) {
    TORCH_CHECK(kv_geom.has_value() && kv_geom->size() == 4, "CROSSKV needs kv_geom = [S, B, D, H]");
    for (int i = 0; i < 4; ++i) geom[i] = (int)(*kv_geom)[i];
    TORCH_CHECK(out.is_contiguous(), "CROSSKV out must be contiguous");
    TORCH_CHECK(out.numel() >= (int64_t)M * N, "CROSSKV out too small");
  } else {
    rows(out, "out");
    TORCH_CHECK(out.size(0) >= M && out.size(1) >= N, "out too small");
    ldo = (int)out.stride(0);
    // (the bf16 epilogues store 16-byte vectors: rows must start 16-byte aligned)
    TORCH_CHECK(!bf_out || ldo % 8 == 0, "bf16 out needs a row stride that is a multiple of 8 elements");
  }
  if (epi == TW_EPI_GELU_POS_F32) {
    TORCH_CHECK(aux.has_value() && aux->defined() && aux_rows > 0, "GELU_POS_F32 needs aux and aux_rows");
    // aux[m % aux_rows][n] is indexed with the output's row stride
    TORCH_CHECK(ldo == N, "GELU_POS_F32 needs out rows of exactly N (the aux stride)");
    holds(A, *aux, at::kFloat, (int64_t)aux_rows * N, "aux");
  } else {
    opt_holds(A, aux, at::kFloat, 0, "aux");
  }
  ok(tw_gemm_bf16(ptr<uint16_t>(A), ptr<uint16_t>(W), M, N, K, (int)A.stride(0), (int)W.stride(0), (int)epi,
                  out.data_ptr(), ldo, optr<float>(bias), optr<float>(aux), (int)aux_rows,
                  epi == TW_EPI_CROSSKV ? geom : nullptr, cur_stream(A)),
     "gemm_bf16");
}

at::ScalarType gemm_out_type(int64_t epi) {
  TORCH_CHECK(epi == TW_EPI_BF16 || epi == TW_EPI_GELU_BF16 || epi == TW_EPI_F32,
              "tw::gemm_bf16 (functional) takes the BF16, GELU_BF16 or F32 epilogue; the in-place ones: gemm_bf16_out");
  return epi == TW_EPI_F32 ? at::kFloat : at::kBFloat16;
}

Tensor gemm_bf16(const Tensor& A, const Tensor& W, int64_t epi, const c10::optional<Tensor>& bias) {
  Tensor out = at::empty({A.size(0), W.size(0)}, A.options().dtype(gemm_out_type(epi)));
  gemm_bf16_out(A, W, epi, out, bias, c10::nullopt, 0, c10::nullopt);
  return out;
}

Tensor gemm_bf16_meta(const Tensor& A, const Tensor& W, int64_t epi, const c10::optional<Tensor>&) {
  return at::empty({A.size(0), W.size(0)}, A.options().dtype(gemm_out_type(epi)));
}

// ---- encoder self-attention (WhisperSdpaAttention / eager attention, modeling_whisper.py:215-238) ----------------
void attn_encoder_out(const Tensor& qkv, int64_t batch, int64_t heads, Tensor& out) {
  TW_OP_DEVICE(qkv);
  dev(qkv, at::kBFloat16, "qkv");
  dev(out, at::kBFloat16, "out");
  TORCH_CHECK(qkv.is_contiguous() && out.is_contiguous(), "qkv / out must be contiguous");
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(1) == 3 * heads * 64 && qkv.size(0) % batch == 0,
              "qkv must be [batch * S][3 * heads * 64]");
  TORCH_CHECK(out.numel() >= qkv.size(0) * heads * 64, "out too small");
  same_device(qkv, out, "out");
  ok(tw_attn_encoder(ptr<uint16_t>(qkv), (int)batch, (int)(qkv.size(0) / batch), (int)heads, ptr<uint16_t>(out),
                     cur_stream(qkv)),
     "attn_encoder");
}

Tensor attn_encoder(const Tensor& qkv, int64_t batch, int64_t heads) {
  Tensor out = at::empty({qkv.size(0), heads * 64}, qkv.options());
  attn_encoder_out(qkv, batch, heads, out);
  return out;
}

Tensor attn_encoder_meta(const Tensor& qkv, int64_t, int64_t heads) {
  return at::empty({qkv.size(0), heads * 64}, qkv.options());
}

// ---- encoder LayerNorm ---------------------------------------------------------------------------------------------
void layernorm_out(const Tensor& x, const Tensor& gamma, const Tensor& beta, double eps, Tensor& out) {
  TW_OP_DEVICE(x);
  dev(x, at::kFloat, "x");
  dev(out, at::kBFloat16, "out");
  dev(gamma, at::kFloat, "gamma");
  dev(beta, at::kFloat, "beta");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.dim() == 2 && out.numel() >= x.numel(), "x [M][D]");
  holds(x, gamma, at::kFloat, x.size(1), "gamma");
  holds(x, beta, at::kFloat, x.size(1), "beta");
  same_device(x, out, "out");
  ok(tw_layernorm(ptr<float>(x), ptr<float>(gamma), ptr<float>(beta), (int)x.size(0), (int)x.size(1), (float)eps,
                  ptr<uint16_t>(out), cur_stream(x)),
     "layernorm");
}

Tensor layernorm(const Tensor& x, const Tensor& gamma, const Tensor& beta, double eps) {
  Tensor out = at::empty(x.sizes(), x.options().dtype(at::kBFloat16));
  layernorm_out(x, gamma, beta, eps, out);
  return out;
}

Tensor layernorm_meta(const Tensor& x, const Tensor&, const Tensor&, double) {
  return at::empty(x.sizes(), x.options().dtype(at::kBFloat16));
}

// ---- decoder step pieces (WhisperDecoderLayer.forward, modeling_whisper.py:448-505) ---------------------------------
void gemv_packed_out(const Tensor& A, bool a_packed, const Tensor& Wp, int64_t M, int64_t N, int64_t K, int64_t epi,
                     Tensor& out, const c10::optional<Tensor>& bias, int64_t splits) {
  TW_OP_DEVICE(A);
  dev(A, at::kBFloat16, "A");
  dev(Wp, at::kBFloat16, "Wp");
  TORCH_CHECK(Wp.numel() >= ((N + 15) / 16) * 16 * K, "Wp too small for [N][K] packed");
  same_device(A, Wp, "Wp");
  TORCH_CHECK(M >= 1 && M <= 64 && K % 32 == 0 && N >= 1, "gemv_packed: 1 <= M <= 64 rows, K % 32 == 0");
  TORCH_CHECK(splits >= 1 && (splits == 1 || epi == TW_EPI_PARTIAL_F32), "splits > 1 only with PARTIAL_F32");
  // a packed activation spans [K/32][M <= 32 ? 2 : 4][64][8]; a row-major one [M][lda]
  TORCH_CHECK(A.numel() >= (a_packed ? (K / 32) * (M > 32 ? 4 : 2) * 512 : (M - 1) * A.stride(0) + K),
              "A too small for ", M, " rows of K = ", K);
  const bool f32 = epi == TW_EPI_F32 || epi == TW_EPI_RESID_F32 || epi == TW_EPI_PARTIAL_F32;
  const int ldo = epi == TW_EPI_GELU_PACKED ? 0 : (int)N;
  holds(A, out, f32 ? at::kFloat : at::kBFloat16,
        epi == TW_EPI_GELU_PACKED ? (K > 0 ? ((N + 31) / 32) * (M > 32 ? 4 : 2) * 512 : 0)
                                  : (epi == TW_EPI_PARTIAL_F32 ? splits : 1) * M * N,
        "out");
  opt_holds(A, bias, at::kFloat, N, "bias");
  ok(tw_gemv_packed(ptr<uint16_t>(A), a_packed ? 1 : 0, a_packed ? (int)K : (int)A.stride(0), ptr<uint16_t>(Wp),
                    (int)M, (int)N, (int)K, (int)epi, out.data_ptr(), ldo, optr<float>(bias), (int)splits,
                    cur_stream(A)),
     "gemv_packed");
}

void resid_layernorm_packed_(Tensor& x, const c10::optional<Tensor>& parts, int64_t nparts,
                             const c10::optional<Tensor>& bias, const Tensor& gamma, const Tensor& beta, double eps,
                             Tensor& out) {
  TW_OP_DEVICE(x);
  dev(x, at::kFloat, "x");
  dev(out, at::kBFloat16, "out");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "x must be [M][D]");
  const int64_t M = x.size(0), D = x.size(1);
  TORCH_CHECK(M >= 1 && M <= 64 && D % 32 == 0, "resid_layernorm_packed: M <= 64, D % 32 == 0");
  opt_holds(x, parts, at::kFloat, nparts * M * D, "parts");
  opt_holds(x, bias, at::kFloat, D, "bias");
  holds(x, gamma, at::kFloat, D, "gamma");
  holds(x, beta, at::kFloat, D, "beta");
  holds(x, out, at::kBFloat16, (D / 32) * (M > 32 ? 4 : 2) * 512, "out");
  ok(tw_resid_layernorm_packed(ptr<float>(x), optr<float>(parts), (int)nparts, optr<float>(bias), ptr<float>(gamma),
                               ptr<float>(beta), (int)x.size(0), (int)x.size(1), (float)eps, ptr<uint16_t>(out),
                               cur_stream(x)),
     "resid_layernorm_packed");
}

void attn_decode_self_(const Tensor& qkv, int64_t heads, int64_t max_pos, const Tensor& pos, Tensor& k_cache,
                       Tensor& v_cache, Tensor& out) {
  TW_OP_DEVICE(qkv);
  dev(qkv, at::kBFloat16, "qkv");
  TORCH_CHECK(qkv.dim() == 2 && qkv.is_contiguous() && qkv.size(1) == 3 * heads * 64, "qkv must be [B][3 H 64]");
  const int64_t B = qkv.size(0);
  holds(qkv, pos, at::kInt, B, "pos");
  holds(qkv, k_cache, at::kBFloat16, B * heads * max_pos * 64, "k_cache");
  holds(qkv, v_cache, at::kBFloat16, B * heads * max_pos * 64, "v_cache");
  holds(qkv, out, at::kBFloat16, B * heads * 64, "out");
  ok(tw_attn_decode_self(ptr<uint16_t>(qkv), (int)qkv.size(0), (int)heads, (int)max_pos, ptr<int>(pos),
                         ptr<uint16_t>(k_cache), ptr<uint16_t>(v_cache), ptr<uint16_t>(out), cur_stream(qkv)),
     "attn_decode_self");
}

void attn_decode_cross_out(const Tensor& q, int64_t heads, int64_t S, int64_t Bt, const c10::optional<Tensor>& row_map,
                           const Tensor& cross_kv, Tensor& out) {
  TW_OP_DEVICE(q);
  dev(q, at::kBFloat16, "q");
  TORCH_CHECK(q.dim() == 2 && q.is_contiguous() && q.size(1) == heads * 64, "q must be [B][H 64]");
  const int64_t B = q.size(0);
  TORCH_CHECK(row_map.has_value() && row_map->defined() ? true : B <= Bt, "without row_map B must be <= Bt");
  holds(q, cross_kv, at::kBFloat16, 2 * Bt * heads * S * 64, "cross_kv");
  opt_holds(q, row_map, at::kInt, B, "row_map");
  holds(q, out, at::kBFloat16, B * heads * 64, "out");
  ok(tw_attn_decode_cross(ptr<uint16_t>(q), (int)q.size(0), (int)heads, (int)S, (int)Bt, optr<int>(row_map),
                          ptr<uint16_t>(cross_kv), ptr<uint16_t>(out), cur_stream(q)),
     "attn_decode_cross");
}

// the Whisper logits processors + greedy argmax (logits_process.py:1816-2047, generation/utils.py:2876-2941);
// params = TwSelectParams as 20 ints (V, eos, pad, ts_begin, no_timestamps, max_initial_ts, use_timestamps, max_new,
// mode, lo, hi, n_begin_suppress, begin_suppress[8])
void logits_select_(const Tensor& logits, const Tensor& suppress_bits, at::IntArrayRef params, Tensor& state,
                    const c10::optional<Tensor>& tokens, Tensor& ids, Tensor& pos, Tensor& workspace) {
  TW_OP_DEVICE(logits);
  dev(logits, at::kFloat, "logits");
  rows(logits, "logits");
  TORCH_CHECK(params.size() == 20, "params: 20 ints (TwSelectParams)");
  const int64_t B = logits.size(0), V = params[0];
  TORCH_CHECK(logits.size(1) >= V, "logits narrower than V");
  holds(logits, suppress_bits, at::kInt, (V + 31) / 32, "suppress_bits");
  holds(logits, state, at::kInt, B * TW_STATE_STRIDE, "state");
  holds(logits, ids, at::kInt, B, "ids");
  holds(logits, pos, at::kInt, B, "pos");
  holds(logits, workspace, at::kFloat, B * TW_SELECT_WS_PER_ROW, "workspace");
  if (tokens.has_value() && tokens->defined()) {
    dev(*tokens, at::kInt, "tokens");
    same_device(logits, *tokens, "tokens");
    rows(*tokens, "tokens");
    TORCH_CHECK(tokens->size(0) >= B, "tokens must hold B rows");
  }
  TwSelectParams p;
  int32_t* f = &p.V;
  for (int i = 0; i < 12; ++i) f[i] = (int32_t)params[i];
  for (int i = 0; i < 8; ++i) p.begin_suppress[i] = (int32_t)params[12 + i];
  const Tensor* tk = tokens.has_value() && tokens->defined() ? &*tokens : nullptr;
  ok(tw_logits_select(ptr<float>(logits), (int)logits.size(0), (int)logits.stride(0), ptr<uint32_t>(suppress_bits),
                      &p, ptr<int>(state), tk ? ptr<int>(*tk) : nullptr, tk ? (int)tk->stride(0) : 0, ptr<int>(ids),
                      ptr<int>(pos), ptr<float>(workspace), cur_stream(logits)),
     "logits_select");
}

}  // namespace

TORCH_LIBRARY(tw, m) {
  m.def("logmel(Tensor wave, Tensor basis_cos, Tensor basis_sin, Tensor mel_fb, int n_mels) -> Tensor");
  m.def("logmel_out(Tensor wave, Tensor basis_cos, Tensor basis_sin, Tensor mel_fb, int n_mels, Tensor(a!) out, "
        "Tensor(b!) maxkeys) -> ()");
  m.def("gemm_bf16(Tensor A, Tensor W, int epi, Tensor? bias=None) -> Tensor");
  m.def("gemm_bf16_out(Tensor A, Tensor W, int epi, Tensor(a!) out, Tensor? bias=None, Tensor? aux=None, "
        "int aux_rows=0, int[]? kv_geom=None) -> ()");
  m.def("attn_encoder(Tensor qkv, int batch, int heads) -> Tensor");
  m.def("attn_encoder_out(Tensor qkv, int batch, int heads, Tensor(a!) out) -> ()");
  m.def("layernorm(Tensor x, Tensor gamma, Tensor beta, float eps) -> Tensor");
  m.def("layernorm_out(Tensor x, Tensor gamma, Tensor beta, float eps, Tensor(a!) out) -> ()");
  m.def("gemv_packed_out(Tensor A, bool a_packed, Tensor Wp, int M, int N, int K, int epi, Tensor(a!) out, "
        "Tensor? bias=None, int splits=1) -> ()");
  m.def("resid_layernorm_packed_(Tensor(a!) x, Tensor? parts, int nparts, Tensor? bias, Tensor gamma, Tensor beta, "
        "float eps, Tensor(b!) out) -> ()");
  m.def("attn_decode_self_(Tensor qkv, int heads, int max_pos, Tensor pos, Tensor(a!) k_cache, Tensor(b!) v_cache, "
        "Tensor(c!) out) -> ()");
  m.def("attn_decode_cross_out(Tensor q, int heads, int S, int Bt, Tensor? row_map, Tensor cross_kv, "
        "Tensor(a!) out) -> ()");
  m.def("logits_select_(Tensor logits, Tensor suppress_bits, int[] params, Tensor(a!) state, Tensor(b!)? tokens, "
        "Tensor(c!) ids, Tensor(d!) pos, Tensor(e!) workspace) -> ()");
}

TORCH_LIBRARY_IMPL(tw, CUDA, m) {  // (the dispatch key of device tensors; on this ROCm build they are HIP tensors)
  m.impl("logmel", &logmel);
  m.impl("logmel_out", &logmel_out);
  m.impl("gemm_bf16", &gemm_bf16);
  m.impl("gemm_bf16_out", &gemm_bf16_out);
  m.impl("attn_encoder", &attn_encoder);
  m.impl("attn_encoder_out", &attn_encoder_out);
  m.impl("layernorm", &layernorm);
  m.impl("layernorm_out", &layernorm_out);
  m.impl("gemv_packed_out", &gemv_packed_out);
  m.impl("resid_layernorm_packed_", &resid_layernorm_packed_);
  m.impl("attn_decode_self_", &attn_decode_self_);
  m.impl("attn_decode_cross_out", &attn_decode_cross_out);
  m.impl("logits_select_", &logits_select_);
}

TORCH_LIBRARY_IMPL(tw, Meta, m) {  // shape functions (FakeTensor / tracing); the out= and in-place ops write nothing
  m.impl("logmel", &logmel_meta);
  m.impl("gemm_bf16", &gemm_bf16_meta);
  m.impl("attn_encoder", &attn_encoder_meta);
  m.impl("layernorm", &layernorm_meta);
  m.impl("logmel_out", [](const Tensor&, const Tensor&, const Tensor&, const Tensor&, int64_t, Tensor&, Tensor&) {});
  m.impl("gemm_bf16_out", [](const Tensor&, const Tensor&, int64_t, Tensor&, const c10::optional<Tensor>&,
                             const c10::optional<Tensor>&, int64_t, at::OptionalIntArrayRef) {});
  m.impl("attn_encoder_out", [](const Tensor&, int64_t, int64_t, Tensor&) {});
  m.impl("layernorm_out", [](const Tensor&, const Tensor&, const Tensor&, double, Tensor&) {});
  m.impl("gemv_packed_out", [](const Tensor&, bool, const Tensor&, int64_t, int64_t, int64_t, int64_t, Tensor&,
                               const c10::optional<Tensor>&, int64_t) {});
  m.impl("resid_layernorm_packed_", [](Tensor&, const c10::optional<Tensor>&, int64_t, const c10::optional<Tensor>&,
                                       const Tensor&, const Tensor&, double, Tensor&) {});
  m.impl("attn_decode_self_", [](const Tensor&, int64_t, int64_t, const Tensor&, Tensor&, Tensor&, Tensor&) {});
  m.impl("attn_decode_cross_out", [](const Tensor&, int64_t, int64_t, int64_t, const c10::optional<Tensor>&,
                                     const Tensor&, Tensor&) {});
  m.impl("logits_select_", [](const Tensor&, const Tensor&, at::IntArrayRef, Tensor&, const c10::optional<Tensor>&,
                              Tensor&, Tensor&, Tensor&) {});
}
