// Whisper log-mel front end on CDNA4.
//
// Restates WhisperFeatureExtractor._torch_extract_fbank_features
// ($TF/models/whisper/feature_extraction_whisper.py:135-168): periodic-Hann STFT (n_fft 400,
// hop 160, center=True reflect pad), |X|^2 of the first 3000 of 3001 frames, slaney mel
// filterbank (mel_filter_bank, $TF/audio_utils.py:638), log10(max(.,1e-10)), per-chunk
// max(x, max-8), (x+4)/4.
//
// Design: one workgroup = 32 frames of one chunk. The 32x400 frame matrix is staged once in LDS
// (row stride 401 floats -> conflict-free column reads), the windowed DFT runs as an exact-f32
// MFMA GEMM (v_mfma_f32_32x32x2_f32, a bit-exact fmaf chain) against a [400][224] cos/sin basis
// that stays L2-resident, |X|^2 goes to LDS (stride 225), and the mel projection is a second f32
// MFMA GEMM. The per-chunk max is an order-preserving uint atomicMax; a second tiny kernel applies
// clamp + affine. Output layout matches the reference: feats[b][mel][3000] f32.
#include "tw_common.h"
#include "../../include/tw_whisper.h"

#define LM_NFFT 400
#define LM_HOP 160
#define LM_FRAMES 3000
#define LM_SAMPLES 480000
#define LM_FP 224   // 201 frequency bins padded to 7 tiles of 32
#define LM_XS 401   // LDS row stride (floats) of the frame matrix
#define LM_PS 225   // LDS row stride (floats) of the power tile

__global__ __launch_bounds__(256) void k_logmel(const float* __restrict__ wave, const float* __restrict__ bcos,
                                                const float* __restrict__ bsin, const float* __restrict__ fb,
                                                int n_mels, int mp, float* __restrict__ feats,
                                                uint32_t* __restrict__ maxkeys) {
  extern __shared__ __attribute__((aligned(16))) float lm_smem[];
  float* xs = lm_smem;                 // [32][401]
  float* ps = lm_smem + 32 * LM_XS;    // [32][225]
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * 32;
  const float* w = wave + (size_t)b * LM_SAMPLES;

  for (int e = threadIdx.x; e < 32 * LM_NFFT; e += 256) {
    int i = e / LM_NFFT, n = e - i * LM_NFFT;
    int t = t0 + i;
    float v = 0.f;
    if (t < LM_FRAMES) {
      int j = t * LM_HOP - LM_NFFT / 2 + n;
      if (j < 0) j = -j;
      else if (j >= LM_SAMPLES) j = 2 * (LM_SAMPLES - 1) - j;
      v = w[j];
    }
    xs[i * LM_XS + n] = v;
  }
  __syncthreads();

  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int li = lane & 31, lk = lane >> 5;
  for (int ft = wid; ft < LM_FP / 32; ft += 4) {
    f32x16 re = {0}, im = {0};
    const int f = ft * 32 + li;
#pragma unroll 8
    for (int n0 = 0; n0 < LM_NFFT; n0 += 2) {
      float a = xs[li * LM_XS + n0 + lk];
      float bc = bcos[(n0 + lk) * LM_FP + f];
      float bs = bsin[(n0 + lk) * LM_FP + f];
      re = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bc, re, 0, 0, 0);
      im = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bs, im, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int row = (r & 3) + 8 * (r >> 2) + 4 * lk;
      ps[row * LM_PS + f] = re[r] * re[r] + im[r] * im[r];
    }
  }
  __syncthreads();

  float lmax = -INFINITY;
  if (wid * 32 < mp) {
    f32x16 acc = {0};
    const int m = wid * 32 + li;
#pragma unroll 8
    for (int f0 = 0; f0 < LM_FP; f0 += 2) {
      float a = ps[li * LM_PS + f0 + lk];
      float bb = fb[(f0 + lk) * mp + m];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc, 0, 0, 0);
    }
    if (m < n_mels) {
      float* dst = feats + ((size_t)b * n_mels + m) * LM_FRAMES;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int t = t0 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (t < LM_FRAMES) {
          float v = log10f(fmaxf(acc[r], 1e-10f));
          dst[t] = v;
          lmax = fmaxf(lmax, v);
        }
      }
    }
  }
  lmax = wave_max(lmax);
  if (lane == 0 && lmax > -INFINITY) atomicMax(&maxkeys[b], f32_order_key(lmax));
}

__global__ void k_logmel_finalize(float* __restrict__ feats, const uint32_t* __restrict__ maxkeys, long per_chunk,
                                  long total) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < total; i += stride) {
    float mx = f32_from_order_key(maxkeys[i / per_chunk]);
    float v = fmaxf(feats[i], mx - 8.0f);
    feats[i] = (v + 4.0f) / 4.0f;
  }
}

extern "C" int tw_logmel(const float* wave, int n_chunks, const float* basis_cos, const float* basis_sin,
                         const float* mel_fb, int n_mels, float* feats, uint32_t* maxkeys, void* stream) {
  TW_REQUIRE(wave && basis_cos && basis_sin && mel_fb && feats && maxkeys, "tw_logmel: null pointer");
  TW_REQUIRE(n_chunks > 0 && n_mels > 0 && n_mels <= 128, "tw_logmel: n_chunks=%d n_mels=%d", n_chunks, n_mels);
  hipStream_t s = (hipStream_t)stream;
  int mp = (n_mels + 31) / 32 * 32;
  (void)hipMemsetAsync(maxkeys, 0, sizeof(uint32_t) * n_chunks, s);
  size_t lds = sizeof(float) * 32 * (LM_XS + LM_PS);
  hipLaunchKernelGGL(k_logmel, dim3(tw_cdiv(LM_FRAMES, 32), n_chunks), dim3(256), lds, s, wave, basis_cos, basis_sin,
                     mel_fb, n_mels, mp, feats, maxkeys);
  int rc = tw_check_launch("tw_logmel");
  if (rc) return rc;
  long total = (long)n_chunks * n_mels * LM_FRAMES;
  unsigned grid = tw_cdiv(total, 256);
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(k_logmel_finalize, dim3(grid), dim3(256), 0, s, feats, maxkeys, (long)n_mels * LM_FRAMES, total);
  return tw_check_launch("tw_logmel_finalize");
}
