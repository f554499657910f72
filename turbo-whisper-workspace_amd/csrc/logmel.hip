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
// The basis and the filterbank arrive in "k8" order (tw_whisper.h: [K/8][cols][2][4]), so one 16-byte load
// gives a lane its B values for four MFMA steps: the kernel was bound by the L2 latency of one 4-byte load
// per MFMA (every workgroup streams the 717 KB basis), 1.18 ms for 24 windows.
#include "tw_common.h"
#include "../../include/tw_whisper.h"

#define LM_NFFT 400
#define LM_HOP 160
#define LM_FRAMES 3000
#define LM_SAMPLES 480000
#define LM_FP 224   // 201 frequency bins padded to 7 tiles of 32
#define LM_XS 401   // LDS row stride (floats) of the frame matrix
#define LM_PS 225   // LDS row stride (floats) of the power tile

// Geometry: row b of the wave holds n_samples samples at stride wave_ld; its n_frames frames go to
// feats[b][mel][0 .. n_frames) at row stride feats_ld (30-s windows: 480000, 3000, 3000; a long-form input: its own
// length, n_samples / 160 frames, reflect padding only at its two ends).
__global__ __launch_bounds__(256) void k_logmel(const float* __restrict__ wave, const float* __restrict__ bcos,
                                                const float* __restrict__ bsin, const float* __restrict__ fb,
                                                int n_mels, int mp, float* __restrict__ feats,
                                                uint32_t* __restrict__ maxkeys, long n_samples, long wave_ld,
                                                int n_frames, long feats_ld) {
  extern __shared__ __attribute__((aligned(16))) float lm_smem[];
  float* xs = lm_smem;                 // [32][401]
  float* ps = lm_smem + 32 * LM_XS;    // [32][225]
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * 32;
  const float* w = wave + (size_t)b * wave_ld;

  for (int e = threadIdx.x; e < 32 * LM_NFFT; e += 256) {
    int i = e / LM_NFFT, n = e - i * LM_NFFT;
    int t = t0 + i;
    float v = 0.f;
    if (t < n_frames) {
      long j = (long)t * LM_HOP - LM_NFFT / 2 + n;
      if (j < 0) j = -j;
      else if (j >= n_samples) j = 2 * (n_samples - 1) - j;
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
    // step n0 = 8 g + 2 j: lane (li, lk) multiplies frame li's sample n0 + lk by basis[n0 + lk][f] = k8[g][f][lk][j]
    const float4* pc = (const float4*)bcos + f * 2 + lk;
    const float4* psn = (const float4*)bsin + f * 2 + lk;
#pragma unroll 5
    for (int g = 0; g < LM_NFFT / 8; ++g) {
      const float4 bc = pc[g * LM_FP * 2], bs = psn[g * LM_FP * 2];
      const float* xr = xs + li * LM_XS + 8 * g + lk;
      const float bcv[4] = {bc.x, bc.y, bc.z, bc.w}, bsv[4] = {bs.x, bs.y, bs.z, bs.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = xr[2 * j];
        re = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bcv[j], re, 0, 0, 0);
        im = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bsv[j], im, 0, 0, 0);
      }
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
    const float4* pf = (const float4*)fb + m * 2 + lk;  // fb[f0 + lk][m] = k8[g][m][lk][j], f0 = 8 g + 2 j
#pragma unroll 7
    for (int g = 0; g < LM_FP / 8; ++g) {
      const float4 b4 = pf[g * mp * 2];
      const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
      const float* pr = ps + li * LM_PS + 8 * g + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(pr[2 * j], bv[j], acc, 0, 0, 0);
    }
    if (m < n_mels) {
      float* dst = feats + ((size_t)b * n_mels + m) * feats_ld;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int t = t0 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (t < n_frames) {
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

__global__ void k_logmel_finalize(float* __restrict__ feats, const uint32_t* __restrict__ maxkeys, int n_mels,
                                  int n_frames, long feats_ld, long total) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < total; i += stride) {
    const long row = i / n_frames;  // b * n_mels + mel
    float* p = feats + row * feats_ld + (i - row * n_frames);
    float mx = f32_from_order_key(maxkeys[row / n_mels]);
    float v = fmaxf(*p, mx - 8.0f);
    *p = (v + 4.0f) / 4.0f;
  }
}

static int logmel_launch(const float* wave, int n_chunks, long n_samples, long wave_ld, const float* basis_cos,
                         const float* basis_sin, const float* mel_fb, int n_mels, float* feats, int n_frames,
                         long feats_ld, uint32_t* maxkeys, hipStream_t s) {
  int mp = (n_mels + 31) / 32 * 32;
  (void)hipMemsetAsync(maxkeys, 0, sizeof(uint32_t) * n_chunks, s);
  size_t lds = sizeof(float) * 32 * (LM_XS + LM_PS);
  hipLaunchKernelGGL(k_logmel, dim3(tw_cdiv(n_frames, 32), n_chunks), dim3(256), lds, s, wave, basis_cos, basis_sin,
                     mel_fb, n_mels, mp, feats, maxkeys, n_samples, wave_ld, n_frames, feats_ld);
  int rc = tw_check_launch("tw_logmel");
  if (rc) return rc;
  long total = (long)n_chunks * n_mels * n_frames;
  unsigned grid = tw_cdiv(total, 256);
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(k_logmel_finalize, dim3(grid), dim3(256), 0, s, feats, maxkeys, n_mels, n_frames, feats_ld, total);
  return tw_check_launch("tw_logmel_finalize");
}

extern "C" int tw_logmel(const float* wave, int n_chunks, const float* basis_cos, const float* basis_sin,
                         const float* mel_fb, int n_mels, float* feats, uint32_t* maxkeys, void* stream) {
  TW_REQUIRE(wave && basis_cos && basis_sin && mel_fb && feats && maxkeys, "tw_logmel: null pointer");
  TW_REQUIRE(n_chunks > 0 && n_mels > 0 && n_mels <= 128, "tw_logmel: n_chunks=%d n_mels=%d", n_chunks, n_mels);
  return logmel_launch(wave, n_chunks, LM_SAMPLES, LM_SAMPLES, basis_cos, basis_sin, mel_fb, n_mels, feats, LM_FRAMES,
                       LM_FRAMES, maxkeys, (hipStream_t)stream);
}

extern "C" int tw_logmel_long(const float* wave, long n_samples, const float* basis_cos, const float* basis_sin,
                              const float* mel_fb, int n_mels, float* feats, long feats_ld, uint32_t* maxkey,
                              void* stream) {
  TW_REQUIRE(wave && basis_cos && basis_sin && mel_fb && feats && maxkey, "tw_logmel_long: null pointer");
  TW_REQUIRE(n_mels > 0 && n_mels <= 128 && n_samples > LM_NFFT / 2 && n_samples / LM_HOP <= feats_ld &&
                 n_samples / LM_HOP < (1L << 30),
             "tw_logmel_long: n_samples=%ld n_mels=%d feats_ld=%ld", n_samples, n_mels, feats_ld);
  return logmel_launch(wave, 1, n_samples, n_samples, basis_cos, basis_sin, mel_fb, n_mels, feats,
                       (int)(n_samples / LM_HOP), feats_ld, maxkey, (hipStream_t)stream);
}
