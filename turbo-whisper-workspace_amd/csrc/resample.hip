// Downmix + polyphase resampling to 16 kHz on the GPU (include/tw_audio.h), the resampling half of the
// reference's `ffmpeg -ac 1 -ar 16000 -f f32le` ingest ($TF/pipelines/audio_utils.py:9-45). The filter bank is
// designed on the host (twamd/audio.py: swr_filter_bank, libswresample's default Kaiser-windowed sinc).
//
// One block = 256 consecutive outputs. Their input footprint (256*down/up + ntaps samples) is converted once
// (int32 -> f32 * scale, channel mean, end reflection) into LDS with coalesced loads; the bank lives in LDS
// too when it fits in 64 KiB with the footprint (every rate pair from 8 kHz to 192 kHz does). Each thread then
// runs its output's ntaps-long dot product out of LDS. For one hour of 192 kHz mono this is 2.8 GB of int32
// reads (~0.5 ms of HBM time) and 23 GMAC — a few ms of VALU time, negligible next to the transcription.
#include "tw_common.h"
#include "../../include/tw_audio.h"

namespace {

constexpr int RS_BLOCK = 256;
constexpr long RS_LDS_FLOATS = 16384;  // 64 KiB of dynamic LDS

__device__ __forceinline__ long reflect_idx(long j, long n) {
  if (j < 0) j = -j;
  if (j >= n) j = 2 * (n - 1) - j;
  return j < 0 ? 0 : (j >= n ? n - 1 : j);  // inputs shorter than the reflection span
}

template <typename In>
__device__ __forceinline__ float load_mono(const In* x, long t, int ch, float scale) {
  float s = 0.f;
  for (int c = 0; c < ch; c++) s += (float)x[t * ch + c];
  return ch == 1 ? s * scale : s * (scale / (float)ch);
}

template <typename In, bool TAPS_LDS>
__global__ __launch_bounds__(RS_BLOCK) void k_resample(const In* __restrict__ x, long n_in, int ch, float scale,
                                                       int up, int down, const float* __restrict__ taps, int T,
                                                       float* __restrict__ y, long n_out) {
  extern __shared__ float sm[];
  const int tid = threadIdx.x;
  const long n0 = (long)blockIdx.x * RS_BLOCK;
  const long n1 = min(n0 + RS_BLOCK, n_out) - 1;
  const long c = (T - 1) / 2;
  const long i_lo = (n0 * down) / up - c;
  const long cnt = (n1 * down) / up - c + T - i_lo;
  float* tb = sm;
  float* xs = TAPS_LDS ? sm + (long)up * T : sm;
  if (TAPS_LDS)
    for (long j = tid; j < (long)up * T; j += RS_BLOCK) tb[j] = taps[j];
  for (long j = tid; j < cnt; j += RS_BLOCK) xs[j] = load_mono(x, reflect_idx(i_lo + j, n_in), ch, scale);
  __syncthreads();
  const long n = n0 + tid;
  if (n > n1) return;
  const long q = n * down;
  const int ph = (int)(q % up);
  const float* h = (TAPS_LDS ? tb : taps) + (long)ph * T;
  const float* xv = xs + (q / up - c - i_lo);
  float acc = 0.f;
  for (int i = 0; i < T; i++) acc = fmaf(h[i], xv[i], acc);
  y[n] = acc;
}

template <typename In>
int launch(const In* x, long n_in, int ch, float scale, int up, int down, const float* taps, int T, float* y,
           long n_out, void* stream, const char* name) {
  TW_REQUIRE(x && taps && y && n_in > 0 && n_out > 0, "%s: null pointer or empty signal", name);
  TW_REQUIRE(ch >= 1 && ch <= 8 && up >= 1 && down >= 1 && T >= 1, "%s: bad channels/ratio/taps", name);
  TW_REQUIRE(n_out <= (n_in * up + down - 1) / down, "%s: n_out exceeds ceil(n_in*up/down)", name);
  const long foot = (long)(RS_BLOCK - 1) * down / up + 2 + T;
  TW_REQUIRE(foot <= RS_LDS_FLOATS, "%s: ratio %d/%d with %d taps needs %ld LDS floats", name, up, down, T, foot);
  const bool taps_lds = foot + (long)up * T <= RS_LDS_FLOATS;
  const size_t lds = sizeof(float) * (size_t)(foot + (taps_lds ? (long)up * T : 0));
  const unsigned grid = tw_cdiv(n_out, RS_BLOCK);
  hipStream_t s = (hipStream_t)stream;
  if (taps_lds)
    hipLaunchKernelGGL((k_resample<In, true>), dim3(grid), dim3(RS_BLOCK), lds, s, x, n_in, ch, scale, up, down,
                       taps, T, y, n_out);
  else
    hipLaunchKernelGGL((k_resample<In, false>), dim3(grid), dim3(RS_BLOCK), lds, s, x, n_in, ch, scale, up, down,
                       taps, T, y, n_out);
  return tw_check_launch(name);
}

}  // namespace

extern "C" int tw_resample_pcm_i32(const int32_t* pcm, int64_t n_in, int32_t channels, float scale, int32_t up,
                                   int32_t down, const float* taps, int32_t ntaps, float* y, int64_t n_out,
                                   void* stream) {
  return launch(pcm, (long)n_in, channels, scale, up, down, taps, ntaps, y, (long)n_out, stream,
                "tw_resample_pcm_i32");
}

extern "C" int tw_resample_pcm_f32(const float* x, int64_t n_in, int32_t channels, int32_t up, int32_t down,
                                   const float* taps, int32_t ntaps, float* y, int64_t n_out, void* stream) {
  return launch(x, (long)n_in, channels, 1.0f, up, down, taps, ntaps, y, (long)n_out, stream,
                "tw_resample_pcm_f32");
}
