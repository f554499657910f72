// Dynamic time warping for token-level timestamps (host side, include/tw_whisper.h: tw_dtw).
//
// The alignment step of return_timestamps="word": WhisperGenerationMixin._extract_token_timestamps runs
// _dynamic_time_warping ($TF/models/whisper/generation_whisper.py:64-114) on -mean(alignment-head attention) in a
// pure-Python double loop; this is the same recurrence (float32 cost table, the diagonal move only when strictly
// cheaper than both others, the vertical move only when strictly cheaper than both others, otherwise horizontal)
// and the same backtrace, in C++.
#include <stdint.h>

#include <cmath>
#include <vector>

void tw_set_error(const char* fmt, ...);

extern "C" int tw_dtw(const double* matrix, int32_t n, int32_t m, int32_t* text_idx, int32_t* time_idx,
                      int32_t* path_len) {
  if (!matrix || !text_idx || !time_idx || !path_len || n <= 0 || m <= 0) {
    tw_set_error("tw_dtw: bad arguments");
    return 1;
  }
  const size_t W = (size_t)m + 1;
  std::vector<float> cost((size_t)(n + 1) * W, INFINITY);
  std::vector<int8_t> trace((size_t)(n + 1) * W, -1);
  cost[0] = 0.f;
  for (int j = 1; j <= m; ++j) {
    for (int i = 1; i <= n; ++i) {
      const float c0 = cost[(size_t)(i - 1) * W + (j - 1)];
      const float c1 = cost[(size_t)(i - 1) * W + j];
      const float c2 = cost[(size_t)i * W + (j - 1)];
      float c;
      int8_t t;
      if (c0 < c1 && c0 < c2) {
        c = c0;
        t = 0;
      } else if (c1 < c0 && c1 < c2) {
        c = c1;
        t = 1;
      } else {
        c = c2;
        t = 2;
      }
      cost[(size_t)i * W + j] = (float)(matrix[(size_t)(i - 1) * m + (j - 1)] + (double)c);
      trace[(size_t)i * W + j] = t;
    }
  }
  for (int j = 0; j <= m; ++j) trace[j] = 2;
  for (int i = 0; i <= n; ++i) trace[(size_t)i * W] = 1;
  int i = n, j = m, k = 0;
  std::vector<int32_t> ti, tj;
  ti.reserve(n + m);
  tj.reserve(n + m);
  while (i > 0 || j > 0) {
    ti.push_back(i - 1);
    tj.push_back(j - 1);
    const int8_t t = trace[(size_t)i * W + j];
    if (t == 0) {
      --i;
      --j;
    } else if (t == 1) {
      --i;
    } else {
      --j;
    }
  }
  const int L = (int)ti.size();
  for (k = 0; k < L; ++k) {
    text_idx[k] = ti[L - 1 - k];
    time_idx[k] = tj[L - 1 - k];
  }
  *path_len = L;
  return 0;
}
