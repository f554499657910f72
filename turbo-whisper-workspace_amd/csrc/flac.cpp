// Native FLAC decoder (host side of the audio ingest, include/tw_audio.h).
//
// Replaces the container-decode half of the reference's ffmpeg_read ($TF/pipelines/audio_utils.py:9-45), which
// the reference reaches for every file path it transcribes (vocalis/core/audio_pipeline.py:351 hands the path to
// the ASR pipeline; examples/Test1/ChrisAndAlexDiTest.flac is 192 kHz / 16-bit / mono FLAC). The decode follows
// the FLAC format specification (RFC 9639): STREAMINFO, frame header with UTF-8 coded frame/sample number and
// CRC-8, CONSTANT / VERBATIM / FIXED(0..4) / LPC(1..32) subframes with wasted bits, partitioned Rice residuals
// (4- and 5-bit parameters, escape codes), inter-channel decorrelation (left/side, side/right, mid/side), CRC-16.
//
// Parallelism: frames are independent, so the compressed stream is split into n_threads byte ranges; each worker
// finds the first genuine frame at or after its range start (sync code + header CRC-8 + full decode with a
// matching CRC-16) and decodes until it reaches the next worker's first frame. Each frame's position in the
// output comes from its own header (frame number x block size, or the sample number for variable blocking), so
// workers write disjoint slices without coordination. A worker that overruns its neighbour's start (a stream
// whose sync search was fooled) makes the whole decode fall back to one sequential pass.
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tw_audio.h"

void tw_set_error(const char* fmt, ...);

namespace {

uint8_t g_crc8[256];
uint16_t g_crc16[256];
struct CrcInit {
  CrcInit() {
    for (int i = 0; i < 256; i++) {
      uint8_t c = (uint8_t)i;
      for (int b = 0; b < 8; b++) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
      g_crc8[i] = c;
      uint16_t d = (uint16_t)(i << 8);
      for (int b = 0; b < 8; b++) d = (uint16_t)((d & 0x8000) ? (d << 1) ^ 0x8005 : (d << 1));
      g_crc16[i] = d;
    }
  }
} g_crc_init;

uint8_t crc8(const uint8_t* p, size_t n) {
  uint8_t c = 0;
  for (size_t i = 0; i < n; i++) c = g_crc8[c ^ p[i]];
  return c;
}
uint16_t crc16(const uint8_t* p, size_t n) {
  uint16_t c = 0;
  for (size_t i = 0; i < n; i++) c = (uint16_t)((c << 8) ^ g_crc16[(c >> 8) ^ p[i]]);
  return c;
}

// MSB-first bit reader over [d, d+n). Reads past the end return zeros and set `bad`.
struct Bits {
  const uint8_t* d;
  size_t n;
  uint64_t bit = 0;
  bool bad = false;

  Bits(const uint8_t* d_, size_t n_, size_t byte0) : d(d_), n(n_), bit((uint64_t)byte0 * 8) {}

  // 64 bits starting at `bit`; at least 57 of them are stream bits (the low bit&7 are zero fill)
  inline uint64_t peek() const {
    size_t b = (size_t)(bit >> 3);
    uint64_t v;
    if (b + 8 <= n) {
      memcpy(&v, d + b, 8);
      v = __builtin_bswap64(v);
    } else {
      v = 0;
      for (int i = 0; i < 8; i++) v = (v << 8) | (b + i < n ? d[b + i] : 0);
    }
    return v << (bit & 7);
  }
  inline uint32_t u(int k) {  // k in [0, 32]
    if (k == 0) return 0;
    uint32_t r = (uint32_t)(peek() >> (64 - k));
    bit += (uint64_t)k;
    if (bit > (uint64_t)n * 8) bad = true;
    return r;
  }
  inline int32_t s(int k) {  // k in [0, 32], two's complement
    if (k == 0) return 0;
    uint32_t v = u(k);
    return (int32_t)(v << (32 - k)) >> (32 - k);
  }
  inline uint32_t unary() {  // number of 0 bits before the next 1 bit
    uint32_t q = 0;
    for (;;) {
      uint64_t v = peek();
      if (v) {
        int lz = __builtin_clzll(v);
        if (lz < 57) {
          q += (uint32_t)lz;
          bit += (uint64_t)lz + 1;
          if (bit > (uint64_t)n * 8) bad = true;
          return q;
        }
      }
      q += 56;
      bit += 56;
      if (bit > (uint64_t)n * 8) {
        bad = true;
        return q;
      }
    }
  }
  inline void align() { bit = (bit + 7) & ~(uint64_t)7; }
  inline size_t byte() const { return (size_t)(bit >> 3); }
};

struct Header {
  int blocksize, channels, chan_assign, bps;
  int64_t first_sample;  // position of this frame's first sample in the stream (per channel)
  size_t hdr_bytes;
};

// Parse the frame header at byte `pos` (sync code included). Returns false if it is not a valid header.
bool parse_header(const uint8_t* d, size_t n, size_t pos, const TwFlacInfo& si, Header* h) {
  if (pos + 6 > n || d[pos] != 0xFF || (d[pos + 1] & 0xFE) != 0xF8) return false;
  Bits b(d, n, pos);
  b.u(15);
  int variable = (int)b.u(1);
  int bs_code = (int)b.u(4), sr_code = (int)b.u(4), ch_code = (int)b.u(4), ss_code = (int)b.u(3);
  if (b.u(1) != 0 || bs_code == 0 || sr_code == 15 || ch_code > 10 || ss_code == 3) return false;
  // UTF-8 style coded number (frame number for fixed blocking, sample number for variable blocking)
  uint32_t x = b.u(8);
  uint64_t num;
  int extra;
  if (!(x & 0x80)) {
    num = x;
    extra = 0;
  } else if ((x & 0xE0) == 0xC0) {
    num = x & 0x1F;
    extra = 1;
  } else if ((x & 0xF0) == 0xE0) {
    num = x & 0x0F;
    extra = 2;
  } else if ((x & 0xF8) == 0xF0) {
    num = x & 0x07;
    extra = 3;
  } else if ((x & 0xFC) == 0xF8) {
    num = x & 0x03;
    extra = 4;
  } else if ((x & 0xFE) == 0xFC) {
    num = x & 0x01;
    extra = 5;
  } else if (x == 0xFE) {
    num = 0;
    extra = 6;
  } else {
    return false;
  }
  for (int i = 0; i < extra; i++) {
    uint32_t c = b.u(8);
    if ((c & 0xC0) != 0x80) return false;
    num = (num << 6) | (c & 0x3F);
  }
  int bs;
  if (bs_code == 1) bs = 192;
  else if (bs_code <= 5) bs = 576 << (bs_code - 2);
  else if (bs_code == 6) bs = (int)b.u(8) + 1;
  else if (bs_code == 7) bs = (int)b.u(16) + 1;
  else bs = 256 << (bs_code - 8);
  if (sr_code == 12) b.u(8);
  else if (sr_code == 13 || sr_code == 14) b.u(16);
  static const int kSS[8] = {0, 8, 12, 0, 16, 20, 24, 32};
  int bps = ss_code == 0 ? si.bits_per_sample : kSS[ss_code];
  size_t hb = b.byte();
  if (b.bad || hb + 1 > n) return false;
  if (crc8(d + pos, hb - pos) != d[hb]) return false;
  h->blocksize = bs;
  h->chan_assign = ch_code;
  h->channels = ch_code < 8 ? ch_code + 1 : 2;
  h->bps = bps;
  if (variable) {
    h->first_sample = (int64_t)num;
  } else {
    if (si.min_blocksize != si.max_blocksize && si.max_blocksize != 0 && num != 0) return false;
    h->first_sample = (int64_t)num * (int64_t)si.max_blocksize;
  }
  h->hdr_bytes = hb + 1 - pos;
  if (h->channels != si.channels || bps < 4 || bps > 32) return false;
  if (si.max_blocksize && bs > si.max_blocksize) return false;
  return true;
}

bool residual(Bits& b, int bs, int order, int32_t* out) {
  int method = (int)b.u(2);
  if (method > 1) return false;
  int pbits = method == 0 ? 4 : 5, esc = method == 0 ? 15 : 31;
  int porder = (int)b.u(4);
  int psize = bs >> porder;
  if ((psize << porder) != bs || psize < order) return false;
  int i = order;
  for (int p = 0; p < (1 << porder); p++) {
    int cnt = psize - (p == 0 ? order : 0);
    int k = (int)b.u(pbits);
    if (k == esc) {
      int nb = (int)b.u(5);
      for (int j = 0; j < cnt; j++) out[i++] = b.s(nb);
    } else {
      for (int j = 0; j < cnt; j++) {
        uint32_t v;
        uint64_t w = b.peek();
        int lz = w ? __builtin_clzll(w) : 64;
        if (lz + 1 + k <= 57) {  // quotient, stop bit and remainder all inside one 64-bit window
          uint64_t rest = w << (lz + 1);
          v = ((uint32_t)lz << k) | (k ? (uint32_t)(rest >> (64 - k)) : 0u);
          b.bit += (uint64_t)(lz + 1 + k);
        } else {
          uint32_t q = b.unary();
          v = (q << k) | b.u(k);
        }
        out[i++] = (int32_t)(v >> 1) ^ -(int32_t)(v & 1);
      }
    }
    if (b.bit > (uint64_t)b.n * 8) b.bad = true;
    if (b.bad) return false;
  }
  return true;
}

// Sample arithmetic wraps modulo 2^32 (unsigned), never signed-overflows: a valid stream's samples and predictions
// fit their 32 bits, so the wrapped results are the exact ones, while a damaged upload (residuals far outside the
// frame's bit depth) decodes to garbage that its CRC-16 then rejects — not to undefined behaviour (found by the
// -fsanitize=undefined fuzz build, tests/test_codec_sanitize.py).
static inline int32_t wrap_add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }

template <typename Acc>
struct LpcAcc;
template <>
struct LpcAcc<int32_t> {  // the narrow path: exact for valid streams (see subframe()), modular otherwise
  static inline uint32_t mul(int32_t c, int32_t x) { return (uint32_t)c * (uint32_t)x; }
  static inline int32_t shifted(uint32_t acc, int shift) { return (int32_t)acc >> shift; }
  using T = uint32_t;
};
template <>
struct LpcAcc<int64_t> {  // |coef| < 2^15, |x| < 2^31: 32 terms stay far inside 64 bits
  static inline int64_t mul(int32_t c, int32_t x) { return (int64_t)c * (int64_t)x; }
  static inline int32_t shifted(int64_t acc, int shift) { return (int32_t)(acc >> shift); }
  using T = int64_t;
};

template <int ORDER, typename Acc>
void lpc_fixed_order(int32_t* out, int bs, const int32_t* coef, int shift) {
  int32_t c[ORDER];
  for (int j = 0; j < ORDER; j++) c[j] = coef[j];
  for (int i = ORDER; i < bs; i++) {
    typename LpcAcc<Acc>::T acc = 0;
#pragma GCC unroll 16
    for (int j = 0; j < ORDER; j++) acc += LpcAcc<Acc>::mul(c[j], out[i - 1 - j]);
    out[i] = wrap_add(out[i], LpcAcc<Acc>::shifted(acc, shift));
  }
}

template <typename Acc>
bool lpc_dispatch(int32_t* out, int bs, const int32_t* coef, int order, int shift) {
  switch (order) {
#define TW_LPC_CASE(k) \
  case k:              \
    lpc_fixed_order<k, Acc>(out, bs, coef, shift); \
    return true;
    TW_LPC_CASE(1) TW_LPC_CASE(2) TW_LPC_CASE(3) TW_LPC_CASE(4) TW_LPC_CASE(5) TW_LPC_CASE(6) TW_LPC_CASE(7)
    TW_LPC_CASE(8) TW_LPC_CASE(9) TW_LPC_CASE(10) TW_LPC_CASE(11) TW_LPC_CASE(12) TW_LPC_CASE(13) TW_LPC_CASE(14)
    TW_LPC_CASE(15) TW_LPC_CASE(16)
#undef TW_LPC_CASE
    default:
      for (int i = order; i < bs; i++) {
        int64_t acc = 0;
        for (int j = 0; j < order; j++) acc += (int64_t)coef[j] * out[i - 1 - j];
        out[i] = wrap_add(out[i], (int32_t)(acc >> shift));
      }
      return true;
  }
}

// LPC synthesis: out[i] += (sum_j coef[j] * out[i-1-j]) >> shift, specialised per order (orders 1..16 cover
// every libFLAC compression level; 17..32 take the generic loop)
bool lpc_restore(int32_t* out, int bs, const int32_t* coef, int order, int shift, bool narrow) {
  return narrow ? lpc_dispatch<int32_t>(out, bs, coef, order, shift)
                : lpc_dispatch<int64_t>(out, bs, coef, order, shift);
}

bool subframe(Bits& b, int bs, int bps, int32_t* out) {
  if (b.u(1) != 0) return false;
  int type = (int)b.u(6);
  int wasted = 0;
  if (b.u(1)) wasted = (int)b.unary() + 1;
  bps -= wasted;
  if (bps <= 0 || bps > 32) return false;
  if (type == 0) {
    int32_t v = b.s(bps);
    for (int i = 0; i < bs; i++) out[i] = v;
  } else if (type == 1) {
    for (int i = 0; i < bs; i++) out[i] = b.s(bps);
  } else if (type >= 8 && type <= 12) {
    int order = type - 8;
    if (order > bs) return false;
    for (int i = 0; i < order; i++) out[i] = b.s(bps);
    if (!residual(b, bs, order, out)) return false;
    uint32_t* u = (uint32_t*)out;  // fixed polynomial predictors, modulo 2^32 (see wrap_add)
    switch (order) {
      case 1:
        for (int i = 1; i < bs; i++) u[i] += u[i - 1];
        break;
      case 2:
        for (int i = 2; i < bs; i++) u[i] += 2u * u[i - 1] - u[i - 2];
        break;
      case 3:
        for (int i = 3; i < bs; i++) u[i] += 3u * u[i - 1] - 3u * u[i - 2] + u[i - 3];
        break;
      case 4:
        for (int i = 4; i < bs; i++) u[i] += 4u * u[i - 1] - 6u * u[i - 2] + 4u * u[i - 3] - u[i - 4];
        break;
      default:
        break;
    }
  } else if (type >= 32) {
    int order = (type & 31) + 1;
    if (order > bs) return false;
    for (int i = 0; i < order; i++) out[i] = b.s(bps);
    int prec = (int)b.u(4) + 1;
    if (prec == 16) return false;
    int shift = b.s(5);
    if (shift < 0) return false;
    int32_t coef[32];
    for (int j = 0; j < order; j++) coef[j] = b.s(prec);
    if (!residual(b, bs, order, out)) return false;
    // 32-bit accumulation is exact when |sample| < 2^bps, |coef| < 2^(prec-1) and order terms fit in 31 bits
    bool narrow = bps + prec + 32 - __builtin_clz((unsigned)order) <= 32;
    if (!lpc_restore(out, bs, coef, order, shift, narrow)) return false;
  } else {
    return false;
  }
  if (wasted)
    for (int i = 0; i < bs; i++) out[i] = (int32_t)((uint32_t)out[i] << wasted);
  return !b.bad;
}

// Decode the frame at `pos` into out (interleaved) if it fits; returns the frame's byte length, 0 on failure.
size_t decode_frame(const uint8_t* d, size_t n, size_t pos, const TwFlacInfo& si, int32_t* out, int64_t out_frames,
                    std::vector<int32_t>& scratch, int64_t* first_sample, int* blocksize) {
  Header h;
  if (!parse_header(d, n, pos, si, &h)) return 0;
  const int bs = h.blocksize, nch = h.channels;
  if (h.first_sample < 0 || h.first_sample + bs > out_frames) return 0;
  scratch.resize((size_t)bs * nch);
  Bits b(d, n, pos + h.hdr_bytes);
  for (int c = 0; c < nch; c++) {
    int sbps = h.bps;
    if ((h.chan_assign == 8 && c == 1) || (h.chan_assign == 9 && c == 0) || (h.chan_assign == 10 && c == 1))
      sbps += 1;  // side channel carries one extra bit
    if (sbps > 32) return 0;
    if (!subframe(b, bs, sbps, scratch.data() + (size_t)c * bs)) return 0;
  }
  b.align();
  size_t end = b.byte();
  if (end + 2 > n) return 0;
  if (crc16(d + pos, end - pos) != (uint16_t)((d[end] << 8) | d[end + 1])) return 0;
  *first_sample = h.first_sample;
  *blocksize = bs;
  if (!out) return end + 2 - pos;  // (a validating pass: no output)
  int32_t* s0 = scratch.data();
  int32_t* s1 = nch > 1 ? scratch.data() + bs : nullptr;
  int32_t* o = out + h.first_sample * nch;
  if (h.chan_assign < 8) {
    for (int i = 0; i < bs; i++)
      for (int c = 0; c < nch; c++) o[(size_t)i * nch + c] = scratch[(size_t)c * bs + i];
  } else if (h.chan_assign == 8) {  // left, side
    for (int i = 0; i < bs; i++) {
      o[2 * i] = s0[i];
      o[2 * i + 1] = (int32_t)((uint32_t)s0[i] - (uint32_t)s1[i]);
    }
  } else if (h.chan_assign == 9) {  // side, right
    for (int i = 0; i < bs; i++) {
      o[2 * i] = wrap_add(s0[i], s1[i]);
      o[2 * i + 1] = s1[i];
    }
  } else {  // mid, side
    for (int i = 0; i < bs; i++) {
      int64_t mid = (int64_t)s0[i] * 2 + (s1[i] & 1);  // (s0 << 1 | side's low bit; no shift of a negative)
      o[2 * i] = (int32_t)((mid + s1[i]) >> 1);
      o[2 * i + 1] = (int32_t)((mid - s1[i]) >> 1);
    }
  }
  return end + 2 - pos;
}

struct Worker {
  size_t start = 0;     // byte offset of the first frame this worker owns (SIZE_MAX: none found)
  int64_t decoded = 0;  // max(first_sample + blocksize) over its frames
  int64_t first = -1;   // first sample of its first frame
  int64_t next = -1;    // first sample + blocksize of its last frame (frames must follow each other gap-free)
  bool ok = true;
  std::string err;
};

// First genuine frame at or after `from` (sync + CRC-8 + CRC-16 of a full decode); SIZE_MAX if none.
size_t find_frame(const uint8_t* d, size_t n, size_t from, const TwFlacInfo& si, int32_t* out, int64_t out_frames,
                  std::vector<int32_t>& scratch) {
  for (size_t p = from; p + 1 < n; p++) {
    if (d[p] != 0xFF || (d[p + 1] & 0xFE) != 0xF8) continue;
    int64_t fs;
    int bsz;
    if (decode_frame(d, n, p, si, out, out_frames, scratch, &fs, &bsz)) return p;
  }
  return SIZE_MAX;
}

}  // namespace

extern "C" int tw_flac_probe(const uint8_t* data, int64_t size, TwFlacInfo* info) {
  if (!data || !info || size < 42 || memcmp(data, "fLaC", 4) != 0) {
    tw_set_error("tw_flac_probe: not a FLAC stream");
    return 1;
  }
  memset(info, 0, sizeof(*info));
  size_t pos = 4;
  bool have_si = false;
  for (;;) {
    if (pos + 4 > (size_t)size) {
      tw_set_error("tw_flac_probe: truncated metadata");
      return 1;
    }
    int last = data[pos] >> 7, type = data[pos] & 0x7F;
    size_t len = ((size_t)data[pos + 1] << 16) | ((size_t)data[pos + 2] << 8) | data[pos + 3];
    const uint8_t* p = data + pos + 4;
    if (pos + 4 + len > (size_t)size) {
      tw_set_error("tw_flac_probe: truncated metadata block");
      return 1;
    }
    if (type == 0) {
      if (len < 34) {
        tw_set_error("tw_flac_probe: short STREAMINFO");
        return 1;
      }
      info->min_blocksize = (p[0] << 8) | p[1];
      info->max_blocksize = (p[2] << 8) | p[3];
      uint64_t x = 0;
      for (int i = 10; i < 18; i++) x = (x << 8) | p[i];
      info->sample_rate = (int32_t)(x >> 44);
      info->channels = (int32_t)((x >> 41) & 7) + 1;
      info->bits_per_sample = (int32_t)((x >> 36) & 31) + 1;
      info->total_samples = (int64_t)(x & ((1ull << 36) - 1));
      memcpy(info->md5, p + 18, 16);
      have_si = true;
    } else if (type == 127) {
      tw_set_error("tw_flac_probe: invalid metadata block type");
      return 1;
    }
    pos += 4 + len;
    if (last) break;
  }
  if (!have_si) {
    tw_set_error("tw_flac_probe: missing STREAMINFO");
    return 1;
  }
  info->audio_offset = (int64_t)pos;
  if (info->total_samples == 0) {
    // STREAMINFO leaves the length unknown (a stream written to a pipe): the last genuine frame (sync, CRC-8 and the
    // CRC-16 of a full decode, searched back from the end) gives it, as its first sample + its block size
    std::vector<int32_t> scratch;
    for (size_t p = (size_t)size - 2; p + 1 > pos; p--) {
      if (data[p] != 0xFF || (data[p + 1] & 0xFE) != 0xF8) continue;
      int64_t fs;
      int bsz;
      if (decode_frame(data, (size_t)size, p, *info, nullptr, INT64_MAX, scratch, &fs, &bsz)) {
        info->total_samples = fs + bsz;
        info->total_from_frames = 1;
        break;
      }
    }
  }
  return 0;
}

extern "C" int tw_flac_decode(const uint8_t* data, int64_t size, int32_t* out, int64_t out_frames, int32_t n_threads,
                              int64_t* frames_decoded) {
  TwFlacInfo si;
  if (tw_flac_probe(data, size, &si)) return 1;
  if (!out || si.total_samples <= 0 || out_frames < si.total_samples) {
    tw_set_error("tw_flac_decode: %s", si.total_samples <= 0 ? "stream length unknown (STREAMINFO total = 0)"
                                                              : "output buffer smaller than total_samples");
    return 1;
  }
  const uint8_t* d = data;
  const size_t n = (size_t)size, a0 = (size_t)si.audio_offset;
  int T = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  // at least ~256 KiB of compressed data per worker
  T = (int)std::max<int64_t>(1, std::min<int64_t>(T, (int64_t)(n - a0) / (256 << 10)));
  const int64_t total = si.total_samples;

  auto run = [&](int nw) -> std::vector<Worker> {
    std::vector<Worker> w(nw);
    // phase 1: each worker locates its first frame
    auto locate = [&](int t) {
      std::vector<int32_t> scratch;
      size_t from = a0 + (n - a0) * (size_t)t / (size_t)nw;
      w[t].start = t == 0 ? a0 : find_frame(d, n, from, si, out, total, scratch);
    };
    // phase 2: decode [start_t, start_{t+1})
    auto decode = [&](int t) {
      std::vector<int32_t> scratch;
      size_t p = w[t].start, stop = n;
      for (int u = t + 1; u < nw; u++)
        if (w[u].start != SIZE_MAX) {
          stop = w[u].start;
          break;
        }
      if (p == SIZE_MAX) return;
      while (p < stop && p + 2 < n) {
        int64_t fs;
        int bsz;
        size_t len = decode_frame(d, n, p, si, out, total, scratch, &fs, &bsz);
        if (!len) {
          w[t].ok = false;
          char msg[160];
          snprintf(msg, sizeof msg, "corrupt or unsupported FLAC frame at byte %zu", p);
          w[t].err = msg;
          return;
        }
        if (w[t].next >= 0 && fs != w[t].next) {  // a skipped or repeated sample range: not a valid stream
          w[t].ok = false;
          w[t].err = "frame sample numbers are not contiguous";
          return;
        }
        if (w[t].first < 0) w[t].first = fs;
        w[t].next = fs + bsz;
        w[t].decoded = std::max(w[t].decoded, fs + bsz);
        p += len;
        if (fs + bsz >= total) break;  // the last frame: what follows (an ID3v1 / APE tag, padding) is not audio
      }
      if (p != stop && stop != n) {
        w[t].ok = false;
        w[t].err = "frame boundary mismatch";
      }
    };
    if (nw == 1) {
      locate(0);
      decode(0);
      return w;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nw; t++) th.emplace_back(locate, t);
    for (auto& x : th) x.join();
    th.clear();
    for (int t = 0; t < nw; t++) th.emplace_back(decode, t);
    for (auto& x : th) x.join();
    return w;
  };

  std::vector<Worker> w = run(T);
  bool ok = true;
  for (auto& x : w) ok = ok && x.ok;
  if (!ok && T > 1) {  // a fooled sync search: one sequential pass decides
    w = run(1);
    ok = w[0].ok;
  }
  if (!ok) {
    for (auto& x : w)
      if (!x.ok) {
        tw_set_error("tw_flac_decode: %s", x.err.c_str());
        break;
      }
    return 1;
  }
  // every output sample written exactly once: the workers' frame runs tile [0, total) in order
  int64_t got = 0;
  for (auto& x : w) {
    if (x.first < 0) continue;  // (a worker whose range held no frame start)
    if (x.first != got) {
      tw_set_error("tw_flac_decode: samples [%lld, %lld) missing or repeated", (long long)std::min(got, x.first),
                   (long long)std::max(got, x.first));
      return 1;
    }
    got = x.next;
  }
  if (got != total) {
    tw_set_error("tw_flac_decode: decoded %lld of %lld samples", (long long)got, (long long)total);
    return 1;
  }
  if (frames_decoded) *frames_decoded = got;
  return 0;
}
