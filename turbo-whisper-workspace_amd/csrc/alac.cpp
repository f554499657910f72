// Apple Lossless (ALAC) decoder for the access units of an MP4 / M4A 'alac' track (host side of the audio ingest,
// include/tw_audio.h). The reference's ffmpeg_read ($TF/pipelines/audio_utils.py:9-45) takes any .m4a upload
// (vocalis/security/security_monitor.py:355, scripts/normalize_audio.py:226 list the extension), and ffmpeg's mov
// demuxer + alac decoder decode an Apple Lossless track in it; this restates that decoder's behaviour (ffmpeg 6.x
// libavcodec/alac.c, which follows Apple's published ALAC sources): the 24-byte ALACSpecificConfig (frame length,
// bit depth, Rice parameters pb / mb / kb, channels, rate); per frame, elements (SCE / CPE / LFE, up to END) with
// their header (partial-frame sample count, shifted-out low bytes, an uncompressed escape); the adaptive Rice /
// Golomb residuals with their zero-run mode; the sign-adaptive LPC predictor (type 15 runs a first-order pass first);
// stereo decorrelation (mix shift / weight); the shifted-out low bits appended. Frames are independent, so packets
// decode on threads. Output: f32 interleaved, sample / 2^(bit depth - 1), as ffmpeg's s16p / s32p output converted by
// `-f f32le` (16-bit samples truncated to s16, 20 / 24-bit shifted into s32).
//
// ffmpeg drops a packet its decoder refuses; so does this decoder (the packet contributes no samples).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/tw_audio.h"

void tw_set_error(const char* fmt, ...);

namespace {

struct Cfg {
  uint32_t frame_length = 0;
  int bit_depth = 0, pb = 0, mb = 0, kb = 0, channels = 0;
  uint32_t sample_rate = 0;
};

bool parse_cfg(const uint8_t* c, int64_t n, Cfg& g, const char** err) {
  if (n >= 36 && memcmp(c + 4, "alac", 4) == 0) c += 12, n -= 12;  // the 'alac' atom with its header
  if (n < 24) {
    *err = "ALAC: magic cookie shorter than 24 bytes";
    return false;
  }
  auto be32 = [](const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; };
  g.frame_length = be32(c);
  g.bit_depth = c[5], g.pb = c[6], g.mb = c[7], g.kb = c[8], g.channels = c[9];
  g.sample_rate = be32(c + 20);
  if (!g.frame_length || g.frame_length > 4096u * 4096u) {
    *err = "ALAC: frame length out of range";
    return false;
  }
  if (g.bit_depth != 16 && g.bit_depth != 20 && g.bit_depth != 24 && g.bit_depth != 32) {
    *err = "ALAC: unsupported bit depth (16 / 20 / 24 / 32)";
    return false;
  }
  if (g.channels < 1 || g.channels > 2) {
    *err = "ALAC: only mono and stereo tracks are decoded";
    return false;
  }
  return true;
}

// MSB-first bit reader; reads past the end as zeros, `left()` goes negative there
struct Bits {
  const uint8_t* d;
  int64_t nbits, pos = 0;
  uint32_t peek(int n) const {  // n <= 32
    if (n <= 0) return 0;
    uint64_t w = 0;
    const int64_t b = pos >> 3;
    for (int i = 0; i < 8; i++) w = w << 8 | ((b + i) * 8 < nbits ? d[b + i] : 0);
    return (uint32_t)((w << (pos & 7)) >> (64 - n));
  }
  uint32_t get(int n) {
    const uint32_t v = peek(n);
    pos += n;
    return v;
  }
  int32_t sget(int n) {  // n <= 32, sign-extended
    const uint32_t v = get(n);
    return n >= 32 ? (int32_t)v : (int32_t)(v << (32 - n)) >> (32 - n);
  }
  int64_t left() const { return nbits - pos; }
};

inline int ilog2(uint32_t v) { return v ? 31 - __builtin_clz(v) : 0; }
inline int32_t sext(uint32_t v, int bits) { return bits >= 32 ? (int32_t)v : (int32_t)(v << (32 - bits)) >> (32 - bits); }
inline int sign_only(int v) { return v > 0 ? 1 : v < 0 ? -1 : 0; }

// one Rice / Golomb value: a unary prefix of up to 9 ones, then k bits (escape: `bps` raw bits)
uint32_t scalar(Bits& br, int k, int bps) {
  uint32_t x = 0;
  while (x < 9 && br.get(1)) x++;
  if (x > 8) return br.get(bps);
  if (k != 1) {
    const uint32_t extra = br.peek(k);
    x = (x << k) - x;
    if (extra > 1) {
      x += extra - 1;
      br.pos += k;
    } else {
      br.pos += k - 1;
    }
  }
  return x;
}

bool rice(Bits& br, int32_t* out, int n, int bps, uint32_t mult, const Cfg& g) {
  uint32_t history = (uint32_t)g.mb;
  int sign_mod = 0;
  for (int i = 0; i < n; i++) {
    if (br.left() <= 0) return false;
    int k = std::min(ilog2((history >> 9) + 3), g.kb);
    uint32_t x = scalar(br, k, bps) + sign_mod;
    sign_mod = 0;
    out[i] = (int32_t)((x >> 1) ^ (0u - (x & 1)));
    if (x > 0xffff)
      history = 0xffff;
    else
      history += x * mult - ((history * mult) >> 9);
    if (history < 128 && i + 1 < n) {
      k = std::min(7 - ilog2(history) + (int)((history + 16) >> 6), g.kb);
      int block = (int)scalar(br, k, 16);
      if (block > 0) {
        if (block >= n - i) block = n - i - 1;
        memset(out + i + 1, 0, sizeof(int32_t) * block);
        i += block;
      }
      if (block <= 0xffff) sign_mod = 1;
      history = 0;
    }
  }
  return true;
}

// the adaptive LPC: warm-up by first differences, then prediction from the `order` previous samples relative to the
// oldest one, coefficients nudged by the sign of each error (ffmpeg's lpc_prediction, coefficients oldest first)
void lpc(const int32_t* err, int32_t* out, int n, int bps, int16_t* coefs, int order, int quant) {
  out[0] = err[0];
  if (n <= 1) return;
  if (!order) {
    memcpy(out + 1, err + 1, sizeof(int32_t) * (n - 1));
    return;
  }
  if (order == 31) {
    for (int i = 1; i < n; i++) out[i] = sext((uint32_t)out[i - 1] + (uint32_t)err[i], bps);
    return;
  }
  int i = 1;
  for (; i <= order && i < n; i++) out[i] = sext((uint32_t)out[i - 1] + (uint32_t)err[i], bps);
  for (; i < n; i++) {
    const uint32_t* pred = (const uint32_t*)out + (i - order);
    const int d = out[i - order - 1];
    uint32_t acc = 0;
    for (int j = 0; j < order; j++) acc += (pred[j] - (uint32_t)d) * (uint32_t)(int32_t)coefs[j];
    int64_t v = ((int64_t)(int32_t)acc + (1LL << (quant - 1))) >> quant;
    uint32_t errv = (uint32_t)err[i];
    out[i] = sext((uint32_t)(int32_t)v + (uint32_t)d + errv, bps);
    const int es = sign_only((int32_t)errv);
    if (es)
      for (int j = 0; j < order && (int32_t)(errv * (uint32_t)es) > 0; j++) {
        int dv = d - (int32_t)pred[j];
        const int s = sign_only(dv) * es;
        coefs[j] -= s;
        dv *= s;
        errv -= (uint32_t)((dv >> quant) * (j + 1));
      }
  }
}

struct Scratch {
  std::vector<int32_t> err[2], out[2], extra[2];
  void size(uint32_t n) {
    for (int c = 0; c < 2; c++) err[c].resize(n), out[c].resize(n), extra[c].resize(n);
  }
};

// the sample count of a packet (its first element's header), 0 when it does not start with a valid element
uint32_t packet_samples(const uint8_t* p, int64_t n, const Cfg& g) {
  Bits br{p, n * 8};
  if (br.left() < 3 + 4 + 12 + 4) return 0;
  const uint32_t tag = br.get(3);
  if (tag != 0 && tag != 1 && tag != 3) return 0;
  br.get(16);
  const uint32_t has_size = br.get(1);
  br.get(3);
  const uint32_t ns = has_size ? br.get(32) : g.frame_length;
  return (ns && ns <= g.frame_length) ? ns : 0;
}

// decode one packet into pcm (interleaved f32, `ns` frames); false: the packet is refused
bool decode_packet(const uint8_t* p, int64_t n, const Cfg& g, uint32_t ns, float* pcm, Scratch& S) {
  Bits br{p, n * 8};
  int ch = 0;
  uint32_t nb = 0;
  while (br.left() >= 3) {
    const uint32_t tag = br.get(3);
    if (tag == 7) break;
    if (tag != 0 && tag != 1 && tag != 3) return false;
    const int channels = tag == 1 ? 2 : 1;
    if (ch + channels > g.channels) return false;
    br.get(4 + 12);
    const uint32_t has_size = br.get(1);
    int extra_bits = (int)br.get(2) << 3;
    const int bps = g.bit_depth - extra_bits + channels - 1;
    if (bps > 32 || bps < 1) return false;
    const bool compressed = !br.get(1);
    const uint32_t out_n = has_size ? br.get(32) : g.frame_length;
    if (!out_n || out_n > g.frame_length) return false;
    if (nb && out_n != nb) return false;
    nb = out_n;
    if (nb != ns) return false;
    int shift = 0, weight = 0;
    if (compressed) {
      if (!g.kb) return false;
      shift = (int)br.get(8), weight = (int)br.get(8);
      if (channels == 2 && weight && shift > 31) return false;
      int ptype[2], quant[2], hmult[2], order[2];
      int16_t coefs[2][32];
      for (int c = 0; c < channels; c++) {
        ptype[c] = (int)br.get(4), quant[c] = (int)br.get(4), hmult[c] = (int)br.get(3), order[c] = (int)br.get(5);
        if ((uint32_t)order[c] >= g.frame_length || !quant[c]) return false;
        for (int i = order[c] - 1; i >= 0; i--) coefs[c][i] = (int16_t)br.sget(16);
      }
      if (extra_bits)
        for (uint32_t i = 0; i < nb; i++) {
          if (br.left() <= 0) return false;
          for (int c = 0; c < channels; c++) S.extra[c][i] = (int32_t)br.get(extra_bits);
        }
      for (int c = 0; c < channels; c++) {
        if (!rice(br, S.err[c].data(), (int)nb, bps, (uint32_t)(hmult[c] * g.pb / 4), g)) return false;
        if (ptype[c] == 15) lpc(S.err[c].data(), S.err[c].data(), (int)nb, bps, nullptr, 31, 0);
        lpc(S.err[c].data(), S.out[c].data(), (int)nb, bps, coefs[c], order[c], quant[c]);
      }
    } else {
      for (uint32_t i = 0; i < nb; i++)
        for (int c = 0; c < channels; c++) S.out[c][i] = br.sget(g.bit_depth);
      extra_bits = 0;
    }
    if (channels == 2 && weight)
      for (uint32_t i = 0; i < nb; i++) {
        int32_t a = S.out[0][i], b = S.out[1][i];
        a -= (int32_t)(((int64_t)b * weight) >> shift);
        b += a;
        S.out[0][i] = b, S.out[1][i] = a;
      }
    if (extra_bits)
      for (int c = 0; c < channels; c++)
        for (uint32_t i = 0; i < nb; i++)
          S.out[c][i] = (int32_t)(((uint32_t)S.out[c][i] << extra_bits) | (uint32_t)S.extra[c][i]);
    for (int c = 0; c < channels; c++)
      for (uint32_t i = 0; i < nb; i++) {
        const int32_t v = S.out[c][i];
        float f;
        if (g.bit_depth == 16)
          f = (float)(int16_t)v / 32768.f;
        else
          f = (float)((double)(int32_t)((uint32_t)v << (32 - g.bit_depth)) / 2147483648.0);
        pcm[(size_t)i * g.channels + ch + c] = f;
      }
    ch += channels;
  }
  return nb == ns && ch > 0;
}

}  // namespace

extern "C" {

int tw_alac_parse_cookie(const uint8_t* cookie, int64_t size, TwAlacInfo* info) {
  if (!cookie || !info) {
    tw_set_error("tw_alac_parse_cookie: null argument");
    return 1;
  }
  Cfg g;
  const char* err = nullptr;
  if (!parse_cfg(cookie, size, g, &err)) {
    tw_set_error("%s", err);
    return 2;
  }
  memset(info, 0, sizeof(*info));
  info->sample_rate = (int32_t)g.sample_rate;
  info->channels = g.channels;
  info->bit_depth = g.bit_depth;
  info->frame_length = (int32_t)g.frame_length;
  info->pb = g.pb, info->mb = g.mb, info->kb = g.kb;
  return 0;
}

int tw_alac_decode(const uint8_t* cookie, int64_t cookie_size, const uint8_t* data, int64_t size,
                   const int64_t* offsets, const int64_t* sizes, int64_t n_packets, float* out, int64_t out_frames,
                   int32_t n_threads, int64_t* frames_decoded) {
  if (!cookie || !data || !offsets || !sizes || !out || !frames_decoded || n_packets < 0) {
    tw_set_error("tw_alac_decode: null argument");
    return 1;
  }
  Cfg g;
  const char* err = nullptr;
  if (!parse_cfg(cookie, cookie_size, g, &err)) {
    tw_set_error("%s", err);
    return 2;
  }
  std::vector<uint32_t> ns((size_t)n_packets);
  std::vector<int64_t> at((size_t)n_packets + 1, 0);
  for (int64_t k = 0; k < n_packets; k++) {
    if (offsets[k] < 0 || sizes[k] < 0 || offsets[k] + sizes[k] > size) {
      tw_set_error("tw_alac_decode: packet %lld lies outside the data", (long long)k);
      return 3;
    }
    ns[k] = packet_samples(data + offsets[k], sizes[k], g);
    at[k + 1] = at[k] + ns[k];
  }
  if (at[n_packets] > out_frames) {
    tw_set_error("tw_alac_decode: out_frames %lld < %lld samples", (long long)out_frames, (long long)at[n_packets]);
    return 4;
  }
  std::vector<uint8_t> ok((size_t)n_packets, 0);
  int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n_packets / 4));
  auto work = [&](int64_t a, int64_t b) {
    Scratch S;
    S.size(g.frame_length);
    for (int64_t k = a; k < b; k++)
      if (ns[k]) ok[k] = decode_packet(data + offsets[k], sizes[k], g, ns[k], out + at[k] * g.channels, S);
  };
  if (nt == 1) {
    work(0, n_packets);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++) th.emplace_back(work, n_packets * t / nt, n_packets * (t + 1) / nt);
    for (auto& x : th) x.join();
  }
  // refused packets contribute no samples (ffmpeg drops them): close the gaps
  int64_t w = 0;
  for (int64_t k = 0; k < n_packets; k++) {
    if (!ok[k]) continue;
    if (w != at[k]) memmove(out + w * g.channels, out + at[k] * g.channels, sizeof(float) * ns[k] * g.channels);
    w += ns[k];
  }
  *frames_decoded = w;
  return 0;
}

}  // extern "C"
