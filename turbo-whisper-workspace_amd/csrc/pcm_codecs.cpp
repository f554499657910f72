// Telephony codecs of the containers ffmpeg_read accepts besides PCM and FLAC ($TF/pipelines/audio_utils.py:9-45:
// ffmpeg decodes every codec to s16, and `-f f32le` divides by 32768). HOST memory, no GPU.
//   G.711 mu-law / A-law (ITU-T G.711; WAV format tags 7 / 6, AU encodings 1 / 27, AIFF-C 'ulaw' / 'alaw'): the
//     classic expansion (Sun's g711.c, which ffmpeg's pcm_tablegen and CPython's audioop also restate), 8 bits -> s16.
//   IMA ADPCM (WAV format tag 0x11, Microsoft's block layout; ffmpeg's adpcm_ima_wav): per block and channel a
//     4-byte header {s16 predictor, u8 step index, u8 0} whose predictor is the block's first sample, then 4-byte words
//     of 8 nibbles per channel, interleaved channel by channel, low nibble first; every nibble is the IMA/DVI step
//     (stepsize table of 89, index table, shift-add difference, s16 clamp).
//   Microsoft ADPCM (WAV format tag 2; ffmpeg's adpcm_ms) and Apple IMA4 (AIFF-C 'ima4'; ffmpeg's adpcm_ima_qt):
//     below, at their decoders.
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "../../include/tw_audio.h"

void tw_set_error(const char* fmt, ...);

static int16_t ulaw_to_s16(uint8_t u) {
  u = (uint8_t)~u;
  int t = ((u & 0x0f) << 3) + 0x84;
  t <<= (u & 0x70) >> 4;
  return (int16_t)((u & 0x80) ? (0x84 - t) : (t - 0x84));
}

static int16_t alaw_to_s16(uint8_t a) {
  a ^= 0x55;
  int t = (a & 0x0f) << 4;
  const int seg = (a & 0x70) >> 4;
  if (seg == 0) t += 8;
  else if (seg == 1) t += 0x108;
  else t = (t + 0x108) << (seg - 1);
  return (int16_t)((a & 0x80) ? t : -t);
}

extern "C" int tw_g711_decode(const uint8_t* in, int64_t n, int32_t alaw, int16_t* out) {
  if ((!in || !out) && n > 0) {
    tw_set_error("tw_g711_decode: null pointer");
    return 1;
  }
  if (alaw)
    for (int64_t i = 0; i < n; ++i) out[i] = alaw_to_s16(in[i]);
  else
    for (int64_t i = 0; i < n; ++i) out[i] = ulaw_to_s16(in[i]);
  return 0;
}

static const int kImaStep[89] = {
    7,     8,     9,     10,    11,    12,    13,    14,    16,    17,    19,    21,    23,    25,    28,
    31,    34,    37,    41,    45,    50,    55,    60,    66,    73,    80,    88,    97,    107,   118,
    130,   143,   157,   173,   190,   209,   230,   253,   279,   307,   337,   371,   408,   449,   494,
    544,   598,   658,   724,   796,   876,   963,   1060,  1166,  1282,  1411,  1552,  1707,  1878,  2066,
    2272,  2499,  2749,  3024,  3327,  3660,  4026,  4428,  4871,  5358,  5894,  6484,  7132,  7845,  8630,
    9493,  10442, 11487, 12635, 13899, 15289, 16818, 18500, 20350, 22385, 24623, 27086, 29794, 32767};
static const int kImaIndex[16] = {-1, -1, -1, -1, 2, 4, 6, 8, -1, -1, -1, -1, 2, 4, 6, 8};

static inline int16_t ima_step(int& pred, int& index, int nib) {
  const int step = kImaStep[index];
  int diff = step >> 3;
  if (nib & 4) diff += step;
  if (nib & 2) diff += step >> 1;
  if (nib & 1) diff += step >> 2;
  pred = (nib & 8) ? pred - diff : pred + diff;
  pred = std::min(32767, std::max(-32768, pred));
  index = std::min(88, std::max(0, index + kImaIndex[nib]));
  return (int16_t)pred;
}

static int64_t tw_ima_wav_block_frames(int32_t bytes, int32_t channels) {
  if (channels < 1 || bytes < 4 * channels) return 0;
  return 1 + (int64_t)((bytes - 4 * channels) / (4 * channels)) * 8;
}

extern "C" int tw_ima_adpcm_wav_decode(const uint8_t* data, int64_t size, int32_t channels, int32_t block_align,
                                       int16_t* out, int64_t out_frames, int64_t* frames_decoded) {
  if (!data || !out || !frames_decoded || channels < 1 || channels > 8 || block_align < 4 * channels) {
    tw_set_error("tw_ima_adpcm_wav_decode: bad arguments (channels %d, block_align %d)", channels, block_align);
    return 1;
  }
  int64_t f = 0;
  for (int64_t pos = 0; pos + 4 * channels <= size; pos += block_align) {
    const int32_t len = (int32_t)std::min<int64_t>(block_align, size - pos);
    const int64_t nb = tw_ima_wav_block_frames(len, channels);
    if (f + nb > out_frames) {
      tw_set_error("tw_ima_adpcm_wav_decode: output holds %lld frames, the stream has more", (long long)out_frames);
      return 1;
    }
    const uint8_t* b = data + pos;
    for (int c = 0; c < channels; ++c) {
      int pred = (int16_t)(b[4 * c] | (b[4 * c + 1] << 8));
      int index = b[4 * c + 2];
      if (index > 88) {
        tw_set_error("tw_ima_adpcm_wav_decode: step index %d > 88 in the block at byte %lld", index, (long long)pos);
        return 1;
      }
      int16_t* o = out + f * channels + c;
      o[0] = (int16_t)pred;
      const uint8_t* w = b + 4 * channels + 4 * c;  // this channel's first 4-byte word
      for (int64_t k = 0; k < (nb - 1) / 8; ++k, w += 4 * channels) {
        for (int j = 0; j < 4; ++j) {
          o[(1 + 8 * k + 2 * j) * channels] = ima_step(pred, index, w[j] & 0x0f);
          o[(2 + 8 * k + 2 * j) * channels] = ima_step(pred, index, w[j] >> 4);
        }
      }
    }
    f += nb;
  }
  *frames_decoded = f;
  return 0;
}

// ---- Microsoft ADPCM (WAV format tag 2; ffmpeg's adpcm_ms) ------------------------------------------------------------
// Per block: for each channel a predictor index (u8, 0..6), then each channel's s16 delta, s16 sample1, s16 sample2.
// The block's first two output frames are sample2 then sample1; every following byte holds two nibbles, high first
// (stereo: high nibble channel 0, low nibble channel 1). A nibble n (4-bit two's complement) predicts
// (s1 c1 + s2 c2) / 256 (C division) + n delta, clamped to s16, and scales delta by the adaptation table / 256
// (floor 16). The coefficient pairs are the standard seven (ffmpeg uses its built-in table and refuses an index > 6:
// such a block is dropped, as its decode error drops the packet).
static const int kMsCoef1[7] = {256, 512, 0, 192, 240, 460, 392};
static const int kMsCoef2[7] = {0, -256, 0, 64, 0, -208, -232};
static const int kMsAdapt[16] = {230, 230, 230, 230, 307, 409, 512, 614, 768, 614, 512, 409, 307, 230, 230, 230};

struct MsState {
  int c1, c2, delta, s1, s2;
};

static inline int16_t ms_step(MsState& s, int nib) {
  int pred = (s.s1 * s.c1 + s.s2 * s.c2) / 256;
  pred += ((nib & 8) ? nib - 16 : nib) * s.delta;
  s.s2 = s.s1;
  s.s1 = std::min(32767, std::max(-32768, pred));
  s.delta = (int)(((int64_t)kMsAdapt[nib] * s.delta) >> 8);
  if (s.delta < 16) s.delta = 16;
  if (s.delta > 2147483647 / 768) s.delta = 2147483647 / 768;
  return (int16_t)s.s1;
}

extern "C" int tw_ms_adpcm_wav_decode(const uint8_t* data, int64_t size, int32_t channels, int32_t block_align,
                                      int16_t* out, int64_t out_frames, int64_t* frames_decoded) {
  if (!data || !out || !frames_decoded || channels < 1 || channels > 2 || block_align < 7 * channels) {
    tw_set_error("tw_ms_adpcm_wav_decode: bad arguments (channels %d, block_align %d)", channels, block_align);
    return 1;
  }
  const int st = channels - 1;
  int64_t f = 0;
  for (int64_t pos = 0; pos + 7 * channels <= size; pos += block_align) {
    const int32_t len = (int32_t)std::min<int64_t>(block_align, size - pos);
    const int64_t nb = (int64_t)(len - 6 * channels) * 2 / channels;  // frames in this block
    const uint8_t* b = data + pos;
    MsState s[2];
    bool ok = true;
    for (int c = 0; c < channels; ++c) {
      if (b[c] > 6) ok = false;
      else s[c].c1 = kMsCoef1[b[c]], s[c].c2 = kMsCoef2[b[c]];
    }
    if (!ok) continue;
    if (f + nb > out_frames) {
      tw_set_error("tw_ms_adpcm_wav_decode: output holds %lld frames, the stream has more", (long long)out_frames);
      return 1;
    }
    auto s16 = [&](int off) { return (int)(int16_t)(b[off] | (b[off + 1] << 8)); };
    for (int c = 0; c < channels; ++c) {
      s[c].delta = s16(channels + 2 * c);
      s[c].s1 = s16(3 * channels + 2 * c);
      s[c].s2 = s16(5 * channels + 2 * c);
    }
    int16_t* o = out + f * channels;
    for (int c = 0; c < channels; ++c) o[c] = (int16_t)s[c].s2, o[channels + c] = (int16_t)s[c].s1;
    o += 2 * channels;
    const uint8_t* p = b + 7 * channels;
    for (int64_t n = (nb - 2) >> (1 - st); n > 0; --n, ++p) {
      *o++ = ms_step(s[0], *p >> 4);
      *o++ = ms_step(s[st], *p & 15);
    }
    f += nb;
  }
  *frames_decoded = f;
  return 0;
}

// ---- Apple IMA4 (AIFF-C / QuickTime 'ima4'; ffmpeg's adpcm_ima_qt) ------------------------------------------------------
// Packets of 34 bytes per channel, channel after channel: a big-endian u16 whose top 9 bits are the predictor's top 9
// bits (low 7 zero) and whose low 7 bits are the step index, then 32 bytes of 64 nibbles, low nibble first. As ffmpeg
// decodes it, a channel's running state carries over a packet boundary when the header's step index equals the
// running one and its predictor is within 0x7f of the running predictor; otherwise the header resets it.
extern "C" int tw_ima_qt_decode(const uint8_t* data, int64_t size, int32_t channels, int16_t* out, int64_t out_frames,
                                int64_t* frames_decoded) {
  if (!data || !out || !frames_decoded || channels < 1 || channels > 8) {
    tw_set_error("tw_ima_qt_decode: bad arguments (channels %d)", channels);
    return 1;
  }
  int pred[8] = {0}, index[8] = {0};
  int64_t f = 0;
  for (int64_t pos = 0; pos + 34 * channels <= size; pos += 34 * channels) {
    if (f + 64 > out_frames) {
      tw_set_error("tw_ima_qt_decode: output holds %lld frames, the stream has more", (long long)out_frames);
      return 1;
    }
    for (int c = 0; c < channels; ++c) {
      const uint8_t* b = data + pos + 34 * c;
      const int hdr = (int16_t)(b[0] << 8 | b[1]);
      const int si = hdr & 0x7f, hp = hdr & ~0x7f;
      if (!(index[c] == si && std::abs(hp - pred[c]) <= 0x7f)) index[c] = si, pred[c] = hp;
      if (index[c] > 88) {
        tw_set_error("tw_ima_qt_decode: step index %d > 88 in the packet at byte %lld", index[c], (long long)pos);
        return 1;
      }
      int16_t* o = out + f * channels + c;
      for (int m = 0; m < 32; ++m) {
        o[(2 * m) * channels] = ima_step(pred[c], index[c], b[2 + m] & 15);
        o[(2 * m + 1) * channels] = ima_step(pred[c], index[c], b[2 + m] >> 4);
      }
    }
    f += 64;
  }
  *frames_decoded = f;
  return 0;
}
