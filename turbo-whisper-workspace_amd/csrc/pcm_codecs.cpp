// Telephony codecs of the containers ffmpeg_read accepts besides PCM and FLAC ($TF/pipelines/audio_utils.py:9-45:
// ffmpeg decodes every codec to s16, and `-f f32le` divides by 32768). HOST memory, no GPU.
//   G.711 mu-law / A-law (ITU-T G.711; WAV format tags 7 / 6, AU encodings 1 / 27, AIFF-C 'ulaw' / 'alaw'): the
//     classic expansion (Sun's g711.c, which ffmpeg's pcm_tablegen and CPython's audioop also restate), 8 bits -> s16.
//   IMA ADPCM (WAV format tag 0x11, Microsoft's block layout; ffmpeg's adpcm_ima_wav): per block and channel a
//     4-byte header {s16 predictor, u8 step index, u8 0} whose predictor is the block's first sample, then 4-byte words
//     of 8 nibbles per channel, interleaved channel by channel, low nibble first; every nibble is the IMA/DVI step
//     (stepsize table of 89, index table, shift-add difference, s16 clamp).
#include <stdint.h>

#include <algorithm>

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
