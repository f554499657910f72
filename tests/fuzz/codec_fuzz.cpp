// Sanitizer driver for the host parsers of untrusted upload bytes (csrc/flac.cpp, vorbis.cpp, pcm_codecs.cpp, mp3.cpp,
// aac.cpp): every
// input file, then `mutations` damaged copies of it (truncations, bit flips, byte overwrites, chunk duplications;
// a fixed-seed PRNG), through probe + decode of every codec, single- and multi-threaded. Built with
// -fsanitize=address,undefined and -fno-sanitize-recover (make -C turbo-whisper-workspace_amd/csrc sanitize): any
// out-of-bounds access, leak or undefined behaviour aborts the run. Test infrastructure (tests/test_codec_sanitize.py),
// CPU only; the decoders' return codes are not judged here, only memory safety.
//   codec_fuzz [-m mutations] [-s seed] file...
#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "tw_audio.h"

// the library's error sink (tw_runtime.hip in the GPU build); host-only here
static char g_err[512];
void tw_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {  // splitmix64
  uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static long g_runs = 0, g_ok = 0;

static void run_all(const std::vector<uint8_t>& buf) {
  const uint8_t* d = buf.empty() ? nullptr : buf.data();
  const int64_t n = (int64_t)buf.size();
  ++g_runs;
  {  // FLAC
    TwFlacInfo info;
    if (tw_flac_probe(d, n, &info) == 0 && info.channels > 0 && info.total_samples > 0 &&
        info.total_samples < (1 << 22)) {
      std::vector<int32_t> out((size_t)info.total_samples * info.channels);
      int64_t got = 0;
      for (int th : {1, 3})
        if (tw_flac_decode(d, n, out.data(), info.total_samples, th, &got) == 0) ++g_ok;
    }
  }
  {  // Ogg Vorbis
    TwVorbisInfo info;
    if (tw_vorbis_probe(d, n, &info) == 0 && info.channels > 0 && info.total_samples > 0 &&
        info.total_samples < (1 << 22)) {
      std::vector<float> out((size_t)info.total_samples * info.channels);
      int64_t got = 0;
      for (int th : {1, 4})
        if (tw_vorbis_decode(d, n, out.data(), info.total_samples, th, &got) == 0) ++g_ok;
    }
  }
  {  // MP3 / MPEG audio (Layers I, II, III)
    TwMp3Info info;
    if (tw_mp3_probe(d, n, &info) == 0 && info.channels > 0 && info.total_samples >= 0 &&
        info.total_samples < (1 << 22)) {
      std::vector<float> out((size_t)info.total_samples * info.channels + 1);
      int64_t got = 0;
      for (int th : {1, 3})
        if (tw_mp3_decode(d, n, out.data(), info.total_samples, th, &got) == 0) ++g_ok;
    }
  }
  {  // AAC: ADTS framing, and the same bytes as raw access units of 1..3 fixed sizes (the MP4 path) for two configs
    TwAacInfo info;
    if (tw_aac_adts_probe(d, n, &info) == 0 && info.channels > 0 && info.total_samples > 0 &&
        info.total_samples < (1 << 22)) {
      std::vector<float> out((size_t)info.total_samples * info.channels);
      int64_t got = 0;
      for (int th : {1, 3})
        if (tw_aac_adts_decode(d, n, out.data(), info.total_samples, th, &got) == 0) ++g_ok;
    }
    const uint8_t ascs[2][2] = {{0x11, 0x88}, {0x12, 0x10}};  // 48 kHz mono, 44.1 kHz stereo
    for (int a = 0; a < 2; a++)
      for (int64_t unit : {(int64_t)37, (int64_t)200, (int64_t)700}) {
        const int64_t nau = std::min<int64_t>(n / unit, 64);
        if (nau <= 0) continue;
        std::vector<int64_t> off(nau), sz(nau);
        for (int64_t i = 0; i < nau; i++) off[i] = i * unit, sz[i] = unit;
        std::vector<float> out((size_t)nau * 1024 * 2);
        int64_t got = 0;
        if (tw_aac_decode_raw(ascs[a], 2, d, n, off.data(), sz.data(), nau, out.data(), nau * 1024, 2, &got) == 0)
          ++g_ok;
      }
  }
  {  // ALAC: the bytes as access units of a few fixed sizes under mono / stereo, 16 / 24-bit configs
    const uint8_t base[24] = {0, 0, 16, 0, 0, 16, 40, 10, 14, 1, 0, 255, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 172, 68};
    for (int v = 0; v < 3; v++) {
      uint8_t ck[24];
      memcpy(ck, base, 24);
      ck[2] = v == 2 ? 4 : 16;                // frame length 4096 or 1024 (big-endian u32 0x00001000 / 0x00000400)
      ck[5] = v == 1 ? 24 : 16, ck[9] = (uint8_t)(1 + (v & 1));
      for (int64_t unit : {(int64_t)64, (int64_t)900, (int64_t)3000}) {
        const int64_t nau = std::min<int64_t>(n / unit, 32);
        if (nau <= 0) continue;
        std::vector<int64_t> off(nau), sz(nau);
        for (int64_t i = 0; i < nau; i++) off[i] = i * unit, sz[i] = unit;
        std::vector<float> out((size_t)nau * 4096 * 2);
        int64_t got = 0;
        if (tw_alac_decode(ck, 24, d, n, off.data(), sz.data(), nau, out.data(), nau * 4096, 1 + v, &got) == 0) ++g_ok;
      }
    }
  }
  {  // G.711 (raw payload) and IMA ADPCM (Microsoft block layout) over the same bytes
    std::vector<int16_t> pcm(buf.size() + 1);
    if (tw_g711_decode(d, n, 0, pcm.data()) == 0) ++g_ok;
    if (tw_g711_decode(d, n, 1, pcm.data()) == 0) ++g_ok;
    for (int ch : {1, 2})
      for (int ba : {36, 256, 1024}) {
        const int64_t cap = (n / ba + 1) * (int64_t)((ba - 4 * ch) * 2 + 1) + 16;
        std::vector<int16_t> o((size_t)cap * ch);
        int64_t got = 0;
        if (tw_ima_adpcm_wav_decode(d, n, ch, ba, o.data(), cap, &got) == 0) ++g_ok;
        const int64_t mcap = (n / ba + 1) * (int64_t)((ba - 6 * ch) * 2 / ch);  // MS ADPCM, as twamd sizes it
        std::vector<int16_t> m((size_t)std::max<int64_t>(mcap, 1) * ch);
        if (tw_ms_adpcm_wav_decode(d, n, ch, ba, m.data(), mcap, &got) == 0) ++g_ok;
      }
    for (int ch : {1, 2, 5}) {  // Apple IMA4 packets
      const int64_t cap = n / (34 * ch) * 64;
      std::vector<int16_t> o((size_t)std::max<int64_t>(cap, 1) * ch);
      int64_t got = 0;
      if (tw_ima_qt_decode(d, n, ch, o.data(), cap, &got) == 0) ++g_ok;
    }
  }
}

static void mutate_and_run(const std::vector<uint8_t>& src, int mutations) {
  run_all(src);
  for (int m = 0; m < mutations; ++m) {
    std::vector<uint8_t> b = src;
    const int kind = (int)(rnd() % 5);
    if (b.empty()) break;
    if (kind == 0) {  // truncation
      b.resize(rnd() % b.size());
    } else if (kind == 1) {  // 1-8 bit flips
      const int k = 1 + (int)(rnd() % 8);
      for (int i = 0; i < k; ++i) b[rnd() % b.size()] ^= (uint8_t)(1u << (rnd() % 8));
    } else if (kind == 2) {  // a run of bytes overwritten (0x00, 0xFF or random)
      const size_t at = rnd() % b.size(), len = 1 + rnd() % 16;
      const int how = (int)(rnd() % 3);
      for (size_t i = at; i < b.size() && i < at + len; ++i) b[i] = how == 0 ? 0 : how == 1 ? 0xFF : (uint8_t)rnd();
    } else if (kind == 3) {  // a chunk duplicated in place (lengths / page sequence disagree)
      const size_t at = rnd() % b.size(), len = 1 + rnd() % 64;
      std::vector<uint8_t> c(b.begin() + at, b.begin() + std::min(b.size(), at + len));
      b.insert(b.begin() + at, c.begin(), c.end());
    } else {  // a header-sized prefix kept, the rest random
      const size_t keep = std::min(b.size(), (size_t)(rnd() % 256));
      for (size_t i = keep; i < b.size(); ++i) b[i] = (uint8_t)rnd();
    }
    run_all(b);
  }
}

int main(int argc, char** argv) {
  int mutations = 200;
  int i = 1;
  for (; i < argc && argv[i][0] == '-'; i += 2) {
    if (i + 1 >= argc) return 2;
    if (!strcmp(argv[i], "-m")) mutations = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "-s")) g_rng ^= strtoull(argv[i + 1], nullptr, 10);
    else return 2;
  }
  for (; i < argc; ++i) {
    FILE* f = fopen(argv[i], "rb");
    if (!f) {
      fprintf(stderr, "cannot open %s\n", argv[i]);
      return 2;
    }
    std::vector<uint8_t> buf;
    uint8_t tmp[65536];
    size_t r;
    while ((r = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + r);
    fclose(f);
    mutate_and_run(buf, mutations);
  }
  printf("codec_fuzz: %ld inputs, %ld decodes accepted, no sanitizer report\n", g_runs, g_ok);
  return 0;
}
