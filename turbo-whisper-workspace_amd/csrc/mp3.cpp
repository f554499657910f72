// Native MPEG audio decoder: MPEG-1 / MPEG-2 LSF / MPEG-2.5 Layer III ("MP3"), and Layers I and II (host side of the
// audio ingest, include/tw_audio.h).
//
// Replaces the codec half of the reference's ffmpeg_read ($TF/pipelines/audio_utils.py:9-45) for MP3 uploads: the
// reference's POST /api/transcribe stores any upload under its own suffix (vocalis/api/main.py:67-75) and its own
// callers list .mp3 (vocalis/security/security_monitor.py:353, scripts/normalize_audio.py:226); ffmpeg's mp3 demuxer
// takes MPEG audio of any layer under that name (mp1 / mp2 / mp3float decoders). Written from ISO/IEC 11172-3 and
// 13818-3: frame sync and header, side information, the bit reservoir (main_data_begin), scalefactors
// (MPEG-1 scfsi sharing; the LSF scalefac_compress partitions incl. the intensity-stereo right channel), Huffman
// big-values / count1 decoding with the standard's tables (mp3_tables.h), requantisation (|is|^(4/3), global gain,
// subblock gain, scalefac_scale, pre-emphasis), short-block reordering, mid/side and intensity stereo (MPEG-1 tan
// ratios, LSF intensity_scale powers), alias reduction, the IMDCT with the four window shapes and overlap-add,
// frequency inversion and the 32-band polyphase synthesis filter bank. The Xing / Info / VBRI frame is skipped and
// a LAME (or Lavf / Lavc) tag's encoder delay and padding trim the output to the encoded length, as ffmpeg's mp3
// demuxer does (delay + 529 decoder-delay samples skipped at the start, padding - 529 at the end). Layers I / II:
// bit allocation (Layer II's tables B.2a-d by rate and bitrate per channel, 13818-3's for LSF), scfsi, grouped
// codewords, joint-stereo subband sharing above the bound, then the same filter bank; no tag, no trim.
//
// Parallel decode: a Layer III frame depends on earlier frames only through (a) reservoir bytes, read here from one
// concatenated main-data buffer by offset, and (b) the IMDCT overlap and the synthesis buffer, which one decoded
// frame (>= 18 subband slots >= the filter bank's 16) fully determines; a Layer I / II frame only through the
// synthesis buffer (36 slots a Layer II frame, 12 a Layer I frame: two frames prime it). Threads therefore decode
// frame ranges, each starting one (Layer I: two) frames early with that output discarded: bit-identical to a serial
// decode for any thread count.
//
// Output: f32 samples, interleaved [frames][channels], nominal full scale +-1 (what ffmpeg's float decoders hand to
// its resampler).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/tw_audio.h"
#include "mp3_tables.h"

void tw_set_error(const char* fmt, ...);

namespace {

using namespace mp3t;

// ---- frame header ---------------------------------------------------------------------------------------------------
struct Header {
  int layer = 3;  // 1, 2 or 3
  int lsf = 0;  // 1: MPEG-2 / MPEG-2.5 (Layer III: one granule per frame, LSF scalefactors)
  int version = 1;  // 1, 2 or 25
  int crc = 0;  // a 16-bit CRC follows the header
  int bitrate = 0, sr_index = 0, sample_rate = 0, padding = 0;
  int mode = 0, mode_ext = 0, channels = 0;
  int frame_bytes = 0, side_bytes = 0, granules = 0;
  int spf = 0;  // samples per channel per frame: 384 (Layer I), 1152 (Layer II, MPEG-1 Layer III), 576 (LSF III)
};

bool parse_header(const uint8_t* p, Header& h) {
  const uint32_t v = (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
  if ((v >> 21) != 0x7ffu) return false;
  const int ver = (v >> 19) & 3, lbits = (v >> 17) & 3, bri = (v >> 12) & 15, sri = (v >> 10) & 3;
  if (ver == 1 || lbits == 0 || bri == 0 || bri == 15 || sri == 3) return false;  // reserved / free format
  h.layer = 4 - lbits;
  h.lsf = ver != 3;
  h.version = ver == 3 ? 1 : ver == 2 ? 2 : 25;
  h.crc = !((v >> 16) & 1);
  h.sr_index = (ver == 3 ? 0 : ver == 2 ? 3 : 6) + sri;
  h.sample_rate = kSampleRate[h.sr_index];
  h.padding = (v >> 9) & 1;
  h.mode = (v >> 6) & 3;
  h.mode_ext = (v >> 4) & 3;
  h.channels = h.mode == 3 ? 1 : 2;
  if (h.layer == 3) {
    h.bitrate = kBitrate[h.lsf][bri];
    h.frame_bytes = (h.lsf ? 72000 : 144000) * h.bitrate / h.sample_rate + h.padding;
    h.side_bytes = h.lsf ? (h.channels == 1 ? 9 : 17) : (h.channels == 1 ? 17 : 32);
    h.granules = h.lsf ? 1 : 2;
    h.spf = 576 * h.granules;
  } else if (h.layer == 2) {  // 1152 samples in every version; 144 bytes per kbit/s / kHz
    h.bitrate = h.lsf ? kBitrate[1][bri] : kBitrateL12[1][bri];
    h.frame_bytes = 144000 * h.bitrate / h.sample_rate + h.padding;
    h.spf = 1152;
  } else {  // Layer I: 384 samples in 4-byte slots
    h.bitrate = kBitrateL12[h.lsf ? 2 : 0][bri];
    h.frame_bytes = (12000 * h.bitrate / h.sample_rate + h.padding) * 4;
    h.spf = 384;
  }
  return h.frame_bytes >= 4 + 2 * h.crc + h.side_bytes;
}

bool same_stream(const Header& a, const Header& b) {
  return a.layer == b.layer && a.lsf == b.lsf && a.version == b.version && a.sr_index == b.sr_index &&
         a.channels == b.channels;
}

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// a tag that may follow the last frame (ID3v1, APEv2, a trailing ID3v2): the stream ends there
bool trailing_tag(const uint8_t* d, int64_t pos, int64_t n) {
  return (pos + 3 <= n && memcmp(d + pos, "TAG", 3) == 0) || (pos + 8 <= n && memcmp(d + pos, "APETAGEX", 8) == 0) ||
         (pos + 3 <= n && memcmp(d + pos, "ID3", 3) == 0);
}

struct Stream {
  Header first;
  std::vector<int64_t> pos;  // byte offset of every audio frame
  std::vector<Header> hdr;
  int flags = 0;             // 1 Xing / Info frame, 2 LAME gapless fields, 4 VBRI frame
  int64_t tag_frames = -1;   // the Xing frame count (flags & 1 and its frames field present)
  int enc_delay = -1, enc_padding = -1;
  int64_t total = 0, skip = 0;  // output samples per channel after the trim, and samples skipped at the start
};

// a header at `pos` that the next frame (or the end of the data, or a trailing tag) confirms
bool confirmed(const uint8_t* d, int64_t n, int64_t pos, Header& h) {
  if (pos + 4 > n || !parse_header(d + pos, h) || pos + h.frame_bytes > n) return false;
  const int64_t nx = pos + h.frame_bytes;
  if (nx == n || trailing_tag(d, nx, n)) return true;
  Header g;
  return nx + 4 <= n && parse_header(d + nx, g) && same_stream(h, g);
}

bool scan(const uint8_t* d, int64_t n, Stream& s, const char** err) {
  int64_t pos = 0;
  while (pos + 10 <= n && memcmp(d + pos, "ID3", 3) == 0) {  // ID3v2 tags (several may precede the audio)
    const int64_t sz = (int64_t)(d[pos + 6] & 127) << 21 | (d[pos + 7] & 127) << 14 | (d[pos + 8] & 127) << 7 |
                       (d[pos + 9] & 127);
    pos += 10 + sz + ((d[pos + 5] & 0x10) ? 10 : 0);
  }
  Header h;
  while (pos + 4 <= n && !confirmed(d, n, pos, h)) pos++;
  if (pos + 4 > n) {
    *err = "MP3: no MPEG audio frame found";
    return false;
  }
  s.first = h;
  while (pos + 4 <= n) {
    if (parse_header(d + pos, h) && same_stream(h, s.first) && pos + h.frame_bytes <= n) {
      s.pos.push_back(pos);
      s.hdr.push_back(h);
      pos += h.frame_bytes;
      continue;
    }
    if (trailing_tag(d, pos, n) || pos + 4 + 32 > n) break;
    // lost sync (junk between frames): resynchronise on the next header of the same stream (version, rate and
    // channel count fixed by the confirmed first frame)
    int64_t q = pos + 1;
    while (q + 4 <= n && !(parse_header(d + q, h) && same_stream(h, s.first) && q + h.frame_bytes <= n)) q++;
    pos = q;
  }
  // the first frame may be a Xing / Info (LAME) or VBRI header frame instead of audio (Layer III only: the tag
  // sits after the Layer III side information)
  const int64_t p0 = s.pos[0];
  const Header& h0 = s.hdr[0];
  const int64_t fend = p0 + h0.frame_bytes;
  const int64_t xo = p0 + 4 + h0.side_bytes;  // (the offset ignores the CRC, as encoders and ffmpeg place it)
  const bool l3 = h0.layer == 3;
  if (l3 && xo + 8 <= fend && (memcmp(d + xo, "Xing", 4) == 0 || memcmp(d + xo, "Info", 4) == 0)) {
    s.flags |= 1;
    const uint32_t fl = be32(d + xo + 4);
    int64_t q = xo + 8;
    if ((fl & 1) && q + 4 <= fend) s.tag_frames = be32(d + q);
    q += (fl & 1) ? 4 : 0;
    q += (fl & 2) ? 4 : 0;
    q += (fl & 4) ? 100 : 0;
    q += (fl & 8) ? 4 : 0;
    // LAME extension: 9-byte encoder string, then (after 12 bytes of rev / lowpass / peak / gains / flags / abr)
    // 12 bits of encoder delay and 12 bits of padding
    if (q + 24 <= fend && (memcmp(d + q, "LAME", 4) == 0 || memcmp(d + q, "Lavf", 4) == 0 ||
                           memcmp(d + q, "Lavc", 4) == 0)) {
      const uint8_t* g = d + q + 21;
      s.enc_delay = g[0] << 4 | g[1] >> 4;
      s.enc_padding = (g[1] & 15) << 8 | g[2];
      s.flags |= 2;
    }
  } else if (l3 && p0 + 4 + 32 + 4 <= fend && memcmp(d + p0 + 4 + 32, "VBRI", 4) == 0) {
    s.flags |= 4;
  }
  if (s.flags & 5) {
    s.pos.erase(s.pos.begin());
    s.hdr.erase(s.hdr.begin());
  }
  const int64_t spf = s.first.spf;
  const int64_t decoded = (int64_t)s.pos.size() * spf;
  if (s.flags & 2) {
    const int64_t frames = s.tag_frames >= 0 ? s.tag_frames : (int64_t)s.pos.size();
    s.skip = s.enc_delay + 529;
    const int64_t end = std::min(decoded, frames * spf - s.enc_padding + 529);
    s.total = std::max<int64_t>(0, end - s.skip);
  } else {
    s.skip = 0;
    s.total = decoded;
  }
  return true;
}

// ---- bit reader (MSB first), reads past the end as zeros -------------------------------------------------------------
struct Bits {
  const uint8_t* d;
  int64_t nbytes;
  int64_t pos = 0;  // bit position
  uint32_t peek32() const {
    const int64_t b = pos >> 3;
    uint64_t w = 0;
    if (b >= 0 && b + 8 <= nbytes) {
      for (int i = 0; i < 8; i++) w = w << 8 | d[b + i];
    } else {
      for (int i = 0; i < 8; i++) w = w << 8 | ((b + i >= 0 && b + i < nbytes) ? d[b + i] : 0);
    }
    return (uint32_t)((w << (pos & 7)) >> 32);
  }
  uint32_t get(int n) {
    if (n <= 0) return 0;
    const uint32_t v = peek32() >> (32 - n);
    pos += n;
    return v;
  }
};

// ---- Huffman decoders built from the code tables ------------------------------------------------------------------
constexpr int kLutBits = 8;
struct Huff {
  // tree: node pairs; child >= 1 another node, child < 0 a leaf ~value, 0 absent
  std::vector<int32_t> tree;
  // lut[peek 8 bits]: leaf -> (len << 16 | value | 0x8000'0000), else (node index) with bit 31 clear; -1 invalid
  int32_t lut[1 << kLutBits];
  bool ok = false;
  void build(const uint16_t* code, const uint8_t* len, int n) {
    tree.assign(2, 0);
    for (int v = 0; v < n; v++) {
      int node = 0;
      for (int b = len[v] - 1; b >= 0; b--) {
        const int bit = (code[v] >> b) & 1;
        if (b == 0) {
          tree[2 * node + bit] = ~v;
        } else {
          if (tree[2 * node + bit] <= 0) {
            tree[2 * node + bit] = (int32_t)(tree.size() / 2);
            tree.push_back(0);
            tree.push_back(0);
          }
          node = tree[2 * node + bit];
        }
      }
    }
    for (int p = 0; p < (1 << kLutBits); p++) {
      int node = 0, l = 0;
      int32_t e = -1;
      for (; l < kLutBits; l++) {
        const int c = tree[2 * node + ((p >> (kLutBits - 1 - l)) & 1)];
        if (c < 0) {
          e = (int32_t)(0x80000000u | (uint32_t)(l + 1) << 16 | (uint32_t)~c);
          break;
        }
        if (c == 0) break;  // (a hole: a complete code has none)
        node = c;
      }
      if (l == kLutBits) e = node;
      lut[p] = e;
    }
    ok = true;
  }
  // value, or -1 for a codeword the table lacks
  inline int decode(Bits& br) const {
    const uint32_t w = br.peek32();
    const int32_t e = lut[w >> (32 - kLutBits)];
    if (e < -1 || (uint32_t)e & 0x80000000u) {
      if (e == -1) return -1;
      br.pos += ((uint32_t)e >> 16) & 0x7fff;
      return e & 0xffff;
    }
    int node = e, l = kLutBits;
    for (; l < 32; l++) {
      const int c = tree[2 * node + ((w >> (31 - l)) & 1)];
      if (c < 0) {
        br.pos += l + 1;
        return ~c;
      }
      if (c == 0) return -1;
      node = c;
    }
    return -1;
  }
};

struct Tables {
  Huff pair[32];  // by table_select (shared tables built once per distinct code table)
  Huff quadA;
  float pow43[8207];
  float win[4][36];     // long block windows by block_type (2: the short window in [0, 12))
  float cos36[18][36];  // IMDCT-36: cos(pi/72 (2i + 19)(2k + 1)) x window, per block type below
  float imdct_long[4][18][36];  // [block type][k][i]: the inner loops run over i (vectorised)
  float imdct_short[6][12];     // [k][i]: cos(pi/24 (2i + 7)(2k + 1)) x short window
  float cs[8], ca[8];
  float N[32][64];  // synthesis matrixing cos((16 + i)(2k + 1) pi / 64), [k][i]
  float D[512];     // synthesis window
  float is_ratio[16][2];  // MPEG-1 intensity (left, right) by is_pos
  Tables() {
    for (int t = 0; t < 32; t++) {
      const HuffSpec& sp = kHuff[t];
      if (!sp.code) continue;
      int same = -1;
      for (int u = 0; u < t; u++)
        if (kHuff[u].code == sp.code) same = u;
      if (same >= 0) {
        pair[t] = pair[same];
      } else {
        pair[t].build(sp.code, sp.len, sp.dim * sp.dim);
      }
    }
    {
      uint16_t c[16];
      for (int i = 0; i < 16; i++) c[i] = hAc[i];
      quadA.build(c, hAl, 16);
    }
    for (int i = 0; i < 8207; i++) pow43[i] = (float)pow((double)i, 4.0 / 3.0);
    for (int i = 0; i < 36; i++) {
      const double s36 = sin(M_PI / 36 * (i + 0.5));
      win[0][i] = (float)s36;
      win[1][i] = (float)(i < 18 ? s36 : i < 24 ? 1.0 : i < 30 ? sin(M_PI / 12 * (i - 18 + 0.5)) : 0.0);
      win[3][i] = (float)(i < 6 ? 0.0 : i < 12 ? sin(M_PI / 12 * (i - 6 + 0.5)) : i < 18 ? 1.0 : s36);
      win[2][i] = (float)(i < 12 ? sin(M_PI / 12 * (i + 0.5)) : 0.0);
    }
    for (int bt = 0; bt < 4; bt++)
      for (int i = 0; i < 36; i++)
        for (int k = 0; k < 18; k++)
          imdct_long[bt][k][i] =
              (float)(cos(M_PI / 72 * (2 * i + 19) * (2 * k + 1)) * (bt == 2 ? 0.0 : (double)win[bt][i]));
    for (int i = 0; i < 12; i++)
      for (int k = 0; k < 6; k++)
        imdct_short[k][i] = (float)(cos(M_PI / 24 * (2 * i + 7) * (2 * k + 1)) * sin(M_PI / 12 * (i + 0.5)));
    for (int i = 0; i < 8; i++) {
      const double c = kAliasC[i], r = sqrt(1.0 + c * c);
      cs[i] = (float)(1.0 / r);
      ca[i] = (float)(c / r);
    }
    for (int i = 0; i < 64; i++)
      for (int k = 0; k < 32; k++) N[k][i] = (float)cos((16 + i) * (2 * k + 1) * M_PI / 64);
    for (int i = 0; i < 512; i++) {
      const int j = i <= 256 ? i : 512 - i;
      D[i] = (float)(kWin[j] * (((i >> 6) & 1) ? -1.0 : 1.0) / 65536.0);
    }
    for (int p = 0; p < 16; p++) {
      if (p < 7) {
        const double t = tan(p * M_PI / 12);
        is_ratio[p][0] = (float)(t / (1 + t));
        is_ratio[p][1] = (float)(1 / (1 + t));
      } else {
        is_ratio[p][0] = is_ratio[p][1] = 0.f;
      }
    }
  }
};

const Tables& tables() {
  static const Tables t;
  return t;
}

// ---- side information -------------------------------------------------------------------------------------------
struct Granule {
  int part2_3_length = 0, big_values = 0, global_gain = 0, scalefac_compress = 0;
  int window_switching = 0, block_type = 0, mixed = 0;
  int table_select[3] = {0, 0, 0}, subblock_gain[3] = {0, 0, 0};
  int region0_count = 0, region1_count = 0;
  int preflag = 0, scalefac_scale = 0, count1table_select = 0;
  bool bad = false;  // reserved combination: decoded as silence
};

struct SideInfo {
  int main_data_begin = 0;
  int scfsi[2][4] = {{0}};
  Granule gr[2][2];
};

void parse_side(const uint8_t* p, int bytes, const Header& h, SideInfo& si) {
  Bits br{p, bytes};
  const int nch = h.channels;
  if (!h.lsf) {
    si.main_data_begin = br.get(9);
    br.get(nch == 1 ? 5 : 3);
    for (int ch = 0; ch < nch; ch++)
      for (int b = 0; b < 4; b++) si.scfsi[ch][b] = br.get(1);
  } else {
    si.main_data_begin = br.get(8);
    br.get(nch == 1 ? 1 : 2);
  }
  for (int gr = 0; gr < h.granules; gr++)
    for (int ch = 0; ch < nch; ch++) {
      Granule& g = si.gr[gr][ch];
      g.part2_3_length = br.get(12);
      g.big_values = br.get(9);
      g.global_gain = br.get(8);
      g.scalefac_compress = br.get(h.lsf ? 9 : 4);
      g.window_switching = br.get(1);
      if (g.window_switching) {
        g.block_type = br.get(2);
        g.mixed = br.get(1);
        for (int r = 0; r < 2; r++) g.table_select[r] = br.get(5);
        for (int w = 0; w < 3; w++) g.subblock_gain[w] = br.get(3);
        if (g.block_type == 0) g.bad = true;
        g.region0_count = (g.block_type == 2 && !g.mixed) ? 8 : 7;
        g.region1_count = 20 - g.region0_count;
      } else {
        for (int r = 0; r < 3; r++) g.table_select[r] = br.get(5);
        g.region0_count = br.get(4);
        g.region1_count = br.get(3);
      }
      if (!h.lsf) g.preflag = br.get(1);
      g.scalefac_scale = br.get(1);
      g.count1table_select = br.get(1);
      if (g.big_values > 288) g.bad = true;
    }
}

// scalefactors of one granule / channel
struct Scalefac {
  int l[22];             // long bands (21: none transmitted)
  int s[13][3];          // short bands x windows (12: none transmitted)
  int l_bad[22];         // LSF: the illegal intensity position of the band ((1 << slen) - 1)
  int s_bad[13][3];
  int intensity_scale;   // LSF intensity stereo, right channel
};

// ---- one decoder state (overlap + synthesis buffers per channel) ------------------------------------------------------
struct State {
  float overlap[2][32][18];
  float V[2][1024];
  int voff[2];
  void reset() {
    memset(overlap, 0, sizeof(overlap));
    memset(V, 0, sizeof(V));
    voff[0] = voff[1] = 0;
  }
};

struct Decoder {
  const uint8_t* data;
  const Stream& st;
  const std::vector<uint8_t>& md;       // concatenated main data of every audio frame
  const std::vector<int64_t>& md_off;   // where each frame's own main data starts in md
  const Tables& T = tables();

  // MPEG-1 scalefactors (scfsi copies the first granule's groups)
  void read_scalefac_v1(Bits& br, const Granule& g, const SideInfo& si, int gr, int ch, Scalefac& sf) const {
    const int s1 = kSlen[0][g.scalefac_compress], s2 = kSlen[1][g.scalefac_compress];
    if (g.window_switching && g.block_type == 2) {
      if (g.mixed) {
        for (int b = 0; b < 8; b++) sf.l[b] = br.get(s1);
        for (int b = 3; b < 12; b++)
          for (int w = 0; w < 3; w++) sf.s[b][w] = br.get(b < 6 ? s1 : s2);
      } else {
        for (int b = 0; b < 12; b++)
          for (int w = 0; w < 3; w++) sf.s[b][w] = br.get(b < 6 ? s1 : s2);
      }
      for (int w = 0; w < 3; w++) sf.s[12][w] = 0;
    } else {
      static const int edge[5] = {0, 6, 11, 16, 21};
      for (int k = 0; k < 4; k++) {
        if (gr == 1 && si.scfsi[ch][k]) continue;  // kept from granule 0
        for (int b = edge[k]; b < edge[k + 1]; b++) sf.l[b] = br.get(k < 2 ? s1 : s2);
      }
      sf.l[21] = 0;
    }
  }

  // MPEG-2 LSF scalefactors (13818-3 2.4.3.2): scalefac_compress selects four slen and a partition of the bands
  void read_scalefac_lsf(Bits& br, const Granule& g, const Header& h, int ch, Scalefac& sf, int& preflag) const {
    int sfc = g.scalefac_compress, slen[4] = {0, 0, 0, 0}, tab;
    preflag = 0;
    const bool is_right = ch == 1 && h.mode == 1 && (h.mode_ext & 1);
    if (!is_right) {
      if (sfc < 400) {
        slen[0] = (sfc >> 4) / 5, slen[1] = (sfc >> 4) % 5, slen[2] = (sfc & 15) >> 2, slen[3] = sfc & 3, tab = 0;
      } else if (sfc < 500) {
        sfc -= 400;
        slen[0] = (sfc >> 2) / 5, slen[1] = (sfc >> 2) % 5, slen[2] = sfc & 3, tab = 1;
      } else {
        sfc -= 500;
        slen[0] = sfc / 3, slen[1] = sfc % 3, tab = 2;
        preflag = 1;
      }
      sf.intensity_scale = 0;
    } else {
      sf.intensity_scale = sfc & 1;
      sfc >>= 1;
      if (sfc < 180) {
        slen[0] = sfc / 36, slen[1] = (sfc % 36) / 6, slen[2] = (sfc % 36) % 6, tab = 3;
      } else if (sfc < 244) {
        sfc -= 180;
        slen[0] = (sfc & 63) >> 4, slen[1] = (sfc & 15) >> 2, slen[2] = sfc & 3, tab = 4;
      } else {
        sfc -= 244;
        slen[0] = sfc / 3, slen[1] = sfc % 3, tab = 5;
      }
    }
    const int kind = (g.window_switching && g.block_type == 2) ? (g.mixed ? 2 : 1) : 0;
    int vals[40], bad[40], k = 0;
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < kNrOfSfb[tab][kind][i]; j++, k++) {
        vals[k] = br.get(slen[i]);
        bad[k] = (1 << slen[i]) - 1;
      }
    for (; k < 40; k++) vals[k] = 0, bad[k] = 0;
    if (kind == 0) {
      for (int b = 0; b < 21; b++) sf.l[b] = vals[b], sf.l_bad[b] = bad[b];
      sf.l[21] = 0, sf.l_bad[21] = sf.l_bad[20];
    } else {
      int q = 0, b0 = 0;
      if (kind == 2) {
        for (int b = 0; b < 6; b++) sf.l[b] = vals[b], sf.l_bad[b] = bad[b];
        q = 6, b0 = 3;
      }
      for (int b = b0; b < 12; b++)
        for (int w = 0; w < 3; w++, q++) sf.s[b][w] = vals[q], sf.s_bad[b][w] = bad[q];
      for (int w = 0; w < 3; w++) sf.s[12][w] = 0, sf.s_bad[12][w] = sf.s_bad[11][w];
    }
  }

  // Huffman data of one granule / channel into is[576]; returns the end of the coded (possibly non-zero) lines
  int huffman(Bits& br, int64_t end, const Granule& g, int sri, int* is) const {
    const int big = std::min(g.big_values * 2, 576);
    int r1, r2;
    if (g.window_switching) {
      r1 = (g.block_type == 2 && !g.mixed) ? 3 * kSfbShort[sri][3] : kSfbLong[sri][8];
      r2 = 576;
    } else {
      r1 = kSfbLong[sri][std::min(g.region0_count + 1, 22)];
      r2 = kSfbLong[sri][std::min(g.region0_count + g.region1_count + 2, 22)];
    }
    r1 = std::min(r1, big), r2 = std::min(r2, big);
    int i = 0;
    for (; i < big; i += 2) {
      const int t = g.table_select[i < r1 ? 0 : i < r2 ? 1 : 2];
      const HuffSpec& sp = kHuff[t];
      int x = 0, y = 0;
      if (sp.code) {
        const int v = T.pair[t].decode(br);
        if (v < 0) break;  // (a damaged stream: the rest of the granule is silent)
        x = v / sp.dim, y = v % sp.dim;
        if (sp.linbits && x == 15) x += br.get(sp.linbits);
        if (x && br.get(1)) x = -x;
        if (sp.linbits && y == 15) y += br.get(sp.linbits);
        if (y && br.get(1)) y = -y;
      }
      is[i] = x, is[i + 1] = y;
    }
    const int bigend = i;
    for (; bigend == big && i + 4 <= 576 && br.pos < end;) {
      const int64_t at = br.pos;
      int v;
      if (g.count1table_select) {
        v = 15 - (int)br.get(4);
      } else {
        v = T.quadA.decode(br);
        if (v < 0) break;
      }
      int q[4] = {(v >> 3) & 1, (v >> 2) & 1, (v >> 1) & 1, v & 1};
      for (int j = 0; j < 4; j++)
        if (q[j] && br.get(1)) q[j] = -1;
      if (br.pos > end) {  // the last quadruple overran part2_3_length: dropped (as ffmpeg / mpg123)
        br.pos = at;
        break;
      }
      for (int j = 0; j < 4; j++) is[i + j] = q[j];
      i += 4;
    }
    for (int j = i; j < 576; j++) is[j] = 0;
    return i;
  }

  // requantise into xr (bitstream order: short bands window after window)
  void requantize(const Granule& g, const Scalefac& sf, int preflag, int sri, const int* is, int nz, float* xr) const {
    const double sfm = g.scalefac_scale ? 1.0 : 0.5;
    const double gain = 0.25 * (g.global_gain - 210);
    for (int j = 0; j < 576; j++) xr[j] = 0.f;
    auto put = [&](int a, int b, double e) {
      const double m = exp2(e);
      for (int j = a; j < b && j < nz; j++) {
        const int v = is[j];
        if (!v) continue;
        const double q = (double)T.pow43[std::min(v < 0 ? -v : v, 8206)] * m;
        xr[j] = (float)(v < 0 ? -q : q);
      }
    };
    const bool shortb = g.window_switching && g.block_type == 2;
    int long_end = 576, short_start = 13;
    if (shortb) {
      long_end = g.mixed ? 3 * kSfbShort[sri][3] : 0;
      short_start = g.mixed ? 3 : 0;
    }
    for (int b = 0; b < 22 && kSfbLong[sri][b] < long_end; b++)
      put(kSfbLong[sri][b], std::min<int>(kSfbLong[sri][b + 1], long_end),
          gain - sfm * (sf.l[b] + (preflag ? kPretab[b] : 0)));
    if (shortb)
      for (int b = short_start; b < 13; b++) {
        const int w0 = kSfbShort[sri][b], W = kSfbShort[sri][b + 1] - w0;
        for (int w = 0; w < 3; w++)
          put(3 * w0 + w * W, 3 * w0 + (w + 1) * W, gain - 2.0 * g.subblock_gain[w] - sfm * sf.s[b][w]);
      }
  }

  // short bands from window-after-window to frequency-major order (line f of window w at 3 f + w within the band)
  static void reorder(const Granule& g, int sri, float* xr) {
    if (!(g.window_switching && g.block_type == 2)) return;
    float tmp[576];
    for (int b = g.mixed ? 3 : 0; b < 13; b++) {
      const int w0 = kSfbShort[sri][b], W = kSfbShort[sri][b + 1] - w0;
      float* p = xr + 3 * w0;
      for (int f = 0; f < W; f++)
        for (int w = 0; w < 3; w++) tmp[3 * f + w] = p[w * W + f];
      memcpy(p, tmp, sizeof(float) * 3 * W);
    }
  }

  // joint stereo: intensity above the right channel's last non-zero band (per window for short blocks), mid/side
  // below it or everywhere (11172-3 2.4.3.4.9.2-3; 13818-3 2.4.3.2 for the LSF intensity positions)
  void stereo(const Header& h, const Granule& g1, const Scalefac& sf1, int sri, float* L, float* R) const {
    if (h.mode != 1 || h.channels != 2) return;
    const bool ms = h.mode_ext & 2, ist = h.mode_ext & 1;
    const float r2 = (float)(1.0 / sqrt(2.0));
    auto do_ms = [&](int idx) {
      const float m = L[idx], s = R[idx];
      L[idx] = (m + s) * r2;
      R[idx] = (m - s) * r2;
    };
    if (!ist) {
      if (ms)
        for (int j = 0; j < 576; j++) do_ms(j);
      return;
    }
    const double io = h.lsf ? (sf1.intensity_scale ? 1.0 / sqrt(2.0) : 1.0 / sqrt(sqrt(2.0))) : 0.0;
    // (left, right) gains of an intensity position; false: illegal (no intensity: mid/side if enabled)
    auto is_gain = [&](int pos, int bad, float& kl, float& kr) {
      if (!h.lsf) {
        if (pos == 7) return false;
        kl = T.is_ratio[pos & 15][0], kr = T.is_ratio[pos & 15][1];
        return true;
      }
      if (pos == bad) return false;
      kl = kr = 1.f;
      if (pos & 1)
        kl = (float)pow(io, (pos + 1) / 2);
      else if (pos)
        kr = (float)pow(io, pos / 2);
      return true;
    };
    auto band = [&](const int* idx, int n, bool above, int pos, int bad) {
      float kl, kr;
      if (above && is_gain(pos, bad, kl, kr)) {
        for (int j = 0; j < n; j++) {
          const float v = L[idx[j]];
          L[idx[j]] = v * kl;
          R[idx[j]] = v * kr;
        }
      } else if (ms) {
        for (int j = 0; j < n; j++) do_ms(idx[j]);
      }
    };
    int idx[576];
    const bool shortb = g1.window_switching && g1.block_type == 2;
    bool long_above = true;  // the long bands (of a long or mixed block) lie above every non-zero right line
    if (shortb) {
      const int sstart = g1.mixed ? 3 : 0;
      bool any_nz = false;
      for (int w = 0; w < 3; w++) {
        bool above = true;
        for (int b = 12; b >= sstart; b--) {
          const int w0 = kSfbShort[sri][b], W = kSfbShort[sri][b + 1] - w0;
          for (int f = 0; f < W; f++) idx[f] = 3 * w0 + 3 * f + w;
          if (above)
            for (int f = 0; f < W; f++)
              if (R[idx[f]] != 0.f) {
                above = false;
                break;
              }
          const int bb = b == 12 ? 11 : b;
          band(idx, W, above, sf1.s[bb][w], h.lsf ? sf1.s_bad[bb][w] : 7);
        }
        if (!above) any_nz = true;
      }
      if (!g1.mixed) return;
      long_above = !any_nz;
    }
    const int long_end = shortb ? 3 * kSfbShort[sri][3] : 576;
    int top = 0;
    while (top < 22 && kSfbLong[sri][top] < long_end) top++;
    bool above = long_above;
    for (int b = top - 1; b >= 0; b--) {
      const int a = kSfbLong[sri][b], e = std::min<int>(kSfbLong[sri][b + 1], long_end);
      for (int j = a; j < e; j++) idx[j - a] = j;
      if (above)
        for (int j = a; j < e; j++)
          if (R[j] != 0.f) {
            above = false;
            break;
          }
      const int bb = b == 21 ? 20 : b;
      band(idx, e - a, above, sf1.l[bb], h.lsf ? sf1.l_bad[bb] : 7);
    }
  }

  void antialias(const Granule& g, float* xr) const {
    int n = 31;
    if (g.window_switching && g.block_type == 2) {
      if (!g.mixed) return;
      n = 1;
    }
    for (int sb = 0; sb < n; sb++) {
      float* a = xr + 18 * sb + 17;
      float* b = xr + 18 * sb + 18;
      for (int i = 0; i < 8; i++) {
        const float u = a[-i], v = b[i];
        a[-i] = u * T.cs[i] - v * T.ca[i];
        b[i] = v * T.cs[i] + u * T.ca[i];
      }
    }
  }

  // IMDCT + overlap-add + frequency inversion -> sb[18][32]
  void imdct(const Granule& g, const float* xr, float (*ov)[18], float (*out)[32]) const {
    const bool shortb = g.window_switching && g.block_type == 2;
    const int long_end = shortb ? (g.mixed ? 2 : 0) : 32;
    for (int sb = 0; sb < 32; sb++) {
      const float* X = xr + 18 * sb;
      float z[36];
      bool zero = true;
      for (int k = 0; k < 18; k++)
        if (X[k] != 0.f) zero = false;
      if (zero) {
        for (int i = 0; i < 36; i++) z[i] = 0.f;
      } else if (sb < long_end) {
        const int bt = shortb ? 0 : g.block_type;
        for (int i = 0; i < 36; i++) z[i] = 0.f;
        for (int k = 0; k < 18; k++) {
          const float xk = X[k];
          const float* c = T.imdct_long[bt][k];
          for (int i = 0; i < 36; i++) z[i] += c[i] * xk;
        }
      } else {
        for (int i = 0; i < 36; i++) z[i] = 0.f;
        for (int w = 0; w < 3; w++) {
          float y[12] = {0.f};
          for (int k = 0; k < 6; k++) {
            const float xk = X[3 * k + w];
            for (int i = 0; i < 12; i++) y[i] += T.imdct_short[k][i] * xk;
          }
          for (int i = 0; i < 12; i++) z[6 + 6 * w + i] += y[i];
        }
      }
      for (int i = 0; i < 18; i++) {
        float v = z[i] + ov[sb][i];
        if ((sb & 1) && (i & 1)) v = -v;
        out[i][sb] = v;
        ov[sb][i] = z[18 + i];
      }
    }
  }

  // polyphase synthesis of `nslot` subband slots of one channel: pcm[slot * 32 + j] (stride `stride` floats)
  void synth(const float (*sbs)[32], int nslot, float* V, int& voff, float* pcm, int stride) const {
    for (int s = 0; s < nslot; s++) {
      voff = (voff - 64) & 1023;
      const float* S = sbs[s];
      // matrixing into the newest 64-value block of V (voff is a multiple of 64, so every block is contiguous)
      float* vv = V + voff;
      for (int i = 0; i < 64; i++) vv[i] = 0.f;
      for (int k = 0; k < 32; k++) {
        const float sk = S[k];
        if (sk == 0.f) continue;
        const float* n = T.N[k];
        for (int i = 0; i < 64; i++) vv[i] += n[i] * sk;
      }
      // windowing: out[j] = sum_i V[128 i + j] D[64 i + j] + V[128 i + 96 + j] D[64 i + 32 + j] over 32 contiguous j
      float acc[32] = {0.f};
      for (int i = 0; i < 8; i++) {
        const float* v0 = V + ((voff + 128 * i) & 1023);
        const float* v1 = V + ((voff + 128 * i + 96) & 1023);
        const float* d0 = T.D + 64 * i;
        for (int j = 0; j < 32; j++) acc[j] += v0[j] * d0[j] + v1[j] * d0[32 + j];
      }
      for (int j = 0; j < 32; j++) pcm[(size_t)(s * 32 + j) * stride] = acc[j];
    }
  }

  // ---- Layers I and II (11172-3 2.4.3.2 / 2.4.3.3; 13818-3 2.4.3.2 for LSF Layer II's table) -----------------------
  // A frame is self-contained: bit allocation, scalefactors and samples of the 32 subbands, then the same synthesis
  // filter bank as Layer III. A sample code v of a class with L steps dequantises to (2 v + 1 - L) / L times the
  // scalefactor 2^(1 - index / 3) (the standard's C (s'' + D) with s'' the code read as a two's-complement fraction,
  // MSB inverted, written in closed form).
  static float scale(int idx) { return (float)exp2(1.0 - idx / 3.0); }
  static float dequant(int v, int steps) { return (float)((2.0 * v + 1.0 - steps) / steps); }

  // Layer I: 12 slots; joint stereo shares the allocation and samples of subbands >= bound (each channel keeps its
  // own scalefactor). An allocation of 15 (forbidden) makes the frame silent.
  bool layer1(Bits& br, const Header& h, int bound, float (*sbs)[36][32]) const {
    const int nch = h.channels;
    int alloc[2][32], scf[2][32];
    for (int sb = 0; sb < 32; sb++) {
      if (sb < bound) {
        for (int ch = 0; ch < nch; ch++) alloc[ch][sb] = br.get(4);
      } else {
        alloc[0][sb] = alloc[1][sb] = br.get(4);
      }
      for (int ch = 0; ch < nch; ch++)
        if (alloc[ch][sb] == 15) return false;
    }
    for (int sb = 0; sb < 32; sb++)
      for (int ch = 0; ch < nch; ch++) scf[ch][sb] = alloc[ch][sb] ? br.get(6) : 0;
    for (int s = 0; s < 12; s++)
      for (int sb = 0; sb < 32; sb++) {
        if (sb < bound) {
          for (int ch = 0; ch < nch; ch++)
            if (const int n = alloc[ch][sb])
              sbs[ch][s][sb] = dequant(br.get(n + 1), (2 << n) - 1) * scale(scf[ch][sb]);
        } else if (const int n = alloc[0][sb]) {
          const float q = dequant(br.get(n + 1), (2 << n) - 1);
          for (int ch = 0; ch < nch; ch++) sbs[ch][s][sb] = q * scale(scf[ch][sb]);
        }
      }
    return true;
  }

  // the Layer II allocation table (11172-3 Annex B Table B.2 by sampling rate and bitrate per channel; LSF: 13818-3
  // Table B.1)
  static int l2_table(const Header& h) {
    if (h.lsf) return 4;
    const int chb = h.bitrate / h.channels;
    if ((h.sample_rate == 48000 && chb >= 56) || (chb >= 56 && chb <= 80)) return 0;
    if (h.sample_rate != 48000 && chb >= 96) return 1;
    if (h.sample_rate != 32000 && chb <= 48) return 2;
    return 3;
  }

  // Layer II: 36 slots in 12 granules of 3; scfsi selects how the three scalefactors of a subband are shared across
  // the frame's three parts of 12 slots
  bool layer2(Bits& br, const Header& h, int bound, float (*sbs)[36][32]) const {
    const int nch = h.channels, tab = l2_table(h), sblimit = kL2Sblimit[tab];
    bound = std::min(bound, sblimit);
    int cls[2][32], scf[2][32][3];
    for (int sb = 0; sb < sblimit; sb++) {
      const int row = kL2SbRow[tab][sb], nbal = kL2RowBits[row];
      int a[2] = {0, 0};
      if (sb < bound) {
        for (int ch = 0; ch < nch; ch++) a[ch] = br.get(nbal);
      } else {
        a[0] = a[1] = br.get(nbal);
      }
      for (int ch = 0; ch < 2; ch++) cls[ch][sb] = a[ch] ? kL2Row[row][a[ch] - 1] : -1;
    }
    int scfsi[2][32];
    for (int sb = 0; sb < sblimit; sb++)
      for (int ch = 0; ch < nch; ch++) scfsi[ch][sb] = cls[ch][sb] >= 0 ? br.get(2) : 0;
    for (int sb = 0; sb < sblimit; sb++)
      for (int ch = 0; ch < nch; ch++) {
        int* f = scf[ch][sb];
        if (cls[ch][sb] < 0) {
          f[0] = f[1] = f[2] = 0;
          continue;
        }
        switch (scfsi[ch][sb]) {
          case 0: f[0] = br.get(6), f[1] = br.get(6), f[2] = br.get(6); break;
          case 1: f[0] = f[1] = br.get(6), f[2] = br.get(6); break;
          case 2: f[0] = f[1] = f[2] = br.get(6); break;
          default: f[0] = br.get(6), f[1] = f[2] = br.get(6); break;
        }
      }
    // one triple of sample codes of class c (grouped: one codeword; the third value is the quotient left after two
    // divisions, as ffmpeg's division tables hold it for codewords past steps^3)
    auto triple = [&](int c, float* q) {
      const int L = kL2Steps[c];
      if (kL2Grouped[c]) {
        int v = br.get(kL2Bits[c]);
        const int a = v % L;
        v /= L;
        const int b = v % L;
        q[0] = dequant(a, L), q[1] = dequant(b, L), q[2] = dequant(v / L, L);
      } else {
        for (int j = 0; j < 3; j++) q[j] = dequant(br.get(kL2Bits[c]), L);
      }
    };
    for (int gr = 0; gr < 12; gr++)
      for (int sb = 0; sb < sblimit; sb++) {
        float q[3];
        if (sb < bound) {
          for (int ch = 0; ch < nch; ch++)
            if (cls[ch][sb] >= 0) {
              triple(cls[ch][sb], q);
              const float f = scale(scf[ch][sb][gr >> 2]);
              for (int j = 0; j < 3; j++) sbs[ch][3 * gr + j][sb] = q[j] * f;
            }
        } else if (cls[0][sb] >= 0) {
          triple(cls[0][sb], q);
          for (int ch = 0; ch < nch; ch++) {
            const float f = scale(scf[ch][sb][gr >> 2]);
            for (int j = 0; j < 3; j++) sbs[ch][3 * gr + j][sb] = q[j] * f;
          }
        }
      }
    return true;
  }

  void frame_l12(int64_t k, State& S, float* pcm) const {
    const Header& h = st.hdr[k];
    Bits br{data + st.pos[k], h.frame_bytes};
    br.pos = 32 + 16 * h.crc;
    const int nch = h.channels, nslot = h.spf / 32;
    static thread_local float sbs[2][36][32];
    memset(sbs, 0, sizeof(sbs));
    const int bound = h.mode == 1 ? 4 * (h.mode_ext + 1) : 32;
    if (!(h.layer == 1 ? layer1(br, h, bound, sbs) : layer2(br, h, bound, sbs))) memset(sbs, 0, sizeof(sbs));
    for (int ch = 0; ch < nch; ch++) {
      static thread_local float scratch[1152];
      synth(sbs[ch], nslot, S.V[ch], S.voff[ch], pcm ? pcm + ch : scratch, pcm ? nch : 1);
    }
  }

  // decode frame k into pcm[spf][channels] (nullptr: state only)
  void frame(int64_t k, State& S, float* pcm) const {
    const Header& h = st.hdr[k];
    if (h.layer != 3) return frame_l12(k, S, pcm);
    const int64_t p = st.pos[k];
    SideInfo si;
    parse_side(data + p + 4 + 2 * h.crc, h.side_bytes, h, si);
    const int nch = h.channels, sri = h.sr_index;
    Bits br{md.data(), (int64_t)md.size()};
    const int64_t start = md_off[k] - si.main_data_begin;
    const bool have_data = start >= 0;
    br.pos = std::max<int64_t>(start, 0) * 8;
    Scalefac sf[2];
    memset(sf, 0, sizeof(sf));
    static thread_local float xr[2][576];
    static thread_local int is[576];
    static thread_local float sbs[18][32];
    for (int gr = 0; gr < h.granules; gr++) {
      int nz[2] = {0, 0};
      for (int ch = 0; ch < nch; ch++) {
        const Granule& g = si.gr[gr][ch];
        const int64_t g0 = br.pos, end = g0 + g.part2_3_length;
        int preflag = g.preflag;
        if (!h.lsf)
          read_scalefac_v1(br, g, si, gr, ch, sf[ch]);
        else
          read_scalefac_lsf(br, g, h, ch, sf[ch], preflag);
        if (have_data && !g.bad && br.pos <= end) {
          nz[ch] = huffman(br, end, g, sri, is);
          requantize(g, sf[ch], preflag, sri, is, nz[ch], xr[ch]);
          reorder(g, sri, xr[ch]);
        } else {
          memset(xr[ch], 0, sizeof(xr[ch]));
        }
        br.pos = end;
      }
      if (nch == 2) stereo(h, si.gr[gr][1], sf[1], sri, xr[0], xr[1]);
      for (int ch = 0; ch < nch; ch++) {
        const Granule& g = si.gr[gr][ch];
        antialias(g, xr[ch]);
        imdct(g, xr[ch], S.overlap[ch], sbs);
        float scratch[576];
        float* out = pcm ? pcm + (size_t)gr * 576 * nch + ch : scratch;
        synth(sbs, 18, S.V[ch], S.voff[ch], out, pcm ? nch : 1);
      }
    }
  }
};

bool build_main_data(const uint8_t* d, const Stream& s, std::vector<uint8_t>& md, std::vector<int64_t>& off) {
  md.clear();
  off.resize(s.pos.size());
  for (size_t k = 0; k < s.pos.size(); k++) {
    const Header& h = s.hdr[k];
    off[k] = (int64_t)md.size();
    if (h.layer != 3) continue;  // (Layers I / II: no reservoir)
    const int64_t a = s.pos[k] + 4 + 2 * h.crc + h.side_bytes, b = s.pos[k] + h.frame_bytes;
    md.insert(md.end(), d + a, d + b);
  }
  return true;
}

}  // namespace

extern "C" {

int tw_mp3_probe(const uint8_t* data, int64_t size, TwMp3Info* info) {
  if (!data || size < 4 || !info) {
    tw_set_error("tw_mp3_probe: empty input");
    return 1;
  }
  Stream s;
  const char* err = nullptr;
  if (!scan(data, size, s, &err)) {
    tw_set_error("%s", err);
    return 2;
  }
  memset(info, 0, sizeof(*info));
  info->sample_rate = s.first.sample_rate;
  info->channels = s.first.channels;
  info->version = s.first.version;
  info->bitrate_kbps = s.pos.empty() ? s.first.bitrate : s.hdr[0].bitrate;
  info->total_samples = s.total;
  info->n_frames = (int64_t)s.pos.size();
  info->samples_per_frame = s.first.spf;
  info->layer = s.first.layer;
  info->enc_delay = s.enc_delay;
  info->enc_padding = s.enc_padding;
  info->flags = s.flags;
  info->skip_samples = s.skip;
  return 0;
}

int tw_mp3_decode(const uint8_t* data, int64_t size, float* out, int64_t out_frames, int32_t n_threads,
                  int64_t* frames_decoded) {
  if (!data || size < 4 || !out) {
    tw_set_error("tw_mp3_decode: null or empty argument");
    return 1;
  }
  Stream s;
  const char* err = nullptr;
  if (!scan(data, size, s, &err)) {
    tw_set_error("%s", err);
    return 2;
  }
  if (out_frames < s.total) {
    tw_set_error("tw_mp3_decode: out_frames %lld < %lld samples", (long long)out_frames, (long long)s.total);
    return 3;
  }
  std::vector<uint8_t> md;
  std::vector<int64_t> off;
  build_main_data(data, s, md, off);
  const int nch = s.first.channels;
  const int64_t spf = s.first.spf, nf = (int64_t)s.pos.size();
  // frames of priming before a thread's range: enough subband slots for the synthesis buffer's 16 (Layer I's 12 slots
  // per frame need two frames)
  const int64_t warm = s.first.layer == 1 ? 2 : 1;
  Decoder dec{data, s, md, off};
  int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, nf / 8));
  auto work = [&](int64_t a, int64_t b) {
    State S;
    S.reset();
    std::vector<float> pcm((size_t)spf * nch);
    for (int64_t k = std::max<int64_t>(0, a - warm); k < b; k++) {
      dec.frame(k, S, pcm.data());
      if (k < a) continue;  // warm-up frames: prime the overlap and synthesis buffers only
      const int64_t g0 = k * spf - s.skip;
      for (int64_t i = 0; i < spf; i++) {
        const int64_t o = g0 + i;
        if (o < 0 || o >= s.total) continue;
        memcpy(out + o * nch, pcm.data() + i * nch, sizeof(float) * nch);
      }
    }
  };
  if (nt == 1) {
    work(0, nf);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++) th.emplace_back(work, nf * t / nt, nf * (t + 1) / nt);
    for (auto& x : th) x.join();
  }
  if (frames_decoded) *frames_decoded = s.total;
  return 0;
}

}  // extern "C"
