// Native Ogg Vorbis decoder (host side of the audio ingest, include/tw_audio.h).
//
// Replaces the container + codec half of the reference's ffmpeg_read ($TF/pipelines/audio_utils.py:9-45) for Ogg
// Vorbis uploads (the reference's POST /api/transcribe stores any upload under its own suffix and hands the path to
// the ASR pipeline, vocalis/api/main.py:67-75; vocalis' normalize_audio.py lists .ogg among its inputs). Written from
// the Ogg framing specification (RFC 3533) and the Vorbis I specification: Ogg pages (CRC-32 checked) and packet
// lacing; the identification / setup headers (Huffman codebooks with VQ lookup types 1 and 2, floor type 1,
// residue types 0 / 1 / 2, mappings with channel coupling, modes); audio packets: floor-1 curve synthesis, residue
// decode, inverse coupling, the floor x residue product, the inverse MDCT (an N/4-point complex FFT), the power-sine
// windows with short / long transitions, overlap-add, and the end trim to the last page's granule position.
// Floor type 0 (LSP) is refused: no encoder in use emits it (libvorbis has written floor 1 since 2002).
//
// Output: f32 samples, interleaved [frames][channels], in the codec's own scale (the inverse MDCT unnormalised, as
// libvorbis's mdct_backward), the values ffmpeg's libvorbis / native decoder hand to its resampler.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/tw_audio.h"

void tw_set_error(const char* fmt, ...);

namespace {

// ---- Ogg framing ----------------------------------------------------------------------------------------------------
uint32_t g_crc32[256];
struct Crc32Init {
  Crc32Init() {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t r = i << 24;
      for (int b = 0; b < 8; b++) r = (r & 0x80000000u) ? (r << 1) ^ 0x04c11db7u : (r << 1);
      g_crc32[i] = r;
    }
  }
} g_crc32_init;

struct OggPacket {
  std::vector<uint8_t> data;
  int64_t granule;  // the granule position of the page this packet ends on (-1: the page ends no packet)
  bool last_on_page;
};

// Every packet of the first logical stream (the serial of the first page). Returns false with an error message.
bool ogg_packets(const uint8_t* d, int64_t n, std::vector<OggPacket>& out, const char** err) {
  int64_t pos = 0;
  bool have_serial = false;
  uint32_t serial = 0;
  std::vector<uint8_t> cur;
  while (pos + 27 <= n) {
    if (memcmp(d + pos, "OggS", 4) != 0) {
      *err = "Ogg: lost page sync";
      return false;
    }
    if (d[pos + 4] != 0) {
      *err = "Ogg: unknown page version";
      return false;
    }
    const uint8_t htype = d[pos + 5];
    int64_t granule;
    memcpy(&granule, d + pos + 6, 8);
    uint32_t ser, crc;
    memcpy(&ser, d + pos + 14, 4);
    memcpy(&crc, d + pos + 22, 4);
    const int nseg = d[pos + 26];
    if (pos + 27 + nseg > n) {
      *err = "Ogg: truncated page header";
      return false;
    }
    const uint8_t* lace = d + pos + 27;
    int64_t body = 0;
    for (int i = 0; i < nseg; i++) body += lace[i];
    const int64_t hlen = 27 + nseg;
    if (pos + hlen + body > n) {
      *err = "Ogg: truncated page";
      return false;
    }
    uint32_t c = 0;
    for (int64_t i = 0; i < hlen + body; i++) {
      const uint8_t b = (i >= 22 && i < 26) ? 0 : d[pos + i];
      c = (c << 8) ^ g_crc32[((c >> 24) & 0xff) ^ b];
    }
    if (c != crc) {
      *err = "Ogg: page CRC mismatch";
      return false;
    }
    if (!have_serial) {
      serial = ser;
      have_serial = true;
    }
    if (ser == serial) {
      if (!(htype & 1)) cur.clear();  // (not a continuation: a dangling partial packet is dropped)
      const uint8_t* p = d + pos + hlen;
      size_t first_new = out.size();
      for (int i = 0; i < nseg; i++) {
        cur.insert(cur.end(), p, p + lace[i]);
        p += lace[i];
        if (lace[i] < 255) {
          out.push_back(OggPacket{cur, -1, false});
          cur.clear();
        }
      }
      if (out.size() > first_new) {
        out.back().granule = granule;
        out.back().last_on_page = true;
      }
    }
    pos += hlen + body;
  }
  if (!have_serial) {
    *err = "Ogg: no page";
    return false;
  }
  return true;
}

// ---- bit reader (Vorbis packs LSB first) ----------------------------------------------------------------------------
struct BitReader {
  const uint8_t* d;
  size_t n;
  size_t bit = 0;
  bool eop = false;  // read past the end of the packet (sticky; every later read returns 0)
  BitReader(const uint8_t* d_, size_t n_) : d(d_), n(n_) {}
  size_t left() const { return eop ? 0 : n * 8 - bit; }
  uint32_t peek24() const {  // the next 24 bits, zero-padded past the end
    const size_t b = bit >> 3;
    uint32_t w = 0;
    if (b + 4 <= n) {
      memcpy(&w, d + b, 4);
    } else {
      for (size_t i = 0; b + i < n && i < 4; i++) w |= (uint32_t)d[b + i] << (8 * i);
    }
    return (w >> (bit & 7)) & 0xffffffu;
  }
  uint32_t get(int k) {  // k <= 32; a read that runs past the end returns 0
    if (eop || bit + k > n * 8) {
      eop = true;
      bit = n * 8;
      return 0;
    }
    uint32_t v;
    if (k <= 24) {
      v = peek24() & ((1u << k) - 1);
    } else {
      const uint32_t lo = peek24();
      bit += 24;
      v = lo | ((peek24() & ((1u << (k - 24)) - 1)) << 24);
      bit -= 24;
    }
    bit += k;
    return v;
  }
  uint32_t get1() { return get(1); }
};

int ilog(uint32_t x) {
  int r = 0;
  while (x) {
    r++;
    x >>= 1;
  }
  return r;
}

float float32_unpack(uint32_t x) {
  double mant = (double)(x & 0x1fffff);
  const int exp = (int)((x & 0x7fe00000u) >> 21);
  if (x & 0x80000000u) mant = -mant;
  return (float)ldexp(mant, exp - 788);
}

// ---- codebooks -------------------------------------------------------------------------------------------------------
struct Codebook {
  int dims = 0, entries = 0;
  std::vector<int8_t> len;        // codeword length per entry, 0 = unused
  std::vector<int32_t> tree;      // binary tree: node i has children tree[2i], tree[2i+1]; < 0: leaf -(entry+1)
  int lookup = 0;
  std::vector<float> vq;          // [entries][dims] decoded VQ vectors (lookup 1 / 2)
  int used = 0;                   // used entries

  bool build(const char** err) {
    // codewords in entry order, each the lowest free one of its length (Vorbis I §3.2.1)
    uint32_t avail[33] = {0};
    tree.assign(2, 0);
    int nodes = 1;
    used = 0;
    for (int e = 0; e < entries; e++) used += len[e] > 0;
    if (used == 0) return true;  // (a single used entry gets codeword 0 of its length, read like any other)
    bool first = true;
    for (int e = 0; e < entries; e++) {
      const int L = len[e];
      if (L <= 0) continue;
      uint32_t code;
      if (first) {
        code = 0;
        for (int i = 1; i <= L; i++) avail[i] = 1u << (32 - i);
        first = false;
      } else {
        int z = L;
        while (z > 0 && !avail[z]) z--;
        if (z == 0) {
          *err = "Vorbis: overspecified Huffman codebook";
          return false;
        }
        code = avail[z];
        avail[z] = 0;
        for (int y = L; y > z; y--) avail[y] = code + (1u << (32 - y));
      }
      // insert code (its top L bits, MSB first = first bit read)
      int node = 0;
      for (int i = 0; i < L; i++) {
        const int bitv = (code >> (31 - i)) & 1;
        int32_t& child = tree[2 * node + bitv];
        if (i == L - 1) {
          if (child != 0) {
            *err = "Vorbis: Huffman codeword collision";
            return false;
          }
          child = -(e + 1);
        } else {
          if (child < 0) {
            *err = "Vorbis: Huffman prefix collision";
            return false;
          }
          if (child == 0) {
            child = nodes++;
            tree.resize(2 * (size_t)nodes, 0);
          }
          node = tree[2 * node + bitv];
        }
      }
    }
    return true;
  }

  // codewords of up to FB bits by one table lookup on the next FB bits (first bit read = lowest index bit):
  // fast[idx] = entry | length << 24, -1 for no codeword, -2 for the prefix of a longer codeword (tree walk)
  static constexpr int FB = 10;
  std::vector<int32_t> fast;

  void build_fast() {
    fast.assign(1 << FB, -1);
    std::vector<std::pair<int, int>> stack{{0, 0}};  // (node, depth) ; path bits kept alongside
    std::vector<uint32_t> path{0};
    while (!stack.empty()) {
      const auto [node, depth] = stack.back();
      const uint32_t bits = path.back();
      stack.pop_back();
      path.pop_back();
      for (int b = 0; b < 2; b++) {
        const int32_t c = tree[2 * node + b];
        const uint32_t nb = bits | ((uint32_t)b << depth);
        if (c < 0) {
          for (uint32_t f = 0; f < (1u << (FB - depth - 1)); f++)
            fast[nb | (f << (depth + 1))] = (-c - 1) | ((depth + 1) << 24);
        } else if (c > 0) {
          if (depth + 1 < FB) {
            stack.push_back({c, depth + 1});
            path.push_back(nb);
          } else {
            fast[nb] = -2;
          }
        }
      }
    }
  }

  int decode(BitReader& br) const {  // entry number, -1 at the end of the packet
    if (used == 0) return -1;
    const int32_t t = fast[br.peek24() & ((1u << FB) - 1)];
    if (t >= 0) {
      const int L = t >> 24;
      if ((size_t)L > br.left()) {
        br.get(L);  // (runs past the end: sets eop)
        return -1;
      }
      br.bit += L;
      return t & 0xffffff;
    }
    if (t == -1) return -1;
    int node = 0;
    for (int depth = 0; depth < 33; depth++) {
      const int b = (int)br.get1();
      if (br.eop) return -1;
      const int32_t c = tree[2 * node + b];
      if (c < 0) return -c - 1;
      if (c == 0) return -1;  // (an unassigned codeword: treated as the end of the packet)
      node = c;
    }
    return -1;
  }
};

int lookup1_values(int entries, int dims) {
  int r = (int)floor(exp(log((double)entries) / dims));
  while (true) {  // the largest r with r^dims <= entries
    double p1 = pow((double)(r + 1), dims);
    if (p1 <= entries) {
      r++;
      continue;
    }
    double p = pow((double)r, dims);
    if (p > entries) {
      r--;
      continue;
    }
    break;
  }
  return r;
}

bool read_codebook(BitReader& br, Codebook& cb, const char** err) {
  if (br.get(24) != 0x564342) {
    *err = "Vorbis: bad codebook sync";
    return false;
  }
  cb.dims = (int)br.get(16);
  cb.entries = (int)br.get(24);
  if (cb.dims <= 0 || cb.entries <= 0) {
    *err = "Vorbis: empty codebook";
    return false;
  }
  // (bounds no encoder comes near — libvorbis's largest books hold a few thousand entries of <= 8 dimensions — that
  // keep a damaged or hostile header from allocating gigabytes for its tree or VQ table)
  if (cb.entries > (1 << 20) || (long)cb.entries * cb.dims > (1L << 24)) {
    *err = "Vorbis: codebook too large";
    return false;
  }
  cb.len.assign(cb.entries, 0);
  const bool ordered = br.get1();
  if (!ordered) {
    const bool sparse = br.get1();
    for (int e = 0; e < cb.entries; e++) {
      if (sparse && !br.get1()) continue;
      cb.len[e] = (int8_t)(br.get(5) + 1);
    }
  } else {
    int cur = 0, L = (int)br.get(5) + 1;
    while (cur < cb.entries) {
      const int num = (int)br.get(ilog((uint32_t)(cb.entries - cur)));
      if (cur + num > cb.entries || L > 32) {
        *err = "Vorbis: bad ordered codebook";
        return false;
      }
      for (int i = 0; i < num; i++) cb.len[cur + i] = (int8_t)L;
      cur += num;
      L++;
    }
  }
  cb.lookup = (int)br.get(4);
  if (cb.lookup == 1 || cb.lookup == 2) {
    const float minv = float32_unpack(br.get(32)), delta = float32_unpack(br.get(32));
    const int vbits = (int)br.get(4) + 1;
    const bool seq = br.get1();
    const long nvals = cb.lookup == 1 ? lookup1_values(cb.entries, cb.dims) : (long)cb.entries * cb.dims;
    if (nvals <= 0 || nvals > (1L << 24)) {
      *err = "Vorbis: bad VQ lookup size";
      return false;
    }
    std::vector<uint32_t> mult(nvals);
    for (long i = 0; i < nvals; i++) mult[i] = br.get(vbits);
    cb.vq.assign((size_t)cb.entries * cb.dims, 0.f);
    for (int e = 0; e < cb.entries; e++) {
      float last = 0.f;
      long div = 1;
      for (int i = 0; i < cb.dims; i++) {
        const long off = cb.lookup == 1 ? (e / div) % nvals : (long)e * cb.dims + i;
        const float v = (float)mult[off] * delta + minv + last;
        cb.vq[(size_t)e * cb.dims + i] = v;
        if (seq) last = v;
        if (cb.lookup == 1) div *= nvals;
      }
    }
  } else if (cb.lookup != 0) {
    *err = "Vorbis: bad codebook lookup type";
    return false;
  }
  if (br.eop) {
    *err = "Vorbis: truncated setup header";
    return false;
  }
  if (!cb.build(err)) return false;
  if (cb.used > 0) cb.build_fast();
  return true;
}

// ---- floor 1 ---------------------------------------------------------------------------------------------------------
struct Floor1 {
  std::vector<int> part_class;
  int cdim[16], csub[16], cmaster[16], subbook[16][8];
  int mult = 1;
  std::vector<int> X;        // post x positions in header order
  std::vector<int> order;    // post indices sorted by X
  std::vector<int> lo, hi;   // low / high neighbour of each post (index >= 2)
};

float g_inv_db[256];
struct InvDbInit {
  // floor1_inverse_dB_table (Vorbis I §10.1): a geometric table from 1.0649863e-07 to 1 over 256 steps (the spec's
  // literals are this ratio's powers rounded to 8 digits)
  InvDbInit() {
    const double r = pow(1.0 / 1.0649863e-07, 1.0 / 255.0);
    for (int i = 0; i < 256; i++) g_inv_db[i] = (float)pow(r, (double)(i - 255));
  }
} g_inv_db_init;

void render_line(int x0, int y0, int x1, int y1, int n, std::vector<int>& v) {
  const int dy = y1 - y0, adx = x1 - x0;
  int ady = abs(dy);
  const int base = dy / adx;
  const int sy = dy < 0 ? base - 1 : base + 1;
  int x = x0, y = y0, err = 0;
  ady -= abs(base) * adx;
  if (x < n) v[x] = y;
  for (x = x0 + 1; x < x1; x++) {
    err += ady;
    if (err >= adx) {
      err -= adx;
      y += sy;
    } else {
      y += base;
    }
    if (x < n) v[x] = y;
  }
}

int render_point(int x0, int y0, int x1, int y1, int X) {
  const int dy = y1 - y0, adx = x1 - x0, ady = abs(dy);
  const long long err = (long long)ady * (X - x0);  // (64-bit: no overflow for any post values)
  const int off = (int)(err / adx);
  return dy < 0 ? y0 - off : y0 + off;
}

// ---- residues, mappings, modes ----------------------------------------------------------------------------------------
struct Residue {
  int type = 0, begin = 0, end = 0, psize = 1, classes = 1, classbook = 0;
  int books[64][8];
};

struct Mapping {
  int submaps = 1;
  std::vector<int> mag, ang;   // coupling steps
  std::vector<int> mux;        // submap per channel
  int floor_of[16], residue_of[16];
};

struct Mode {
  int blockflag = 0, mapping = 0;
};

// ---- inverse MDCT ------------------------------------------------------------------------------------------------------
// y[i] = sum_{k < M} X[k] cos(pi / M (i + 1/2 + M/2)(k + 1/2)), i < N = 2M. With u = DCT-IV(X),
// u[j] = sum_k X[k] cos(pi / M (j + 1/2)(k + 1/2)), the output unfolds as y[i] = u[i + M/2] (i < M/2),
// -u[3M/2 - 1 - i] (i < 3M/2), -u[i - 3M/2] (i < 2M); u comes from one M/2-point complex FFT:
// v[j] = (X[2j] + i X[M-1-2j]) e^{-i pi (j + 1/4) / M}, V = FFT(v), V[j] *= e^{-i pi j / M}, u[2j] = Re V[j],
// u[M-1-2j] = -Im V[j].
struct Imdct {
  int N = 0, M = 0, H = 0;
  std::vector<float> twr, twi;                  // per stage len: twiddles e^{-2 pi i j / len}, j < len/2, at [len/2 + j]
  std::vector<float> prer, prei, postr, posti;  // e^{-i pi (j + 1/4) / M}, e^{-i pi j / M}
  std::vector<int> rev;
  void init(int n) {
    N = n;
    M = n / 2;
    H = M / 2;
    int lg = 0;
    while ((1 << lg) < H) lg++;
    rev.resize(H);
    for (int i = 0; i < H; i++) {
      int r = 0;
      for (int b = 0; b < lg; b++) r |= ((i >> b) & 1) << (lg - 1 - b);
      rev[i] = r;
    }
    twr.assign(std::max(H, 2), 0.f);
    twi.assign(std::max(H, 2), 0.f);
    for (int len = 2; len <= H; len <<= 1)
      for (int j = 0; j < len / 2; j++) {
        twr[len / 2 + j] = (float)cos(-2.0 * M_PI * j / len);
        twi[len / 2 + j] = (float)sin(-2.0 * M_PI * j / len);
      }
    prer.resize(H);
    prei.resize(H);
    postr.resize(H);
    posti.resize(H);
    for (int j = 0; j < H; j++) {
      prer[j] = (float)cos(-M_PI * (j + 0.25) / M);
      prei[j] = (float)sin(-M_PI * (j + 0.25) / M);
      postr[j] = (float)cos(-M_PI * j / M);
      posti[j] = (float)sin(-M_PI * j / M);
    }
  }
  // y[0 .. N) from X[0 .. M) in float (as libvorbis and ffmpeg's decoder compute it); re / im: scratch
  void run(const float* X, float* y, std::vector<float>& re, std::vector<float>& im) const {
    re.resize(H);
    im.resize(H);
    float* ar = re.data();
    float* ai = im.data();
    for (int j = 0; j < H; j++) {
      const float xr = X[2 * j], xi = X[M - 1 - 2 * j];
      ar[rev[j]] = xr * prer[j] - xi * prei[j];
      ai[rev[j]] = xr * prei[j] + xi * prer[j];
    }
    for (int len = 2; len <= H; len <<= 1) {
      const int half = len >> 1;
      const float* wr = twr.data() + half;
      const float* wi = twi.data() + half;
      for (int s0 = 0; s0 < H; s0 += len) {
        float* pr = ar + s0;
        float* pi = ai + s0;
        float* qr = pr + half;
        float* qi = pi + half;
        for (int j = 0; j < half; j++) {
          const float tr = qr[j] * wr[j] - qi[j] * wi[j], ti = qr[j] * wi[j] + qi[j] * wr[j];
          qr[j] = pr[j] - tr;
          qi[j] = pi[j] - ti;
          pr[j] += tr;
          pi[j] += ti;
        }
      }
    }
    // u[2j] = Re(V[j] post[j]), u[M-1-2j] = -Im(V[j] post[j]); y unfolds u (see above), written directly
    const int q = M / 2;
    auto u = [&](int k) -> float {
      const int j = (k & 1) ? (M - 1 - k) >> 1 : k >> 1;
      return (k & 1) ? -(ar[j] * posti[j] + ai[j] * postr[j]) : ar[j] * postr[j] - ai[j] * posti[j];
    };
    for (int i = 0; i < q; i++) y[i] = u(i + q);
    for (int i = q; i < 3 * q; i++) y[i] = -u(3 * q - 1 - i);
    for (int i = 3 * q; i < N; i++) y[i] = -u(i - 3 * q);
  }
};

struct Decoder {
  int channels = 0, rate = 0, bs[2] = {0, 0};
  std::vector<Codebook> books;
  std::vector<Floor1> floors;
  std::vector<Residue> residues;
  std::vector<Mapping> maps;
  std::vector<Mode> modes;
  Imdct mdct[2];
  std::vector<float> win_slope[2];  // rising half-window of length bs[b] / 2
  std::vector<float> windows[5];    // [0]: short block; [1 + 2 prev + next]: long block with its neighbours' sizes

  bool ident(const std::vector<uint8_t>& p, const char** err) {
    if (p.size() < 30 || p[0] != 1 || memcmp(p.data() + 1, "vorbis", 6) != 0) {
      *err = "Vorbis: no identification header";
      return false;
    }
    BitReader br(p.data() + 7, p.size() - 7);
    if (br.get(32) != 0) {
      *err = "Vorbis: unknown version";
      return false;
    }
    channels = (int)br.get(8);
    rate = (int)br.get(32);
    br.get(32);
    br.get(32);
    br.get(32);
    bs[0] = 1 << br.get(4);
    bs[1] = 1 << br.get(4);
    if (channels < 1 || channels > 16 || rate <= 0 || bs[0] < 64 || bs[1] < bs[0] || bs[1] > 8192 || !br.get1()) {
      *err = "Vorbis: bad identification header";
      return false;
    }
    for (int b = 0; b < 2; b++) {
      mdct[b].init(bs[b]);
      const int h = bs[b] / 2;
      win_slope[b].resize(h);
      for (int i = 0; i < h; i++) {
        const double s = sin((i + 0.5) / h * M_PI / 2);
        win_slope[b][i] = (float)sin(M_PI / 2 * s * s);
      }
    }
    window(0, 0, 0, windows[0]);
    for (int pf = 0; pf < 2; pf++)
      for (int nf = 0; nf < 2; nf++) window(1, pf, nf, windows[1 + 2 * pf + nf]);
    return true;
  }

  bool setup(const std::vector<uint8_t>& p, const char** err) {
    if (p.size() < 8 || p[0] != 5 || memcmp(p.data() + 1, "vorbis", 6) != 0) {
      *err = "Vorbis: no setup header";
      return false;
    }
    BitReader br(p.data() + 7, p.size() - 7);
    const int nbooks = (int)br.get(8) + 1;
    books.resize(nbooks);
    for (auto& cb : books)
      if (!read_codebook(br, cb, err)) return false;
    const int ntime = (int)br.get(6) + 1;
    for (int i = 0; i < ntime; i++)
      if (br.get(16) != 0) {
        *err = "Vorbis: bad time-domain transform";
        return false;
      }
    const int nfloors = (int)br.get(6) + 1;
    floors.resize(nfloors);
    for (auto& f : floors) {
      const int type = (int)br.get(16);
      if (type == 0) {
        *err = "Vorbis: floor type 0 (LSP) is not decoded by this engine";
        return false;
      }
      if (type != 1) {
        *err = "Vorbis: bad floor type";
        return false;
      }
      const int parts = (int)br.get(5);
      f.part_class.resize(parts);
      int maxc = -1;
      for (int i = 0; i < parts; i++) {
        f.part_class[i] = (int)br.get(4);
        maxc = std::max(maxc, f.part_class[i]);
      }
      for (int c = 0; c <= maxc; c++) {
        f.cdim[c] = (int)br.get(3) + 1;
        f.csub[c] = (int)br.get(2);
        f.cmaster[c] = f.csub[c] ? (int)br.get(8) : -1;
        for (int j = 0; j < (1 << f.csub[c]); j++) f.subbook[c][j] = (int)br.get(8) - 1;
      }
      f.mult = (int)br.get(2) + 1;
      const int rbits = (int)br.get(4);
      f.X = {0, 1 << rbits};
      for (int i = 0; i < parts; i++)
        for (int j = 0; j < f.cdim[f.part_class[i]]; j++) f.X.push_back((int)br.get(rbits));
      if (f.X.size() > 65) {
        *err = "Vorbis: too many floor posts";
        return false;
      }
      const int nx = (int)f.X.size();
      f.order.resize(nx);
      for (int i = 0; i < nx; i++) f.order[i] = i;
      std::stable_sort(f.order.begin(), f.order.end(), [&](int a, int b) { return f.X[a] < f.X[b]; });
      for (int i = 1; i < nx; i++)
        if (f.X[f.order[i]] == f.X[f.order[i - 1]]) {
          *err = "Vorbis: repeated floor post";
          return false;
        }
      f.lo.assign(nx, 0);
      f.hi.assign(nx, 1);
      for (int i = 2; i < nx; i++) {
        int lo = 0, hi = 1, lox = -1, hix = 1 << 30;
        for (int j = 0; j < i; j++) {
          if (f.X[j] < f.X[i] && f.X[j] > lox) {
            lox = f.X[j];
            lo = j;
          }
          if (f.X[j] > f.X[i] && f.X[j] < hix) {
            hix = f.X[j];
            hi = j;
          }
        }
        f.lo[i] = lo;
        f.hi[i] = hi;
      }
      for (int i = 0; i < parts; i++) {
        const int c = f.part_class[i];
        if (f.cmaster[c] >= nbooks) {
          *err = "Vorbis: bad floor book";
          return false;
        }
        for (int j = 0; j < (1 << f.csub[c]); j++)
          if (f.subbook[c][j] >= nbooks) {
            *err = "Vorbis: bad floor book";
            return false;
          }
      }
    }
    const int nres = (int)br.get(6) + 1;
    residues.resize(nres);
    for (auto& r : residues) {
      r.type = (int)br.get(16);
      if (r.type > 2) {
        *err = "Vorbis: bad residue type";
        return false;
      }
      r.begin = (int)br.get(24);
      r.end = (int)br.get(24);
      r.psize = (int)br.get(24) + 1;
      r.classes = (int)br.get(6) + 1;
      r.classbook = (int)br.get(8);
      int cascade[64];
      for (int c = 0; c < r.classes; c++) {
        const int low = (int)br.get(3);
        const int high = br.get1() ? (int)br.get(5) : 0;
        cascade[c] = high * 8 + low;
      }
      for (int c = 0; c < r.classes; c++)
        for (int j = 0; j < 8; j++) r.books[c][j] = (cascade[c] >> j) & 1 ? (int)br.get(8) : -1;
      if (r.classbook >= nbooks || books[r.classbook].dims <= 0) {
        *err = "Vorbis: bad residue classbook";
        return false;
      }
      for (int c = 0; c < r.classes; c++)
        for (int j = 0; j < 8; j++)
          if (r.books[c][j] >= nbooks || (r.books[c][j] >= 0 && books[r.books[c][j]].vq.empty())) {
            *err = "Vorbis: bad residue book";
            return false;
          }
    }
    const int nmaps = (int)br.get(6) + 1;
    maps.resize(nmaps);
    for (auto& m : maps) {
      if (br.get(16) != 0) {
        *err = "Vorbis: bad mapping type";
        return false;
      }
      m.submaps = br.get1() ? (int)br.get(4) + 1 : 1;
      const int steps = br.get1() ? (int)br.get(8) + 1 : 0;
      const int cb = ilog((uint32_t)(channels - 1));
      for (int s = 0; s < steps; s++) {
        m.mag.push_back((int)br.get(cb));
        m.ang.push_back((int)br.get(cb));
        if (m.mag.back() == m.ang.back() || m.mag.back() >= channels || m.ang.back() >= channels) {
          *err = "Vorbis: bad channel coupling";
          return false;
        }
      }
      if (br.get(2) != 0) {
        *err = "Vorbis: bad mapping reserved bits";
        return false;
      }
      m.mux.assign(channels, 0);
      if (m.submaps > 1)
        for (int c = 0; c < channels; c++) {
          m.mux[c] = (int)br.get(4);
          if (m.mux[c] >= m.submaps) {
            *err = "Vorbis: bad mapping mux";
            return false;
          }
        }
      for (int s = 0; s < m.submaps; s++) {
        br.get(8);
        m.floor_of[s] = (int)br.get(8);
        m.residue_of[s] = (int)br.get(8);
        if (m.floor_of[s] >= nfloors || m.residue_of[s] >= nres) {
          *err = "Vorbis: bad mapping submap";
          return false;
        }
      }
    }
    const int nmodes = (int)br.get(6) + 1;
    modes.resize(nmodes);
    for (auto& md : modes) {
      md.blockflag = (int)br.get1();
      if (br.get(16) != 0 || br.get(16) != 0) {
        *err = "Vorbis: bad mode";
        return false;
      }
      md.mapping = (int)br.get(8);
      if (md.mapping >= nmaps) {
        *err = "Vorbis: bad mode mapping";
        return false;
      }
    }
    if (!br.get1() || br.eop) {
      *err = "Vorbis: bad setup header framing";
      return false;
    }
    return true;
  }

  // floor 1 of one channel: false = unused; else fl[0 .. n/2) = the curve
  bool floor1(const Floor1& f, BitReader& br, int n2, std::vector<float>& fl, std::vector<int>& v) const {
    if (!br.get1()) return false;
    static const int ranges[4] = {256, 128, 86, 64};
    const int range = ranges[f.mult - 1], rb = ilog((uint32_t)(range - 1));
    const int nx = (int)f.X.size();
    int Y[65];
    Y[0] = (int)br.get(rb);
    Y[1] = (int)br.get(rb);
    int off = 2;
    for (size_t p = 0; p < f.part_class.size(); p++) {
      const int c = f.part_class[p];
      const int cdim = f.cdim[c], cbits = f.csub[c], csub = (1 << cbits) - 1;
      int cval = 0;
      if (cbits > 0) {
        cval = books[f.cmaster[c]].decode(br);
        if (cval < 0) return false;  // (end of packet inside the floor: the channel is unused)
      }
      for (int j = 0; j < cdim; j++) {
        const int book = f.subbook[c][cval & csub];
        cval >>= cbits;
        if (book >= 0) {
          const int v = books[book].decode(br);
          if (v < 0) return false;
          Y[off + j] = v;
        } else {
          Y[off + j] = 0;
        }
      }
      off += cdim;
    }
    if (br.eop) return false;
    // amplitude value synthesis (§7.2.4 step 1)
    int fy[65];
    bool step2[65];
    fy[0] = Y[0];  // (read with ilog(range - 1) bits: < 2^16)
    fy[1] = Y[1];
    step2[0] = step2[1] = true;
    for (int i = 2; i < nx; i++) {
      const int lo = f.lo[i], hi = f.hi[i];
      const int pred = render_point(f.X[lo], fy[lo], f.X[hi], fy[hi], f.X[i]);
      const int val = Y[i], highroom = range - pred, lowroom = pred;
      const int room = (highroom < lowroom ? highroom : lowroom) * 2;
      if (val) {
        step2[lo] = step2[hi] = step2[i] = true;
        if (val >= room) fy[i] = highroom > lowroom ? val - lowroom + pred : pred - val + highroom - 1;
        else fy[i] = (val & 1) ? pred - (val + 1) / 2 : pred + val / 2;
      } else {
        step2[i] = false;
        fy[i] = pred;
      }
      // a hostile codebook entry (up to 2^20) can put a post far outside [0, range): clipped to [0, 65535] as ffmpeg's
      // decoder (the one ffmpeg_read runs) clips floor1_Y_final with av_clip_uint16, so neither the predictions
      // (render_point, 64-bit) nor the curve arithmetic can overflow; a valid stream's posts are unchanged
      fy[i] = std::min(std::max(fy[i], 0), 65535);
    }
    // curve synthesis (step 2): lines between the used posts in x order, then the dB table
    v.assign(n2, 0);
    int lx = 0, ly = fy[f.order[0]] * f.mult, hx = 0, hy = ly;
    for (int k = 1; k < nx; k++) {
      const int i = f.order[k];
      if (!step2[i]) continue;
      hy = fy[i] * f.mult;
      hx = f.X[i];
      render_line(lx, ly, hx, hy, n2, v);
      lx = hx;
      ly = hy;
    }
    if (hx < n2) render_line(hx, hy, n2, hy, n2, v);
    fl.resize(n2);
    for (int i = 0; i < n2; i++) fl[i] = g_inv_db[std::min(std::max(v[i], 0), 255)];
    return true;
  }

  // residue decode into the vectors of one submap (§8.6)
  void residue(const Residue& r, BitReader& br, int n2, std::vector<std::vector<float>*>& vecs,
               const std::vector<bool>& skip) const {
    const int ch = (int)vecs.size();
    if (r.type == 2) {
      bool any = false;
      for (int j = 0; j < ch; j++) any = any || !skip[j];
      if (!any) return;
      std::vector<float> il((size_t)n2 * ch, 0.f);
      std::vector<std::vector<float>*> one{&il};
      std::vector<bool> no{false};
      residue_core(r, 1, br, n2 * ch, one, no);
      for (int i = 0; i < n2; i++)
        for (int j = 0; j < ch; j++) (*vecs[j])[i] += il[(size_t)i * ch + j];
      return;
    }
    residue_core(r, r.type, br, n2, vecs, skip);
  }

  void residue_core(const Residue& r, int format, BitReader& br, int size, std::vector<std::vector<float>*>& vecs,
                    const std::vector<bool>& skip) const {
    const int ch = (int)vecs.size();
    const int lb = std::min(r.begin, size), le = std::min(r.end, size);
    const int nread = le - lb;
    if (nread <= 0) return;
    const int parts = nread / r.psize;
    const Codebook& cbk = books[r.classbook];
    const int cpw = cbk.dims;
    std::vector<std::vector<int>> cls(ch, std::vector<int>(parts + cpw, 0));
    for (int pass = 0; pass < 8; pass++) {
      int pc = 0;
      while (pc < parts) {
        if (pass == 0)
          for (int j = 0; j < ch; j++) {
            if (skip[j]) continue;
            int temp = cbk.decode(br);
            if (temp < 0) return;  // end of packet: the rest stays zero
            for (int i = cpw - 1; i >= 0; i--) {
              cls[j][i + pc] = temp % r.classes;
              temp /= r.classes;
            }
          }
        for (int i = 0; i < cpw && pc < parts; i++, pc++)
          for (int j = 0; j < ch; j++) {
            if (skip[j]) continue;
            const int book = r.books[cls[j][pc]][pass];
            if (book < 0) continue;
            const Codebook& vb = books[book];
            float* v = vecs[j]->data() + lb + pc * r.psize;
            const int d = vb.dims;
            if (format == 0) {
              const int step = r.psize / d;
              for (int s = 0; s < step; s++) {
                const int e = vb.decode(br);
                if (e < 0) return;
                for (int k = 0; k < d; k++) v[s + k * step] += vb.vq[(size_t)e * d + k];
              }
            } else {
              for (int s = 0; s < r.psize;) {
                const int e = vb.decode(br);
                if (e < 0) return;
                for (int k = 0; k < d && s < r.psize; k++) v[s++] += vb.vq[(size_t)e * d + k];
              }
            }
          }
      }
    }
  }

  struct Scratch {
    std::vector<std::vector<float>> resid, flo;
    std::vector<int> curve;
    std::vector<float> re, im;
  };

  // One audio packet -> its windowed block, channel-major [channels][n] in `block`. Returns n, 0 for a packet that
  // is skipped (not an audio packet, or it ends before its window flags), -1 for a bad mode number.
  int packet(const std::vector<uint8_t>& pk, Scratch& sc, std::vector<float>& block) const {
    if (pk.empty()) return 0;
    BitReader br(pk.data(), pk.size());
    if (br.get1() != 0) return 0;
    const int mode = (int)br.get(ilog((uint32_t)(modes.size() - 1)));
    if (mode >= (int)modes.size()) return -1;
    const int flag = modes[mode].blockflag, n = bs[flag], n2 = n / 2;
    int prevflag = 0, nextflag = 0;
    if (flag) {
      prevflag = (int)br.get1();
      nextflag = (int)br.get1();
    }
    if (br.eop) return 0;
    const int C = channels;
    sc.resid.resize(C);
    sc.flo.resize(C);
    const Mapping& m = maps[modes[mode].mapping];
    bool unused[16], noresid[16];
    for (int c = 0; c < C; c++) {
      unused[c] = !floor1(floors[m.floor_of[m.mux[c]]], br, n2, sc.flo[c], sc.curve);
      noresid[c] = unused[c];
      sc.resid[c].assign(n2, 0.f);
    }
    for (size_t k = 0; k < m.mag.size(); k++)
      if (!noresid[m.mag[k]] || !noresid[m.ang[k]]) noresid[m.mag[k]] = noresid[m.ang[k]] = false;
    for (int sm = 0; sm < m.submaps; sm++) {
      std::vector<std::vector<float>*> vecs;
      std::vector<bool> skip;
      for (int c = 0; c < C; c++)
        if (m.mux[c] == sm) {
          vecs.push_back(&sc.resid[c]);
          skip.push_back(noresid[c]);
        }
      if (!vecs.empty()) residue(residues[m.residue_of[sm]], br, n2, vecs, skip);
    }
    for (int k = (int)m.mag.size() - 1; k >= 0; k--) {  // inverse coupling (§9.3.5)
      float* M = sc.resid[m.mag[k]].data();
      float* A = sc.resid[m.ang[k]].data();
      for (int j = 0; j < n2; j++) {
        const float mv = M[j], av = A[j];
        float nm, na;
        if (mv > 0) {
          if (av > 0) {
            nm = mv;
            na = mv - av;
          } else {
            na = mv;
            nm = mv + av;
          }
        } else {
          if (av > 0) {
            nm = mv;
            na = mv + av;
          } else {
            na = mv;
            nm = mv - av;
          }
        }
        M[j] = nm;
        A[j] = na;
      }
    }
    const float* w = windows[flag ? 1 + 2 * prevflag + nextflag : 0].data();
    block.resize((size_t)C * n);
    for (int c = 0; c < C; c++) {
      float* y = block.data() + (size_t)c * n;
      if (unused[c]) {
        std::fill(y, y + n, 0.f);
        continue;
      }
      float* r = sc.resid[c].data();
      const float* f = sc.flo[c].data();
      for (int j = 0; j < n2; j++) r[j] *= f[j];
      mdct[flag].run(r, y, sc.re, sc.im);
      for (int i = 0; i < n; i++) y[i] *= w[i];
    }
    return n;
  }

  // window value i of an n-sample block with left / right halves from the neighbouring block sizes
  void window(int flag, int prevflag, int nextflag, std::vector<float>& w) const {
    const int n = bs[flag];
    w.assign(n, 0.f);
    const int ln = (flag && !prevflag) ? bs[0] / 2 : n / 2;
    const int rn = (flag && !nextflag) ? bs[0] / 2 : n / 2;
    const int ls = n / 4 - ln / 2, rs = 3 * n / 4 - rn / 2;
    const std::vector<float>& lsl = win_slope[ln == bs[0] / 2 ? 0 : 1];
    const std::vector<float>& rsl = win_slope[rn == bs[0] / 2 ? 0 : 1];
    for (int i = 0; i < ln; i++) w[ls + i] = lsl[i];
    for (int i = ls + ln; i < rs; i++) w[i] = 1.f;
    for (int i = 0; i < rn; i++) w[rs + i] = rsl[rn - 1 - i];
  }
};

}  // namespace

struct TwVorbisStream {
  Decoder dec;
  std::vector<OggPacket> packets;
};

static int vorbis_open(const uint8_t* data, int64_t size, TwVorbisStream& s) {
  const char* err = nullptr;
  if (!data || size <= 0) {
    tw_set_error("tw_vorbis: empty input");
    return 1;
  }
  if (!ogg_packets(data, size, s.packets, &err)) {
    tw_set_error("tw_vorbis: %s", err);
    return 1;
  }
  if (s.packets.size() < 3 || !s.dec.ident(s.packets[0].data, &err) ||
      (s.packets[1].data.size() < 7 || s.packets[1].data[0] != 3) || !s.dec.setup(s.packets[2].data, &err)) {
    tw_set_error("tw_vorbis: %s", err ? err : "Vorbis: missing comment header");
    return 1;
  }
  return 0;
}

extern "C" int tw_vorbis_probe(const uint8_t* data, int64_t size, TwVorbisInfo* info) {
  TwVorbisStream s;
  if (vorbis_open(data, size, s)) return 1;
  info->sample_rate = s.dec.rate;
  info->channels = s.dec.channels;
  info->blocksize0 = s.dec.bs[0];
  info->blocksize1 = s.dec.bs[1];
  int64_t g = 0;
  for (size_t i = 3; i < s.packets.size(); i++)
    if (s.packets[i].granule >= 0) g = s.packets[i].granule;
  info->total_samples = g;
  return 0;
}

extern "C" int tw_vorbis_decode(const uint8_t* data, int64_t size, float* out, int64_t out_frames, int32_t n_threads,
                                int64_t* frames_decoded) {
  TwVorbisStream s;
  if (vorbis_open(data, size, s)) return 1;
  if (!out || !frames_decoded || out_frames < 0) {
    tw_set_error("tw_vorbis_decode: null output");
    return 1;
  }
  const Decoder& d = s.dec;
  const int C = d.channels;
  int64_t end_granule = -1;
  for (size_t i = 3; i < s.packets.size(); i++)
    if (s.packets[i].granule >= 0) end_granule = s.packets[i].granule;
  // Packets decode independently (floor, residue, IMDCT, window); only the overlap-add chains them. Rounds of RP
  // packets: the round's blocks in parallel (packet p on thread p mod T), then the overlap-add in order.
  int T = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  T = std::max(1, std::min(T, 64));
  constexpr size_t RP = 1024;
  std::vector<std::vector<float>> blocks(RP);
  std::vector<int> bn(RP);
  std::vector<Decoder::Scratch> scr(T);
  std::vector<float> prev;
  int prev_n = 0;
  int64_t total = 0;
  for (size_t r0 = 3; r0 < s.packets.size(); r0 += RP) {
    const size_t r1 = std::min(s.packets.size(), r0 + RP), cnt = r1 - r0;
    auto work = [&](int t, int nt) {
      for (size_t p = r0 + t; p < r1; p += nt) bn[p - r0] = d.packet(s.packets[p].data, scr[t], blocks[p - r0]);
    };
    const int nt = (int)std::min<size_t>(T, (cnt + 7) / 8);
    if (nt <= 1) {
      work(0, 1);
    } else {
      std::vector<std::thread> th;
      for (int t = 1; t < nt; t++) th.emplace_back(work, t, nt);
      work(0, nt);
      for (auto& x : th) x.join();
    }
    for (size_t k = 0; k < cnt; k++) {
      const int n = bn[k];
      if (n < 0) {
        tw_set_error("tw_vorbis_decode: bad mode number in packet %zu", r0 + k);
        return 1;
      }
      if (n == 0) continue;
      const std::vector<float>& cur = blocks[k];
      if (prev_n) {  // overlap-add: from the previous block's centre to this block's centre
        // output i = prev[prev_n / 2 + i] (i < prev_n / 2) + cur[i + shift] (i + shift >= 0): prev alone on [0, a),
        // both on [a, b), cur alone on [b, cnt)
        const int shift = n / 4 - prev_n / 4;
        const int cnt = (int)std::min<int64_t>(prev_n / 4 + n / 4, out_frames - total);
        const int a = std::min(cnt, std::max(0, -shift)), b = std::max(a, std::min(cnt, prev_n / 2));
        for (int c = 0; c < C; c++) {
          const float* P = prev.data() + (size_t)c * prev_n + prev_n / 2;
          const float* Q = cur.data() + (size_t)c * n + shift;
          float* o = out + total * C + c;
          for (int i = 0; i < a; i++) o[(size_t)i * C] = P[i];
          for (int i = a; i < b; i++) o[(size_t)i * C] = P[i] + Q[i];
          for (int i = b; i < cnt; i++) o[(size_t)i * C] = Q[i];
        }
        total += std::max(cnt, 0);
      }
      prev.swap(blocks[k]);
      prev_n = n;
    }
  }
  if (end_granule >= 0 && total > end_granule) total = end_granule;  // the last page's granule ends the stream
  *frames_decoded = total;
  return 0;
}

extern "C" int tw_vorbis_imdct(const float* X, int32_t n, float* y) {
  if (!X || !y || n < 4 || (n & (n - 1))) {
    tw_set_error("tw_vorbis_imdct: n=%d (a power of two >= 4)", n);
    return 1;
  }
  Imdct t;
  t.init(n);
  std::vector<float> re, im;
  t.run(X, y, re, im);
  return 0;
}
