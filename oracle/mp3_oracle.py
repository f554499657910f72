"""CPU oracle for MP3 (MPEG-1 / MPEG-2 LSF / MPEG-2.5 Layer III, and Layers I / II) ingest —
TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module; the product (turbo-whisper-workspace_amd/twamd, csrc/mp3.cpp) never does.

The reference decodes .mp3 uploads (vocalis/api/main.py:67-75 keeps the client's suffix; vocalis/security/
security_monitor.py:353 and scripts/normalize_audio.py:226 list .mp3) through ffmpeg_read
($TF/pipelines/audio_utils.py:9-45, ffmpeg's mp3float decoder), which this image does not have, and there is no other
MP3 decoder here. This is a second restatement of ISO/IEC 11172-3 / 13818-3 Layer III in float64, written for clarity
in a different shape from the native decoder: Huffman codewords looked up as bit strings in a dict; scalefactor gains,
intensity / mid-side decisions as whole-spectrum numpy masks; the IMDCT as the standard's cosine sum (a matrix
product); the synthesis filter bank literally as the standard's V / U / W vectors. The standard's tables are read as
text from the product's `csrc/mp3_tables.h` (data, one source of truth): they are pinned by `table_checks()` (complete
prefix codes, band sums, a smooth window) and by the image's one real MP3, not by this module.

* `decode(data)` -> (f32 [frames, channels], sample_rate, info dict) — clean streams (no resynchronisation).
* `write_stream(rng, ...)` — a random *syntax* writer: frames of any version / sample rate / channel mode (mid-side
  and intensity, MPEG-1 and LSF), CRC words, padding, the bit reservoir, long / start / short / stop / mixed blocks,
  every Huffman table with linbits escapes, count1 tables A and B, MPEG-1 scfsi sharing and every LSF scalefactor
  partition (incl. the intensity right channel's), random scalefactors and gains; optionally an ID3v2 tag and a
  Xing / Info + LAME gapless header frame.
* Layers I / II (11172-3 2.4.3.2-3; 13818-3's LSF Layer II table): `decode_frame_l12` reads allocation, scfsi,
  scalefactors and (grouped) sample codes into subband samples with the standard's C (s'' + D) dequantiser;
  `write_stream_l12(rng, layer, ...)` is the matching random-syntax writer. Their tables are restated here in the
  standard's per-subband-range form and compared with the product's arrays (`l12_table_checks`).

Pinning: the only real MP3 in this image is MathJax's a11y/invalid_keypress.mp3 (Lavf56 / libmp3lame, MPEG-1 128 kb/s
44.1 kHz joint stereo, 21 audio frames + an Info frame whose LAME tag holds delay 576, padding 0). Against ffmpeg's own
decoder the decoded samples are UNPINNED (no ffmpeg here); the cross-codec check is that file's Vorbis twin.
"""
from __future__ import annotations

import math
import os
import re
from typing import Dict, List, Optional, Tuple

import numpy as np

_HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "turbo-whisper-workspace_amd", "csrc",
                    "mp3_tables.h")


def _read_tables() -> Dict[str, np.ndarray]:
    txt = open(_HDR).read()
    out = {}
    for m in re.finditer(r"static const (\w+) (\w+)((?:\[\w*\])+) = (\{.*?\});", txt, re.S):
        typ, name, dims, body = m.groups()
        if typ == "HuffSpec":
            continue
        nums = re.findall(r"-?\d+(?:\.\d+)?", body)
        arr = np.array([float(x) for x in nums]) if typ == "double" else np.array([int(x) for x in nums], np.int64)
        shape = [int(d) for d in re.findall(r"\[(\d+)\]", dims)]
        if len(shape) > 1:
            arr = arr.reshape(shape)
        out[name] = arr
    return out


TAB = _read_tables()
# 11172-3 Table B.7: table_select -> (code table, linbits)
_HUFF_SRC = {1: "h1", 2: "h2", 3: "h3", 5: "h5", 6: "h6", 7: "h7", 8: "h8", 9: "h9", 10: "h10", 11: "h11", 12: "h12",
             13: "h13", 15: "h15"}
_LINBITS = {16: 1, 17: 2, 18: 3, 19: 4, 20: 6, 21: 8, 22: 10, 23: 13, 24: 4, 25: 5, 26: 6, 27: 7, 28: 8, 29: 9,
            30: 11, 31: 13}
for _t in range(16, 24):
    _HUFF_SRC[_t] = "h16"
for _t in range(24, 32):
    _HUFF_SRC[_t] = "h24"


def huff_table(t: int):
    """(codes, lengths, dim, linbits) of table_select t, or None for tables 0 / 4 / 14."""
    if t not in _HUFF_SRC:
        return None
    c, ln = TAB[_HUFF_SRC[t] + "c"], TAB[_HUFF_SRC[t] + "l"]
    return c, ln, int(round(math.sqrt(len(c)))), _LINBITS.get(t, 0)


def _bitstrings(codes, lens) -> List[str]:
    return [format(int(c), "0%db" % int(n)) for c, n in zip(codes, lens)]


_DECODE: Dict[str, Dict[str, int]] = {}
for _name in ("h1", "h2", "h3", "h5", "h6", "h7", "h8", "h9", "h10", "h11", "h12", "h13", "h15", "h16", "h24", "hA"):
    _DECODE[_name] = {s: i for i, s in enumerate(_bitstrings(TAB[_name + "c"], TAB[_name + "l"]))}
_QUAD_B = {format(15 - i, "04b"): i for i in range(16)}


def table_checks() -> Dict[str, object]:
    """Structural checks of the standard's tables: every Huffman table a complete prefix code (Kraft sum 1, no
    codeword the prefix of another), the band tables summing to 576 / 192 lines, the window smooth."""
    from fractions import Fraction

    res = {}
    for name in ("h1", "h2", "h3", "h5", "h6", "h7", "h8", "h9", "h10", "h11", "h12", "h13", "h15", "h16", "h24", "hA"):
        strs = _bitstrings(TAB[name + "c"], TAB[name + "l"])
        kraft = sum(Fraction(1, 2 ** len(s)) for s in strs)
        srt = sorted(strs)
        prefix_free = all(not srt[i + 1].startswith(srt[i]) for i in range(len(srt) - 1))
        fits = all(int(c) < 2 ** int(n) for c, n in zip(TAB[name + "c"], TAB[name + "l"]))
        res[name] = (kraft == 1 and prefix_free and fits)
    res["sfb_long"] = bool(all(r[-1] == 576 and np.all(np.diff(r) > 0) for r in TAB["kSfbLong"]))
    res["sfb_short"] = bool(all(r[-1] == 192 and np.all(np.diff(r) > 0) for r in TAB["kSfbShort"]))
    d3 = np.abs(np.diff(TAB["kWin"].astype(np.float64), 3))
    res["window_smooth"] = bool(d3.max() <= 8)
    return res


# ---- Layers I / II, restated in the standard's own form (a second transcription; the product's compact arrays in
# mp3_tables.h are checked against these by l12_table_checks()) --------------------------------------------------------
# bitrate (kbit/s) by bitrate_index, 11172-3 2.4.2.3 / 13818-3 2.4.2.3, keyed (layer, lsf)
L12_BITRATE = {(1, 0): [0, 32, 64, 96, 128, 160, 192, 224, 256, 288, 320, 352, 384, 416, 448],
               (2, 0): [0, 32, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 384],
               (1, 1): [0, 32, 48, 56, 64, 80, 96, 112, 128, 144, 160, 176, 192, 224, 256],
               (2, 1): [0, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 144, 160]}
_FULL = [3, 7, 15, 31, 63, 127, 255, 511, 1023, 2047, 4095, 8191, 16383, 32767, 65535]
_MID = [3, 5, 7, 9, 15, 31, 63, 127, 255, 511, 1023, 2047, 4095, 8191, 65535]
_LOWR = [3, 5, 9, 15, 31, 63, 127, 255, 511, 1023, 2047, 4095, 8191, 16383, 32767]
# Annex B Table B.2a-d and 13818-3 Table B.1: (first subband, last subband, steps of allocation codes 1..2^nbal - 1)
L2_ALLOC = {
    "a": [(0, 2, _FULL), (3, 10, _MID), (11, 22, [3, 5, 7, 9, 15, 31, 65535]), (23, 26, [3, 5, 65535])],
    "b": [(0, 2, _FULL), (3, 10, _MID), (11, 22, [3, 5, 7, 9, 15, 31, 65535]), (23, 29, [3, 5, 65535])],
    "c": [(0, 1, _LOWR), (2, 7, [3, 5, 9, 15, 31, 63, 127])],
    "d": [(0, 1, _LOWR), (2, 11, [3, 5, 9, 15, 31, 63, 127])],
    "lsf": [(0, 3, _LOWR), (4, 10, [3, 5, 9, 15, 31, 63, 127]), (11, 29, [3, 5, 9])],
}


def l2_codeword(steps: int) -> Tuple[int, bool]:
    """(bits per codeword, grouped) of a Layer II quantisation class (Table B.4): 3, 5 and 9 steps code three samples
    in one word of ceil(log2(steps^3)) bits, the others one sample in log2(steps + 1) bits."""
    if steps in (3, 5, 9):
        return int(math.ceil(math.log2(steps ** 3))), True
    return int(round(math.log2(steps + 1))), False


def l2_table_name(h) -> str:
    """Table B.2's choice by sampling rate and bitrate per channel (LSF: Table B.1)."""
    if h["lsf"]:
        return "lsf"
    chb = h["bitrate"] // h["channels"]
    fs = h["sample_rate"]
    if chb >= 96:  # 96..192 kbit/s per channel: a at 48 kHz, b at 44.1 / 32 kHz
        return "a" if fs == 48000 else "b"
    if chb >= 56:  # 56..80
        return "a"
    return "c" if fs != 32000 else "d"  # 32..48


def l2_alloc(name: str):
    """[(nbal, [steps of codes 1..]) per subband] of an allocation table."""
    out = []
    for a, b, steps in L2_ALLOC[name]:
        nbal = int(math.log2(len(steps) + 1))
        out += [(nbal, steps)] * (b - a + 1)
    return out


def l12_table_checks() -> Dict[str, bool]:
    """The product's compact Layer I / II arrays against this module's transcription, plus structure."""
    res = {}
    res["bitrates"] = (TAB["kBitrateL12"][0].tolist() == L12_BITRATE[(1, 0)] and
                       TAB["kBitrateL12"][1].tolist() == L12_BITRATE[(2, 0)] and
                       TAB["kBitrateL12"][2].tolist() == L12_BITRATE[(1, 1)] and
                       TAB["kBitrate"][1].tolist() == L12_BITRATE[(2, 1)])
    steps, bits, grp = TAB["kL2Steps"], TAB["kL2Bits"], TAB["kL2Grouped"]
    res["classes"] = all((int(b), bool(g)) == l2_codeword(int(st)) for st, b, g in zip(steps, bits, grp))
    res["grouped_fit"] = all(int(st) ** 3 <= 2 ** int(b) for st, b, g in zip(steps, bits, grp) if g)
    ok = True
    for t, name in enumerate(("a", "b", "c", "d", "lsf")):
        want = l2_alloc(name)
        ok &= int(TAB["kL2Sblimit"][t]) == len(want)
        for sb in range(30):
            row = int(TAB["kL2SbRow"][t][sb])
            if sb >= len(want):
                ok &= row == -1
                continue
            nbal, st = want[sb]
            got = [int(steps[c]) for c in TAB["kL2Row"][row] if c >= 0]
            ok &= int(TAB["kL2RowBits"][row]) == nbal and got == st and len(got) == 2 ** nbal - 1
            ok &= got == sorted(got)
    res["alloc_tables"] = bool(ok)
    return res


# ---- frame header --------------------------------------------------------------------------------------------------
def parse_header(b: bytes) -> Optional[dict]:
    if len(b) < 4:
        return None
    v = int.from_bytes(b[:4], "big")
    if v >> 21 != 0x7FF:
        return None
    ver, layer, bri, sri = (v >> 19) & 3, (v >> 17) & 3, (v >> 12) & 15, (v >> 10) & 3
    if ver == 1 or layer == 0 or bri in (0, 15) or sri == 3:
        return None
    lsf = int(ver != 3)
    h = dict(layer=4 - layer, lsf=lsf, version={3: 1, 2: 2, 0: 25}[ver], crc=int(not (v >> 16) & 1),
             sr_index={3: 0, 2: 3, 0: 6}[ver] + sri, padding=(v >> 9) & 1, mode=(v >> 6) & 3, mode_ext=(v >> 4) & 3)
    h["sample_rate"] = int(TAB["kSampleRate"][h["sr_index"]])
    h["channels"] = 1 if h["mode"] == 3 else 2
    if h["layer"] != 3:
        h["bitrate"] = L12_BITRATE[(h["layer"], lsf)][bri]
        if h["layer"] == 2:
            h["frame_bytes"] = 144000 * h["bitrate"] // h["sample_rate"] + h["padding"]
        else:
            h["frame_bytes"] = (12000 * h["bitrate"] // h["sample_rate"] + h["padding"]) * 4
        h["side_bytes"], h["granules"], h["spf"] = 0, 0, 1152 if h["layer"] == 2 else 384
        return h
    h["bitrate"] = int(TAB["kBitrate"][lsf][bri])
    h["frame_bytes"] = (72000 if lsf else 144000) * h["bitrate"] // h["sample_rate"] + h["padding"]
    h["side_bytes"] = (9 if h["channels"] == 1 else 17) if lsf else (17 if h["channels"] == 1 else 32)
    h["granules"] = 1 if lsf else 2
    h["spf"] = 576 * h["granules"]
    return h


class Bits:
    def __init__(self, data: bytes):
        self.s = "".join(format(x, "08b") for x in data)
        self.pos = 0

    def get(self, n: int) -> int:
        if n <= 0:
            return 0
        seg = self.s[self.pos: self.pos + n]
        self.pos += n
        return int((seg + "0" * (n - len(seg))) or "0", 2)

    def huff(self, table: Dict[str, int]) -> int:
        for n in range(1, 20):
            seg = self.s[self.pos: self.pos + n]
            if seg in table:
                self.pos += n
                return table[seg]
        raise ValueError("codeword not in table")


def parse_side(b: bytes, h: dict) -> dict:
    br = Bits(b)
    nch, si = h["channels"], {"scfsi": [[0] * 4 for _ in range(2)], "gr": [[None, None], [None, None]]}
    if not h["lsf"]:
        si["main_data_begin"] = br.get(9)
        br.get(5 if nch == 1 else 3)
        for ch in range(nch):
            si["scfsi"][ch] = [br.get(1) for _ in range(4)]
    else:
        si["main_data_begin"] = br.get(8)
        br.get(1 if nch == 1 else 2)
    for gr in range(h["granules"]):
        for ch in range(nch):
            g = dict(part2_3_length=br.get(12), big_values=br.get(9), global_gain=br.get(8),
                     scalefac_compress=br.get(9 if h["lsf"] else 4), window_switching=br.get(1))
            g["bad"] = False
            if g["window_switching"]:
                g["block_type"], g["mixed"] = br.get(2), br.get(1)
                g["table_select"] = [br.get(5), br.get(5), 0]
                g["subblock_gain"] = [br.get(3) for _ in range(3)]
                g["bad"] = g["block_type"] == 0
                g["region0_count"] = 8 if (g["block_type"] == 2 and not g["mixed"]) else 7
                g["region1_count"] = 20 - g["region0_count"]
            else:
                g["block_type"], g["mixed"], g["subblock_gain"] = 0, 0, [0, 0, 0]
                g["table_select"] = [br.get(5) for _ in range(3)]
                g["region0_count"], g["region1_count"] = br.get(4), br.get(3)
            g["preflag"] = 0 if h["lsf"] else br.get(1)
            g["scalefac_scale"], g["count1table_select"] = br.get(1), br.get(1)
            g["bad"] = g["bad"] or g["big_values"] > 288
            si["gr"][gr][ch] = g
    return si


def _short(g) -> bool:
    return bool(g["window_switching"] and g["block_type"] == 2)


def lsf_slen(sfc: int, is_right: bool):
    """13818-3 2.4.3.2: (slen[4], partition table index, preflag, intensity_scale)."""
    if not is_right:
        if sfc < 400:
            return [(sfc >> 4) // 5, (sfc >> 4) % 5, (sfc & 15) >> 2, sfc & 3], 0, 0, 0
        if sfc < 500:
            s = sfc - 400
            return [(s >> 2) // 5, (s >> 2) % 5, s & 3, 0], 1, 0, 0
        s = sfc - 500
        return [s // 3, s % 3, 0, 0], 2, 1, 0
    isc, s = sfc & 1, sfc >> 1
    if s < 180:
        return [s // 36, (s % 36) // 6, (s % 36) % 6, 0], 3, 0, isc
    if s < 244:
        s -= 180
        return [(s & 63) >> 4, (s & 15) >> 2, s & 3, 0], 4, 0, isc
    s -= 244
    return [s // 3, s % 3, 0, 0], 5, 0, isc


def _block_kind(g) -> int:
    return (2 if g["mixed"] else 1) if _short(g) else 0


def read_scalefactors(br: Bits, g, h, si, gr, ch, sf):
    """sf: dict with 'l' [22], 's' [13][3], 'lbad' [22], 'sbad' [13][3], 'isc', 'preflag' (updated in place)."""
    if not h["lsf"]:
        s1, s2 = int(TAB["kSlen"][0][g["scalefac_compress"]]), int(TAB["kSlen"][1][g["scalefac_compress"]])
        sf["preflag"] = g["preflag"]
        if _short(g):
            if g["mixed"]:
                for b in range(8):
                    sf["l"][b] = br.get(s1)
            for b in range(3 if g["mixed"] else 0, 12):
                for w in range(3):
                    sf["s"][b][w] = br.get(s1 if b < 6 else s2)
            sf["s"][12] = [0, 0, 0]
        else:
            for k, (a, e) in enumerate(((0, 6), (6, 11), (11, 16), (16, 21))):
                if gr == 1 and si["scfsi"][ch][k]:
                    continue
                for b in range(a, e):
                    sf["l"][b] = br.get(s1 if k < 2 else s2)
            sf["l"][21] = 0
        return
    is_right = ch == 1 and h["mode"] == 1 and bool(h["mode_ext"] & 1)
    slen, tab, sf["preflag"], sf["isc"] = lsf_slen(g["scalefac_compress"], is_right)
    counts = TAB["kNrOfSfb"][tab][_block_kind(g)]
    vals, bad = [], []
    for i in range(4):
        for _ in range(int(counts[i])):
            vals.append(br.get(slen[i]))
            bad.append((1 << slen[i]) - 1)
    vals += [0] * (40 - len(vals))
    bad += [0] * (40 - len(bad))
    kind = _block_kind(g)
    if kind == 0:
        sf["l"][:21], sf["lbad"][:21] = vals[:21], bad[:21]
        sf["l"][21], sf["lbad"][21] = 0, sf["lbad"][20]
        return
    q, b0 = 0, 0
    if kind == 2:
        sf["l"][:6], sf["lbad"][:6] = vals[:6], bad[:6]
        q, b0 = 6, 3
    for b in range(b0, 12):
        for w in range(3):
            sf["s"][b][w], sf["sbad"][b][w] = vals[q], bad[q]
            q += 1
    sf["s"][12] = [0, 0, 0]
    sf["sbad"][12] = list(sf["sbad"][11])


def huffman(br: Bits, end: int, g, sri: int) -> np.ndarray:
    is_ = np.zeros(576, np.int64)
    big = min(2 * g["big_values"], 576)
    if g["window_switching"]:
        r1 = 3 * int(TAB["kSfbShort"][sri][3]) if (g["block_type"] == 2 and not g["mixed"]) else int(TAB["kSfbLong"][sri][8])
        r2 = 576
    else:
        r1 = int(TAB["kSfbLong"][sri][min(g["region0_count"] + 1, 22)])
        r2 = int(TAB["kSfbLong"][sri][min(g["region0_count"] + g["region1_count"] + 2, 22)])
    r1, r2 = min(r1, big), min(r2, big)
    for i in range(0, big, 2):
        t = g["table_select"][0 if i < r1 else 1 if i < r2 else 2]
        ht = huff_table(t)
        if ht is None:
            continue
        _, _, dim, lb = ht
        v = br.huff(_DECODE[_HUFF_SRC[t]])
        x, y = divmod(v, dim)
        if lb and x == 15:
            x += br.get(lb)
        if x and br.get(1):
            x = -x
        if lb and y == 15:
            y += br.get(lb)
        if y and br.get(1):
            y = -y
        is_[i], is_[i + 1] = x, y
    i = big
    while i + 4 <= 576 and br.pos < end:
        at = br.pos
        v = br.huff(_QUAD_B) if g["count1table_select"] else br.huff(_DECODE["hA"])
        q = [(v >> 3) & 1, (v >> 2) & 1, (v >> 1) & 1, v & 1]
        q = [-1 if (x and br.get(1)) else x for x in q]
        if br.pos > end:
            br.pos = at
            break
        is_[i: i + 4] = q
        i += 4
    return is_


def requantize(g, sf, sri, is_) -> np.ndarray:
    """xr = sign(is) |is|^(4/3) 2^(exponent), the exponent per line from its band (bitstream order)."""
    sfm = 1.0 if g["scalefac_scale"] else 0.5
    expo = np.zeros(576)
    gain = 0.25 * (g["global_gain"] - 210)
    lo = TAB["kSfbLong"][sri]
    so = TAB["kSfbShort"][sri]
    long_end = (3 * int(so[3]) if g["mixed"] else 0) if _short(g) else 576
    for b in range(22):
        a, e = int(lo[b]), min(int(lo[b + 1]), long_end)
        if a >= long_end:
            break
        expo[a:e] = gain - sfm * (sf["l"][b] + (int(TAB["kPretab"][b]) if sf["preflag"] else 0))
    if _short(g):
        for b in range(3 if g["mixed"] else 0, 13):
            w0, W = int(so[b]), int(so[b + 1] - so[b])
            for w in range(3):
                expo[3 * w0 + w * W: 3 * w0 + (w + 1) * W] = gain - 2.0 * g["subblock_gain"][w] - sfm * sf["s"][b][w]
    return np.sign(is_) * np.abs(is_).astype(np.float64) ** (4.0 / 3.0) * np.exp2(expo)


def reorder(g, sri, xr):
    if not _short(g):
        return xr
    xr = xr.copy()
    so = TAB["kSfbShort"][sri]
    for b in range(3 if g["mixed"] else 0, 13):
        w0, W = int(so[b]), int(so[b + 1] - so[b])
        blk = xr[3 * w0: 3 * w0 + 3 * W].reshape(3, W)  # [window][line]
        xr[3 * w0: 3 * w0 + 3 * W] = blk.T.reshape(-1)  # [line][window]
    return xr


def stereo(h, g1, sf1, sri, L, R):
    if h["mode"] != 1 or h["channels"] != 2:
        return L, R
    ms, ist = bool(h["mode_ext"] & 2), bool(h["mode_ext"] & 1)
    if not ist:
        if ms:
            return (L + R) / math.sqrt(2.0), (L - R) / math.sqrt(2.0)
        return L, R
    is_mask = np.zeros(576, bool)
    kl, kr = np.zeros(576), np.zeros(576)
    ms_mask = np.full(576, ms)
    lo, so = TAB["kSfbLong"][sri], TAB["kSfbShort"][sri]

    def gains(pos, bad):
        if not h["lsf"]:
            if pos == 7:
                return None
            if pos > 7:
                return 0.0, 0.0
            t = math.tan(pos * math.pi / 12)
            return t / (1 + t), 1 / (1 + t)
        if pos == bad:
            return None
        io = 1 / math.sqrt(2.0) if sf1["isc"] else 2.0 ** -0.25
        if pos == 0:
            return 1.0, 1.0
        return (io ** ((pos + 1) // 2), 1.0) if pos & 1 else (1.0, io ** (pos // 2))

    def mark(idx, pos, bad):
        gg = gains(pos, bad)
        if gg is not None:
            is_mask[idx] = True
            ms_mask[idx] = False
            kl[idx], kr[idx] = gg

    long_ok = True
    if _short(g1):
        start = 3 if g1["mixed"] else 0
        any_nz = False
        for w in range(3):
            # the short band of window w's highest non-zero right line: bands above it are intensity-coded
            bands = [(b, 3 * int(so[b]) + 3 * np.arange(int(so[b + 1] - so[b])) + w) for b in range(start, 13)]
            nzb = [b for b, idx in bands if np.any(R[idx] != 0)]
            bound = max(nzb) if nzb else start - 1
            any_nz |= bool(nzb)
            for b, idx in bands:
                if b > bound:
                    bb = 11 if b == 12 else b
                    mark(idx, sf1["s"][bb][w], sf1["sbad"][bb][w] if h["lsf"] else 7)
        if not g1["mixed"]:
            long_top = 0
        else:
            long_top = int(np.searchsorted(lo, 3 * int(so[3])))
        long_ok = not any_nz
    else:
        long_top = 22
    if long_top:
        end = int(lo[long_top]) if long_top < 22 else 576
        nz = np.nonzero(R[:end])[0]
        hb = int(np.searchsorted(lo, nz.max(), side="right")) - 1 if (len(nz) and long_ok) else (-1 if long_ok else 99)
        for b in range(long_top):
            if b > hb:
                bb = 20 if b == 21 else b
                mark(np.arange(int(lo[b]), min(int(lo[b + 1]), end)), sf1["l"][bb], sf1["lbad"][bb] if h["lsf"] else 7)
    r2 = 1 / math.sqrt(2.0)
    Ln = np.where(is_mask, L * kl, np.where(ms_mask, (L + R) * r2, L))
    Rn = np.where(is_mask, L * kr, np.where(ms_mask, (L - R) * r2, R))
    return Ln, Rn


_CA = TAB["kAliasC"]
_CS_A = 1 / np.sqrt(1 + _CA ** 2)
_CA_A = _CA / np.sqrt(1 + _CA ** 2)


def antialias(g, xr):
    xr = xr.copy()
    if _short(g) and not g["mixed"]:
        return xr
    n = 1 if _short(g) else 31
    for sb in range(n):
        for i in range(8):
            a, b = xr[18 * sb + 17 - i], xr[18 * sb + 18 + i]
            xr[18 * sb + 17 - i] = a * _CS_A[i] - b * _CA_A[i]
            xr[18 * sb + 18 + i] = b * _CS_A[i] + a * _CA_A[i]
    return xr


def _windows():
    i = np.arange(36)
    s36 = np.sin(np.pi / 36 * (i + 0.5))
    w = np.zeros((4, 36))
    w[0] = s36
    w[1] = np.where(i < 18, s36, np.where(i < 24, 1.0, np.where(i < 30, np.sin(np.pi / 12 * (i - 18 + 0.5)), 0.0)))
    w[3] = np.where(i < 6, 0.0, np.where(i < 12, np.sin(np.pi / 12 * (i - 6 + 0.5)), np.where(i < 18, 1.0, s36)))
    return w


_WIN = _windows()
_C36 = np.cos(np.pi / 72 * np.outer(2 * np.arange(36) + 19, 2 * np.arange(18) + 1))  # [i][k]
_C12 = np.cos(np.pi / 24 * np.outer(2 * np.arange(12) + 7, 2 * np.arange(6) + 1))
_W12 = np.sin(np.pi / 12 * (np.arange(12) + 0.5))


def imdct(g, xr, overlap):
    """-> (subband samples [18][32], new overlap [32][18])."""
    out = np.zeros((18, 32))
    new = np.zeros((32, 18))
    long_end = (2 if g["mixed"] else 0) if _short(g) else 32
    for sb in range(32):
        X = xr[18 * sb: 18 * sb + 18]
        if sb < long_end:
            bt = 0 if _short(g) else g["block_type"]
            z = (_C36 @ X) * _WIN[bt]
        else:
            z = np.zeros(36)
            for w in range(3):
                z[6 + 6 * w: 18 + 6 * w] += (_C12 @ X[w::3]) * _W12
        y = z[:18] + overlap[sb]
        if sb & 1:
            y[1::2] = -y[1::2]
        out[:, sb] = y
        new[sb] = z[18:]
    return out, new


_N = np.cos(np.outer(16 + np.arange(64), 2 * np.arange(32) + 1) * np.pi / 64)  # [i][k]


def synthesis_window() -> np.ndarray:
    i = np.arange(512)
    h = TAB["kWin"][np.where(i <= 256, i, 512 - i)].astype(np.float64)
    return h * np.where((i // 64) % 2, -1.0, 1.0) / 65536.0


_D = synthesis_window()


def synthesize(S, V):
    """11172-3 Annex A synthesis: S [slots][32] -> pcm [slots * 32]; V (1024) updated in place."""
    pcm = []
    for s in range(S.shape[0]):
        V[64:] = V[:-64].copy()
        V[:64] = _N @ S[s]
        U = np.zeros(512)
        for i in range(8):
            U[64 * i: 64 * i + 32] = V[128 * i: 128 * i + 32]
            U[64 * i + 32: 64 * i + 64] = V[128 * i + 96: 128 * i + 128]
        W = U * _D
        pcm.append(W.reshape(16, 32).sum(0))
    return np.concatenate(pcm)


def scan(data: bytes):
    """(first header, [(pos, header) of audio frames], tag info dict) for a clean stream."""
    pos = 0
    while data[pos: pos + 3] == b"ID3" and pos + 10 <= len(data):
        sz = (data[pos + 6] & 127) << 21 | (data[pos + 7] & 127) << 14 | (data[pos + 8] & 127) << 7 | (data[pos + 9] & 127)
        pos += 10 + sz + (10 if data[pos + 5] & 0x10 else 0)
    while pos + 4 <= len(data) and parse_header(data[pos: pos + 4]) is None:
        pos += 1
    frames = []
    while pos + 4 <= len(data):
        h = parse_header(data[pos: pos + 4])
        if h is None or pos + h["frame_bytes"] > len(data):
            break
        frames.append((pos, h))
        pos += h["frame_bytes"]
    if not frames:
        raise ValueError("no frame")
    info = {"flags": 0, "enc_delay": -1, "enc_padding": -1, "tag_frames": -1}
    p0, h0 = frames[0]
    xo = p0 + 4 + h0["side_bytes"]
    if h0["layer"] != 3:
        return h0, frames, info
    if data[xo: xo + 4] in (b"Xing", b"Info"):
        info["flags"] |= 1
        fl = int.from_bytes(data[xo + 4: xo + 8], "big")
        q = xo + 8
        if fl & 1:
            info["tag_frames"] = int.from_bytes(data[q: q + 4], "big")
        q += 4 * bool(fl & 1) + 4 * bool(fl & 2) + 100 * bool(fl & 4) + 4 * bool(fl & 8)
        if data[q: q + 4] in (b"LAME", b"Lavf", b"Lavc"):
            g = data[q + 21: q + 24]
            info["enc_delay"] = g[0] << 4 | g[1] >> 4
            info["enc_padding"] = (g[1] & 15) << 8 | g[2]
            info["flags"] |= 2
    elif data[p0 + 36: p0 + 40] == b"VBRI":
        info["flags"] |= 4
    if info["flags"] & 5:
        frames = frames[1:]
    return h0, frames, info


def _dequant(v: int, steps: int) -> float:
    """11172-3 2.4.3.2.1 / 2.4.3.3.4: s''' = C (s'' + D), s'' the code as a two's-complement fraction with its MSB
    inverted; for L = steps levels that is (2 v + 1 - L) / L."""
    nb = int(math.ceil(math.log2(steps + 1)))
    frac = v / 2 ** (nb - 1) - 1.0
    c = 2 ** nb / steps if steps == 2 ** nb - 1 else {3: 4 / 3, 5: 8 / 5, 9: 16 / 9}[steps]
    d = 2.0 ** (1 - nb) if steps == 2 ** nb - 1 else 0.5
    return c * (frac + d)


def _scalefactor(i: int) -> float:
    return 2.0 ** (1 - i / 3)  # Table B.1: 2.0, 1.5874..., 1.2599..., ...


def decode_frame_l12(fr: bytes, h) -> np.ndarray:
    """One Layer I / II frame -> subband samples [channels][slots][32] (float64)."""
    nch, layer = h["channels"], h["layer"]
    br = Bits(fr)
    br.pos = 32 + 16 * h["crc"]
    bound = 4 * (h["mode_ext"] + 1) if h["mode"] == 1 else 32
    S = np.zeros((nch, 12 if layer == 1 else 36, 32))
    if layer == 1:
        alloc = [[0] * 32 for _ in range(2)]
        for sb in range(32):
            for ch in (range(nch) if sb < bound else [0]):
                alloc[ch][sb] = br.get(4)
            if sb >= bound:
                alloc[1][sb] = alloc[0][sb]
        if any(alloc[ch][sb] == 15 for ch in range(nch) for sb in range(32)):
            return S * 0
        scf = [[br.get(6) if alloc[ch][sb] else 0 for ch in range(nch)] for sb in range(32)]
        for s in range(12):
            for sb in range(32):
                if sb < bound:
                    for ch in range(nch):
                        n = alloc[ch][sb]
                        if n:
                            S[ch, s, sb] = _dequant(br.get(n + 1), 2 ** (n + 1) - 1) * _scalefactor(scf[sb][ch])
                elif alloc[0][sb]:
                    n = alloc[0][sb]
                    q = _dequant(br.get(n + 1), 2 ** (n + 1) - 1)
                    for ch in range(nch):
                        S[ch, s, sb] = q * _scalefactor(scf[sb][ch])
        return S
    table = l2_alloc(l2_table_name(h))
    sblimit = len(table)
    bound = min(bound, sblimit)
    steps = [[0] * 32 for _ in range(2)]  # 0: no allocation
    for sb in range(sblimit):
        nbal, st = table[sb]
        codes = [br.get(nbal) for _ in range(nch)] if sb < bound else [br.get(nbal)] * 2
        for ch in range(2 if sb >= bound else nch):
            steps[ch][sb] = st[codes[ch] - 1] if codes[ch] else 0
    scfsi = {(ch, sb): br.get(2) for sb in range(sblimit) for ch in range(nch) if steps[ch][sb]}
    scf = {}
    for sb in range(sblimit):
        for ch in range(nch):
            if not steps[ch][sb]:
                continue
            sel = scfsi[(ch, sb)]
            if sel == 0:
                scf[(ch, sb)] = [br.get(6), br.get(6), br.get(6)]
            elif sel == 1:
                a = br.get(6)
                scf[(ch, sb)] = [a, a, br.get(6)]
            elif sel == 2:
                a = br.get(6)
                scf[(ch, sb)] = [a, a, a]
            else:
                a, b = br.get(6), br.get(6)
                scf[(ch, sb)] = [a, b, b]

    def triple(L):
        nb, grouped = l2_codeword(L)
        if not grouped:
            return [_dequant(br.get(nb), L) for _ in range(3)]
        c = br.get(nb)
        return [_dequant(c % L, L), _dequant((c // L) % L, L), _dequant(c // L // L, L)]

    for gr in range(12):
        for sb in range(sblimit):
            if sb < bound:
                for ch in range(nch):
                    if steps[ch][sb]:
                        S[ch, 3 * gr: 3 * gr + 3, sb] = np.array(triple(steps[ch][sb])) * _scalefactor(
                            scf[(ch, sb)][gr // 4])
            elif steps[0][sb]:
                q = np.array(triple(steps[0][sb]))
                for ch in range(nch):
                    S[ch, 3 * gr: 3 * gr + 3, sb] = q * _scalefactor(scf[(ch, sb)][gr // 4])
    return S


def decode(data: bytes, stats: Optional[dict] = None):
    """MP3 bytes -> (f32 [frames, channels], sample_rate, info). stats (optional) collects per-granule bit accounting
    ('exact': Huffman data ended exactly at part2_3_length) and the Huffman tables used."""
    h0, frames, info = scan(data)
    nch, spf = h0["channels"], h0["spf"]
    if h0["layer"] != 3:  # Layers I / II: self-contained frames into the synthesis bank, no trim
        V = [np.zeros(1024) for _ in range(nch)]
        pcm = np.zeros((len(frames) * spf, nch))
        for k, (p, h) in enumerate(frames):
            S = decode_frame_l12(data[p: p + h["frame_bytes"]], h)
            if stats is not None:
                stats.setdefault("l2_tables", set()).add(l2_table_name(h) if h["layer"] == 2 else "I")
            for ch in range(nch):
                pcm[k * spf: (k + 1) * spf, ch] = synthesize(S[ch], V[ch])
        info.update(skip=0, total=len(pcm), n_frames=len(frames), sample_rate=h0["sample_rate"], channels=nch)
        return pcm.astype(np.float32), h0["sample_rate"], info
    md, off = bytearray(), []
    for p, h in frames:
        off.append(len(md))
        md += data[p + 4 + 2 * h["crc"] + h["side_bytes"]: p + h["frame_bytes"]]
    br = Bits(bytes(md))
    overlap = [np.zeros((32, 18)) for _ in range(nch)]
    V = [np.zeros(1024) for _ in range(nch)]
    pcm = np.zeros((len(frames) * spf, nch))
    for k, (p, h) in enumerate(frames):
        si = parse_side(data[p + 4 + 2 * h["crc"]: p + 4 + 2 * h["crc"] + h["side_bytes"]], h)
        start = off[k] - si["main_data_begin"]
        br.pos = max(start, 0) * 8
        sfs = [dict(l=[0] * 22, s=[[0] * 3 for _ in range(13)], lbad=[0] * 22, sbad=[[0] * 3 for _ in range(13)],
                    isc=0, preflag=0) for _ in range(2)]
        for gr in range(h["granules"]):
            xr = [np.zeros(576), np.zeros(576)]
            for ch in range(nch):
                g = si["gr"][gr][ch]
                end = br.pos + g["part2_3_length"]
                read_scalefactors(br, g, h, si, gr, ch, sfs[ch])
                if start >= 0 and not g["bad"] and br.pos <= end:
                    is_ = huffman(br, end, g, h["sr_index"])
                    if stats is not None:
                        stats.setdefault("exact", []).append(br.pos == end)
                        for t in g["table_select"][: (2 if g["window_switching"] else 3)]:
                            stats.setdefault("tables", set()).add(int(t))
                        stats.setdefault("count1", set()).add(g["count1table_select"])
                        stats.setdefault("blocks", set()).add((g["block_type"], g["mixed"]))
                    xr[ch] = reorder(g, h["sr_index"], requantize(g, sfs[ch], h["sr_index"], is_))
                br.pos = end
            if nch == 2:
                xr[0], xr[1] = stereo(h, si["gr"][gr][1], sfs[1], h["sr_index"], xr[0], xr[1])
            for ch in range(nch):
                g = si["gr"][gr][ch]
                S, overlap[ch] = imdct(g, antialias(g, xr[ch]), overlap[ch])
                base = k * spf + gr * 576
                pcm[base: base + 576, ch] = synthesize(S, V[ch])
    skip, total = 0, len(pcm)
    if info["flags"] & 2:
        nfr = info["tag_frames"] if info["tag_frames"] >= 0 else len(frames)
        skip = info["enc_delay"] + 529
        total = max(0, min(len(pcm), nfr * spf - info["enc_padding"] + 529) - skip)
    info.update(skip=skip, total=total, n_frames=len(frames), sample_rate=h0["sample_rate"], channels=nch)
    return pcm[skip: skip + total].astype(np.float32), h0["sample_rate"], info


# ---- random-syntax writer --------------------------------------------------------------------------------------------
class BitWriter:
    def __init__(self):
        self.parts: List[str] = []
        self.n = 0

    def put(self, v: int, n: int):
        if n:
            self.parts.append(format(int(v), "0%db" % n))
            self.n += n

    def bits(self) -> str:
        return "".join(self.parts)


def _bytes(bits: str) -> bytes:
    bits += "0" * (-len(bits) % 8)
    return bytes(int(bits[i: i + 8], 2) for i in range(0, len(bits), 8))


_TABLES_OK = [0, 1, 2, 3, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15] + list(range(16, 32))


def _rand_granule(rng, h, ch, gr, si, max_big):
    lsf, sri = h["lsf"], h["sr_index"]
    g = {"window_switching": int(rng.random() < 0.45)}
    if g["window_switching"]:
        g["block_type"] = int(rng.choice([1, 2, 2, 3]))
        g["mixed"] = int(g["block_type"] == 2 and rng.random() < 0.4)
        g["table_select"] = [int(rng.choice(_TABLES_OK)) for _ in range(2)] + [0]
        g["subblock_gain"] = [int(x) for x in rng.integers(0, 8, 3)]
        g["region0_count"] = 8 if (g["block_type"] == 2 and not g["mixed"]) else 7
        g["region1_count"] = 20 - g["region0_count"]
    else:
        g["block_type"], g["mixed"], g["subblock_gain"] = 0, 0, [0, 0, 0]
        g["table_select"] = [int(rng.choice(_TABLES_OK)) for _ in range(3)]
        g["region0_count"], g["region1_count"] = int(rng.integers(0, 16)), int(rng.integers(0, 8))
    g["global_gain"] = int(rng.integers(150, 215))
    g["scalefac_compress"] = int(rng.integers(0, 512 if lsf else 16))
    g["preflag"] = 0 if lsf else int(rng.integers(0, 2))
    g["scalefac_scale"], g["count1table_select"] = int(rng.integers(0, 2)), int(rng.integers(0, 2))
    g["big_values"] = int(rng.integers(0, max_big + 1))
    # scalefactor values (written below in the order the decoder reads them)
    w = BitWriter()
    if not lsf:
        s1, s2 = int(TAB["kSlen"][0][g["scalefac_compress"]]), int(TAB["kSlen"][1][g["scalefac_compress"]])
        if _short(g):
            if g["mixed"]:
                for _ in range(8):
                    w.put(rng.integers(0, 1 << s1), s1)
            for b in range(3 if g["mixed"] else 0, 12):
                s = s1 if b < 6 else s2
                for _ in range(3):
                    w.put(rng.integers(0, 1 << s), s)
        else:
            for k, (a, e) in enumerate(((0, 6), (6, 11), (11, 16), (16, 21))):
                if gr == 1 and si["scfsi"][ch][k]:
                    continue
                s = s1 if k < 2 else s2
                for _ in range(a, e):
                    w.put(rng.integers(0, 1 << s), s)
    else:
        is_right = ch == 1 and h["mode"] == 1 and bool(h["mode_ext"] & 1)
        slen, tab, _, _ = lsf_slen(g["scalefac_compress"], is_right)
        for i in range(4):
            for _ in range(int(TAB["kNrOfSfb"][tab][_block_kind(g)][i])):
                w.put(rng.integers(0, 1 << slen[i]), slen[i])
    # Huffman data
    big = 2 * g["big_values"]
    if g["window_switching"]:
        r1 = 3 * int(TAB["kSfbShort"][sri][3]) if (g["block_type"] == 2 and not g["mixed"]) else int(TAB["kSfbLong"][sri][8])
        r2 = 576
    else:
        r1 = int(TAB["kSfbLong"][sri][min(g["region0_count"] + 1, 22)])
        r2 = int(TAB["kSfbLong"][sri][min(g["region0_count"] + g["region1_count"] + 2, 22)])
    r1, r2 = min(r1, big), min(r2, big)
    for i in range(0, big, 2):
        t = g["table_select"][0 if i < r1 else 1 if i < r2 else 2]
        ht = huff_table(t)
        if ht is None:
            continue
        codes, lens, dim, lb = ht
        x, y = int(rng.integers(0, dim)), int(rng.integers(0, dim))
        if rng.random() < 0.6:  # mostly small values, as real spectra
            x, y = min(x, int(rng.integers(0, 3))), min(y, int(rng.integers(0, 3)))
        w.put(codes[x * dim + y], int(lens[x * dim + y]))
        for v in (x, y):
            if lb and v == 15:
                w.put(rng.integers(0, min(1 << lb, 64)), lb)
            if v:
                w.put(rng.integers(0, 2), 1)
    nq = int(rng.integers(0, min((576 - big) // 4, 30) + 1))
    for _ in range(nq):
        v = int(rng.integers(0, 16))
        if g["count1table_select"]:
            w.put(15 - v, 4)
        else:
            w.put(TAB["hAc"][v], int(TAB["hAl"][v]))
        for j in range(4):
            if (v >> (3 - j)) & 1:
                w.put(rng.integers(0, 2), 1)
    g["part2_3_length"] = w.n
    return g, w


def _write_side(h, si) -> bytes:
    w = BitWriter()
    nch = h["channels"]
    if not h["lsf"]:
        w.put(si["main_data_begin"], 9)
        w.put(0, 5 if nch == 1 else 3)
        for ch in range(nch):
            for b in range(4):
                w.put(si["scfsi"][ch][b], 1)
    else:
        w.put(si["main_data_begin"], 8)
        w.put(0, 1 if nch == 1 else 2)
    for gr in range(h["granules"]):
        for ch in range(nch):
            g = si["gr"][gr][ch]
            w.put(g["part2_3_length"], 12)
            w.put(g["big_values"], 9)
            w.put(g["global_gain"], 8)
            w.put(g["scalefac_compress"], 9 if h["lsf"] else 4)
            w.put(g["window_switching"], 1)
            if g["window_switching"]:
                w.put(g["block_type"], 2)
                w.put(g["mixed"], 1)
                w.put(g["table_select"][0], 5)
                w.put(g["table_select"][1], 5)
                for x in g["subblock_gain"]:
                    w.put(x, 3)
            else:
                for x in g["table_select"]:
                    w.put(x, 5)
                w.put(g["region0_count"], 4)
                w.put(g["region1_count"], 3)
            if not h["lsf"]:
                w.put(g["preflag"], 1)
            w.put(g["scalefac_scale"], 1)
            w.put(g["count1table_select"], 1)
    b = _bytes(w.bits())
    assert len(b) == h["side_bytes"], (len(b), h["side_bytes"])
    return b


_VER_BITS = {1: 3, 2: 2, 25: 0}


def _header_bytes(version, sr_sub, bri, crc, pad, mode, mode_ext) -> bytes:
    v = (0x7FF << 21) | (_VER_BITS[version] << 19) | (1 << 17) | ((0 if crc else 1) << 16) | (bri << 12)
    v |= (sr_sub << 10) | (pad << 9) | (mode << 6) | (mode_ext << 4)
    return v.to_bytes(4, "big")


def write_stream(rng, version: int = 1, sr_sub: Optional[int] = None, mode: Optional[int] = None, nframes: int = 6,
                 crc: Optional[bool] = None, xing: bool = False, enc_delay: int = 576, enc_padding: int = 1200,
                 id3: bool = False, max_big: int = 120, junk: bool = False) -> bytes:
    """A random-syntax Layer III stream (see the module docstring). With xing=True an Info frame with a LAME tag
    (delay / padding as given) precedes the audio frames. junk=True puts random non-sync bytes between some frames
    (decoders resynchronise; the clean scan of this module does not — use it only for the native decoder)."""
    lsf = version != 1
    sr_sub = int(rng.integers(0, 3)) if sr_sub is None else sr_sub
    bri = int(rng.integers(9, 15)) if not lsf else int(rng.integers(11, 15))
    mode = int(rng.integers(0, 4)) if mode is None else mode
    out = bytearray()
    if id3:
        body = bytes(rng.integers(0, 128, 40, dtype=np.uint8))
        out += b"ID3\x04\x00\x00" + bytes([0, 0, 0, len(body)]) + body
    md_stream = bytearray()
    used = 0
    frames = []
    for k in range(nframes):
        pad = int(rng.integers(0, 2))
        use_crc = bool(rng.integers(0, 2)) if crc is None else crc
        mode_ext = int(rng.integers(0, 4)) if mode == 1 else 0
        hdr = _header_bytes(version, sr_sub, bri, use_crc, pad, mode, mode_ext)
        h = parse_header(hdr)
        cap = h["frame_bytes"] - 4 - 2 * use_crc - h["side_bytes"]
        off = len(md_stream)
        limit = 255 if lsf else 511
        for attempt in range(12):
            si = {"scfsi": [[int(x) for x in rng.integers(0, 2, 4)] for _ in range(2)],
                  "gr": [[None, None], [None, None]]}
            writers = []
            mb = max(0, max_big >> attempt)
            for gr in range(h["granules"]):
                for ch in range(h["channels"]):
                    g, w = _rand_granule(rng, h, ch, gr, si, mb)
                    si["gr"][gr][ch] = g
                    writers.append(w)
            data_bits = "".join(w.bits() for w in writers)
            nbytes = (len(data_bits) + 7) // 8
            free = off - used
            mdb = min(free, limit)
            if nbytes <= mdb + cap and all(g["part2_3_length"] < 4096 for r in si["gr"] for g in r if g):
                break
        else:
            raise RuntimeError("writer: granule data does not fit")
        # place the data as early as the reservoir allows (random amount of reservoir use)
        mdb = int(rng.integers(max(0, nbytes - cap), mdb + 1))
        si["main_data_begin"] = mdb
        side = _write_side(h, si)
        slot = bytearray(rng.integers(0, 256, cap, dtype=np.uint8).tobytes())  # ancillary / stuffing bytes
        md_stream += slot
        start = off - mdb
        payload = _bytes(data_bits)
        md_stream[start: start + len(payload)] = payload
        used = start + len(payload)
        frames.append((hdr, use_crc, side, off, cap))
    if xing:
        h = parse_header(frames[0][0])
        hdr = _header_bytes(version, sr_sub, bri, False, 0, mode, frames[0][0][3] >> 4 & 3)
        h = parse_header(hdr)
        fr = bytearray(h["frame_bytes"])
        fr[:4] = hdr
        q = 4 + h["side_bytes"]
        fr[q: q + 4] = b"Info"
        fr[q + 4: q + 8] = (0x0F).to_bytes(4, "big")
        fr[q + 8: q + 12] = nframes.to_bytes(4, "big")
        fr[q + 12: q + 16] = (0).to_bytes(4, "big")
        q += 8 + 4 + 4 + 100 + 4
        fr[q: q + 9] = b"LAME3.100"
        fr[q + 21: q + 24] = ((enc_delay << 12) | enc_padding).to_bytes(3, "big")
        out += fr
    for k, (hdr, use_crc, side, off, cap) in enumerate(frames):
        if junk and k and rng.random() < 0.5:
            out += bytes(rng.integers(0, 0x7F, int(rng.integers(1, 20)), dtype=np.uint8))
        out += hdr
        if use_crc:
            out += bytes(rng.integers(0, 256, 2, dtype=np.uint8))
        out += side + md_stream[off: off + cap]
    return bytes(out)


def _header_bytes_l12(layer, version, sr_sub, bri, crc, pad, mode, mode_ext) -> bytes:
    v = (0x7FF << 21) | (_VER_BITS[version] << 19) | ((4 - layer) << 17) | ((0 if crc else 1) << 16) | (bri << 12)
    v |= (sr_sub << 10) | (pad << 9) | (mode << 6) | (mode_ext << 4)
    return v.to_bytes(4, "big")


def write_stream_l12(rng, layer: int = 2, version: int = 1, sr_sub: Optional[int] = None, mode: Optional[int] = None,
                     bri: Optional[int] = None, nframes: int = 6, crc: Optional[bool] = None, id3: bool = False,
                     fill: float = 0.7, bad_groups: bool = True) -> bytes:
    """A random-syntax Layer I or II stream: random bit allocations (every code of every row, dropped at random until
    the frame's bits fit; `fill` the share of subbands allocated), scfsi patterns, scalefactors and sample codes —
    grouped codewords past steps^3 included when bad_groups — with joint-stereo bounds, CRC words and padding;
    ancillary bytes fill each frame."""
    sr_sub = int(rng.integers(0, 3)) if sr_sub is None else sr_sub
    mode = int(rng.integers(0, 4)) if mode is None else mode
    if bri is None:
        bri = int(rng.integers(6, 15))
    out = bytearray()
    if id3:
        body = bytes(rng.integers(0, 128, 30, dtype=np.uint8))
        out += b"ID3\x03\x00\x00" + bytes([0, 0, 0, len(body)]) + body
    for _ in range(nframes):
        pad = int(rng.integers(0, 2))
        use_crc = bool(rng.integers(0, 2)) if crc is None else crc
        mode_ext = int(rng.integers(0, 4)) if mode == 1 else 0
        hdr = _header_bytes_l12(layer, version, sr_sub, bri, use_crc, pad, mode, mode_ext)
        h = parse_header(hdr)
        nch = h["channels"]
        bound = 4 * (mode_ext + 1) if mode == 1 else 32
        cap = 8 * h["frame_bytes"] - 32 - 16 * use_crc
        if layer == 1:
            rows = [(4, None)] * 32
        else:
            rows = l2_alloc(l2_table_name(h))
        sblimit = len(rows)
        bound = min(bound, sblimit)
        # allocation codes [ch][sb]
        codes = [[0] * 32 for _ in range(2)]
        for sb in range(sblimit):
            nbal = rows[sb][0]
            top = 14 if layer == 1 else 2 ** nbal - 1
            for ch in range(nch if sb < bound else 1):
                if rng.random() < fill:
                    codes[ch][sb] = int(rng.integers(1, top + 1))
            if sb >= bound:
                codes[1][sb] = codes[0][sb]
        scfsi = [[int(x) for x in rng.integers(0, 4, 32)] for _ in range(2)]

        def cost():
            n = sum(rows[sb][0] * (nch if sb < bound else 1) for sb in range(sblimit))
            for sb in range(sblimit):
                for ch in range(nch):
                    if codes[ch][sb]:
                        if layer == 1:
                            n += 6
                        else:
                            n += 2 + 6 * {0: 3, 1: 2, 2: 1, 3: 2}[scfsi[ch][sb]]
            for sb in range(sblimit):
                chans = range(nch) if sb < bound else [0]
                for ch in chans:
                    c = codes[ch][sb]
                    if not c:
                        continue
                    if layer == 1:
                        n += 12 * (c + 1)
                    else:
                        nb, grouped = l2_codeword(rows[sb][1][c - 1])
                        n += 12 * (nb if grouped else 3 * nb)
            return n

        while cost() > cap:
            live = [(ch, sb) for sb in range(sblimit) for ch in range(2) if codes[ch][sb]]
            ch, sb = live[int(rng.integers(0, len(live)))]
            if sb >= bound:
                codes[0][sb] = codes[1][sb] = 0
            else:
                codes[ch][sb] = 0
        w = BitWriter()
        for sb in range(sblimit):
            for ch in range(nch if sb < bound else 1):
                w.put(codes[ch][sb], rows[sb][0])
        if layer == 1:
            for sb in range(32):
                for ch in range(nch):
                    if codes[ch][sb]:
                        w.put(rng.integers(0, 63), 6)
            for _s in range(12):
                for sb in range(32):
                    for ch in (range(nch) if sb < bound else [0]):
                        c = codes[ch][sb]
                        if c:
                            w.put(rng.integers(0, 2 ** (c + 1) - 1), c + 1)  # (all-ones is forbidden)
        else:
            for sb in range(sblimit):
                for ch in range(nch):
                    if codes[ch][sb]:
                        w.put(scfsi[ch][sb], 2)
            for sb in range(sblimit):
                for ch in range(nch):
                    if codes[ch][sb]:
                        for _k in range({0: 3, 1: 2, 2: 1, 3: 2}[scfsi[ch][sb]]):
                            w.put(rng.integers(0, 63), 6)
            for _gr in range(12):
                for sb in range(sblimit):
                    for ch in (range(nch) if sb < bound else [0]):
                        c = codes[ch][sb]
                        if not c:
                            continue
                        L = rows[sb][1][c - 1]
                        nb, grouped = l2_codeword(L)
                        if grouped:
                            top = 2 ** nb if (bad_groups and rng.random() < 0.05) else L ** 3
                            w.put(rng.integers(0, top), nb)
                        else:
                            for _k in range(3):
                                w.put(rng.integers(0, L), nb)
        assert w.n <= cap, (w.n, cap)
        body = bytearray(_bytes(w.bits()))
        nbody = h["frame_bytes"] - 4 - 2 * use_crc
        body += bytes(rng.integers(0, 256, nbody - len(body), dtype=np.uint8))  # ancillary data
        out += hdr
        if use_crc:
            out += bytes(rng.integers(0, 256, 2, dtype=np.uint8))
        out += body
    return bytes(out)
