"""CPU oracle for AAC-LC ingest (ADTS and MP4 / M4A) — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module; the product (turbo-whisper-workspace_amd/twamd, csrc/aac.cpp) never does.

The reference decodes .m4a uploads (vocalis/security/security_monitor.py:353 lists the suffix; vocalis/api/main.py:67-75
stores any upload under its own suffix) through ffmpeg_read ($TF/pipelines/audio_utils.py:9-45, ffmpeg's aac decoder
and mov demuxer), which this image does not have, and there is no other AAC decoder here. This is a second
restatement of ISO/IEC 14496-3 AAC-LC in float64, in a different shape from the native decoder: Huffman codewords
looked up as bit strings in dicts; the IMDCT as the standard's cosine sum (a matrix product, with its 2/N factor);
the windows built whole; TNS as the standard's tns_ar_filter with its state vector. The standard's tables are read as
text from the product's `csrc/aac_tables.h` (one source of truth), pinned by `table_checks()` and by the image's one
real AAC-LC stream, not by this module. PNS noise follows the native decoder's own documented generator (ffmpeg's
noise is another random sequence: PNS bands are unpinned by construction).

* `decode_raw(asc, units)` / `decode_adts(data)` -> (f32 [frames, channels], sample_rate, stats).
* `write_adts(rng, ...)` / `write_mp4(rng, ...)` — a random *syntax* writer: SCE / CPE (common and separate windows,
  mid-side masks of both kinds), all four window sequences with both shapes and random grouping, every spectral
  codebook incl. escapes, intensity and noise bands, pulse data, TNS filters of every resolution / direction /
  compression; DSE, FIL and PCE elements to skip. write_mp4 wraps the units in a minimal MP4 (ftyp, moov with one
  sound track: stsd mp4a + esds, stts, stsc, stsz, stco, an optional edit list, mdat).

Pinning: the only real AAC in this image is imageio's realshort.mp4 (48 kHz mono AAC-LC, 55 access units): every unit
must parse to its END element with only byte-alignment padding left. Against ffmpeg's decoder the samples are UNPINNED.
"""
from __future__ import annotations

import math
import os
import re
import struct
from typing import Dict, List, Optional, Tuple

import numpy as np

_HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "turbo-whisper-workspace_amd", "csrc",
                    "aac_tables.h")


def _read_tables() -> Dict[str, np.ndarray]:
    txt = open(_HDR).read()
    out = {}
    for m in re.finditer(r"static const (\w+) (\w+)\[(\d*)\] = (\{.*?\});", txt, re.S):
        typ, name, _, body = m.groups()
        if typ in ("Codebook", "SwbTables"):
            continue
        nums = re.findall(r"0x[0-9a-fA-F]+|-?\d+", body)
        out[name] = np.array([int(x, 0) for x in nums], np.int64)
    return out


TAB = _read_tables()
# 14496-3 4.A.1: (dim, lav, signed, mod, off) per spectral codebook
CB = {1: (4, 1, 1, 3, 1), 2: (4, 1, 1, 3, 1), 3: (4, 2, 0, 3, 0), 4: (4, 2, 0, 3, 0), 5: (2, 4, 1, 9, 4),
      6: (2, 4, 1, 9, 4), 7: (2, 7, 0, 8, 0), 8: (2, 7, 0, 8, 0), 9: (2, 12, 0, 13, 0), 10: (2, 12, 0, 13, 0),
      11: (2, 16, 0, 17, 0)}
RATES = [96000, 88200, 64000, 48000, 44100, 32000, 24000, 22050, 16000, 12000, 11025, 8000, 7350]
_LONG = {0: "96", 1: "96", 2: "64", 3: "48", 4: "48", 5: "32", 6: "24", 7: "24", 8: "16", 9: "16", 10: "16", 11: "8",
         12: "8"}
_SHORT = {0: "96", 1: "96", 2: "96", 3: "48", 4: "48", 5: "48", 6: "24", 7: "24", 8: "16", 9: "16", 10: "16",
          11: "8", 12: "8"}
CHANNELS = [0, 1, 2, 3, 4, 5, 6, 8]
# elements of each channel configuration (SCE / CPE / LFE in bitstream order)
CONFIG_ELEMENTS = {1: "S", 2: "C", 3: "SC", 4: "SCS", 5: "SCC", 6: "SCCL", 7: "SCCCL"}


def swb_long(sri):
    return TAB["kSwbLong" + _LONG[sri]]


def swb_short(sri):
    return TAB["kSwbShort" + _SHORT[sri]]


def _strings(c, l):
    return [format(int(a), "0%db" % int(b)) for a, b in zip(c, l)]


_DEC = {k: {s: i for i, s in enumerate(_strings(TAB["cb%dc" % k], TAB["cb%dl" % k]))} for k in range(1, 12)}
_DEC_SF = {s: i for i, s in enumerate(_strings(TAB["sfc"], TAB["sfl"]))}


def table_checks() -> Dict[str, bool]:
    from fractions import Fraction

    res = {}
    for name in ["cb%d" % k for k in range(1, 12)] + ["sf"]:
        strs = _strings(TAB[name + "c"], TAB[name + "l"])
        srt = sorted(strs)
        res[name] = (sum(Fraction(1, 2 ** len(s)) for s in strs) == 1
                     and all(not srt[i + 1].startswith(srt[i]) for i in range(len(srt) - 1))
                     and all(int(c) < 2 ** int(n) for c, n in zip(TAB[name + "c"], TAB[name + "l"])))
    bands = {"96": 41, "64": 47, "48": 49, "32": 51, "24": 47, "16": 43, "8": 40}
    res["swb_long"] = all(TAB["kSwbLong" + k][-1] == 1024 and len(TAB["kSwbLong" + k]) == n + 1
                          and np.all(np.diff(TAB["kSwbLong" + k]) > 0) for k, n in bands.items())
    sb = {"96": 12, "48": 14, "24": 15, "16": 15, "8": 15}
    res["swb_short"] = all(TAB["kSwbShort" + k][-1] == 128 and len(TAB["kSwbShort" + k]) == n + 1
                           and np.all(np.diff(TAB["kSwbShort" + k]) > 0) for k, n in sb.items())
    return res


class Bits:
    def __init__(self, data: bytes):
        self.s = "".join(format(x, "08b") for x in data)
        self.pos = 0

    def get(self, n):
        if n <= 0:
            return 0
        seg = self.s[self.pos: self.pos + n]
        self.pos += n
        if len(seg) < n:
            raise ValueError("read past the end of the access unit")
        return int(seg, 2)

    def huff(self, table):
        for n in range(1, 20):
            seg = self.s[self.pos: self.pos + n]
            if seg in table:
                self.pos += n
                return table[seg]
        raise ValueError("codeword not in table")


def parse_asc(asc: bytes) -> dict:
    br = Bits(asc)
    aot = br.get(5)
    sri = br.get(4)
    cc = br.get(4)
    if aot != 2 or sri > 12 or not 1 <= cc <= 7:
        raise ValueError("not an AAC-LC configuration this oracle decodes")
    return {"sri": sri, "sample_rate": RATES[sri], "chan_config": cc, "channels": CHANNELS[cc]}


# ---- windows / IMDCT ----------------------------------------------------------------------------------------------
def kbd_window(N, alpha):
    p = np.arange(N // 2 + 1)
    k = np.i0(np.pi * alpha * np.sqrt(np.maximum(0.0, 1 - ((p - N / 4) / (N / 4)) ** 2)))
    rise = np.sqrt(np.cumsum(k)[: N // 2] / k.sum())
    return np.concatenate([rise, rise[::-1]])


def sine_window(N):
    return np.sin(np.pi / N * (np.arange(N) + 0.5))


WIN_LONG = [sine_window(2048), kbd_window(2048, 4.0)]
WIN_SHORT = [sine_window(256), kbd_window(256, 6.0)]
_IM = {}


def imdct(X):
    N = 2 * len(X)
    if N not in _IM:
        n, k = np.arange(N), np.arange(N // 2)
        _IM[N] = (2.0 / N) * np.cos(2 * np.pi / N * np.outer(n + N / 4 + 0.5, k + 0.5))
    return _IM[N] @ X


# ---- one access unit ----------------------------------------------------------------------------------------------
def _ics_info(br, sri):
    br.get(1)
    ws, shape = br.get(2), br.get(1)
    if ws == 2:
        max_sfb, grouping = br.get(4), br.get(7)
        groups = [1]
        for i in range(7):
            if grouping & (1 << (6 - i)):
                groups[-1] += 1
            else:
                groups.append(1)
        if max_sfb > len(swb_short(sri)) - 1:
            raise ValueError("max_sfb")
    else:
        max_sfb, groups = br.get(6), [1]
        if br.get(1):
            raise ValueError("prediction")
        if max_sfb > len(swb_long(sri)) - 1:
            raise ValueError("max_sfb")
    return {"ws": ws, "shape": shape, "max_sfb": max_sfb, "groups": groups}


def _noise(width, sf, seed):
    """The native decoder's PNS generator: a 32-bit LCG seeded from (frame, channel, window, band)."""
    st = ((seed * 2654435761) & 0xFFFFFFFF) ^ 0x9E3779B9
    out = np.zeros(width)
    for k in range(width):
        st = (st * 1664525 + 1013904223) & 0xFFFFFFFF
        out[k] = float(np.float32(st - (1 << 32) if st >= 1 << 31 else st))
    e = float(np.sum(out * out))
    return out * (2.0 ** (0.25 * sf) / math.sqrt(max(e, 1e-30)))


def _ics(br, ics, common, sri, seed):
    gg = br.get(8)
    if not common:
        ics = _ics_info(br, sri)
    short = ics["ws"] == 2
    off = swb_short(sri) if short else swb_long(sri)
    ng, ms = len(ics["groups"]), ics["max_sfb"]
    cb = np.zeros((ng, 64), int)
    for g in range(ng):
        k = 0
        sb = 3 if short else 5
        while k < ms:
            c = br.get(4)
            if c == 12:
                raise ValueError("codebook 12")
            n = 0
            while True:
                inc = br.get(sb)
                n += inc
                if inc != (1 << sb) - 1:
                    break
            if k + n > ms:
                raise ValueError("section")
            cb[g, k: k + n] = c
            k += n
    sf = np.zeros((ng, 64), int)
    v, isp, nrg, first_noise = gg, 0, gg - 90, True
    for g in range(ng):
        for s in range(ms):
            c = cb[g, s]
            if c == 0:
                continue
            if c in (14, 15):
                isp += br.huff(_DEC_SF) - 60
                sf[g, s] = isp
            elif c == 13:
                if first_noise:
                    first_noise = False
                    nrg += br.get(9) - 256
                else:
                    nrg += br.huff(_DEC_SF) - 60
                sf[g, s] = nrg
            else:
                v += br.huff(_DEC_SF) - 60
                if not 0 <= v <= 255:
                    raise ValueError("scalefactor range")
                sf[g, s] = v
    pulses = []
    if br.get(1):
        if short:
            raise ValueError("pulse in short")
        n, start = br.get(2) + 1, br.get(6)
        k = int(swb_long(sri)[start])
        for _ in range(n):
            k += br.get(5)
            pulses.append((k, br.get(4)))
    tns = None
    if br.get(1):
        tns = []
        for w in range(8 if short else 1):
            nf = br.get(1 if short else 2)
            res = br.get(1) if nf else 0
            fl = []
            for _ in range(nf):
                length, order = br.get(4 if short else 6), br.get(3 if short else 5)
                if order > (7 if short else 12):
                    raise ValueError("tns order")
                d = comp = 0
                coefs = []
                if order:
                    d, comp = br.get(1), br.get(1)
                    bits = res + 3 - comp
                    for _ in range(order):
                        c = br.get(bits)
                        coefs.append(c - (1 << bits) if c & (1 << (bits - 1)) else c)
                fl.append((length, order, d, res + 3, coefs))
            tns.append(fl)
    if br.get(1):
        raise ValueError("gain control")
    q = np.zeros(1024, np.int64)
    w0 = 0
    for g, gl in enumerate(ics["groups"]):
        for s in range(ms):
            c = cb[g, s]
            if c == 0 or c >= 13:
                continue
            dim, lav, signed, mod, o = CB[c]
            width = int(off[s + 1] - off[s])
            for w in range(w0, w0 + gl):
                base = w * 128 + int(off[s])
                for k in range(0, width, dim):
                    idx = br.huff(_DEC[c])
                    vals = []
                    for _ in range(dim):
                        vals.append(idx % mod - o)
                        idx //= mod
                    vals = vals[::-1]
                    if not signed:
                        vals = [-x if (x and br.get(1)) else x for x in vals]
                    if c == 11:
                        for i in range(2):
                            if abs(vals[i]) == 16:
                                n = 0
                                while br.get(1):
                                    n += 1
                                e = (1 << (n + 4)) + br.get(n + 4)
                                vals[i] = -e if vals[i] < 0 else e
                    q[base + k: base + k + dim] = vals
        w0 += gl
    for k, amp in pulses:
        q[k] = q[k] + amp if q[k] > 0 else q[k] - amp
    spec = np.zeros(1024)
    w0 = 0
    for g, gl in enumerate(ics["groups"]):
        for s in range(ms):
            c = cb[g, s]
            a, b = int(off[s]), int(off[s + 1])
            for w in range(w0, w0 + gl):
                if c == 13:
                    spec[w * 128 + a: w * 128 + b] = _noise(b - a, sf[g, s], seed * 4096 + w * 64 + s)
                elif 0 < c < 13:
                    qq = q[w * 128 + a: w * 128 + b].astype(np.float64)
                    spec[w * 128 + a: w * 128 + b] = np.sign(qq) * np.abs(qq) ** (4 / 3) * 2.0 ** (0.25 * (sf[g, s] - 100))
        w0 += gl
    return {"ics": ics, "cb": cb, "sf": sf, "tns": tns, "spec": spec}


def _stereo(L, R, msp, ms_used, sri):
    ics = L["ics"]
    off = swb_short(sri) if ics["ws"] == 2 else swb_long(sri)
    w0 = 0
    for g, gl in enumerate(ics["groups"]):
        for s in range(ics["max_sfb"]):
            a, b = int(off[s]), int(off[s + 1])
            ms = msp == 2 or (msp == 1 and ms_used[g][s])
            cl, cr = L["cb"][g, s], R["cb"][g, s]
            for w in range(w0, w0 + gl):
                sl = slice(w * 128 + a, w * 128 + b)
                if cr in (14, 15):
                    c = (1.0 if cr == 15 else -1.0) * (-1.0 if (msp and ms) else 1.0)
                    R["spec"][sl] = L["spec"][sl] * c * 2.0 ** (-0.25 * R["sf"][g, s])
                elif cl == 13 and cr == 13 and ms:
                    v = L["spec"][sl]
                    R["spec"][sl] = v * (2.0 ** (0.25 * R["sf"][g, s]) / math.sqrt(max(float(v @ v), 1e-30)))
                elif ms and cl != 13 and cr != 13:
                    m, d = L["spec"][sl].copy(), R["spec"][sl].copy()
                    L["spec"][sl], R["spec"][sl] = m + d, m - d
        w0 += gl


def _tns(ch, sri):
    if ch["tns"] is None:
        return
    ics = ch["ics"]
    short = ics["ws"] == 2
    off = swb_short(sri) if short else swb_long(sri)
    nb = len(off) - 1
    maxb = min(int(TAB["kTnsMaxBandsShort" if short else "kTnsMaxBandsLong"][sri]), ics["max_sfb"])
    for w, fl in enumerate(ch["tns"]):
        top = nb
        for length, order, direction, res, coefs in fl:
            bottom = max(top - length, 0)
            lo, hi = int(off[min(bottom, maxb)]), int(off[min(top, maxb)])
            top = bottom
            if not order or hi <= lo:
                continue
            iq = ((1 << (res - 1)) - 0.5) / (math.pi / 2)
            iqm = ((1 << (res - 1)) + 0.5) / (math.pi / 2)
            tmp = [math.sin(c / (iq if c >= 0 else iqm)) for c in coefs]
            a = [1.0] + [0.0] * order
            for m in range(1, order + 1):
                b = a[:]
                for i in range(1, m):
                    b[i] = a[i] + tmp[m - 1] * a[m - i]
                a = b
                a[m] = tmp[m - 1]
            seg = ch["spec"][w * 128 + lo: w * 128 + hi]
            idx = range(len(seg) - 1, -1, -1) if direction else range(len(seg))
            state = [0.0] * order
            for i in idx:
                y = seg[i] - sum(a[j + 1] * state[j] for j in range(order))
                state = [y] + state[:-1]
                seg[i] = y


def _filterbank(ch, st):
    ics = ch["ics"]
    ws, cs, ps = ics["ws"], ics["shape"], st["shape"]
    z = np.zeros(2048)
    if ws == 2:
        for w in range(8):
            y = imdct(ch["spec"][w * 128: w * 128 + 128])
            win = np.concatenate([WIN_SHORT[ps if w == 0 else cs][:128], WIN_SHORT[cs][128:]])
            z[448 + 128 * w: 448 + 128 * w + 256] += y * win
    else:
        y = imdct(ch["spec"])
        win = np.ones(2048)
        if ws == 3:
            win[:448] = 0
            win[448:576] = WIN_SHORT[ps][:128]
        else:
            win[:1024] = WIN_LONG[ps][:1024]
        if ws == 1:
            win[1472:1600] = WIN_SHORT[cs][128:]
            win[1600:] = 0
        else:
            win[1024:] = WIN_LONG[cs][1024:]
        z = y * win
    out = (st["overlap"] + z[:1024]) / 32768.0
    st["overlap"], st["shape"] = z[1024:], cs
    return out


def decode_unit(unit: bytes, cfg: dict, states: list, frame_index: int, stats: Optional[dict] = None) -> np.ndarray:
    br = Bits(unit)
    sri, nch = cfg["sri"], cfg["channels"]
    pcm = np.zeros((1024, nch))
    c = 0
    while True:
        eid = br.get(3)
        if eid == 7:
            break
        if eid in (0, 3):
            br.get(4)
            ch = _ics(br, None, False, sri, frame_index * 8 + c)
            _tns(ch, sri)
            pcm[:, c] = _filterbank(ch, states[c])
            c += 1
        elif eid == 1:
            br.get(4)
            common = br.get(1)
            ics, msp, ms_used = None, 0, np.zeros((8, 64), int)
            if common:
                ics = _ics_info(br, sri)
                msp = br.get(2)
                if msp == 1:
                    for g in range(len(ics["groups"])):
                        for s in range(ics["max_sfb"]):
                            ms_used[g, s] = br.get(1)
            L = _ics(br, ics, common, sri, frame_index * 8 + c)
            R = _ics(br, ics, common, sri, frame_index * 8 + c + 1)
            if common:
                _stereo(L, R, msp, ms_used, sri)
            for j, ch in enumerate((L, R)):
                _tns(ch, sri)
                pcm[:, c + j] = _filterbank(ch, states[c + j])
            c += 2
        elif eid == 4:
            br.get(4)
            align = br.get(1)
            n = br.get(8)
            n += br.get(8) if n == 255 else 0
            if align:
                br.pos = (br.pos + 7) // 8 * 8
            br.pos += 8 * n
        elif eid == 5:
            br.get(10)
            nf, ns, nb, nl, na, nc = br.get(4), br.get(4), br.get(4), br.get(2), br.get(3), br.get(4)
            for _ in range(3):
                if br.get(1):
                    br.get(4 if _ < 2 else 3)
            br.pos += 5 * (nf + ns + nb) + 4 * (nl + na) + 5 * nc
            br.pos = (br.pos + 7) // 8 * 8
            br.pos += 8 * br.get(8)
        elif eid == 6:
            n = br.get(4)
            if n == 15:
                n += br.get(8) - 1
            br.pos += 8 * n
        else:
            raise ValueError("coupling element")
    if stats is not None:  # the END element closes the unit: only byte-alignment padding may follow
        stats.setdefault("end_exact", []).append((br.pos + 7) // 8 == len(unit))
    return pcm


def decode_raw(asc: bytes, units: List[bytes], stats: Optional[dict] = None):
    cfg = parse_asc(asc)
    states = [{"overlap": np.zeros(1024), "shape": 0} for _ in range(cfg["channels"])]
    out = [decode_unit(u, cfg, states, k, stats) for k, u in enumerate(units)]
    pcm = np.concatenate(out) if out else np.zeros((0, cfg["channels"]))
    return pcm.astype(np.float32), cfg["sample_rate"], stats


def adts_units(data: bytes):
    pos, units, cfg = 0, [], None
    while pos + 7 <= len(data):
        if data[pos] != 0xFF or (data[pos + 1] & 0xF6) != 0xF0:
            break
        prot = data[pos + 1] & 1
        sri, cc = (data[pos + 2] >> 2) & 15, ((data[pos + 2] & 1) << 2) | (data[pos + 3] >> 6)
        flen = ((data[pos + 3] & 3) << 11) | (data[pos + 4] << 3) | (data[pos + 5] >> 5)
        hl = 7 if prot else 9
        cfg = cfg or bytes([0x10 | (sri >> 1), ((sri & 1) << 7) | (cc << 3)])
        units.append(data[pos + hl: pos + flen])
        pos += flen
    return cfg, units


def decode_adts(data: bytes, stats: Optional[dict] = None):
    asc, units = adts_units(data)
    return decode_raw(asc, units, stats)


# ---- random-syntax writer -----------------------------------------------------------------------------------------
class BitWriter:
    def __init__(self):
        self.parts: List[str] = []
        self.n = 0

    def put(self, v, n):
        if n:
            self.parts.append(format(int(v), "0%db" % n))
            self.n += n

    def align(self):
        self.put(0, -self.n % 8)

    def bytes(self) -> bytes:
        s = "".join(self.parts)
        s += "0" * (-len(s) % 8)
        return bytes(int(s[i: i + 8], 2) for i in range(0, len(s), 8))


def _put_huff(w, table, idx):
    w.put(TAB[table + "c"][idx], int(TAB[table + "l"][idx]))


def _rand_ics_info(rng, sri, ws=None):
    ws = int(rng.integers(0, 4)) if ws is None else ws
    shape = int(rng.integers(0, 2))
    if ws == 2:
        return {"ws": 2, "shape": shape, "max_sfb": int(rng.integers(0, len(swb_short(sri)))),
                "grouping": int(rng.integers(0, 128))}
    return {"ws": ws, "shape": shape, "max_sfb": int(rng.integers(0, len(swb_long(sri))))}


def _groups(info):
    if info["ws"] != 2:
        return [1]
    g = [1]
    for i in range(7):
        if info["grouping"] & (1 << (6 - i)):
            g[-1] += 1
        else:
            g.append(1)
    return g


def _write_ics_info(w, info):
    w.put(0, 1)
    w.put(info["ws"], 2)
    w.put(info["shape"], 1)
    if info["ws"] == 2:
        w.put(info["max_sfb"], 4)
        w.put(info["grouping"], 7)
    else:
        w.put(info["max_sfb"], 6)
        w.put(0, 1)


def _write_ics(w, rng, info, common, sri, right=False, allow_is=False):
    short = info["ws"] == 2
    off = swb_short(sri) if short else swb_long(sri)
    groups = _groups(info)
    ms = info["max_sfb"]
    gg = int(rng.integers(110, 170))
    w.put(gg, 8)
    if not common:
        _write_ics_info(w, info)
    choices = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 11, 13] + ([14, 15] if allow_is and right else [])
    cbs = np.zeros((len(groups), 64), int)
    sb = 3 if short else 5
    for g in range(len(groups)):
        k = 0
        while k < ms:
            c = int(rng.choice(choices))
            n = int(rng.integers(1, ms - k + 1))
            w.put(c, 4)
            left = n
            while left >= (1 << sb) - 1:
                w.put((1 << sb) - 1, sb)
                left -= (1 << sb) - 1
            w.put(left, sb)
            cbs[g, k: k + n] = c
            k += n
    v, isp, nrg, first = gg, 0, gg - 90, True
    for g in range(len(groups)):
        for s in range(ms):
            c = cbs[g, s]
            if c == 0:
                continue
            if c in (14, 15):
                d = int(rng.integers(-8, 9))
                isp += d
                _put_huff(w, "sf", d + 60)
            elif c == 13:
                if first:
                    first = False
                    d = int(rng.integers(-20, 21))
                    w.put(d + 256, 9)
                else:
                    d = int(rng.integers(-10, 11))
                    _put_huff(w, "sf", d + 60)
                nrg += d
            else:
                d = int(rng.integers(-6, 7))
                if not 0 <= v + d <= 255:
                    d = 0
                v += d
                _put_huff(w, "sf", d + 60)
    # pulse data (long windows)
    if not short and ms > 0 and rng.random() < 0.3:
        w.put(1, 1)
        n = int(rng.integers(1, 5))
        start = int(rng.integers(0, ms))
        w.put(n - 1, 2)
        w.put(start, 6)
        k = int(off[start])
        for _ in range(n):
            step = int(rng.integers(0, min(32, 1024 - k)))
            k += step
            w.put(step, 5)
            w.put(int(rng.integers(0, 16)), 4)
    else:
        w.put(0, 1)
    # TNS
    if rng.random() < 0.5:
        w.put(1, 1)
        for _ in range(8 if short else 1):
            nf = int(rng.integers(0, 2 if short else 4))
            w.put(nf, 1 if short else 2)
            if nf:
                res = int(rng.integers(0, 2))
                w.put(res, 1)
                for _ in range(nf):
                    w.put(int(rng.integers(0, 16 if short else 64)), 4 if short else 6)
                    order = int(rng.integers(0, 8 if short else 13))
                    w.put(order, 3 if short else 5)
                    if order:
                        w.put(int(rng.integers(0, 2)), 1)
                        comp = int(rng.integers(0, 2))
                        w.put(comp, 1)
                        bits = res + 3 - comp
                        for _ in range(order):
                            w.put(int(rng.integers(0, 1 << bits)), bits)
    else:
        w.put(0, 1)
    w.put(0, 1)  # gain control
    w0 = 0
    for g, gl in enumerate(groups):
        for s in range(ms):
            c = cbs[g, s]
            if c == 0 or c >= 13:
                continue
            dim, lav, signed, mod, o = CB[c]
            width = int(off[s + 1] - off[s])
            for _ in range(gl):
                for _ in range(0, width, dim):
                    vals = [int(rng.integers(-lav, lav + 1)) for _ in range(dim)]
                    if rng.random() < 0.5:
                        vals = [max(-1, min(1, x)) for x in vals]
                    idx = 0
                    for x in vals:
                        idx = idx * mod + ((x + o) if signed else abs(x))
                    _put_huff(w, "cb%d" % c, idx)
                    if not signed:
                        for x in vals:
                            if x:
                                w.put(1 if x < 0 else 0, 1)
                    if c == 11:
                        for x in vals:
                            if abs(x) == 16:
                                n = int(rng.integers(0, 4))
                                w.put((1 << (n + 1)) - 2, n + 1)  # n ones, then a zero
                                w.put(int(rng.integers(0, 1 << (n + 4))), n + 4)
        w0 += gl


def write_unit(rng, cfg_channels: int, sri: int, extras: bool = True) -> bytes:
    w = BitWriter()
    elems = CONFIG_ELEMENTS[[k for k, v in enumerate(CHANNELS) if v == cfg_channels][0]]
    for e in elems:
        if extras and rng.random() < 0.2:  # a FIL element to skip (extension type 0: fill), count < 15 or escaped
            n = int(rng.integers(1, 30))
            w.put(6, 3)
            if n < 15:
                w.put(n, 4)
            else:
                w.put(15, 4)
                w.put(n - 14, 8)
            for i in range(n):
                w.put(int(rng.integers(0, 16 if i == 0 else 256)), 8)
        if extras and rng.random() < 0.1:  # a DSE
            w.put(4, 3)
            w.put(0, 4)
            al = int(rng.integers(0, 2))
            n = int(rng.integers(0, 10))
            w.put(al, 1)
            w.put(n, 8)
            if al:
                w.align()
            for _ in range(n):
                w.put(int(rng.integers(0, 256)), 8)
        if e in "SL":
            w.put(0 if e == "S" else 3, 3)
            w.put(0, 4)
            _write_ics(w, rng, _rand_ics_info(rng, sri), False, sri)
        else:
            w.put(1, 3)
            w.put(0, 4)
            common = int(rng.integers(0, 2))
            w.put(common, 1)
            if common:
                info = _rand_ics_info(rng, sri)
                _write_ics_info(w, info)
                msp = int(rng.integers(0, 3))
                w.put(msp, 2)
                if msp == 1:
                    for _ in range(len(_groups(info)) * info["max_sfb"]):
                        w.put(int(rng.integers(0, 2)), 1)
                _write_ics(w, rng, info, True, sri)
                _write_ics(w, rng, info, True, sri, right=True, allow_is=True)
            else:
                _write_ics(w, rng, _rand_ics_info(rng, sri), False, sri)
                _write_ics(w, rng, _rand_ics_info(rng, sri), False, sri)
    w.put(7, 3)
    return w.bytes()


def asc_bytes(sri: int, chan_config: int) -> bytes:
    return bytes([0x10 | (sri >> 1), ((sri & 1) << 7) | (chan_config << 3)])


def write_adts(rng, sri: int = 4, chan_config: int = 2, nframes: int = 6, crc: bool = False) -> bytes:
    out = bytearray()
    for _ in range(nframes):
        unit = write_unit(rng, CHANNELS[chan_config], sri)
        hl = 9 if crc else 7
        flen = hl + len(unit)
        h = bytearray(hl)
        h[0] = 0xFF
        h[1] = 0xF0 | (0 if crc else 1)
        h[2] = (1 << 6) | (sri << 2) | (chan_config >> 2)
        h[3] = ((chan_config & 3) << 6) | (flen >> 11)
        h[4] = (flen >> 3) & 0xFF
        h[5] = ((flen & 7) << 5) | 0x1F
        h[6] = 0xFC
        out += h + unit
    return bytes(out)


def _box(typ: bytes, body: bytes) -> bytes:
    return struct.pack(">I", 8 + len(body)) + typ + body


def write_mp4(rng, sri: int = 3, chan_config: int = 1, nframes: int = 8, edit: Optional[Tuple[int, int]] = None,
              units: Optional[List[bytes]] = None, chunk: int = 3) -> Tuple[bytes, List[bytes]]:
    """A minimal MP4 holding one AAC-LC sound track of random-syntax units (or the given ones); edit = (media_time,
    duration) in samples for an edit list. Returns (file bytes, the units)."""
    units = units if units is not None else [write_unit(rng, CHANNELS[chan_config], sri) for _ in range(nframes)]
    rate = RATES[sri]
    asc = asc_bytes(sri, chan_config)
    dsi = b"\x05" + bytes([len(asc)]) + asc
    dcd = bytes([0x40, 0x15]) + b"\x00\x00\x00" + struct.pack(">II", 0, 0) + dsi
    es = struct.pack(">HB", 1, 0) + b"\x04" + bytes([len(dcd)]) + dcd + b"\x06\x01\x02"
    esds = _box(b"esds", b"\x00\x00\x00\x00" + b"\x03" + bytes([len(es)]) + es)
    mp4a = _box(b"mp4a", bytes(6) + struct.pack(">H", 1) + bytes(8) + struct.pack(">HHHHI", CHANNELS[chan_config], 16,
                                                                              0, 0, rate << 16) + esds)
    stsd = _box(b"stsd", struct.pack(">II", 0, 1) + mp4a)
    n = len(units)
    stts = _box(b"stts", struct.pack(">III", 0, 1, n) + struct.pack(">I", 1024))
    nchunks = (n + chunk - 1) // chunk
    stsc = _box(b"stsc", struct.pack(">II", 0, 2 if n % chunk else 1) + struct.pack(">III", 1, chunk, 1)
                + (struct.pack(">III", nchunks, n % chunk, 1) if n % chunk else b""))
    stsz = _box(b"stsz", struct.pack(">III", 0, 0, n) + b"".join(struct.pack(">I", len(u)) for u in units))

    def moov(chunk_offsets):
        stco = _box(b"stco", struct.pack(">II", 0, len(chunk_offsets)) + b"".join(struct.pack(">I", o) for o in
                                                                                   chunk_offsets))
        stbl = _box(b"stbl", stsd + stts + stsc + stsz + stco)
        minf = _box(b"minf", _box(b"smhd", bytes(8)) + stbl)
        hdlr = _box(b"hdlr", bytes(8) + b"soun" + bytes(12) + b"snd\x00")
        mdhd = _box(b"mdhd", struct.pack(">IIIIIHH", 0, 0, 0, rate, n * 1024, 0, 0))
        trak_body = _box(b"tkhd", bytes(84))
        if edit is not None:
            trak_body += _box(b"edts", _box(b"elst", struct.pack(">IIIiI", 0, 1, edit[1], edit[0], 1 << 16)))
        trak_body += _box(b"mdia", mdhd + hdlr + minf)
        mvhd = _box(b"mvhd", struct.pack(">IIIII", 0, 0, 0, rate, 0) + bytes(80))  # (movie timescale = the rate)
        return _box(b"moov", mvhd + _box(b"trak", trak_body))

    ftyp = _box(b"ftyp", b"M4A \x00\x00\x00\x00M4A mp42isom")
    payload = b"".join(units)
    head = len(ftyp) + len(moov([0] * nchunks)) + 8
    offs, pos = [], head
    for c in range(nchunks):
        offs.append(pos)
        pos += sum(len(u) for u in units[c * chunk: (c + 1) * chunk])
    return ftyp + moov(offs) + _box(b"mdat", payload), units
