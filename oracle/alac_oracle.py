"""CPU oracle for Apple Lossless (ALAC) in MP4 / M4A — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module; the product (turbo-whisper-workspace_amd/twamd, csrc/alac.cpp) never does.

The reference decodes .m4a uploads (vocalis/security/security_monitor.py:355 and scripts/normalize_audio.py:226 list
the extension) through ffmpeg_read ($TF/pipelines/audio_utils.py:9-45); an Apple Lossless track in one goes through
ffmpeg's alac decoder (ffmpeg 6.x libavcodec/alac.c, not in this image; it follows Apple's published ALAC sources).
This module restates that decoder per sample in pure Python integers, in a different shape from the native one
(a dict-based element parser, the Rice coder as explicit prefix / remainder arithmetic), and holds an ENCODER that
drives every decoder path: mono SCE and stereo CPE elements, mix shift / weight decorrelation, 0-2 shifted-out low
bytes (20 / 24 / 32-bit), LPC orders 0-30 with random coefficients and quantisers, order 31 (first-order), prediction
type 15 (a first-order pre-pass), Rice escapes, zero runs, uncompressed (escape) frames and a short last frame.

Pinning: no ALAC file or decoder exists in this image, so parity with ffmpeg is UNPINNED. The encoder works the
decoder's adaptive predictor forward (the residual it writes is the one that makes the decoder reproduce its input),
so the lossless round trip pins the semantics the two share: a wrong coefficient order, adaptation sign, Rice
remainder rule, zero-run modifier or decorrelation formula loses samples.
"""
from __future__ import annotations

import struct
from typing import List, Optional, Tuple

import numpy as np


def sext(v: int, bits: int) -> int:
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def s32(v: int) -> int:
    return sext(v, 32)


def _log2(v: int) -> int:
    return v.bit_length() - 1 if v > 0 else 0


def _sign(v: int) -> int:
    return (v > 0) - (v < 0)


class BitReader:
    def __init__(self, data: bytes):
        self.s = "".join(format(b, "08b") for b in data)
        self.pos = 0

    def left(self) -> int:
        return len(self.s) - self.pos

    def peek(self, n: int) -> int:
        if n <= 0:
            return 0
        seg = self.s[self.pos: self.pos + n]
        return int((seg + "0" * (n - len(seg))) or "0", 2)

    def get(self, n: int) -> int:
        v = self.peek(n)
        self.pos += n
        return v

    def sget(self, n: int) -> int:
        return sext(self.get(n), n)


def parse_cookie(c: bytes) -> dict:
    if len(c) >= 36 and c[4:8] == b"alac":
        c = c[12:]
    fl, _ver, depth, pb, mb, kb, ch, _run, _mfb, _abr, rate = struct.unpack(">IBBBBBBHIII", c[:24])
    return dict(frame_length=fl, bit_depth=depth, pb=pb, mb=mb, kb=kb, channels=ch, rate=rate)


def _scalar(br: BitReader, k: int, bps: int) -> int:
    q = 0
    while q < 9 and br.get(1):
        q += 1
    if q == 9:
        return br.get(bps)
    if k == 1:
        return q
    v = br.peek(k)
    if v > 1:
        br.pos += k
        return q * ((1 << k) - 1) + v - 1
    br.pos += k - 1
    return q * ((1 << k) - 1)


def _rice(br: BitReader, n: int, bps: int, mult: int, cfg: dict) -> List[int]:
    out = [0] * n
    history, mod, i = cfg["mb"], 0, 0
    while i < n:
        if br.left() <= 0:
            raise ValueError("residuals run past the packet")
        k = min(_log2((history >> 9) + 3), cfg["kb"])
        x = (_scalar(br, k, bps) + mod) & 0xFFFFFFFF
        mod = 0
        out[i] = s32((x >> 1) ^ (-(x & 1) & 0xFFFFFFFF))
        history = 0xFFFF if x > 0xFFFF else (history + x * mult - ((history * mult) >> 9)) & 0xFFFFFFFF
        if history < 128 and i + 1 < n:
            k = min(7 - _log2(history) + ((history + 16) >> 6), cfg["kb"])
            block = s32(_scalar(br, k, 16))
            if block > 0:
                block = min(block, n - i - 1)
                i += block
            if block <= 0xFFFF:
                mod = 1
            history = 0
        i += 1
    return out


def _lpc(err: List[int], n: int, bps: int, coefs: Optional[List[int]], order: int, quant: int) -> List[int]:
    """ffmpeg's lpc_prediction; coefs (oldest sample first) adapt in place."""
    out = [0] * n
    if not n:
        return out
    out[0] = err[0]
    if n <= 1:
        return out
    if order == 0:
        out[1:] = err[1:n]
        return out
    if order == 31:
        for i in range(1, n):
            out[i] = sext(out[i - 1] + err[i], bps)
        return out
    i = 1
    while i <= order and i < n:
        out[i] = sext(out[i - 1] + err[i], bps)
        i += 1
    while i < n:
        d = out[i - order - 1]
        base = i - order
        acc = s32(sum((out[base + j] - d) * coefs[j] for j in range(order)))
        v = (acc + (1 << (quant - 1))) >> quant
        e = err[i] & 0xFFFFFFFF
        out[i] = sext(v + d + e, bps)
        es = _sign(s32(e))
        if es:
            j = 0
            while j < order and s32(e * es) > 0:
                dv = d - out[base + j]
                sg = _sign(dv) * es
                coefs[j] -= sg
                dv = s32(dv * sg)
                e = (e - (dv >> quant) * (j + 1)) & 0xFFFFFFFF
                j += 1
        i += 1
    return out


def decode_packet(pkt: bytes, cfg: dict) -> np.ndarray:
    """One access unit -> int32 [frames, channels] (the decoder's integer samples before the output scaling)."""
    br = BitReader(pkt)
    nch, depth = cfg["channels"], cfg["bit_depth"]
    cols: List[Optional[List[int]]] = [None] * nch
    ch, nb = 0, 0
    while br.left() >= 3:
        tag = br.get(3)
        if tag == 7:
            break
        if tag not in (0, 1, 3):
            raise ValueError(f"element {tag}")
        chans = 2 if tag == 1 else 1
        if ch + chans > nch:
            raise ValueError("too many channels")
        br.get(16)
        has_size = br.get(1)
        extra = br.get(2) << 3
        bps = depth - extra + chans - 1
        compressed = not br.get(1)
        nout = br.get(32) if has_size else cfg["frame_length"]
        if not 0 < nout <= cfg["frame_length"] or (nb and nout != nb):
            raise ValueError("sample count")
        nb = nout
        shift = weight = 0
        if compressed:
            shift, weight = br.get(8), br.get(8)
            params = []
            for _ in range(chans):
                ptype, quant, hmult, order = br.get(4), br.get(4), br.get(3), br.get(5)
                if order >= cfg["frame_length"] or not quant:
                    raise ValueError("predictor")
                coefs = [0] * order
                for i in range(order - 1, -1, -1):
                    coefs[i] = br.sget(16)
                params.append((ptype, quant, hmult, order, coefs))
            lows = [[0] * nb for _ in range(chans)]
            if extra:
                for i in range(nb):
                    for c in range(chans):
                        lows[c][i] = br.get(extra)
            outs = []
            for c in range(chans):
                ptype, quant, hmult, order, coefs = params[c]
                err = _rice(br, nb, bps, hmult * cfg["pb"] // 4, cfg)
                if ptype == 15:
                    err = _lpc(err, nb, bps, None, 31, 0)
                outs.append(_lpc(err, nb, bps, coefs, order, quant))
        else:
            raw = [[0] * nb for _ in range(chans)]
            for i in range(nb):
                for c in range(chans):
                    raw[c][i] = br.sget(depth)
            outs, extra = raw, 0
        if chans == 2 and weight:
            for i in range(nb):
                a, b = outs[0][i], outs[1][i]
                a = s32(a - ((b * weight) >> shift))
                b = s32(b + a)
                outs[0][i], outs[1][i] = b, a
        if extra:
            outs = [[s32((outs[c][i] << extra) | lows[c][i]) for i in range(nb)] for c in range(chans)]
        for c in range(chans):
            cols[ch + c] = outs[c]
        ch += chans
    return np.array(cols, np.int64).T.reshape(nb, nch)


def to_float(x: np.ndarray, depth: int) -> np.ndarray:
    """The decoder's integer samples as ffmpeg_read sees them (s16 truncation / s32 shift, then f32)."""
    if depth == 16:
        return (((x + 32768) % 65536) - 32768).astype(np.float64).astype(np.float32) / np.float32(32768.0)
    y = ((x << (32 - depth)) + 2 ** 31) % 2 ** 32 - 2 ** 31
    return (y.astype(np.float64) / 2147483648.0).astype(np.float32)


def decode(cookie: bytes, packets: List[bytes]) -> np.ndarray:
    cfg = parse_cookie(cookie)
    parts = [to_float(decode_packet(p, cfg), cfg["bit_depth"]) for p in packets]
    return np.concatenate(parts) if parts else np.zeros((0, cfg["channels"]), np.float32)


# ---- encoder ---------------------------------------------------------------------------------------------------------
class BitWriter:
    def __init__(self):
        self.bits: List[str] = []

    def put(self, v: int, n: int):
        if n:
            self.bits.append(format(v & ((1 << n) - 1), "0%db" % n))

    def bytes(self) -> bytes:
        s = "".join(self.bits)
        s += "0" * (-len(s) % 8)
        return bytes(int(s[i: i + 8], 2) for i in range(0, len(s), 8))


def _put_scalar(w: BitWriter, x: int, k: int, bps: int):
    if k == 1:
        q, r = x, 0
    else:
        q, r = divmod(x, (1 << k) - 1)
    if q > 8:
        w.put(0x1FF, 9)
        w.put(x, bps)
        return
    w.put((1 << (q + 1)) - 2, q + 1)  # q ones and a zero
    if k != 1:
        if r == 0:
            w.put(0, k - 1)
        else:
            w.put(r + 1, k)


def _put_rice(w: BitWriter, err: List[int], bps: int, mult: int, cfg: dict):
    n = len(err)
    history, mod, i = cfg["mb"], 0, 0
    while i < n:
        e = err[i]
        x = ((e << 1) ^ (e >> 31)) & 0xFFFFFFFF
        x -= mod
        assert x >= 0
        mod = 0
        k = min(_log2((history >> 9) + 3), cfg["kb"])
        _put_scalar(w, x, k, bps)
        xd = ((e << 1) ^ (e >> 31)) & 0xFFFFFFFF  # the value the decoder reconstructs (after its modifier)
        history = 0xFFFF if xd > 0xFFFF else (history + xd * mult - ((history * mult) >> 9)) & 0xFFFFFFFF
        if history < 128 and i + 1 < n:
            run = 0
            while i + 1 + run < n and err[i + 1 + run] == 0 and run < 0xFFFF:
                run += 1
            k2 = min(7 - _log2(history) + ((history + 16) >> 6), cfg["kb"])
            _put_scalar(w, run, k2, 16)
            i += run
            mod = 1
            history = 0
        i += 1


def _forward_lpc(s: List[int], bps: int, coefs: List[int], order: int, quant: int) -> List[int]:
    """The residuals that make _lpc(residuals) reproduce s (coefs adapt exactly as the decoder's)."""
    n = len(s)
    err = [0] * n
    if not n:
        return err
    err[0] = s[0]
    if order == 0:
        err[1:] = s[1:]
        return err
    if order == 31:
        for i in range(1, n):
            err[i] = sext(s[i] - s[i - 1], bps)
        return err
    i = 1
    while i <= order and i < n:
        err[i] = sext(s[i] - s[i - 1], bps)
        i += 1
    while i < n:
        d = s[i - order - 1]
        base = i - order
        acc = s32(sum((s[base + j] - d) * coefs[j] for j in range(order)))
        v = (acc + (1 << (quant - 1))) >> quant
        err[i] = sext(s[i] - v - d, bps)
        e = err[i] & 0xFFFFFFFF
        es = _sign(s32(e))
        if es:
            j = 0
            while j < order and s32(e * es) > 0:
                dv = d - s[base + j]
                sg = _sign(dv) * es
                coefs[j] -= sg
                dv = s32(dv * sg)
                e = (e - (dv >> quant) * (j + 1)) & 0xFFFFFFFF
                j += 1
        i += 1
    return err


def encode_packet(x: np.ndarray, cfg: dict, rng: np.random.Generator, mode: str = "random") -> bytes:
    """int samples [n, channels] (in the bit depth's range) -> one ALAC access unit."""
    n, nch = x.shape
    depth = cfg["bit_depth"]
    w = BitWriter()
    w.put(1 if nch == 2 else 0, 3)
    w.put(0, 4)
    w.put(0, 12)
    partial = n != cfg["frame_length"]
    w.put(int(partial), 1)
    uncompressed = mode == "raw" or (mode == "random" and rng.random() < 0.1)
    extra_bytes = 0 if (depth == 16 or uncompressed) else int(rng.integers(0, 3 if depth >= 24 else 2))
    if depth == 32 and nch == 2 and not uncompressed:
        extra_bytes = max(extra_bytes, 1)  # (33 significant bits of a side channel are refused)
    extra = 8 * extra_bytes
    w.put(extra_bytes, 2)
    w.put(int(uncompressed), 1)
    if partial:
        w.put(n, 32)
    cols = [[int(v) for v in x[:, c]] for c in range(nch)]
    if uncompressed:
        for i in range(n):
            for c in range(nch):
                w.put(cols[c][i], depth)
        w.put(7, 3)
        return w.bytes()
    lows = [[v & ((1 << extra) - 1) for v in col] for col in cols] if extra else None
    highs = [[v >> extra for v in col] for col in cols]
    shift, weight = 0, 0
    if nch == 2:
        shift, weight = (2, int(rng.choice([0, 1, 2, 3, 4])))
        if weight:
            L, R = highs
            v_ = [L[i] - R[i] for i in range(n)]
            u_ = [R[i] + ((v_[i] * weight) >> shift) for i in range(n)]
            highs = [u_, v_]
    bps = depth - extra + nch - 1
    w.put(shift, 8)
    w.put(weight, 8)
    params = []
    for c in range(nch):
        order = int(rng.choice([0, 1, 2, 4, 8, 12, 16, 24, 30, 31]))
        quant = int(rng.integers(6, 16))
        ptype = 15 if rng.random() < 0.2 else 0
        hmult = int(rng.integers(1, 8))
        coefs = [int(v) for v in rng.integers(-(1 << (quant - 3)), 1 << (quant - 2), order)] if order != 31 else \
            [int(v) for v in rng.integers(-300, 300, 31)]
        params.append((ptype, quant, hmult, order, coefs))
        w.put(ptype, 4), w.put(quant, 4), w.put(hmult, 3), w.put(order, 5)
        for i in range(order - 1, -1, -1):
            w.put(coefs[i], 16)
    if extra:
        for i in range(n):
            for c in range(nch):
                w.put(lows[c][i], extra)
    for c in range(nch):
        ptype, quant, hmult, order, coefs = params[c]
        err = _forward_lpc(highs[c], bps, list(coefs), order, quant)
        if ptype == 15:  # the decoder integrates the residuals first: difference them here
            err = [err[0]] + [sext(err[i] - err[i - 1], bps) for i in range(1, n)]
        _put_rice(w, err, bps, hmult * cfg["pb"] // 4, cfg)
    w.put(7, 3)
    return w.bytes()


def cookie_bytes(cfg: dict, atom: bool = True) -> bytes:
    body = struct.pack(">IBBBBBBHIII", cfg["frame_length"], 0, cfg["bit_depth"], cfg["pb"], cfg["mb"], cfg["kb"],
                       cfg["channels"], 255, 0, 0, cfg["rate"])
    return struct.pack(">I", 36) + b"alac" + bytes(4) + body if atom else body


def signal(n: int, nch: int, depth: int, rng: np.random.Generator) -> np.ndarray:
    """Speech-like test material in the depth's range: tones, noise, silent stretches (zero runs) and a few full-scale
    samples (Rice escapes)."""
    t = np.arange(n)
    top = 2 ** (depth - 1) - 1
    out = np.zeros((n, nch), np.int64)
    for c in range(nch):
        x = 0.3 * np.sin(2 * np.pi * (200 + 50 * c) * t / 16000) + 0.05 * rng.standard_normal(n)
        x[(t // 700) % 3 == 2] = 0.0
        y = np.round(x * top).astype(np.int64)
        y[rng.integers(0, n, 3)] = rng.choice([top, -top - 1], 3)
        out[:, c] = np.clip(y, -top - 1, top)
    return out


def write_stream(rng, nch: int = 2, depth: int = 16, frames: int = 4, frame_length: int = 4096, tail: int = 1000,
                 pb: int = 40, mb: int = 10, kb: int = 14, rate: int = 44100, mode: str = "random"):
    """(cookie, packets, the encoded int samples)."""
    cfg = dict(frame_length=frame_length, bit_depth=depth, pb=pb, mb=mb, kb=kb, channels=nch, rate=rate)
    total = frames * frame_length + tail
    x = signal(total, nch, depth, rng)
    packets = []
    for a in range(0, total, frame_length):
        packets.append(encode_packet(x[a: a + frame_length], cfg, rng, mode))
    return cookie_bytes(cfg), packets, x


def _box(typ: bytes, body: bytes) -> bytes:
    return struct.pack(">I", 8 + len(body)) + typ + body


def write_m4a(cookie: bytes, packets: List[bytes], cfg: dict, chunk: int = 3,
              edit: Optional[Tuple[int, int]] = None) -> bytes:
    """A minimal M4A holding one 'alac' sound track (sample entry + its 'alac' cookie atom, stts / stsc / stsz / stco,
    an optional edit list)."""
    rate, nch, fl = cfg["rate"], cfg["channels"], cfg["frame_length"]
    entry = _box(b"alac", bytes(6) + struct.pack(">H", 1) + bytes(8) +
                 struct.pack(">HHHHI", nch, cfg["bit_depth"], 0, 0, rate << 16) + cookie)
    stsd = _box(b"stsd", struct.pack(">II", 0, 1) + entry)
    n = len(packets)
    stts = _box(b"stts", struct.pack(">III", 0, 1, n) + struct.pack(">I", fl))
    nchunks = (n + chunk - 1) // chunk
    stsc = _box(b"stsc", struct.pack(">II", 0, 2 if n % chunk else 1) + struct.pack(">III", 1, chunk, 1)
                + (struct.pack(">III", nchunks, n % chunk, 1) if n % chunk else b""))
    stsz = _box(b"stsz", struct.pack(">III", 0, 0, n) + b"".join(struct.pack(">I", len(p)) for p in packets))

    def moov(offs):
        stco = _box(b"stco", struct.pack(">II", 0, len(offs)) + b"".join(struct.pack(">I", o) for o in offs))
        stbl = _box(b"stbl", stsd + stts + stsc + stsz + stco)
        minf = _box(b"minf", _box(b"smhd", bytes(8)) + stbl)
        hdlr = _box(b"hdlr", bytes(8) + b"soun" + bytes(12) + b"snd\x00")
        mdhd = _box(b"mdhd", struct.pack(">IIIIIHH", 0, 0, 0, rate, n * fl, 0, 0))
        trak = _box(b"tkhd", bytes(84))
        if edit is not None:
            trak += _box(b"edts", _box(b"elst", struct.pack(">IIIiI", 0, 1, edit[1], edit[0], 1 << 16)))
        trak += _box(b"mdia", mdhd + hdlr + minf)
        mvhd = _box(b"mvhd", struct.pack(">IIIII", 0, 0, 0, rate, 0) + bytes(80))
        return _box(b"moov", mvhd + _box(b"trak", trak))

    ftyp = _box(b"ftyp", b"M4A \x00\x00\x00\x00M4A mp42isom")
    head = len(ftyp) + len(moov([0] * nchunks)) + 8
    offs, pos = [], head
    for c in range(nchunks):
        offs.append(pos)
        pos += sum(len(p) for p in packets[c * chunk: (c + 1) * chunk])
    return ftyp + moov(offs) + _box(b"mdat", b"".join(packets))
