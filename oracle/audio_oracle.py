"""CPU oracle for the audio ingest — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module; the product
(turbo-whisper-workspace_amd/twamd) never does.

What it restates, and what pins it:

* `swr_resample` — the resampler `ffmpeg -ac 1 -ar 16000` runs inside the reference's ffmpeg_read
  ($TF/pipelines/audio_utils.py:9-45): libswresample's default (swr filter_size 32, cutoff 0.97, Kaiser beta 9,
  exact rational phase count, linear interpolation unused because the phases are exact), with its start-of-
  stream mirror (invert_initial_buffer) and end-of-stream reflection (resample_flush). Written here per output
  sample in float64 with its own Bessel-I0 series, independently of twamd/audio.py's vectorised filter design.
  ffmpeg is not in this image and its SIMD float accumulation order is not reproducible, so parity of resampled
  audio against ffmpeg itself is UNPINNED; the GPU kernel is held to this float64 restatement.

* `flac_encode` — a small FLAC *encoder* (RFC 9639 bitstream: STREAMINFO with MD5, fixed or variable blocking,
  CONSTANT / VERBATIM / FIXED / LPC subframes, wasted bits, Rice partitions with escapes, all four stereo
  decorrelation modes, CRC-8/CRC-16). It exists to produce streams that exercise every decoder path; the native
  decoder must return the encoder's input PCM exactly. Real-encoder parity is pinned separately by
  examples/Test1/ChrisAndAlexDiTest.flac (libFLAC 1.4.2): its STREAMINFO MD5 must match the decoded PCM.

* `ms_adpcm_decode` / `ms_adpcm_encode` — Microsoft ADPCM (WAV format tag 2) as ffmpeg's adpcm_ms decodes it
  (ffmpeg 6.x libavcodec/adpcm.c, absent from this image; restated from Microsoft's published algorithm and that
  decoder's documented behaviour: the standard seven coefficient pairs, a predictor index > 6 drops the block), per
  nibble in pure Python; and a greedy encoder whose streams exercise every nibble, the delta floor and the s16 clamp.
  No MS ADPCM file or decoder exists in this image: parity against ffmpeg is UNPINNED; the encoder round trip pins
  the semantics (a wrong sign, order or coefficient scale breaks the reconstruction of its input).
"""
from __future__ import annotations

import hashlib
import math
from typing import List, Optional, Sequence

import numpy as np


# ---------------------------------------------------------------------------------------------- resampler
def _bessel_i0(x: float) -> float:
    s, t, k = 1.0, 1.0, 1
    while True:
        t *= (x / (2.0 * k)) ** 2
        s += t
        if t < 1e-17 * s:
            return s
        k += 1


def swr_taps(sr_in: int, sr_out: int, filter_size: int = 32, cutoff: float = 0.97, beta: float = 9.0):
    g = math.gcd(sr_in, sr_out)
    up, down = sr_out // g, sr_in // g
    factor = min(up / down * cutoff, 1.0)
    T = max(int(math.ceil(filter_size / factor)), 1)
    c = (T - 1) // 2
    bank = np.zeros((up, T))
    for ph in range(up):
        for i in range(T):
            x = math.pi * ((i - c) - ph / up) * factor
            y = 1.0 if x == 0 else math.sin(x) / x
            w = 2.0 * x / (factor * T * math.pi)
            bank[ph, i] = y * _bessel_i0(beta * math.sqrt(max(1.0 - w * w, 0.0)))
    bank /= bank[0].sum()
    return up, down, bank


def swr_resample(x: np.ndarray, sr_in: int, sr_out: int) -> np.ndarray:
    """float64 mono resampling; len = ceil(len(x) * up / down)."""
    x = np.asarray(x, np.float64)
    if sr_in == sr_out:
        return x.copy()
    up, down, bank = swr_taps(sr_in, sr_out)
    T = bank.shape[1]
    c = (T - 1) // 2
    n_in = len(x)
    n_out = -(-n_in * up // down)
    out = np.empty(n_out)
    for n in range(n_out):
        q = n * down
        ph, idx = q % up, q // up
        j = np.arange(idx - c, idx - c + T)
        j = np.where(j < 0, -j, j)  # mirror at the start (invert_initial_buffer)
        j = np.where(j >= n_in, 2 * (n_in - 1) - j, j)  # reflection at the end (resample_flush)
        j = np.clip(j, 0, n_in - 1)
        out[n] = float(np.dot(bank[ph], x[j]))
    return out


# ---------------------------------------------------------------------------------------------- FLAC writer
class _BitWriter:
    def __init__(self):
        self.acc = 0
        self.n = 0
        self.out = bytearray()

    def put(self, v: int, k: int):
        if k == 0:
            return
        v &= (1 << k) - 1
        self.acc = (self.acc << k) | v
        self.n += k
        while self.n >= 8:
            self.n -= 8
            self.out.append((self.acc >> self.n) & 0xFF)
        self.acc &= (1 << self.n) - 1

    def put_signed(self, v: int, k: int):
        assert -(1 << (k - 1)) <= v < (1 << (k - 1)), (v, k)
        self.put(v, k)

    def unary(self, q: int):
        while q >= 32:
            self.put(0, 32)
            q -= 32
        self.put(1, q + 1)

    def align(self):
        if self.n:
            self.put(0, 8 - self.n)

    def bytes(self) -> bytes:
        assert self.n == 0
        return bytes(self.out)


def _crc8(b: bytes) -> int:
    c = 0
    for x in b:
        c ^= x
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def _crc16(b: bytes) -> int:
    c = 0
    for x in b:
        c ^= x << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def _utf8_num(v: int) -> bytes:
    if v < 0x80:
        return bytes([v])
    for n_extra, lead_bits in ((1, 5), (2, 4), (3, 3), (4, 2), (5, 1), (6, 0)):
        if v < (1 << (lead_bits + 6 * n_extra)):
            lead = (0xFF << (7 - n_extra)) & 0xFF
            out = [lead | (v >> (6 * n_extra))]
            for i in range(n_extra - 1, -1, -1):
                out.append(0x80 | ((v >> (6 * i)) & 0x3F))
            return bytes(out)
    raise ValueError("number too large")


def _fixed_residual(x: np.ndarray, order: int) -> np.ndarray:
    r = x.astype(np.int64)
    for _ in range(order):
        r = np.concatenate([r[:1], np.diff(r)])
    # FLAC's fixed predictors = repeated differencing; the first `order` values are warm-up
    return r


def _rice_write(w: _BitWriter, res: Sequence[int], order: int, bs: int, porder: int, method: int,
                escape_parts: Sequence[int] = ()):
    w.put(method, 2)
    w.put(porder, 4)
    pbits, esc = (4, 15) if method == 0 else (5, 31)
    psize = bs >> porder
    pos = 0
    for p in range(1 << porder):
        cnt = psize - (order if p == 0 else 0)
        part = [int(v) for v in res[pos: pos + cnt]]
        pos += cnt
        if p in escape_parts:
            nb = max([abs(v).bit_length() + 1 for v in part] + [0])
            w.put(esc, pbits)
            w.put(nb, 5)
            for v in part:
                if nb:
                    w.put_signed(v, nb)
            continue
        u = [(v << 1) ^ (v >> 63) if v >= 0 else ((-v) << 1) - 1 for v in part]
        mean = (sum(u) / len(u)) if u else 0
        k = max(0, min(esc - 1, int(math.log2(mean + 1)) if mean > 0 else 0))
        w.put(k, pbits)
        for v in u:
            w.unary(v >> k)
            w.put(v & ((1 << k) - 1), k)


def _write_subframe(w: _BitWriter, x: np.ndarray, bps: int, kind: str, rng: np.random.Generator, opts: dict):
    bs = len(x)
    wasted = 0
    if opts.get("wasted", True) and np.any(x):
        tz = int(min((int(v) & -int(v)).bit_length() - 1 for v in x if v != 0))
        wasted = min(tz, bps - 1)
    if kind == "constant" and not np.all(x == x[0]):
        kind = "verbatim"
    xs = (x.astype(np.int64) >> wasted) if wasted else x.astype(np.int64)
    sbps = bps - wasted
    porder = opts.get("porder", 2)
    while bs % (1 << porder) or (bs >> porder) < 33:
        porder -= 1
        if porder == 0:
            break
    method = opts.get("rice_method", 0)
    esc = opts.get("escape_parts", ())

    def header(t):
        w.put(0, 1)
        w.put(t, 6)
        if wasted:
            w.put(1, 1)
            w.unary(wasted - 1)
        else:
            w.put(0, 1)

    if kind == "constant":
        header(0)
        w.put_signed(int(xs[0]), sbps)
    elif kind == "verbatim":
        header(1)
        for v in xs:
            w.put_signed(int(v), sbps)
    elif kind.startswith("fixed"):
        order = int(kind[5:])
        header(8 + order)
        for v in xs[:order]:
            w.put_signed(int(v), sbps)
        r = _fixed_residual(xs, order)
        _rice_write(w, r[order:], order, bs, porder, method, esc)
    elif kind.startswith("lpc"):
        order = int(kind[3:])
        prec = opts.get("qlp_precision", 12)
        shift = opts.get("qlp_shift", 10)
        # least-squares predictor, quantised; any integer coefficients give a valid stream
        X = np.stack([xs[order - 1 - j: bs - 1 - j] for j in range(order)], 1).astype(np.float64)
        y = xs[order:].astype(np.float64)
        try:
            a = np.linalg.lstsq(X, y, rcond=None)[0]
        except np.linalg.LinAlgError:
            a = np.zeros(order)
        lim = (1 << (prec - 1)) - 1
        q = np.clip(np.round(a * (1 << shift)), -lim - 1, lim).astype(np.int64)
        header(32 + order - 1)
        for v in xs[:order]:
            w.put_signed(int(v), sbps)
        w.put(prec - 1, 4)
        w.put_signed(shift, 5)
        for cf in q:
            w.put_signed(int(cf), prec)
        r = [int(xs[i]) - (int(sum(int(q[j]) * int(xs[i - 1 - j]) for j in range(order))) >> shift)
             for i in range(order, bs)]
        _rice_write(w, r, order, bs, porder, method, esc)
    else:
        raise ValueError(kind)


_BS_CODES = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12, 8192: 13,
             16384: 14, 32768: 15}
_SR_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9,
             48000: 10, 96000: 11}
_SS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def flac_encode(pcm: np.ndarray, sample_rate: int, bps: int, blocksizes: Sequence[int] = (4096,),
                subframe_kinds: Sequence[str] = ("lpc8",), stereo_modes: Sequence[int] = (0,),
                variable: bool = False, seed: int = 0, opts: Optional[dict] = None) -> bytes:
    """Encode int PCM [frames, channels] (values in [-2^(bps-1), 2^(bps-1))). Frame f uses
    blocksizes[f % len], subframe_kinds[(f + ch) % len] and, for 2 channels, channel assignment
    stereo_modes[f % len] (0 = independent, 8 = left/side, 9 = side/right, 10 = mid/side)."""
    opts = dict(opts or {})
    pcm = np.asarray(pcm, np.int64)
    if pcm.ndim == 1:
        pcm = pcm[:, None]
    n, nch = pcm.shape
    rng = np.random.default_rng(seed)
    frames: List[bytes] = []
    pos, f = 0, 0
    bsz_seen = []
    while pos < n:
        bs = min(blocksizes[f % len(blocksizes)], n - pos)
        bsz_seen.append(bs)
        blk = pcm[pos: pos + bs]
        mode = stereo_modes[f % len(stereo_modes)] if nch == 2 else 0
        if mode == 8:
            chans, extra = [blk[:, 0], blk[:, 0] - blk[:, 1]], [0, 1]
        elif mode == 9:
            chans, extra = [blk[:, 0] - blk[:, 1], blk[:, 1]], [1, 0]
        elif mode == 10:
            chans, extra = [(blk[:, 0] + blk[:, 1]) >> 1, blk[:, 0] - blk[:, 1]], [0, 1]
        else:
            mode = nch - 1
            chans, extra = [blk[:, c] for c in range(nch)], [0] * nch
        w = _BitWriter()
        w.put(0x3FFE, 14)
        w.put(0, 1)
        w.put(1 if variable else 0, 1)
        code = _BS_CODES.get(bs)
        if code is None or (not variable and pos + bs < n and bs != blocksizes[0]):
            code = 6 if bs <= 256 else 7
        w.put(code, 4)
        w.put(_SR_CODES.get(sample_rate, 0), 4)
        w.put(mode, 4)
        w.put(_SS_CODES.get(bps, 0), 3)
        w.put(0, 1)
        for byte in _utf8_num(pos if variable else f):
            w.put(byte, 8)
        if code == 6:
            w.put(bs - 1, 8)
        elif code == 7:
            w.put(bs - 1, 16)
        hdr = w.bytes()
        w.put(_crc8(hdr), 8)
        for c, x in enumerate(chans):
            kind = subframe_kinds[(f + c) % len(subframe_kinds)]
            order = int("".join(ch for ch in kind if ch.isdigit()) or 0)
            if order >= bs:
                kind = "verbatim"
            _write_subframe(w, x, bps + extra[c], kind, rng, opts)
        w.align()
        body = w.bytes()
        crc = _crc16(body)
        frames.append(body + bytes([crc >> 8, crc & 0xFF]))
        pos += bs
        f += 1
    nb = (bps + 7) // 8
    md5 = hashlib.md5(np.ascontiguousarray(pcm.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :nb]).tobytes())
    si = _BitWriter()
    bmin = min(bsz_seen[:-1] or bsz_seen) if variable else blocksizes[0]
    bmax = max(bsz_seen) if variable else blocksizes[0]
    si.put(bmin, 16)
    si.put(bmax, 16)
    si.put(min(len(x) for x in frames), 24)
    si.put(max(len(x) for x in frames), 24)
    si.put(sample_rate, 20)
    si.put(nch - 1, 3)
    si.put(bps - 1, 5)
    si.put(n, 36)
    streaminfo = si.bytes() + md5.digest()
    meta = bytes([0x80 | 0]) + len(streaminfo).to_bytes(3, "big") + streaminfo
    return b"fLaC" + meta + b"".join(frames)


# ---------------------------------------------------------------------------------------------- MS ADPCM
MS_COEF = [(256, 0), (512, -256), (0, 0), (192, 64), (240, 0), (460, -208), (392, -232)]
MS_ADAPT = [230, 230, 230, 230, 307, 409, 512, 614, 768, 614, 512, 409, 307, 230, 230, 230]


def _c_div(a: int, b: int) -> int:
    """C integer division (truncation toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def _ms_nibble(st: list, nib: int) -> int:
    """st = [coef1, coef2, delta, sample1, sample2] updated in place; returns the new sample."""
    c1, c2, delta, s1, s2 = st
    pred = _c_div(s1 * c1 + s2 * c2, 256) + (nib - 16 if nib & 8 else nib) * delta
    pred = max(-32768, min(32767, pred))
    delta = max(16, (MS_ADAPT[nib] * delta) >> 8)
    st[:] = [c1, c2, min(delta, 2147483647 // 768), pred, s1]
    return pred


def ms_adpcm_decode(payload: bytes, ch: int, align: int) -> np.ndarray:
    """WAV MS ADPCM blocks -> int16 [frames, ch] (1 or 2 channels)."""
    out = []
    for pos in range(0, len(payload), align):
        blk = payload[pos: pos + align]
        if len(blk) < 7 * ch:
            break
        if any(blk[c] > 6 for c in range(ch)):
            continue
        nb = (len(blk) - 6 * ch) * 2 // ch
        sts = []
        for c in range(ch):
            c1, c2 = MS_COEF[blk[c]]
            delta = int.from_bytes(blk[ch + 2 * c: ch + 2 * c + 2], "little", signed=True)
            s1 = int.from_bytes(blk[3 * ch + 2 * c: 3 * ch + 2 * c + 2], "little", signed=True)
            s2 = int.from_bytes(blk[5 * ch + 2 * c: 5 * ch + 2 * c + 2], "little", signed=True)
            sts.append([c1, c2, delta, s1, s2])
        rows = [[st[4] for st in sts], [st[3] for st in sts]]
        flat = []
        nbytes = (nb - 2) // 2 if ch == 1 else nb - 2
        for byte in blk[7 * ch: 7 * ch + nbytes]:
            flat.append(_ms_nibble(sts[0], byte >> 4))
            flat.append(_ms_nibble(sts[ch - 1], byte & 15))
        rows += [flat[i: i + ch] for i in range(0, len(flat), ch)]
        out += rows[:nb]
    return np.array(out, np.int16).reshape(-1, ch)


def ms_adpcm_encode(x: np.ndarray, ch: int, align: int, rng: np.random.Generator, predictors=None) -> bytes:
    """int16 [frames, ch] -> MS ADPCM blocks: per block and channel a predictor index (given, or random), an initial
    delta, the first two samples verbatim, then per sample the nibble whose decoded value is nearest the input
    (searching all 16, so the decoder's own update is what follows)."""
    per = (align - 6 * ch) * 2 // ch
    out = bytearray()
    for b0 in range(0, len(x), per):
        seg = x[b0: b0 + per]
        if len(seg) < 2:
            break
        pidx = [int(rng.integers(0, 7)) if predictors is None else predictors[c] for c in range(ch)]
        sts = [[*MS_COEF[pidx[c]], int(rng.integers(16, 512)), int(seg[1, c]), int(seg[0, c])] for c in range(ch)]
        hdr = bytes(pidx)
        hdr += b"".join(int(sts[c][2]).to_bytes(2, "little", signed=True) for c in range(ch))
        hdr += b"".join(int(seg[1, c]).to_bytes(2, "little", signed=True) for c in range(ch))
        hdr += b"".join(int(seg[0, c]).to_bytes(2, "little", signed=True) for c in range(ch))
        nibs = []
        for i in range(2, len(seg)):
            for c in range(ch):
                best = None
                for nib in range(16):
                    trial = list(sts[c])
                    v = _ms_nibble(trial, nib)
                    e = abs(v - int(seg[i, c]))
                    if best is None or e < best[0]:
                        best = (e, nib, trial)
                nibs.append(best[1])
                sts[c] = best[2]
        if len(nibs) % 2:
            nibs.append(0)
        body = bytes((nibs[i] << 4) | nibs[i + 1] for i in range(0, len(nibs), 2))
        out += hdr + body
    return bytes(out)
