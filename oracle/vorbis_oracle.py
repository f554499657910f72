"""CPU oracle for Ogg Vorbis ingest — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module; the product (turbo-whisper-workspace_amd/twamd, csrc/vorbis.cpp) never does.

The reference decodes Ogg uploads through ffmpeg_read ($TF/pipelines/audio_utils.py:9-45; ffmpeg's native Vorbis
decoder), which this image does not have, and there is no other Vorbis decoder here (no libvorbis, soundfile,
torchaudio). So this is a second, independent restatement of the Vorbis I specification and Ogg framing (RFC 3533),
written for clarity rather than speed, in a different shape from the native decoder: codewords assigned by a
leftmost-free-node search over an explicit binary tree and looked up by (length, value); the inverse MDCT as a
float64 cosine-matrix product; every block windowed and added into one global timeline at its own offset.

* `decode(data)` -> (f32 [frames, channels], sample_rate).
* `write_stream(rng, ...)` — a random *syntax* writer: identification / comment / setup headers with random
  codebooks (ordered / sparse / dense length coding, VQ lookup types 1 and 2), floor-1 configurations, residues of
  types 0 / 1 / 2, mappings with coupling and submaps, two modes; then audio packets of random payload bits (any bit
  string is a decodable Vorbis audio packet: decoders stop at the end of the packet). It exercises every decoder
  path the one real-encoder file does not.

Pinning: the only real Vorbis stream in this image is MathJax's a11y/invalid_keypress.ogg (libVorbis I 20101101,
44.1 kHz stereo, shipped by the kaleido / notebook Python packages); it must decode without error to exactly the
granule length of its last page. Against ffmpeg's own decoder the decoded samples are UNPINNED (no ffmpeg here).
"""
from __future__ import annotations

import math
import struct
from typing import List, Optional, Tuple

import numpy as np

# ---- Ogg ---------------------------------------------------------------------------------------------------------------


def _crc_table():
    t = []
    for i in range(256):
        r = i << 24
        for _ in range(8):
            r = ((r << 1) ^ 0x04C11DB7) if r & 0x80000000 else (r << 1)
            r &= 0xFFFFFFFF
        t.append(r)
    return t


_CRC = _crc_table()


def ogg_crc(b: bytes) -> int:
    c = 0
    for x in b:
        c = ((c << 8) & 0xFFFFFFFF) ^ _CRC[(c >> 24) ^ x]
    return c


def ogg_packets(data: bytes) -> Tuple[List[bytes], List[int]]:
    """Packets of the first logical stream, and the granule position of each page's last completed packet (-1
    for packets that do not end a page)."""
    pos, serial, cur = 0, None, b""
    packets, granules = [], []
    while pos + 27 <= len(data):
        assert data[pos:pos + 4] == b"OggS", "lost page sync"
        htype = data[pos + 5]
        granule, ser, _, crc = struct.unpack_from("<qIII", data, pos + 6)
        nseg = data[pos + 26]
        lace = data[pos + 27: pos + 27 + nseg]
        hlen = 27 + nseg
        body = sum(lace)
        page = bytearray(data[pos: pos + hlen + body])
        page[22:26] = b"\0\0\0\0"
        assert ogg_crc(bytes(page)) == crc, "page CRC"
        if serial is None:
            serial = ser
        if ser == serial:
            if not htype & 1:
                cur = b""
            p, ended = pos + hlen, False
            for L in lace:
                cur += data[p: p + L]
                p += L
                if L < 255:
                    packets.append(cur)
                    granules.append(-1)
                    cur, ended = b"", True
            if ended:
                granules[-1] = granule
        pos += hlen + body
    return packets, granules


def ogg_write(packets: List[bytes], granules: List[int], serial: int = 0x5EED) -> bytes:
    """One page per packet (header packets with granule 0), lacing per RFC 3533."""
    out = b""
    for seq, (pk, g) in enumerate(zip(packets, granules)):
        lace = [255] * (len(pk) // 255) + [len(pk) % 255]
        assert len(lace) <= 255
        htype = 2 if seq == 0 else (4 if seq == len(packets) - 1 else 0)
        hdr = b"OggS" + bytes([0, htype]) + struct.pack("<qIII", g, serial, seq, 0) + bytes([len(lace)]) + bytes(lace)
        page = bytearray(hdr + pk)
        struct.pack_into("<I", page, 22, ogg_crc(bytes(page)))
        out += bytes(page)
    return out


# ---- bits ----------------------------------------------------------------------------------------------------------------


class Bits:
    """LSB-first reader; reads past the end return zeros and set `eop`."""

    def __init__(self, b: bytes):
        self.bits = np.unpackbits(np.frombuffer(b, np.uint8), bitorder="little")
        self.p = 0
        self.eop = False

    def read(self, n: int) -> int:
        v = 0
        for i in range(n):
            if self.p >= len(self.bits):
                self.eop = True
                return 0
            v |= int(self.bits[self.p]) << i
            self.p += 1
        return v


class BitWriter:
    def __init__(self):
        self.bits: List[int] = []

    def write(self, v: int, n: int):
        for i in range(n):
            self.bits.append((v >> i) & 1)

    def bytes(self) -> bytes:
        b = self.bits + [0] * (-len(self.bits) % 8)
        return np.packbits(np.array(b, np.uint8), bitorder="little").tobytes()


def ilog(x: int) -> int:
    return x.bit_length() if x > 0 else 0


def float32_unpack(x: int) -> float:
    mant = x & 0x1FFFFF
    exp = (x & 0x7FE00000) >> 21
    return float(np.float32((-mant if x & 0x80000000 else mant) * 2.0 ** (exp - 788)))


def lookup1_values(entries: int, dims: int) -> int:
    r = 0
    while (r + 1) ** dims <= entries:
        r += 1
    return r


# ---- codebooks -------------------------------------------------------------------------------------------------------------


def assign_codewords(lengths: List[int]) -> Optional[dict]:
    """{(length, value): entry} — each used entry in order takes the leftmost free node at its depth of the code
    tree (the numerically lowest codeword that no earlier codeword prefixes or extends). None if overspecified."""
    full = {}  # (depth, value) -> True when the node's subtree is fully taken

    def taken(d, v):
        return full.get((d, v), False)

    def find(d, v, L):  # leftmost free node at depth L below node (d, v), or None
        if taken(d, v) or (d, v) in used_leaf:
            return None
        if d == L:
            return v if not has_child.get((d, v)) else None
        for b in (0, 1):
            r = find(d + 1, 2 * v + b, L)
            if r is not None:
                return r
        return None

    used_leaf, has_child, table = set(), {}, {}
    for e, L in enumerate(lengths):
        if L <= 0:
            continue
        v = find(0, 0, L)
        if v is None:
            return None
        used_leaf.add((L, v))
        table[(L, v)] = e
        full[(L, v)] = True
        d, x = L, v
        while d > 0:  # mark ancestors: they have a child; full when both children are
            d, x = d - 1, x >> 1
            has_child[(d, x)] = True
            if taken(d + 1, 2 * x) and taken(d + 1, 2 * x + 1):
                full[(d, x)] = True
    return table


class Book:
    def __init__(self, dims, lengths, vq):
        self.dims, self.lengths, self.vq = dims, lengths, vq
        self.table = assign_codewords(lengths)
        if self.table is None:
            raise ValueError("overspecified codebook")
        self.maxlen = max([L for L in lengths if L > 0], default=0)

    def decode(self, br: Bits) -> int:
        v = 0
        for L in range(1, self.maxlen + 1):
            v = (v << 1) | br.read(1)
            if br.eop:
                return -1
            e = self.table.get((L, v))
            if e is not None:
                return e
        return -1


def read_book(br: Bits) -> Book:
    assert br.read(24) == 0x564342, "codebook sync"
    dims, entries = br.read(16), br.read(24)
    lengths = [0] * entries
    if br.read(1):  # ordered
        e, L = 0, br.read(5) + 1
        while e < entries:
            num = br.read(ilog(entries - e))
            for i in range(num):
                lengths[e + i] = L
            e += num
            L += 1
    else:
        sparse = br.read(1)
        for e in range(entries):
            if sparse and not br.read(1):
                continue
            lengths[e] = br.read(5) + 1
    lookup = br.read(4)
    vq = None
    if lookup in (1, 2):
        mn, delta = np.float32(float32_unpack(br.read(32))), np.float32(float32_unpack(br.read(32)))
        vbits, seq = br.read(4) + 1, br.read(1)
        nv = lookup1_values(entries, dims) if lookup == 1 else entries * dims
        mult = [br.read(vbits) for _ in range(nv)]
        vq = np.zeros((entries, dims), np.float32)
        for e in range(entries):
            last, div = np.float32(0), 1
            for i in range(dims):
                off = (e // div) % nv if lookup == 1 else e * dims + i
                val = np.float32(np.float32(np.float32(mult[off]) * delta) + mn) + last
                vq[e, i] = val
                if seq:
                    last = val
                if lookup == 1:
                    div *= nv
    else:
        assert lookup == 0, "lookup type"
    return Book(dims, lengths, vq)


# ---- setup -------------------------------------------------------------------------------------------------------------------


def parse_headers(p0: bytes, p1: bytes, p2: bytes) -> dict:
    assert p0[:7] == b"\x01vorbis" and p1[:7] == b"\x03vorbis" and p2[:7] == b"\x05vorbis"
    br = Bits(p0[7:])
    assert br.read(32) == 0
    ch, rate = br.read(8), br.read(32)
    br.read(32), br.read(32), br.read(32)
    bs0, bs1 = 1 << br.read(4), 1 << br.read(4)
    assert br.read(1) == 1
    br = Bits(p2[7:])
    books = [read_book(br) for _ in range(br.read(8) + 1)]
    for _ in range(br.read(6) + 1):
        assert br.read(16) == 0
    floors = []
    for _ in range(br.read(6) + 1):
        assert br.read(16) == 1, "floor type 1 only"
        pc = [br.read(4) for _ in range(br.read(5))]
        cls = []
        for _c in range(max(pc, default=-1) + 1):
            cdim, csub = br.read(3) + 1, br.read(2)
            master = br.read(8) if csub else -1
            sub = [br.read(8) - 1 for _ in range(1 << csub)]
            cls.append((cdim, csub, master, sub))
        mult, rb = br.read(2) + 1, br.read(4)
        X = [0, 1 << rb]
        for c in pc:
            X += [br.read(rb) for _ in range(cls[c][0])]
        floors.append(dict(pc=pc, cls=cls, mult=mult, X=X))
    residues = []
    for _ in range(br.read(6) + 1):
        rtype, begin, end, psize, classes, cbook = br.read(16), br.read(24), br.read(24), br.read(24) + 1, \
            br.read(6) + 1, br.read(8)
        casc = []
        for _c in range(classes):
            low = br.read(3)
            casc.append((br.read(5) if br.read(1) else 0) * 8 + low)
        rbooks = [[br.read(8) if (casc[c] >> j) & 1 else -1 for j in range(8)] for c in range(classes)]
        residues.append(dict(type=rtype, begin=begin, end=end, psize=psize, classes=classes, cbook=cbook,
                             books=rbooks))
    maps = []
    for _ in range(br.read(6) + 1):
        assert br.read(16) == 0
        submaps = br.read(4) + 1 if br.read(1) else 1
        coupling = []
        if br.read(1):
            for _s in range(br.read(8) + 1):
                coupling.append((br.read(ilog(ch - 1)), br.read(ilog(ch - 1))))
        assert br.read(2) == 0
        mux = [br.read(4) for _ in range(ch)] if submaps > 1 else [0] * ch
        sm = []
        for _s in range(submaps):
            br.read(8)
            sm.append((br.read(8), br.read(8)))
        maps.append(dict(coupling=coupling, mux=mux, submaps=sm))
    modes = []
    for _ in range(br.read(6) + 1):
        flag = br.read(1)
        assert br.read(16) == 0 and br.read(16) == 0
        modes.append((flag, br.read(8)))
    assert br.read(1) == 1 and not br.eop, "setup framing"
    return dict(ch=ch, rate=rate, bs=(bs0, bs1), books=books, floors=floors, residues=residues, maps=maps,
                modes=modes)


# ---- floor 1 ---------------------------------------------------------------------------------------------------------------

_RANGES = (256, 128, 86, 64)
_INV_DB = np.array([(1.0 / 1.0649863e-07) ** ((i - 255) / 255.0) for i in range(256)], np.float32)


def _render_point(x0, y0, x1, y1, X):
    dy, adx = y1 - y0, x1 - x0
    off = abs(dy) * (X - x0) // adx
    return y0 - off if dy < 0 else y0 + off


def _render_line(x0, y0, x1, y1, v):
    dy, adx = y1 - y0, x1 - x0
    base = int(dy / adx)  # C division: toward zero
    sy = base - 1 if dy < 0 else base + 1
    ady = abs(dy) - abs(base) * adx
    y, err = y0, 0
    if x0 < len(v):
        v[x0] = y
    for x in range(x0 + 1, x1):
        err += ady
        if err >= adx:
            err -= adx
            y += sy
        else:
            y += base
        if x < len(v):
            v[x] = y


def floor1(f, books, br: Bits, n2: int):
    """The floor curve f32[n2], or None for an unused channel (including an end of packet inside the floor)."""
    if not br.read(1):
        return None
    rng = _RANGES[f["mult"] - 1]
    Y = [br.read(ilog(rng - 1)), br.read(ilog(rng - 1))]
    for c in f["pc"]:
        cdim, csub, master, sub = f["cls"][c]
        cval = 0
        if csub:
            cval = books[master].decode(br)
            if cval < 0:
                return None
        for _ in range(cdim):
            b = sub[cval & ((1 << csub) - 1)]
            cval >>= csub
            if b >= 0:
                y = books[b].decode(br)
                if y < 0:
                    return None
                Y.append(y)
            else:
                Y.append(0)
    if br.eop:
        return None
    X = f["X"]
    n = len(X)
    fy, used = list(Y[:2]), [True, True]
    for i in range(2, n):
        lo = max((j for j in range(i) if X[j] < X[i]), key=lambda j: X[j])
        hi = min((j for j in range(i) if X[j] > X[i]), key=lambda j: X[j])
        pred = _render_point(X[lo], fy[lo], X[hi], fy[hi], X[i])
        val, hroom, lroom = Y[i], rng - pred, pred
        room = 2 * min(hroom, lroom)
        if val:
            used[lo] = used[hi] = True
            used.append(True)
            if val >= room:
                fy.append(val - lroom + pred if hroom > lroom else pred - val + hroom - 1)
            else:
                fy.append(pred - (val + 1) // 2 if val & 1 else pred + val // 2)
        else:
            used.append(False)
            fy.append(pred)
        # ffmpeg's vorbis decoder (the decoder ffmpeg_read runs, $TF/pipelines/audio_utils.py:9-45) clips every final
        # post to 16 bits (av_clip_uint16); the specification leaves out-of-range posts of a malformed stream open
        fy[i] = min(max(fy[i], 0), 65535)
    v = np.zeros(n2, np.int64)
    order = sorted(range(n), key=lambda i: X[i])
    lx, ly = 0, fy[order[0]] * f["mult"]
    hx, hy = 0, ly
    for i in order[1:]:
        if used[i]:
            hx, hy = X[i], fy[i] * f["mult"]
            _render_line(lx, ly, hx, hy, v)
            lx, ly = hx, hy
    if hx < n2:
        _render_line(hx, hy, n2, hy, v)
    return _INV_DB[np.clip(v, 0, 255)]


# ---- residue -----------------------------------------------------------------------------------------------------------------


def _residue_vectors(r, books, br: Bits, size: int, vecs: List[np.ndarray], skip: List[bool], fmt: int):
    lb, le = min(r["begin"], size), min(r["end"], size)
    if le - lb <= 0:
        return
    ps, nparts = r["psize"], (le - lb) // r["psize"]
    cb = books[r["cbook"]]
    cls = [[0] * (nparts + cb.dims) for _ in vecs]
    for pas in range(8):
        pc = 0
        while pc < nparts:
            if pas == 0:
                for j in range(len(vecs)):
                    if skip[j]:
                        continue
                    t = cb.decode(br)
                    if t < 0:
                        return
                    for i in reversed(range(cb.dims)):
                        cls[j][pc + i] = t % r["classes"]
                        t //= r["classes"]
            i = 0
            while i < cb.dims and pc < nparts:
                for j in range(len(vecs)):
                    if skip[j]:
                        continue
                    b = r["books"][cls[j][pc]][pas]
                    if b < 0:
                        continue
                    book, off = books[b], lb + pc * ps
                    if fmt == 0:
                        step = ps // book.dims
                        for s in range(step):
                            e = book.decode(br)
                            if e < 0:
                                return
                            for k in range(book.dims):
                                vecs[j][off + s + k * step] += book.vq[e, k]
                    else:
                        s = 0
                        while s < ps:
                            e = book.decode(br)
                            if e < 0:
                                return
                            for k in range(book.dims):
                                if s < ps:
                                    vecs[j][off + s] += book.vq[e, k]
                                s += 1
                i += 1
                pc += 1


def residue(r, books, br: Bits, n2: int, vecs: List[np.ndarray], skip: List[bool]):
    if r["type"] != 2:
        return _residue_vectors(r, books, br, n2, vecs, skip, r["type"])
    if all(skip):
        return
    il = np.zeros(n2 * len(vecs), np.float32)
    _residue_vectors(r, books, br, n2 * len(vecs), [il], [False], 1)
    for j, v in enumerate(vecs):
        v += il[j::len(vecs)]


# ---- synthesis --------------------------------------------------------------------------------------------------------------

_MDCT = {}


def imdct(X: np.ndarray) -> np.ndarray:
    """y[i] = sum_k X[k] cos(2 pi / N (i + 1/2 + N/4)(k + 1/2)), N = 2 len(X) (float64 matrix)."""
    N = 2 * len(X)
    if N not in _MDCT:
        i = np.arange(N, dtype=np.float64)[:, None]
        k = np.arange(N // 2, dtype=np.float64)[None, :]
        _MDCT[N] = np.cos(2 * np.pi / N * (i + 0.5 + N / 4) * (k + 0.5))
    return _MDCT[N] @ X.astype(np.float64)


def window(n: int, ln: int, rn: int) -> np.ndarray:
    def slope(h):
        x = (np.arange(h) + 0.5) / h * np.pi / 2
        return np.sin(np.pi / 2 * np.sin(x) ** 2)

    w = np.zeros(n)
    ls, rs = n // 4 - ln // 2, 3 * n // 4 - rn // 2
    w[ls: ls + ln] = slope(ln)
    w[ls + ln: rs] = 1.0
    w[rs: rs + rn] = slope(rn)[::-1]
    return w


def decode(data: bytes) -> Tuple[np.ndarray, int]:
    packets, granules = ogg_packets(data)
    h = parse_headers(*packets[:3])
    ch, (bs0, bs1), books = h["ch"], h["bs"], h["books"]
    blocks = []  # (n, f64 [ch][n] windowed time data)
    for pk in packets[3:]:
        if not pk:
            continue
        br = Bits(pk)
        if br.read(1):
            continue
        mode = br.read(ilog(len(h["modes"]) - 1))
        flag, mapping = h["modes"][mode]
        n = bs1 if flag else bs0
        pf = nf = 0
        if flag:
            pf, nf = br.read(1), br.read(1)
        if br.eop:
            continue
        m = h["maps"][mapping]
        n2 = n // 2
        fl = [floor1(h["floors"][m["submaps"][m["mux"][c]][0]], books, br, n2) for c in range(ch)]
        nores = [f is None for f in fl]
        for a, b in m["coupling"]:
            if not nores[a] or not nores[b]:
                nores[a] = nores[b] = False
        res = [np.zeros(n2, np.float32) for _ in range(ch)]
        for s, (_fl, ri) in enumerate(m["submaps"]):
            idx = [c for c in range(ch) if m["mux"][c] == s]
            if idx:
                residue(h["residues"][ri], books, br, n2, [res[c] for c in idx], [nores[c] for c in idx])
        for a, b in reversed(m["coupling"]):
            M, A = res[a].copy(), res[b].copy()
            pos = M > 0
            apos = A > 0
            res[a] = np.where(pos, np.where(apos, M, M + A), np.where(apos, M, M - A)).astype(np.float32)
            res[b] = np.where(pos, np.where(apos, M - A, M), np.where(apos, M + A, M)).astype(np.float32)
        ln = bs0 // 2 if (flag and not pf) else n // 2
        rn = bs0 // 2 if (flag and not nf) else n // 2
        w = window(n, ln, rn)
        out = np.zeros((ch, n))
        for c in range(ch):
            if fl[c] is not None:
                out[c] = imdct((res[c] * fl[c]).astype(np.float32)) * w
        blocks.append((n, out))
    if len(blocks) < 2:
        return np.zeros((0, ch), np.float32), h["rate"]
    # block k's centre sits at c_k on one timeline, c_{k+1} = c_k + n_k / 4 + n_{k+1} / 4; output = [c_0, c_last)
    centres = [bs1]  # (a margin: a long block after a short one starts before the short block does)
    for (na, _), (nb, _) in zip(blocks, blocks[1:]):
        centres.append(centres[-1] + na // 4 + nb // 4)
    tl = np.zeros((ch, centres[-1] + blocks[-1][0]))
    for (n, out), c in zip(blocks, centres):
        tl[:, c - n // 2: c + n // 2] += out
    y = tl[:, centres[0]: centres[-1]].T
    ends = [g for g in granules[3:] if g >= 0]  # the last page's granule position ends the stream
    end = ends[-1] if ends else -1
    if 0 <= end < len(y):
        y = y[:end]
    return y.astype(np.float32), h["rate"]


# ---- random stream writer -------------------------------------------------------------------------------------------


def _float32_pack(x: float) -> int:
    m, e = math.frexp(abs(x))  # x = m 2^e, m in [0.5, 1)
    mant = int(round(m * (1 << 21)))
    exp = e - 21 + 788
    if mant == 1 << 21:
        mant, exp = mant >> 1, exp + 1
    return (0x80000000 if x < 0 else 0) | (exp << 21) | mant


def _random_lengths(rng, entries: int, maxlen: int = 12) -> List[int]:
    """Codeword lengths of a complete prefix code (Kraft sum 1) over `entries` leaves, shuffled."""
    leaves = [0]
    while len(leaves) < entries:
        cand = [i for i, d in enumerate(leaves) if d < maxlen]
        i = cand[rng.integers(len(cand))]
        d = leaves.pop(i)
        leaves += [d + 1, d + 1]
    rng.shuffle(leaves)
    return [max(d, 1) for d in leaves]


def _write_book(bw: BitWriter, rng, dims: int, entries: int, lookup: int, mode: str):
    if entries == 1:
        lengths = [int(rng.integers(1, 4))]
    else:
        lengths = _random_lengths(rng, entries)
        while assign_codewords(lengths) is None:
            lengths = _random_lengths(rng, entries)
    if mode == "ordered":
        lengths = sorted(lengths)
    bw.write(0x564342, 24)
    bw.write(dims, 16)
    bw.write(entries, 24)
    if mode == "ordered":
        bw.write(1, 1)
        bw.write(lengths[0] - 1, 5)
        e, L = 0, lengths[0]
        while e < entries:
            num = sum(1 for x in lengths[e:] if x == L)
            bw.write(num, ilog(entries - e))
            e += num
            L += 1
    else:
        bw.write(0, 1)
        sparse = mode == "sparse"
        bw.write(int(sparse), 1)
        for L in lengths:
            if sparse:
                bw.write(1, 1)
            bw.write(L - 1, 5)
    bw.write(lookup, 4)
    if lookup:
        bw.write(_float32_pack(-float(rng.uniform(0.2, 2.0))), 32)
        bw.write(_float32_pack(float(rng.uniform(0.01, 0.3))), 32)
        vbits = int(rng.integers(1, 6))
        bw.write(vbits - 1, 4)
        bw.write(int(rng.integers(2)), 1)
        nv = lookup1_values(entries, dims) if lookup == 1 else entries * dims
        for _ in range(nv):
            bw.write(int(rng.integers(1 << vbits)), vbits)


def write_stream(rng, channels: int = 2, bs_exp=(7, 9), n_packets: int = 12, rate: int = 22050,
                 packet_bytes=(8, 160), end_trim: int = 17) -> bytes:
    """A random but syntactically valid Ogg Vorbis stream (see the module docstring)."""
    bs = (1 << bs_exp[0], 1 << bs_exp[1])
    ident = BitWriter()
    ident.write(0, 32)
    ident.write(channels, 8)
    ident.write(rate, 32)
    for _ in range(3):
        ident.write(0, 32)
    ident.write(bs_exp[0], 4)
    ident.write(bs_exp[1], 4)
    ident.write(1, 1)
    comment = BitWriter()
    vendor = b"tw random syntax writer"
    comment.write(len(vendor), 32)
    for c in vendor:
        comment.write(c, 8)
    comment.write(0, 32)
    comment.write(1, 1)

    sb = BitWriter()
    # books: 0..3 scalar (floor masters / subbooks / classbooks), 4.. VQ books for residues
    scalar = [(1, 4), (1, 16), (1, 32), (1, 1)]
    vq_specs = [(1, 8, 1), (2, 16, 1), (4, 16, 2), (2, 9, 1), (8, 6, 2), (4, 81, 1)]
    n_books = len(scalar) + len(vq_specs) + 1
    sb.write(n_books - 1, 8)
    modes_cycle = ["dense", "sparse", "ordered"]
    for i, (d, e) in enumerate(scalar):
        _write_book(sb, rng, d, e, 0, modes_cycle[i % 3])
    for i, (d, e, lk) in enumerate(vq_specs):
        _write_book(sb, rng, d, e, lk, modes_cycle[i % 3])
    # residue classbook (dims 2 over 3 classes: 9 entries)
    cls_book = n_books - 1
    _write_book(sb, rng, 2, 9, 0, "dense")
    sb.write(0, 6)
    sb.write(0, 16)
    # floors: two floor-1 configurations
    n_floors = 2
    sb.write(n_floors - 1, 6)
    for fi in range(n_floors):
        sb.write(1, 16)
        nparts = int(rng.integers(1, 5))
        nclasses = int(rng.integers(1, 4))
        pc = [int(rng.integers(nclasses)) for _ in range(nparts)]
        pc[0] = nclasses - 1
        sb.write(nparts, 5)
        for c in pc:
            sb.write(c, 4)
        cdims = []
        for c in range(nclasses):
            cdim, csub = int(rng.integers(1, 4)), int(rng.integers(0, 3))
            cdims.append(cdim)
            sb.write(cdim - 1, 3)
            sb.write(csub, 2)
            if csub:
                sb.write(int(rng.integers(0, 3)), 8)  # master: a 4 / 16 / 32 entry scalar book
            for _ in range(1 << csub):
                sb.write(int(rng.integers(0, 4)), 8)  # subbook + 1 (0 = none)
        mult = int(rng.integers(1, 5))
        sb.write(mult - 1, 2)
        rb = bs_exp[fi] - 1  # x range = n / 2 of the block size this floor serves
        sb.write(rb, 4)
        npost = sum(cdims[c] for c in pc)
        xs = rng.choice(np.arange(1, 1 << rb), size=npost, replace=False)
        for x in xs:
            sb.write(int(x), rb)
    # residues: types 0, 1, 2
    sb.write(2, 6)
    for rtype in (0, 1, 2):
        sb.write(rtype, 16)
        full = bs[1] // 2 * (channels if rtype == 2 else 1)
        begin = int(rng.integers(0, 4)) * 8
        end = int(rng.integers(full // 2, full + 64))
        sb.write(begin, 24)
        sb.write(end, 24)
        sb.write(int(rng.choice([8, 16, 32])) - 1, 24)
        sb.write(3 - 1, 6)
        sb.write(cls_book, 8)
        casc = [int(rng.integers(0, 256)) for _ in range(3)]
        for c in casc:
            sb.write(c & 7, 3)
            sb.write(1, 1)
            sb.write(c >> 3, 5)
        for c in casc:
            for j in range(8):
                if (c >> j) & 1:
                    sb.write(len(scalar) + int(rng.integers(len(vq_specs))), 8)
    # mappings: 0 = one submap (+ coupling when stereo+), 1 = two submaps
    sb.write(1, 6)
    for mi in range(2):
        sb.write(0, 16)
        submaps = 1 if mi == 0 or channels == 1 else 2
        if submaps > 1:
            sb.write(1, 1)
            sb.write(submaps - 1, 4)
        else:
            sb.write(0, 1)
        if channels > 1:
            sb.write(1, 1)
            steps = [(0, 1)] + ([(2, 0)] if channels > 2 else [])
            sb.write(len(steps) - 1, 8)
            for a, b in steps:
                sb.write(a, ilog(channels - 1))
                sb.write(b, ilog(channels - 1))
        else:
            sb.write(0, 1)
        sb.write(0, 2)
        if submaps > 1:
            for c in range(channels):
                sb.write(c % submaps, 4)
        for s in range(submaps):
            sb.write(0, 8)
            sb.write(int(rng.integers(n_floors)), 8)
            sb.write(int(rng.integers(3)) if mi == 0 else (s + 1) % 3, 8)
    # modes: 0 short, 1 long
    sb.write(1, 6)
    for flag in (0, 1):
        sb.write(flag, 1)
        sb.write(0, 16)
        sb.write(0, 16)
        sb.write(flag, 8)  # mode 0 -> mapping 0, mode 1 -> mapping 1
    sb.write(1, 1)

    flags = [int(rng.integers(2)) for _ in range(n_packets)]
    audio = []
    for k, f in enumerate(flags):
        bw = BitWriter()
        bw.write(0, 1)
        bw.write(f, 1)  # mode number (1 bit for 2 modes)
        if f:
            bw.write(flags[k - 1] if k > 0 else 1, 1)
            bw.write(flags[k + 1] if k + 1 < n_packets else 1, 1)
        payload = np.frombuffer(rng.bytes(int(rng.integers(*packet_bytes))), np.uint8)
        bw.bits.extend(np.unpackbits(payload, bitorder="little").tolist())
        audio.append(bw.bytes())
    ns = [bs[f] for f in flags]
    total = sum(a // 4 + b // 4 for a, b in zip(ns, ns[1:]))
    heads = [b"\x01vorbis" + ident.bytes(), b"\x03vorbis" + comment.bytes(), b"\x05vorbis" + sb.bytes()]
    gran = [0, 0, 0] + [-1] * (n_packets - 1) + [max(total - end_trim, 0)]
    # one page per packet: granule of non-final audio pages = samples so far
    acc = 0
    for k in range(n_packets - 1):
        if k > 0:
            acc += ns[k - 1] // 4 + ns[k] // 4
        gran[3 + k] = acc
    return ogg_write(heads + audio, gran)
