"""Telephony-codec ingest (G.711 mu-law / A-law, IMA ADPCM) and the AU / AIFF / AIFF-C containers, pinned bit-exactly
against CPython's own implementations of the same formats: audioop (ulaw2lin / alaw2lin / adpcm2lin), sunau, aifc and
wave. The reference decodes uploads with ffmpeg (transformers' ffmpeg_read, $TF/pipelines/audio_utils.py:9-45: every
codec to s16, then f32le = s16 / 32768); ffmpeg is absent here, so these stdlib decoders are the pinned restatement of
the same published formats. Host code only (libtwhip.so's tw_g711_decode / tw_ima_adpcm_wav_decode), no GPU."""
from __future__ import annotations

import audioop
import aifc
import io
import struct
import sunau
import wave

import numpy as np
import pytest

from twamd import audio

RNG = np.random.default_rng(711)


def _s16(b: bytes) -> np.ndarray:
    return np.frombuffer(b, "=i2")  # audioop works in native byte order


@pytest.mark.parametrize("alaw", [False, True])
def test_g711_all_codes_match_audioop(alaw):
    codes = bytes(range(256))
    want = _s16(audioop.alaw2lin(codes, 2) if alaw else audioop.ulaw2lin(codes, 2))
    got = audio.g711_decode(codes, alaw)
    np.testing.assert_array_equal(got, want)
    assert audio.g711_decode(b"", alaw).shape == (0,)


def _wav_bytes(tag: int, ch: int, sr: int, bits: int, align: int, payload: bytes, extensible: bool = False,
               extra_chunk: bool = True) -> bytes:
    if extensible:
        guid = struct.pack("<H", tag) + bytes.fromhex("000000001000800000aa00389b71")
        fmt = struct.pack("<HHIIHHHHI", 0xFFFE, ch, sr, sr * align, align, bits, 22, bits, 0) + guid
    else:
        fmt = struct.pack("<HHIIHH", tag, ch, sr, sr * align, align, bits)
        if tag == 0x11:
            per = 1 + ((align - 4 * ch) // (4 * ch)) * 8
            fmt += struct.pack("<HH", 2, per)
    chunks = b"fmt " + struct.pack("<I", len(fmt)) + fmt
    if extra_chunk:  # a chunk the decoder must skip, odd-sized (pad byte)
        chunks += b"LIST" + struct.pack("<I", 3) + b"abc\x00"
    chunks += b"data" + struct.pack("<I", len(payload)) + payload + (b"\x00" if len(payload) & 1 else b"")
    return b"RIFF" + struct.pack("<I", 4 + len(chunks)) + b"WAVE" + chunks


@pytest.mark.parametrize("tag,extensible", [(7, False), (6, False), (7, True), (6, True)])
@pytest.mark.parametrize("ch", [1, 2])
def test_wav_g711(tag, extensible, ch):
    n = 1001 * ch
    payload = RNG.integers(0, 256, n, dtype=np.uint8).tobytes()
    x, sr = audio.decode_wav(_wav_bytes(tag, ch, 8000, 8, ch, payload, extensible))
    lin = audioop.alaw2lin(payload, 2) if tag == 6 else audioop.ulaw2lin(payload, 2)
    want = _s16(lin).astype(np.float32).reshape(-1, ch) / 32768.0
    assert sr == 8000 and x.shape == (1001, ch)
    np.testing.assert_array_equal(x, want)


def _ima_reference(payload: bytes, ch: int, align: int) -> np.ndarray:
    """Decode Microsoft IMA ADPCM blocks with audioop.adpcm2lin: per block and channel, the header predictor is the
    first sample and (predictor, index) audioop's state; the channel's 4-byte words are gathered, and each byte's
    nibbles swapped (WAV codes the earlier sample in the low nibble, audioop in the high one)."""
    frames = []
    for pos in range(0, len(payload), align):
        blk = payload[pos: pos + align]
        if len(blk) < 4 * ch:
            break
        words = (len(blk) - 4 * ch) // (4 * ch)
        cols = []
        for c in range(ch):
            pred, idx = struct.unpack("<hB", blk[4 * c: 4 * c + 3])
            data = b"".join(blk[4 * ch + 4 * (k * ch + c): 4 * ch + 4 * (k * ch + c) + 4] for k in range(words))
            swapped = bytes(((b & 0x0F) << 4) | (b >> 4) for b in data)
            lin, _ = audioop.adpcm2lin(swapped, 2, (pred, idx))
            cols.append(np.concatenate([[pred], _s16(lin)]).astype(np.int16))
        frames.append(np.stack(cols, axis=1))
    return np.concatenate(frames) if frames else np.zeros((0, ch), np.int16)


def _ima_payload(ch: int, align: int, blocks: int, tail: int) -> bytes:
    out = bytearray()
    for b in range(blocks + (1 if tail else 0)):
        blk = bytearray(RNG.integers(0, 256, align, dtype=np.uint8).tobytes())
        for c in range(ch):
            pred = int(RNG.integers(-32768, 32768))
            idx = int(RNG.integers(0, 89)) if b else 88  # first block at the largest step: exercises the s16 clamp
            blk[4 * c: 4 * c + 4] = struct.pack("<hBB", pred, idx, 0)
        out += blk[:tail] if b == blocks else blk
    return bytes(out)


@pytest.mark.parametrize("ch,align,tail", [(1, 256, 0), (1, 512, 100), (2, 512, 0), (2, 1024, 37)])
def test_wav_ima_adpcm_matches_audioop(ch, align, tail):
    payload = _ima_payload(ch, align, 5, tail)
    x, sr = audio.decode_wav(_wav_bytes(0x11, ch, 22050, 4, align, payload))
    want = _ima_reference(payload, ch, align)
    per = 1 + ((align - 4 * ch) // (4 * ch)) * 8
    assert x.shape[0] == want.shape[0] and x.shape[0] >= 5 * per
    np.testing.assert_array_equal(x, want.astype(np.float32) / 32768.0)
    assert sr == 22050


def test_ima_adpcm_rejects_bad_step_index_and_short_block_align():
    payload = bytearray(_ima_payload(1, 256, 1, 0))
    payload[2] = 89
    with pytest.raises(ValueError, match="step index"):
        audio.decode_wav(_wav_bytes(0x11, 1, 8000, 4, 256, bytes(payload)))
    with pytest.raises(ValueError, match="block_align"):
        audio.ima_adpcm_wav_decode(bytes(64), 2, 4)


@pytest.mark.parametrize("bits", [8, 16, 24, 32])
@pytest.mark.parametrize("ch", [1, 2])
def test_wav_pcm_matches_wave_module(bits, ch):
    buf = io.BytesIO()
    frames = RNG.integers(0, 256, 333 * ch * bits // 8, dtype=np.uint8).tobytes()
    with wave.open(buf, "wb") as w:
        w.setnchannels(ch)
        w.setsampwidth(bits // 8)
        w.setframerate(16000)
        w.writeframes(frames)
    x, sr = audio.decode_wav(buf.getvalue())
    with wave.open(io.BytesIO(buf.getvalue()), "rb") as r:
        raw = r.readframes(r.getnframes())
    if bits == 8:  # WAV 8-bit is unsigned
        want = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128) / 128
    else:
        want = np.frombuffer(audioop.lin2lin(raw, bits // 8, 4), "<i4").astype(np.float64) / 2.0 ** 31
    assert sr == 16000
    np.testing.assert_array_equal(x, want.astype(np.float32).reshape(-1, ch))


def _au(writer_setup, frames: bytes) -> bytes:
    buf = io.BytesIO()
    w = sunau.open(buf, "wb")
    writer_setup(w)
    w.writeframes(frames)
    w._patchheader() if hasattr(w, "_patchheader") else None
    data = buf.getvalue()
    w._file = None  # the stream stays open: sunau would close the BytesIO
    return data


@pytest.mark.parametrize("kind", ["ulaw", "pcm8", "pcm16", "pcm24", "pcm32"])
@pytest.mark.parametrize("ch", [1, 2])
def test_au_matches_sunau(kind, ch):
    width = {"ulaw": 2, "pcm8": 1, "pcm16": 2, "pcm24": 3, "pcm32": 4}[kind]
    lin = RNG.integers(0, 256, 257 * ch * width, dtype=np.uint8).tobytes()

    def setup(w):
        w.setnchannels(ch)
        w.setsampwidth(width)
        w.setframerate(8000)
        w.setcomptype("ULAW" if kind == "ulaw" else "NONE", "")  # sunau's writer defaults to ULAW

    data = _au(setup, lin)
    x, sr = audio.decode_au(data)
    r = sunau.open(io.BytesIO(data), "rb")
    raw = r.readframes(r.getnframes())  # sunau expands mu-law with audioop.ulaw2lin; PCM stays big-endian
    if kind == "ulaw":
        want = _s16(raw).astype(np.float64) / 32768.0
        assert struct.unpack(">I", data[12:16])[0] == 1
    else:
        want = np.frombuffer(audioop.lin2lin(audioop.byteswap(raw, width), width, 4), "<i4") / 2.0 ** 31
    assert sr == 8000 and r.getnchannels() == ch
    np.testing.assert_array_equal(x, want.astype(np.float32).reshape(-1, ch))


def test_au_alaw_and_float_and_unknown_size():
    codes = RNG.integers(0, 256, 400, dtype=np.uint8).tobytes()
    hdr = b".snd" + struct.pack(">IIIII", 32, 0xFFFFFFFF, 27, 8000, 1) + b"\x00" * 8  # data size "unknown"
    x, _ = audio.decode_au(hdr + codes)
    np.testing.assert_array_equal(x[:, 0], _s16(audioop.alaw2lin(codes, 2)).astype(np.float32) / 32768.0)
    f = RNG.standard_normal(300).astype(">f4")
    x, _ = audio.decode_au(b".snd" + struct.pack(">IIIII", 24, 1200, 6, 16000, 2) + f.tobytes())
    np.testing.assert_array_equal(x, f.astype(np.float32).reshape(-1, 2))
    with pytest.raises(ValueError, match="unsupported .au encoding 23"):
        audio.decode_au(b".snd" + struct.pack(">IIIII", 24, 4, 23, 8000, 1) + bytes(4))


def _aiff(comptype: bytes, ch: int, width: int, frames: bytes, aifc_form: bool = True) -> bytes:
    """aifc's writer; 'sowt' (which CPython 3.10's aifc neither writes nor reads) by rewriting a NONE file:
    compression type in COMM, little-endian SSND samples."""
    buf = io.BytesIO()
    w = aifc.open(buf, "wb")
    if not aifc_form:
        w.aiff()
    w.setnchannels(ch)
    w.setsampwidth(width)
    w.setframerate(11025)
    if comptype not in (b"NONE", b"sowt"):
        w.setcomptype(comptype, b"")
    w.writeframes(frames)
    w._patchheader()
    data = buf.getvalue()
    w._file = None
    if comptype == b"sowt":
        i = data.index(b"SSND") + 16
        n = len(frames)
        data = data.replace(b"NONE", b"sowt", 1)
        data = data[:i] + audioop.byteswap(data[i: i + n], width) + data[i + n:]
    return data


@pytest.mark.parametrize("comptype,width,aifc_form", [(b"NONE", 2, False), (b"NONE", 3, False), (b"NONE", 1, True),
                                                      (b"NONE", 4, True), (b"sowt", 2, True), (b"sowt", 3, True),
                                                      (b"ulaw", 2, True), (b"alaw", 2, True)])
@pytest.mark.parametrize("ch", [1, 2])
def test_aiff_matches_aifc(comptype, width, aifc_form, ch):
    lin = RNG.integers(0, 256, 201 * ch * width, dtype=np.uint8).tobytes()
    data = _aiff(comptype, ch, width, lin, aifc_form)
    assert data[8:12] == (b"AIFC" if aifc_form else b"AIFF")
    x, sr = audio.decode_aiff(data)
    # sowt is checked against aifc's reading of the same samples as a big-endian NONE file
    r = aifc.open(io.BytesIO(_aiff(b"NONE", ch, width, lin) if comptype == b"sowt" else data), "rb")
    assert r.getcomptype() == (b"NONE" if comptype == b"sowt" else comptype)
    raw, sw = r.readframes(r.getnframes()), r.getsampwidth()
    if comptype in (b"ulaw", b"alaw"):  # aifc expands G.711 with audioop: native-endian s16
        want = _s16(raw).astype(np.float64) / 32768.0
    else:  # big-endian linear PCM (sowt byteswapped back)
        want = np.frombuffer(audioop.lin2lin(audioop.byteswap(raw, sw), sw, 4), "<i4") / 2.0 ** 31
    assert sr == 11025 and x.shape == (r.getnframes(), ch)
    np.testing.assert_array_equal(x, want.astype(np.float32).reshape(-1, ch))


@pytest.mark.parametrize("ctype,width", [(b"in24", 3), (b"in32", 4), (b"raw ", 1)])
def test_aifc_in24_in32_raw_equal_their_none_twins(ctype, width):
    """in24 / in32 are big-endian s24 / s32 under their own compression types, 'raw ' is unsigned 8-bit (ffmpeg's
    aiff tags): each decodes to the samples of the NONE file it was rewritten from."""
    lin = RNG.integers(0, 256, 301 * 2 * width, dtype=np.uint8).tobytes()
    none = _aiff(b"NONE", 2, width, lin)
    data = none.replace(b"NONE", ctype, 1)
    if ctype == b"raw ":
        i = data.index(b"SSND") + 16
        data = data[:i] + bytes(b ^ 0x80 for b in data[i: i + len(lin)]) + data[i + len(lin):]
    x, sr = audio.decode_aiff(data)
    y, _ = audio.decode_aiff(none)
    assert x.shape == (301, 2)
    np.testing.assert_array_equal(x, y)


def test_aiff_float_and_extended_rates():
    for rate in (8000, 11025, 22050, 44100, 48000, 96000):
        ext = aifc._write_float  # noqa: SLF001 - the stdlib's own 80-bit writer pins the reader
        b = io.BytesIO()
        ext(b, float(rate))
        assert audio._ieee_extended(b.getvalue()) == rate
    f = RNG.standard_normal(64).astype(">f4")
    b = io.BytesIO()
    aifc._write_float(b, 16000.0)
    comm = struct.pack(">hIh", 1, 64, 32) + b.getvalue() + b"fl32" + b"\x00"
    ssnd = struct.pack(">II", 0, 0) + f.tobytes()
    body = b"AIFC" + b"COMM" + struct.pack(">I", len(comm)) + comm + b"\x00" + b"SSND" + struct.pack(">I", len(ssnd)) + ssnd
    x, sr = audio.decode_aiff(b"FORM" + struct.pack(">I", len(body)) + body)
    assert sr == 16000
    np.testing.assert_array_equal(x[:, 0], f.astype(np.float32))


def test_containers_are_recognised_and_dispatched():
    au = b".snd" + struct.pack(">IIIII", 24, 8, 3, 16000, 1) + struct.pack(">4h", 0, 16384, -16384, 32767)
    assert audio.container_name(au) == "AU"
    np.testing.assert_array_equal(audio.decode_bytes(au), np.array([0, 0.5, -0.5, 32767 / 32768], np.float32))
    aif = _aiff(b"ulaw", 1, 2, bytes(32), aifc_form=True)
    assert audio.container_name(aif) == "AIFF"
    wav = _wav_bytes(7, 2, 16000, 8, 2, bytes([0xFF, 0x7F] * 10))
    x = audio.decode_bytes(wav)
    mono = (_s16(audioop.ulaw2lin(bytes([0xFF, 0x7F]), 2)).astype(np.float32) / 32768.0).reshape(1, 2)
    np.testing.assert_array_equal(x, np.repeat(mono.mean(axis=1, dtype=np.float32), 10))
    with pytest.raises(ValueError, match="unsupported WAVE format tag 49"):  # GSM 6.10
        audio.decode_wav(_wav_bytes(49, 1, 8000, 0, 65, bytes(65)))


def test_duration_of_telephony_files(tmp_path):
    p = tmp_path / "call.wav"
    p.write_bytes(_wav_bytes(0x11, 1, 8000, 4, 256, _ima_payload(1, 256, 4, 0)))
    assert audio.duration_seconds(str(p)) == pytest.approx(4 * 505 / 8000)
    p = tmp_path / "call.au"
    p.write_bytes(b".snd" + struct.pack(">IIIII", 24, 8000, 1, 8000, 1) + bytes(8000))
    assert audio.duration_seconds(str(p)) == 1.0
