"""More of what ffmpeg's wav / aiff demuxers hand the reference's ffmpeg_read ($TF/pipelines/audio_utils.py:9-45):
Microsoft ADPCM (WAV tag 2), MPEG audio in a WAV wrapper (tags 0x55 MP3, 0x50 MPEG Layer I / II) and Apple IMA4
(AIFF-C 'ima4'). Host code only (libtwhip.so's tw_ms_adpcm_wav_decode / tw_ima_qt_decode; the MPEG decoder of
tests/test_audio_mp3.py).

Pins: IMA4 bit-exactly against CPython's audioop.adpcm2lin (the IMA/DVI nibble decoder) under ffmpeg's
packet-boundary state rule; MS ADPCM bit-exactly against the oracle's per-nibble restatement
(oracle/audio_oracle.py, "parity unpinned vs ffmpeg": no MS ADPCM decoder or file exists in this image) and by the
round trip of its greedy encoder (a wrong sign, order or coefficient scale breaks the reconstruction); MPEG-in-WAV
equals the bare stream's decode."""
from __future__ import annotations

import audioop
import struct

import numpy as np
import pytest

from oracle import audio_oracle as ao
from oracle import mp3_oracle as mo
from twamd import audio


def _wav(tag: int, ch: int, sr: int, bits: int, align: int, payload: bytes, fmt_extra: bytes = b"") -> bytes:
    fmt = struct.pack("<HHIIHH", tag, ch, sr, sr * align, align, bits) + fmt_extra
    chunks = b"fmt " + struct.pack("<I", len(fmt)) + fmt
    chunks += b"data" + struct.pack("<I", len(payload)) + payload + (b"\x00" if len(payload) & 1 else b"")
    return b"RIFF" + struct.pack("<I", 4 + len(chunks)) + b"WAVE" + chunks


def _ms_fmt_extra(ch: int, align: int) -> bytes:
    per = (align - 6 * ch) * 2 // ch
    coefs = b"".join(struct.pack("<hh", a, b) for a, b in ao.MS_COEF)
    return struct.pack("<HHH", 4 + len(coefs), per, 7) + coefs


def _tone(n, ch, sr, amp=12000.0, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / sr
    x = np.stack([amp * np.sin(2 * np.pi * (330 + 110 * c) * t) + 300 * rng.standard_normal(n) for c in range(ch)], 1)
    return np.clip(np.round(x), -32768, 32767).astype(np.int16)


@pytest.mark.parametrize("ch,align,n", [(1, 256, 2000), (2, 512, 1500), (1, 1024, 777), (2, 256, 901)])
def test_ms_adpcm_matches_oracle_and_round_trips(ch, align, n):
    x = _tone(n, ch, 22050, seed=ch * align)
    payload = ao.ms_adpcm_encode(x, ch, align, np.random.default_rng(align))
    got, sr = audio.decode_wav(_wav(2, ch, 22050, 4, align, payload, _ms_fmt_extra(ch, align)))
    want = ao.ms_adpcm_decode(payload, ch, align)
    assert sr == 22050 and got.shape == want.shape and len(got) >= n
    np.testing.assert_array_equal(got, want.astype(np.float32) / 32768.0)
    # the round trip: 4 bits per sample of a tone + noise, every predictor pair in use
    err = want[:n].astype(np.float64) - x
    snr = 10 * np.log10((x.astype(np.float64) ** 2).mean() / (err ** 2).mean())
    assert snr > 20, snr


def test_ms_adpcm_clamp_floor_and_bad_predictor_block():
    """Full-scale square waves drive the s16 clamp and large deltas; silence drives the delta floor of 16; a block
    naming predictor 7 is dropped (ffmpeg drops the packet it cannot decode) and the rest decode."""
    n = 1200
    sq = np.where((np.arange(n) // 37) % 2, 32767, -32768).astype(np.int16)[:, None]
    x = np.concatenate([sq, np.zeros((n, 1), np.int16)])
    align = 256
    payload = bytearray(ao.ms_adpcm_encode(x, 1, align, np.random.default_rng(1), predictors=[1]))
    want_all = ao.ms_adpcm_decode(bytes(payload), 1, align)
    assert want_all.max() == 32767 and want_all.min() == -32768
    payload[2 * align] = 7
    got, _ = audio.decode_wav(_wav(2, 1, 8000, 4, align, bytes(payload), _ms_fmt_extra(1, align)))
    want = ao.ms_adpcm_decode(bytes(payload), 1, align)
    per = (align - 6) * 2
    assert len(want) == len(want_all) - per
    np.testing.assert_array_equal(got, want.astype(np.float32) / 32768.0)
    with pytest.raises(ValueError, match="MS ADPCM"):
        audio.ms_adpcm_wav_decode(bytes(64), 3, 64)


def _qt_reference(payload: bytes, ch: int) -> np.ndarray:
    """IMA4 with audioop.adpcm2lin: per packet and channel the state is audioop's running (valprev, index) when the
    header's step index equals it and its predictor is within 0x7f, else the header's; nibbles swapped (IMA4 codes
    the earlier sample in the low nibble, audioop in the high one)."""
    state = [(0, 0)] * ch
    cols = [[] for _ in range(ch)]
    for pos in range(0, len(payload) - 34 * ch + 1, 34 * ch):
        for c in range(ch):
            pk = payload[pos + 34 * c: pos + 34 * c + 34]
            hdr = struct.unpack(">h", pk[:2])[0]
            si, hp = hdr & 0x7F, hdr & ~0x7F
            pred, idx = state[c]
            if not (idx == si and abs(hp - pred) <= 0x7F):
                pred, idx = hp, si
            swapped = bytes(((b & 15) << 4) | (b >> 4) for b in pk[2:])
            lin, state[c] = audioop.adpcm2lin(swapped, 2, (pred, idx))
            cols[c].append(np.frombuffer(lin, "=i2"))
    return np.stack([np.concatenate(c) for c in cols], axis=1)


def _qt_payload(ch: int, packets: int, rng) -> bytes:
    """Random packets; every third header restates the running state (so ffmpeg carries it over), the others reset
    it to a random predictor / step index."""
    out = bytearray()
    state = [(0, 0)] * ch
    for k in range(packets):
        for c in range(ch):
            body = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
            if k % 3 == 2:
                pred, idx = state[c]
                hdr = (pred & ~0x7F) | idx
            else:
                pred, idx = int(rng.integers(-32768, 32768)) & ~0x7F, int(rng.integers(0, 89))
                hdr = pred | idx
            out += struct.pack(">h", hdr) + body
            # the running state after this packet, as the decoder will have it
            if not (state[c][1] == (hdr & 0x7F) and abs((hdr & ~0x7F) - state[c][0]) <= 0x7F):
                state[c] = (hdr & ~0x7F, hdr & 0x7F)
            swapped = bytes(((b & 15) << 4) | (b >> 4) for b in body)
            _, state[c] = audioop.adpcm2lin(swapped, 2, state[c])
    return bytes(out)


def _aifc(ch: int, sr: int, ctype: bytes, ssnd: bytes, nframes: int) -> bytes:
    ext = struct.pack(">H", 16383 + 15) + struct.pack(">Q", int(sr) << (63 - 15)) if sr < 65536 else None
    comm = struct.pack(">hIh", ch, nframes, 16) + ext + ctype + b"\x00\x00"
    ch_ = b"COMM" + struct.pack(">I", len(comm)) + comm
    ch_ += b"SSND" + struct.pack(">I", 8 + len(ssnd)) + struct.pack(">II", 0, 0) + ssnd
    return b"FORM" + struct.pack(">I", 4 + len(ch_)) + b"AIFC" + ch_


@pytest.mark.parametrize("ch", [1, 2])
def test_aifc_ima4_matches_audioop(ch):
    rng = np.random.default_rng(40 + ch)
    payload = _qt_payload(ch, 9, rng) + bytes(5)  # a partial trailing packet is not decoded
    data = _aifc(ch, 16000, b"ima4", payload, 9)
    assert audio.container_name(data) == "AIFF"
    got, sr = audio.decode_aiff(data)
    want = _qt_reference(payload, ch)
    assert sr == 16000 and got.shape == (9 * 64, ch) == want.shape
    np.testing.assert_array_equal(got, want.astype(np.float32) / 32768.0)
    # 16 kHz: no resampler, load_input is the channel mean
    np.testing.assert_array_equal(audio.load_input(data), got.mean(axis=1, dtype=np.float32))


def test_ima4_rejects_bad_step_index():
    bad = struct.pack(">h", 89) + bytes(32)
    with pytest.raises(ValueError, match="step index"):
        audio.ima_qt_decode(bad, 1)


@pytest.mark.parametrize("tag,layer", [(0x55, 3), (0x50, 2), (0x50, 1)])
def test_mpeg_audio_in_wav_equals_the_bare_stream(tag, layer):
    rng = np.random.default_rng(tag + layer)
    if layer == 3:
        stream = mo.write_stream(rng, version=1, sr_sub=0, mode=1, nframes=5)
    else:
        stream = mo.write_stream_l12(rng, layer=layer, version=1, sr_sub=1, mode=1, bri=12, nframes=5)
    h = mo.parse_header(stream[:4])
    data = _wav(tag, h["channels"], h["sample_rate"], 0, 1, stream)
    assert audio.container_name(data) == "WAV"
    got, sr = audio.decode_wav(data)
    want, wsr = audio.decode_mp3(stream)
    assert sr == wsr == h["sample_rate"]
    np.testing.assert_array_equal(got, want)
