"""Native audio ingest, CPU side: the FLAC decoder in libtwhip.so (host code) and the
resampler's filter design. The GPU resampler is tested in tests/test_gpu_audio.py.

Pins: the reference's own example file (examples/Test1/ChrisAndAlexDiTest.flac, libFLAC 1.4.2, 192 kHz 16-bit
mono) must decode to PCM whose MD5 equals its STREAMINFO MD5 (runs where /root/reference exists); streams from
the oracle's FLAC writer (oracle/audio_oracle.py) cover every subframe type, stereo mode, bit depth and blocking
strategy and must round-trip exactly."""
import os
import re

import numpy as np
import pytest

from oracle import audio_oracle as ao
from twamd import audio
from twamd.synth_audio import speech_like

REF_FLAC = "/root/reference/examples/Test1/ChrisAndAlexDiTest.flac"


def _pcm(n, ch, bps, seed):
    """Speech-like integer PCM with some structure (LPC has something to predict) and full-scale peaks."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 16000.0
    cols = []
    for c in range(ch):
        x = 0.6 * speech_like(n / 16000.0 + 0.01, seed + c)[:n] + 0.05 * rng.standard_normal(n)
        x += 0.2 * np.sin(2 * np.pi * (220 + 30 * c) * t)
        cols.append(x)
    x = np.clip(np.stack(cols, 1), -1, 1)
    lim = (1 << (bps - 1)) - 1
    return np.round(x * lim).astype(np.int32)


def _roundtrip(pcm, bps, threads=1, **kw):
    data = ao.flac_encode(pcm, 44100, bps, **kw)
    fl = audio.decode_flac(data, threads=threads)
    np.testing.assert_array_equal(fl.pcm, pcm.reshape(len(pcm), -1))
    assert audio.pcm_md5(fl.pcm, bps) == fl.md5
    return data


@pytest.mark.skipif(not os.path.exists(REF_FLAC), reason="reference example not present")
@pytest.mark.parametrize("threads", [1, 4])
def test_reference_example_md5(threads):
    data = open(REF_FLAC, "rb").read()
    fl = audio.decode_flac(data, threads=threads)
    assert (fl.sample_rate, fl.bits_per_sample, fl.pcm.shape) == (192000, 16, (3788416, 1))
    assert audio.pcm_md5(fl.pcm, 16) == fl.md5 == bytes.fromhex("ad59c8238990b312513c3de75bda098e")
    assert abs(audio.duration_seconds(REF_FLAC) - 19.731333) < 1e-5  # output.json's last timestamp is 19.74


@pytest.mark.parametrize("kind", ["verbatim", "constant", "fixed0", "fixed1", "fixed2", "fixed3", "fixed4",
                                  "lpc1", "lpc8", "lpc12", "lpc32"])
def test_subframe_kinds_mono16(kind):
    pcm = _pcm(5000, 1, 16, 3)
    if kind == "constant":
        pcm[:] = -1234
    _roundtrip(pcm, 16, blocksizes=(1152,), subframe_kinds=(kind,))


@pytest.mark.parametrize("mode", [0, 8, 9, 10])
@pytest.mark.parametrize("bps", [16, 24])
def test_stereo_decorrelation(mode, bps):
    _roundtrip(_pcm(6000, 2, bps, 5), bps, blocksizes=(2048,), subframe_kinds=("lpc10", "fixed2"),
               stereo_modes=(mode,))


@pytest.mark.parametrize("bps", [8, 12, 20])
def test_bit_depths(bps):
    _roundtrip(_pcm(3000, 1, bps, 7), bps, blocksizes=(576,), subframe_kinds=("lpc6", "fixed3", "verbatim"))


def test_multichannel_wasted_bits_and_escapes():
    pcm = _pcm(4000, 3, 16, 9) & ~7  # three trailing zero bits in every sample -> wasted-bits subframes
    _roundtrip(pcm, 16, blocksizes=(1024,), subframe_kinds=("lpc4", "fixed1", "verbatim"),
               opts={"escape_parts": (1, 3), "porder": 3})
    _roundtrip(_pcm(3000, 1, 16, 10), 16, blocksizes=(1000,), subframe_kinds=("fixed2",),
               opts={"rice_method": 1, "porder": 0})


def test_variable_blocking_and_odd_sizes():
    _roundtrip(_pcm(9000, 2, 16, 11), 16, blocksizes=(4096, 192, 1000, 256, 333), subframe_kinds=("lpc8",),
               stereo_modes=(10, 8, 0, 9), variable=True)
    _roundtrip(_pcm(70, 1, 16, 12), 16, blocksizes=(4096,), subframe_kinds=("lpc8",))  # one short frame


def test_threaded_decode_matches_sequential():
    pcm = _pcm(16000 * 24, 2, 16, 13)
    data = ao.flac_encode(pcm, 48000, 16, blocksizes=(4096,), subframe_kinds=("verbatim",), stereo_modes=(0, 10))
    assert len(data) > 4 * 256 * 1024  # large enough for the decoder to split it
    a = audio.decode_flac(data, threads=1).pcm
    b = audio.decode_flac(data, threads=8).pcm
    np.testing.assert_array_equal(a, pcm)
    np.testing.assert_array_equal(b, pcm)


def test_damaged_and_truncated_streams_raise():
    pcm = _pcm(8000, 1, 16, 14)
    data = bytearray(ao.flac_encode(pcm, 16000, 16, blocksizes=(1024,), subframe_kinds=("lpc8",)))
    bad = bytearray(data)
    bad[len(bad) // 2] ^= 0x10
    with pytest.raises(ValueError, match="corrupt|decoded"):
        audio.decode_flac(bytes(bad))
    with pytest.raises(ValueError):
        audio.decode_flac(bytes(data[: len(data) - 300]))
    with pytest.raises(ValueError, match="not a FLAC"):
        audio.decode_flac(b"RIFF" + bytes(60))


def _frames(pcm, bs, **kw):
    """(header bytes, [frame bytes]) of a fixed-blocksize stream: frame k ends where the stream of the first k
    blocks ends (the writer numbers and codes frames independently of what follows)."""
    full = ao.flac_encode(pcm, 16000, 16, blocksizes=(bs,), **kw)
    a0 = int(audio.flac_probe(full).audio_offset)
    ends = [len(ao.flac_encode(pcm[: bs * k], 16000, 16, blocksizes=(bs,), **kw)) for k in range(1, len(pcm) // bs + 1)]
    starts = [a0] + ends[:-1]
    frames = [full[s:e] for s, e in zip(starts, ends)]
    assert b"".join(frames) == full[a0:]
    return full[:a0], frames


@pytest.mark.parametrize("threads", [1, 4])
def test_skipped_or_repeated_frames_raise(threads):
    """frames [0, 2, 3, 3] still reach the STREAMINFO sample count; samples 1024..2047 would be left
    unwritten. The decoder requires the frames to tile [0, total) and the output buffer starts zeroed."""
    pcm = _pcm(4 * 1024, 1, 16, 15)
    hdr, fr = _frames(pcm, 1024, subframe_kinds=("fixed2",))
    assert np.array_equal(audio.decode_flac(hdr + b"".join(fr), threads=threads).pcm, pcm)
    for order in ([0, 2, 3, 3], [0, 1, 1, 3], [1, 0, 2, 3]):
        with pytest.raises(ValueError, match="contiguous|missing|repeated|decoded"):
            audio.decode_flac(hdr + b"".join(fr[i] for i in order), threads=threads)


def test_oversized_header_rejected_before_allocation():
    """A STREAMINFO total of 2^36 - 1 samples on a few-kB stream is refused before anything is allocated."""
    pcm = _pcm(2048, 1, 16, 16)
    data = bytearray(ao.flac_encode(pcm, 16000, 16, blocksizes=(1024,), subframe_kinds=("fixed2",)))
    # STREAMINFO: 4 (fLaC) + 4 (block header) + 13 bytes in: low 4 bits of byte 13 and bytes 14..17 = total samples
    data[8 + 13] |= 0x0F
    data[8 + 14: 8 + 18] = b"\xff\xff\xff\xff"
    assert int(audio.flac_probe(bytes(data)).total_samples) == (1 << 36) - 1
    with pytest.raises(ValueError, match="larger than"):
        audio.decode_flac(bytes(data))


@pytest.mark.parametrize("rates", [(192000, 16000), (44100, 16000), (48000, 16000), (8000, 16000),
                                   (22050, 16000), (16000, 16000)])
def test_filter_bank_matches_oracle_design(rates):
    up, down, taps = audio.swr_filter_bank(*rates)
    if rates[0] == rates[1]:
        assert (up, down, taps.tolist()) == (1, 1, [[1.0]])
        return
    ou, od, ob = ao.swr_taps(*rates)
    assert (up, down) == (ou, od) and taps.shape == ob.shape
    np.testing.assert_allclose(taps, ob, rtol=0, atol=2e-7)
    if rates == (192000, 16000):
        assert taps.shape == (1, 396)  # ceil(32 / (0.97 / 12))


def test_flac_needs_gpu_to_resample_on_cpu():
    """No CPU resampler in the product: FLAC (decoded on the host) still resamples on the GPU."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    data = ao.flac_encode(_pcm(4000, 1, 16, 15), 44100, 16, blocksizes=(1024,))
    with pytest.raises(RuntimeError, match="GPU"):
        audio.load_input(data)


def test_constant_subframe_stream_over_duration_cap(monkeypatch):
    """constant subframes code 4096 samples in a few bytes, so a small valid stream can claim hours; the
    claimed length is checked against TW_MAX_AUDIO_S x sample_rate (from STREAMINFO) before anything is allocated."""
    pcm = np.full((4096 * 64, 1), 7, np.int32)
    data = ao.flac_encode(pcm, 16000, 16, blocksizes=(4096,), subframe_kinds=("constant",))
    assert len(data) < 4096  # ~16 s of audio in a few hundred bytes
    assert np.array_equal(audio.decode_flac(data).pcm, pcm)
    monkeypatch.setenv("TW_MAX_AUDIO_S", "10")
    with pytest.raises(ValueError, match="TW_MAX_AUDIO_S=10"):
        audio.decode_flac(data)


def test_undecoded_containers_named_and_garbage_reported_as_reference():
    """Ogg Opus (and Ogg of another codec) and WebM uploads are refused by name; bytes no container matches get the
    reference's own decode-failure message (transformers' ffmpeg_read), which its transcribe() returns as
    {"error": ...}. (MPEG audio of every layer and AAC / M4A are decoded: tests/test_audio_mp3.py,
    tests/test_audio_mpeg_l12.py, tests/test_audio_aac.py.)"""
    cases = {b"OggS\x00\x02" + bytes(22) + b"OpusHead" + bytes(32): "Ogg Opus", b"OggS\x00\x02" + bytes(64): "Ogg",
             b"\x1aE\xdf\xa3" + bytes(64): "Matroska/WebM"}
    for data, name in cases.items():
        assert audio.container_name(data) == name
        with pytest.raises(ValueError, match=f"^{re.escape(name)} audio is not decoded"):
            audio.load_input(data)
    # a lone Layer I / II header (no frame the next header confirms): named, refused by the decoder's frame search
    for data, name in ((b"\xff\xfd\x90\x00" + bytes(64), "MPEG audio Layer II"),
                       (b"\xff\xff\x90\x00" + bytes(64), "MPEG audio Layer I")):
        assert audio.container_name(data) == name
        with pytest.raises(ValueError, match="no MPEG audio frame"):
            audio.load_input(data)
    # an ID3 tag before ADTS frames names AAC; an MP4 without a moov box is refused by the demuxer
    assert audio.container_name(b"ID3\x04\x00\x00\x00\x00\x00\x04" + bytes(4) + b"\xff\xf1\x50\x80" + bytes(64)) == \
        "AAC (ADTS)"
    with pytest.raises(ValueError, match="no moov"):
        audio.load_input(b"\x00\x00\x00\x20ftypM4A " + bytes(64))
    # an ID3 tag over bytes holding no MPEG audio frame: named MP3, refused by the decoder's frame search
    assert audio.container_name(b"ID3\x04\x00" + bytes(64)) == "MP3"
    with pytest.raises(ValueError, match="no MPEG audio frame"):
        audio.load_input(b"ID3\x04\x00" + bytes(64))
    with pytest.raises(ValueError) as e:
        audio.load_input(b"hello, not audio" * 8)
    assert str(e.value) == audio.MALFORMED and str(e.value).startswith("Soundfile is either not in the correct format")
