"""Ogg Vorbis ingest, CPU side: the native decoder (csrc/vorbis.cpp in libtwhip.so) against
the oracle's independent restatement of the Vorbis I specification (oracle/vorbis_oracle.py).

Pins: the one real-encoder Vorbis stream in this image (MathJax's a11y/invalid_keypress.ogg, libVorbis I 20101101,
44.1 kHz stereo, blocksizes 256 / 2048) must decode to exactly its last page's granule length and agree with the
oracle; random-syntax streams from the oracle's writer cover what that file does not (VQ lookup type 1, residues
0 and 1, floor classes with master books, coupling over three channels, two submaps, single-entry and ordered
codebooks). Against ffmpeg's own Vorbis decoder (what the reference's ffmpeg_read runs) the samples are unpinned:
no ffmpeg or libvorbis exists in this image. Tolerance: 1e-6 of the stream's peak (float32 IMDCT / windowing in
the native decoder vs float64 in the oracle)."""
import ctypes
import os

import numpy as np
import pytest

from oracle import vorbis_oracle as vo
from twamd import _lib, audio

REAL_OGG = "/usr/local/lib/python3.10/dist-packages/kaleido/executable/etc/mathjax/extensions/a11y/invalid_keypress.ogg"
REL = 1e-6


def _close(got, ref):
    assert got.shape == ref.shape
    scale = max(float(np.abs(ref).max()), 1e-6)
    assert np.abs(got - ref).max() <= REL * scale, float(np.abs(got - ref).max() / scale)


@pytest.mark.skipif(not os.path.exists(REAL_OGG), reason="the image's MathJax Ogg file is not present")
def test_real_libvorbis_stream():
    data = open(REAL_OGG, "rb").read()
    assert audio.container_name(data) == "Ogg Vorbis"
    info = audio.vorbis_probe(data)
    assert (info.sample_rate, info.channels, info.blocksize0, info.blocksize1, info.total_samples) == \
        (44100, 2, 256, 2048, 22050)
    x, sr = audio.decode_vorbis(data)
    ref, rsr = vo.decode(data)
    assert sr == rsr == 44100 and x.shape == (22050, 2)
    _close(x, ref)
    # a short beep: both channels carry it, its energy sits at 150-170 Hz, no block-edge clicks
    assert np.corrcoef(x[:, 0], x[:, 1])[0, 1] > 0.999 and 0.3 < np.abs(x).max() < 1.0
    f = np.abs(np.fft.rfft(x[:, 0]))
    peak_hz = np.argmax(f) * 44100 / len(x)
    assert 140 < peak_hz < 180
    assert np.abs(np.diff(x[:, 0], 2)).max() < 0.05
    assert abs(audio.duration_seconds(REAL_OGG) - 0.5) < 1e-9


@pytest.mark.parametrize("seed", range(16))
def test_random_syntax_streams_match_oracle(seed):
    rng = np.random.default_rng(seed)
    ch = 1 + seed % 3
    data = vo.write_stream(rng, channels=ch, bs_exp=(6 + seed % 2, 8 + (seed // 2) % 2), n_packets=10 + seed % 5)
    x, sr = audio.decode_vorbis(data)
    ref, _ = vo.decode(data)
    assert x.shape[1] == ch and len(x) > 0
    _close(x, ref)


def test_imdct_matches_definition():
    lib = _lib.load()
    for n in (8, 64, 256, 2048):
        X = np.random.default_rng(n).standard_normal(n // 2).astype(np.float32)
        y = np.zeros(n, np.float32)
        assert lib.tw_vorbis_imdct(X.ctypes.data, n, y.ctypes.data) == 0
        ref = vo.imdct(X)
        assert np.abs(y - ref).max() < 1e-6 * np.abs(ref).max() * np.sqrt(n)
    assert lib.tw_vorbis_imdct(X.ctypes.data, 100, y.ctypes.data) != 0


def test_damaged_streams_are_errors():
    data = bytearray(vo.write_stream(np.random.default_rng(3), channels=2))
    bad = bytearray(data)
    bad[200] ^= 0x40  # inside the setup header's page: its CRC no longer matches
    with pytest.raises(ValueError, match="CRC"):
        audio.decode_vorbis(bytes(bad))
    with pytest.raises(ValueError, match="truncated"):
        audio.decode_vorbis(bytes(data[: len(data) - 7]))
    with pytest.raises(ValueError):
        audio.decode_vorbis(b"OggS" + bytes(40))


def test_ogg_container_names():
    opus = vo.ogg_write([b"OpusHead" + bytes(11)], [0])
    assert audio.container_name(opus) == "Ogg Opus"
    with pytest.raises(ValueError, match="^Ogg Opus audio is not decoded"):
        audio.load_input(opus)
    vorbis = vo.write_stream(np.random.default_rng(0), channels=1, n_packets=3)
    assert audio.container_name(vorbis) == "Ogg Vorbis"


def test_header_length_claims_are_bounded(monkeypatch):
    data = vo.write_stream(np.random.default_rng(5), channels=1, n_packets=6)
    packets, gran = vo.ogg_packets(data)
    gran[-1] = 1 << 40  # a final granule no stream of this size can reach
    with pytest.raises(ValueError, match="larger than the stream can code"):
        audio.decode_vorbis(vo.ogg_write(packets, gran))
    monkeypatch.setenv("TW_MAX_AUDIO_S", "0.001")
    with pytest.raises(ValueError, match="TW_MAX_AUDIO_S"):
        audio.decode_vorbis(data)


def test_native_entry_points_declared():
    lib = _lib.load()
    info = _lib.TwVorbisInfo()
    assert lib.tw_vorbis_probe(ctypes.c_char_p(b"nope"), 4, ctypes.byref(info)) != 0
    assert b"Ogg" in lib.tw_last_error()


def test_threads_do_not_change_the_output():
    """Packets decode in parallel rounds of 1024 (the overlap-add after each round, in order): a stream longer than
    one round gives the same samples on 1 and 3 threads, and the oracle's."""
    data = vo.write_stream(np.random.default_rng(11), channels=2, bs_exp=(6, 8), n_packets=1100, packet_bytes=(4, 40))
    x1, _ = audio.decode_vorbis(data, threads=1)
    x3, _ = audio.decode_vorbis(data, threads=3)
    assert np.array_equal(x1, x3) and len(x1) > 50000
    _close(x1, vo.decode(data)[0])


def test_hostile_codebook_sizes_are_refused():
    """A setup header claiming a 2^24 - 1-entry, 1000-dimension codebook is an error, not a multi-gigabyte
    allocation."""
    packets, gran = vo.ogg_packets(vo.write_stream(np.random.default_rng(2), channels=1, n_packets=3))
    bw = vo.BitWriter()
    bw.write(0, 8)  # one codebook
    bw.write(0x564342, 24)
    bw.write(1000, 16)
    bw.write((1 << 24) - 1, 24)
    bw.write(0, 1)  # unordered
    bw.write(0, 1)  # dense
    packets[2] = b"\x05vorbis" + bw.bytes() + bytes(64)
    with pytest.raises(ValueError, match="too large"):
        audio.decode_vorbis(vo.ogg_write(packets, gran))
