"""MP3 (MPEG-1 / MPEG-2 LSF / MPEG-2.5 Layer III) ingest, CPU side: the native decoder
(csrc/mp3.cpp in libtwhip.so) against the oracle's float64 restatement of ISO/IEC 11172-3 / 13818-3
(oracle/mp3_oracle.py).

Pins, in the absence of ffmpeg (what the reference's ffmpeg_read runs; $TF/pipelines/audio_utils.py:9-45) — the
samples are "parity unpinned vs ffmpeg":
* the standard's tables (csrc/mp3_tables.h): every Huffman table a complete prefix code, band tables summing to
  576 / 192 lines, a smooth synthesis window whose analysis / synthesis pair reconstructs;
* the image's one real MP3 (MathJax's a11y/invalid_keypress.mp3, Lavf56 / libmp3lame, MPEG-1 128 kb/s 44.1 kHz joint
  stereo, 21 audio frames after an Info frame with a LAME tag of delay 576, padding 0): every granule's Huffman data
  ends exactly at its part2_3_length, the output has the 21 x 1152 - (576 + 529) = 23087 samples ffmpeg's gapless
  trim implies, and it matches the Vorbis encoding of the same sound (invalid_keypress.ogg, decoded by the native
  Vorbis decoder) at lag 0 with correlation >= 0.95 (measured 0.99999998; the MP3 encode is 0.950 x the Vorbis
  level, a constant gain);
* random-syntax streams from the oracle's writer (every version, sample rate, channel mode, block type, table,
  scalefactor partition, the reservoir, CRC words, ID3v2 / Info + LAME frames) against the oracle.
Tolerance: 1e-6 of the stream's peak (float32 IMDCT / synthesis in the native decoder vs float64 in the oracle)."""
import ctypes
import os

import numpy as np
import pytest

from oracle import mp3_oracle as mo
from twamd import _lib, audio

A11Y = "/usr/local/lib/python3.10/dist-packages/kaleido/executable/etc/mathjax/extensions/a11y/"
REAL_MP3, REAL_OGG = A11Y + "invalid_keypress.mp3", A11Y + "invalid_keypress.ogg"
REL = 1e-6
real = pytest.mark.skipif(not os.path.exists(REAL_MP3), reason="the image's MathJax MP3 file is not present")


def _close(got, ref):
    assert got.shape == ref.shape
    scale = max(float(np.abs(ref).max()), 1e-30)
    assert np.abs(got - ref).max() <= REL * scale, float(np.abs(got - ref).max() / scale)


def test_tables_are_structurally_sound():
    checks = mo.table_checks()
    assert all(checks.values()), {k: v for k, v in checks.items() if not v}


def test_synthesis_window_reconstructs():
    """The window defines the 32-band pseudo-QMF bank: analysis (C[i] = D[i] / 32 ... 11172-3 Annex C's encoder
    bank) followed by the standard's synthesis reconstructs a signal delayed by 481 samples to the bank's design
    error (~1e-4 of full scale); a wrong coefficient of the window breaks that."""
    D = mo.synthesis_window()
    C = D / 32.0
    n = 32 * 120
    rng = np.random.default_rng(0)
    x = np.convolve(rng.standard_normal(n), np.ones(8) / 8, "same") * 0.3
    M = np.cos(np.outer(2 * np.arange(32) + 1, np.arange(64) - 16) * np.pi / 64)  # [k][i] analysis matrixing
    buf = np.zeros(512)
    S = []
    for t in range(n // 32):
        buf = np.concatenate([x[32 * t: 32 * t + 32][::-1], buf[:-32]])
        Z = buf * C
        Y = Z.reshape(8, 64).sum(0)
        S.append(M @ Y)
    y = mo.synthesize(np.array(S), np.zeros(1024))
    d = 481
    err = np.abs(y[d + 512: n - 512] - x[512: n - 512 - d]).max()
    assert err < 2e-3 * np.abs(x).max(), err


@real
def test_real_file_probe_and_gapless_length():
    data = open(REAL_MP3, "rb").read()
    assert audio.container_name(data) == "MP3"
    info = audio.mp3_probe(data)
    assert (info.sample_rate, info.channels, info.version, info.bitrate_kbps, info.n_frames,
            info.samples_per_frame) == (44100, 2, 1, 128, 21, 1152)
    assert (info.enc_delay, info.enc_padding, info.flags, info.skip_samples) == (576, 0, 3, 576 + 529)
    assert info.total_samples == 21 * 1152 - 576 - 529 == 23087
    assert abs(audio.duration_seconds(REAL_MP3) - 23087 / 44100) < 1e-12


@real
def test_real_file_matches_oracle_and_every_granule_is_exact():
    data = open(REAL_MP3, "rb").read()
    x, sr = audio.decode_mp3(data)
    st = {}
    ref, rsr, info = mo.decode(data, st)
    assert sr == rsr == 44100 and x.shape == (23087, 2) and info["total"] == 23087
    _close(x, ref)
    assert len(st["exact"]) == 21 * 2 * 2 and all(st["exact"])  # Huffman data ends at part2_3_length, all 84
    # what the file exercises (tables 10, 16-18, 20-23 do not occur in it; the random-syntax tests cover them)
    assert {1, 2, 3, 5, 6, 7, 8, 9, 11, 12, 13, 15, 19, 24} <= st["tables"] and st["count1"] == {0, 1}
    assert {(0, 0), (1, 0), (2, 0), (3, 0)} <= st["blocks"]


@real
@pytest.mark.skipif(not os.path.exists(REAL_OGG), reason="the Vorbis twin is not present")
def test_real_file_against_its_vorbis_twin():
    """The cross-codec pin: the same MathJax sound encoded as Vorbis (22050 frames) and MP3. At 44.1 kHz the MP3
    decode equals the Vorbis decode up to a constant gain (0.950), correlation >= 0.95 at lag 0 (measured
    0.99999998), lag 0 the best of +-1197 (the gapless trim is exact), and the MP3's 1037 samples past the Vorbis
    length are digital silence."""
    m, _ = audio.decode_mp3(open(REAL_MP3, "rb").read())
    v, _ = audio.decode_vorbis(open(REAL_OGG, "rb").read())
    n = len(v)
    a, b = v.mean(1).astype(np.float64), m.mean(1).astype(np.float64)
    corr = lambda p, q: float(p @ q / np.sqrt((p @ p) * (q @ q)))
    c0 = corr(a, b[:n])
    assert c0 >= 0.95 and c0 > 0.9999
    lags = {lag: corr(a[max(0, -lag): n - max(0, lag)], b[max(0, lag): n - max(0, -lag)]) for lag in range(-1197, 1198, 7)}
    assert max(lags, key=lags.get) == 0
    assert abs(float(b[:n] @ a / (a @ a)) - 0.950) < 0.002
    assert np.abs(m[n:]).max() == 0.0


SEEDS = range(30)


def _stream(seed):
    rng = np.random.default_rng(seed)
    version = (1, 2, 25)[seed % 3]
    return mo.write_stream(rng, version=version, sr_sub=(seed // 3) % 3, mode=(1, 0, 1, 2, 1, 3)[(seed // 3) % 6],
                           nframes=4 + seed % 3, xing=seed % 4 == 0, id3=seed % 5 == 0,
                           crc=None if seed % 2 else True, enc_padding=(1200, 300, 0)[seed % 3])


@pytest.mark.parametrize("seed", SEEDS)
def test_random_syntax_streams_match_oracle(seed):
    data = _stream(seed)
    x, sr = audio.decode_mp3(data)
    ref, rsr, info = mo.decode(data)
    assert sr == rsr and x.shape[1] == info["channels"]
    _close(x, ref)


def test_random_streams_cover_the_syntax():
    """The writer reaches every decoder path over SEEDS: each version and sample rate, each channel mode with every
    mode extension (mid-side, intensity, both), every block kind (long / start / short / stop / mixed), every
    table_select the standard defines, both count1 tables and (LSF) every scalefactor partition incl. the
    intensity right channel's."""
    seen = {"sr": set(), "modes": set(), "blocks": set(), "tables": set(), "count1": set(), "lsf_tab": set()}
    for seed in SEEDS:
        data = _stream(seed)
        h0, frames, _ = mo.scan(data)
        for p, h in frames:
            seen["sr"].add(h["sr_index"])
            seen["modes"].add((h["mode"], h["mode_ext"] if h["mode"] == 1 else 0, h["lsf"]))
            si = mo.parse_side(data[p + 4 + 2 * h["crc"]: p + 4 + 2 * h["crc"] + h["side_bytes"]], h)
            for gr in range(h["granules"]):
                for ch in range(h["channels"]):
                    g = si["gr"][gr][ch]
                    seen["blocks"].add((g["block_type"], g["mixed"]))
                    seen["count1"].add(g["count1table_select"])
                    nreg = 2 if g["window_switching"] else 3
                    if g["big_values"]:
                        seen["tables"].update(g["table_select"][:nreg])
                    if h["lsf"]:
                        is_right = ch == 1 and h["mode"] == 1 and bool(h["mode_ext"] & 1)
                        seen["lsf_tab"].add(mo.lsf_slen(g["scalefac_compress"], is_right)[1])
    assert seen["sr"] == set(range(9))
    assert {(1, e, lsf) for e in range(4) for lsf in (0, 1)} <= seen["modes"]
    assert {(m, lsf) for m, _, lsf in seen["modes"]} == {(m, lsf) for m in range(4) for lsf in (0, 1)}
    assert {(0, 0), (1, 0), (2, 0), (2, 1), (3, 0)} <= seen["blocks"]
    assert set(mo._TABLES_OK) - {0} <= seen["tables"]
    assert seen["count1"] == {0, 1} and seen["lsf_tab"] == set(range(6))


def test_threads_do_not_change_the_output():
    """Frame ranges decode on threads, each primed by the frame before it: 1 and 4 threads give identical samples
    on a 240-frame stream, and they equal the oracle's."""
    data = mo.write_stream(np.random.default_rng(77), version=1, mode=1, nframes=240, max_big=60)
    x1, _ = audio.decode_mp3(data, threads=1)
    x4, _ = audio.decode_mp3(data, threads=4)
    assert np.array_equal(x1, x4) and len(x1) == 240 * 1152
    _close(x1, mo.decode(data)[0])


def _frames(data):
    h0, frames, _ = mo.scan(data)
    bounds = [p for p, _ in frames] + [frames[-1][0] + frames[-1][1]["frame_bytes"]]
    return data[: bounds[0]], [data[a:b] for a, b in zip(bounds[:-1], bounds[1:])]


def test_junk_between_frames_and_trailing_tags():
    """Bytes between frames (no sync) are skipped by resynchronisation on the next header of the same stream; ID3v1 / APEv2 tags after the last frame end
    the stream: the samples equal the clean stream's."""
    data = mo.write_stream(np.random.default_rng(5), version=1, mode=0, nframes=8)
    head, frames = _frames(data)
    rng = np.random.default_rng(1)
    # (the first frame must be confirmed by the next one, as every decoder's probe requires)
    dirty = head + frames[0] + b"".join(f + bytes(rng.integers(0, 0x7F, int(rng.integers(1, 30)), dtype=np.uint8))
                                        for f in frames[1:])
    clean, _ = audio.decode_mp3(data)
    x, _ = audio.decode_mp3(dirty)
    assert np.array_equal(x, clean)
    for tail in (b"TAG" + bytes(125), b"APETAGEX" + bytes(24)):
        y, _ = audio.decode_mp3(data + tail)
        assert np.array_equal(y, clean)


def test_lame_tag_trims_the_full_decode():
    """With a LAME tag the output is the full decode from sample delay + 529 on, nframes x 1152 - delay - padding
    samples long; replacing the tag's encoder string (no gapless fields) gives the untrimmed decode."""
    for delay, padding in ((576, 1200), (1105, 529), (0, 100)):
        data = mo.write_stream(np.random.default_rng(delay), version=1, mode=1, nframes=6, xing=True,
                               enc_delay=delay, enc_padding=padding)
        x, _ = audio.decode_mp3(data)
        info = audio.mp3_probe(data)
        i = data.index(b"LAME3.100")
        full, _ = audio.decode_mp3(data[:i] + b"XXXX" + data[i + 4:])
        assert len(full) == 6 * 1152 and info.n_frames == 6
        want = min(6 * 1152, 6 * 1152 - padding + 529) - (delay + 529)
        assert len(x) == info.total_samples == want
        assert np.array_equal(x, full[delay + 529: delay + 529 + want])


def test_16khz_lsf_stream_through_load_input_without_resampling():
    """An MPEG-2 LSF stream at 16 kHz needs no resampler (so no GPU): load_input is the channel mean of the decode."""
    data = mo.write_stream(np.random.default_rng(3), version=2, sr_sub=2, mode=1, nframes=5)
    assert audio.mp3_probe(data).sample_rate == 16000
    x, _ = audio.decode_mp3(data)
    y = audio.load_input(data)
    assert np.array_equal(y, x.mean(axis=1, dtype=np.float32))


def test_refusals():
    lib = _lib.load()
    info = _lib.TwMp3Info()
    assert lib.tw_mp3_probe(ctypes.c_char_p(b"nope"), 4, ctypes.byref(info)) != 0
    assert b"no MPEG audio frame" in lib.tw_last_error()
    layer2 = b"\xff\xfd\x90\x00" + bytes(400)  # an MPEG-1 Layer II header whose frame runs past the data
    with pytest.raises(ValueError, match="no MPEG audio frame"):
        audio.load_input(layer2)
    data = mo.write_stream(np.random.default_rng(4), version=1, mode=3, nframes=4)
    n = audio.mp3_probe(data).total_samples
    out = np.zeros((n - 1, 1), np.float32)
    got = ctypes.c_int64()
    assert lib.tw_mp3_decode(ctypes.c_char_p(data), len(data), out.ctypes.data, n - 1, 1, ctypes.byref(got)) != 0
    # a truncated last frame is dropped, not an error
    x, _ = audio.decode_mp3(data[:-10])
    assert len(x) == 3 * 1152


def test_length_cap(monkeypatch):
    data = mo.write_stream(np.random.default_rng(6), version=1, mode=3, nframes=4)
    monkeypatch.setenv("TW_MAX_AUDIO_S", "0.01")
    with pytest.raises(ValueError, match="TW_MAX_AUDIO_S"):
        audio.decode_mp3(data)
