"""AAC-LC ingest (ADTS and MP4 / M4A), CPU side: the native decoder (csrc/aac.cpp in libtwhip.so)
and the MP4 demuxer (twamd/audio.py: mp4_audio_track, decode_mp4) against the oracle's float64 restatement of
ISO/IEC 14496-3 (oracle/aac_oracle.py); an MP4's MP3 track through the MP3 decoder.

Pins, in the absence of ffmpeg (the reference's ffmpeg_read, $TF/pipelines/audio_utils.py:9-45, for the .m4a
uploads vocalis/security/security_monitor.py:353 lists) — the samples are "parity unpinned vs ffmpeg":
* the standard's tables (csrc/aac_tables.h): every spectral codebook and the scalefactor codebook a complete prefix
  code; the scalefactor-band tables with the standard's band counts, rising to 1024 / 128 lines;
* the image's one real AAC-LC stream (imageio's realshort.mp4: 48 kHz mono, 55 access units, no edit list): every
  access unit parses to its END element with only byte-alignment padding left (a wrong codebook entry derails the
  parse), and the track decodes to its mdhd duration of 55 x 1024 samples;
* the image's one MP4 with an MP3 track (imageio's cockatoo.mp4: MPEG-2 LSF 16 kHz mono, 388 frames, an edit list
  skipping 1105 = 576 + 529 samples and keeping 13.898 s): every granule's Huffman data ends at its part2_3_length and
  the output has the 222368 samples the edit keeps (the track is digital silence: a syntax pin only);
* random-syntax streams from the oracle's writer (SCE / CPE / LFE, common and separate windows, every window sequence
  and shape, grouping, every codebook incl. escapes, intensity, noise, pulses, TNS, mid/side masks, DSE / FIL) in
  ADTS and in the oracle's MP4 writer (chunked sample tables, edit lists) against the oracle.
Tolerance: 1e-6 of the stream's peak (float32 IMDCT in the native decoder vs float64 in the oracle)."""
import ctypes
import os

import numpy as np
import pytest

from oracle import aac_oracle as ao
from oracle import mp3_oracle as mo
from twamd import _lib, audio

IMAGES = "/opt/conda/lib/python3.9/site-packages/imageio/resources/images/"
REALSHORT, COCKATOO = IMAGES + "realshort.mp4", IMAGES + "cockatoo.mp4"
REL = 1e-6


def _close(got, ref):
    assert got.shape == ref.shape, (got.shape, ref.shape)
    scale = max(float(np.abs(ref).max()), 1e-30)
    assert np.abs(got - ref).max() <= REL * scale, float(np.abs(got - ref).max() / scale)


def test_tables_are_structurally_sound():
    checks = ao.table_checks()
    assert all(checks.values()), {k: v for k, v in checks.items() if not v}


@pytest.mark.skipif(not os.path.exists(REALSHORT), reason="imageio's realshort.mp4 is not present")
def test_real_aac_track_parses_exactly_and_matches_oracle():
    data = open(REALSHORT, "rb").read()
    assert audio.container_name(data) == "MP4/M4A"
    tr = audio.mp4_audio_track(data)
    assert (tr.codec, tr.config, tr.sample_rate, tr.channels, len(tr.sizes), tr.timescale, tr.edit, tr.duration) == \
        ("aac", bytes.fromhex("1188"), 48000, 1, 55, 48000, None, 55 * 1024)
    x, sr = audio.decode_mp4(data)
    units = [data[o: o + s] for o, s in zip(tr.offsets.tolist(), tr.sizes.tolist())]
    st = {}
    ref, rsr, _ = ao.decode_raw(tr.config, units, st)
    assert sr == rsr == 48000 and x.shape == (55 * 1024, 1)
    assert len(st["end_exact"]) == 55 and all(st["end_exact"])  # END closes every unit
    _close(x, ref)
    assert np.isfinite(x).all() and 1e-4 < float(np.sqrt(np.mean(x ** 2))) < 0.5
    assert abs(audio.duration_seconds(REALSHORT) - 55 * 1024 / 48000) < 1e-12


@pytest.mark.skipif(not os.path.exists(COCKATOO), reason="imageio's cockatoo.mp4 is not present")
def test_real_mp4_mp3_track_through_the_edit_list():
    data = open(COCKATOO, "rb").read()
    tr = audio.mp4_audio_track(data)
    assert (tr.codec, tr.sample_rate, len(tr.sizes), tr.timescale, tr.edit, tr.duration) == \
        ("mp3", 16000, 388, 16000, (1105, 222368), 388 * 576)
    au = b"".join(data[o: o + s] for o, s in zip(tr.offsets.tolist(), tr.sizes.tolist()))
    st = {}
    ref, _, info = mo.decode(au, st)
    assert info["n_frames"] == 388 and len(st["exact"]) == 388 and all(st["exact"])
    x, sr = audio.decode_mp4(data)
    assert sr == 16000 and x.shape == (222368, 1)
    _close(x, ref[1105: 1105 + 222368])


SEEDS = range(24)
_CFG = [(1, 3), (2, 4), (1, 8), (2, 11), (3, 0), (6, 6), (2, 3), (4, 7), (7, 5), (5, 9), (2, 1), (1, 12)]


def _adts(seed):
    cc, sri = _CFG[seed % len(_CFG)]
    return ao.write_adts(np.random.default_rng(seed), sri=sri, chan_config=cc, nframes=4, crc=seed % 2 == 1)


@pytest.mark.parametrize("seed", SEEDS)
def test_random_adts_streams_match_oracle(seed):
    data = _adts(seed)
    assert audio.container_name(data) == "AAC (ADTS)"
    x, sr = audio.decode_aac_adts(data)
    st = {}
    ref, rsr, _ = ao.decode_adts(data, st)
    assert sr == rsr and all(st["end_exact"])
    _close(x, ref)


def test_random_streams_cover_the_syntax():
    """Over SEEDS the writer reaches: every window sequence and shape, grouping, every spectral codebook 1..11, the
    intensity and noise codebooks, pulses, TNS, CPEs with and without a common window and every ms_mask_present."""
    seen = {"ws": set(), "shape": set(), "cb": set(), "msp": set(), "common": set(), "pulse": 0, "tns": 0}
    orig_info, orig_ics = ao._ics_info, ao._ics

    def info(br, sri):
        r = orig_info(br, sri)
        seen["ws"].add(r["ws"])
        seen["shape"].add(r["shape"])
        return r

    def ics(br, i, common, sri, seed):
        seen["common"].add(common)
        r = orig_ics(br, i, common, sri, seed)
        seen["cb"].update(int(c) for c in np.unique(r["cb"][:, : r["ics"]["max_sfb"]]))
        seen["tns"] += r["tns"] is not None
        return r

    ao._ics_info, ao._ics = info, ics
    try:
        for seed in SEEDS:
            ao.decode_adts(_adts(seed))
    finally:
        ao._ics_info, ao._ics = orig_info, orig_ics
    assert seen["ws"] == {0, 1, 2, 3} and seen["shape"] == {0, 1} and seen["common"] == {0, 1}
    assert set(range(16)) - {12} <= seen["cb"] and seen["tns"] > 10


def test_mp4_writer_tracks_with_edit_lists_and_chunks():
    """The demuxer over the oracle writer's MP4s: samples spread over chunks of 3 (a two-run stsc), the first edit's
    media time skipped and its duration kept, against the oracle's decode of the same units."""
    for seed, (cc, sri, edit) in enumerate([(1, 3, (1024, 5000)), (2, 4, (2112, 4 * 1024)), (2, 8, None),
                                            (1, 11, (0, 8 * 1024))]):
        data, units = ao.write_mp4(np.random.default_rng(100 + seed), sri=sri, chan_config=cc, nframes=10, edit=edit)
        tr = audio.mp4_audio_track(data)
        assert tr.codec == "aac" and len(tr.sizes) == 10
        assert [data[o: o + s] for o, s in zip(tr.offsets.tolist(), tr.sizes.tolist())] == units
        x, sr = audio.decode_mp4(data)
        ref, _, _ = ao.decode_raw(ao.asc_bytes(sri, cc), units)
        if edit is not None:
            ref = ref[edit[0]: edit[0] + edit[1]]
        _close(x, ref)


def test_threads_do_not_change_the_output():
    data = ao.write_adts(np.random.default_rng(9), sri=4, chan_config=2, nframes=120)
    x1, _ = audio.decode_aac_adts(data, threads=1)
    x4, _ = audio.decode_aac_adts(data, threads=4)
    assert np.array_equal(x1, x4) and len(x1) == 120 * 1024


def test_16khz_aac_through_load_input_without_resampling():
    data, _ = ao.write_mp4(np.random.default_rng(5), sri=8, chan_config=2, nframes=6)
    x, sr = audio.decode_mp4(data)
    assert sr == 16000
    assert np.array_equal(audio.load_input(data), x.mean(axis=1, dtype=np.float32))


def test_refusals():
    lib = _lib.load()
    info = _lib.TwAacInfo()
    for asc, msg in ((bytes([0x2B, 0x92, 0x08, 0x00]), b"HE-AAC"), (bytes([0x0A, 0x10]), b"Main"),
                     (bytes([0x11, 0x80]), b"configuration 0"), (bytes([0x11, 0x94]), b"960")):
        assert lib.tw_aac_parse_asc(ctypes.c_char_p(asc), len(asc), ctypes.byref(info)) != 0
        assert msg in lib.tw_last_error(), (asc.hex(), lib.tw_last_error())
    assert lib.tw_aac_parse_asc(ctypes.c_char_p(bytes([0x11, 0x90])), 2, ctypes.byref(info)) == 0
    assert (info.sample_rate, info.channels, info.object_type) == (48000, 2, 2)
    # an ADTS stream whose FIL element carries SBR data (implicit HE-AAC): refused, not decoded at half rate
    w = ao.BitWriter()
    w.put(6, 3)
    w.put(2, 4)
    w.put(13, 4)
    w.put(0, 12)
    w.put(7, 3)
    unit = w.bytes()
    flen = 7 + len(unit)
    hdr = bytes([0xFF, 0xF1, (1 << 6) | (3 << 2), (1 << 6) | (flen >> 11), (flen >> 3) & 0xFF,
                 ((flen & 7) << 5) | 0x1F, 0xFC])
    with pytest.raises(ValueError, match="HE-AAC"):
        audio.decode_aac_adts(hdr + unit)
    # an access unit cut short (its ADTS frame_length shortened by 8 bytes) is an error naming the unit
    data = bytearray(_adts(0))  # (seed 0: 7-byte headers, no CRC)
    flen = ((data[3] & 3) << 11) | (data[4] << 3) | (data[5] >> 5)
    short = flen - 8
    data[3] = (data[3] & 0xFC) | (short >> 11)
    data[4] = (short >> 3) & 0xFF
    data[5] = ((short & 7) << 5) | (data[5] & 0x1F)
    with pytest.raises(ValueError, match="access unit 0"):
        audio.decode_aac_adts(bytes(data[:short]))
    # MP4 codecs other than AAC-LC / MP3
    mp4, _ = ao.write_mp4(np.random.default_rng(1), nframes=2)
    bad = mp4.replace(b"\x04\x11\x40\x15", b"\x04\x11\xdd\x15")
    with pytest.raises(ValueError, match="not decoded"):
        audio.decode_mp4(bad)


def test_container_names():
    assert audio.container_name(_adts(0)) == "AAC (ADTS)"
    mp4, _ = ao.write_mp4(np.random.default_rng(0), nframes=2)
    assert audio.container_name(mp4) == "MP4/M4A"
    assert "AAC-LC" in audio.DECODED and "M4A" in audio.DECODED
