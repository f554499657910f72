"""Fragmented MP4 / M4A (what browsers' MediaRecorder and live writers produce: an empty sample table in moov, mvex /
trex defaults, then moof / traf / trun fragments each followed by its mdat), demuxed as ffmpeg's mov demuxer reads it
(ISO/IEC 14496-12 8.8) for the reference's .m4a uploads (ffmpeg_read, $TF/pipelines/audio_utils.py:9-45). The access
units are the AAC oracle's random-syntax units (oracle/aac_oracle.py); the demuxed units must be exactly them, and
the decode equal the oracle's decode of the same units. Base offsets covered: default-base-is-moof with trun data
offsets, an explicit tfhd base data offset, and runs following one another without offsets; sizes per sample, from
tfhd's default and from trex's; a second (video) track's fragments interleaved and skipped."""
import struct

import numpy as np
import pytest

from oracle import aac_oracle as ao
from twamd import audio


def _box(t, body):
    return struct.pack(">I", 8 + len(body)) + t + body


def _full(t, ver_flags, body):
    return _box(t, struct.pack(">I", ver_flags) + body)


def _stsd_of(mp4: bytes) -> bytes:
    i = mp4.index(b"stsd") - 4
    n = struct.unpack(">I", mp4[i: i + 4])[0]
    return mp4[i: i + n]


def _moov(stsd, rate, trex_size=0, with_video=False, edit=None):
    def trak(tid, handler, stsd_box):
        empty = (_full(b"stts", 0, struct.pack(">I", 0)) + _full(b"stsc", 0, struct.pack(">I", 0)) +
                 _full(b"stsz", 0, struct.pack(">II", 0, 0)) + _full(b"stco", 0, struct.pack(">I", 0)))
        stbl = _box(b"stbl", stsd_box + empty)
        mdia = _box(b"mdia", _full(b"mdhd", 0, struct.pack(">IIII", 0, 0, rate, 0) + bytes(4)) +
                    _full(b"hdlr", 0, bytes(4) + handler + bytes(12) + b"x\x00") + _box(b"minf", stbl))
        tkhd = _full(b"tkhd", 0, struct.pack(">III", 0, 0, tid) + bytes(68))
        edts = _box(b"edts", _full(b"elst", 0, struct.pack(">IIiI", 1, edit[1], edit[0], 1 << 16))) if edit else b""
        return _box(b"trak", tkhd + edts + mdia)

    traks = trak(1, b"soun", stsd)
    if with_video:
        traks += trak(2, b"vide", _full(b"stsd", 0, struct.pack(">I", 0)))
    trex = _full(b"trex", 0, struct.pack(">IIIII", 1, 1, 1024, trex_size, 0))
    if with_video:
        trex += _full(b"trex", 0, struct.pack(">IIIII", 2, 1, 1, 0, 0))
    mvhd = _full(b"mvhd", 0, struct.pack(">IIII", 0, 0, rate, 0) + bytes(80))
    return _box(b"moov", mvhd + traks + _box(b"mvex", trex))


def _fragment(seq, units, mode, video=None):
    """One moof + mdat. mode: 'moof' (default-base-is-moof + trun data offset + per-sample sizes), 'explicit'
    (tfhd base data offset, filled in by the caller), 'chained' (two truns, the second without a data offset),
    'tfhd' / 'trex' (no per-sample sizes: tfhd's default sample size, or the track's trex default; equal-size units)."""
    sizes = [len(u) for u in units]
    if mode in ("tfhd", "trex"):
        assert len(set(sizes)) == 1
        tfhd = _full(b"tfhd", 0x20000 | (0x10 if mode == "tfhd" else 0),
                     struct.pack(">I", 1) + (struct.pack(">I", sizes[0]) if mode == "tfhd" else b""))
        truns = [_full(b"trun", 0x001, struct.pack(">Ii", len(units), 0))]
    elif mode == "moof":
        tfhd = _full(b"tfhd", 0x20000, struct.pack(">I", 1))
        trun = _full(b"trun", 0x201, struct.pack(">Ii", len(units), 0) + b"".join(struct.pack(">I", s) for s in sizes))
        truns = [trun]
    elif mode == "explicit":
        tfhd = _full(b"tfhd", 0x01, struct.pack(">IQ", 1, 0))
        truns = [_full(b"trun", 0x200, struct.pack(">I", len(units)) + b"".join(struct.pack(">I", s) for s in sizes))]
    else:
        h = len(units) // 2
        tfhd = _full(b"tfhd", 0x20000, struct.pack(">I", 1))
        truns = [_full(b"trun", 0x201, struct.pack(">Ii", h, 0) + b"".join(struct.pack(">I", s) for s in sizes[:h])),
                 _full(b"trun", 0x200, struct.pack(">I", len(units) - h) +
                       b"".join(struct.pack(">I", s) for s in sizes[h:]))]
    traf = _box(b"traf", tfhd + _full(b"tfdt", 0, struct.pack(">I", 0)) + b"".join(truns))
    vtraf = b""
    if video is not None:  # a video track's run (track 2, its own data after the audio's)
        vtfhd = _full(b"tfhd", 0x20000 | 0x10, struct.pack(">II", 2, len(video)))
        vtraf = _box(b"traf", vtfhd + _full(b"trun", 0x001, struct.pack(">Ii", 1, 0)))
    moof = _box(b"moof", _full(b"mfhd", 0, struct.pack(">I", seq)) + traf + vtraf)
    payload = b"".join(units) + (video or b"")
    # patch offsets now that the moof size is known
    moof = bytearray(moof)
    data_start = len(moof) + 8
    if mode in ("moof", "chained", "tfhd", "trex"):
        i = moof.index(b"trun") + 4 + 4 + 4
        moof[i: i + 4] = struct.pack(">i", data_start)
    if video is not None:
        j = moof.rindex(b"trun") + 4 + 4 + 4
        moof[j: j + 4] = struct.pack(">i", data_start + sum(sizes))
    return bytes(moof), _box(b"mdat", payload)


def _fmp4(rng, mode, nfrag=3, per=4, with_video=False, edit=None, trex_size=0):
    mp4, _ = ao.write_mp4(rng, sri=4, chan_config=2, nframes=1)
    stsd = _stsd_of(mp4)
    units = [ao.write_unit(rng, 2, 4) for _ in range(nfrag * per)]
    if mode in ("tfhd", "trex"):  # equal sizes: zero bytes after each unit's END element (ignored by decoders)
        top = max(len(u) for u in units)
        units = [u + bytes(top - len(u)) for u in units]
        trex_size = top if mode == "trex" else 0
    out = bytearray(_box(b"ftyp", b"iso5\x00\x00\x02\x00iso5iso6mp41") + _moov(stsd, 44100, trex_size, with_video, edit))
    for f in range(nfrag):
        chunk = units[f * per: (f + 1) * per]
        video = bytes(rng.integers(0, 256, 37, dtype=np.uint8)) if with_video else None
        moof, mdat = _fragment(f + 1, chunk, mode, video)
        if mode == "explicit":
            moof = bytearray(moof)
            i = moof.index(b"tfhd") + 4 + 4 + 4
            moof[i: i + 8] = struct.pack(">Q", len(out) + len(moof) + 8)
            moof = bytes(moof)
        out += moof + mdat
    return bytes(out), units


@pytest.mark.parametrize("mode,video", [("moof", False), ("explicit", False), ("chained", False), ("tfhd", False),
                                        ("trex", False), ("moof", True)])
def test_fragmented_mp4_units_and_decode(mode, video):
    seed = ["moof", "explicit", "chained", "tfhd", "trex"].index(mode) + 10 * video
    data, units = _fmp4(np.random.default_rng(seed), mode, with_video=video)
    assert audio.container_name(data) == "MP4/M4A"
    tr = audio.mp4_audio_track(data)
    assert tr.codec == "aac"
    assert [data[o: o + s] for o, s in zip(tr.offsets.tolist(), tr.sizes.tolist())] == units
    x, sr = audio.decode_mp4(data)
    ref, _, _ = ao.decode_raw(ao.asc_bytes(4, 2), units)
    assert sr == 44100 and x.shape == ref.shape
    assert np.abs(x - ref).max() <= 1e-6 * max(1.0, float(np.abs(ref).max()))


def test_fragmented_mp4_zero_length_edit_keeps_everything_after_the_skip():
    """Fragmented writers put a zero segment duration in their edit (the length is unknown when moov is written):
    the media time is skipped and the rest kept."""
    data, units = _fmp4(np.random.default_rng(3), "moof", edit=(2112, 0))
    x, _ = audio.decode_mp4(data)
    ref, _, _ = ao.decode_raw(ao.asc_bytes(4, 2), units)
    assert x.shape == ref[2112:].shape
    assert np.abs(x - ref[2112:]).max() <= 1e-6 * max(1.0, float(np.abs(ref).max()))
