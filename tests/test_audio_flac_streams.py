"""FLAC as it arrives from streaming writers (the reference's example input is FLAC,
examples/Test1/ChrisAndAlexDiTest.flac, read by ffmpeg_read, $TF/pipelines/audio_utils.py:9-45):
* a STREAMINFO whose total-samples field is 0 (a FLAC written to a pipe: the muxer cannot seek back to fill it) — ffmpeg
  decodes such a stream frame by frame; the native probe takes the length from the last genuine frame (sync, CRC-8,
  CRC-16 of a full decode, searched back from the end);
* Ogg FLAC (the FLAC-to-Ogg mapping ffmpeg's ogg demuxer reads: "\\x7fFLAC" mapping header carrying "fLaC" +
  STREAMINFO, metadata-block packets, then frames), demuxed to the native stream it carries.
The samples are pinned by the oracle's FLAC encoder (oracle/audio_oracle.py): the decode must return its input."""
import struct

import numpy as np
import pytest

from oracle import audio_oracle as ao
from oracle import vorbis_oracle as vo
from twamd import audio


def _pcm(n, ch, bps, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    top = 2 ** (bps - 1)
    x = np.stack([0.4 * np.sin(2 * np.pi * (300 + 70 * c) * t / 16000) + 0.02 * rng.standard_normal(n)
                  for c in range(ch)], 1)
    return np.clip(np.round(x * top), -top, top - 1).astype(np.int64)


def _zero_total(flac: bytes) -> bytes:
    b = bytearray(flac)
    si = 8  # "fLaC" + the STREAMINFO block header
    x = int.from_bytes(b[si + 10: si + 18], "big") & ~((1 << 36) - 1)
    b[si + 10: si + 18] = x.to_bytes(8, "big")
    b[si + 18: si + 34] = bytes(16)  # (a piped writer leaves the MD5 unset too)
    return bytes(b)


@pytest.mark.parametrize("variable,bs", [(False, (4096,)), (True, (1152, 576, 4608)), (False, (1024,))])
def test_unknown_total_from_last_frame(variable, bs):
    pcm = _pcm(10000 + 333, 2, 16, 3)
    flac = ao.flac_encode(pcm, 16000, 16, blocksizes=bs, variable=variable, stereo_modes=(0, 10))
    z = _zero_total(flac)
    info = audio.flac_probe(z)
    assert info.total_samples == len(pcm) and info.total_from_frames == 1
    assert audio.flac_probe(flac).total_from_frames == 0
    got = audio.decode_flac(z)
    np.testing.assert_array_equal(got.pcm, pcm)
    # trailing junk after the last frame (an ID3v1 tag) does not hide it
    got = audio.decode_flac(z + b"TAG" + bytes(125))
    np.testing.assert_array_equal(got.pcm, pcm)


def _ogg_flac(flac: bytes, chunk: int = 700, with_comment: bool = True) -> bytes:
    info = audio.flac_probe(flac)
    si = bytearray(flac[4: 4 + 38])
    si[0] &= 0x7F
    comment = b"\x84" + (12).to_bytes(3, "big") + struct.pack("<I", 4) + b"test" + struct.pack("<I", 0)
    first = b"\x7fFLAC\x01\x00" + struct.pack(">H", 1 if with_comment else 0) + b"fLaC" + bytes(si)
    audio_bytes = flac[int(info.audio_offset):]
    packets = [first] + ([comment] if with_comment else [])
    packets += [audio_bytes[i: i + chunk] for i in range(0, len(audio_bytes), chunk)]
    return vo.ogg_write(packets, [0] * (len(packets) - 1) + [int(info.total_samples)])


@pytest.mark.parametrize("ch,bps,zero", [(1, 16, False), (2, 24, False), (2, 16, True)])
def test_ogg_flac(ch, bps, zero, tmp_path):
    pcm = _pcm(9000, ch, bps, ch * bps)
    flac = ao.flac_encode(pcm, 16000, bps, blocksizes=(2048,))
    data = _ogg_flac(_zero_total(flac) if zero else flac, with_comment=not zero)
    assert audio.container_name(data) == "Ogg FLAC"
    native = audio.ogg_flac_to_native(data)
    got = audio.decode_flac(native)
    np.testing.assert_array_equal(got.pcm, pcm)
    if not zero:
        assert audio.pcm_md5(got.pcm, bps) == got.md5
    p = tmp_path / "upload.ogg"
    p.write_bytes(data)
    assert audio.duration_seconds(str(p)) == pytest.approx(9000 / 16000)


def test_ogg_flac_without_mapping_header_is_refused():
    bad = vo.ogg_write([b"\x7fFLAX" + bytes(60)], [0])
    with pytest.raises(ValueError):
        audio.ogg_flac_to_native(bad)
