"""Apple Lossless (ALAC) in M4A: the native decoder (csrc/alac.cpp, tw_alac_decode) behind the MP4
demuxer (twamd.audio.decode_mp4), against the oracle's pure-integer restatement of ffmpeg's alac decoder
(oracle/alac_oracle.py) and against the input of the oracle's encoder (lossless: the decode must return it exactly).

Parity with ffmpeg is UNPINNED (no ALAC file or decoder in this image); what pins the semantics is the lossless round
trip of an encoder that runs the decoder's adaptive predictor forward, over every path: mono / stereo, 16 / 20 / 24-bit,
mix weights, shifted-out low bytes, LPC orders 0-30 and 31, prediction type 15, Rice escapes and zero runs,
uncompressed frames, a short last frame. The native output must equal the oracle's bit for bit."""
import ctypes

import numpy as np
import pytest

from oracle import alac_oracle as al
from twamd import _lib, audio

CASES = [(1, 16), (2, 16), (2, 24), (1, 24), (2, 20), (1, 20)]


def _m4a(seed, nch, depth, frames=3, frame_length=4096, tail=1000, mode="random", edit=None):
    rng = np.random.default_rng(seed)
    cookie, packets, x = al.write_stream(rng, nch=nch, depth=depth, frames=frames, frame_length=frame_length,
                                         tail=tail, mode=mode)
    cfg = al.parse_cookie(cookie)
    return al.write_m4a(cookie, packets, cfg, edit=edit), cookie, packets, x


@pytest.mark.parametrize("nch,depth", CASES)
def test_lossless_and_equal_to_oracle(nch, depth):
    data, cookie, packets, x = _m4a(nch * 100 + depth, nch, depth, frames=2, frame_length=2048, tail=777)
    assert audio.container_name(data) == "MP4/M4A"
    tr = audio.mp4_audio_track(data)
    assert tr.codec == "alac" and len(tr.sizes) == len(packets)
    got, sr = audio.decode_mp4(data)
    assert sr == 44100 and got.shape == x.shape
    ref = al.decode(cookie, packets)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(ref, al.to_float(x, depth))  # lossless: the encoder's input comes back


def test_paths_are_exercised():
    """What the encoder writes over CASES: LPC orders 0 and 31 and several between, type 15, uncompressed frames,
    0 / 1 / 2 shifted bytes, several mix weights (re-parsed from the packets' element headers)."""
    seen = {"orders": set(), "ptype15": False, "extra": set(), "weights": set(), "raw": False}
    for nch, depth in CASES:
        rng = np.random.default_rng(nch * 100 + depth)
        cookie, packets, _ = al.write_stream(rng, nch=nch, depth=depth, frames=5, frame_length=512, tail=77)
        for p in packets:
            br = al.BitReader(p)
            chans = 2 if br.get(3) == 1 else 1
            br.get(16)
            has_size, extra, raw = br.get(1), br.get(2), br.get(1)
            if has_size:
                br.get(32)
            seen["extra"].add(extra)
            if raw:
                seen["raw"] = True
                continue
            br.get(8)
            seen["weights"].add(br.get(8))
            for _ in range(chans):
                ptype, _q, _h, order = br.get(4), br.get(4), br.get(3), br.get(5)
                seen["orders"].add(order)
                seen["ptype15"] |= ptype == 15
                br.get(16 * order)
    assert {0, 31} <= seen["orders"] and len(seen["orders"]) >= 6 and seen["ptype15"] and seen["raw"]
    assert seen["extra"] >= {0, 1, 2} and len(seen["weights"]) >= 3


def test_threads_and_partial_frame():
    data, cookie, packets, x = _m4a(7, 2, 16, frames=12, frame_length=1024, tail=100)
    x1, _ = audio.decode_mp4(data, threads=1)
    x4, _ = audio.decode_mp4(data, threads=4)
    assert np.array_equal(x1, x4) and len(x1) == 12 * 1024 + 100


def test_edit_list():
    """An edit list trims an ALAC track as it trims AAC (media_time skipped, the edit's duration kept)."""
    data, cookie, packets, x = _m4a(9, 1, 16, frames=2, frame_length=1024, tail=300, edit=(100, 2000))
    got, _ = audio.decode_mp4(data)
    np.testing.assert_array_equal(got, al.to_float(x, 16)[100: 2100])


def test_refused_packet_is_dropped_and_cookie_checks():
    """A packet the decoder refuses (here: an element tag 5) contributes no samples, as ffmpeg drops it; a cookie
    of an unsupported depth or channel count is refused by name."""
    rng = np.random.default_rng(11)
    cookie, packets, x = al.write_stream(rng, nch=1, depth=16, frames=3, frame_length=1024, tail=0)
    bad = bytearray(packets[1])
    bad[0] = (5 << 5) | (bad[0] & 31)
    cfg = al.parse_cookie(cookie)
    data = al.write_m4a(cookie, [packets[0], bytes(bad), packets[2]], cfg)
    got, _ = audio.decode_mp4(data)
    want = al.to_float(np.concatenate([x[:1024], x[2048:]]), 16)
    np.testing.assert_array_equal(got, want)
    lib = _lib.load()
    info = _lib.TwAlacInfo()
    odd = bytearray(cookie)
    odd[12 + 5] = 8  # 8-bit depth
    assert lib.tw_alac_parse_cookie(bytes(odd), len(odd), ctypes.byref(info)) != 0 and b"bit depth" in lib.tw_last_error()
    odd = bytearray(cookie)
    odd[12 + 9] = 6  # 5.1
    assert lib.tw_alac_parse_cookie(bytes(odd), len(odd), ctypes.byref(info)) != 0 and b"mono and stereo" in lib.tw_last_error()
    assert lib.tw_alac_parse_cookie(cookie, len(cookie), ctypes.byref(info)) == 0 and (info.bit_depth, info.channels) == (16, 1)
