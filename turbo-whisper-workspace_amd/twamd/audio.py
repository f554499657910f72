"""Audio ingest for the transcriber (host decode + GPU resample, before the log-mel).

Mirrors the input handling of AutomaticSpeechRecognitionPipeline.preprocess
($TF/pipelines/automatic_speech_recognition.py:345-420): a path is read as bytes, bytes are decoded to mono f32
at 16 kHz (the reference shells out to `ffmpeg -ac 1 -ar 16000 -f f32le`, $TF/pipelines/audio_utils.py:9-45,
which this image does not have), dicts carry {"raw"|"array", "sampling_rate"} and are resampled when the rate
differs, multi-channel arrays are averaged to mono.

Containers: FLAC (native multi-threaded decoder in libtwhip.so, include/tw_audio.h; bit-exact, verifiable
against the stream's STREAMINFO MD5), Ogg Vorbis (native decoder, csrc/vorbis.cpp), MP3 (MPEG-1 / 2 / 2.5 Layer III,
native multi-threaded decoder csrc/mp3.cpp, gapless-trimmed by the LAME tag as ffmpeg trims it; Layers I / II too), AAC-LC (native
decoder csrc/aac.cpp) in ADTS or in an MP4 / M4A track (demuxed here: stsz / stsc / stco, trimmed by the edit list;
an MP4's MP3 track goes to the MP3 decoder), RIFF/WAVE (PCM 8/16/24/32-bit, IEEE float 32/64, G.711 A-law / mu-law, IMA
ADPCM), Sun AU and AIFF / AIFF-C (PCM, float, G.711) — the telephony codecs through native decoders
(tw_g711_decode, tw_ima_adpcm_wav_decode), pinned to CPython's audioop / aifc / sunau / wave.
Resampling runs on the GPU (tw_resample_pcm_*) with libswresample's default filter restated in
swr_filter_bank. There is no CPU resampler in the product: resampling without a GPU raises.
"""
from __future__ import annotations

import ctypes
import io
import math
import os
import struct
from typing import List, NamedTuple, Optional, Tuple, Union

import numpy as np

TARGET_SR = 16000


class FlacStream(NamedTuple):
    pcm: np.ndarray  # int32 [frames, channels], sample values as coded
    sample_rate: int
    bits_per_sample: int
    md5: bytes  # STREAMINFO MD5 of the unencoded PCM


def _flac_lib():
    from . import _lib

    return _lib, _lib.load()


def flac_probe(data: bytes):
    _lib, lib = _flac_lib()
    info = _lib.TwFlacInfo()
    buf = ctypes.c_char_p(data)
    if lib.tw_flac_probe(buf, len(data), ctypes.byref(info)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return info


def decode_flac(data: bytes, threads: int = 0) -> FlacStream:
    """FLAC bytes -> int32 PCM through the native decoder (frame CRCs checked; no concealment)."""
    _lib, lib = _flac_lib()
    info = flac_probe(data)
    total, ch = int(info.total_samples), int(info.channels)
    # bound the allocation before trusting the header: a frame codes at most 65535 samples per channel in no fewer
    # than ~(6 + channels) bytes, and the stream may last at most max_audio_seconds() (constant-subframe frames code
    # 65535 samples in a few bytes, so the byte bound alone admits ~0.2 Gsamples per MB)
    max_s = max_audio_seconds()
    if total > (len(data) // (6 + ch) + 1) * 65535 or total > max_s * int(info.sample_rate):
        raise ValueError(f"FLAC header claims {total} samples x {ch} channels at {int(info.sample_rate)} Hz: larger "
                         f"than the stream can code or longer than TW_MAX_AUDIO_S={max_s:g} s")
    pcm = np.zeros((total, ch), np.int32)  # never hand out uninitialised memory, whatever the decoder reports
    got = ctypes.c_int64()
    if lib.tw_flac_decode(ctypes.c_char_p(data), len(data), pcm.ctypes.data, pcm.shape[0], int(threads),
                          ctypes.byref(got)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return FlacStream(pcm, int(info.sample_rate), int(info.bits_per_sample), bytes(info.md5))


def pcm_md5(pcm: np.ndarray, bits_per_sample: int) -> bytes:
    """FLAC's STREAMINFO checksum definition: MD5 over interleaved little-endian samples of ceil(bps/8) bytes."""
    import hashlib

    nb = (bits_per_sample + 7) // 8
    raw = np.ascontiguousarray(pcm, dtype="<i4").view(np.uint8).reshape(-1, 4)[:, :nb]
    return hashlib.md5(np.ascontiguousarray(raw).tobytes()).digest()


def swr_filter_bank(sr_in: int, sr_out: int, filter_size: int = 32, cutoff: float = 0.97,
                    kaiser_beta: float = 9.0) -> Tuple[int, int, np.ndarray]:
    """libswresample's default resampler design (what `ffmpeg -ar 16000` runs): exact rational phases
    up/down = sr_out/sr_in reduced, Kaiser-windowed sinc of filter_length = ceil(filter_size / factor) taps with
    factor = min(up/down * cutoff, 1), each phase normalised by the sum of phase 0.
    Returns (up, down, taps f32[up][ntaps]); tap i of phase ph sits at offset (i - center) - ph/up input samples,
    center = (ntaps - 1) // 2."""
    g = math.gcd(int(sr_in), int(sr_out))
    up, down = int(sr_out) // g, int(sr_in) // g
    if up == down:
        return 1, 1, np.ones((1, 1), np.float32)
    factor = min(up / down * cutoff, 1.0)
    T = max(int(math.ceil(filter_size / factor)), 1)
    center = (T - 1) // 2
    i = np.arange(T, dtype=np.float64)[None, :]
    ph = np.arange(up, dtype=np.float64)[:, None]
    x = np.pi * ((i - center) - ph / up) * factor
    with np.errstate(invalid="ignore", divide="ignore"):
        y = np.where(x == 0, 1.0, np.sin(x) / np.where(x == 0, 1.0, x))
    w = 2.0 * x / (factor * T * np.pi)
    y = y * np.i0(kaiser_beta * np.sqrt(np.maximum(1.0 - w * w, 0.0)))
    y = y / y[0].sum()
    return up, down, y.astype(np.float32)


def resample_device(x: np.ndarray, sr_in: int, sr_out: int = TARGET_SR, scale: float = 1.0,
                    device=None):
    """Downmix + resample on the GPU: x is int32 PCM [frames, ch] (times `scale`) or float [frames] /
    [frames, ch]. Returns a float32 torch tensor [n_out] on `device` (default: the current GPU)."""
    import torch

    from . import _lib

    if not torch.cuda.is_available():
        raise RuntimeError("resampling runs on the GPU (tw_resample_pcm_*); no GPU is visible")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    up, down, taps = swr_filter_bank(sr_in, sr_out)
    x = np.asarray(x)
    if x.ndim == 1:
        x = x[:, None]
    n_in, ch = x.shape
    n_out = -(-n_in * up // down)
    with torch.cuda.device(dev):
        xd = torch.from_numpy(np.ascontiguousarray(x)).to(dev, non_blocking=False)
        td = torch.from_numpy(taps).to(dev)
        y = torch.empty(n_out, dtype=torch.float32, device=dev)
        st = _lib.stream_handle()
        if x.dtype == np.int32:
            _lib.call("tw_resample_pcm_i32", xd.data_ptr(), n_in, ch, float(scale), up, down, td.data_ptr(),
                      taps.shape[1], y.data_ptr(), n_out, st)
        else:
            xd = xd.float()
            _lib.call("tw_resample_pcm_f32", xd.data_ptr(), n_in, ch, up, down, td.data_ptr(), taps.shape[1],
                      y.data_ptr(), n_out, st)
    return y


def vorbis_probe(data: bytes):
    _lib, lib = _flac_lib()
    info = _lib.TwVorbisInfo()
    if lib.tw_vorbis_probe(ctypes.c_char_p(data), len(data), ctypes.byref(info)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return info


def decode_vorbis(data: bytes, threads: int = 0) -> Tuple[np.ndarray, int]:
    """Ogg Vorbis bytes -> f32 [frames, channels] through the native decoder (csrc/vorbis.cpp; Ogg page CRCs
    checked, the end trimmed to the last page's granule position)."""
    _lib, lib = _flac_lib()
    info = vorbis_probe(data)
    total, ch, sr = int(info.total_samples), int(info.channels), int(info.sample_rate)
    # bound the allocation before trusting the granule: a packet of >= 1 byte codes at most blocksize1 / 2 frames
    if total < 0 or total > (len(data) + 1) * int(info.blocksize1) // 2 or total > max_audio_seconds() * sr:
        raise ValueError(f"Ogg Vorbis stream claims {total} frames x {ch} channels at {sr} Hz: larger than the "
                         f"stream can code or longer than TW_MAX_AUDIO_S={max_audio_seconds():g} s")
    out = np.zeros((total, ch), np.float32)
    got = ctypes.c_int64()
    if lib.tw_vorbis_decode(ctypes.c_char_p(data), len(data), out.ctypes.data, total, int(threads),
                            ctypes.byref(got)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return out[: got.value], sr


def mp3_probe(data: bytes):
    _lib, lib = _flac_lib()
    info = _lib.TwMp3Info()
    if lib.tw_mp3_probe(ctypes.c_char_p(data), len(data), ctypes.byref(info)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return info


def decode_mp3(data: bytes, threads: int = 0) -> Tuple[np.ndarray, int]:
    """MP3 (or MPEG audio Layer I / II) bytes -> f32 [frames, channels] through the native decoder (csrc/mp3.cpp; for
    Layer III the Xing / Info frame skipped, the LAME tag's delay + 529 samples dropped at the start and its
    padding - 529 at the end, as ffmpeg's mp3 demuxer does)."""
    _lib, lib = _flac_lib()
    info = mp3_probe(data)
    total, ch, sr = int(info.total_samples), int(info.channels), int(info.sample_rate)
    if total > max_audio_seconds() * sr:
        raise ValueError(f"MP3 stream of {total} frames at {sr} Hz is longer than TW_MAX_AUDIO_S="
                         f"{max_audio_seconds():g} s")
    out = np.zeros((total, ch), np.float32)
    got = ctypes.c_int64()
    if lib.tw_mp3_decode(ctypes.c_char_p(data), len(data), out.ctypes.data, total, int(threads),
                         ctypes.byref(got)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return out[: got.value], sr


def aac_adts_probe(data: bytes):
    _lib, lib = _flac_lib()
    info = _lib.TwAacInfo()
    if lib.tw_aac_adts_probe(ctypes.c_char_p(data), len(data), ctypes.byref(info)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return info


def decode_aac_adts(data: bytes, threads: int = 0) -> Tuple[np.ndarray, int]:
    """ADTS AAC-LC bytes (.aac) -> f32 [frames, channels] through the native decoder (csrc/aac.cpp): every frame's 1024
    samples, untrimmed (ADTS carries no priming information; ffmpeg does not trim it either)."""
    _lib, lib = _flac_lib()
    info = aac_adts_probe(data)
    total, ch, sr = int(info.total_samples), int(info.channels), int(info.sample_rate)
    if total > max_audio_seconds() * sr:
        raise ValueError(f"AAC stream longer than TW_MAX_AUDIO_S={max_audio_seconds():g} s")
    out = np.zeros((total, ch), np.float32)
    got = ctypes.c_int64()
    if lib.tw_aac_adts_decode(ctypes.c_char_p(data), len(data), out.ctypes.data, total, int(threads),
                              ctypes.byref(got)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return out[: got.value], sr


class Mp4Track(NamedTuple):
    codec: str               # "aac", "mp3" or "alac"
    config: bytes            # AAC AudioSpecificConfig / ALACSpecificConfig (b"" for MP3)
    sample_rate: int
    channels: int
    offsets: np.ndarray      # int64 byte offset of each access unit in the file
    sizes: np.ndarray        # int64 size of each access unit
    timescale: int           # the track's (mdhd) time units per second
    edit: Optional[Tuple[int, int]]  # first non-empty edit: (media_time, duration), both in the track's timescale
    duration: int            # mdhd duration (track timescale)


def _mp4_boxes(data: bytes, start: int, end: int):
    pos = start
    while pos + 8 <= end:
        size, typ = struct.unpack(">I4s", data[pos: pos + 8])
        hdr = 8
        if size == 1:
            if pos + 16 > end:
                break
            size, hdr = struct.unpack(">Q", data[pos + 8: pos + 16])[0], 16
        elif size == 0:
            size = end - pos
        if size < hdr or pos + size > end:
            raise ValueError(f"MP4: box {typ!r} at {pos} overruns its parent")
        yield typ, pos + hdr, pos + size
        pos += size


def _desc(data: bytes, pos: int):
    """An MPEG-4 descriptor at pos: (tag, body start, body end)."""
    tag, pos, n = data[pos], pos + 1, 0
    for _ in range(4):
        b = data[pos]
        pos += 1
        n = (n << 7) | (b & 0x7F)
        if not b & 0x80:
            break
    return tag, pos, pos + n


def _esds_config(data: bytes, a: int, b: int) -> Tuple[int, bytes]:
    """(objectTypeIndication, DecoderSpecificInfo) of an esds box body."""
    tag, p, e = _desc(data, a + 4)  # (version / flags)
    if tag != 3:
        raise ValueError("MP4: esds without an ES_Descriptor")
    flags = data[p + 2]
    p += 3 + (2 if flags & 0x80 else 0)
    if flags & 0x40:
        p += 1 + data[p]
    p += 2 if flags & 0x20 else 0
    tag, q, qe = _desc(data, p)
    if tag != 4:
        raise ValueError("MP4: esds without a DecoderConfigDescriptor")
    oti = data[q]
    cfg = b""
    if q + 13 < qe:
        tag, r, re_ = _desc(data, q + 13)
        if tag == 5:
            cfg = data[r: re_]
    return oti, cfg


def _fragment_samples(data: bytes, moov: Tuple[int, int], trak_a: int, trak_b: int) -> Tuple[np.ndarray, np.ndarray]:
    """Fragmented MP4 (what browsers' MediaRecorder and live writers produce): the byte offset and size of every sample
    of this track in the file's moof / traf / trun boxes (ISO/IEC 14496-12 8.8, as ffmpeg's mov demuxer reads them):
    sizes from trun, else tfhd's default, else the track's trex default; offsets from the base data offset (tfhd's
    explicit one, the moof start under default-base-is-moof or for a moof's first traf, else where the previous
    traf's data ended) plus trun's data offset, samples contiguous after it."""
    tid = None
    for t, a, b in _mp4_boxes(data, trak_a, trak_b):
        if t == b"tkhd":
            tid = struct.unpack(">I", data[a + (20 if data[a] == 1 else 12): a + (24 if data[a] == 1 else 16)])[0]
    trex_size = 0
    for t, a, b in _mp4_boxes(data, *moov):
        if t == b"mvex":
            for tt, aa, bb in _mp4_boxes(data, a, b):
                if tt == b"trex" and struct.unpack(">I", data[aa + 4: aa + 8])[0] == tid:
                    trex_size = struct.unpack(">I", data[aa + 16: aa + 20])[0]
    offs: List[int] = []
    sizes: List[int] = []
    for t, ma, mb in _mp4_boxes(data, 0, len(data)):
        if t != b"moof":
            continue
        moof_start, prev_end = ma - 8, None
        for tt, ta, tb in _mp4_boxes(data, ma, mb):
            if tt != b"traf":
                continue
            base, dflt_size, this_track = None, trex_size, False
            for t3, a3, b3 in _mp4_boxes(data, ta, tb):
                if t3 == b"tfhd":
                    fl = int.from_bytes(data[a3 + 1: a3 + 4], "big")
                    this_track = struct.unpack(">I", data[a3 + 4: a3 + 8])[0] == tid
                    q = a3 + 8
                    if fl & 0x01:
                        base = struct.unpack(">Q", data[q: q + 8])[0]
                        q += 8
                    q += 4 * bool(fl & 0x02) + 4 * bool(fl & 0x08)
                    if fl & 0x10:
                        dflt_size = struct.unpack(">I", data[q: q + 4])[0]
                    if base is None:
                        base = moof_start if (fl & 0x20000 or prev_end is None) else prev_end
                elif t3 == b"trun":
                    fl = int.from_bytes(data[a3 + 1: a3 + 4], "big")
                    n = struct.unpack(">I", data[a3 + 4: a3 + 8])[0]
                    q = a3 + 8
                    pos = base if base is not None else moof_start
                    if fl & 0x01:
                        pos = base + struct.unpack(">i", data[q: q + 4])[0]
                        q += 4
                    elif prev_end is not None:
                        pos = prev_end
                    q += 4 * bool(fl & 0x04)
                    per = 4 * (bool(fl & 0x100) + bool(fl & 0x200) + bool(fl & 0x400) + bool(fl & 0x800))
                    for i in range(n):
                        rec = q + i * per
                        sz = dflt_size
                        if fl & 0x200:
                            sz = struct.unpack(">I", data[rec + 4 * bool(fl & 0x100): rec + 4 * bool(fl & 0x100) + 4])[0]
                        if this_track:
                            offs.append(pos)
                            sizes.append(sz)
                        pos += sz
                    prev_end = pos
    return np.array(offs, np.int64), np.array(sizes, np.int64)


def mp4_audio_track(data: bytes) -> Mp4Track:
    """The first sound track of an MP4 / M4A / MOV file: its codec configuration, the file offset and size of every
    access unit (stsz, stsc, stco / co64, then any moof fragments) and its first edit (elst), as ffmpeg's mov demuxer
    reads them."""
    moov = next(((a, b) for t, a, b in _mp4_boxes(data, 0, len(data)) if t == b"moov"), None)
    if moov is None:
        raise ValueError("MP4: no moov box" + (" (fragments without their initialization segment)" if b"moof" in
                                               data[:4096] else ""))
    movie_ts = 1000
    for t, a, b in _mp4_boxes(data, *moov):
        if t == b"mvhd":
            movie_ts = struct.unpack(">I", data[a + (20 if data[a] == 1 else 12): a + (24 if data[a] == 1 else 16)])[0]
    for t, a, b in _mp4_boxes(data, *moov):
        if t != b"trak":
            continue
        box = {}

        def walk(lo, hi):
            for tt, aa, bb in _mp4_boxes(data, lo, hi):
                if tt in (b"mdia", b"minf", b"stbl", b"edts"):
                    walk(aa, bb)
                else:
                    box.setdefault(tt, (aa, bb))
        walk(a, b)
        if b"hdlr" not in box or data[box[b"hdlr"][0] + 8: box[b"hdlr"][0] + 12] != b"soun":
            continue
        ha, _ = box[b"mdhd"]
        if data[ha] == 1:
            ts, dur = struct.unpack(">IQ", data[ha + 20: ha + 32])
        else:
            ts, dur = struct.unpack(">II", data[ha + 12: ha + 20])
        sa, sb = box[b"stsd"]
        ea = sa + 8  # (version / flags, entry count)
        esize, etype = struct.unpack(">I4s", data[ea: ea + 8])
        ver = struct.unpack(">H", data[ea + 16: ea + 18])[0]
        channels = struct.unpack(">H", data[ea + 24: ea + 26])[0]
        rate = struct.unpack(">I", data[ea + 32: ea + 36])[0] >> 16
        child = ea + 36 + {0: 0, 1: 16, 2: 36}.get(ver, 0)
        codec, cfg = None, b""
        if etype in (b".mp3", b"mp3 "):
            codec = "mp3"
        elif etype == b"alac":  # Apple Lossless: the ALACSpecificConfig in the entry's 'alac' child box
            for tt, aa, bb in _mp4_boxes(data, child, ea + esize):
                if tt == b"alac":
                    codec, cfg = "alac", data[aa + 4: bb]
        elif etype == b"mp4a":
            for tt, aa, bb in _mp4_boxes(data, child, ea + esize):
                if tt == b"esds":
                    oti, cfg = _esds_config(data, aa, bb)
                    codec = {0x40: "aac", 0x66: "aac-main", 0x67: "aac", 0x68: "aac-ssr", 0x69: "mp3",
                             0x6B: "mp3"}.get(oti, f"object type 0x{oti:02x}")
                    if oti == 0x67:  # MPEG-2 AAC LC: no AudioSpecificConfig object type of its own
                        cfg = cfg or bytes([0x10 | 0, 0])
        if codec is None:
            raise ValueError(f"MP4: sound track codec {etype.decode(errors='replace')!r} is not decoded")
        # sample table
        za, _ = box[b"stsz"]
        fixed, count = struct.unpack(">II", data[za + 4: za + 12])
        sizes = (np.full(count, fixed, np.int64) if fixed else
                 np.frombuffer(data, ">u4", count, za + 12).astype(np.int64))
        if b"co64" in box:
            ca, _ = box[b"co64"]
            chunks = np.frombuffer(data, ">u8", struct.unpack(">I", data[ca + 4: ca + 8])[0], ca + 8).astype(np.int64)
        else:
            ca, _ = box[b"stco"]
            chunks = np.frombuffer(data, ">u4", struct.unpack(">I", data[ca + 4: ca + 8])[0], ca + 8).astype(np.int64)
        qa, _ = box[b"stsc"]
        runs = np.frombuffer(data, ">u4", 3 * struct.unpack(">I", data[qa + 4: qa + 8])[0], qa + 8).reshape(-1, 3)
        per_chunk = np.zeros(len(chunks), np.int64)
        for i, (first, spc, _) in enumerate(runs):
            last = runs[i + 1][0] - 1 if i + 1 < len(runs) else len(chunks)
            per_chunk[int(first) - 1: int(last)] = int(spc)
        if int(per_chunk.sum()) < count:
            raise ValueError("MP4: the sample-to-chunk table covers fewer samples than stsz")
        chunk_of = np.repeat(np.arange(len(chunks)), per_chunk)[:count]
        first_in_chunk = np.concatenate([[0], np.cumsum(per_chunk)[:-1]])[chunk_of]
        csum = np.concatenate([[0], np.cumsum(sizes)])
        offsets = chunks[chunk_of] + csum[np.arange(count)] - csum[first_in_chunk]
        if b"trex" in box or any(t == b"mvex" for t, _, _ in _mp4_boxes(data, *moov)):
            extra_off, extra_siz = _fragment_samples(data, moov, a, b)
            offsets = np.concatenate([offsets, extra_off])
            sizes = np.concatenate([sizes, extra_siz])
            count = len(sizes)
        if count and int((offsets + sizes).max()) > len(data):
            raise ValueError("MP4: an access unit lies beyond the end of the file (truncated upload)")
        edit = None
        if b"elst" in box:
            la, _ = box[b"elst"]
            v, n = data[la], struct.unpack(">I", data[la + 4: la + 8])[0]
            fmt, w = (">Qq", 16) if v == 1 else (">Ii", 8)
            for i in range(n):
                sdur, mtime = struct.unpack(fmt, data[la + 8 + i * (w + 4): la + 8 + i * (w + 4) + w])
                if mtime >= 0:
                    edit = (int(mtime), int(round(sdur * ts / movie_ts)))
                    break
        return Mp4Track(codec, cfg, int(rate), int(channels), offsets, sizes, int(ts), edit, int(dur))
    raise ValueError("MP4: no sound track")


def decode_mp4(data: bytes, threads: int = 0) -> Tuple[np.ndarray, int]:
    """MP4 / M4A bytes -> f32 [frames, channels]: the first sound track (AAC-LC through tw_aac_decode_raw, MP3 through
    tw_mp3_decode, Apple Lossless through tw_alac_decode), trimmed by its first edit (elst media_time skipped, the edit's duration kept), as ffmpeg's mov
    demuxer presents it."""
    _lib, lib = _flac_lib()
    tr = mp4_audio_track(data)
    n = len(tr.sizes)
    if tr.codec == "mp3":
        au = b"".join(data[o: o + s] for o, s in zip(tr.offsets.tolist(), tr.sizes.tolist()))
        x, sr = decode_mp3(au, threads)
    elif tr.codec == "aac":
        info = _lib.TwAacInfo()
        if lib.tw_aac_parse_asc(ctypes.c_char_p(tr.config), len(tr.config), ctypes.byref(info)) != 0:
            raise ValueError(lib.tw_last_error().decode(errors="replace"))
        sr, ch = int(info.sample_rate), int(info.channels)
        if n * 1024 > max_audio_seconds() * sr:
            raise ValueError(f"MP4 track longer than TW_MAX_AUDIO_S={max_audio_seconds():g} s")
        x = np.zeros((n * 1024, ch), np.float32)
        off = np.ascontiguousarray(tr.offsets, np.int64)
        siz = np.ascontiguousarray(tr.sizes, np.int64)
        got = ctypes.c_int64()
        if lib.tw_aac_decode_raw(ctypes.c_char_p(tr.config), len(tr.config), ctypes.c_char_p(data), len(data),
                                 off.ctypes.data, siz.ctypes.data, n, x.ctypes.data, len(x), int(threads),
                                 ctypes.byref(got)) != 0:
            raise ValueError(lib.tw_last_error().decode(errors="replace"))
    elif tr.codec == "alac":
        info = _lib.TwAlacInfo()
        if lib.tw_alac_parse_cookie(ctypes.c_char_p(tr.config), len(tr.config), ctypes.byref(info)) != 0:
            raise ValueError(lib.tw_last_error().decode(errors="replace"))
        sr, ch = int(info.sample_rate) or tr.sample_rate, int(info.channels)
        cap = n * int(info.frame_length)
        if cap > max_audio_seconds() * sr:
            raise ValueError(f"MP4 track longer than TW_MAX_AUDIO_S={max_audio_seconds():g} s")
        x = np.zeros((cap, ch), np.float32)
        off = np.ascontiguousarray(tr.offsets, np.int64)
        siz = np.ascontiguousarray(tr.sizes, np.int64)
        got = ctypes.c_int64()
        if lib.tw_alac_decode(ctypes.c_char_p(tr.config), len(tr.config), ctypes.c_char_p(data), len(data),
                              off.ctypes.data, siz.ctypes.data, n, x.ctypes.data, cap, int(threads),
                              ctypes.byref(got)) != 0:
            raise ValueError(lib.tw_last_error().decode(errors="replace"))
        x = x[: got.value]
    else:
        raise ValueError(f"MP4 sound track codec {tr.codec} is not decoded (AAC-LC, MP3 and ALAC are)")
    if tr.edit is not None:
        scale = sr / tr.timescale
        skip, keep = int(round(tr.edit[0] * scale)), int(round(tr.edit[1] * scale))
        x = x[skip: skip + keep] if keep else x[skip:]  # (a zero-length edit, as fragmented files write: to the end)
    return x, sr


def g711_decode(codes: bytes, alaw: bool) -> np.ndarray:
    """G.711 mu-law / A-law bytes -> int16 (native tw_g711_decode: the ITU-T tables ffmpeg's pcm_mulaw / pcm_alaw
    use)."""
    _lib, lib = _flac_lib()
    src = np.frombuffer(codes, np.uint8)
    out = np.empty(len(src), np.int16)
    if lib.tw_g711_decode(src.ctypes.data, len(src), int(alaw), out.ctypes.data) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return out


def ima_adpcm_wav_decode(data: bytes, channels: int, block_align: int) -> np.ndarray:
    """Microsoft IMA ADPCM blocks (WAV format tag 0x11) -> int16 [frames, channels] (native
    tw_ima_adpcm_wav_decode; ffmpeg's adpcm_ima_wav)."""
    _lib, lib = _flac_lib()
    if block_align < 4 * channels:
        raise ValueError(f"IMA ADPCM block_align {block_align} < 4 x {channels} channels")
    per = 1 + ((block_align - 4 * channels) // (4 * channels)) * 8
    cap = (len(data) // block_align + 1) * per
    if cap > max_audio_seconds() * 192000:
        raise ValueError("IMA ADPCM stream longer than TW_MAX_AUDIO_S")
    out = np.zeros((cap, channels), np.int16)
    got = ctypes.c_int64()
    src = np.frombuffer(data, np.uint8)
    if lib.tw_ima_adpcm_wav_decode(src.ctypes.data, len(src), channels, block_align, out.ctypes.data, cap,
                                   ctypes.byref(got)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return out[: got.value]


def ms_adpcm_wav_decode(data: bytes, channels: int, block_align: int) -> np.ndarray:
    """Microsoft ADPCM blocks (WAV format tag 2) -> int16 [frames, channels] (native tw_ms_adpcm_wav_decode;
    ffmpeg's adpcm_ms)."""
    _lib, lib = _flac_lib()
    if channels not in (1, 2) or block_align < 7 * channels:
        raise ValueError(f"MS ADPCM with {channels} channels, block_align {block_align} (1-2 channels, >= 7 each)")
    cap = (len(data) // block_align + 1) * ((block_align - 6 * channels) * 2 // channels)
    if cap > max_audio_seconds() * 192000:
        raise ValueError("MS ADPCM stream longer than TW_MAX_AUDIO_S")
    out = np.zeros((cap, channels), np.int16)
    got = ctypes.c_int64()
    src = np.frombuffer(data, np.uint8)
    if lib.tw_ms_adpcm_wav_decode(src.ctypes.data, len(src), channels, block_align, out.ctypes.data, cap,
                                  ctypes.byref(got)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return out[: got.value]


def ima_qt_decode(data: bytes, channels: int) -> np.ndarray:
    """Apple IMA4 packets (AIFF-C 'ima4') -> int16 [frames, channels] (native tw_ima_qt_decode; ffmpeg's
    adpcm_ima_qt)."""
    _lib, lib = _flac_lib()
    if not 1 <= channels <= 8:
        raise ValueError(f"IMA4 with {channels} channels (1-8 supported)")
    cap = len(data) // (34 * channels) * 64
    if cap > max_audio_seconds() * 192000:
        raise ValueError("IMA4 stream longer than TW_MAX_AUDIO_S")
    out = np.zeros((cap, channels), np.int16)
    got = ctypes.c_int64()
    src = np.frombuffer(data, np.uint8)
    if lib.tw_ima_qt_decode(src.ctypes.data, len(src), channels, out.ctypes.data, cap, ctypes.byref(got)) != 0:
        raise ValueError(lib.tw_last_error().decode(errors="replace"))
    return out[: got.value]


def _pcm_to_float(raw: bytes, bits: int, big_endian: bool = False, unsigned8: bool = True) -> np.ndarray:
    """Integer PCM -> float32 in [-1, 1) the way ffmpeg's s8/s16/s24/s32/s64 -> flt conversion scales
    (2^-(bits-1))."""
    e = ">" if big_endian else "<"
    if bits == 64:
        return (np.frombuffer(raw[: len(raw) // 8 * 8], e + "i8").astype(np.float64) / 9223372036854775808.0
                ).astype(np.float32)
    if bits == 8:
        v = np.frombuffer(raw, np.uint8 if unsigned8 else np.int8).astype(np.float32)
        return (v - 128.0) / 128.0 if unsigned8 else v / 128.0
    if bits == 16:
        return np.frombuffer(raw[: len(raw) // 2 * 2], e + "i2").astype(np.float32) / 32768.0
    if bits == 24:
        b = np.frombuffer(raw[: len(raw) // 3 * 3], np.uint8).reshape(-1, 3).astype(np.int32)
        if big_endian:
            b = b[:, ::-1]
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        return v.astype(np.float32) / float(1 << 23)
    if bits == 32:
        return np.frombuffer(raw[: len(raw) // 4 * 4], e + "i4").astype(np.float32) / 2147483648.0
    raise ValueError(f"unsupported PCM width {bits}")


def _frames(x: np.ndarray, ch: int) -> np.ndarray:
    n = len(x) // ch
    return x[: n * ch].reshape(n, ch)


def decode_wav(data: bytes) -> Tuple[np.ndarray, int]:
    """RIFF/WAVE bytes -> (float32 [frames, channels] in [-1, 1], sample_rate), as ffmpeg's wav demuxer reads them
    (libavformat/wavdec.c): "RIFF" little-endian, "RIFX" big-endian, "RF64" with its ds64 chunk's 64-bit data size.
    Format tags: 1 PCM in 1 / 2 / 3 / 4 / 8-byte containers (bits per sample rounded up to whole bytes, as
    ff_get_pcm_codec_id maps them: a 20-bit stream is s24, a 12-bit one s16, a 5-bit one u8; 5-7-byte containers are
    refused, as ffmpeg refuses them), 3 IEEE float 32 / 64, 6 A-law, 7 mu-law, 0x11 IMA ADPCM, 2 Microsoft ADPCM,
    0x55 MP3 and 0x50 MPEG Layer I / II (the data chunk through the MPEG audio decoder), and WAVE_FORMAT_EXTENSIBLE
    carrying any of them. A data chunk that runs past the end of the bytes is read up to it."""
    if len(data) < 12 or data[:4] not in (b"RIFF", b"RIFX", b"RF64") or data[8:12] != b"WAVE":
        raise ValueError("not a RIFF/WAVE stream")
    be = data[:4] == b"RIFX"
    e = ">" if be else "<"
    u16, u32 = e + "H", e + "I"
    pos, fmt, pcm, ds64_data = 12, None, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos: pos + 4], struct.unpack(u32, data[pos + 4: pos + 8])[0]
        if cid == b"ds64" and size >= 16:  # RF64: riff size, data size (64-bit each), sample count
            ds64_data = struct.unpack("<Q", data[pos + 16: pos + 24])[0]
        if cid == b"data" and size == 0xFFFFFFFF and ds64_data is not None:
            size = ds64_data
        body = data[pos + 8: pos + 8 + size]
        if cid == b"fmt ":
            if len(body) < 16:
                raise ValueError("WAVE fmt chunk too short")
            tag, ch = struct.unpack(e + "HH", body[:4])
            sr = struct.unpack(u32, body[4:8])[0]
            align, bits = struct.unpack(e + "HH", body[12:16])
            if tag == 0xFFFE and len(body) >= 28:  # WAVE_FORMAT_EXTENSIBLE: the subformat GUID's Data1 (its low 16
                tag = struct.unpack(u32, body[24:28])[0] & 0xFFFF  # bits are the format tag), in the file's byte order
            fmt = (tag, ch, sr, bits, align)
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError("WAVE stream without fmt/data chunks")
    tag, ch, sr, bits, align = fmt
    if ch < 1:
        raise ValueError("WAVE stream with no channels")
    if tag == 1:
        width = (bits + 7) // 8
        if bits < 1 or width not in (1, 2, 3, 4, 8):
            raise ValueError(f"unsupported PCM width {bits}")
        x = _pcm_to_float(pcm, 8 * width, big_endian=be)
    elif tag == 3:
        if bits not in (32, 64):
            raise ValueError(f"unsupported IEEE float width {bits}")
        w = bits // 8
        x = np.frombuffer(pcm[: len(pcm) // w * w], e + ("f4" if w == 4 else "f8")).astype(np.float32)
    elif tag in (6, 7):
        x = g711_decode(pcm, alaw=tag == 6).astype(np.float32) / 32768.0
    elif tag == 0x11:
        if bits != 4:
            raise ValueError(f"IMA ADPCM with {bits} bits per sample (4 supported)")
        return ima_adpcm_wav_decode(pcm, ch, align).astype(np.float32) / 32768.0, sr
    elif tag == 2:
        return ms_adpcm_wav_decode(pcm, ch, align).astype(np.float32) / 32768.0, sr
    elif tag in (0x50, 0x55):  # MPEG audio in a WAV wrapper: the stream's own headers give rate and channels
        return decode_mp3(bytes(pcm))
    else:
        raise ValueError(f"unsupported WAVE format tag {tag}")
    return _frames(x, ch), sr


# Sun/NeXT .au encodings (ffmpeg's au demuxer): 1 mu-law, 2/3/4/5 big-endian signed PCM 8/16/24/32, 6/7 float 32/64,
# 27 A-law
def decode_au(data: bytes) -> Tuple[np.ndarray, int]:
    """Sun .au / .snd bytes -> (float32 [frames, channels], sample_rate)."""
    if len(data) < 24 or data[:4] != b".snd":
        raise ValueError("not a Sun .au stream")
    off, size, enc, sr, ch = struct.unpack(">IIIII", data[4:24])
    if ch < 1 or off < 24:
        raise ValueError("bad .au header")
    body = data[off:] if size == 0xFFFFFFFF else data[off: off + size]
    if enc == 1 or enc == 27:
        x = g711_decode(body, alaw=enc == 27).astype(np.float32) / 32768.0
    elif enc in (2, 3, 4, 5):
        x = _pcm_to_float(body, 8 * (enc - 1), big_endian=True, unsigned8=False)
    elif enc in (6, 7):
        w = 4 if enc == 6 else 8
        x = np.frombuffer(body[: len(body) // w * w], ">f4" if enc == 6 else ">f8").astype(np.float32)
    else:
        raise ValueError(f"unsupported .au encoding {enc}")
    return _frames(x, ch), sr


def _ieee_extended(b: bytes) -> float:
    """80-bit IEEE 754 extended (AIFF COMM sampleRate)."""
    exp = struct.unpack(">H", b[:2])[0]
    mant = struct.unpack(">Q", b[2:10])[0]
    sign = -1.0 if exp & 0x8000 else 1.0
    exp &= 0x7FFF
    if exp == 0 and mant == 0:
        return 0.0
    return sign * mant * 2.0 ** (exp - 16383 - 63)


def decode_aiff(data: bytes) -> Tuple[np.ndarray, int]:
    """AIFF / AIFF-C bytes -> (float32 [frames, channels], sample_rate). Compression types: NONE / twos (big-endian
    PCM), sowt (little-endian PCM), in24 / in32, raw (unsigned 8-bit), fl32 / fl64, ulaw, alaw, ima4 (Apple IMA
    ADPCM) (ffmpeg's aiff demuxer)."""
    if len(data) < 12 or data[:4] != b"FORM" or data[8:12] not in (b"AIFF", b"AIFC"):
        raise ValueError("not an AIFF stream")
    aifc = data[8:12] == b"AIFC"
    pos, comm, ssnd = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos: pos + 4], struct.unpack(">I", data[pos + 4: pos + 8])[0]
        body = data[pos + 8: pos + 8 + size]
        if cid == b"COMM":
            ch, nframes, bits = struct.unpack(">hIh", body[:8])
            sr = _ieee_extended(body[8:18])
            ctype = body[18:22] if aifc and len(body) >= 22 else b"NONE"
            comm = (ch, nframes, bits, sr, ctype)
        elif cid == b"SSND":
            offset = struct.unpack(">I", body[:4])[0]
            ssnd = body[8 + offset:]
        pos += 8 + size + (size & 1)
    if comm is None or ssnd is None:
        raise ValueError("AIFF stream without COMM/SSND chunks")
    ch, nframes, bits, sr, ctype = comm
    if ch < 1:
        raise ValueError("AIFF stream with no channels")
    if ctype in (b"NONE", b"twos"):
        x = _pcm_to_float(ssnd, (bits + 7) // 8 * 8, big_endian=True, unsigned8=False)
    elif ctype == b"sowt":
        x = _pcm_to_float(ssnd, (bits + 7) // 8 * 8, big_endian=False, unsigned8=False)
    elif ctype in (b"in24", b"in32"):  # big-endian s24 / s32 whatever COMM's depth says
        x = _pcm_to_float(ssnd, 24 if ctype == b"in24" else 32, big_endian=True, unsigned8=False)
    elif ctype == b"raw ":  # unsigned 8-bit
        x = _pcm_to_float(ssnd, 8, unsigned8=True)
    elif ctype in (b"fl32", b"FL32"):
        x = np.frombuffer(ssnd[: len(ssnd) // 4 * 4], ">f4").astype(np.float32)
    elif ctype in (b"fl64", b"FL64"):
        x = np.frombuffer(ssnd[: len(ssnd) // 8 * 8], ">f8").astype(np.float32)
    elif ctype in (b"ulaw", b"ULAW", b"alaw", b"ALAW"):
        x = g711_decode(ssnd, alaw=ctype.lower() == b"alaw").astype(np.float32) / 32768.0
    elif ctype == b"ima4":  # every whole 34-byte-per-channel packet of SSND, as ffmpeg's demuxer hands them over
        return ima_qt_decode(ssnd, ch).astype(np.float32) / 32768.0, int(round(sr))
    else:
        raise ValueError(f"unsupported AIFF-C compression {ctype!r}")
    fr = _frames(x, ch)
    return fr[:nframes], int(round(sr))


def resample(x: np.ndarray, sr_in: int, sr_out: int = TARGET_SR, device=None) -> np.ndarray:
    """Mono/multi-channel float -> mono float32 at sr_out (GPU when the rates differ)."""
    if sr_in == sr_out:
        x = np.asarray(x, np.float32)
        return x if x.ndim == 1 else x.mean(axis=1, dtype=np.float32)
    return resample_device(np.asarray(x, np.float32), sr_in, sr_out, device=device).cpu().numpy()


def max_audio_seconds() -> float:
    """Longest input decoded (env TW_MAX_AUDIO_S, default 4 h): caps a container's claimed length before any
    allocation."""
    return float(os.environ.get("TW_MAX_AUDIO_S", "14400"))


# Containers the engine recognises but does not decode (no AAC / Opus decoder is built in): reported by name, as a
# ValueError like the reference's own decode failure (ffmpeg_read, which its transcribe() turns into its
# {"error": ...} result).
_UNDECODED = ((b"OggS", "Ogg"), (b"\x1aE\xdf\xa3", "Matroska/WebM"))


def _ogg_packets(data: bytes) -> List[bytes]:
    """The packets of an Ogg file's first logical stream (its pages' segments joined by lacing; other streams'
    pages skipped), as ffmpeg's ogg demuxer hands them to a decoder."""
    pos, serial, packets, cur = 0, None, [], b""
    while pos + 27 <= len(data) and data[pos: pos + 4] == b"OggS":
        nseg = data[pos + 26]
        lacing = data[pos + 27: pos + 27 + nseg]
        sn = struct.unpack("<I", data[pos + 14: pos + 18])[0]
        serial = sn if serial is None else serial
        off = pos + 27 + nseg
        for n in lacing:
            if sn == serial:
                cur += data[off: off + n]
                if n < 255:
                    packets.append(cur)
                    cur = b""
            off += n
        pos = off
    return packets


def ogg_flac_to_native(data: bytes) -> bytes:
    """Ogg FLAC (the FLAC-to-Ogg mapping: a first packet "\x7fFLAC" + version + header count + "fLaC" + STREAMINFO,
    then metadata-block packets, then one FLAC frame per packet) -> the native FLAC stream those bytes carry."""
    packets = _ogg_packets(data)
    if not packets or packets[0][:5] != b"\x7fFLAC" or packets[0][9:13] != b"fLaC" or len(packets[0]) < 13 + 38:
        raise ValueError("Ogg FLAC: no FLAC mapping header")
    si = bytearray(packets[0][13: 13 + 38])
    si[0] |= 0x80  # STREAMINFO becomes the last metadata block
    k = 1
    while k < len(packets) and packets[k][:1] != b"\xff":  # the metadata-block packets (their count may be 0 = unknown)
        k += 1
    return b"fLaC" + bytes(si) + b"".join(packets[k:])


def _id3v2_end(data: bytes) -> int:
    pos = 0
    while data[pos: pos + 3] == b"ID3" and pos + 10 <= len(data):
        flags, b = data[pos + 5], data[pos + 6: pos + 10]
        pos += 10 + ((b[0] & 127) << 21 | (b[1] & 127) << 14 | (b[2] & 127) << 7 | (b[3] & 127))
        pos += 10 if flags & 0x10 else 0  # (a footer)
    return pos


def _mpeg_audio_name(data: bytes) -> Optional[str]:
    """MPEG audio frames (after any ID3v2 tags): Layers I, II and III (all decoded by csrc/mp3.cpp, as ffmpeg's mp3
    demuxer takes every layer), or ADTS AAC."""
    pos = _id3v2_end(data)
    h = data[pos: pos + 2]
    if len(h) == 2 and h[0] == 0xFF and (h[1] & 0xE0) == 0xE0:
        layer = (h[1] >> 1) & 3
        if (h[1] & 0xF6) == 0xF0:  # 12-bit sync with layer 00: ADTS
            return "AAC (ADTS)"
        if (h[1] >> 3) & 3 != 1 and layer:
            return {1: "MP3", 2: "MPEG audio Layer II", 3: "MPEG audio Layer I"}[layer]
    if pos:  # an ID3v2 tag followed by something else: let the MP3 frame search decide
        return "MP3"
    return None
# transformers' ffmpeg_read message for a payload ffmpeg cannot decode (pipelines/audio_utils.py)
MALFORMED = ("Soundfile is either not in the correct format or is malformed. Ensure that the soundfile has a valid "
             "audio file extension (e.g. wav, flac or mp3) and is not corrupted. If reading from a remote URL, ensure "
             "that the URL is the full address to **download** the audio file.")


def container_name(data: bytes) -> Optional[str]:
    if data[:4] in (b"RIFF", b"RIFX", b"RF64") and data[8:12] == b"WAVE":
        return "WAV"
    if data[:4] == b"fLaC":
        return "FLAC"
    if data[:4] == b".snd":
        return "AU"
    if data[:4] == b"FORM" and data[8:12] in (b"AIFF", b"AIFC"):
        return "AIFF"
    if data[4:8] == b"ftyp":
        return "MP4/M4A"
    if data[:4] == b"OggS":
        head = data[28: 28 + 8]  # the first packet of a one-segment first page (every Ogg codec's header packet)
        if head[:7] == b"\x01vorbis":
            return "Ogg Vorbis"
        if head[:5] == b"\x7fFLAC":
            return "Ogg FLAC"
        return "Ogg Opus" if head == b"OpusHead" else "Ogg"
    for magic, name in _UNDECODED:
        if data.startswith(magic):
            return name
    return _mpeg_audio_name(data)


_DECODERS = {"WAV": decode_wav, "AU": decode_au, "AIFF": decode_aiff, "Ogg Vorbis": decode_vorbis, "MP3": decode_mp3,
             "MPEG audio Layer II": decode_mp3, "MPEG audio Layer I": decode_mp3, "AAC (ADTS)": decode_aac_adts,
             "MP4/M4A": decode_mp4}
DECODED = "FLAC (native, Ogg), Ogg Vorbis, MP3 / MPEG audio (MPEG-1 / 2 / 2.5 Layers I, II, III), AAC-LC / ALAC (M4A / MP4), AAC (ADTS), WAV / " \
          "RIFX / RF64 (PCM, float, A-law, mu-law, IMA / MS ADPCM, MPEG), AU, AIFF / AIFF-C"


def decode_bytes(data: bytes, sr_out: int = TARGET_SR, device=None) -> np.ndarray:
    name = container_name(data)
    if name in _DECODERS:
        x, sr = _DECODERS[name](data)
        return resample(x.mean(axis=1) if x.shape[1] > 1 else x[:, 0], sr, sr_out, device)
    if name in ("FLAC", "Ogg FLAC"):
        fl = decode_flac(data if name == "FLAC" else ogg_flac_to_native(data))
        scale = 2.0 ** -(fl.bits_per_sample - 1)  # ffmpeg's s16/s32 -> flt conversion of the coded samples
        return resample_device(fl.pcm, fl.sample_rate, sr_out, scale=scale, device=device).cpu().numpy()
    if name is None:
        raise ValueError(MALFORMED)
    raise ValueError(f"{name} audio is not decoded by this engine (decoded containers: {DECODED}); convert the "
                     "upload to one of them")


def load_input(inputs: Union[str, bytes, np.ndarray, dict], sr_out: int = TARGET_SR, device=None) -> np.ndarray:
    """Any pipeline input -> mono float32 at sr_out."""
    if isinstance(inputs, str):
        if inputs.startswith("http://") or inputs.startswith("https://"):
            raise ValueError("remote audio URLs are not fetched (no network)")
        with open(inputs, "rb") as f:
            inputs = f.read()
    if isinstance(inputs, (bytes, bytearray)):
        return decode_bytes(bytes(inputs), sr_out, device)
    if isinstance(inputs, dict):
        d = dict(inputs)
        if not ("sampling_rate" in d and ("raw" in d or "array" in d)):
            raise ValueError('a dict input needs a "raw" or "array" key and a "sampling_rate" key')
        arr = d.get("raw")
        if arr is None:
            arr = d.get("array")
        arr = np.asarray(arr, dtype=np.float32)
        if arr.ndim != 1:
            arr = arr.mean(axis=0)
        return resample(arr, int(d["sampling_rate"]), sr_out, device)
    if hasattr(inputs, "cpu") and hasattr(inputs, "numpy"):  # torch tensor
        inputs = inputs.cpu().numpy()
    if isinstance(inputs, np.ndarray):
        x = inputs.astype(np.float32, copy=False)
        if x.ndim != 1:
            x = x.mean(axis=0)
        return x
    raise TypeError(f"We expect a numpy ndarray or torch tensor as input, got `{type(inputs)}`")


def duration_seconds(path: str) -> float:
    """Duration of an audio file (the reference's get_audio_duration, vocalis/core/audio_utils.py:78-98, via
    librosa; here from the decoded stream)."""
    with open(path, "rb") as f:
        data = f.read()
    name = container_name(data)
    if name == "Ogg Vorbis":
        info = vorbis_probe(data)
        return int(info.total_samples) / float(info.sample_rate)
    if name in ("MP3", "MPEG audio Layer II", "MPEG audio Layer I"):
        info = mp3_probe(data)
        return int(info.total_samples) / float(info.sample_rate)
    if name == "AAC (ADTS)":
        info = aac_adts_probe(data)
        return int(info.total_samples) / float(info.sample_rate)
    if name in _DECODERS:
        x, sr = _DECODERS[name](data)
        return x.shape[0] / float(sr)
    if name in ("FLAC", "Ogg FLAC"):
        info = flac_probe(data if name == "FLAC" else ogg_flac_to_native(data))
        return int(info.total_samples) / float(info.sample_rate)
    raise ValueError("duration: unsupported container")


def write_wav(path_or_buf, x: np.ndarray, sr: int = TARGET_SR) -> None:
    """16-bit PCM mono WAV writer (test fixtures, examples)."""
    pcm = np.clip(np.round(np.asarray(x, np.float64) * 32767.0), -32768, 32767).astype("<i2").tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(pcm)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, sr, sr * 2, 2, 16)
    hdr += b"data" + struct.pack("<I", len(pcm))
    if isinstance(path_or_buf, (str, bytes)) and not isinstance(path_or_buf, io.IOBase):
        with open(path_or_buf, "wb") as f:
            f.write(hdr + pcm)
    else:
        path_or_buf.write(hdr + pcm)
