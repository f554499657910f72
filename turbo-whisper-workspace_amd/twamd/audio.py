"""Audio ingest for the transcriber (host side, before the GPU path).

Mirrors the input handling of AutomaticSpeechRecognitionPipeline.preprocess
($TF/pipelines/automatic_speech_recognition.py:345-420): a path is read as bytes, bytes are decoded
to mono f32 at 16 kHz (the reference shells out to ffmpeg, $TF/pipelines/audio_utils.py:9-45, which
this image does not have), dicts carry {"raw"|"array", "sampling_rate"} and are resampled when the
rate differs, multi-channel arrays are averaged to mono.

Decoders here: RIFF/WAVE (PCM 8/16/24/32-bit, IEEE float 32/64). Resampling uses a polyphase
windowed-sinc filter (scipy.signal.resample_poly); ffmpeg's resampler is not bit-reproducible,
so no reference value is claimed for resampled input.
"""
from __future__ import annotations

import io
import struct
from fractions import Fraction
from typing import Tuple, Union

import numpy as np

TARGET_SR = 16000


def decode_wav(data: bytes) -> Tuple[np.ndarray, int]:
    """RIFF/WAVE bytes -> (float32 [frames, channels] in [-1, 1], sample_rate)."""
    if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError("not a RIFF/WAVE stream")
    pos, fmt, pcm = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos: pos + 4], struct.unpack("<I", data[pos + 4: pos + 8])[0]
        body = data[pos + 8: pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, sr, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:  # WAVE_FORMAT_EXTENSIBLE: subformat GUID's first 2 bytes
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, sr, bits)
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError("WAVE stream without fmt/data chunks")
    tag, ch, sr, bits = fmt
    if tag == 1:
        if bits == 8:
            x = (np.frombuffer(pcm, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif bits == 16:
            x = np.frombuffer(pcm[: len(pcm) // 2 * 2], "<i2").astype(np.float32) / 32768.0
        elif bits == 24:
            b = np.frombuffer(pcm[: len(pcm) // 3 * 3], np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = v.astype(np.float32) / float(1 << 23)
        elif bits == 32:
            x = np.frombuffer(pcm[: len(pcm) // 4 * 4], "<i4").astype(np.float32) / 2147483648.0
        else:
            raise ValueError(f"unsupported PCM width {bits}")
    elif tag == 3:
        x = np.frombuffer(pcm, "<f4" if bits == 32 else "<f8").astype(np.float32)
    else:
        raise ValueError(f"unsupported WAVE format tag {tag}")
    n = len(x) // ch
    return x[: n * ch].reshape(n, ch), sr


def resample(x: np.ndarray, sr_in: int, sr_out: int = TARGET_SR) -> np.ndarray:
    if sr_in == sr_out:
        return x.astype(np.float32, copy=False)
    from scipy.signal import resample_poly

    fr = Fraction(sr_out, sr_in).limit_denominator(1000)
    return resample_poly(x.astype(np.float64), fr.numerator, fr.denominator).astype(np.float32)


def decode_bytes(data: bytes, sr_out: int = TARGET_SR) -> np.ndarray:
    if data[:4] == b"RIFF":
        x, sr = decode_wav(data)
        return resample(x.mean(axis=1) if x.shape[1] > 1 else x[:, 0], sr, sr_out)
    if data[:4] == b"fLaC":
        raise NotImplementedError("FLAC decoding is not implemented yet (the reference relies on ffmpeg); "
                                  "convert to WAV or pass a decoded array")
    raise ValueError("unrecognised audio container (supported: RIFF/WAVE)")


def load_input(inputs: Union[str, bytes, np.ndarray, dict], sr_out: int = TARGET_SR) -> np.ndarray:
    """Any pipeline input -> mono float32 at sr_out."""
    if isinstance(inputs, str):
        if inputs.startswith("http://") or inputs.startswith("https://"):
            raise ValueError("remote audio URLs are not fetched (no network)")
        with open(inputs, "rb") as f:
            inputs = f.read()
    if isinstance(inputs, (bytes, bytearray)):
        return decode_bytes(bytes(inputs), sr_out)
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
        return resample(arr, int(d["sampling_rate"]), sr_out)
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
    if data[:4] == b"RIFF":
        x, sr = decode_wav(data)
        return x.shape[0] / float(sr)
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
