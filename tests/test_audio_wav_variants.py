"""WAV variants of the reference's upload path (ffmpeg_read: $TF/pipelines/audio_utils.py:9-45, ffmpeg's wav demuxer
libavformat/wavdec.c), pinned to an independent reader: scipy.io.wavfile over scipy's own WAV test files (present in
this image), scaled the way ffmpeg converts integer PCM to float (2^-(container bits - 1); u8 centred at 128).

Covered: RIFF little-endian, RIFX big-endian, RF64 (ds64 data size), WAVE_FORMAT_EXTENSIBLE, PCM in 1 / 2 / 3 / 4 /
8-byte containers including sub-container bit depths (5-bit in u8, 12-bit in s16, 20-bit in s24, left-justified:
the container's scale, as ff_get_pcm_codec_id maps them), IEEE float 32 / 64 little- and big-endian, a data chunk
running past the end of the file (read up to it), a header whose nAvgBytesPerSec disagrees (ignored). Refused as
ffmpeg refuses them: 5-7-byte PCM containers (36 / 45 / 53-bit), a stream without a data chunk."""
import glob
import os
import struct
import warnings

import numpy as np
import pytest

from twamd import audio

DATA = "/usr/local/lib/python3.10/dist-packages/scipy/io/tests/data/"
FILES = sorted(glob.glob(DATA + "test-*.wav"))
REFUSED = {"36bit", "45bit", "53bit"}  # 5-7-byte containers: no ffmpeg PCM codec


def _ffmpeg_scale(ref: np.ndarray, bits: int) -> np.ndarray:
    """scipy's integer samples -> ffmpeg's float: scipy returns sub-container depths left-justified in the container
    (so the container's scale applies), u8 unsigned."""
    if ref.dtype == np.uint8:
        return (ref.astype(np.float64) - 128.0) / 128.0
    if ref.dtype.kind == "f":
        return ref.astype(np.float64)
    return ref.astype(np.float64) / float(2 ** (8 * ref.dtype.itemsize - 1))


@pytest.mark.skipif(not FILES, reason="scipy's WAV test data is not in this image")
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_scipy_wav_files(path):
    name = os.path.basename(path)
    data = open(path, "rb").read()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            sr, ref = __import__("scipy.io.wavfile", fromlist=["read"]).read(path)
        except ValueError:
            ref = None
    if any(r in name for r in REFUSED) or "no-data" in name or "incomplete-chunk" in name:
        with pytest.raises(ValueError):
            audio.decode_wav(data)
        return
    if "ulaw" in name:  # (scipy does not read mu-law; the G.711 decoder has its own pins, test_audio_codecs.py)
        x, sr2 = audio.decode_wav(data)
        assert sr2 == 8000 and x.shape[1] == 1
        return
    x, sr2 = audio.decode_wav(data)
    assert audio.container_name(data) == "WAV"
    if "inconsistent" in name:  # scipy refuses the header; ffmpeg reads it: compare with the consistent twin
        ref_x, _ = audio.decode_wav(open(path.replace("-inconsistent", ""), "rb").read())
        assert np.array_equal(x, ref_x)
        return
    assert ref is not None, name
    if ref.ndim == 1:
        ref = ref[:, None]
    exp = _ffmpeg_scale(ref, 0)
    assert sr2 == sr and x.shape == exp.shape, (name, x.shape, exp.shape)
    tol = 1e-7 if ref.dtype.kind == "f" else 2.0 ** -23  # float32 rounding of the scaled integers
    assert np.abs(x.astype(np.float64) - exp).max() <= tol, name


def _wav(fourcc: bytes, fmt_body: bytes, pcm: bytes, be: bool = False, ds64: bool = False) -> bytes:
    u32 = ">I" if be else "<I"
    chunks = b""
    if ds64:
        chunks += b"ds64" + struct.pack("<I", 28) + struct.pack("<QQQI", 0, len(pcm), 0, 0)
    chunks += b"fmt " + struct.pack(u32, len(fmt_body)) + fmt_body
    chunks += b"data" + (struct.pack("<I", 0xFFFFFFFF) if ds64 else struct.pack(u32, len(pcm))) + pcm
    return fourcc + struct.pack(u32, 0xFFFFFFFF if ds64 else 4 + len(chunks)) + b"WAVE" + chunks


@pytest.mark.parametrize("bits,width", [(5, 1), (8, 1), (12, 2), (16, 2), (20, 3), (24, 3), (32, 4), (64, 8)])
@pytest.mark.parametrize("form", ["RIFF", "RIFX", "RF64"])
def test_written_streams(bits, width, form):
    """Synthetic streams of every container width and byte order: values left-justified in their containers."""
    rng = np.random.default_rng(bits * 7 + len(form))
    n, ch, be = 33, 2, form == "RIFX"
    top = 2 ** (bits - 1)
    v = rng.integers(-top, top, size=(n, ch), dtype=np.int64) << (8 * width - bits)  # left-justified
    if width == 1:
        raw = (v + 128).astype(np.uint8).tobytes()
        exp = v.astype(np.float64) / 128.0
    else:
        dt = {2: "i2", 3: None, 4: "i4", 8: "i8"}[width]
        if dt is None:
            u = (v & 0xFFFFFF).astype(np.uint32)
            b = np.stack([(u >> s) & 0xFF for s in ((16, 8, 0) if be else (0, 8, 16))], -1).astype(np.uint8)
            raw = b.tobytes()
        else:
            raw = v.astype((">" if be else "<") + dt).tobytes()
        exp = v.astype(np.float64) / float(2 ** (8 * width - 1))
    e = ">" if be else "<"
    fmt = struct.pack(e + "HHIIHH", 1, ch, 16000, 16000 * ch * width, ch * width, bits)
    data = _wav(form.encode(), fmt, raw, be=be, ds64=form == "RF64")
    x, sr = audio.decode_wav(data)
    assert sr == 16000 and x.shape == (n, ch)
    assert np.abs(x.astype(np.float64) - exp).max() <= 2.0 ** -23 * (1 if width < 8 else 2)
    assert audio.container_name(data) == "WAV"


def test_float_big_endian_and_truncated_data():
    x = np.linspace(-1, 1, 40, dtype=np.float32).reshape(20, 2)
    fmt = struct.pack(">HHIIHH", 3, 2, 22050, 22050 * 8, 8, 32)
    data = _wav(b"RIFX", fmt, x.astype(">f4").tobytes(), be=True)
    got, sr = audio.decode_wav(data)
    assert sr == 22050 and np.array_equal(got, x)
    # a data chunk announcing more bytes than the file holds: read up to the end (whole frames)
    cut = data[:-12]
    got2, _ = audio.decode_wav(cut)
    assert np.array_equal(got2, x[: len(got2)]) and len(got2) == 18
