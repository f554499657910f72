"""Audio ingest on the MI355X: the GPU resampler (tw_resample_pcm_*) against the oracle's float64 restatement of
libswresample's default filter, and FLAC / Ogg Vorbis / MP3 (and MPEG Layers I / II) / AAC (M4A, ADTS) / ALAC files through
the full product path (host decode -> GPU resample -> transcription). Tolerance: 2e-6 absolute on [-1, 1] signals (float32 accumulation of <= 396 taps)."""
import numpy as np
import pytest
import torch

from oracle import audio_oracle as ao
from twamd import audio
from twamd.synth_audio import speech_like

pytestmark = pytest.mark.gpu
TOL = 2e-6


def _sig(sr, seconds, ch, seed):
    rng = np.random.default_rng(seed)
    n = int(sr * seconds)
    t = np.arange(n) / sr
    x = np.stack([0.5 * np.sin(2 * np.pi * (440 + 97 * c) * t) + 0.1 * rng.standard_normal(n) for c in range(ch)], 1)
    return np.clip(x, -1, 1)


@pytest.mark.parametrize("sr_in,ch", [(192000, 1), (44100, 2), (48000, 1), (22050, 1), (8000, 1), (32000, 2)])
def test_resample_f32_matches_oracle(sr_in, ch):
    x = _sig(sr_in, 0.37, ch, sr_in).astype(np.float32)
    got = audio.resample_device(x, sr_in, 16000).cpu().numpy()
    ref = ao.swr_resample(x.astype(np.float64).mean(axis=1), sr_in, 16000)
    assert got.shape == ref.shape == (-(-len(x) * 16000 // sr_in),)
    assert np.abs(got - ref).max() < TOL


def test_resample_i32_pcm_matches_oracle():
    pcm = np.round(_sig(192000, 0.5, 2, 3) * 32767).astype(np.int32)
    got = audio.resample_device(pcm, 192000, 16000, scale=2.0 ** -15).cpu().numpy()
    ref = ao.swr_resample(pcm.astype(np.float64).mean(axis=1) / 32768.0, 192000, 16000)
    assert np.abs(got - ref).max() < TOL


def test_resample_long_signal_properties():
    """Full-size sanity at one hour of 192 kHz audio would be 2.8 GB; use 60 s: a 1 kHz tone stays a 1 kHz tone
    of the same amplitude, a tone above the 8 kHz cutoff is removed."""
    sr = 192000
    t = np.arange(sr * 60) / sr
    lo = (0.5 * np.sin(2 * np.pi * 1000 * t)).astype(np.float32)
    hi = (0.5 * np.sin(2 * np.pi * 9500 * t)).astype(np.float32)
    y_lo = audio.resample_device(lo, sr, 16000).cpu().numpy()
    y_hi = audio.resample_device(hi, sr, 16000).cpu().numpy()
    tt = np.arange(len(y_lo)) / 16000
    mid = slice(1000, -1000)
    assert np.abs(y_lo[mid] - 0.5 * np.sin(2 * np.pi * 1000 * tt[mid])).max() < 2e-3
    assert np.abs(y_hi[mid]).max() < 2e-3


def test_flac_bytes_through_load_input():
    pcm = np.round(_sig(44100, 1.3, 2, 5) * 8388607).astype(np.int32)
    data = ao.flac_encode(pcm, 44100, 24, blocksizes=(4096,), subframe_kinds=("lpc8",), stereo_modes=(10,))
    got = audio.load_input(data)
    ref = ao.swr_resample(pcm.astype(np.float64).mean(axis=1) / 2.0 ** 23, 44100, 16000)
    assert np.abs(got - ref).max() < TOL


def test_ogg_vorbis_bytes_through_load_input():
    """Native Vorbis decode (host) -> GPU downmix + resample, against the oracle's decoder + float64 resampler:
    the image's real libVorbis file when present, and a random-syntax stream from the oracle's writer."""
    import os

    from oracle import vorbis_oracle as vo

    real = "/usr/local/lib/python3.10/dist-packages/kaleido/executable/etc/mathjax/extensions/a11y/invalid_keypress.ogg"
    streams = [open(real, "rb").read()] if os.path.exists(real) else []
    streams.append(vo.write_stream(np.random.default_rng(7), channels=2, bs_exp=(7, 9), n_packets=14, rate=44100))
    for data in streams:
        x, sr = vo.decode(data)
        got = audio.load_input(data)
        ref = ao.swr_resample(x.astype(np.float64).mean(axis=1), sr, 16000)
        scale = max(1.0, float(np.abs(ref).max()))
        assert got.shape == ref.shape and np.abs(got - ref).max() < TOL * scale


def test_mp3_bytes_through_load_input():
    """Native MP3 decode (host) -> GPU downmix + resample, against the oracle's float64 decoder + resampler (the
    image's real MP3 and a random-syntax MPEG-2 LSF 22.05 kHz stream); and the cross-codec pin at 16 kHz: the real
    MP3's ingest correlates >= 0.95 at lag 0 with the ingest of its Vorbis twin (the same MathJax sound; measured
    0.99999998 at 44.1 kHz on the CPU, tests/test_audio_mp3.py). Parity with ffmpeg is unpinned."""
    import os

    from oracle import mp3_oracle as mo

    a11y = "/usr/local/lib/python3.10/dist-packages/kaleido/executable/etc/mathjax/extensions/a11y/"
    streams = [open(a11y + "invalid_keypress.mp3", "rb").read()] if os.path.exists(a11y + "invalid_keypress.mp3") else []
    streams.append(mo.write_stream(np.random.default_rng(8), version=2, sr_sub=0, mode=1, nframes=12))
    for data in streams:
        x, sr, _ = mo.decode(data)
        got = audio.load_input(data)
        ref = ao.swr_resample(x.astype(np.float64).mean(axis=1), sr, 16000)
        scale = max(1.0, float(np.abs(ref).max()))
        assert got.shape == ref.shape and np.abs(got - ref).max() < TOL * scale
    if os.path.exists(a11y + "invalid_keypress.ogg") and len(streams) == 2:
        m = audio.load_input(streams[0]).astype(np.float64)
        v = audio.load_input(open(a11y + "invalid_keypress.ogg", "rb").read()).astype(np.float64)
        n = len(v)  # 8000 samples (0.5 s); the MP3 runs 377 samples of digital silence longer
        c = float(m[:n] @ v / np.sqrt((m[:n] @ m[:n]) * (v @ v)))
        assert len(m) == -(-23087 * 16000 // 44100) and c >= 0.95, c
        print(f"mp3 vs vorbis at 16 kHz: correlation {c:.8f}")


def test_mpeg_layer1_layer2_bytes_through_load_input():
    """MPEG audio Layers I / II (host decode) -> GPU downmix + resample: random-syntax streams against the oracle's
    float64 decoder + resampler, and the signal pin at 16 kHz — the test-side Annex C encoder's two-tone 48 kHz
    signal (tests/test_audio_mpeg_l12.py) comes out of the ingest as the float64 resampling of that signal delayed by
    the filter bank's 481 samples, to the bank's design error."""
    from oracle import mp3_oracle as mo
    from test_audio_mpeg_l12 import _encode

    for layer, version, sr_sub in ((2, 1, 0), (1, 1, 1), (2, 2, 1)):
        data = mo.write_stream_l12(np.random.default_rng(layer * 10 + version), layer=layer, version=version,
                                   sr_sub=sr_sub, mode=1, bri=12, nframes=6)
        x, sr, _ = mo.decode(data)
        got = audio.load_input(data)
        ref = ao.swr_resample(x.astype(np.float64).mean(axis=1), sr, 16000)
        scale = max(1.0, float(np.abs(ref).max()))
        assert got.shape == ref.shape and np.abs(got - ref).max() < TOL * scale
    n = 48000 // 2
    t = np.arange(n) / 48000.0
    mono = 0.4 * np.sin(2 * np.pi * 440 * t) + 0.25 * np.sin(2 * np.pi * 2500 * t + 0.3)
    for layer in (1, 2):
        data = _encode(np.stack([mono, 0.5 * mono], axis=1), layer)
        got = audio.load_input(data).astype(np.float64)
        m = len(got) * 3
        ref = ao.swr_resample(np.concatenate([np.zeros(481), 0.75 * mono])[:m], 48000, 16000)
        mid = slice(1000, len(got) - 1000)
        err = np.abs(got[mid] - ref[mid]).max()
        assert got.shape == ref.shape and err < 3e-4 * np.abs(ref).max(), (layer, err)


def test_alac_m4a_bytes_through_load_input():
    """Apple Lossless in M4A (host decode behind the MP4 demuxer) -> GPU downmix + resample, against the oracle's
    integer decode (lossless: the encoder's input) through the float64 resampler."""
    from oracle import alac_oracle as al

    for seed, (nch, depth) in enumerate(((2, 16), (1, 24))):
        cookie, packets, x = al.write_stream(np.random.default_rng(seed), nch=nch, depth=depth, frames=3,
                                             frame_length=4096, tail=1234)
        data = al.write_m4a(cookie, packets, al.parse_cookie(cookie))
        got = audio.load_input(data)
        ref = ao.swr_resample(al.to_float(x, depth).astype(np.float64).mean(axis=1), 44100, 16000)
        assert got.shape == ref.shape and np.abs(got - ref).max() < TOL


def test_mp3_file_through_process_audio(tmp_path):
    """An MP3 upload (the image's real file when present, else a random-syntax stream) through
    AudioProcessingPipeline.process_audio and the drop-in callable on the tiny.en engine: the duration is the
    gapless-trimmed length, and the transcript equals the one of the same upload handed over as the ingest's 16 kHz
    array."""
    import os

    from oracle import mp3_oracle as mo
    from twamd.audio_pipeline import AudioProcessingPipeline
    from twamd.pipeline import TurboTranscriber

    real = "/usr/local/lib/python3.10/dist-packages/kaleido/executable/etc/mathjax/extensions/a11y/invalid_keypress.mp3"
    data = open(real, "rb").read() if os.path.exists(real) else mo.write_stream(np.random.default_rng(9), mode=1)
    path = str(tmp_path / "upload.mp3")
    with open(path, "wb") as f:
        f.write(data)
    tr = TurboTranscriber.from_pretrained("tiny.en", seed=1234, max_batch=4)
    pipe = AudioProcessingPipeline(transcriber=tr)
    orig = pipe.transcribe
    kw = dict(chunk_length_s=60, stride_length_s=5, generate_kwargs={"max_new_tokens": 32}, return_timestamps=True)

    def _tr(audio_path, task="transcribe", **_):  # tiny.en is English-only: the reference's task kwarg raises
        return tr(audio_path, **kw)

    pipe.transcribe = _tr
    res = pipe.process_audio(path)
    pipe.transcribe = orig
    assert "error" not in res, res
    x, sr, _ = mo.decode(data)
    assert abs(res["duration"] - len(x) / sr) < 1e-6
    wav = audio.load_input(data)
    ref = tr(wav, **kw)
    assert res["text"] == ref["text"] == tr(path, **kw)["text"] == tr(data, **kw)["text"]


def test_aac_bytes_through_load_input():
    """Native AAC-LC decode (host; the MP4 demuxer or ADTS framing) -> GPU downmix + resample, against the oracle's
    float64 decoder + resampler: the image's real AAC-LC track (realshort.mp4, 48 kHz mono) and a random-syntax
    44.1 kHz stereo ADTS stream. Parity with ffmpeg is unpinned."""
    import os

    from oracle import aac_oracle as aao

    real = "/opt/conda/lib/python3.9/site-packages/imageio/resources/images/realshort.mp4"
    cases = []
    if os.path.exists(real):
        data = open(real, "rb").read()
        tr = audio.mp4_audio_track(data)
        units = [data[o: o + s] for o, s in zip(tr.offsets.tolist(), tr.sizes.tolist())]
        cases.append((data, aao.decode_raw(tr.config, units)))
    adts = aao.write_adts(np.random.default_rng(12), sri=4, chan_config=2, nframes=10)
    cases.append((adts, aao.decode_adts(adts)))
    for data, (x, sr, _) in cases:
        got = audio.load_input(data)
        ref = ao.swr_resample(x.astype(np.float64).mean(axis=1), sr, 16000)
        scale = max(1.0, float(np.abs(ref).max()))
        assert got.shape == ref.shape and np.abs(got - ref).max() < TOL * scale


def test_m4a_file_through_process_audio(tmp_path):
    """An .m4a upload (the image's real AAC-LC track when present, else a random-syntax MP4) through
    AudioProcessingPipeline.process_audio and the drop-in callable on the tiny.en engine: the duration is the
    track's decoded length, and the transcript equals the one of the same upload handed over as the ingest's 16 kHz
    array."""
    import os

    from oracle import aac_oracle as aao
    from twamd.audio_pipeline import AudioProcessingPipeline
    from twamd.pipeline import TurboTranscriber

    real = "/opt/conda/lib/python3.9/site-packages/imageio/resources/images/realshort.mp4"
    data = open(real, "rb").read() if os.path.exists(real) else aao.write_mp4(np.random.default_rng(3))[0]
    path = str(tmp_path / "upload.m4a")
    with open(path, "wb") as f:
        f.write(data)
    tr = TurboTranscriber.from_pretrained("tiny.en", seed=1234, max_batch=4)
    pipe = AudioProcessingPipeline(transcriber=tr)
    orig = pipe.transcribe
    kw = dict(chunk_length_s=60, stride_length_s=5, generate_kwargs={"max_new_tokens": 32}, return_timestamps=True)

    def _tr(audio_path, task="transcribe", **_):  # tiny.en is English-only: the reference's task kwarg raises
        return tr(audio_path, **kw)

    pipe.transcribe = _tr
    res = pipe.process_audio(path)
    pipe.transcribe = orig
    assert "error" not in res, res
    x, sr = audio.decode_mp4(data)
    assert abs(res["duration"] - len(x) / sr) < 1e-6
    wav = audio.load_input(data)
    ref = tr(wav, **kw)
    assert res["text"] == ref["text"] == tr(path, **kw)["text"]


def test_flac_file_through_process_audio(tmp_path):
    """BASELINE config 1 shape: a single FLAC file at 192 kHz through AudioProcessingPipeline.process_audio on the
    tiny.en engine; the transcript equals the one of the same audio handed over as a decoded 16 kHz array."""
    from twamd.audio_pipeline import AudioProcessingPipeline
    from twamd.pipeline import TurboTranscriber

    x = speech_like(19.7, 21)
    src = np.interp(np.arange(int(len(x) * 12)) / 12.0, np.arange(len(x)), x)  # 192 kHz version
    pcm = np.round(np.clip(src, -1, 1) * 32767).astype(np.int32)
    path = str(tmp_path / "clip.flac")
    with open(path, "wb") as f:
        f.write(ao.flac_encode(pcm, 192000, 16, blocksizes=(4096,), subframe_kinds=("lpc12", "fixed2")))
    tr = TurboTranscriber.from_pretrained("tiny.en", seed=1234, max_batch=4)
    pipe = AudioProcessingPipeline(transcriber=tr)
    orig = pipe.transcribe

    def _tr(audio_path, task="transcribe", **kw):  # tiny.en is English-only: the reference's task kwarg raises
        return tr(audio_path, chunk_length_s=60, stride_length_s=5, generate_kwargs={"max_new_tokens": 32},
                  return_timestamps=True)

    pipe.transcribe = _tr
    res = pipe.process_audio(path)
    pipe.transcribe = orig
    assert "error" not in res, res
    assert set(res) >= {"text", "segments", "merged_segments", "duration", "processing_times"}
    assert abs(res["duration"] - len(pcm) / 192000) < 1e-6
    wav = ao.swr_resample(pcm / 32768.0, 192000, 16000).astype(np.float32)
    ref = tr(wav, chunk_length_s=60, stride_length_s=5, generate_kwargs={"max_new_tokens": 32}, return_timestamps=True)
    assert res["text"] == ref["text"]


def test_ogg_file_through_process_audio(tmp_path):
    """An Ogg Vorbis upload (the image's real libVorbis file when present, else a random-syntax stream) through
    AudioProcessingPipeline.process_audio on the tiny.en engine: the duration is the stream's granule length (the
    oracle's decode), and the transcript equals the one of the same upload handed over as the ingest's 16 kHz array
    (native decode + GPU resampler, held to the oracle by test_ogg_vorbis_bytes_through_load_input)."""
    import os

    from oracle import vorbis_oracle as vo
    from twamd.audio_pipeline import AudioProcessingPipeline
    from twamd.pipeline import TurboTranscriber

    real = "/usr/local/lib/python3.10/dist-packages/kaleido/executable/etc/mathjax/extensions/a11y/invalid_keypress.ogg"
    data = open(real, "rb").read() if os.path.exists(real) else vo.write_stream(np.random.default_rng(9), channels=2)
    path = str(tmp_path / "upload.ogg")
    with open(path, "wb") as f:
        f.write(data)
    tr = TurboTranscriber.from_pretrained("tiny.en", seed=1234, max_batch=4)
    pipe = AudioProcessingPipeline(transcriber=tr)
    orig = pipe.transcribe

    def _tr(audio_path, task="transcribe", **kw):  # tiny.en is English-only: the reference's task kwarg raises
        return tr(audio_path, chunk_length_s=60, stride_length_s=5, generate_kwargs={"max_new_tokens": 32},
                  return_timestamps=True)

    pipe.transcribe = _tr
    res = pipe.process_audio(path)
    pipe.transcribe = orig
    assert "error" not in res, res
    x, sr = vo.decode(data)
    assert abs(res["duration"] - len(x) / sr) < 1e-6
    wav = audio.load_input(data)
    ref = tr(wav, chunk_length_s=60, stride_length_s=5, generate_kwargs={"max_new_tokens": 32}, return_timestamps=True)
    assert res["text"] == ref["text"]


@pytest.mark.parametrize("kind", ["wav_ulaw", "wav_ima", "au_alaw", "aifc_ulaw", "wav_msadpcm", "aifc_ima4"])
def test_telephony_files_through_load_input(kind):
    """8 kHz call recordings (G.711 / IMA / MS ADPCM, Apple IMA4) through the product path: native host decode, then
    the GPU resampler to 16 kHz, against the oracle resampler applied to the stdlib (audioop) decode of the same
    bytes (MS ADPCM: the oracle's decode, tests/test_audio_adpcm_mpeg_wav.py)."""
    import audioop
    import struct

    x = np.clip(_sig(8000, 2.1, 1, 11)[:, 0] * 0.8, -1, 1)
    lin = np.round(x * 32767).astype("<i2").tobytes()
    if kind == "wav_ima":
        # a Microsoft IMA encoder: per 505-sample block, the header carries the first sample and the running step
        # index; audioop codes the other 504 (high nibble first, swapped to WAV's low-nibble-first order)
        s16 = np.frombuffer(lin, "<i2")
        payload, index = bytearray(), 0
        for i in range(0, len(s16) - 504, 505):
            codes, (_, nxt) = audioop.lin2adpcm(s16[i + 1: i + 505].tobytes(), 2, (int(s16[i]), index))
            payload += struct.pack("<hBB", int(s16[i]), index, 0) + bytes(((b & 0x0F) << 4) | (b >> 4) for b in codes)
            index = nxt
        fmt = struct.pack("<HHIIHHHH", 0x11, 1, 8000, 4055, 256, 4, 2, 505)
        data = b"RIFF" + struct.pack("<I", 4 + 8 + len(fmt) + 8 + len(payload)) + b"WAVEfmt " + \
            struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(payload)) + bytes(payload)
        ref_lin = audio.decode_wav(data)[0][:, 0].astype(np.float64)  # checked against audioop in test_audio_codecs
    elif kind == "wav_msadpcm":
        s16 = np.frombuffer(lin, "<i2")[:, None]
        payload = ao.ms_adpcm_encode(s16, 1, 256, np.random.default_rng(5), predictors=[0])
        coefs = b"".join(struct.pack("<hh", a, b) for a, b in ao.MS_COEF)
        fmt = struct.pack("<HHIIHH", 2, 1, 8000, 4096, 256, 4) + struct.pack("<HHH", 4 + len(coefs), 500, 7) + coefs
        data = b"RIFF" + struct.pack("<I", 4 + 8 + len(fmt) + 8 + len(payload)) + b"WAVEfmt " + \
            struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(payload)) + payload
        ref_lin = ao.ms_adpcm_decode(payload, 1, 256)[:, 0] / 32768.0
    elif kind == "aifc_ima4":
        # an IMA4 encoder: audioop codes each 64-sample packet from the running state, which the packet header
        # restates (so the decoder carries its exact state over, as ffmpeg's adpcm_ima_qt does)
        s16 = np.frombuffer(lin, "<i2")
        payload, state = bytearray(), (0, 0)
        for i in range(0, len(s16) - 63, 64):
            codes, nxt = audioop.lin2adpcm(s16[i: i + 64].tobytes(), 2, state)
            payload += struct.pack(">h", (state[0] & ~0x7F) | state[1])
            payload += bytes(((b & 0x0F) << 4) | (b >> 4) for b in codes)
            state = nxt
        comm = struct.pack(">hIh", 1, len(payload) // 34, 16) + struct.pack(">H", 16383 + 15) + \
            struct.pack(">Q", 8000 << 48) + b"ima4\x00\x00"
        body = b"COMM" + struct.pack(">I", len(comm)) + comm + b"SSND" + struct.pack(">I", 8 + len(payload)) + \
            bytes(8) + bytes(payload)
        data = b"FORM" + struct.pack(">I", 4 + len(body)) + b"AIFC" + body
        ref_lin = audio.decode_aiff(data)[0][:, 0].astype(np.float64)  # checked against audioop on the CPU
    else:
        alaw = kind == "au_alaw"
        codes = audioop.lin2alaw(lin, 2) if alaw else audioop.lin2ulaw(lin, 2)
        ref_lin = np.frombuffer(audioop.alaw2lin(codes, 2) if alaw else audioop.ulaw2lin(codes, 2), "=i2") / 32768.0
        if kind == "wav_ulaw":
            fmt = struct.pack("<HHIIHH", 7, 1, 8000, 8000, 1, 8)
            data = b"RIFF" + struct.pack("<I", 4 + 8 + len(fmt) + 8 + len(codes)) + b"WAVEfmt " + \
                struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(codes)) + codes
        elif kind == "au_alaw":
            data = b".snd" + struct.pack(">IIIII", 24, len(codes), 27, 8000, 1) + codes
        else:
            import aifc
            import io

            buf = io.BytesIO()
            w = aifc.open(buf, "wb")
            w.setnchannels(1), w.setsampwidth(2), w.setframerate(8000), w.setcomptype(b"ulaw", b"")
            w.writeframes(lin)
            w._patchheader()
            data = buf.getvalue()
            w._file = None
    got = audio.load_input(data)
    ref = ao.swr_resample(ref_lin, 8000, 16000)
    assert got.shape == ref.shape == (2 * len(ref_lin),)
    assert np.abs(got - ref).max() < TOL
    clean = ao.swr_resample(x[: len(ref_lin)], 8000, 16000)
    assert np.abs(ref - clean)[100:-100].mean() < 0.03  # codec noise, not garbage
