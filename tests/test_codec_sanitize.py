"""The host parsers of untrusted upload bytes under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

POST /api/transcribe stores any upload and the pipeline decodes it (/root/reference/vocalis/api/main.py:67-75;
ffmpeg_read, $TF/pipelines/audio_utils.py:9-45); here the FLAC, Ogg Vorbis, G.711 and IMA ADPCM decoders do that in
host C++ (csrc/flac.cpp, vorbis.cpp, pcm_codecs.cpp incl. MS ADPCM and IMA4, mp3.cpp, aac.cpp, alac.cpp). `make sanitize` builds
them with -fsanitize=address,undefined and -fno-sanitize-recover into tests/fuzz/codec_fuzz.cpp, which runs probe + decode over every corpus file and
hundreds of damaged copies of each (truncations, bit flips, overwritten runs, duplicated chunks, random tails). Any
out-of-bounds access, leak or undefined behaviour aborts the run. The corpus: the oracle's FLAC writer over every
subframe kind / stereo mode / bit depth / blocking, its random-syntax Vorbis writer, the image's one libVorbis
stream, the MP3 oracle's random-syntax Layer III writer (MPEG-1 / 2 / 2.5, every channel mode, Info + LAME frames,
ID3v2 tags, junk between frames) and its Layer I / II writer, the image's one real MP3, the AAC oracle's random-syntax ADTS streams, the access
units of the image's one real AAC-LC track as ADTS, and the reference's example FLAC (first 256 KB, when present in
this container)."""
import os
import subprocess

import numpy as np
import pytest

from oracle import audio_oracle as ao
from oracle import aac_oracle as aao
from oracle import alac_oracle as alo
from oracle import mp3_oracle as mo
from oracle import vorbis_oracle as vo

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "turbo-whisper-workspace_amd", "csrc")
REAL_OGG = "/usr/local/lib/python3.10/dist-packages/kaleido/executable/etc/mathjax/extensions/a11y/invalid_keypress.ogg"
REAL_MP3 = REAL_OGG[:-3] + "mp3"
REAL_AAC_MP4 = "/opt/conda/lib/python3.9/site-packages/imageio/resources/images/realshort.mp4"
REF_FLAC = "/root/reference/examples/Test1/ChrisAndAlexDiTest.flac"


def _corpus(tmp_path):
    files = []

    def put(name, data):
        p = tmp_path / name
        p.write_bytes(bytes(data))
        files.append(str(p))

    rng = np.random.default_rng(7)
    for i, (bps, kinds, modes, bs, var) in enumerate([
            (16, ("lpc8",), (0,), (1024,), False), (24, ("fixed2", "verbatim"), (8, 9, 10), (576, 1152), True),
            (8, ("constant", "lpc2"), (10,), (256,), False), (12, ("fixed0", "lpc12"), (0, 8), (4608,), False),
            (20, ("fixed4", "lpc32"), (9,), (192, 4096), True)]):
        nch = 1 if i == 0 else 2
        pcm = rng.integers(-(1 << (bps - 1)), 1 << (bps - 1), size=(3000 + 700 * i, nch))
        put(f"gen{i}.flac", ao.flac_encode(pcm, 16000 if i % 2 else 44100, bps, blocksizes=bs, subframe_kinds=kinds,
                                           stereo_modes=modes, variable=var, seed=i))
    for seed in range(6):
        put(f"gen{seed}.ogg", vo.write_stream(np.random.default_rng(seed), channels=1 + seed % 3, n_packets=6))
    if os.path.exists(REAL_OGG):
        put("real.ogg", open(REAL_OGG, "rb").read())
    for seed in range(6):
        put(f"gen{seed}.mp3", mo.write_stream(np.random.default_rng(seed), version=(1, 2, 25)[seed % 3], nframes=5,
                                              mode=seed % 4, xing=seed % 2 == 0, id3=seed == 1, junk=seed == 3))
    for seed in range(6):
        put(f"gen{seed}.mp2", mo.write_stream_l12(np.random.default_rng(seed), layer=1 + seed % 2,
                                                  version=(1, 2, 25)[seed % 3], mode=seed % 4, nframes=4,
                                                  id3=seed == 2))
    if os.path.exists(REAL_MP3):
        put("real.mp3", open(REAL_MP3, "rb").read())
    for seed in range(6):
        put(f"gen{seed}.aac", aao.write_adts(np.random.default_rng(seed), sri=(3, 4, 8, 11, 6, 0)[seed],
                                             chan_config=(1, 2, 1, 2, 3, 6)[seed], nframes=4, crc=seed % 2 == 1))
    if os.path.exists(REAL_AAC_MP4):
        from twamd import audio
        data = open(REAL_AAC_MP4, "rb").read()
        tr = audio.mp4_audio_track(data)
        adts = b""
        for o, sz in zip(tr.offsets.tolist(), tr.sizes.tolist()):
            fl = 7 + sz
            adts += bytes([0xFF, 0xF1, 0x4C, 0x40 | (fl >> 11), (fl >> 3) & 0xFF, ((fl & 7) << 5) | 0x1F, 0xFC])
            adts += data[o: o + sz]
        put("real_aac.aac", adts)
    if os.path.exists(REF_FLAC):
        put("ref_prefix.flac", open(REF_FLAC, "rb").read()[: 256 * 1024])
    put("adpcm_like.bin", rng.integers(0, 256, size=4096, dtype=np.uint8))
    tone = np.round(9000 * np.sin(np.arange(3000) / 7.0)).astype(np.int16)
    put("ms_adpcm.bin", ao.ms_adpcm_encode(np.stack([tone, tone[::-1]], 1), 2, 256, np.random.default_rng(2)))
    for seed, (nch, depth) in enumerate(((1, 16), (2, 24))):  # ALAC packets back to back (the driver cuts them up)
        ck, pk, _ = alo.write_stream(np.random.default_rng(seed), nch=nch, depth=depth, frames=2, frame_length=1024,
                                     tail=200)
        put(f"alac{seed}.bin", b"".join(pk))
    return files


def test_upload_parsers_clean_under_asan_ubsan(tmp_path):
    r = subprocess.run(["make", "-C", CSRC, "sanitize"], capture_output=True, text=True)
    if r.returncode != 0 and ("fsanitize" in r.stderr or "libasan" in r.stderr):
        pytest.skip("the sanitizer runtime is not available to g++ here")
    assert r.returncode == 0, r.stderr[-2000:]
    # (verify_asan_link_order=0: the environment may preload a library ahead of the sanitizer runtime)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([os.path.join(CSRC, "build_asan", "codec_fuzz"), "-m", "150", *_corpus(tmp_path)],
                       capture_output=True, text=True, env=env, timeout=600)
    report = (p.stdout + p.stderr)[-4000:]
    assert p.returncode == 0 and "no sanitizer report" in p.stdout, report
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, report
