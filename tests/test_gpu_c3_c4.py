"""BASELINE configs[2] and configs[3] on the MI355X at the benchmarked depth (large-v3-turbo dims, seeded weights):

  configs[2]  one TurboTranscriber call on 1 h of audio (120 x 30-s windows, the product call bench.py --config c3
              times): equal to per-batch generate() window for window, the windows that have an fp32 golden within
              tau of it; and the same call sharded over two ranks (gloo, both on this GPU) equal to one process
  configs[3]  process_audio with the transcription on the GPU and a host diarizer overlapped beside it
              (twamd.audio_pipeline.install(..., overlap_diarization=True)) on a stand-in of the reference's class
              (built here: no reference code runs on the GPU box): the same result dict as the serial run, and the
              diarizer's time hidden behind the GPU work

The reference runs transcription then diarization back to back (vocalis/core/audio_pipeline.py:589-624); the hour is
the reference call shape of configs[2] (30-s mode: chunk_length_s=30, stride 0)."""
import os
import socket
import sys
import time
import wave

import numpy as np
import pytest
import torch

from twamd.pipeline import TurboTranscriber
from twamd.synth_audio import speech_like, workload

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import turbo_parity as tp  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T = 128


@pytest.fixture(scope="module")
def turbo():
    tr = TurboTranscriber.from_pretrained("large-v3-turbo", seed=1234, max_batch=24, max_beams=1)
    yield tr
    del tr
    torch.cuda.empty_cache()


def _suppress_eos(tr, on):
    g = tr.gen
    tr.engine.set_suppress_tokens(list(g.suppress_tokens) + ([g.special.eot] if on else []))


def test_c3_hour_call_equals_per_batch_generate(turbo):
    """One call on the hour (bench.py --config c3's call: 30-s mode, greedy, EOS suppressed, 128 new tokens, one
    seek pass): 120 windows in 5 pipelined engine batches. Every window's tokens equal a plain generate() of its
    batch of 24, and the hour's windows 0, 5, 11, 17 (the same seeded clips as bench windows 0, 5, 11, 17) pass the
    fp32 golden's first-divergence check (turbo_bench.npz, tau 0.15 logits) with the fp32 language."""
    eng = turbo.engine
    hour = workload(120, 30.0, seed=1234)
    kw = dict(chunk_length_s=30, stride_length_s=0, batch_size=24, return_timestamps=True,
              generate_kwargs={"task": "transcribe", "num_beams": 1, "max_new_tokens": T, "max_passes": 1})
    _suppress_eos(turbo, True)
    try:
        t0 = time.perf_counter()
        out = turbo(hour.reshape(-1), **kw)
        wall = time.perf_counter() - t0
        passes = [p[0] for p in turbo.last_window_passes]
        langs = list(turbo.last_window_langs)
        assert len(passes) == 120 and all(len(p) == T for p in passes)
        assert out["text"] and len(out["chunks"]) > 0
        for b in range(5):
            eng.wave[:24].copy_(torch.from_numpy(hour[b * 24:(b + 1) * 24]))
            eng.logmel(24)
            eng.generate(24, task="transcribe", max_new_tokens=T, max_passes=1)
            assert [p[0] for p in eng.last_passes] == passes[b * 24:(b + 1) * 24], b
            assert eng.last_langs == langs[b * 24:(b + 1) * 24], b
    finally:
        _suppress_eos(turbo, False)
    zb = tp.load_bench()
    bench = workload(24, 30.0, seed=1234)
    checked = 0
    for w in (int(x) for x in zb["windows"]):
        if not np.array_equal(hour[w], bench[w]):
            continue  # (the bench's silent windows 22, 23 are speech in the hour)
        k = f"w{w}_"
        r = tp.check_pass(passes[w], zb[k + "tokens"], zb[k + "top_idx"], zb[k + "top_val"], zb[k + "ts_margin"])
        print(f"c3 hour window {w}: {r}")
        assert r["status"] in ("exact", "within_tau"), (w, r)
        assert langs[w] == int(zb[k + "lang"][0])
        checked += 1
    assert checked == 4
    print(f"c3: one call on 1 h of audio, {wall * 1000:.0f} ms (first call, graphs captured inside)")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


_SHARD_KW = dict(chunk_length_s=30, stride_length_s=0, batch_size=24, return_timestamps=True,
                 generate_kwargs={"task": "transcribe", "num_beams": 1, "max_new_tokens": 32, "max_passes": 1})


def _shard_input():
    return workload(7, 30.0, seed=4321).reshape(-1)[: 7 * 480000 - 16000 * 9]  # 7 windows, the last one ragged


def _rank_worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "turbo-whisper-workspace_amd")]
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from twamd.pipeline import TurboTranscriber as TT

        tr = TT.from_pretrained("large-v3-turbo", seed=1234, max_batch=24, max_beams=1)
        out = tr(_shard_input() if rank == 0 else None, **_SHARD_KW)
        q.put((rank, out, [p[0] for p in tr.last_window_passes]))
    finally:
        dist.destroy_process_group()


def test_c3_two_rank_turbo_sharded_equals_single_process(turbo):
    """configs[2]'s sharding at turbo depth on a shortened input (7 windows, 32 new tokens): two ranks (gloo, both on
    this GPU) each decode their contiguous shard (3 + 4 windows, twamd.dist.shard_range) with their own engine, the token arrays are
    all-gathered and rank 0 stitches; both ranks return exactly the single-process transcript."""
    import torch.multiprocessing as mp

    ref = turbo(_shard_input(), **_SHARD_KW)
    ref_passes = [p[0] for p in turbo.last_window_passes]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, out, passes = q.get(timeout=400)
        got[r] = (out, passes)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert got[0][0] == ref and got[1][0] == ref
    assert got[0][1] == ref_passes[:3] and got[1][1] == ref_passes[3:]  # each rank decoded its own shard


# ---- configs[3]: process_audio with the diarizer overlapped ------------------------------------------------------
class _StandInDiarizer:
    """Host diarizer stand-in: GIL-releasing numpy work (BLAS on 4 threads, as the reference's sherpa-onnx runs with
    4, vocalis/core/model.py:451-470) of a calibrated amount, then speaker turns from the waveform's energy
    (deterministic)."""

    def __init__(self, segmentation_model, embedding_model, num_speakers, threshold, units):
        self.segmentation_model, self.embedding_model = segmentation_model, embedding_model
        self.num_speakers, self.threshold, self.units = num_speakers, threshold, units

    @staticmethod
    def work(units):
        from threadpoolctl import threadpool_limits

        a = np.random.default_rng(0).standard_normal((768, 768)).astype(np.float32)
        with threadpool_limits(limits=4):
            for _ in range(units):
                a = np.tanh(a @ a * 1e-3)
        return float(a[0, 0])

    def process(self, path, num_speakers):
        self.work(self.units)
        with wave.open(path, "rb") as f:
            x = np.frombuffer(f.readframes(f.getnframes()), np.int16).astype(np.float32)
        sec = x[: len(x) // 16000 * 16000].reshape(-1, 16000)
        loud = (np.abs(sec).mean(1) > np.median(np.abs(sec).mean(1))).astype(int)
        turns, start = [], 0
        for i in range(1, len(loud) + 1):
            if i == len(loud) or loud[i] != loud[start]:
                turns.append({"speaker": f"Speaker {loud[start] % num_speakers}", "start": float(start),
                              "end": float(i)})
                start = i
        return turns


def _stand_in_module(units):
    """A module shaped like vocalis.core.audio_pipeline for what install() patches and process_audio does
    (reference :171-208 load_transcription_model, :323-369 transcribe's call, :567-688 process_audio: transcribe,
    then load_diarizer / diarize, merge, result dict), with the merge of the root layout (chunks' timestamps ->
    start / end, root audio_pipeline.py:774-799)."""
    import types

    from twamd.audio_pipeline import create_transcript_with_speakers

    class AudioProcessingPipeline:
        def __init__(self):
            self.transcription_model = None
            self.diarizer = None

        def load_transcription_model(self, model_name="openai/whisper-large-v3"):
            raise AssertionError("install() replaces this")

        def transcribe(self, audio_path, task="transcribe", return_timestamps=True):
            if self.transcription_model is None and not self.load_transcription_model():
                return {"error": "Failed to load transcription model"}
            try:
                return self.transcription_model(audio_path, chunk_length_s=60, batch_size=512, stride_length_s=5,
                                                generate_kwargs={"task": task}, return_timestamps=return_timestamps)
            except Exception as e:
                return {"error": f"Transcription error: {e}"}

        def load_diarizer(self, segmentation_model, embedding_model, num_speakers=2, threshold=0.5):
            self.diarizer = _StandInDiarizer(segmentation_model, embedding_model, num_speakers, threshold, units)
            return True

        def diarize(self, audio_path, num_speakers=2):
            return self.diarizer.process(audio_path, num_speakers)

        def process_audio(self, audio_path, task="transcribe", segmentation_model="pyannote/segmentation-3.0",
                          embedding_model="3dspeaker_speech_eres2net_sv_en_voxceleb_16k.onnx|25.3MB",
                          num_speakers=2, threshold=0.5):
            t_start, times = time.time(), {}
            try:
                t = time.time()
                tr = self.transcribe(audio_path, task)
                times["transcription"] = time.time() - t
                if "error" in tr:
                    return tr
                segments = tr.get("chunks", [])
                t = time.time()
                if self.diarizer is None or self.diarizer.segmentation_model != segmentation_model or \
                        self.diarizer.embedding_model != embedding_model:
                    self.load_diarizer(segmentation_model, embedding_model, num_speakers, threshold)
                diar = self.diarize(audio_path, num_speakers)
                times["diarization"] = time.time() - t
                conv = [{"text": c["text"], "start": c["timestamp"][0],
                         "end": c["timestamp"][1] if c["timestamp"][1] is not None else c["timestamp"][0]}
                        for c in segments]
                merged = create_transcript_with_speakers(conv, diar)
                times["total"] = time.time() - t_start
                return {"text": tr.get("text", ""), "segments": segments, "diarization_segments": diar,
                        "merged_segments": merged, "duration": max((s["end"] for s in merged), default=0),
                        "processing_times": times}
            except Exception as e:
                return {"error": f"Processing error: {e}"}

    return types.SimpleNamespace(AudioProcessingPipeline=AudioProcessingPipeline,
                                 _PIPELINE_CACHE={"transcription_model": None, "diarization_model": None})


def _write_wav(path, x):
    with wave.open(str(path), "wb") as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(16000)
        f.writeframes((np.clip(x, -1, 1) * 32767).astype(np.int16).tobytes())


def test_c4_process_audio_with_overlapped_diarization(tmp_path, monkeypatch):
    """configs[3]: install(module, overlap_diarization=True) on the stand-in class with the real turbo engine as the
    reference loads it (load_transcription_model -> the as-shipped beam-5 call through the drop-in) and a host
    diarizer doing GIL-releasing numpy work sized to ~60 % of the transcription. The overlapped process_audio returns
    the serial run's result dict (processing_times aside) and its wall time is below serial - 80 % of the shorter of
    the diarizer's and the transcription's time (the part one can hide behind the other)."""
    from twamd import audio_pipeline as tw_ap

    monkeypatch.setenv("TW_ALLOW_SYNTHETIC", "1")
    path = tmp_path / "upload.wav"
    _write_wav(path, speech_like(75.0, 99) * 0.5)
    # calibration: the transcription alone (also captures its graphs), the diarizer's work per unit
    probe = _stand_in_module(0)
    tw_ap.install(probe)
    p0 = probe.AudioProcessingPipeline()
    assert p0.load_transcription_model("openai/whisper-large-v3-turbo")  # configs[3]'s model (synthetic weights)
    assert p0.transcription_model.engine.d.decoder_layers == 4
    ref_asr = p0.transcribe(str(path))  # (the first call captures the engine's graphs)
    t = time.perf_counter()
    ref_asr = p0.transcribe(str(path))  # warm: the time process_audio's transcription takes
    t_asr = time.perf_counter() - t
    assert "error" not in ref_asr, ref_asr
    _StandInDiarizer.work(4)  # (BLAS threads started)
    t = time.perf_counter()
    _StandInDiarizer.work(16)
    per_unit = (time.perf_counter() - t) / 16
    units = max(4, int(0.6 * t_asr / per_unit))

    def run(overlap):
        mod = _stand_in_module(units)
        mod._PIPELINE_CACHE["transcription_model"] = probe._PIPELINE_CACHE["transcription_model"]
        tw_ap.install(mod, overlap_diarization=overlap)
        p = mod.AudioProcessingPipeline()
        t = time.perf_counter()
        r = p.process_audio(str(path), "transcribe", num_speakers=2)
        return r, time.perf_counter() - t

    serial, t_serial = run(False)
    over, t_over = run(True)
    assert "error" not in serial, serial
    d = serial["processing_times"]["diarization"]
    print(f"c4: transcription {t_asr:.3f} s alone; serial {t_serial:.3f} s (diarization {d:.3f} s, {units} units); "
          f"overlapped {t_over:.3f} s")
    strip = lambda r: {k: v for k, v in r.items() if k != "processing_times"}  # noqa: E731
    assert strip(over) == strip(serial)
    assert strip(serial)["text"] == ref_asr["text"] and serial["segments"] == ref_asr["chunks"]
    assert d >= 0.3 * t_asr, (d, t_asr)  # the diarizer is a real share of the call
    # the hideable share is the shorter of the two (the diarizer behind the GPU work, or the reverse)
    assert t_over < t_serial - 0.8 * min(d, t_serial - d), (t_over, t_serial, d)
