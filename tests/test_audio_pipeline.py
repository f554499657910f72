"""The AudioProcessingPipeline surface on CPU with a stand-in transcription callable:
the reference's call kwargs, cache protocol, result schema and error conventions
(/root/reference/vocalis/core/audio_pipeline.py:171-208, 323-369, 567-726)."""
import types

import numpy as np

from twamd import audio
from twamd import audio_pipeline as ap


class FakeASR:
    def __init__(self, result=None, exc=None):
        self.calls = []
        self.result = result or {"text": " hello world", "chunks": [{"timestamp": (0.0, 1.5), "text": " hello"},
                                                                   {"timestamp": (1.5, 3.0), "text": " world"}]}
        self.exc = exc

    def __call__(self, inputs, **kw):
        self.calls.append((inputs, kw))
        if self.exc:
            raise self.exc
        return dict(self.result)


def _wav(tmp_path, seconds=3.0):
    p = str(tmp_path / "a.wav")
    audio.write_wav(p, np.zeros(int(16000 * seconds), np.float32))
    return p


def test_transcribe_uses_reference_kwargs(tmp_path):
    f = FakeASR()
    pipe = ap.AudioProcessingPipeline(transcriber=f)
    out = pipe.transcribe(_wav(tmp_path), task="translate")
    assert out["text"] == " hello world"
    (inp, kw), = f.calls
    # batch_size=512 on a GPU, 32 on CPU (:353): this container has no GPU
    assert kw == {"chunk_length_s": 60, "batch_size": 512 if pipe.gpu_available else 32, "stride_length_s": 5,
                  "generate_kwargs": {"task": "translate"}, "return_timestamps": True}


def test_transcribe_error_convention(tmp_path):
    pipe = ap.AudioProcessingPipeline(transcriber=FakeASR(exc=RuntimeError("boom")))
    assert pipe.transcribe(_wav(tmp_path)) == {"error": "Transcription error: boom"}


def test_load_failure_returns_reference_error(tmp_path, monkeypatch):
    ap._PIPELINE_CACHE["transcription_model"] = None
    monkeypatch.setattr(ap, "build_transcriber", lambda *a, **k: (_ for _ in ()).throw(RuntimeError("no gpu")))
    pipe = ap.AudioProcessingPipeline()
    assert pipe.load_transcription_model() is False
    assert pipe.transcribe(_wav(tmp_path)) == {"error": "Failed to load transcription model"}


def test_no_checkpoint_is_a_load_failure_not_gibberish(tmp_path, monkeypatch):
    """the reference loads real weights or fails; without TW_CHECKPOINT the drop-in must not serve the
    seeded synthetic preset under the reference's model name (opt-in: TW_ALLOW_SYNTHETIC=1)."""
    monkeypatch.delenv("TW_CHECKPOINT", raising=False)
    monkeypatch.delenv("TW_ALLOW_SYNTHETIC", raising=False)
    built = []
    monkeypatch.setattr(ap.TurboTranscriber, "from_pretrained", staticmethod(lambda *a, **k: built.append(a) or FakeASR()))
    try:
        ap.build_transcriber()
        raise AssertionError("build_transcriber accepted no checkpoint")
    except RuntimeError as e:
        assert "TW_CHECKPOINT" in str(e)
    ap._PIPELINE_CACHE["transcription_model"] = None
    pipe = ap.AudioProcessingPipeline()
    assert pipe.load_transcription_model() is False
    assert pipe.transcribe(_wav(tmp_path)) == {"error": "Failed to load transcription model"}
    assert built == []
    # explicit opt-in, and a local checkpoint directory, both build
    monkeypatch.setenv("TW_ALLOW_SYNTHETIC", "1")
    ap.build_transcriber()
    monkeypatch.delenv("TW_ALLOW_SYNTHETIC")
    ap.build_transcriber(str(tmp_path))
    assert len(built) == 2
    ap._PIPELINE_CACHE["transcription_model"] = None


def test_process_audio_schema_without_diarization(tmp_path):
    pipe = ap.AudioProcessingPipeline(transcriber=FakeASR())
    r = pipe.process_audio(_wav(tmp_path, 3.0))
    assert set(r) == {"text", "segments", "diarization_segments", "merged_segments", "duration", "processing_times"}
    assert r["duration"] == 3.0 and r["diarization_segments"] == []
    # reference merge, no diarization: alternating speakers, HF chunks have no start/end -> 0
    assert r["merged_segments"] == [{"speaker": "Speaker 0", "text": " hello", "start": 0, "end": 0},
                                    {"speaker": "Speaker 1", "text": " world", "start": 0, "end": 0}]
    assert set(r["processing_times"]) == {"transcription", "diarization", "total"}


def test_process_audio_with_diarization_reproduces_reference_keyerror(tmp_path):
    """vocalis merges raw HF chunks ({"timestamp","text"}) through create_transcript_with_speakers, which reads
    seg['start']: any non-empty diarization gives {"error": "Processing error: 'start'"}."""
    pipe = ap.AudioProcessingPipeline(transcriber=FakeASR(),
                                      diarize_fn=lambda p, n: [{"speaker": "Speaker 0", "start": 0.0, "end": 2.0}])
    assert pipe.process_audio(_wav(tmp_path)) == {"error": "Processing error: 'start'"}


def test_process_audio_propagates_transcription_error(tmp_path):
    pipe = ap.AudioProcessingPipeline(transcriber=FakeASR(exc=ValueError("bad")))
    assert pipe.process_audio(_wav(tmp_path)) == {"error": "Transcription error: bad"}


def test_install_patches_reference_class(monkeypatch):
    class RefPipeline:
        def __init__(self):
            self.transcription_model = None

        def load_transcription_model(self, model_name="openai/whisper-large-v3"):
            raise AssertionError("reference loader must not run")

    mod = types.SimpleNamespace(AudioProcessingPipeline=RefPipeline, _PIPELINE_CACHE={"transcription_model": None})
    built = []
    monkeypatch.setattr(ap, "build_transcriber", lambda name, **k: built.append(name) or FakeASR())
    ap.install(mod)
    a, b = RefPipeline(), RefPipeline()
    assert a.load_transcription_model() is True and b.load_transcription_model() is True
    assert built == ["openai/whisper-large-v3"]          # built once, then served from the module cache
    assert a.transcription_model is b.transcription_model is mod._PIPELINE_CACHE["transcription_model"]


def test_overlapped_diarization_same_result_and_concurrent(tmp_path):
    """BASELINE config 4: the host diarizer runs beside the (GPU) transcription; results are identical."""
    import threading
    import time

    started = threading.Event()

    class SlowASR(FakeASR):
        def __call__(self, inputs, **kw):
            assert started.wait(5), "diarizer did not start before transcription finished"
            time.sleep(0.2)
            return super().__call__(inputs, **kw)

    def diar(path, n):
        started.set()
        time.sleep(0.2)
        return []

    p = _wav(tmp_path)
    seq = ap.AudioProcessingPipeline(transcriber=FakeASR(), diarize_fn=lambda a, n: []).process_audio(p)
    t0 = time.time()
    ovl = ap.AudioProcessingPipeline(transcriber=SlowASR(), diarize_fn=diar, overlap_diarization=True).process_audio(p)
    wall = time.time() - t0
    assert wall < 0.39  # 0.2 s + 0.2 s, overlapped
    for k in ("text", "segments", "diarization_segments", "merged_segments", "duration"):
        assert ovl[k] == seq[k]
