"""The standalone mirror of the reference's result/merge surface (twamd.audio_pipeline) against the reference's OWN
behaviour, captured from /root/reference by tests/golden/make_ref_merge.py into tests/golden/ref_merge.json (SURVEY
§8c(v), rows a2/a18/f2): the exact kwargs `transcribe` hands the ASR callable, its error convention, the vocalis
`process_audio` result and merge (including the KeyError 'start' on raw HF chunks), the root layout's
timestamp -> start/end merge (and its failures), the diarizer's speaker assignment, and install(...,
overlap_diarization=True) on the reference's own class. CPU only; no reference code is imported here."""
import copy
import dataclasses
import json
import os
import threading
import time

import pytest

from twamd import audio as tw_audio
from twamd import audio_pipeline as ap

G = os.path.join(os.path.dirname(__file__), "golden")
GOLD = json.load(open(os.path.join(G, "ref_merge.json")))


@dataclasses.dataclass
class DiarizationSegment:  # the shape of the root diar.py's segment objects (not subscriptable)
    speaker_id: int
    start_time: float
    end_time: float
    score: float = 1.0


class FakeASR:
    def __init__(self, output):
        self.output, self.calls = output, []

    def __call__(self, inputs, **kw):
        self.calls.append({"inputs": inputs, **kw})
        if isinstance(self.output, Exception):
            raise self.output
        return json.loads(json.dumps(self.output))


def _cases(layout, fn):
    return [c for c in GOLD["cases"] if c["layout"] == layout and c["fn"] == fn]


def _diar_for(layout, asr, turns):
    """The diarization the reference's diarize() produced for this case, as the mirror's diarize_fn returns it."""
    if layout == "root":  # DiarizationSegment objects, sorted by start (sort_by_start_time)
        return [DiarizationSegment(s, a, b) for s, a, b in sorted(GOLD["turns"][turns], key=lambda t: t[1])]
    (c,) = [c for c in _cases(layout, "diarize") if c["asr"] == asr and c["turns"] == turns]
    return copy.deepcopy(c["result"])


def _norm(r):
    r = json.loads(json.dumps(r, default=repr))
    if isinstance(r, dict) and "processing_times" in r:
        r["processing_times"] = sorted(r["processing_times"])
    return r


@pytest.fixture(autouse=True)
def _duration(monkeypatch):
    monkeypatch.setattr(tw_audio, "duration_seconds", lambda path: GOLD["audio_s"])
    saved = dict(ap._PIPELINE_CACHE)
    yield
    ap._PIPELINE_CACHE.clear()
    ap._PIPELINE_CACHE.update(saved)


def _mirror(layout, asr, turns):
    cls = ap.AudioProcessingPipeline if layout == "vocalis" else ap.RootAudioProcessingPipeline
    p = cls(diarize_fn=lambda path, n: _diar_for(layout, asr, turns))
    p.transcription_model = FakeASR(GOLD["asr_outputs"][asr])
    return p


@pytest.mark.parametrize("layout", ["vocalis", "root", "root_dict_segments"])
def test_process_audio_matches_reference(layout):
    cases = _cases(layout, "process_audio")
    assert len(cases) == 9
    for c in cases:
        p = _mirror(layout, c["asr"], c["turns"])
        seg = "pyannote/segmentation-3.0" if layout == "vocalis" else ""
        emb = "3dspeaker_speech_eres2net_sv_en_voxceleb_16k.onnx|25.3MB" if layout == "vocalis" else ""
        got = _norm(p.process_audio("/tmp/upload.flac", "transcribe", seg, emb, 2, 0.5))
        assert got == c["result"], (layout, c["asr"], c["turns"])
        assert p.transcription_model.calls == [{**k, "batch_size": 32} for k in c["asr_calls"]]


@pytest.mark.parametrize("layout", ["vocalis", "root", "root_dict_segments"])
def test_merge_matches_reference(layout):
    for c in _cases(layout, "merge"):
        p = _mirror(layout, c["asr"], c["turns"])
        tr = json.loads(json.dumps(GOLD["asr_outputs"][c["asr"]]))
        try:
            got = _norm(p._merge_transcription_with_diarization(tr, _diar_for(layout, c["asr"], c["turns"])))
        except Exception as e:
            got = None
            assert f"{type(e).__name__}: {e}" == c.get("exception"), (layout, c["asr"], c["turns"])
        assert got == c["result"], (layout, c["asr"], c["turns"])


@pytest.mark.parametrize("layout", ["vocalis", "root"])
def test_transcribe_call_and_errors_match_reference(layout):
    """The mirror calls the ASR callable with the reference's exact kwargs (chunk_length_s=60, stride_length_s=5,
    batch_size=32 without a GPU, generate_kwargs={"task": task}, return_timestamps=True) and keeps its error
    strings."""
    cls = ap.AudioProcessingPipeline if layout == "vocalis" else ap.RootAudioProcessingPipeline
    for c in _cases(layout, "transcribe"):
        p = cls()
        if c["asr"] == "raises":
            p.transcription_model = FakeASR(RuntimeError("boom"))
        elif c["asr"] == "load_fails":
            p.transcription_model = None
            p.load_transcription_model = lambda *a, **k: False
        else:
            p.transcription_model = FakeASR(GOLD["asr_outputs"][c["asr"]])
        got = _norm(p.transcribe("/tmp/upload.wav", c["task"]))
        assert got == c["result"], c
        if c["asr_calls"]:
            assert p.transcription_model.calls == c["asr_calls"]


def test_speaker_assignment_matches_reference_diarizer():
    for c in _cases("vocalis", "create_transcript_with_speakers"):
        dsegs = [{"speaker": f"Speaker {s}", "start": a, "end": b, "score": 1.0} for s, a, b in GOLD["turns"][c["turns"]]]
        assert ap.create_transcript_with_speakers(c["segments"], dsegs) == c["result"]


def test_reference_call_kwargs_reach_turbo_transcriber_signature():
    """The kwargs the reference's transcribe() passes (recorded from its own code) are accepted by
    TurboTranscriber.__call__'s signature (bound without calling the engine)."""
    import inspect

    from twamd.pipeline import TurboTranscriber

    sig = inspect.signature(TurboTranscriber.__call__)
    for c in _cases("vocalis", "transcribe") + _cases("root", "transcribe"):
        for call in c["asr_calls"]:
            kw = dict(call)
            sig.bind(None, kw.pop("inputs"), **kw)


def test_install_overlap_on_reference_class_fixture():
    """Recorded on the reference's own class (make_ref_merge.py): install(..., overlap_diarization=True) returns the
    serial run's result dict exactly, and runs diarization beside transcription (0.4 s + 0.4 s of fake work)."""
    (c,) = _cases("vocalis", "install_overlap")
    assert c["serial"] == c["overlapped"]
    assert c["asr_calls"] == c["asr_calls_serial"]
    assert c["wall_overlapped_s"] < 0.75 * c["wall_serial_s"]


class _RefShaped:
    """A stand-in with the reference's process_audio call order (transcribe, then load_diarizer when the diarizer
    is missing or different, then diarize, then merge; vocalis/core/audio_pipeline.py:567-624)."""

    def __init__(self):
        self.transcription_model = None
        self.diarizer = None
        self.log = []

    def transcribe(self, audio_path, task="transcribe"):
        self.log.append(("transcribe", threading.current_thread().name))
        time.sleep(0.3)
        return {"text": "x", "chunks": []}

    def load_diarizer(self, segmentation_model, embedding_model, num_speakers=2, threshold=0.5):
        self.log.append(("load", threading.current_thread().name))
        self.diarizer = type("D", (), {"segmentation_model": segmentation_model, "embedding_model": embedding_model})()
        return True

    def diarize(self, audio_path, num_speakers=2):
        self.log.append(("diarize", threading.current_thread().name))
        time.sleep(0.3)
        return [{"speaker": "Speaker 0", "start": 0.0, "end": 1.0, "score": 1.0}]

    def process_audio(self, audio_path, task="transcribe", segmentation_model="seg", embedding_model="emb",
                      num_speakers=2, threshold=0.5):
        tr = self.transcribe(audio_path, task)
        if self.diarizer is None or self.diarizer.segmentation_model != segmentation_model:
            self.load_diarizer(segmentation_model, embedding_model, num_speakers, threshold)
        return {"t": tr, "d": self.diarize(audio_path, num_speakers)}


def test_install_overlap_runs_diarizer_beside_transcription():
    import types

    mod = types.SimpleNamespace(AudioProcessingPipeline=type("P", (_RefShaped,), {}), _PIPELINE_CACHE={})
    serial = mod.AudioProcessingPipeline()
    t0 = time.time()
    r_serial = serial.process_audio("/a.wav", num_speakers=3)
    t_serial = time.time() - t0
    ap.install(mod, overlap_diarization=True)
    p = mod.AudioProcessingPipeline()
    t0 = time.time()
    r = p.process_audio("/a.wav", num_speakers=3)
    t_over = time.time() - t0
    assert r == r_serial
    assert t_over < 0.8 * t_serial
    names = dict((k, n) for k, n in p.log)
    assert names["diarize"].startswith("tw-diarize") and not names["transcribe"].startswith("tw-diarize")
    assert [k for k, _ in p.log].count("load") == 1 and [k for k, _ in p.log].count("diarize") == 1
    # a later diarize() with other arguments is the reference's own call, not the prefetched result
    assert p.diarize("/b.wav", 2) == r["d"] and p.log[-1][0] == "diarize"


@pytest.mark.parametrize("layout", ["vocalis", "root"])
def test_undecodable_upload_reaches_reference_error_convention(layout, tmp_path):
    """An upload the engine cannot decode (here Ogg Opus) surfaces as the reference's transcribe() error result,
    {"error": "Transcription error: <message>"} (the "raises" fixture above), not as an exception."""
    cls = ap.AudioProcessingPipeline if layout == "vocalis" else ap.RootAudioProcessingPipeline
    p = cls()
    p.transcription_model = lambda inputs, **kw: tw_audio.load_input(inputs)
    f = tmp_path / "upload.ogg"
    f.write_bytes(b"OggS\x00\x02" + bytes(22) + b"OpusHead" + bytes(256))
    got = p.transcribe(str(f), "transcribe")
    assert got == {"error": "Transcription error: Ogg Opus audio is not decoded by this engine (decoded containers: "
                            "FLAC (native, Ogg), Ogg Vorbis, MP3 / MPEG audio (MPEG-1 / 2 / 2.5 Layers I, II, III), "
                            "AAC-LC / ALAC (M4A / MP4), AAC (ADTS), WAV / RIFX / RF64 (PCM, float, A-law, mu-law, IMA / "
                            "MS ADPCM, MPEG), AU, AIFF / AIFF-C); convert the upload to one of them"}
