"""Capture the reference's OWN result / merge behaviour as fixtures; build-container only.

Imports the reference's `vocalis.core.audio_pipeline` and the root `audio_pipeline` from /root/reference (read-only)
with `sys.modules` stand-ins for the audio/diarization libraries this image lacks (librosa, soundfile, pydub,
sherpa-onnx via `model` / `vocalis.core.model`) and with the LLM helpers made unimportable (LLM_AVAILABLE = False:
the summariser is out of scope), then drives `transcribe`, `process_audio`, `diarize` and
`_merge_transcription_with_diarization` with a fake ASR callable that records the keyword arguments it is called with
and returns Hugging-Face-shaped outputs. The diarizer is the reference's own `SpeakerDiarizer` whose sherpa-onnx
backend (`get_speaker_diarization`) is a stand-in returning fixed speaker turns.

Writes tests/golden/ref_merge.json (inputs, the ASR call kwargs, result dicts with processing_times reduced to their
keys, and exception strings, e.g. the vocalis merge's KeyError 'start'). Nothing from the reference travels: only the
JSON data does.

Usage: python tests/golden/make_ref_merge.py
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
AUDIO_S = 19.73  # duration the librosa stand-in reports


class _Turn:
    def __init__(self, speaker, start, end):
        self.speaker, self.start, self.end = speaker, start, end


class _Result(list):
    def sort_by_start_time(self):
        return sorted(self, key=lambda t: t.start)


class _FakeSherpa:
    """Stand-in for sherpa_onnx.OfflineSpeakerDiarization: fixed turns (unsorted, to exercise the sort)."""

    turns = []
    delay = 0.0

    def process(self, samples):
        if self.delay:
            import time

            time.sleep(self.delay)
        return _Result(_Turn(*t) for t in self.turns)


def _install_stubs():
    librosa = types.ModuleType("librosa")
    librosa.load = lambda path, sr=None, **k: (np.zeros(int(AUDIO_S * 16000), np.float32), 16000)
    librosa.get_duration = lambda y=None, sr=None, path=None, **k: AUDIO_S
    soundfile = types.ModuleType("soundfile")
    pydub = types.ModuleType("pydub")

    class AudioSegment:  # never reached: librosa answers first
        @staticmethod
        def from_file(p):
            raise RuntimeError("pydub stand-in")

    pydub.AudioSegment = AudioSegment
    model = types.ModuleType("model")
    model.get_speaker_diarization = lambda **kw: _FakeSherpa()
    model.read_wave = lambda path: (np.zeros(16000, np.float32), 16000)
    sys.modules.update({"librosa": librosa, "soundfile": soundfile, "pydub": pydub, "model": model,
                        "vocalis.core.model": model})
    # LLM helpers unimportable -> LLM_AVAILABLE = False in both pipelines (out of scope)
    sys.modules.update({"llm_helper": None, "vocalis.llm": None, "vocalis.llm.llm_helper": None})


class FakeASR:
    """Records each call's kwargs; returns a Hugging-Face-pipeline-shaped output."""

    def __init__(self, output):
        self.output = output
        self.calls = []

    def __call__(self, inputs, **kwargs):
        self.calls.append({"inputs": inputs, **kwargs})
        if isinstance(self.output, Exception):
            raise self.output
        return json.loads(json.dumps(self.output))


ASR_OUTPUTS = {
    "three_chunks": {"text": " Hello there. How are you? Fine.",
                     "chunks": [{"timestamp": [0.0, 3.2], "text": " Hello there."},
                                {"timestamp": [3.2, 7.84], "text": " How are you?"},
                                {"timestamp": [9.5, 12.02], "text": " Fine."}]},
    "open_end": {"text": " one two",
                 "chunks": [{"timestamp": [0.0, 1.5], "text": " one"}, {"timestamp": [1.5, None], "text": " two"}]},
    "no_chunks": {"text": " nothing", "chunks": []},
}
TURNS = {"two_speakers": [(1, 3.0, 8.0), (0, 0.0, 3.1), (0, 9.0, 13.0)],
         "none": [],
         "no_overlap": [(0, 20.0, 25.0)]}


def _clean(r):
    if isinstance(r, dict):
        r = dict(r)
        if "processing_times" in r:
            r["processing_times"] = sorted(r["processing_times"])
        for k in ("diarization_segments", "merged_segments", "segments"):
            if k in r and isinstance(r[k], list):
                r[k] = [x if isinstance(x, dict) else {"__repr__": repr(x)} for x in r[k]]
    return json.loads(json.dumps(r, default=repr))


def _overlap_case(voc_ap, voc_diar):
    """twamd.audio_pipeline.install(..., overlap_diarization=True) on the reference's own class: the same result
    dict as the serial reference run, in less wall time (0.4 s of fake ASR work beside 0.4 s of fake diarization)."""
    import time

    sys.path[:0] = [os.path.dirname(os.path.dirname(HERE)),
                    os.path.join(os.path.dirname(os.path.dirname(HERE)), "turbo-whisper-workspace_amd")]
    from twamd import audio_pipeline as tw_ap

    class SlowASR(FakeASR):
        def __call__(self, inputs, **kw):
            time.sleep(0.4)
            return super().__call__(inputs, **kw)

    def run():
        voc_ap._PIPELINE_CACHE.update(transcription_model=None, diarizer=None)
        p = voc_ap.AudioProcessingPipeline()
        asr = SlowASR(ASR_OUTPUTS["three_chunks"])
        p.transcription_model = asr
        voc_ap._PIPELINE_CACHE["transcription_model"] = asr
        _FakeSherpa.turns, _FakeSherpa.delay = [], 0.4
        t = time.time()
        r = p.process_audio("/tmp/upload.flac", "transcribe")
        return r, time.time() - t, asr.calls

    orig = voc_ap.AudioProcessingPipeline.load_diarizer

    def load_diarizer(self, segmentation_model, embedding_model, num_speakers=2, threshold=0.5):
        # the reference's load_diarizer probes sherpa_onnx for GPU support; with the stand-in backend only the
        # SpeakerDiarizer construction it ends in matters
        self.diarizer = voc_diar.SpeakerDiarizer(segmentation_model=segmentation_model, embedding_model=embedding_model,
                                                 num_speakers=num_speakers, threshold=threshold)
        return True

    voc_ap.AudioProcessingPipeline.load_diarizer = load_diarizer
    serial, t_serial, calls_s = run()
    tw_ap.install(voc_ap, overlap_diarization=True)
    over, t_over, calls_o = run()
    voc_ap.AudioProcessingPipeline.load_diarizer = orig
    _FakeSherpa.delay = 0.0
    return {"layout": "vocalis", "fn": "install_overlap", "serial": _clean(serial), "overlapped": _clean(over),
            "wall_serial_s": round(t_serial, 3), "wall_overlapped_s": round(t_over, 3), "asr_calls": calls_o,
            "asr_calls_serial": calls_s}


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    import audio_pipeline as root_ap  # noqa: E402 (root copy: `from diar import ...`)
    import diar as root_diar  # noqa: E402
    from vocalis.core import audio_pipeline as voc_ap  # noqa: E402
    from vocalis.core import diar as voc_diar  # noqa: E402

    out = {"reference": "crmorton/Turbo-Whisper-Workspace @ /root/reference", "audio_s": AUDIO_S,
           "asr_outputs": ASR_OUTPUTS, "turns": TURNS, "cases": []}

    def add(layout, fn, asr, turns, result, calls, **extra):
        out["cases"].append({"layout": layout, "fn": fn, "asr": asr, "turns": turns, "result": _clean(result),
                             "asr_calls": calls, **extra})

    class DictDiarizer(root_diar.SpeakerDiarizer):
        """The root diarizer handing out dict segments (as vocalis' diarize() does): the root process_audio then
        gets past its `segment["start"]` subscripts (audio_pipeline.py:676-682) and reaches the merge."""

        def process_file(self, audio_path):
            return [s.to_dict() for s in super().process_file(audio_path)]

    for layout, mod, dmod in (("vocalis", voc_ap, voc_diar), ("root", root_ap, root_diar),
                              ("root_dict_segments", root_ap, None)):
        seg_model = "pyannote/segmentation-3.0" if layout == "vocalis" else ""
        emb_model = "3dspeaker_speech_eres2net_sv_en_voxceleb_16k.onnx|25.3MB" if layout == "vocalis" else ""
        if dmod is None:
            dmod = types.SimpleNamespace(SpeakerDiarizer=DictDiarizer)
        for asr_name, asr_out in ASR_OUTPUTS.items():
            for tname, turns in TURNS.items():
                mod._PIPELINE_CACHE.update(transcription_model=None, diarizer=None)
                p = mod.AudioProcessingPipeline()
                asr = FakeASR(asr_out)
                p.transcription_model = asr
                mod._PIPELINE_CACHE["transcription_model"] = asr
                dz = dmod.SpeakerDiarizer(segmentation_model=seg_model, embedding_model=emb_model, num_speakers=2,
                                          threshold=0.5)
                _FakeSherpa.turns = list(turns)
                p.diarizer = dz
                mod._PIPELINE_CACHE["diarizer"] = dz
                r = p.process_audio("/tmp/upload.flac", "transcribe", seg_model, emb_model, 2, 0.5)
                add(layout, "process_audio", asr_name, tname, r, asr.calls)
                _FakeSherpa.turns = list(turns)
                d = p.diarize("/tmp/upload.flac", 2)
                add(layout, "diarize", asr_name, tname, d, [])
                try:
                    m = p._merge_transcription_with_diarization(json.loads(json.dumps(asr_out)), d)
                    add(layout, "merge", asr_name, tname, m, [])
                except Exception as e:  # the vocalis merge on raw HF chunks: KeyError 'start'
                    add(layout, "merge", asr_name, tname, None, [], exception=f"{type(e).__name__}: {e}")
        if layout == "root_dict_segments":
            continue
        # transcribe(): the exact call the reference makes, and its error convention
        for task in ("transcribe", "translate"):
            p = mod.AudioProcessingPipeline()
            asr = FakeASR(ASR_OUTPUTS["three_chunks"])
            p.transcription_model = asr
            r = p.transcribe("/tmp/upload.wav", task)
            add(layout, "transcribe", "three_chunks", None, r, asr.calls, task=task)
        p = mod.AudioProcessingPipeline()
        p.transcription_model = FakeASR(RuntimeError("boom"))
        add(layout, "transcribe", "raises", None, p.transcribe("/tmp/upload.wav"), [], task="transcribe")
        mod._PIPELINE_CACHE.update(transcription_model=None)
        p = mod.AudioProcessingPipeline()
        p.load_transcription_model = lambda *a, **k: False
        add(layout, "transcribe", "load_fails", None, p.transcribe("/tmp/upload.wav"), [], task="transcribe")
    # the diarizer's own merge and conversation formatting on segment-shaped input
    segs = [{"text": " a", "start": 0.0, "end": 2.0}, {"text": " b", "start": 2.0, "end": 5.0},
            {"text": " c", "start": 5.0, "end": 5.0}, {"text": " d", "start": 30.0, "end": 31.0}]
    for tname, turns in TURNS.items():
        dsegs = [{"speaker": f"Speaker {s}", "start": a, "end": b, "score": 1.0} for s, a, b in turns]
        m = voc_diar.SpeakerDiarizer().create_transcript_with_speakers(segs, dsegs)
        out["cases"].append({"layout": "vocalis", "fn": "create_transcript_with_speakers", "turns": tname,
                             "segments": segs, "result": m, "conversation": voc_diar.format_as_conversation(m)})
    out["cases"].append(_overlap_case(voc_ap, voc_diar))
    with open(os.path.join(HERE, "ref_merge.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote ref_merge.json:", len(out["cases"]), "cases")


if __name__ == "__main__":
    main()
