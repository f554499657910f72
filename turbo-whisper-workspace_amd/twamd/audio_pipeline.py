"""AudioProcessingPipeline surface of the transcription hot path (§8b).

Two ways to use it:

1. Inside the reference (the drop-in): `install(vocalis.core.audio_pipeline)` replaces
   `AudioProcessingPipeline.load_transcription_model` (/root/reference/vocalis/core/audio_pipeline.py:171-208) so
   the callable it caches in `_PIPELINE_CACHE['transcription_model']` is a `TurboTranscriber` instead of
   `transformers.pipeline(...)`. `transcribe` (:323-369), `process_audio` (:567-688), diarization, the LLM helpers
   and `POST /api/transcribe` (vocalis/api/main.py:89-131) stay the reference's own code.
2. Standalone: `AudioProcessingPipeline` below mirrors the reference class's transcription surface with the same
   names, arguments, result schema and error conventions, for deployments without the reference package.
   Diarization stays a host-CPU concern (north_star): pass `diarize_fn(audio_path, num_speakers) -> [segments]`
   to run one; without it the reference's no-diarization merge branch applies (alternating speakers, :709-720).
"""
from __future__ import annotations

import os
import time
from typing import Any, Callable, Dict, List, Optional

from . import audio
from .pipeline import TurboTranscriber

# process-wide model cache, as the reference's module-level _PIPELINE_CACHE (:28-32)
_PIPELINE_CACHE: Dict[str, Any] = {"transcription_model": None, "diarization_model": None}

DEFAULT_MODEL = "openai/whisper-large-v3"  # the reference's default name (:171)


def _engine_options() -> Dict[str, Any]:
    """Engine construction from the environment (the reference reads LLM_MODEL etc. the same way):
    TW_CHECKPOINT = local HF Whisper directory (no hub access offline), TW_MAX_BATCH, TW_SEED, TW_DEVICE, and
    TW_PRECISION = bf16 (default) or fp32 (BASELINE configs[0]: the reference's torch_dtype=torch.float32 load,
    /root/reference/vocalis/core/audio_pipeline.py:199)."""
    return {"checkpoint": os.environ.get("TW_CHECKPOINT") or None,
            "max_batch": int(os.environ.get("TW_MAX_BATCH", "24")),
            "seed": int(os.environ.get("TW_SEED", "1234")),
            "device": os.environ.get("TW_DEVICE", "cuda"),
            "precision": os.environ.get("TW_PRECISION", "bf16")}


def build_transcriber(model_name: str = DEFAULT_MODEL, **overrides) -> TurboTranscriber:
    """The engine for `model_name` from a LOCAL checkpoint (TW_CHECKPOINT, or model_name naming a directory). The
    reference either loads real weights or fails, so without a checkpoint this raises (load_transcription_model
    turns that into its False / "Failed to load transcription model" convention) instead of serving gibberish from
    seeded synthetic weights; TW_ALLOW_SYNTHETIC=1 opts into the synthetic preset (tests, benchmarks)."""
    opts = _engine_options()
    opts.update(overrides)
    if opts.get("checkpoint") is None and not os.path.isdir(model_name) and \
            os.environ.get("TW_ALLOW_SYNTHETIC", "0") != "1":
        raise RuntimeError(f"no local checkpoint for {model_name!r}: set TW_CHECKPOINT to a Hugging Face Whisper "
                           f"directory (config.json, *.safetensors, vocab.json), or TW_ALLOW_SYNTHETIC=1 for seeded "
                           f"synthetic weights")
    return TurboTranscriber.from_pretrained(model_name, **opts)


def load_transcription_model(self, model_name: str = DEFAULT_MODEL) -> bool:
    """Replacement body of AudioProcessingPipeline.load_transcription_model (:171-208): same cache protocol,
    same return convention (True, or False after printing the error)."""
    cache = getattr(self, "_tw_cache", _PIPELINE_CACHE)
    if cache.get("transcription_model") is not None:
        self.transcription_model = cache["transcription_model"]
        print(f"Using cached transcription model: {model_name}")
        return True
    try:
        print(f"Loading MI355X transcription engine for {model_name}...")
        self.transcription_model = build_transcriber(model_name)
        cache["transcription_model"] = self.transcription_model
        return True
    except Exception as e:  # the reference's convention: print, return False
        print(f"Error loading transcription model: {e}")
        return False


def install(reference_module, overlap_diarization: bool = False) -> None:
    """Patch the reference's AudioProcessingPipeline (module `vocalis.core.audio_pipeline` or the root
    `audio_pipeline`) so its transcription callable is the MI355X engine. Its own _PIPELINE_CACHE is used.

    overlap_diarization (BASELINE config 4): `process_audio` still runs the reference's own code, but the host-CPU
    diarizer (sherpa-onnx, vocalis/core/model.py:451-470) is started in a worker thread when the call begins, so it
    runs while the GPU transcribes instead of after it (the reference runs them back to back,
    vocalis/core/audio_pipeline.py:589-624). The reference's later `load_diarizer` / `diarize` calls with the same
    arguments then return the worker's results, so every result key is identical and only processing_times
    change."""
    cls = reference_module.AudioProcessingPipeline
    cache = reference_module._PIPELINE_CACHE

    def _load(self, model_name: str = DEFAULT_MODEL) -> bool:
        self._tw_cache = cache
        return load_transcription_model(self, model_name)

    _load.__doc__ = load_transcription_model.__doc__
    cls.load_transcription_model = _load
    if overlap_diarization and not getattr(cls, "_tw_overlap", False):
        _install_overlap(cls)


def _install_overlap(cls) -> None:
    import concurrent.futures
    import inspect
    import threading

    orig_process, orig_load, orig_diarize = cls.process_audio, cls.load_diarizer, cls.diarize
    defaults = {k: v.default for k, v in inspect.signature(orig_process).parameters.items()
                if v.default is not inspect.Parameter.empty}

    def process_audio(self, audio_path, *args, **kwargs):
        bound = inspect.signature(orig_process).bind(self, audio_path, *args, **kwargs)
        a = {**defaults, **bound.arguments}
        load_key = (a["segmentation_model"], a["embedding_model"], a["num_speakers"], a["threshold"])
        diar_key = (audio_path, a["num_speakers"])
        pool = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="tw-diarize")
        loaded = threading.Event()
        state = {"load_key": load_key, "diar_key": diar_key, "loaded": loaded}

        def work():
            try:
                need = self.diarizer is None or self.diarizer.segmentation_model != load_key[0] or \
                    self.diarizer.embedding_model != load_key[1]
                state["load_result"] = orig_load(self, *load_key) if need else True
            finally:
                loaded.set()
            return orig_diarize(self, *diar_key)

        state["future"] = pool.submit(work)
        pool.shutdown(wait=False)
        self._tw_prefetch = state
        try:
            return orig_process(self, audio_path, *args, **kwargs)
        finally:
            self._tw_prefetch = None

    def load_diarizer(self, segmentation_model, embedding_model, num_speakers=2, threshold=0.5):
        st = getattr(self, "_tw_prefetch", None)
        if st is not None and st["load_key"] == (segmentation_model, embedding_model, num_speakers, threshold):
            st["loaded"].wait()
            if "load_result" in st:
                return st["load_result"]
        return orig_load(self, segmentation_model, embedding_model, num_speakers, threshold)

    def diarize(self, audio_path, num_speakers=2):
        st = getattr(self, "_tw_prefetch", None)
        if st is not None and st.get("future") is not None and st["diar_key"] == (audio_path, num_speakers):
            fut, st["future"] = st["future"], None
            return fut.result()
        return orig_diarize(self, audio_path, num_speakers)

    process_audio.__doc__ = orig_process.__doc__
    cls.process_audio, cls.load_diarizer, cls.diarize = process_audio, load_diarizer, diarize
    cls._tw_overlap = True


def create_transcript_with_speakers(transcript_segments, diarization_segments, layout: str = "vocalis"):
    """SpeakerDiarizer.create_transcript_with_speakers: vocalis/core/diar.py:184-247 (dict or DiarizationSegment
    diarization entries) and, for layout="root", diar.py:171-228 (attribute access only, so dict entries raise
    AttributeError there, as in the reference). Transcript segments need 'text', 'start', 'end' (HF chunks lack
    'start': KeyError, as in the reference)."""
    result: List[Dict[str, Any]] = []
    if not diarization_segments:
        return [{"speaker": f"Speaker {i % 2}", "text": seg["text"], "start": seg["start"], "end": seg["end"]}
                for i, seg in enumerate(transcript_segments)]
    for seg in transcript_segments:
        start_time, end_time, text = seg["start"], seg["end"], seg["text"]
        speaker, max_overlap = "Unknown", 0
        for d in diarization_segments:
            if layout == "vocalis" and isinstance(d, dict):
                ds, de, sp = d["start"], d["end"], d["speaker"]
            else:
                ds, de, sp = d.start_time, d.end_time, f"Speaker {d.speaker_id}"
            overlap = max(0, min(end_time, de) - max(start_time, ds))
            if overlap > max_overlap:
                max_overlap, speaker = overlap, sp
        if max_overlap == 0:
            speaker = f"Speaker {len(result) % 2}"
        result.append({"speaker": speaker, "text": text, "start": start_time, "end": end_time})
    return result


class AudioProcessingPipeline:
    """Standalone mirror of the reference class's transcription surface."""

    def __init__(self, diarize_fn: Optional[Callable[[str, int], List[Dict[str, Any]]]] = None,
                 transcriber: Optional[TurboTranscriber] = None, overlap_diarization: bool = False):
        self.transcription_model = transcriber
        self.diarize_fn = diarize_fn
        # BASELINE config 4: run the host-CPU diarizer concurrently with the GPU transcription (the reference runs
        # them back to back, :589-624); results are identical, only processing_times change
        self.overlap_diarization = overlap_diarization
        import torch

        self.gpu_available = torch.cuda.is_available()  # the reference's _setup_gpu result (:49-114)
        if transcriber is not None and _PIPELINE_CACHE["transcription_model"] is None:
            _PIPELINE_CACHE["transcription_model"] = transcriber

    load_transcription_model = load_transcription_model

    def transcribe(self, audio_path: str, task: str = "transcribe", return_timestamps: bool = True) -> Dict[str, Any]:
        """:323-369 — the reference's exact call (chunk_length_s=60, batch_size=512 on a GPU / 32 on CPU,
        stride_length_s=5, generate_kwargs={"task": task}) on the engine."""
        if self.transcription_model is None:
            if not self.load_transcription_model():
                return {"error": "Failed to load transcription model"}
        try:
            return self.transcription_model(audio_path, chunk_length_s=60,
                                            batch_size=512 if self.gpu_available else 32, stride_length_s=5,
                                            generate_kwargs={"task": task}, return_timestamps=return_timestamps)
        except Exception as e:
            print(f"Error during transcription: {e}")
            return {"error": f"Transcription error: {str(e)}"}

    def _merge_transcription_with_diarization(self, transcription, diarization_segments):
        """:690-726. With no diarization segments: alternating speakers over the transcript chunks, whose
        `start`/`end` keys HF chunks do not carry (the reference reads them with .get(..., 0))."""
        if isinstance(transcription, dict) and "segments" in transcription:
            segs = transcription["segments"]
        elif isinstance(transcription, dict) and "chunks" in transcription:
            segs = transcription["chunks"]
        else:
            segs = transcription
        if not diarization_segments:
            return [{"speaker": f"Speaker {i % 2}", "text": s.get("text", ""), "start": s.get("start", 0),
                     "end": s.get("end", 0)} for i, s in enumerate(segs)]
        # the reference hands these to SpeakerDiarizer.create_transcript_with_speakers (vocalis/core/diar.py:
        # 184-247), which reads seg['start'] and so raises KeyError on HF chunks; reproduced as-is
        return create_transcript_with_speakers(segs, diarization_segments)

    def process_audio(self, audio_path: str, task: str = "transcribe",
                      segmentation_model: str = "pyannote/segmentation-3.0",
                      embedding_model: str = "3dspeaker_speech_eres2net_sv_en_voxceleb_16k.onnx|25.3MB",
                      num_speakers: int = 2, threshold: float = 0.5) -> Dict[str, Any]:
        """:567-688 — transcription + (host) diarization + merge; same result keys and error convention."""
        start_time = time.time()
        processing_times: Dict[str, float] = {}
        try:
            diar_future = None
            if self.overlap_diarization and self.diarize_fn:
                import concurrent.futures

                pool = concurrent.futures.ThreadPoolExecutor(max_workers=1)
                t_d = time.time()
                diar_future = pool.submit(self.diarize_fn, audio_path, num_speakers)
                pool.shutdown(wait=False)
            t0 = time.time()
            transcription = self.transcribe(audio_path, task)
            processing_times["transcription"] = time.time() - t0
            if isinstance(transcription, dict) and "error" in transcription:
                return transcription
            text = transcription.get("text", "")
            segments = transcription.get("chunks", [])
            if not segments and "segments" in transcription:
                segments = transcription["segments"]
            if not segments:
                segments = [{"text": text, "start": 0, "end": 0}]
            if diar_future is not None:
                diarization_segments = diar_future.result()
                processing_times["diarization"] = time.time() - t_d
            else:
                t0 = time.time()
                diarization_segments = self.diarize_fn(audio_path, num_speakers) if self.diarize_fn else []
                processing_times["diarization"] = time.time() - t0
            merged_segments = self._merge_transcription_with_diarization(transcription, diarization_segments)
            try:
                duration = audio.duration_seconds(audio_path)
            except Exception:
                duration = max([s.get("end", 0) for s in merged_segments]) if merged_segments else 0
            processing_times["total"] = time.time() - start_time
            return {"text": text, "segments": segments, "diarization_segments": diarization_segments,
                    "merged_segments": merged_segments, "duration": duration, "processing_times": processing_times}
        except Exception as e:
            import traceback

            traceback.print_exc()
            return {"error": f"Processing error: {str(e)}"}


class RootAudioProcessingPipeline(AudioProcessingPipeline):
    """Mirror of the ROOT copy's result layout (/root/reference/audio_pipeline.py:610-799; used by app.py:66,
    security_monitor.py:21 and the bar scripts): the result carries audio_path/task/num_speakers/threshold, the
    transcript under "chunks", the diarization as "segments", and the merge converts each chunk's `timestamp` into
    start/end (:779-789) before SpeakerDiarizer.create_transcript_with_speakers (diar.py:171-228, attribute access:
    dict diarization entries raise AttributeError, and the root diarizer's DiarizationSegment objects are not
    subscriptable at :676-682, so any non-empty diarization ends in the reference's "Processing error" result)."""

    def _merge_transcription_with_diarization(self, transcription, diarization_segments):
        chunks = transcription.get("chunks", [])
        if not chunks:
            return []
        segs = [{"text": c["text"], "start": c["timestamp"][0], "end": c["timestamp"][1]} for c in chunks
                if "timestamp" in c]
        if not segs:
            return []
        return create_transcript_with_speakers(segs, diarization_segments, layout="root")

    def process_audio(self, audio_path: str, task: str = "transcribe", segmentation_model: str = "",
                      embedding_model: str = "", num_speakers: int = 2, threshold: float = 0.5) -> Dict[str, Any]:
        result: Dict[str, Any] = {"audio_path": audio_path, "task": task, "num_speakers": num_speakers,
                                  "threshold": threshold, "processing_times": {}}
        try:
            start_time = time.time()
            result["duration"] = audio.duration_seconds(audio_path)
            if self.transcription_model is None and not self.load_transcription_model():
                return {"error": "Failed to load transcription model"}
            diar_future = None
            if self.overlap_diarization and self.diarize_fn:
                import concurrent.futures

                pool = concurrent.futures.ThreadPoolExecutor(max_workers=1)
                t_d = time.time()
                diar_future = pool.submit(self.diarize_fn, audio_path, num_speakers)
                pool.shutdown(wait=False)
            t0 = time.time()
            transcription = self.transcribe(audio_path, task)
            result["processing_times"]["transcription"] = time.time() - t0
            if isinstance(transcription, dict) and "error" in transcription:
                return transcription
            result["text"] = transcription.get("text", "")
            result["chunks"] = transcription.get("chunks", [])
            if diar_future is not None:
                diarization_segments = diar_future.result()
                result["processing_times"]["diarization"] = time.time() - t_d
            else:
                t0 = time.time()
                diarization_segments = self.diarize_fn(audio_path, num_speakers) if self.diarize_fn else []
                result["processing_times"]["diarization"] = time.time() - t0
            result["segments"] = [{"start": s["start"], "end": s["end"], "speaker": s["speaker"],
                                   "text": s.get("text", "")} for s in diarization_segments]
            t0 = time.time()
            result["merged_segments"] = self._merge_transcription_with_diarization(transcription,
                                                                                   diarization_segments)
            result["processing_times"]["merge"] = time.time() - t0
            result["processing_times"]["total"] = time.time() - start_time
            return result
        except Exception as e:
            print(f"Error in audio processing pipeline: {e}")
            return {"error": f"Processing error: {str(e)}"}
