"""TurboTranscriber: the drop-in for the ASR callable the reference builds and calls.

Reference: AudioProcessingPipeline.load_transcription_model stores
`transformers.pipeline("automatic-speech-recognition", ...)` in `self.transcription_model`
(/root/reference/vocalis/core/audio_pipeline.py:171-208) and `transcribe` calls it as
    outputs = self.transcription_model(audio_path, chunk_length_s=60, batch_size=512|32,
                                       stride_length_s=5, generate_kwargs={"task": task},
                                       return_timestamps=return_timestamps)      (:351-358)
TurboTranscriber.__call__ accepts the same arguments and returns the same dict
({"text": str, "chunks": [{"timestamp": (start, end), "text": str}, ...]}), following
AutomaticSpeechRecognitionPipeline preprocess / _forward / postprocess
($TF/pipelines/automatic_speech_recognition.py:345-710) with every numeric stage on the GPU engine.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from . import audio, dist
from .config import PRESETS, GenerationSettings, WhisperDims
from .engine import WhisperEngine
from .engine_f32 import WhisperEngineF32
from .frontend import CHUNK_SAMPLES, SAMPLE_RATE, Window, chunk_windows, time_precision
from .segments import FallbackConfig, pad_right
from .tokenizer import LANGUAGE_NAMES, WhisperVocab, decode_asr
from .weights import build_weights

_NAME_TO_CODE = {v: k for k, v in LANGUAGE_NAMES.items()}

# AutomaticSpeechRecognitionPipeline._default_generation_config ($TF/pipelines/automatic_speech_recognition.py:160-163)
PIPELINE_DEFAULT_NUM_BEAMS = 5
PIPELINE_DEFAULT_MAX_NEW_TOKENS = 256
_GLOBAL_DEFAULT_MAX_LENGTH = 20  # GenerationConfig's own max_length default


def resolve_decode(gen: GenerationSettings, gk: Dict[str, Any]) -> Dict[str, Any]:
    """The decode the HF ASR pipeline runs when called the way the reference calls it.

    Pipeline.__init__ ($TF/pipelines/base.py:887-908) prepares the pipeline's generation config from its class
    default {max_new_tokens: 256, num_beams: 5} through `_prepare_generation_config` ($TF/generation/utils.py:
    1771-1830): values the default sets are kept, only unset ones are filled from the checkpoint's
    generation_config.json. So `num_beams` is 5 whatever the checkpoint says, unless the call passes it in
    generate_kwargs (the reference passes only {"task": task}, vocalis/core/audio_pipeline.py:351-358). The pipeline's
    max_new_tokens=256 is then dropped in favour of the checkpoint's max_length when that is set and differs from
    GenerationConfig's global default 20 (Whisper checkpoints set 448). Pinned by tests/golden/defaults.json, made
    by transformers itself (tests/golden/make_golden.py defaults).

    Returns {"num_beams", "max_new_tokens"} (max_new_tokens None = bounded by max_length)."""
    nb = gk.get("num_beams")
    mnt = gk.get("max_new_tokens")
    if mnt is None and "max_new_tokens" not in gk:
        ml = gen.max_length if gen.max_length_set else _GLOBAL_DEFAULT_MAX_LENGTH
        mnt = None if ml != _GLOBAL_DEFAULT_MAX_LENGTH else PIPELINE_DEFAULT_MAX_NEW_TOKENS
    return {"num_beams": int(nb) if nb is not None else PIPELINE_DEFAULT_NUM_BEAMS, "max_new_tokens": mnt}


class TurboTranscriber:
    """Callable with the HF ASR pipeline signature, backed by WhisperEngine (HIP)."""

    def __init__(self, engine: WhisperEngine, vocab: WhisperVocab, sampling_rate: int = SAMPLE_RATE):
        self.engine = engine
        self.vocab = vocab
        self.sampling_rate = sampling_rate
        self.gen = engine.gen
        # A share of n <= max_batch windows is split into two sub-batches when n >= 2 * sub_batch_min, so that
        # run_batches' two-slot pipeline encodes the second beside the first one's decode (a single 1-h request on
        # 8 GPUs gives each rank 15 windows: one batch, no overlap). None: never split (see DESIGN.md §C3 for the
        # measured trade: the decode step is latency-bound, so two decodes of 8 cost about two of 15).
        self.sub_batch_min: Optional[int] = None
        self.sample_seed = 0  # key of the fallback sampler (generate_kwargs "seed" overrides it per call)
        self._staging = None  # two pinned host buffers for the per-batch waveform upload (host-array inputs)

    # -------------------------------------------------------------- construction
    @staticmethod
    def from_pretrained(model: str = "large-v3-turbo", checkpoint: Optional[str] = None, seed: int = 1234,
                        max_batch: int = 24, device: str = "cuda", use_graphs: bool = True,
                        max_beams: int = PIPELINE_DEFAULT_NUM_BEAMS, enc_fp8: Optional[bool] = None,
                        precision: str = "bf16", fused_decode: bool = False) -> "TurboTranscriber":
        """`model`: a preset name (synthetic seeded weights) or, via `checkpoint`, a LOCAL Hugging Face
        Whisper directory (config.json, *.safetensors, vocab.json, generation_config.json). max_beams: decoder rows
        per window (the callable's default decode is beam-5, as the HF pipeline's; 1 = greedy-only engine). enc_fp8:
        run the encoder projections on MX fp8 (BASELINE config 5; default: env TW_ENC_FP8). precision: "bf16" (the
        engine's default arithmetic) or "fp32" (every operand, activation and cache f32: BASELINE configs[0], the
        reference's torch_dtype=torch.float32 load; WhisperEngineF32). fused_decode: greedy / sampled decode passes of
        at most 4 rows run the decoder's layers as one persistent launch (WhisperEngine.dec_fused_alone; 9-14 % less
        per step at 1-4 rows, rounding like, not bit-equal to, the default launch chain)."""
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision {precision!r}: 'bf16' or 'fp32'")
        if checkpoint is None and model not in PRESETS and os.path.isdir(model):
            checkpoint = model
        if checkpoint is not None:
            dims = _dims_from_checkpoint(checkpoint)
            gen = GenerationSettings.from_checkpoint(checkpoint, dims)
            vocab = WhisperVocab.from_checkpoint(checkpoint, gen.special)
        else:
            key = model.split("/")[-1].replace("whisper-", "")
            if key not in PRESETS:
                raise ValueError(f"unknown model {model!r}: give a preset ({sorted(PRESETS)}) or a local checkpoint dir")
            dims = PRESETS[key]
            gen = GenerationSettings.default(dims)
            vocab = WhisperVocab.synthetic(gen.special)
        f32 = precision == "fp32"
        weights = build_weights(dims, seed=seed, checkpoint=checkpoint, dtype=torch.float32 if f32 else torch.bfloat16)
        cls = WhisperEngineF32 if f32 else WhisperEngine
        eng = cls(weights, gen, max_batch=max_batch, device=device, use_graphs=use_graphs, max_beams=max_beams,
                  enc_fp8=enc_fp8)
        eng.dec_fused_alone = bool(fused_decode)
        return TurboTranscriber(eng, vocab)

    # -------------------------------------------------------------- call
    def close(self) -> None:
        """Release the engine (WhisperEngine.close) and the pinned staging buffers; the callable is unusable after."""
        self._staging = None
        if self.engine is not None:
            self.engine.close()

    def __enter__(self) -> "TurboTranscriber":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __call__(self, inputs: Union[str, bytes, np.ndarray, dict], *, chunk_length_s: float = 0,
                 stride_length_s=None, batch_size: int = 1, generate_kwargs: Optional[Dict[str, Any]] = None,
                 return_timestamps: Union[bool, str] = False, return_language: bool = False, **kwargs) -> dict:
        word = return_timestamps == "word"
        if return_timestamps == "char":
            raise ValueError("Whisper cannot return `char` timestamps, only word level or segment level timestamps.")
        gk = dict(generate_kwargs or {})
        gk.update({k: kwargs.pop(k) for k in list(kwargs) if k in ("max_new_tokens", "language", "task", "num_beams")})
        dec = resolve_decode(self.gen, gk)  # as shipped: beam-5, bounded by max_length (see resolve_decode)
        gk.pop("num_beams", None)
        gk.pop("max_new_tokens", None)
        num_beams = dec["num_beams"]
        if num_beams < 1 or num_beams > 8:
            raise ValueError(f"num_beams={num_beams}: the engine supports 1 (greedy) to 8 beams")
        task = gk.pop("task", None)
        language = gk.pop("language", None)
        max_new_tokens = dec["max_new_tokens"]
        # extension (not a transformers generate kwarg): bound the seek loop to this many passes per window
        max_passes = gk.pop("max_passes", None)
        # prompt every seek pass after a window's first with its previous segments (generate()'s
        # condition_on_prev_tokens; the batch then shapes results through the left padding, so batch_size is kept)
        cond = bool(gk.pop("condition_on_prev_tokens", None) or False)
        # generate()'s initial prompt (<|startofprev|> + text tokens, WhisperProcessor.get_prompt_ids) and where it
        # conditions (first-segment / all-segments)
        prompt = {}
        if gk.get("prompt_ids") is not None:
            pid = gk.pop("prompt_ids")
            pid = pid.tolist() if hasattr(pid, "tolist") else list(pid)
            prompt = {"prompt_ids": [int(t) for t in np.asarray(pid).reshape(-1)],
                      "prompt_condition_type": gk.pop("prompt_condition_type", None)}
        gk.pop("prompt_ids", None)
        if "prompt_condition_type" in gk:
            prompt.setdefault("prompt_condition_type", gk.pop("prompt_condition_type"))
        # (_set_prompt_condition_type's checks, generation_whisper.py:1732-1748, before any work is queued)
        pct = prompt.get("prompt_condition_type") or "first-segment"
        if pct not in ("first-segment", "all-segments"):
            raise ValueError(f"`prompt_condition_type={pct} does not exist. Make sure to set `prompt_condition_type` "
                             "to one of first-segment, all-segments")
        if pct == "all-segments" and not cond:
            raise ValueError("Make sure to set `condition_on_prev_tokens=True` when setting "
                             "`prompt_condition_type='all-segments'`.")
        if "prompt_ids" not in prompt:
            prompt = {}
        fallback = self._fallback_config(gk)
        if gk:
            raise ValueError(f"generate_kwargs not supported by this engine: {sorted(gk)}")
        st = self.gen.special
        if not st.is_multilingual and (task is not None or language is not None):
            raise ValueError("Cannot specify `task` or `language` for an English-only model.")

        rank, world = dist.world()
        sharded = dist.collective_path()  # (world > 1, or a forced collective in a world of one)
        dev = getattr(self.engine, "device", None)
        wav, load_err = None, None
        if rank == 0:
            try:
                wav = audio.load_input(inputs, self.sampling_rate, dev)
            except Exception as e:  # raised below, after the other ranks have been told (no rank left waiting)
                load_err = e
        if sharded:  # SPMD: every rank calls with the same arguments; rank 0 decoded the input
            # (the waveform stays in device memory: each rank copies its windows out of it on the GPU)
            wav = dist.broadcast_waveform(wav, failed=load_err is not None, as_tensor=True)
        if load_err is not None:
            raise load_err
        if chunk_length_s:
            windows = list(chunk_windows(len(wav), chunk_length_s, stride_length_s, self.sampling_rate))
            if not windows:  # an empty input: the pipeline's chunk iterator yields nothing and its first next()
                # raises StopIteration (tests/golden/edge.json), which transcribe() reports as "Transcription error: "
                raise StopIteration
            with_stride = True
        elif len(wav) > CHUNK_SAMPLES:  # long-form: one sequential generate() over the whole input (asr:450-457)
            return self._long_form(wav, task=task, language=language, return_timestamps=return_timestamps,
                                   return_language=return_language, max_new_tokens=max_new_tokens,
                                   num_beams=num_beams, max_passes=max_passes, fallback=fallback, condition=cond,
                                   prompt=prompt)
        else:
            windows = [Window(0, len(wav), 0, 0, True)]
            with_stride = False
        lang_id = self._lang_id(language)

        def run(w, ws):
            base = windows.index(ws[0]) if ws else 0  # this shard's first global window (the sampler's row keys)
            # (batch composition shapes results with word timestamps — standardised over the padded batch —, with
            # conditioned prompts — their left padding — and with beams under the fallback — a sampling round turns the
            # rest of that generate() call greedy —, so batch_size is kept there)
            grouped = word or cond or (fallback.active and num_beams > 1)
            kw = dict(task=task, lang_id=lang_id, return_timestamps=bool(return_timestamps) or word,
                      max_new_tokens=max_new_tokens, num_beams=num_beams, max_passes=max_passes,
                      **({"fallback": fallback, "window_base": base} if fallback.active else {}),
                      **({"condition_on_prev_tokens": True} if cond else {}),
                      **({"prompt": prompt} if prompt else {}),
                      **({"group": batch_size} if grouped else {}))
            if word:  # token times ride along as floats after the tokens (one all-gather carries both)
                nf = [-(-min(x.length, CHUNK_SAMPLES) // 160) for x in ws]
                toks = self.transcribe_windows(w, ws, word_timestamps=True, num_frames=nf, **kw)
                return [(t, ts) for t, ts in zip(toks, self.last_window_token_timestamps)]
            return self.transcribe_windows(w, ws, **kw)

        # one window shard per rank + one all-gather of the token arrays (twamd.dist); plain call on 1 GPU
        outputs = dist.transcribe_sharded(run, wav, windows, timed=word) if sharded else run(wav, windows)
        model_outputs = []
        for w, toks in zip(windows, outputs):
            if word:
                toks, tts = toks
                o = {"tokens": toks, "token_timestamps": tts}
            else:
                o = {"tokens": toks}
            if with_stride:
                sr = self.sampling_rate
                o["stride"] = (w.length / sr, w.stride_left / sr, w.stride_right / sr)
            model_outputs.append(o)
        kw = dict(return_timestamps="word" if word else bool(return_timestamps), return_language=return_language,
                  time_precision=time_precision(self.engine.d.max_source_positions))
        # sharded: every rank stitches its own windows and the pieces are merged (dist.stitch_sharded: the serial
        # _decode_asr result, without rank 0 walking every window of the call)
        text, optional = (dist.stitch_sharded(self.vocab, model_outputs, **kw) if sharded else
                          decode_asr(self.vocab, model_outputs, **kw))
        return {"text": text, **optional}

    def _lang_id(self, language: Optional[str]) -> Optional[int]:
        if language is None:
            return None
        code = language.lower()
        code = _NAME_TO_CODE.get(code, code)
        tok = f"<|{code}|>"
        lt = self.gen.special.lang_to_id()
        if tok not in lt:
            raise ValueError(f"Unsupported language: {language}.")
        return lt[tok]

    def _long_form(self, wav, *, task, language, return_timestamps, return_language, max_new_tokens, num_beams,
                   max_passes, fallback, condition=False, prompt=None) -> dict:
        """An input longer than 30 s without chunk_length_s: the pipeline hands generate() the features of the whole
        input (feature extractor with truncation=False, padding="longest", $TF/pipelines/automatic_speech_recognition
        .py:450-457) and generate() runs its seek loop over all of them (generation_whisper.py:647-968: is_shortform
        False, max_frames = the input's frames, every pass the 30-s segment at seek, zero padded). One chunk, no
        stride; every rank computes it (nothing to shard: each pass depends on the previous one's seek)."""
        # (the pipeline never passes return_timestamps=False on to generate(), asr:506-508, so generate() switches
        # timestamps on for a long-form input instead of raising; the text is then decoded without them)
        word = return_timestamps == "word"
        eng = self.engine
        lang_id = self._lang_id(language)
        x = wav if torch.is_tensor(wav) else torch.from_numpy(np.ascontiguousarray(wav, np.float32))
        eng.set_long_input(x)
        try:
            kw = {"fallback": fallback} if fallback.active else {}
            kw.update(prompt or {})
            if word:  # num_frames: the feature extractor's attention mask, one per hop (_set_num_frames)
                kw.update(word_timestamps=True, num_frames=[-(-int(x.shape[0]) // 160)])
            toks = eng.generate(1, task=task, lang_ids=None if lang_id is None else [lang_id],
                                max_new_tokens=max_new_tokens, return_timestamps=True, num_beams=num_beams,
                                max_passes=max_passes, condition_on_prev_tokens=condition, **kw)[0]
        finally:
            eng.set_long_input(None)
        self.last_window_langs = list(eng.last_langs)
        self.last_window_passes = list(eng.last_passes)
        self.last_window_prefixes = list(eng.last_pass_prefixes)
        out = {"tokens": toks}
        if word:
            self.last_window_token_timestamps = list(eng.last_token_timestamps)
            out["token_timestamps"] = eng.last_token_timestamps[0]
        text, optional = decode_asr(self.vocab, [out], return_timestamps="word" if word else bool(return_timestamps),
                                    return_language=return_language,
                                    time_precision=time_precision(self.engine.d.max_source_positions))
        return {"text": text, **optional}

    def transcribe_windows(self, wav: np.ndarray, windows: Sequence[Window], task: Optional[str],
                           lang_id: Optional[int], return_timestamps: bool,
                           max_new_tokens: Optional[int] = None, num_beams: int = 1, word_timestamps: bool = False,
                           num_frames: Optional[Sequence[int]] = None, group: Optional[int] = None,
                           max_passes: Optional[int] = None, fallback: Optional[FallbackConfig] = None,
                           window_base: int = 0, condition_on_prev_tokens: bool = False,
                           prompt: Optional[dict] = None) -> List[List[int]]:
        """Log-mel + generate for every window; returns per-window token sequences (generate() output,
        right-padded with the pad token within each engine batch, as the HF batch output is). Batches of
        max_batch windows go through WhisperEngine.run_batches: batch k+1 is encoded while batch k decodes.

        group: windows per engine batch when the batch's composition changes results. That is the case for
        word timestamps, whose per-pass standardisation runs over the padded batch, and for
        condition_on_prev_tokens, whose prompts are left padded to the batch's longest, so the pipeline's
        `batch_size` (its DataLoader batch, $TF/pipelines/base.py:1319-1339) is honoured there; segment-level
        tokens are per-window results, so batching is then only a schedule: the windows are cut into near-equal
        batches of at most max_batch (and into two when sub_batch_min says so).

        wav: a host array, or a torch tensor (a rank's copy of the broadcast waveform, in device memory)."""
        eng = self.engine
        if group:
            B = max(1, min(int(group), eng.max_batch))
            sizes = [min(B, len(windows) - b0) for b0 in range(0, len(windows), B)]
        else:
            sizes = batch_sizes(len(windows), eng.max_batch, self.sub_batch_min)
        offs = np.cumsum([0] + sizes).tolist()
        parts = [windows[offs[k]: offs[k + 1]] for k in range(len(sizes))]
        on_device = torch.is_tensor(wav)

        def load(k):  # called on the engine's encoder stream
            part = parts[k]
            if on_device:  # device-to-device slices of the rank's waveform copy
                dst = eng.wave[: len(part)]
                for j, w in enumerate(part):
                    n = min(w.length, CHUNK_SAMPLES)  # feature extractor truncation
                    dst[j, :n].copy_(wav[w.start: w.start + n], non_blocking=True)
                    dst[j, n:].zero_()
                return
            host = self._host_staging(k % 2, len(part))
            for j, w in enumerate(part):
                seg = wav[w.start: w.start + min(w.length, CHUNK_SAMPLES)]  # feature extractor truncation
                host[j, : len(seg)] = torch.from_numpy(np.ascontiguousarray(seg, np.float32))
                host[j, len(seg):] = 0
            eng.wave[: len(part)].copy_(host, non_blocking=host.is_pinned())
            if self._staging is not None:
                self._staging[1][k % 2].record(torch.cuda.current_stream(eng.wave.device))

        bkw = None
        if word_timestamps:
            bkw = [{"word_timestamps": True, "num_frames": list(num_frames[offs[k]: offs[k + 1]])}
                   for k in range(len(sizes))]
        res = eng.run_batches(sizes, load=load, batch_kwargs=bkw, task=task,
                              lang_ids=None if lang_id is None else [lang_id] * max(sizes, default=1),
                              max_new_tokens=max_new_tokens, return_timestamps=return_timestamps, num_beams=num_beams,
                              max_passes=max_passes,
                              **({"fallback": fallback, "window_offset": window_base} if fallback is not None else {}),
                              **({"condition_on_prev_tokens": True} if condition_on_prev_tokens else {}),
                              **(prompt or {}))
        out: List[List[int]] = []
        for seqs in res:
            out.extend(pad_right(seqs, self.gen.special.eot))
        # per-window record of the last call (languages, raw tokens of every seek pass) for diagnostics/tests
        self.last_window_langs = [lg for bl in eng.batch_langs for lg in bl]
        self.last_window_passes = [p for bp in eng.batch_passes for p in bp]
        self.last_window_prefixes = [p for bp in eng.batch_prefixes for p in bp]
        if word_timestamps:  # per window the concatenated segments' token times (not padded, as the pipeline's)
            self.last_window_token_timestamps = [t for bt in eng.batch_token_timestamps for t in bt]
        return out

    def _fallback_config(self, gk: Dict[str, Any]) -> FallbackConfig:
        """Pops generate()'s temperature-fallback kwargs (generation_whisper.py:398-401): `temperature` (a float or
        a list / tuple of temperatures tried in turn), the three segment criteria (else the checkpoint's
        generation_config values), `top_k` (sampling; GenerationConfig's default 50), `do_sample` (ignored: the
        temperature decides, as generate_with_fallback does), and the extension `seed` (the sampler's key).
        (condition_on_prev_tokens is popped by the caller.)"""
        g = self.gen
        t = gk.pop("temperature", None)
        temps = tuple(t) if isinstance(t, (list, tuple)) else (t,)
        gk.pop("do_sample", None)
        pick = lambda k: gk.pop(k) if gk.get(k) is not None else (gk.pop(k, None), getattr(g, k))[1]  # noqa: E731
        return FallbackConfig(temperatures=temps, compression_ratio_threshold=pick("compression_ratio_threshold"),
                              logprob_threshold=pick("logprob_threshold"), no_speech_threshold=pick("no_speech_threshold"),
                              top_k=int(gk.pop("top_k", 50) or 0), seed=int(gk.pop("seed", getattr(self, "sample_seed", 0))))

    def _host_staging(self, i: int, rows: int) -> torch.Tensor:
        """Pinned host buffer i (of two, alternating per batch) for a batch's waveforms: the upload is then an async
        copy on the encoder stream; a buffer is refilled only after its previous copy has completed."""
        wave = self.engine.wave
        if not (torch.is_tensor(wave) and wave.is_cuda):
            return torch.zeros(rows, CHUNK_SAMPLES, dtype=torch.float32)
        if self._staging is None:
            bufs = [torch.empty(wave.shape[0], CHUNK_SAMPLES, dtype=torch.float32, pin_memory=True) for _ in range(2)]
            self._staging = (bufs, [torch.cuda.Event() for _ in range(2)])
        self._staging[1][i].synchronize()
        return self._staging[0][i][:rows]


def batch_sizes(n: int, max_batch: int, sub_batch_min: Optional[int] = None) -> List[int]:
    """Engine batch sizes for n windows: ceil(n / max_batch) near-equal batches (e.g. 30 windows at 24 -> 15 + 15,
    so that the encoder of the second overlaps the decode of the first with the same work on each side), and two
    when a single batch would hold >= 2 * sub_batch_min windows."""
    if n <= 0:
        return []
    k = -(-n // max_batch)
    if k == 1 and sub_batch_min is not None and n >= 2 * sub_batch_min:
        k = 2
    base, rem = divmod(n, k)
    return [base + 1] * rem + [base] * (k - rem)


def _dims_from_checkpoint(path: str) -> WhisperDims:
    import json

    with open(os.path.join(path, "config.json")) as f:
        c = json.load(f)
    return WhisperDims(os.path.basename(os.path.normpath(path)), c["d_model"], c["encoder_layers"], c["decoder_layers"],
                       c["encoder_attention_heads"], c["encoder_ffn_dim"], c["num_mel_bins"], c["vocab_size"],
                       c.get("max_source_positions", 1500), c.get("max_target_positions", 448))
